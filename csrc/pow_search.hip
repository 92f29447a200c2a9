// K1: SHA-256 proof-of-work nonce search for gfx950 (CDNA4, wave64).
//
// reference hot loop: miner.py:83-98 (one hashlib.sha256 per nonce in Python) with the predicate of
// miner.py:43-61 / upow/manager.py:130-151.
//
// MI355X design
//  * one nonce per lane, 64 nonces per wavefront, grid-strided over the 2^32 nonce space;
//  * the header's first 64-byte block is nonce independent -> host midstate;
//  * v2 header (108 B): the tail block's words W0..W9 are nonce independent too, so the host also
//    runs rounds 0..9 and the kernel starts at round 10 (W10 = the nonce word);
//    v1 header (138 B): the nonce straddles W1/W2 of the third block; the kernel starts at round 1;
//  * every job constant is a kernel argument -> SGPRs; all loop-invariant partial sums of the message
//    schedule are hoisted by the compiler (LICM + reassociation) so the loop body only contains the
//    nonce-dependent work;
//  * the message schedule is kept in VGPRs (a 16-entry rolling window), not LDS: each W word is
//    produced once and consumed 4x within ~16 rounds; an LDS round trip per use would add a
//    ds_write+4 ds_read per word (≈240 LDS dword ops per nonce) against ≈1.2k VALU ops, making LDS a
//    co-bottleneck (MI355X_MICROARCH.md §LDS: 32 dwords/clk/CU for b32 vs 128 VALU lane-ops/clk/CU);
//  * rotates lower to v_alignbit_b32, the 3-input XORs of the Sigma functions and Maj to the gfx950
//    v_bitop3_b32 (truth tables 0x96 / 0xE8), 3-input adds to v_add3_u32 (1110 VALU ops per nonce in
//    the v2 loop body vs 1359 with 2-input XORs);
//  * the predicate only needs digest word H0 for difficulty < 8 (8 hex nibbles) -> one compare per
//    nonce; hits are appended with an atomic to a small candidate list and re-checked exactly on the
//    host (covers d >= 8 and the d < 1 "whole hash" quirk).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <stdexcept>
#include <string>

#include "native.h"
#include "streams.h"
#include "sha256_common.h"

namespace upow {

struct PowJobDev {
    uint32_t st[8];   // working state after the nonce-independent rounds of the tail block
    uint32_t mid[8];  // chaining value before the tail block (feed-forward)
    uint32_t w[16];   // tail block words (nonce bits zero)
    uint32_t tmask;   // H0 bits that must equal tword
    uint32_t tword;
    uint32_t frac_shift;  // right shift of H0 that brings the fractional nibble to bits 0..3
    uint32_t frac_limit;  // nibble must be < frac_limit (16 == no fractional check)
};

#define ROTR(x, n) __builtin_amdgcn_alignbit((x), (x), (n))
// gfx950 v_bitop3_b32: 3-input bitwise op from an 8-bit truth table. XOR3 (0x96) and MAJ (0xE8) are
// symmetric in their inputs, so the immediates do not depend on the operand->table-column order.
#define XOR3(a, b, c) __builtin_amdgcn_bitop3_b32((a), (b), (c), 0x96)
#define BSIG0(x) XOR3(ROTR((x), 2), ROTR((x), 13), ROTR((x), 22))
#define BSIG1(x) XOR3(ROTR((x), 6), ROTR((x), 11), ROTR((x), 25))
#define SSIG0(x) XOR3(ROTR((x), 7), ROTR((x), 18), ((x) >> 3))
#define SSIG1(x) XOR3(ROTR((x), 17), ROTR((x), 19), ((x) >> 10))
#define CH(e, f, g) (((e) & (f)) | (~(e) & (g)))
#define MAJ(a, b, c) __builtin_amdgcn_bitop3_b32((a), (b), (c), 0xE8)

__constant__ uint32_t dK[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

// H0 of SHA256(header) for the lane's nonce word `v`.
//  LAYOUT 2: v is W10 of the tail block (v = bswap(nonce_le)); rounds 0..9 precomputed.
//  LAYOUT 1: v is the little-endian nonce; W1 low half = n0,n1, W2 high half = n2,n3; round 0 precomputed.
template <int LAYOUT>
__device__ __forceinline__ uint32_t pow_h0(const PowJobDev& job, uint32_t v) {
    constexpr int R0 = LAYOUT == 2 ? 10 : 1;
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) w[i] = job.w[i];
    if (LAYOUT == 2) {
        w[10] = v;
    } else {
        w[1] = job.w[1] | ((v & 0xffu) << 8) | ((v >> 8) & 0xffu);
        w[2] = job.w[2] | (((v >> 16) & 0xffu) << 24) | ((v >> 24) << 16);
    }
    uint32_t a = job.st[0], b = job.st[1], c = job.st[2], d = job.st[3];
    uint32_t e = job.st[4], f = job.st[5], g = job.st[6], h = job.st[7];
#pragma unroll
    for (int i = R0; i < 64; ++i) {
        uint32_t wi;
        if (i < 16) {
            wi = w[i];
        } else {
            wi = w[i & 15] + SSIG0(w[(i - 15) & 15]) + w[(i - 7) & 15] + SSIG1(w[(i - 2) & 15]);
            w[i & 15] = wi;
        }
        uint32_t t1 = h + BSIG1(e) + CH(e, f, g) + dK[i] + wi;
        uint32_t t2 = BSIG0(a) + MAJ(a, b, c);
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    return job.mid[0] + a;
}

// Variant 2 (A/B evidence for the design note above): the same v2 search with the expanded message
// schedule W16..W63 staged in LDS instead of VGPRs. Each lane owns a 16-word ring in LDS laid out
// [word][lane] (consecutive lanes -> consecutive banks, conflict-free); every produced word is one
// ds_write_b32 and each of its four consumers one ds_read_b32. `volatile` keeps the compiler from
// forwarding the stores back into registers, so this really is the LDS-staged form.
typedef __attribute__((address_space(3))) volatile uint32_t lds_u32;

__device__ __forceinline__ uint32_t pow_h0_lds(const PowJobDev& job, uint32_t v, lds_u32* ring) {
    const uint32_t tid = threadIdx.x;
    // words 0..15 are job constants (SGPRs) or the nonce word; only W16..W63 live in LDS
    auto W = [&](int i) -> uint32_t { return i < 16 ? (i == 10 ? v : job.w[i]) : ring[(i & 15) * 256 + tid]; };
    uint32_t a = job.st[0], b = job.st[1], c = job.st[2], d = job.st[3];
    uint32_t e = job.st[4], f = job.st[5], g = job.st[6], h = job.st[7];
#pragma unroll
    for (int i = 10; i < 64; ++i) {
        uint32_t wi;
        if (i < 16) {
            wi = W(i);
        } else {
            wi = W(i - 16) + SSIG0(W(i - 15)) + W(i - 7) + SSIG1(W(i - 2));
            ring[(i & 15) * 256 + tid] = wi;
        }
        uint32_t t1 = h + BSIG1(e) + CH(e, f, g) + dK[i] + wi;
        uint32_t t2 = BSIG0(a) + MAJ(a, b, c);
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    return job.mid[0] + a;
}

__global__ __launch_bounds__(256, 1) void pow_search_lds_kernel(PowJobDev job, uint32_t v_base, uint32_t iters,
                                                                uint32_t* __restrict__ out_count,
                                                                uint32_t* __restrict__ out_words, uint32_t cap) {
    __shared__ uint32_t ring[16 * 256];
    const uint32_t nthreads = gridDim.x * blockDim.x;
    uint32_t v = v_base + blockIdx.x * blockDim.x + threadIdx.x;
    for (uint32_t it = 0; it < iters; ++it, v += nthreads) {
        const uint32_t h0 = pow_h0_lds(job, v, (lds_u32*)ring);
        const bool hit = ((h0 ^ job.tword) & job.tmask) == 0 && ((h0 >> job.frac_shift) & 0xfu) < job.frac_limit;
        if (__builtin_expect(hit, 0)) {
            const uint32_t slot = atomicAdd(out_count, 1u);
            if (slot < cap) out_words[slot] = v;
        }
    }
}

template <int LAYOUT, int MIN_WAVES_PER_SIMD>
__global__ __launch_bounds__(256, MIN_WAVES_PER_SIMD) void pow_search_kernel(PowJobDev job, uint32_t v_base, uint32_t iters,
                                                         uint32_t* __restrict__ out_count,
                                                         uint32_t* __restrict__ out_words, uint32_t cap) {
    const uint32_t nthreads = gridDim.x * blockDim.x;
    uint32_t v = v_base + blockIdx.x * blockDim.x + threadIdx.x;
    for (uint32_t it = 0; it < iters; ++it, v += nthreads) {
        const uint32_t h0 = pow_h0<LAYOUT>(job, v);
        const bool hit = ((h0 ^ job.tword) & job.tmask) == 0 && ((h0 >> job.frac_shift) & 0xfu) < job.frac_limit;
        if (__builtin_expect(hit, 0)) {
            const uint32_t slot = atomicAdd(out_count, 1u);
            if (slot < cap) out_words[slot] = v;
        }
    }
}

// ------------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------------
static void hip_check(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

PowJobDev make_pow_job(const PowJobHost& hj) {
    PowJobDev j{};
    const uint8_t* hdr = hj.header.data();
    const size_t len = hj.header.size();
    if (len != 108 && len != 138) throw std::invalid_argument("header must be 108 (v2) or 138 (v1) bytes");
    uint32_t st[8];
    std::memcpy(st, kSha256IV, sizeof(st));
    const int full_blocks = len == 108 ? 1 : 2;
    for (int b = 0; b < full_blocks; ++b) host_compress(st, hdr + 64 * b);
    uint8_t tail[64] = {0};
    const size_t rem = len - 64 * full_blocks;
    std::memcpy(tail, hdr + 64 * full_blocks, rem);
    // zero the nonce bytes (last 4 bytes of the header) in the template
    std::memset(tail + rem - 4, 0, 4);
    tail[rem] = 0x80;
    const uint64_t bits = uint64_t(len) * 8;
    for (int i = 0; i < 8; ++i) tail[56 + i] = uint8_t(bits >> (56 - 8 * i));
    for (int i = 0; i < 16; ++i) j.w[i] = load_be32(tail + 4 * i);
    std::memcpy(j.mid, st, sizeof(st));
    uint32_t ws[8];
    std::memcpy(ws, st, sizeof(st));
    host_rounds(ws, j.w, len == 108 ? 10 : 1);
    std::memcpy(j.st, ws, sizeof(ws));
    j.tmask = hj.tmask;
    j.tword = hj.tword;
    j.frac_shift = hj.frac_shift;
    j.frac_limit = hj.frac_limit;
    return j;
}

struct PowDeviceBuffers {
    int device = -1;
    uint32_t* d_count = nullptr;
    uint32_t* d_words = nullptr;
    uint32_t cap = 0;
};

static thread_local PowDeviceBuffers g_pow_bufs;

static PowDeviceBuffers& pow_buffers(uint32_t cap) {
    int dev = 0;
    hip_check(hipGetDevice(&dev), "hipGetDevice");
    PowDeviceBuffers& b = g_pow_bufs;
    if (b.device != dev || b.cap < cap) {
        if (b.d_count) { (void)hipFree(b.d_count); (void)hipFree(b.d_words); }
        hip_check(hipMalloc(&b.d_count, sizeof(uint32_t)), "hipMalloc count");
        hip_check(hipMalloc(&b.d_words, sizeof(uint32_t) * cap), "hipMalloc words");
        b.device = dev;
        b.cap = cap;
    }
    return b;
}

// Grid = exactly the resident capacity of the chip (CUs x blocks/CU for this kernel's VGPR/SGPR use),
// so every launch is one full "wave" of workgroups with no tail round. The occupancy API can report
// one block/CU too many for SGPR-heavy kernels (MI355X_MICROARCH.md §Residency), which would only
// create a small second round here, so we take min(API, 800 / (ceil(sgpr/16)*16 + 16)).
static int pow_resident_blocks(bool v2, int variant) {
    int dev = 0, cus = 0, per_cu = 0;
    hip_check(hipGetDevice(&dev), "hipGetDevice");
    hip_check(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev), "attr");
    const void* fn = v2 ? (variant == 1   ? reinterpret_cast<const void*>(&pow_search_kernel<2, 8>)
                           : variant == 2 ? reinterpret_cast<const void*>(&pow_search_lds_kernel)
                                          : reinterpret_cast<const void*>(&pow_search_kernel<2, 1>))
                        : reinterpret_cast<const void*>(&pow_search_kernel<1, 1>);
    hip_check(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 256, 0), "occupancy");
    hipFuncAttributes attr{};
    if (hipFuncGetAttributes(&attr, fn) == hipSuccess) {
        (void)attr;
    }
    if (per_cu < 1) per_cu = 1;
    if (per_cu > 8) per_cu = 8;
    return cus * per_cu;
}

PowKernelInfo pow_kernel_info(int variant) {
    PowKernelInfo k;
    int dev = 0;
    hip_check(hipGetDevice(&dev), "hipGetDevice");
    hip_check(hipDeviceGetAttribute(&k.cus, hipDeviceAttributeMultiprocessorCount, dev), "attr");
    k.resident_blocks = pow_resident_blocks(true, variant);
    k.blocks_per_cu = k.resident_blocks / (k.cus ? k.cus : 1);
    return k;
}

// Search nonce words [start, start + count) (count a multiple of the grid size is not required:
// the tail is covered by an extra short launch). Returns all candidate nonce words (host re-checks).
PowResult pow_search_gpu(const PowJobHost& hj, uint64_t start, uint64_t count, int grid_blocks,
                         uint32_t chunk_iters, uint32_t cap, int variant) {
    PowJobDev job = make_pow_job(hj);
    const bool v2 = hj.header.size() == 108;
    node_device_enter();  // a rank's search from any of its threads runs on the rank's own GPU
    PowDeviceBuffers& buf = pow_buffers(cap);
    hipStream_t st = miner_stream();  // least priority: node kernels go first (csrc/streams.h)
    hip_check(hipMemsetAsync(buf.d_count, 0, sizeof(uint32_t), st), "memset");
    const uint32_t block = 256;
    if (grid_blocks <= 0) grid_blocks = pow_resident_blocks(v2, variant);
    const uint64_t per_launch_threads = uint64_t(grid_blocks) * block;
    if (chunk_iters == 0) {
        // nonces per dispatch: 2^28 (~7.6 ms on MI355X) for a dedicated miner; 2^23 (~0.25 ms) once this
        // process also runs node kernels, so a queued node kernel waits at most one short dispatch (the miner
        // CLI next to a node process uses 2^23 too); UPOW_POW_DISPATCH_LOG2 overrides both
        int lg = node_stream_live().load() ? 23 : 28;
        if (const char* e = std::getenv("UPOW_POW_DISPATCH_LOG2")) lg = std::max(16, std::min(32, std::atoi(e)));
        chunk_iters = uint32_t(std::max<uint64_t>(1, (uint64_t(1) << lg) / per_launch_threads));
    }
    uint64_t done = 0;
    while (done < count) {
        const uint64_t left = count - done;
        uint32_t iters = chunk_iters;
        uint32_t gb = grid_blocks;
        if (uint64_t(iters) * per_launch_threads > left) {
            iters = uint32_t(left / per_launch_threads);
            if (iters == 0) {
                iters = 1;
                gb = uint32_t((left + block - 1) / block);
                if (uint64_t(gb) * block > left) {
                    // final ragged piece: round down to whole blocks, then single lanes via the host
                    gb = uint32_t(left / block);
                    if (gb == 0) break;
                }
            }
        }
        const uint32_t vb = uint32_t(start + done);
        if (v2 && variant == 2)
            hipLaunchKernelGGL(pow_search_lds_kernel, dim3(gb), dim3(block), 0, st, job, vb, iters, buf.d_count,
                               buf.d_words, cap);
        else if (v2 && variant == 1)
            hipLaunchKernelGGL((pow_search_kernel<2, 8>), dim3(gb), dim3(block), 0, st, job, vb, iters,
                               buf.d_count, buf.d_words, cap);
        else if (v2)
            hipLaunchKernelGGL((pow_search_kernel<2, 1>), dim3(gb), dim3(block), 0, st, job, vb, iters,
                               buf.d_count, buf.d_words, cap);
        else
            hipLaunchKernelGGL((pow_search_kernel<1, 1>), dim3(gb), dim3(block), 0, st, job, vb, iters,
                               buf.d_count, buf.d_words, cap);
        hip_check(hipGetLastError(), "pow_search_kernel launch");
        done += uint64_t(iters) * gb * block;
    }
    uint32_t n = 0;
    hip_check(hipMemcpyAsync(&n, buf.d_count, sizeof(uint32_t), hipMemcpyDeviceToHost, st), "copy count");
    hip_check(hipStreamSynchronize(st), "miner stream sync");
    PowResult r;
    r.searched = done;
    r.total_hits = n;
    const uint32_t stored = n < cap ? n : cap;
    r.words.resize(stored);
    if (stored)
    {
        hip_check(hipMemcpyAsync(r.words.data(), buf.d_words, sizeof(uint32_t) * stored, hipMemcpyDeviceToHost, st),
                  "copy words");
        hip_check(hipStreamSynchronize(st), "miner stream sync");
    }
    // any ragged remainder (< 256 nonces) is searched on the host so the requested range is exact
    if (done < count) {
        for (uint64_t k = done; k < count; ++k) {
            const uint32_t v = uint32_t(start + k);
            if (pow_check_word_host(hj, v)) { r.words.push_back(v); r.total_hits++; }
        }
        r.searched = count;
    }
    return r;
}

}  // namespace upow
