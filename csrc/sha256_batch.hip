// K3: batched variable-length SHA-256 (txids / merkle leaves) on gfx950.
//
// reference: txid = sha256(tx bytes) computed one at a time in Python (upow/helpers.py:41-44,
// upow/upow_transactions/transaction.py:85-88); merkle leaves (upow/manager.py:365-378).
//
// One message per lane; the host repacks messages at 4-byte aligned offsets so each lane streams
// its message with dword loads (byte-swapped to big-endian words in registers). A 2 MB block holds
// ~8.3k txs -> ~130 waves: latency-bound, a few tens of microseconds, so no LDS staging is needed;
// the whole block is hashed in one launch instead of 8.3k Python calls.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "dev_pool.h"
#include "native.h"
#include "streams.h"
#include "sha256_common.h"

namespace upow {

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

__constant__ uint32_t bK[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

__device__ __forceinline__ void dev_compress(uint32_t st[8], uint32_t w[16]) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
    for (int i = 0; i < 64; ++i) {
        uint32_t wi;
        if (i < 16) {
            wi = w[i];
        } else {
            wi = w[i & 15] + SSIG0(w[(i - 15) & 15]) + w[(i - 7) & 15] + SSIG1(w[(i - 2) & 15]);
            w[i & 15] = wi;
        }
        uint32_t t1 = h + BSIG1(e) + CH(e, f, g) + bK[i] + wi;
        uint32_t t2 = BSIG0(a) + MAJ(a, b, c);
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

// data: 4-byte aligned message starts; offs[i] = byte offset of message i, lens[i] = its length.
__global__ __launch_bounds__(256) void sha256_varlen_kernel(const uint32_t* __restrict__ data,
                                                            const int64_t* __restrict__ offs,
                                                            const uint32_t* __restrict__ lens, int64_t n,
                                                            uint32_t* __restrict__ out) {
    const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t* base = data + (offs[i] >> 2);
    const uint32_t L = lens[i];
    const uint32_t nblocks = (L + 9 + 63) >> 6;
    const uint64_t bits = uint64_t(L) << 3;
    uint32_t st[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                      0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
    for (uint32_t blk = 0; blk < nblocks; ++blk) {
        uint32_t w[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const uint32_t bi = (blk << 6) + 4u * k;
            uint32_t v = 0;
            if (bi + 4 <= L) {
                v = __builtin_bswap32(base[bi >> 2]);
            } else if (bi < L) {
                const uint32_t keep = L - bi;  // 1..3 message bytes in this word
                const uint32_t raw = __builtin_bswap32(base[bi >> 2]);
                const uint32_t mask = 0xffffffffu << (32 - 8 * keep);
                v = (raw & mask) | (0x80u << (24 - 8 * keep));
            } else if (bi == L) {
                v = 0x80000000u;
            }
            w[k] = v;
        }
        if (blk == nblocks - 1) {
            w[14] = uint32_t(bits >> 32);
            w[15] = uint32_t(bits);
        }
        dev_compress(st, w);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) out[i * 8 + k] = st[k];
}

static void hchk(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

std::vector<uint8_t> sha256_batch_gpu(const uint8_t* data, int64_t nbytes, const int64_t* offsets, int64_t n) {
    node_device_enter();
    (void)nbytes;
    std::vector<uint8_t> out(size_t(n) * 32);
    if (n == 0) return out;
    // repack at 4-byte aligned offsets (+4 zero bytes of slack so the partial-word load stays in bounds)
    std::vector<int64_t> aoff(n);
    std::vector<uint32_t> lens(n);
    int64_t total = 0;
    for (int64_t i = 0; i < n; ++i) {
        aoff[i] = total;
        lens[i] = uint32_t(offsets[i + 1] - offsets[i]);
        total += (int64_t(lens[i]) + 3) & ~int64_t(3);
    }
    total += 4;
    std::vector<uint8_t> packed(size_t(total), 0);
    for (int64_t i = 0; i < n; ++i) std::memcpy(packed.data() + aoff[i], data + offsets[i], lens[i]);
    PooledBuf<uint8_t> b_data{size_t(total)};
    PooledBuf<int64_t> b_off{size_t(n)};
    PooledBuf<uint32_t> b_len{size_t(n)}, b_out{size_t(n) * 8};
    uint8_t* d_data = b_data.p;
    int64_t* d_off = b_off.p;
    uint32_t *d_len = b_len.p, *d_out = b_out.p;
    node_h2d(d_data, packed.data(), size_t(total), "h2d data");
    node_h2d(d_off, aoff.data(), sizeof(int64_t) * n, "h2d off");
    node_h2d(d_len, lens.data(), sizeof(uint32_t) * n, "h2d len");
    const int block = 256;
    const int grid = int((n + block - 1) / block);
    hipLaunchKernelGGL(sha256_varlen_kernel, dim3(grid), dim3(block), 0, node_stream(),
                       reinterpret_cast<const uint32_t*>(d_data), d_off, d_len, n, d_out);
    hchk(hipGetLastError(), "sha256_varlen_kernel launch");
    std::vector<uint32_t> words(size_t(n) * 8);
    node_d2h(words.data(), d_out, 32 * size_t(n), "d2h out");
    for (size_t k = 0; k < words.size(); ++k) store_be32(out.data() + 4 * k, words[k]);
    return out;
}

int gpu_device_count() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

std::string gpu_arch_name(int device) {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, device) != hipSuccess) return "";
    return std::string(p.gcnArchName);
}

}  // namespace upow
