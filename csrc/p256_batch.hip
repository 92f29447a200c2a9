// K5 batch path: one lane per signature for batches past kQuadMaxBatch (csrc/p256.hip), where the chip is
// full either way and one lane per signature does a quarter of the quad kernel's redundant work.
//
// This file is compiled with the default (occupancy-first) machine scheduler, unlike p256.hip: the
// default variant runs four waves per SIMD at 128 VGPRs, where the ILP-first schedule that shortens the
// block-latency kernels' dependency chains spills 85 VGPRs instead of 52. The throughput is the same under
// both schedules (19.05 vs 19.11 M sig/s at 132,800 in one session, profiles/r5/p256batch).
//
// reference: fastecdsa ecdsa.verify as called from upow/upow_transactions/transaction_input.py:84-120.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>
#include <string>

#include "native.h"
#include "p256_verify.h"

namespace upow {

// Per-lane window table {1..15}Q lives in global scratch. SOA = false: [lane][k] Jacobian entries
// (each lane's 16 x 96 B contiguous; a table load gathers 64 scattered lines per dword). SOA = true:
// dword-major [k][dword][lane], so the lanes of a wave that picked the same window digit read one
// contiguous run per dword (at most 16 distinct runs per load instead of 64 lines).
template <bool SOA>
__device__ __forceinline__ void tab_store(jac* scratch, int64_t n, int64_t i, int k, const jac& p) {
    if (SOA) {
        uint32_t* s = reinterpret_cast<uint32_t*>(scratch);
        const uint32_t* src = reinterpret_cast<const uint32_t*>(&p);
#pragma unroll
        for (int d = 0; d < 24; ++d) s[(int64_t(k) * 24 + d) * n + i] = src[d];
    } else {
        scratch[i * 16 + k] = p;
    }
}

template <bool SOA>
__device__ __forceinline__ jac tab_load(const jac* scratch, int64_t n, int64_t i, int k) {
    if (SOA) {
        jac p;
        const uint32_t* s = reinterpret_cast<const uint32_t*>(scratch);
        uint32_t* dst = reinterpret_cast<uint32_t*>(&p);
#pragma unroll
        for (int d = 0; d < 24; ++d) dst[d] = s[(int64_t(k) * 24 + d) * n + i];
        return p;
    }
    return scratch[i * 16 + k];
}

template <int MIN_WAVES, bool SOA, int WPB = 1>
__global__ __launch_bounds__(64 * WPB, MIN_WAVES) void p256_verify_kernel(const VerifyItem* __restrict__ items, int64_t n,
                                                          const aff* __restrict__ gtab16, jac* __restrict__ scratch,
                                                          uint8_t* __restrict__ status, int spw) {
    // spw = signatures per 64-lane wave (lanes >= spw idle; A/B of partially filled waves);
    // WPB = waves per workgroup (a workgroup's waves are spread over the CU's SIMDs)
    const int lane = int(threadIdx.x) & 63;
    const int64_t i = (int64_t(blockIdx.x) * WPB + (threadIdx.x >> 6)) * spw + lane;
    if (lane >= spw || i >= n) return;
    const VerifyItem it = items[i];
    aff q;
    fe r, u1, u2;
    const uint8_t pro = verify_prologue(it, q, r, u1, u2);
    if (pro != 255) { status[i] = pro; return; }
    jac t = jac_from_aff(q);  // entry k - 1 = k*Q, k = 1..16 (signed 5-bit windows)
    tab_store<SOA>(scratch, n, i, 0, t);
    for (int k = 2; k <= 16; ++k) {
        t = jac_madd(t, q);
        tab_store<SOA>(scratch, n, i, k - 1, t);
    }
    jac acc = jac_inf();
    BoothW5 bw(u2);
    for (int w = kBoothWindows - 1; w >= 0; --w) {
        acc = jac_dbl(acc); acc = jac_dbl(acc); acc = jac_dbl(acc); acc = jac_dbl(acc); acc = jac_dbl(acc);
        const int d = bw.next();
        if (d) {
            jac e = tab_load<SOA>(scratch, n, i, (d < 0 ? -d : d) - 1);
            if (d < 0) e.y = fe_neg(e.y);
            acc = jac_add(acc, e);
        }
    }
    const jac R = jac_add(mul_g16(u1, gtab16), acc);
    status[i] = verify_epilogue(R, r);
}


void p256_batch_launch(char variant, const void* items, int64_t n, const void* gtab16, void* scratch, uint8_t* status,
                       int spw, void* stream) {
    const VerifyItem* d_items = static_cast<const VerifyItem*>(items);
    const aff* d_tab = static_cast<const aff*>(gtab16);
    jac* d_scratch = static_cast<jac*>(scratch);
    hipStream_t stream_ = static_cast<hipStream_t>(stream);
    const int block = 64;
    const int grid = int((n + spw - 1) / spw);
    // Variant 1 (the one-lane default): __launch_bounds__(64, 4) -> 4 waves/SIMD at 128 VGPRs, 7-9 % faster
    // than the compiler's own choice (variant 0) in the A/B runs of scripts/p256_throughput.py
    // (profiles/p256_variants_ab.txt). Variant 2: dword-major (SoA) window tables, slower (the gathers were
    // not the bottleneck). Variant 3: four waves per workgroup.
    if (variant == '0')
        hipLaunchKernelGGL((p256_verify_kernel<1, false>), dim3(grid), dim3(block), 0, stream_, d_items, n, d_tab, d_scratch,
                           status, spw);
    else if (variant == '2')
        hipLaunchKernelGGL((p256_verify_kernel<1, true>), dim3(grid), dim3(block), 0, stream_, d_items, n, d_tab, d_scratch,
                           status, spw);
    else if (variant == '5')  // 3 waves per SIMD: __launch_bounds__(64, 3), up to 168 VGPRs
        hipLaunchKernelGGL((p256_verify_kernel<3, false>), dim3(grid), dim3(block), 0, stream_, d_items, n, d_tab, d_scratch,
                           status, spw);
    else if (variant == '3')
        hipLaunchKernelGGL((p256_verify_kernel<4, false, 4>), dim3((grid + 3) / 4), dim3(256), 0, stream_, d_items, n, d_tab,
                           d_scratch, status, spw);
    else
        hipLaunchKernelGGL((p256_verify_kernel<4, false>), dim3(grid), dim3(block), 0, stream_, d_items, n, d_tab, d_scratch,
                           status, spw);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) throw std::runtime_error(std::string("p256_verify_kernel launch: ") + hipGetErrorString(e));
}

}  // namespace upow
