// Issue rate of the instructions a 256-bit field product can be built from, on gfx950: 32x32->64 integer
// multiply-add (v_mad_u64_u32), 32-bit add-with-carry, 64-bit add (v_lshl_add_u64), f64 FMA, f64 add.
// Each kernel runs 8 independent chains per lane, so latency hides behind issue; the grid fills the chip
// (4 waves per SIMD). Reported: wave-instructions per SIMD per cycle relative to a plain 32-bit add.
// Build: hipcc --offload-arch=gfx950 -O3 -o build-ab/isa_rates scripts/isa_rates.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#include "../csrc/p256_field.h"

#define CHECK(x)                                                                    \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
            return 1;                                                               \
        }                                                                           \
    } while (0)

constexpr int kIters = 4096;

__global__ void k_add32(uint32_t* out, uint32_t seed) {
    uint32_t a[8];
    for (int k = 0; k < 8; ++k) a[k] = seed + threadIdx.x + k;
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) a[k] = a[k] + (a[k] ^ seed);  // one v_xor + one v_add: 2 per step
    }
    uint32_t s = 0;
    for (int k = 0; k < 8; ++k) s ^= a[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mad64(uint32_t* out, uint32_t seed) {
    uint64_t a[8];
    const uint32_t m = seed | 1u;
    for (int k = 0; k < 8; ++k) a[k] = seed + threadIdx.x + k;
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) a[k] = uint64_t(uint32_t(a[k] >> 32) ^ m) * m + a[k];  // v_xor + v_mad_u64_u32
    }
    uint32_t s = 0;
    for (int k = 0; k < 8; ++k) s ^= uint32_t(a[k]) ^ uint32_t(a[k] >> 32);
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_addc(uint32_t* out, uint32_t seed) {
    uint32_t a[8];
    for (int k = 0; k < 8; ++k) a[k] = seed + threadIdx.x + k;
    unsigned c0 = 0, c1 = 0, c2 = 0, c3 = 0;
    for (int i = 0; i < kIters; ++i) {  // four independent two-limb carry chains
        a[0] = __builtin_addc(a[0], a[4], c0, &c0);
        a[1] = __builtin_addc(a[1], a[5], c1, &c1);
        a[2] = __builtin_addc(a[2], a[6], c2, &c2);
        a[3] = __builtin_addc(a[3], a[7], c3, &c3);
        a[4] = __builtin_addc(a[4], a[0], c0, &c0);
        a[5] = __builtin_addc(a[5], a[1], c1, &c1);
        a[6] = __builtin_addc(a[6], a[2], c2, &c2);
        a[7] = __builtin_addc(a[7], a[3], c3, &c3);
    }
    uint32_t s = c0 ^ c1 ^ c2 ^ c3;
    for (int k = 0; k < 8; ++k) s ^= a[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_add64(uint32_t* out, uint32_t seed) {
    uint64_t a[8];
    for (int k = 0; k < 8; ++k) a[k] = (uint64_t(seed) << 20) + threadIdx.x + k;
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) a[k] = a[k] + (a[k] >> 1);  // v_lshrrev_b64 / v_lshl_add_u64
    }
    uint32_t s = 0;
    for (int k = 0; k < 8; ++k) s ^= uint32_t(a[k]) ^ uint32_t(a[k] >> 32);
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_fma64(uint32_t* out, uint32_t seed) {
    double a[8];
    const double m = 1.0000001 + seed * 1e-12;
    for (int k = 0; k < 8; ++k) a[k] = threadIdx.x + k;
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) a[k] = __builtin_fma(a[k], m, 0.5);  // one v_fma_f64
    }
    double s = 0;
    for (int k = 0; k < 8; ++k) s += a[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = uint32_t(s);
}

__global__ void k_mulhi(uint32_t* out, uint32_t seed) {
    uint32_t a[8];
    const uint32_t m = seed | 1u;
    for (int k = 0; k < 8; ++k) a[k] = seed + threadIdx.x + k;
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) a[k] = __umulhi(a[k], m) ^ a[k];  // v_mul_hi_u32 + v_xor
    }
    uint32_t s = 0;
    for (int k = 0; k < 8; ++k) s ^= a[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// whole field products: two independent fe_mul (or fe_sqr) chains per lane, 256 products per chain
constexpr int kFeIters = 256;
__global__ void k_femul(uint32_t* out, uint32_t seed) {
    using namespace upow::p256;
    fe a, b;
    for (int k = 0; k < 8; ++k) { a.v[k] = seed * 0x9e3779b9u + threadIdx.x + k; b.v[k] = a.v[k] ^ 0x5bd1e995u; }
    for (int i = 0; i < kFeIters; ++i) { a = fe_mul(a, b); b = fe_mul(b, a); }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a.v[0] ^ b.v[7];
}
__global__ void k_fesqr(uint32_t* out, uint32_t seed) {
    using namespace upow::p256;
    fe a, b;
    for (int k = 0; k < 8; ++k) { a.v[k] = seed * 0x9e3779b9u + threadIdx.x + k; b.v[k] = a.v[k] ^ 0x5bd1e995u; }
    for (int i = 0; i < kFeIters; ++i) { a = fe_sqr(a); b = fe_sqr(b); }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a.v[0] ^ b.v[7];
}

int main() {
    int dev = 0;
    CHECK(hipSetDevice(dev));
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, dev));
    const int cus = prop.multiProcessorCount;
    const int blocks = cus * 4, threads = 256;  // 4 waves per SIMD
    uint32_t* out = nullptr;
    CHECK(hipMalloc(&out, size_t(blocks) * threads * sizeof(uint32_t)));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    struct K { const char* name; void (*fn)(uint32_t*, uint32_t); double ops_per_step; };
    // ops_per_step scales kIters * 8 to the number of chain steps the kernel issues
    const K ks[] = {{"add32 (v_xad_u32)", k_add32, 1.0},
                    {"mad_u64_u32 (+ v_xor)", k_mad64, 1.0},
                    {"addc chain", k_addc, 1.0},
                    {"add64 (shift + add)", k_add64, 1.0},
                    {"fma_f64", k_fma64, 1.0},
                    {"mul_hi_u32 (+ v_xor)", k_mulhi, 1.0},
                    {"fe_mul (per product)", k_femul, double(2 * kFeIters) / (kIters * 8)},
                    {"fe_sqr (per product)", k_fesqr, double(2 * kFeIters) / (kIters * 8)}};
    const double clock_hz = double(prop.clockRate) * 1e3;
    std::printf("{\"device\": \"%s\", \"cus\": %d, \"clock_mhz\": %.0f, \"results\": [", prop.name, cus, clock_hz / 1e6);
    for (size_t t = 0; t < sizeof(ks) / sizeof(ks[0]); ++t) {
        hipLaunchKernelGGL(ks[t].fn, dim3(blocks), dim3(threads), 0, 0, out, 7u);  // warm-up
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(e0));
        for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(ks[t].fn, dim3(blocks), dim3(threads), 0, 0, out, 7u + r);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        const double waves = double(blocks) * threads / 64 * 5;
        const double steps = waves * kIters * 8 * ks[t].ops_per_step;  // chain steps issued, in wave instructions
        const double cycles = ms * 1e-3 * clock_hz * cus * 4;  // SIMD-cycles
        std::printf("%s{\"kernel\": \"%s\", \"ms\": %.3f, \"simd_cycles_per_step\": %.2f}", t ? ", " : "", ks[t].name, ms,
                    cycles / steps);
    }
    std::printf("]}\n");
    CHECK(hipFree(out));
    return 0;
}
