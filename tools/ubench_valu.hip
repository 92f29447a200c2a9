// VALU throughput micro-benchmark for the SHA-256 instruction mix on gfx950.
// Each kernel runs ILP independent chains of one opcode per lane; throughput reported as
// lane-ops per clock per CU (128 == one wave64 VALU op per 2 cycles on each of the 4 SIMD32s).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <int OP>
__global__ __launch_bounds__(256) void k(unsigned* out, unsigned seed, int iters) {
    unsigned a0 = seed ^ threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11, a5 = a0 * 13, a6 = a0 * 17, a7 = a0 * 19;
    unsigned b = seed * 0x9e3779b9u + 1, c = seed + 12345;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < 16; ++u) {
#define STEP(x) \
    if (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(b)); \
    if (OP == 1) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(x)); \
    if (OP == 2) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x) : "v"(b), "v"(c)); \
    if (OP == 3) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c)); \
    if (OP == 4) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(b)); \
    if (OP == 5) asm volatile("v_lshl_or_b32 %0, %0, 3, %1" : "+v"(x) : "v"(b)); \
    if (OP == 6) asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(x)); \
    if (OP == 7) asm volatile("v_xad_u32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c)); \
    if (OP == 8) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(x) : "v"(b)); \
    if (OP == 9) asm volatile("v_bfi_b32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c)); \
    if (OP == 10) asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(*(unsigned long long*)&x) : "v"(b), "v"(c) : "s0", "s1"); \
    if (OP == 11) asm volatile("v_lshrrev_b64 %0, 7, %0" : "+v"(*(unsigned long long*)&x)); \
    if (OP == 12) asm volatile("v_alignbyte_b32 %0, %0, %1, 3" : "+v"(x) : "v"(b)); \
    if (OP == 13) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c)); \
    if (OP == 14) asm volatile("v_pk_mov_b32 %0, %0, %0 op_sel:[1,0]" : "+v"(*(unsigned long long*)&x)); \
    if (OP == 15) asm volatile("v_lshl_add_u32 %0, %0, 3, %1" : "+v"(x) : "v"(b));
            if (OP == 10 || OP == 11 || OP == 14) { STEP(a0) STEP(a2) STEP(a4) STEP(a6) }
            else { STEP(a0) STEP(a1) STEP(a2) STEP(a3) STEP(a4) STEP(a5) STEP(a6) STEP(a7) }
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

template <int OP>
double run(const char* name, int blocks_per_cu, int cus, unsigned* d, double ghz_hint) {
    const int grid = cus * blocks_per_cu;
    const int iters = 2000;
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k<OP>, dim3(grid), dim3(256), 0, 0, d, 1u, 10);
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(e0));
    hipLaunchKernelGGL(k<OP>, dim3(grid), dim3(256), 0, 0, d, 1u, iters);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    const double ops_per_lane = double(iters) * 16 * ((OP == 10 || OP == 11 || OP == 14) ? 4 : 8);
    const double lane_ops = ops_per_lane * grid * 256.0;
    const double per_s = lane_ops / (ms * 1e-3);
    printf("%-16s blocks/CU=%d  %8.2f Tlane-op/s  = %6.1f lane-ops/clk/CU @%.2fGHz\n", name, blocks_per_cu,
           per_s / 1e12, per_s / cus / (ghz_hint * 1e9), ghz_hint);
    return per_s;
}

int main(int argc, char** argv) {
    int cus = 0;
    CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    unsigned* d;
    CHK(hipMalloc(&d, sizeof(unsigned) * cus * 8 * 256));
    if (argc > 1 && argv[1][0] == 'c') {
        // PMC calibration: ONE launch with a known VALU count (16 x 8 v_add_u32 per loop iteration plus
        // the loop's own VALU overhead, see the ISA), to read rocprofv3's SQ_INSTS_VALU / SQ_WAVES scale
        // against (docs/PERF.md §1).
        const int grid = cus * 4, iters = 1000;
        hipLaunchKernelGGL(k<0>, dim3(grid), dim3(256), 0, 0, d, 1u, iters);
        CHK(hipDeviceSynchronize());
        printf("calib: waves=%d  v_add_u32 per wave=%d  (expected SQ_INSTS_VALU >= %.4e, SQ_WAVES = %d)\n",
               grid * 4, iters * 128, double(grid) * 4 * iters * 128, grid * 4);
        return 0;
    }
    const double ghz = 2.1;
    for (int bpc : {4, 8}) {
        run<0>("v_add_u32", bpc, cus, d, ghz);
        run<4>("v_xor_b32", bpc, cus, d, ghz);
        run<1>("v_alignbit(x,x)", bpc, cus, d, ghz);
        run<8>("v_alignbit(x,y)", bpc, cus, d, ghz);
        run<2>("v_bitop3_b32", bpc, cus, d, ghz);
        run<3>("v_add3_u32", bpc, cus, d, ghz);
        run<5>("v_lshl_or_b32", bpc, cus, d, ghz);
        run<6>("v_lshrrev_b32", bpc, cus, d, ghz);
        run<7>("v_xad_u32", bpc, cus, d, ghz);
        run<9>("v_bfi_b32", bpc, cus, d, ghz);
        run<10>("v_mad_u64_u32", bpc, cus, d, ghz);
        run<11>("v_lshrrev_b64", bpc, cus, d, ghz);
        run<12>("v_alignbyte_b32", bpc, cus, d, ghz);
        run<13>("v_perm_b32", bpc, cus, d, ghz);
        run<14>("v_pk_mov_b32", bpc, cus, d, ghz);
        run<15>("v_lshl_add_u32", bpc, cus, d, ghz);
    }
    return 0;
}
