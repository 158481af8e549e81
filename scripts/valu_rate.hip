// VALU issue rate on gfx950, per instruction kind and waves per SIMD (measurement only): each
// lane runs 8 independent chains of one instruction kind; grid = 256 CUs x W workgroups of 4
// waves.  Prints cycles per instruction per SIMD = (kernel cycles at the measured s_memtime
// rate) / (instructions issued per SIMD) -- 2 if a wave64 instruction issues in 2 cycles (SIMD
// 32 lanes wide), 4 if in 4.  Settles which reading of SQ_ACTIVE_INST_VALU the DESIGN uses.
//   hipcc --offload-arch=gfx950 -O3 -o scripts/valu_rate scripts/valu_rate.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

constexpr int kIter = 4096;

template <int OP>
__device__ __forceinline__ void op(uint32_t &a, uint32_t b, uint32_t c, uint32_t &s) {
    if constexpr (OP == 0) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a) : "v"(b));
    if constexpr (OP == 1) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a) : "v"(b), "v"(c));
    if constexpr (OP == 2) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x78" : "+v"(a) : "v"(b), "s"(s));
    if constexpr (OP == 3) asm volatile("v_perm_b32 %0, %1, %0, %2" : "+v"(a) : "v"(b), "v"(c));
    if constexpr (OP == 4) asm volatile("v_pk_lshlrev_b16 %0, 3, %0 op_sel_hi:[0,1]" : "+v"(a));
    if constexpr (OP == 5) asm volatile("v_bfe_u32 %0, %0, %1, 4" : "+v"(a) : "v"(b));
    if constexpr (OP == 6) asm volatile("v_lshl_add_u32 %0, %0, 2, %1" : "+v"(a) : "v"(b));
    if constexpr (OP == 7) asm volatile("v_and_b32_e32 %0, 0x7f7f7f7f, %0" : "+v"(a));  // VOP2 + 32-bit literal (8 bytes)
    if constexpr (OP == 8) asm volatile("v_xor_b32_e64 %0, %0, %1" : "+v"(a) : "v"(b));  // VOP2 op in the VOP3 encoding
    if constexpr (OP == 9) asm volatile("v_xor_b32_e32 %0, %1, %0" : "+v"(a) : "s"(s));  // VOP2, SGPR operand
    if constexpr (OP == 10) asm volatile("v_mul_u32_u24_e32 %0, %1, %0" : "+v"(a) : "v"(b));
    if constexpr (OP == 11) asm volatile("v_readlane_b32 %0, %1, 5" : "=s"(s) : "v"(a));
}

template <int OP>
__global__ void __launch_bounds__(256) rate_kernel(uint32_t *out, uint32_t seed, uint64_t *cyc) {
    uint32_t a[8];
    const uint32_t b = seed ^ threadIdx.x, c = seed * 3u + threadIdx.x;
    uint32_t s = seed * 5u;
#pragma unroll
    for (int i = 0; i < 8; i++) a[i] = threadIdx.x * (i + 1);
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < kIter; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) op<OP>(a[i], b, c, s);
#pragma unroll
        for (int i = 0; i < 8; i++) op<OP>(a[i], b, c, s);
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) x ^= a[i];
    x ^= s;
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
    if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

template <int OP>
static void run(const char *name, int W, uint32_t *d_out, uint64_t *d_cyc) {
    const int grid = 256 * W;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(rate_kernel<OP>, dim3(grid), dim3(256), 0, 0, d_out, 7u, d_cyc);  // warm
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(rate_kernel<OP>, dim3(grid), dim3(256), 0, 0, d_out, 9u, d_cyc);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    uint64_t cyc = 0;
    (void)hipMemcpy(&cyc, d_cyc, 8, hipMemcpyDeviceToHost);
    // instructions issued per SIMD: W waves per SIMD (4-wave groups spread over the 4 SIMDs)
    const double per_simd = (double)W * kIter * 16;
    printf("%-18s W=%d  %.3f ms  wave0 %.0f memtime ticks  %.2f ticks/instr/SIMD (wave0 span)  %.2f ns/instr/SIMD (wall)\n",
           name, W, ms, (double)cyc, (double)cyc / per_simd, ms * 1e6 / per_simd);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
}

int main() {
    uint32_t *d_out;
    uint64_t *d_cyc;
    if (hipMalloc(&d_out, 256 * 16 * 256 * 4) != hipSuccess || hipMalloc(&d_cyc, 8) != hipSuccess) return 1;
    int clk = 0;
    (void)hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
    printf("clock attribute %d kHz\n", clk);
    if (getenv("VALU_RATE_EXTRA")) {  // encodings: literal, VOP3-encoded VOP2, SGPR operand, readlane
        for (int W : {4, 8}) {
            run<0>("v_xor_b32", W, d_out, d_cyc);
            run<7>("v_and_b32 literal", W, d_out, d_cyc);
            run<8>("v_xor_b32_e64", W, d_out, d_cyc);
            run<9>("v_xor_b32 sgpr", W, d_out, d_cyc);
            run<10>("v_mul_u32_u24", W, d_out, d_cyc);
            run<11>("v_readlane_b32", W, d_out, d_cyc);
            run<1>("v_bitop3 vvv", W, d_out, d_cyc);
        }
        return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
    }
    for (int W : {1, 2, 4, 8}) {
        run<0>("v_xor_b32", W, d_out, d_cyc);
        run<1>("v_bitop3 vvv", W, d_out, d_cyc);
        run<2>("v_bitop3 vvs", W, d_out, d_cyc);
        run<3>("v_perm_b32", W, d_out, d_cyc);
        run<4>("v_pk_lshlrev_b16", W, d_out, d_cyc);
        run<5>("v_bfe_u32", W, d_out, d_cyc);
        run<6>("v_lshl_add_u32", W, d_out, d_cyc);
    }
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
