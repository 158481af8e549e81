// vmem_bench6.hip -- which store shapes keep HBM writes at streaming rate (not product code).
// Every variant writes the same 14.6 GB; each wave owns a contiguous 64 KB region (64 x 1 KB).
//   T1 full 128-B lines, one dwordx4 instruction per 1 KB (baseline)
//   T2 same wave, each line split over 2 instructions (first halves, then second halves)
//   T3 same wave, 8-B blocks interleaved over 3 dwordx2 instructions (24 B per lane)
//   T4 same wave, contiguous 1 KB per instruction but shifted by +2 B (lines split between
//      consecutive instructions)
//   T5 line halves from two different waves of the workgroup (same time)
//   T6 dwordx2 contiguous (512 B per instruction), aligned
//   T7 dword contiguous (256 B per instruction), aligned
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 -o scripts/vmem_bench6 scripts/vmem_bench6.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr uint32_t kRegion = 64 * 1024;  // bytes per wave

template <int T>
__global__ void __launch_bounds__(256) wr(uint8_t *base, uint32_t nwaves) {
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t gw = blockIdx.x * 4 + wv;
    if (gw >= nwaves) return;
    uint8_t *reg = base + (size_t)gw * kRegion;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(reg, 0, (int)(kRegion + 64), 0x00020000);
    const u32x4 v = {lane, gw, 1u, 2u};
    if constexpr (T == 1) {
        for (uint32_t k = 0; k < 64; k++) __builtin_amdgcn_raw_buffer_store_b128(v, rs, (int)(lane * 16), (int)(k * 1024), 0);
    } else if constexpr (T == 2) {
        // instr A: lane -> line lane/4, quarter (lane&3) of the first half... lane L writes 16 B at
        // line (L>>2), offset (L&3)*16  [first 64 B of 16 lines]; instr B the second 64 B.
        const uint32_t o = (lane >> 2) * 128 + (lane & 3) * 16;
        for (uint32_t k = 0; k < 64; k++) {
            __builtin_amdgcn_raw_buffer_store_b128(v, rs, (int)o, (int)(k * 2048), 0);
            __builtin_amdgcn_raw_buffer_store_b128(v, rs, (int)(o + 64), (int)(k * 2048), 0);
        }
    } else if constexpr (T == 3) {
        // 24 B per lane over 1536 B; instruction j writes 8-B block 3L+j
        for (uint32_t k = 0; k < 42; k++) {
#pragma unroll
            for (int j = 0; j < 3; j++)
                __builtin_amdgcn_raw_buffer_store_b64(u32x2{lane, (uint32_t)j}, rs, (int)(lane * 24 + j * 8), (int)(k * 1536), 0);
        }
    } else if constexpr (T == 4) {
        for (uint32_t k = 0; k < 64; k++) __builtin_amdgcn_raw_buffer_store_b128(v, rs, (int)(lane * 16 + 2), (int)(k * 1024), 0);
    } else if constexpr (T == 6) {
        for (uint32_t k = 0; k < 128; k++) __builtin_amdgcn_raw_buffer_store_b64(u32x2{lane, k}, rs, (int)(lane * 8), (int)(k * 512), 0);
    } else if constexpr (T == 7) {
        for (uint32_t k = 0; k < 256; k++) __builtin_amdgcn_raw_buffer_store_b32(lane ^ k, rs, (int)(lane * 4), (int)(k * 256), 0);
    }
}
// T5: wave pairs (0,1) and (2,3) share a 128 KB region; wave 0 writes the first half of every
// line, wave 1 the second half.
__global__ void __launch_bounds__(256) wr5(uint8_t *base, uint32_t nwaves) {
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t pair = blockIdx.x * 2 + (wv >> 1), half = wv & 1;
    if (pair * 2 >= nwaves) return;
    uint8_t *reg = base + (size_t)pair * 2 * kRegion;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(reg, 0, (int)(2 * kRegion), 0x00020000);
    const u32x4 v = {lane, pair, 1u, 2u};
    const uint32_t o = (lane >> 2) * 128 + (lane & 3) * 16 + half * 64;
    for (uint32_t k = 0; k < 128; k++) __builtin_amdgcn_raw_buffer_store_b128(v, rs, (int)o, (int)(k * 2048), 0);
}


// LDS unaligned access probe: ds_write_b64 / ds_read_b128 at 2-aligned addresses.
__global__ void lds_probe(uint32_t *out) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[4096];
    const uint32_t lane = threadIdx.x;
    for (uint32_t i = lane; i < 4096; i += 64) lds[i] = 0;
    __syncthreads();
    const uint32_t a = 2 + lane * 8;  // 2 mod 8
    const uint64_t v = 0x0807060504030201ull + lane * 0x1010101010101010ull;
    asm volatile("ds_write_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" :: "v"(a), "v"(v) : "memory");
    __syncthreads();
    uint32_t ok = 1;
    for (int b = 0; b < 8; b++) ok &= lds[a + b] == (uint8_t)(v >> (8 * b));
    u32x4 r;
    const uint32_t ra = 6 + lane * 16;  // 6 mod 16
    asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(ra) : "memory");
    uint32_t ok2 = 1;
    for (int b = 0; b < 16; b++) {
        const uint32_t w = b < 4 ? r.x : b < 8 ? r.y : b < 12 ? r.z : r.w;
        ok2 &= (uint8_t)(w >> (8 * (b & 3))) == lds[ra + b];
    }
    out[lane] = ok | (ok2 << 1);
}
// LDS write throughput: aligned vs 2-aligned ds_write_b64, 64 KB per wave pass
template <int MIS>
__global__ void __launch_bounds__(256) lds_wr(uint32_t *sink, int iters) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[65536 + 64];
    const uint32_t t = threadIdx.x;
    uint64_t v = t;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const uint32_t a = MIS + ((t * 8 + k * 2048 + it * 64) & 0xffff);
            asm volatile("ds_write_b64 %0, %1" :: "v"(a), "v"(v) : "memory");
            v += 3;
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
    if (lds[t * 7] == 0x77 && v == 5) sink[0] = 1;
}

template <typename F>
float timeit(F f, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    f();
    CK(hipEventRecord(e0, 0));
    for (int r = 0; r < reps; r++) f();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    CK(hipGetLastError());
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
}

int main() {
    const uint32_t nwaves = 224000;  // 14.7 GB
    const size_t bytes = (size_t)nwaves * kRegion;
    uint8_t *d;
    CK(hipMalloc(&d, bytes + 4096));
    const uint32_t blocks = (nwaves + 3) / 4;
    auto rep = [&](const char *name, float t, double b) { printf("%-52s %8.3f ms  %7.1f GB/s\n", name, t, b / t / 1e6); };
    rep("T1 full lines, 1 x4 instr per 1 KB", timeit([&] { hipLaunchKernelGGL(wr<1>, dim3(blocks), dim3(256), 0, 0, d, nwaves); }, 5), bytes);
    rep("T2 line halves, 2 instrs of one wave", timeit([&] { hipLaunchKernelGGL(wr<2>, dim3(blocks), dim3(256), 0, 0, d, nwaves); }, 5), bytes);
    rep("T3 8-B blocks interleaved over 3 x2 instrs", timeit([&] { hipLaunchKernelGGL(wr<3>, dim3(blocks), dim3(256), 0, 0, d, nwaves); }, 5), (double)nwaves * 42 * 1536);
    rep("T4 contiguous x4 shifted +2 B", timeit([&] { hipLaunchKernelGGL(wr<4>, dim3(blocks), dim3(256), 0, 0, d, nwaves); }, 5), bytes);
    rep("T5 line halves from two waves", timeit([&] { hipLaunchKernelGGL(wr5, dim3(blocks), dim3(256), 0, 0, d, nwaves); }, 5), bytes);
    rep("T6 contiguous x2 aligned", timeit([&] { hipLaunchKernelGGL(wr<6>, dim3(blocks), dim3(256), 0, 0, d, nwaves); }, 5), bytes);
    rep("T7 contiguous dword aligned", timeit([&] { hipLaunchKernelGGL(wr<7>, dim3(blocks), dim3(256), 0, 0, d, nwaves); }, 5), bytes);
    {
        uint32_t *o;
        CK(hipMalloc(&o, 256));
        hipLaunchKernelGGL(lds_probe, dim3(1), dim3(64), 0, 0, o);
        uint32_t h[64];
        CK(hipMemcpy(h, o, 256, hipMemcpyDeviceToHost));
        uint32_t all = 3;
        for (int i = 0; i < 64; i++) all &= h[i];
        printf("LDS unaligned: ds_write_b64 @2 mod 8 %s, ds_read_b128 @6 mod 16 %s\n", (all & 1) ? "OK" : "WRONG", (all & 2) ? "OK" : "WRONG");
        const int it = 4096;
        const double B = 2048.0 * 256 * 8 * 8 * it;  // blocks * thr * 8 writes * 8 B * iters
        rep("LDS ds_write_b64 aligned (2048 WGs)", timeit([&] { hipLaunchKernelGGL(lds_wr<0>, dim3(2048), dim3(256), 0, 0, o, it); }, 3), B);
        rep("LDS ds_write_b64 2-aligned (2048 WGs)", timeit([&] { hipLaunchKernelGGL(lds_wr<2>, dim3(2048), dim3(256), 0, 0, o, it); }, 3), B);
    }
    return 0;
}
