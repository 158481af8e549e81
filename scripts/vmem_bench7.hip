// vmem_bench7.hip -- encode output pattern with ONE wave per stripe (not product code).
// Per plane the wave writes each of the 20 rotated slices' rows itself, so the only lines split
// between instructions are (a) inside the row between its consecutive instructions and (b) at
// row boundaries, across plane steps.  RPS consecutive planes (RPS x 1,430 B) per step; PAD:
// rows padded to 1,536 B (every line whole -- control).
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 -o scripts/vmem_bench7 scripts/vmem_bench7.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t xcd_tile(uint32_t b, uint32_t nb) {
    const uint32_t full = nb & ~7u;
    if (b >= full) return b;
    return (b & 7u) * (full >> 3) + (b >> 3);
}

template <int RPS, bool PAD, int WPG>
__global__ void __launch_bounds__(64 * WPG) enc1(uint8_t *out, uint32_t nst) {
    constexpr uint32_t sc = PAD ? 1536 : 1430, cs = 100 * sc, slen = 5 * cs + (PAD ? 128 : 48);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t job = xcd_tile(blockIdx.x, gridDim.x) * WPG + (threadIdx.x >> 6);
    if (job >= nst) return;
    const uint32_t obj = job / 5, s = job - obj * 5;
    uint8_t *dst = out + (size_t)obj * 20 * slen + (size_t)s * cs;
    const uint32_t rot = (s * 7) % 20;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(dst, 0, (int)(20 * slen - s * cs), 0x00020000);
    constexpr uint32_t run = RPS * sc, ninstr = (run + 1023) / 1024;
    for (uint32_t z = 0; z < 100; z += RPS) {
#pragma unroll
        for (int r = 0; r < 20; r++) {
            uint32_t sl = r + rot;
            sl = sl >= 20 ? sl - 20 : sl;
            const uint32_t so = sl * slen + z * sc;
#pragma unroll
            for (uint32_t k = 0; k < ninstr; k++) {
                const uint32_t b = k * 1024 + lane * 16;
                if (b < run) __builtin_amdgcn_raw_buffer_store_b128(u32x4{z, (uint32_t)r, lane, k}, rs, (int)b, (int)so, 0);
            }
        }
    }
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
    const uint32_t nobj = 1024, nst = nobj * 5;
    uint8_t *d;
    CK(hipMalloc(&d, (size_t)nobj * 20 * (5 * 153600 + 128) + 4096));
    const double B = (double)nobj * 20 * (5 * 143000 + 48);
    auto rep = [&](const char *name, float t, double b) { printf("%-50s %8.3f ms  %7.1f GB/s\n", name, t, b / t / 1e6); };
    rep("1 wave/stripe, 1 plane/step", timeit([&] { hipLaunchKernelGGL((enc1<1, false, 1>), dim3(nst), dim3(64), 0, 0, d, nst); }, 5), B);
    rep("1 wave/stripe, 1 plane/step, 4 waves/WG", timeit([&] { hipLaunchKernelGGL((enc1<1, false, 4>), dim3(nst / 4), dim3(256), 0, 0, d, nst); }, 5), B);
    rep("1 wave/stripe, 2 planes/step", timeit([&] { hipLaunchKernelGGL((enc1<2, false, 1>), dim3(nst), dim3(64), 0, 0, d, nst); }, 5), B);
    rep("1 wave/stripe, 4 planes/step", timeit([&] { hipLaunchKernelGGL((enc1<4, false, 1>), dim3(nst), dim3(64), 0, 0, d, nst); }, 5), B);
    rep("1 wave/stripe, 10 planes/step", timeit([&] { hipLaunchKernelGGL((enc1<10, false, 1>), dim3(nst), dim3(64), 0, 0, d, nst); }, 5), B);
    rep("1 wave/stripe, 1 plane/step, PADDED rows", timeit([&] { hipLaunchKernelGGL((enc1<1, true, 1>), dim3(nst), dim3(64), 0, 0, d, nst); }, 5), B * 1536 / 1430);
    return 0;
}
