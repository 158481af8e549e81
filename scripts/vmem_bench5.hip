// vmem_bench5.hip -- HBM write-ceiling microbenchmark for the encode (not product code).
// Calibrates what the output side (14.6 GB of slices per 1024 x 4 MiB objects) can reach:
// streaming stores vs the encode's 20-rows-per-plane pattern, row alignment, rows per step,
// cache policy and waves per CU.
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 -o scripts/vmem_bench5 scripts/vmem_bench5.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t xcd_tile(uint32_t b, uint32_t nb) {
    const uint32_t full = nb & ~7u;
    if (b >= full) return b;
    return (b & 7u) * (full >> 3) + (b >> 3);
}

// grid-stride streaming store of n16 16-byte blocks
template <int AUX>
__global__ void __launch_bounds__(256) stream_st(uint8_t *p, size_t n16) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(p, 0, 0x7fffffff, 0x00020000);
    (void)rs;
    u32x4 *q = (u32x4 *)p;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
        u32x4 v = {(uint32_t)i, 1u, 2u, 3u};
        if constexpr (AUX == 0) q[i] = v;
        else __builtin_nontemporal_store(v, q + i);
    }
}
__global__ void __launch_bounds__(256) stream_ld(const uint8_t *p, size_t n16, uint32_t *sink) {
    const u32x4 *q = (const u32x4 *)p;
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
        u32x4 v = q[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}
// streaming copy-shaped: each thread reads 1 block and writes 3.4 blocks (encode's 4.3 : 14.6)
__global__ void __launch_bounds__(256) stream_mix(const uint8_t *src, size_t n16in, uint8_t *dst, size_t n16out) {
    const u32x4 *q = (const u32x4 *)src;
    u32x4 *o = (u32x4 *)dst;
    const size_t T = (size_t)gridDim.x * blockDim.x, t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    const size_t iters = (n16in + T - 1) / T;
    const size_t per = (n16out + iters * T - 1) / (iters * T);  // writes per read
    for (size_t it = 0; it < iters; it++) {
        const size_t i = it * T + t;
        u32x4 v = i < n16in ? q[i] : u32x4{0, 0, 0, 0};
        for (size_t k = 0; k < per; k++) {
            const size_t j = (it * per + k) * T + t;
            if (j < n16out) o[j] = v + (uint32_t)k;
        }
    }
}

struct Args { uint8_t *dst; uint32_t nstripes, cs, sc, slen, rows_per_step; };
// encode output pattern: WG per stripe, 100 planes, 20 rotated slices; W16 unaligned stores;
// rows_per_step consecutive planes written per step (one run of rows_per_step*sc bytes per slice)
template <int AUX>
__global__ void __launch_bounds__(512) enc_st(Args a) {
    const uint32_t job = xcd_tile(blockIdx.x, gridDim.x);
    const uint32_t obj = job / 5, s = job - obj * 5;
    uint8_t *dst = a.dst + (size_t)obj * 20 * a.slen + (size_t)s * a.cs;
    const uint32_t rot = (s * 7) % 20;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(dst, 0, (int)(20 * a.slen - s * a.cs), 0x00020000);
    const uint32_t run = a.rows_per_step * a.sc, lanes = (run + 15) / 16;
    for (uint32_t z = 0; z < 100; z += a.rows_per_step) {
        for (uint32_t l = threadIdx.x; l < lanes; l += blockDim.x) {
#pragma unroll
            for (int r = 0; r < 20; r++) {
                uint32_t sl = r + rot;
                sl = sl >= 20 ? sl - 20 : sl;
                const uint32_t so = sl * a.slen + z * a.sc;
                const uint32_t b = l * 16u;
                if (b + 16 <= run)
                    __builtin_amdgcn_raw_buffer_store_b128(u32x4{z, (uint32_t)r, l, 7u}, rs, (int)b, (int)so, AUX);
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

int main(int argc, char **argv) {
    const int nobj = argc > 1 ? atoi(argv[1]) : 1024;
    const size_t L = 4u << 20, cs = 143000, sc = 1430, slen = 5 * cs + 48;
    const size_t out_bytes = (size_t)nobj * 20 * slen, in_bytes = (size_t)nobj * L;
    uint8_t *din, *dout;
    uint32_t *sink;
    CK(hipMalloc(&din, in_bytes));
    CK(hipMalloc(&dout, (size_t)nobj * 20 * (5 * 100 * 1536 + 128) + 4096));  // room for padded rows
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(din, 0x5a, in_bytes));
    const int reps = 5;
    auto rep = [&](const char *name, float t, double b) { printf("%-46s %8.3f ms  %7.1f GB/s\n", name, t, b / t / 1e6); };
    const size_t n16o = out_bytes / 16, n16i = in_bytes / 16;
    for (int g : {1024, 4096, 16384}) {
        char nm[64];
        snprintf(nm, sizeof nm, "stream store x4, grid %d x 256", g);
        rep(nm, timeit([&] { hipLaunchKernelGGL(stream_st<0>, dim3(g), dim3(256), 0, 0, dout, n16o); }, reps), (double)out_bytes);
    }
    rep("stream store x4 nontemporal, grid 4096", timeit([&] { hipLaunchKernelGGL(stream_st<1>, dim3(4096), dim3(256), 0, 0, dout, n16o); }, reps), (double)out_bytes);
    rep("hipMemsetAsync", timeit([&] { (void)hipMemsetAsync(dout, 1, out_bytes, 0); }, reps), (double)out_bytes);
    rep("stream load x4, grid 4096", timeit([&] { hipLaunchKernelGGL(stream_ld, dim3(4096), dim3(256), 0, 0, din, n16i, sink); }, reps), (double)in_bytes);
    rep("stream mix 1 read : 3.4 writes, grid 4096", timeit([&] { hipLaunchKernelGGL(stream_mix, dim3(4096), dim3(256), 0, 0, din, n16i, dout, n16o); }, reps), (double)(in_bytes + out_bytes));
    rep("hipMemcpyAsync d2d (in bytes)", timeit([&] { (void)hipMemcpyAsync(dout, din, in_bytes, hipMemcpyDeviceToDevice, 0); }, reps), 2.0 * in_bytes);
    const uint32_t nst = nobj * 5;
    for (uint32_t rps : {1u, 2u, 4u, 5u, 10u}) {
        for (uint32_t thr : {128u, 256u, 512u}) {
            Args a{dout, nst, (uint32_t)cs, (uint32_t)sc, (uint32_t)slen, rps};
            char nm[96];
            snprintf(nm, sizeof nm, "enc pattern x4, %u planes/step, %u thr/WG", rps, thr);
            rep(nm, timeit([&] { hipLaunchKernelGGL(enc_st<0>, dim3(nst), dim3(thr), 0, 0, a); }, reps), (double)out_bytes);
        }
    }
    {
        Args a{dout, nst, (uint32_t)cs, (uint32_t)sc, (uint32_t)slen, 1};
        rep("enc pattern x4, 1 plane/step, nt (aux 2)", timeit([&] { hipLaunchKernelGGL(enc_st<2>, dim3(nst), dim3(128), 0, 0, a); }, reps), (double)out_bytes);
        Args b{dout, nst, (uint32_t)(100 * 1536), 1536, (uint32_t)(5 * 100 * 1536 + 128), 1};
        rep("enc pattern x4, rows padded to 1536 B", timeit([&] { hipLaunchKernelGGL(enc_st<0>, dim3(nst), dim3(128), 0, 0, b); }, reps), (double)out_bytes * 1536 / 1430);
    }
    return 0;
}
