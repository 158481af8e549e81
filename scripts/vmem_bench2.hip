// vmem_bench2.hip -- store-pattern microbenchmark (not part of the product build).
// All variants write the encode output of 1024 x 4 MiB objects (20 slices x 715,048 B per
// object, sub-chunk 1,430 B, rotated) and differ only in how the writes are shaped:
//   piece  = contiguous bytes one wave-instruction writes (lanes x bytes/lane)
//   order  = which (node, plane, column-range) each workgroup covers
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 -o scripts/vmem_bench2 scripts/vmem_bench2.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

struct Job { uint8_t *dst; uint32_t rot, dst_skew; };

__device__ __forceinline__ uint32_t xcd_tile(uint32_t b, uint32_t nb) {
    const uint32_t full = nb & ~7u;
    if (b >= full) return b;
    return (b & 7u) * (full >> 3) + (b >> 3);
}

__device__ __forceinline__ uint32_t mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return (uint32_t)(z ^ (z >> 31));
}
// Slab-order stores like enc_slab_kernel: WG = 10 waves (slabs) x 64 lanes, lane = W bytes,
// workgroup covers 64*W columns of every plane; step z0 writes planes z0*10+s for 20 nodes.
// SC = sub-chunk stride (1430 real; 1536 = line-aligned rows, output buffer sized for it).
template <int W, int SC, bool XCD>
__global__ void __launch_bounds__(640) slab_store(const Job *jobs, uint32_t gps, uint32_t slen, uint32_t cs) {
    const int slab = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const uint32_t tile = XCD ? xcd_tile(blockIdx.x, gridDim.x) : blockIdx.x;
    const uint32_t job = tile / gps, grp = tile - job * gps;
    const Job J = jobs[job];
    const uint32_t col = (grp * 64u + lane) * W;
    const bool live = col < 1430u;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(J.dst, 0, (int)(20 * slen - J.dst_skew), 0x00020000);
    for (int z0 = 0; z0 < 10; z0++) {
        const uint32_t z = z0 * 10 + slab;
#pragma unroll
        for (int r = 0; r < 20; r++) {
            uint32_t sl = r + J.rot;
            sl = sl >= 20 ? sl - 20 : sl;
            const int vo = live ? (int)(sl * slen + z * SC + col) : (int)0x80000000;
            const uint32_t v = mix(((uint64_t)job << 32) ^ (z * 131 + r) ^ ((uint64_t)col << 12));
            if constexpr (W == 4) __builtin_amdgcn_raw_buffer_store_b32(v, rs, vo, 0, 0);
            if constexpr (W == 8) {
                typedef uint32_t v2 __attribute__((ext_vector_type(2)));
                v2 d = {v, v + 1};
                __builtin_amdgcn_raw_buffer_store_b64(d, rs, vo, 0, 0);
            }
            if constexpr (W == 16) {
                typedef uint32_t v4 __attribute__((ext_vector_type(4)));
                v4 d = {v, v + 1, v + 2, v + 3};
                __builtin_amdgcn_raw_buffer_store_b128(d, rs, vo, 0, 0);
            }
        }
    }
}

// Row order: each wave writes whole 1430-B sub-chunk rows (node r, plane z) with W bytes/lane,
// a workgroup owns one stripe x 10 planes (z0 fixed) -> rows of all 20 nodes.
template <int W>
__global__ void __launch_bounds__(640) row_store(const Job *jobs, uint32_t slen, uint32_t cs) {
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const uint32_t tile = xcd_tile(blockIdx.x, gridDim.x);
    const uint32_t job = tile / 10, z0 = tile - job * 10;
    const Job J = jobs[job];
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(J.dst, 0, (int)(20 * slen - J.dst_skew), 0x00020000);
    // 200 rows (20 nodes x 10 planes) over 10 waves
    for (int i = wv; i < 200; i += 10) {
        const uint32_t r = i / 10, z = z0 * 10 + (i % 10);
        uint32_t sl = r + J.rot;
        sl = sl >= 20 ? sl - 20 : sl;
        const uint32_t base = sl * slen + z * 1430u;
        for (uint32_t c = lane * W; c < 1430u; c += 64 * W) {
            const uint32_t v = mix(((uint64_t)job << 32) ^ (z * 131 + r) ^ ((uint64_t)(c + lane * W) << 12));
            const int vo = (int)(base + c);
            if constexpr (W == 4) __builtin_amdgcn_raw_buffer_store_b32(v, rs, vo, 0, 0);
            if constexpr (W == 16) {
                typedef uint32_t v4 __attribute__((ext_vector_type(4)));
                v4 d = {v, v + 1, v + 2, v + 3};
                __builtin_amdgcn_raw_buffer_store_b128(d, rs, c + 16 <= 1430u ? vo : (int)0x80000000, 0, 0);
            }
        }
    }
}

// Linear write of the same byte count (reference); RND: random payload instead of a counter.
template <bool RND>
__global__ void __launch_bounds__(256) lin_store(uint4 *out, size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += stride) {
        uint4 v = {(uint32_t)j, 1, 2, 3};
        if (RND) v = {mix(4 * j), mix(4 * j + 1), mix(4 * j + 2), mix(4 * j + 3)};
        out[j] = v;
    }
}
// Linear read (reference): XOR-reduce, one store per thread.
__global__ void __launch_bounds__(256) lin_load(const uint4 *in, size_t n, uint32_t *sink) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    uint32_t acc = 0;
    for (size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += stride) {
        uint4 v = in[j];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

template <class F>
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
    const size_t cs = 143000, ns = 5, slen = ns * cs + 48;
    const size_t cs_al = 1536 * 100, slen_al = ns * cs_al + 48;
    uint8_t *dout;
    CK(hipMalloc(&dout, nobj * 20 * slen_al));
    auto mk = [&](size_t c, size_t sl) {
        std::vector<Job> jobs;
        for (int o = 0; o < nobj; o++)
            for (size_t s = 0; s < ns; s++)
                jobs.push_back(Job{dout + (size_t)o * 20 * sl + s * c, (uint32_t)((s * 7) % 20), (uint32_t)(s * c)});
        Job *dj;
        CK(hipMalloc(&dj, jobs.size() * sizeof(Job)));
        CK(hipMemcpy(dj, jobs.data(), jobs.size() * sizeof(Job), hipMemcpyHostToDevice));
        return dj;
    };
    Job *jr = mk(cs, slen), *ja = mk(cs_al, slen_al);
    const uint32_t nj = nobj * ns;
    const double wr = (double)nobj * 20.0 * ns * cs;
    const int reps = 5;
    auto rep = [&](const char *name, float t) { printf("%-52s %8.3f ms  %7.1f GB/s\n", name, t, wr / t / 1e6); };
    rep("linear dwordx4 (same bytes), counter data", timeit([&] { hipLaunchKernelGGL(lin_store<false>, dim3(8192), dim3(256), 0, 0, (uint4 *)dout, (size_t)(wr / 16)); }, reps));
    rep("linear dwordx4 (same bytes), random data", timeit([&] { hipLaunchKernelGGL(lin_store<true>, dim3(8192), dim3(256), 0, 0, (uint4 *)dout, (size_t)(wr / 16)); }, reps));
    rep("linear read x4 of the written bytes (random)", timeit([&] { hipLaunchKernelGGL(lin_load, dim3(8192), dim3(256), 0, 0, (const uint4 *)dout, (size_t)(wr / 16), (uint32_t *)dout); }, reps));
    rep("slab b32 (256B pieces), sc 1430, xcd", timeit([&] { hipLaunchKernelGGL((slab_store<4, 1430, true>), dim3(nj * 6), dim3(640), 0, 0, jr, 6u, (uint32_t)slen, (uint32_t)cs); }, reps));
    rep("slab b32 (256B pieces), sc 1430, no xcd", timeit([&] { hipLaunchKernelGGL((slab_store<4, 1430, false>), dim3(nj * 6), dim3(640), 0, 0, jr, 6u, (uint32_t)slen, (uint32_t)cs); }, reps));
    rep("slab b32 (256B pieces), rows line-aligned (1536)", timeit([&] { hipLaunchKernelGGL((slab_store<4, 1536, true>), dim3(nj * 6), dim3(640), 0, 0, ja, 6u, (uint32_t)slen_al, (uint32_t)cs_al); }, reps));
    rep("slab b64 (512B pieces), sc 1430", timeit([&] { hipLaunchKernelGGL((slab_store<8, 1430, true>), dim3(nj * 3), dim3(640), 0, 0, jr, 3u, (uint32_t)slen, (uint32_t)cs); }, reps));
    rep("slab b128 (1KB pieces), sc 1430 (unaligned)", timeit([&] { hipLaunchKernelGGL((slab_store<16, 1430, true>), dim3(nj * 2), dim3(640), 0, 0, jr, 2u, (uint32_t)slen, (uint32_t)cs); }, reps));
    rep("slab b128 (1KB pieces), rows line-aligned (1536)", timeit([&] { hipLaunchKernelGGL((slab_store<16, 1536, true>), dim3(nj * 2), dim3(640), 0, 0, ja, 2u, (uint32_t)slen_al, (uint32_t)cs_al); }, reps));
    rep("row order b32 (whole 1430B rows)", timeit([&] { hipLaunchKernelGGL((row_store<4>), dim3(nj * 10), dim3(640), 0, 0, jr, (uint32_t)slen, (uint32_t)cs); }, reps));
    rep("row order b128 (whole rows, 16B/lane)", timeit([&] { hipLaunchKernelGGL((row_store<16>), dim3(nj * 10), dim3(640), 0, 0, jr, (uint32_t)slen, (uint32_t)cs); }, reps));
    return 0;
}
