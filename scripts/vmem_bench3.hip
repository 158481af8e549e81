// vmem_bench3.hip -- access-order microbenchmark for the column-wave encode (not product code).
// Workgroup = G waves (one 64-word column group each) covering a stripe's full rows, walking
// the 100 planes in decode order; per plane 7 own + 10 partner word loads (aligned pairs) and
// 20 word stores, exactly the encode kernel's addresses, with no GF arithmetic.
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 -o scripts/vmem_bench3 scripts/vmem_bench3.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

struct Job { const uint8_t *src; uint8_t *dst; uint32_t src_len, rot, dst_skew, pad; };
struct Args { const Job *jobs; uint32_t G, wps, cs, sc, slen; };

__device__ __forceinline__ uint32_t xcd_tile(uint32_t b, uint32_t nb) {
    const uint32_t full = nb & ~7u;
    if (b >= full) return b;
    return (b & 7u) * (full >> 3) + (b >> 3);
}

// LD: 0 none, 1 own+partner, 2 own only.  ST: 0 none, 1 20 stores/plane.  LOCK: s_barrier/plane.
// PF: prefetch next plane's loads.  ORDER: 0 decode order (z0 outer), 1 plane index order.
template <int LD, int ST, bool LOCK, bool PF>
__global__ void __launch_bounds__(512) colwave(Args a) {
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const uint32_t job = xcd_tile(blockIdx.x, gridDim.x);
    const Job J = a.jobs[job];
    uint32_t w = wv * 64u + lane;
    if (w >= a.wps) w = a.wps - 1;
    const uint32_t col = w * 4u, cs = a.cs, sc = a.sc, slen = a.slen;
    const uint32_t src_al = (uint32_t)(uintptr_t)J.src & 3u;
    const __amdgpu_buffer_rsrc_t rs_src = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t *>(J.src - src_al), 0, (int)(J.src_len + src_al), 0x00020000);
    const __amdgpu_buffer_rsrc_t rs_dst =
        __builtin_amdgcn_make_buffer_rsrc(J.dst, 0, (int)(20 * slen - J.dst_skew), 0x00020000);
    const uint32_t dst_al = (uint32_t)(uintptr_t)J.dst & 3u;
    auto ld = [&](uint32_t o) -> uint32_t {
        const uint32_t lo = __builtin_amdgcn_raw_buffer_load_b32(rs_src, (int)(o & ~3u), 0, 0);
        const uint32_t hi = __builtin_amdgcn_raw_buffer_load_b32(rs_src, (int)((o & ~3u) + 4u), 0, 0);
        return __builtin_amdgcn_alignbyte(hi, lo, o & 3u);
    };
    uint32_t own[7], part[10];
    auto load = [&](uint32_t z0, uint32_t s) {
        const uint32_t z = z0 * 10 + s;
#pragma unroll
        for (int x = 0; x < 7; x++) own[x] = LD ? ld(src_al + x * cs + z * sc + col) : z + x;
#pragma unroll
        for (int x = 0; x < 10; x++)
            part[x] = LD == 1 ? ld(src_al + z0 * cs + (x * 10 + s) * sc + col) : x;
    };
    uint32_t acc = 0;
    if (PF) load(0, 0);
    for (uint32_t z0 = 0; z0 < 10; z0++) {
        for (uint32_t s = 0; s < 10; s++) {
            uint32_t co[7], cp[10];
            if (!PF) load(z0, s);
#pragma unroll
            for (int x = 0; x < 7; x++) co[x] = own[x];
#pragma unroll
            for (int x = 0; x < 10; x++) cp[x] = part[x];
            if (PF && z0 * 10 + s + 1 < 100) load(s + 1 < 10 ? z0 : z0 + 1, s + 1 < 10 ? s + 1 : 0);
            uint32_t u = 0;
#pragma unroll
            for (int x = 0; x < 7; x++) u ^= co[x];
#pragma unroll
            for (int x = 0; x < 10; x++) u ^= cp[x];
            acc += u;
            if (ST) {
                const uint32_t z = z0 * 10 + s;
#pragma unroll
                for (int r = 0; r < 20; r++) {
                    uint32_t sl = r + J.rot;
                    sl = sl >= 20 ? sl - 20 : sl;
                    const uint32_t off = sl * slen + z * sc;
                    const int vo = (int)(off + col);
                    if (((dst_al + off) & 3u) == 0) {
                        __builtin_amdgcn_raw_buffer_store_b32(u + r, rs_dst, vo, 0, 0);
                    } else {
                        __builtin_amdgcn_raw_buffer_store_b16((uint16_t)(u + r), rs_dst, vo, 0, 0);
                        __builtin_amdgcn_raw_buffer_store_b16((uint16_t)((u + r) >> 16), rs_dst, vo + 2, 0, 0);
                    }
                }
            }
            if (LOCK) __builtin_amdgcn_s_barrier();
        }
    }
    if (!ST && acc == 0x9e3779b9u) __builtin_amdgcn_raw_buffer_store_b32(acc, rs_dst, (int)col, 0, 0);
}

template <int LD, int ST, bool LOCK, bool PF>
float run(const Args &a, uint32_t blocks, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    hipLaunchKernelGGL((colwave<LD, ST, LOCK, PF>), dim3(blocks), dim3(a.G * 64), 0, 0, a);
    CK(hipEventRecord(e0, 0));
    for (int r = 0; r < reps; r++) hipLaunchKernelGGL((colwave<LD, ST, LOCK, PF>), dim3(blocks), dim3(a.G * 64), 0, 0, a);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    CK(hipGetLastError());
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
}

int main(int argc, char **argv) {
    const int nobj = argc > 1 ? atoi(argv[1]) : 1024;
    const size_t L = 4u << 20, S = 1000000, cs = 143000, sc = 1430, ns = 5, slen = ns * cs + 48;
    uint8_t *din, *dout;
    CK(hipMalloc(&din, nobj * L));
    CK(hipMalloc(&dout, nobj * 20 * slen));
    CK(hipMemset(din, 0x5a, nobj * L));
    std::vector<Job> jobs;
    for (int o = 0; o < nobj; o++)
        for (size_t s = 0; s < ns; s++)
            jobs.push_back(Job{din + (size_t)o * L + s * S, dout + (size_t)o * 20 * slen + s * cs,
                               (uint32_t)std::min<size_t>(S, L - s * S), (uint32_t)((s * 7) % 20), (uint32_t)(s * cs), 0});
    Job *dj;
    CK(hipMalloc(&dj, jobs.size() * sizeof(Job)));
    CK(hipMemcpy(dj, jobs.data(), jobs.size() * sizeof(Job), hipMemcpyHostToDevice));
    Args a{dj, 6, (uint32_t)((sc + 3) / 4), (uint32_t)cs, (uint32_t)sc, (uint32_t)slen};
    const uint32_t blocks = (uint32_t)jobs.size();
    const double rd = (double)nobj * L, wr = (double)nobj * 20.0 * slen;
    const int reps = 5;
    auto rep = [&](const char *name, float t, double b) { printf("%-40s %8.3f ms  %7.1f GB/s\n", name, t, b / t / 1e6); };
    rep("st only", run<0, 1, false, false>(a, blocks, reps), wr);
    rep("st only lockstep", run<0, 1, true, false>(a, blocks, reps), wr);
    rep("ld own+part, prefetch", run<1, 0, false, true>(a, blocks, reps), rd);
    rep("ld own+part, no prefetch", run<1, 0, false, false>(a, blocks, reps), rd);
    rep("ld own only, prefetch", run<2, 0, false, true>(a, blocks, reps), rd);
    rep("ld+st, prefetch", run<1, 1, false, true>(a, blocks, reps), rd + wr);
    rep("ld+st, prefetch, lockstep", run<1, 1, true, true>(a, blocks, reps), rd + wr);
    rep("ld own only + st, prefetch", run<2, 1, false, true>(a, blocks, reps), rd + wr);
    return 0;
}
