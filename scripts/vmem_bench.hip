// vmem_bench.hip -- memory-pattern microbenchmark for the encode kernel's access shape (not part
// of the product build).  Same grid, same addresses as enc_slab_kernel<7> over 1024 x 4 MiB
// objects, but no GF arithmetic: isolates what the loads/stores alone cost per variant.
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 -o scripts/vmem_bench scripts/vmem_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

struct Job { const uint8_t *src; uint8_t *dst; uint32_t src_len, rot, dst_skew, pad; };
struct Args { const Job *jobs; uint32_t gps, wps, cs, sc, slen; };

__device__ __forceinline__ uint32_t xcd_tile(uint32_t b, uint32_t nb) {
    const uint32_t full = nb & ~7u;
    if (b >= full) return b;
    return (b & 7u) * (full >> 3) + (b >> 3);
}

// LD: 0 = none, 1 = own+partner via 2 aligned dwords + alignbyte (production), 2 = same with
//     one unaligned dword, 3 = own only (unaligned dword), 4 = own+partner aligned-fake dword
// ST: 0 = none, 1 = production (b16 pairs on 2-mod-4 planes), 2 = unaligned b32,
//     3 = aligned-fake b32, 4 = unaligned b32 nontemporal
template <int LD, int ST>
__global__ void __launch_bounds__(640) pat_kernel(Args a) {
    const int slab = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const uint32_t tile = xcd_tile(blockIdx.x, gridDim.x);
    const uint32_t job = tile / a.gps, grp = tile - job * a.gps;
    uint32_t w = grp * 64u + lane;
    if (w >= a.wps) w = a.wps - 1;
    const Job J = a.jobs[job];
    const uint32_t col = w * 4u, cs = a.cs, sc = a.sc, slen = a.slen;
    const uint32_t src_al = (uint32_t)(uintptr_t)J.src & 3u;
    const __amdgpu_buffer_rsrc_t rs_src = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t *>(J.src - src_al), 0, (int)(J.src_len + src_al), 0x00020000);
    const __amdgpu_buffer_rsrc_t rs_dst =
        __builtin_amdgcn_make_buffer_rsrc(J.dst, 0, (int)(20 * slen - J.dst_skew), 0x00020000);
    const uint32_t dst_al = (uint32_t)(uintptr_t)J.dst & 3u;
    auto ld = [&](int x, uint32_t z) -> uint32_t {
        const uint32_t o = src_al + x * cs + z * sc + col;
        if constexpr (LD == 1) {
            const uint32_t lo = __builtin_amdgcn_raw_buffer_load_b32(rs_src, (int)(o & ~3u), 0, 0);
            const uint32_t hi = __builtin_amdgcn_raw_buffer_load_b32(rs_src, (int)((o & ~3u) + 4u), 0, 0);
            return __builtin_amdgcn_alignbyte(hi, lo, o & 3u);
        } else if constexpr (LD == 4) {
            return __builtin_amdgcn_raw_buffer_load_b32(rs_src, (int)(o & ~3u), 0, 0);
        } else {
            return __builtin_amdgcn_raw_buffer_load_b32(rs_src, (int)o, 0, 0);
        }
    };
    auto st = [&](int r, uint32_t z, uint32_t v) {
        uint32_t sl = (uint32_t)r + J.rot;
        sl = sl >= 20u ? sl - 20u : sl;
        const uint32_t off = sl * slen + z * sc;
        const uint32_t al = (dst_al + off) & 3u;
        const int vo = (int)(off + col);
        if constexpr (ST == 1) {
            if (al == 0) {
                __builtin_amdgcn_raw_buffer_store_b32(v, rs_dst, vo, 0, 0);
            } else {
                __builtin_amdgcn_raw_buffer_store_b16((uint16_t)v, rs_dst, vo, 0, 0);
                __builtin_amdgcn_raw_buffer_store_b16((uint16_t)(v >> 16), rs_dst, vo + 2, 0, 0);
            }
        } else if constexpr (ST == 2) {
            __builtin_amdgcn_raw_buffer_store_b32(v, rs_dst, vo, 0, 0);
        } else if constexpr (ST == 3) {
            __builtin_amdgcn_raw_buffer_store_b32(v, rs_dst, vo & ~3, 0, 0);
        } else if constexpr (ST == 4) {
            __builtin_amdgcn_raw_buffer_store_b32(v, rs_dst, vo, 0, 2);
        }
    };
    uint32_t acc = 0;
    for (int z0 = 0; z0 < 10; z0++) {
        const uint32_t z = (uint32_t)(z0 * 10 + slab);
        uint32_t own[7], part[10];
        if constexpr (LD != 0) {
#pragma unroll
            for (int x = 0; x < 7; x++) own[x] = ld(x, z);
            if constexpr (LD != 3) {
#pragma unroll
                for (int x = 0; x < 10; x++) part[x] = ld(z0, (uint32_t)(x * 10 + slab));
            } else {
#pragma unroll
                for (int x = 0; x < 10; x++) part[x] = 0;
            }
        } else {
#pragma unroll
            for (int x = 0; x < 7; x++) own[x] = z * 7 + x;
#pragma unroll
            for (int x = 0; x < 10; x++) part[x] = x;
        }
        uint32_t u = 0;
#pragma unroll
        for (int x = 0; x < 7; x++) u ^= own[x];
#pragma unroll
        for (int x = 0; x < 10; x++) u ^= part[x];
        if constexpr (ST != 0) {
#pragma unroll
            for (int r = 0; r < 20; r++) st(r, z, u + r);
        }
        acc += u;
    }
    if constexpr (ST == 0) {
        if (acc == 0x9e3779b9u) __builtin_amdgcn_raw_buffer_store_b32(acc, rs_dst, (int)col, 0, 0);
    }
}

// Streaming reference: read 4 MiB, write 14.3 MB per object, 16 B per lane.
__global__ void __launch_bounds__(256) stream_kernel(const uint4 *in, size_t nin, uint4 *out, size_t nout) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint4 acc = {0, 0, 0, 0};
    for (size_t j = i; j < nin; j += stride) {
        uint4 v = in[j];
        acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
    }
    for (size_t j = i; j < nout; j += stride) {
        uint4 v = {acc.x + (uint32_t)j, acc.y, acc.z, acc.w};
        out[j] = v;
    }
}

template <int LD, int ST>
float run(const Args &a, uint32_t blocks, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    hipLaunchKernelGGL((pat_kernel<LD, ST>), dim3(blocks), dim3(640), 0, 0, a);
    CK(hipEventRecord(e0, 0));
    for (int r = 0; r < reps; r++) hipLaunchKernelGGL((pat_kernel<LD, ST>), dim3(blocks), dim3(640), 0, 0, a);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipGetLastError());
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
        for (size_t s = 0; s < ns; s++) {
            Job j{};
            j.src = din + (size_t)o * L + s * S;
            j.src_len = (uint32_t)std::min<size_t>(S, L - s * S);
            j.dst = dout + (size_t)o * 20 * slen + s * cs;
            j.rot = (uint32_t)((s * 7) % 20);
            j.dst_skew = (uint32_t)(s * cs);
            jobs.push_back(j);
        }
    Job *dj;
    CK(hipMalloc(&dj, jobs.size() * sizeof(Job)));
    CK(hipMemcpy(dj, jobs.data(), jobs.size() * sizeof(Job), hipMemcpyHostToDevice));
    Args a{dj, 0, (uint32_t)((sc + 3) / 4), (uint32_t)cs, (uint32_t)sc, (uint32_t)slen};
    a.gps = (a.wps + 63) / 64;
    const uint32_t blocks = (uint32_t)jobs.size() * a.gps;
    const double rd = (double)nobj * L, wr = (double)nobj * 20.0 * slen;
    const int reps = 5;
    auto rep = [&](const char *name, float t, double bytes) {
        printf("%-44s %8.3f ms  %7.1f GB/s\n", name, t, bytes / t / 1e6);
    };
    {
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
        const size_t nin = nobj * L / 16, nout = (size_t)(wr / 16);
        hipLaunchKernelGGL(stream_kernel, dim3(256 * 8 * 4), dim3(256), 0, 0, (const uint4 *)din, nin, (uint4 *)dout, nout);
        CK(hipEventRecord(e0, 0));
        for (int r = 0; r < reps; r++)
            hipLaunchKernelGGL(stream_kernel, dim3(256 * 8 * 4), dim3(256), 0, 0, (const uint4 *)din, nin, (uint4 *)dout, nout);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        rep("stream x4 (read 4MiB + write 14.3MB /obj)", ms / reps, rd + wr);
    }
    rep("ld prod(2x aligned+alignbyte), no st", run<1, 0>(a, blocks, reps), rd);
    rep("ld unaligned dword, no st", run<2, 0>(a, blocks, reps), rd);
    rep("ld own-only unaligned, no st", run<3, 0>(a, blocks, reps), rd);
    rep("ld aligned-fake, no st", run<4, 0>(a, blocks, reps), rd);
    rep("st prod (b16 pairs), no ld", run<0, 1>(a, blocks, reps), wr);
    rep("st unaligned b32, no ld", run<0, 2>(a, blocks, reps), wr);
    rep("st aligned-fake b32, no ld", run<0, 3>(a, blocks, reps), wr);
    rep("st unaligned b32 nt, no ld", run<0, 4>(a, blocks, reps), wr);
    rep("prod ld + prod st", run<1, 1>(a, blocks, reps), rd + wr);
    rep("unaligned ld + unaligned st", run<2, 2>(a, blocks, reps), rd + wr);
    rep("own-only ld + unaligned st", run<3, 2>(a, blocks, reps), rd + wr);
    rep("aligned-fake ld + aligned-fake st", run<4, 3>(a, blocks, reps), rd + wr);
    rep("unaligned ld + unaligned st nt", run<2, 4>(a, blocks, reps), rd + wr);
    return 0;
}
