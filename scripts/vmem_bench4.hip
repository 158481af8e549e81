// vmem_bench4.hip -- access-width microbenchmark for the encode's HBM pattern (not product code).
// One workgroup per 1 MB stripe walks the 100 planes; per plane it reads the 7 data rows and/or
// writes the 20 output rows (1,430-byte rows, 2-aligned, rotated slices: the encode's exact
// addresses) with W bytes per lane.  ALIGNED: lanes move the 16-byte-aligned blocks covering the
// row instead (ceiling for an in-register realignment; edges overlap neighbours -- timing only).
// Also checks DPP wave_shl:1 semantics.
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 -o scripts/vmem_bench4 scripts/vmem_bench4.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct Job { const uint8_t *src; uint8_t *dst; uint32_t src_len, rot, dst_skew, pad; };
struct Args { const Job *jobs; uint32_t cs, sc, slen; };

__device__ __forceinline__ uint32_t xcd_tile(uint32_t b, uint32_t nb) {
    const uint32_t full = nb & ~7u;
    if (b >= full) return b;
    return (b & 7u) * (full >> 3) + (b >> 3);
}

template <int W>
__device__ __forceinline__ void st(__amdgpu_buffer_rsrc_t rs, int vo, int so, uint32_t v) {
    if constexpr (W == 4) __builtin_amdgcn_raw_buffer_store_b32(v, rs, vo, so, 0);
    if constexpr (W == 8) __builtin_amdgcn_raw_buffer_store_b64(u32x2{v, v + 1}, rs, vo, so, 0);
    if constexpr (W == 12) __builtin_amdgcn_raw_buffer_store_b96(u32x3{v, v + 1, v + 2}, rs, vo, so, 0);
    if constexpr (W == 16) __builtin_amdgcn_raw_buffer_store_b128(u32x4{v, v + 1, v + 2, v + 3}, rs, vo, so, 0);
}
template <int W>
__device__ __forceinline__ uint32_t ld(__amdgpu_buffer_rsrc_t rs, int vo, int so) {
    if constexpr (W == 4) return __builtin_amdgcn_raw_buffer_load_b32(rs, vo, so, 0);
    if constexpr (W == 8) { u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(rs, vo, so, 0); return v.x ^ v.y; }
    if constexpr (W == 12) { u32x3 v = __builtin_amdgcn_raw_buffer_load_b96(rs, vo, so, 0); return v.x ^ v.y ^ v.z; }
    if constexpr (W == 16) { u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, vo, so, 0); return v.x ^ v.y ^ v.z ^ v.w; }
}

// LD: 0 none, 1 the 7 data rows.  ST: 0 none, 1 the 20 output rows.
template <int W, bool ALIGNED, int LD, int ST>
__global__ void __launch_bounds__(512) rows(Args a) {
    const uint32_t lane = threadIdx.x;
    const uint32_t job = xcd_tile(blockIdx.x, gridDim.x);
    const Job J = a.jobs[job];
    const uint32_t cs = a.cs, sc = a.sc, slen = a.slen;
    const uint32_t per_row = (sc + W - 1) / W + (ALIGNED ? 1 : 0);
    if (lane >= per_row) return;
    const __amdgpu_buffer_rsrc_t rs_src = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(J.src), 0, (int)J.src_len, 0x00020000);
    const __amdgpu_buffer_rsrc_t rs_dst = __builtin_amdgcn_make_buffer_rsrc(J.dst, 0, (int)(20 * slen - J.dst_skew), 0x00020000);
    uint32_t acc = lane;
    for (uint32_t z = 0; z < 100; z++) {
        if (LD) {
#pragma unroll
            for (int x = 0; x < 7; x++) {
                uint32_t so = x * cs + z * sc;
                if (ALIGNED) so &= ~15u;
                acc ^= ld<W>(rs_src, (int)(lane * W), (int)so);
            }
        }
        if (ST) {
#pragma unroll
            for (int r = 0; r < 20; r++) {
                uint32_t sl = r + J.rot;
                sl = sl >= 20 ? sl - 20 : sl;
                uint32_t so = sl * slen + z * sc;
                if (ALIGNED) so &= ~15u;
                st<W>(rs_dst, (int)(lane * W), (int)so, acc + r);
            }
        }
        acc = acc * 3u + z;
    }
    if (!ST && acc == 0x9e3779b9u) __builtin_amdgcn_raw_buffer_store_b32(acc, rs_dst, (int)lane, 0, 0);
}

template <int W, bool ALIGNED, int LD, int ST>
float run(const Args &a, uint32_t blocks, int reps) {
    const uint32_t per_row = (a.sc + W - 1) / W + (ALIGNED ? 1 : 0);
    const uint32_t thr = (per_row + 63) / 64 * 64;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    hipLaunchKernelGGL((rows<W, ALIGNED, LD, ST>), dim3(blocks), dim3(thr), 0, 0, a);
    CK(hipEventRecord(e0, 0));
    for (int r = 0; r < reps; r++) hipLaunchKernelGGL((rows<W, ALIGNED, LD, ST>), dim3(blocks), dim3(thr), 0, 0, a);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    CK(hipGetLastError());
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
}

__global__ void dpp_probe(uint32_t *out) {
    const uint32_t v = threadIdx.x * 10u;
    out[threadIdx.x] = __builtin_amdgcn_mov_dpp(v, 0x130, 0xf, 0xf, false);        // wave_shl:1
    out[64 + threadIdx.x] = __builtin_amdgcn_mov_dpp(v, 0x138, 0xf, 0xf, false);   // wave_shr:1
    out[128 + threadIdx.x] = __builtin_amdgcn_update_dpp(7u, v, 0x130, 0xf, 0xf, false);  // wave_shl:1, old = 7
}

int main(int argc, char **argv) {
    const int nobj = argc > 1 ? atoi(argv[1]) : 1024;
    {
        uint32_t *d;
        CK(hipMalloc(&d, 192 * 4));
        hipLaunchKernelGGL(dpp_probe, dim3(1), dim3(64), 0, 0, d);
        uint32_t h[192];
        CK(hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost));
        printf("wave_shl:1 lanes 0,1,15,16,62,63: %u %u %u %u %u %u\n", h[0], h[1], h[15], h[16], h[62], h[63]);
        printf("wave_shr:1 lanes 0,1,15,16,62,63: %u %u %u %u %u %u\n", h[64], h[65], h[79], h[80], h[126], h[127]);
        printf("update wave_shl:1 old=7 lanes 0,62,63: %u %u %u\n", h[128], h[190], h[191]);
    }
    const size_t L = 4u << 20, S = 1000000, cs = 143000, sc = 1430, ns = 5, slen = ns * cs + 48;
    uint8_t *din, *dout;
    CK(hipMalloc(&din, nobj * L));
    CK(hipMalloc(&dout, nobj * 20 * slen + 64));
    CK(hipMemset(din, 0x5a, nobj * L));
    std::vector<Job> jobs;
    for (int o = 0; o < nobj; o++)
        for (size_t s = 0; s < ns; s++)
            jobs.push_back(Job{din + (size_t)o * L + s * S, dout + (size_t)o * 20 * slen + s * cs,
                               (uint32_t)std::min<size_t>(S, L - s * S), (uint32_t)((s * 7) % 20), (uint32_t)(s * cs), 0});
    Job *dj;
    CK(hipMalloc(&dj, jobs.size() * sizeof(Job)));
    CK(hipMemcpy(dj, jobs.data(), jobs.size() * sizeof(Job), hipMemcpyHostToDevice));
    Args a{dj, (uint32_t)cs, (uint32_t)sc, (uint32_t)slen};
    const uint32_t blocks = (uint32_t)jobs.size();
    const double rd = (double)nobj * L, wr = (double)nobj * 20.0 * slen;
    const int reps = 5;
    auto rep = [&](const char *name, float t, double b) { printf("%-34s %8.3f ms  %7.1f GB/s\n", name, t, b / t / 1e6); };
    rep("st  W4  unaligned", run<4, false, 0, 1>(a, blocks, reps), wr);
    rep("st  W8  unaligned", run<8, false, 0, 1>(a, blocks, reps), wr);
    rep("st  W12 unaligned", run<12, false, 0, 1>(a, blocks, reps), wr);
    rep("st  W16 unaligned", run<16, false, 0, 1>(a, blocks, reps), wr);
    rep("st  W16 aligned blocks", run<16, true, 0, 1>(a, blocks, reps), wr);
    rep("st  W8  aligned blocks", run<8, true, 0, 1>(a, blocks, reps), wr);
    rep("ld  W4  unaligned", run<4, false, 1, 0>(a, blocks, reps), rd);
    rep("ld  W8  unaligned", run<8, false, 1, 0>(a, blocks, reps), rd);
    rep("ld  W16 unaligned", run<16, false, 1, 0>(a, blocks, reps), rd);
    rep("ld  W16 aligned blocks", run<16, true, 1, 0>(a, blocks, reps), rd);
    rep("ld+st W4  unaligned", run<4, false, 1, 1>(a, blocks, reps), rd + wr);
    rep("ld+st W8  unaligned", run<8, false, 1, 1>(a, blocks, reps), rd + wr);
    rep("ld+st W12 unaligned", run<12, false, 1, 1>(a, blocks, reps), rd + wr);
    rep("ld+st W16 unaligned", run<16, false, 1, 1>(a, blocks, reps), rd + wr);
    rep("ld+st W16 aligned blocks", run<16, true, 1, 1>(a, blocks, reps), rd + wr);
    return 0;
}
