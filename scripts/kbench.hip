// kbench.hip -- microbenchmark of the encode kernel (not part of the product build).
// Times enc_stage_kernel<7> over a device-resident 1024 x 4 MiB batch and
// times each with hipEvents.  hipcc --offload-arch=gfx950 -O3 -std=c++20 -I tape_amd/csrc
#include "../tape_amd/csrc/encode_stage.hip"
#include "kbench_encode_dma.hip"
#include <cstdio>
#include <vector>
#include <map>
#include <algorithm>
using namespace tec;
namespace tec {  // the library's per-device helper (engine.cpp), single-device here
hipError_t ensure_dyn_lds(const void *fn, size_t bytes) {
    return hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}
}  // namespace tec

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void fill_random(uint32_t *p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint64_t z = (i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = (uint32_t)(z ^ (z >> 31));
    }
}

static bool g_dma = true;
static hipError_t launch_one(const EncArgs &a) { return g_dma ? launch_encode_dma(false, a, 0) : launch_stage<7, false>(a, 0); }
__global__ void diff_kernel(const uint32_t *x, const uint32_t *y, size_t n, unsigned long long *cnt) {
    unsigned long long c = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) c += x[i] != y[i];
    if (c) atomicAdd(cnt, c);
}
template <int MODE>
float run(const EncArgs &a, uint32_t, int reps) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    if (launch_one(a) != hipSuccess) printf("launch failed\n");
    (void)hipEventRecord(e0, 0);
    for (int r = 0; r < reps; r++) (void)launch_one(a);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (hipGetLastError() != hipSuccess) printf("launch error\n");
    return ms / reps;
}

int main(int argc, char **argv) {
    const int nobj = argc > 1 ? atoi(argv[1]) : 1024;
    const size_t L = 4u << 20, S = 1000000, cs = 143000, sc = 1430, ns = 5, slen = ns * cs + 48;
    uint8_t *din, *dout;
    CK(hipMalloc(&din, nobj * L));
    CK(hipMalloc(&dout, nobj * 20 * slen));
    if (argc > 2 && argv[2][0] == 'z') CK(hipMemset(din, 0x5a, nobj * L));
    else hipLaunchKernelGGL(fill_random, dim3(4096), dim3(256), 0, 0, (uint32_t *)din, nobj * L / 4);
    std::vector<EncJob> jobs;
    for (int o = 0; o < nobj; o++)
        for (size_t s = 0; s < ns; s++) {
            EncJob j{};
            j.store_mask = ~0u;
            j.src = din + (size_t)o * L + s * S;
            j.src_len = std::min<size_t>(S, L - s * S);
            j.dst = dout + (size_t)o * 20 * slen + s * cs;
            j.rot = (uint32_t)((s * 7) % 20);
            j.dst_skew = (uint32_t)(s * cs);
            jobs.push_back(j);
        }
    EncJob *dj;
    CK(hipMalloc(&dj, jobs.size() * sizeof(EncJob)));
    CK(hipMemcpy(dj, jobs.data(), jobs.size() * sizeof(EncJob), hipMemcpyHostToDevice));
    EncArgs a{};
    a.jobs = dj; a.njobs = (uint32_t)jobs.size(); a.words_per_stripe = (sc + 3) / 4;
    a.groups_per_stripe = (a.words_per_stripe + 63) / 64; a.cs = cs; a.sc = sc; a.slice_len = slen; a.n = 20;
    CK(hipMalloc(&a.scratch, encode_rows_scratch_bytes(a)));
    const uint32_t blocks = a.njobs * a.groups_per_stripe;
    const double alg = (double)nobj * (L + 20.0 * slen);
    const int reps = 5;
    float t;
    if (argc > 4 && argv[4][0] == 's') g_dma = false;
    {
        int nb_dma = -1, nb_stage = -1;
        (void)hipFuncSetAttribute((const void *)dma::enc_dma_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)dma::kLdsBytes);
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb_dma, dma::enc_dma_kernel<false>, dma::G * 64, dma::kLdsBytes);
        (void)hipFuncSetAttribute((const void *)stage::enc_stage_kernel<7, 6, false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)stage::lds_bytes(6));
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb_stage, stage::enc_stage_kernel<7, 6, false>, 384, stage::lds_bytes(6));
        printf("occupancy: dma %d WG/CU (lds %u), stage %d WG/CU (lds %zu)\n", nb_dma, dma::kLdsBytes, nb_stage, stage::lds_bytes(6));
    }
    if (argc > 3 && argv[3][0] == 'c') {  // check: dma kernel output == stage kernel output
        uint8_t *ref;
        const size_t outb = (size_t)nobj * 20 * slen;
        CK(hipMalloc(&ref, outb));
        CK(hipMemset(dout, 0, outb));
        CK(hipMemset(ref, 0, outb));
        CK((launch_stage<7, false>(a, 0)));
        CK(hipMemcpy(ref, dout, outb, hipMemcpyDeviceToDevice));
        CK(hipMemset(dout, 0, outb));
        CK(launch_encode_dma(false, a, 0));
        unsigned long long *cnt;
        CK(hipMalloc(&cnt, 8));
        CK(hipMemset(cnt, 0, 8));
        hipLaunchKernelGGL(diff_kernel, dim3(4096), dim3(256), 0, 0, (const uint32_t *)ref, (const uint32_t *)dout, outb / 4, cnt);
        unsigned long long h = 0;
        CK(hipMemcpy(&h, cnt, 8, hipMemcpyDeviceToHost));
        printf("check: dma vs stage differing words %llu of %zu\n", h, outb / 4);
        return h != 0;
    }
#ifdef TEC_DMA_CENSUS
    if (argc > 3 && argv[3][0] == 'o') {  // residency census of the DMA kernel
        CK(launch_encode_dma(false, a, 0));
        CK(hipDeviceSynchronize());
        std::vector<uint64_t> rec(3 * a.njobs);
        CK(hipMemcpy(rec.data(), a.scratch, rec.size() * 8, hipMemcpyDeviceToHost));
        // max concurrent workgroups per CU
        std::map<uint64_t, std::vector<std::pair<uint64_t, int>>> ev;
        for (uint32_t i = 0; i < a.njobs; i++) { ev[rec[3 * i]].push_back({rec[3 * i + 1], 1}); ev[rec[3 * i]].push_back({rec[3 * i + 2], -1}); }
        int maxc = 0; std::map<int, int> hist;
        for (auto &kv : ev) { auto v = kv.second; std::sort(v.begin(), v.end(), [](auto x, auto y) { return x.first < y.first || (x.first == y.first && x.second < y.second); });
            int c = 0, m = 0; for (auto &e : v) { c += e.second; m = std::max(m, c); } hist[m]++; maxc = std::max(maxc, m); }
        printf("census: %zu CUs used, max concurrent WGs per CU %d; histogram:", ev.size(), maxc);
        for (auto &h : hist) printf(" %d:%d", h.first, h.second);
        printf("\n");
        return 0;
    }
#endif
    if (argc > 3 && argv[3][0] == 'q') {  // quick: mode 0 only, best of 3
        float best = 1e9f;
        for (int i = 0; i < 5; i++) best = std::min(best, run<0>(a, blocks, 20));
        printf("%s full (best of 5x20) %8.3f ms  %7.1f GB/s\n", g_dma ? "dma  " : "stage", best, alg / best / 1e6);
        return 0;
    }
    t = run<0>(a, blocks, reps); printf("mode0 full            %8.3f ms  %7.1f GB/s\n", t, alg / t / 1e6);
    return 0;
}
