// vmem_ceiling.hip -- microbenchmark (not product code): the HBM ceiling for the encode's traffic
// mix, 4.29 GB read + 14.64 GB written (1024 x 4 MiB objects -> 20 x 715,048 B slices each),
// with loads and stores issued as independent, well-pipelined streams (no compute, no barriers).
// Calibrates what any encode traversal can reach once its excess traffic is gone.
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 -o scripts/vmem_ceiling scripts/vmem_ceiling.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Every workgroup owns one contiguous input range and one contiguous output range (as a stripe
// owns its object bytes and its slice chunks); per iteration a wave issues RL loads of 1 KiB and
// WL stores of 1 KiB (16 B per lane), loads summed into a sink so they are not dropped.
// ROWS: stores walk 1,430-byte rows (row start at any even address, lanes past the row's end
// dropped) instead of contiguous 1 KiB blocks.
template <int RL, int WL, bool ROWS, int AUX>
__global__ void __launch_bounds__(256) mix(const uint8_t *in, size_t in_per_wg, uint8_t *out, size_t out_per_wg,
                                           uint32_t *sink) {
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint8_t *src = in + (size_t)blockIdx.x * in_per_wg;
    uint8_t *dst = out + (size_t)blockIdx.x * out_per_wg;
    const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(src), 0, (int)in_per_wg, 0x00020000);
    const __amdgpu_buffer_rsrc_t wb = __builtin_amdgcn_make_buffer_rsrc(dst, 0, (int)out_per_wg, 0x00020000);
    const uint32_t nin = (uint32_t)(in_per_wg / 1024), nout = (uint32_t)(out_per_wg / (ROWS ? 1432 : 1024));
    const uint32_t iters = RL ? (nin + 4 * RL - 1) / (4 * RL) : (nout + 4 * WL - 1) / (4 * WL);
    u32x4 acc = {0, 0, 0, 0};
    const u32x4 v = {lane, wv, 7u, 9u};
    for (uint32_t it = 0; it < iters; it++) {
#pragma unroll
        for (int r = 0; r < RL; r++) {
            const uint32_t blk = (it * RL + r) * 4 + wv;
            if (blk < nin) acc ^= __builtin_amdgcn_raw_buffer_load_b128(rb, (int)(blk * 1024 + lane * 16), 0, AUX);
        }
        // stores: this iteration's share of the output, in proportion
        const uint32_t w0 = (uint32_t)((uint64_t)it * nout / iters), w1 = (uint32_t)((uint64_t)(it + 1) * nout / iters);
        for (uint32_t b = w0 + wv; b < w1; b += 4) {
            if constexpr (ROWS) {  // row b of 1,430 B: two instructions (1 KiB + 406 B)
                const uint32_t base = 2 + b * 1430u;
                __builtin_amdgcn_raw_buffer_store_b128(v, wb, (int)(lane * 16), (int)base, AUX);
                const uint32_t o1 = lane < 25 ? 1024u + 16u * lane : (lane == 25 ? 1430u - 16u : 0x80000000u);
                __builtin_amdgcn_raw_buffer_store_b128(v, wb, (int)o1, (int)base, AUX);
            } else {
                __builtin_amdgcn_raw_buffer_store_b128(v, wb, (int)(b * 1024 + lane * 16), 0, AUX);
            }
        }
    }
    if (acc.x == 0x12345678u && acc.y == 3u) sink[0] = acc.z;
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
    const size_t nobj = 1024, L = 4u << 20, slen = 5 * 143000 + 48;
    const size_t in_b = nobj * L, out_b = nobj * 20 * slen;
    uint8_t *din, *dout;
    uint32_t *sink;
    CK(hipMalloc(&din, in_b + (1 << 20)));
    CK(hipMalloc(&dout, out_b + (1 << 20)));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(din, 0x5a, in_b));
    auto rep = [&](const char *name, float t, double b) { printf("%-58s %8.3f ms  %7.1f GB/s\n", name, t, b / t / 1e6); };
    const double alg = (double)in_b + (double)out_b;
    for (int wgs : {1024, 2048, 5120}) {
        const size_t ipw = (in_b / wgs) & ~(size_t)1023, opw = (out_b / wgs) & ~(size_t)1023;
        char nm[128];
        snprintf(nm, sizeof nm, "mix 1:3.4 blocks, %d WGs x 256, default", wgs);
        rep(nm, timeit([&] { hipLaunchKernelGGL((mix<1, 4, false, 0>), dim3(wgs), dim3(256), 0, 0, din, ipw, dout, opw, sink); }, 5), alg);
        snprintf(nm, sizeof nm, "mix 1:3.4 blocks, %d WGs x 256, nt", wgs);
        rep(nm, timeit([&] { hipLaunchKernelGGL((mix<1, 4, false, 2>), dim3(wgs), dim3(256), 0, 0, din, ipw, dout, opw, sink); }, 5), alg);
        snprintf(nm, sizeof nm, "mix 1:3.4 ROWS of 1430 B, %d WGs x 256, nt", wgs);
        const size_t opr = out_b / wgs;
        rep(nm, timeit([&] { hipLaunchKernelGGL((mix<1, 4, true, 2>), dim3(wgs), dim3(256), 0, 0, din, ipw, dout, opr, sink); }, 5), alg);
        snprintf(nm, sizeof nm, "store only, %d WGs", wgs);
        rep(nm, timeit([&] { hipLaunchKernelGGL((mix<0, 4, false, 0>), dim3(wgs), dim3(256), 0, 0, din, ipw, dout, opw, sink); }, 5), (double)out_b);
        snprintf(nm, sizeof nm, "load only, %d WGs", wgs);
        rep(nm, timeit([&] { hipLaunchKernelGGL((mix<4, 0, false, 0>), dim3(wgs), dim3(256), 0, 0, din, ipw, dout, 0, sink); }, 5), (double)in_b);
    }
    rep("hipMemsetAsync (slices)", timeit([&] { (void)hipMemsetAsync(dout, 1, out_b, 0); }, 5), (double)out_b);
    rep("hipMemcpyAsync d2d (object bytes)", timeit([&] { (void)hipMemcpyAsync(dout, din, in_b, hipMemcpyDeviceToDevice, 0); }, 5), 2.0 * in_b);
    return 0;
}
