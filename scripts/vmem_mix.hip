// vmem_mix.hip -- microbenchmark (not product code): the encode kernels' memory skeleton without
// the GF arithmetic.  512 workgroups x 6 waves (two per CU); each walks 100 steps, per step
// loading 16 rows of 1,440 B (the plane image) and storing ~20 rows of 1,430 B (the flush),
// with the load path, source/destination alignment and ordering as template knobs.
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 scripts/vmem_mix.hip -o scripts/vmem_mix
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kSteps = 100, kRowsIn = 16, kRowsOut = 20, kRowB = 90;
constexpr uint32_t kRow = 1440, kSub = 1430;
constexpr uint32_t kStripeIn = 1100000;   // per-WG input region (>= 100 steps of distinct rows)
constexpr uint32_t kStripeOut = 3000000;  // per-WG output region

__device__ __forceinline__ u32x4 rsrc(const void *p, uint32_t nrec) {
    const uint64_t a = reinterpret_cast<uint64_t>(p);
    u32x4 r;
    r.x = __builtin_amdgcn_readfirstlane((uint32_t)a);
    r.y = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32) & 0xffffu);
    r.z = nrec;
    r.w = 0x00020000u;
    return r;
}
__device__ __forceinline__ void dma16(u32x4 rs, uint32_t voff, uint32_t soff, uint32_t lds) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(rs), "s"(lds), "s"(soff) : "memory");
}

// LOAD: 0 none, 1 LDS-DMA x4, 2 dword per lane to VGPRs (16 per wave, the stage kernel's shape),
//       3 dwordx4 to VGPRs + ds_write_b128.  AL: byte offset of rows (0 or 2).  ST: stores on.
template <int LOAD, int AL, bool ST>
__global__ void __launch_bounds__(384, 3) mix(const uint8_t *in, uint8_t *out) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const uint32_t lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint8_t *src = in + (size_t)blockIdx.x * kStripeIn;
    uint8_t *dst = out + (size_t)blockIdx.x * kStripeOut;
    const u32x4 rs = rsrc(src, kStripeIn);
    const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(src), 0, kStripeIn, 0x00020000);
    const __amdgpu_buffer_rsrc_t wb = __builtin_amdgcn_make_buffer_rsrc(dst, 0, kStripeOut, 0x00020000);
    const uint32_t slot_bytes = kRowsIn * kRow;
    const uint32_t lds0 = __builtin_amdgcn_groupstaticsize();
    uint32_t acc = 0;
    for (int t = 0; t < kSteps; t++) {
        const uint32_t slot = (t & 1) * slot_bytes;
        const uint32_t soff = AL + (uint32_t)t * kSub;  // rows advance one sub-chunk per step
        if constexpr (LOAD == 1) {
            for (uint32_t i = wv; i < (uint32_t)(kRowsIn * kRowB + 63) / 64; i += 6) {
                const uint32_t b = 64 * i + lane;
                const uint32_t ld = __builtin_amdgcn_readfirstlane(lds0 + slot + 1024u * i);
                if (b < (uint32_t)kRowsIn * kRowB) dma16(rs, (b / kRowB) * 60000u + (b % kRowB) * 16u, soff, ld);
            }
        } else if constexpr (LOAD == 2) {
            for (int r = 0; r < kRowsIn; r++) acc ^= __builtin_amdgcn_raw_buffer_load_b32(rb, (int)(r * 60000u + threadIdx.x * 4u), (int)soff, 0);
        } else if constexpr (LOAD == 3) {
            for (uint32_t i = wv; i < (uint32_t)(kRowsIn * kRowB + 63) / 64; i += 6) {
                const uint32_t b = 64 * i + lane;
                if (b < (uint32_t)kRowsIn * kRowB) {
                    u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rb, (int)((b / kRowB) * 60000u + (b % kRowB) * 16u), (int)soff, 0);
                    *reinterpret_cast<u32x4 *>(lds + slot + 16u * b) = v;
                }
            }
        }
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
        // flush: rows distributed over the waves, 16 B per lane, 2 instructions per row
        if constexpr (ST) {
            for (uint32_t r = wv; r < (uint32_t)kRowsOut; r += 6) {
                const uint8_t *row = lds + (r % kRowsIn) * kRow;
                const u32x4 d0 = *reinterpret_cast<const u32x4 *>(row + 16u * lane);
                const uint32_t o1 = lane < 25 ? 1024u + 16u * lane : (lane == 25 ? kSub - 16u : 0x80000000u);
                const u32x4 d1 = *reinterpret_cast<const u32x4 *>(row + (o1 & 0xffffu));
                const uint32_t base = AL + ((uint32_t)t * kRowsOut + r) * kSub;
                __builtin_amdgcn_raw_buffer_store_b128(d0, wb, (int)(16u * lane), (int)base, 2);
                __builtin_amdgcn_raw_buffer_store_b128(d1, wb, (int)o1, (int)base, 2);
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    if (acc == 0x12345678u) out[threadIdx.x] = 1;
}

// Store patterns only (no loads): PAT 0 = rows of 1,430 B at 1,430-B stride (2-aligned), 2 instr
// per row, rows round-robin over waves; 1 = same at 1,440-B stride (16-B aligned rows); 2 = each
// wave writes its rows as one contiguous run, 1 KiB per instruction (flattened); 3 = like 2 but
// the run starts 16-B aligned
template <int PAT>
__global__ void __launch_bounds__(384, 3) stpat(uint8_t *out) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const uint32_t lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint8_t *dst = out + (size_t)blockIdx.x * kStripeOut;
    const __amdgpu_buffer_rsrc_t wb = __builtin_amdgcn_make_buffer_rsrc(dst, 0, kStripeOut, 0x00020000);
    for (int t = 0; t < kSteps; t++) {
        if constexpr (PAT <= 1) {
            const uint32_t stride = PAT == 0 ? kSub : kRow;
            for (uint32_t r = wv; r < (uint32_t)kRowsOut; r += 6) {
                const uint8_t *row = lds + (r % kRowsIn) * kRow;
                const u32x4 d0 = *reinterpret_cast<const u32x4 *>(row + 16u * lane);
                const uint32_t o1 = lane < 25 ? 1024u + 16u * lane : (lane == 25 ? kSub - 16u : 0x80000000u);
                const u32x4 d1 = *reinterpret_cast<const u32x4 *>(row + (o1 & 0xffffu));
                const uint32_t base = ((uint32_t)t * kRowsOut + r) * stride;
                __builtin_amdgcn_raw_buffer_store_b128(d0, wb, (int)(16u * lane), (int)base, 2);
                __builtin_amdgcn_raw_buffer_store_b128(d1, wb, (int)o1, (int)base, 2);
            }
        } else {
            // this wave's share of the step's 20 rows as one run: 20*1430/6 = 4,767 B
            const uint32_t run = (kRowsOut * kSub) / 6, base = (uint32_t)t * kRowsOut * kSub + wv * run + (PAT == 3 ? 0 : 2);
            for (uint32_t o = 16u * lane; o < run; o += 1024u) {
                const u32x4 d = *reinterpret_cast<const u32x4 *>(lds + (o & 0x3fffu));
                __builtin_amdgcn_raw_buffer_store_b128(d, wb, (int)o, (int)(base & ~(PAT == 3 ? 15u : 0u)), 2);
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
}
template <int PAT>
float time_st(uint8_t *out, int nwg) {
    const size_t lds = 2 * kRowsIn * kRow;
    (void)hipFuncSetAttribute((const void *)stpat<PAT>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipEvent_t a, b;
    (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    hipLaunchKernelGGL(stpat<PAT>, dim3(nwg), dim3(384), lds, 0, out);
    float best = 1e9f;
    for (int r = 0; r < 5; r++) {
        (void)hipEventRecord(a, 0);
        for (int k = 0; k < 5; k++) hipLaunchKernelGGL(stpat<PAT>, dim3(nwg), dim3(384), lds, 0, out);
        (void)hipEventRecord(b, 0);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        best = ms / 5 < best ? ms / 5 : best;
    }
    return best;
}

template <int LOAD, int AL, bool ST>
float time_it(const uint8_t *in, uint8_t *out, int nwg) {
    const size_t lds = 2 * kRowsIn * kRow;
    (void)hipFuncSetAttribute((const void *)mix<LOAD, AL, ST>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipEvent_t a, b;
    (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    hipLaunchKernelGGL((mix<LOAD, AL, ST>), dim3(nwg), dim3(384), lds, 0, in, out);
    float best = 1e9f;
    for (int r = 0; r < 5; r++) {
        (void)hipEventRecord(a, 0);
        for (int k = 0; k < 5; k++) hipLaunchKernelGGL((mix<LOAD, AL, ST>), dim3(nwg), dim3(384), lds, 0, in, out);
        (void)hipEventRecord(b, 0);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        best = ms / 5 < best ? ms / 5 : best;
    }
    return best;
}

#define RUN(L, A, S, name)                                                                                     \
    do {                                                                                                       \
        const float ms = time_it<L, A, S>(in, out, nwg);                                                       \
        const double ld = (L ? (double)nwg * kSteps * kRowsIn * kRow : 0), st = S ? (double)nwg * kSteps * kRowsOut * kSub : 0; \
        printf("%-40s %7.3f ms  loads %6.1f GB/s  stores %6.1f GB/s  total %6.1f GB/s\n", name, ms, ld / ms / 1e6, st / ms / 1e6, (ld + st) / ms / 1e6); \
    } while (0)

int main(int argc, char **argv) {
    const int nwg = argc > 1 ? atoi(argv[1]) : 5120;
    uint8_t *in, *out;
    CK(hipMalloc(&in, (size_t)nwg * kStripeIn));
    CK(hipMalloc(&out, (size_t)nwg * kStripeOut));
    CK(hipMemset(in, 1, (size_t)nwg * kStripeIn));
    for (int p = 0; p < 4; p++) {
        const float ms = p == 0 ? time_st<0>(out, nwg) : p == 1 ? time_st<1>(out, nwg) : p == 2 ? time_st<2>(out, nwg) : time_st<3>(out, nwg);
        const double st = (double)nwg * kSteps * kRowsOut * kSub;
        printf("store pattern %d                          %7.3f ms  stores %6.1f GB/s\n", p, ms, st / ms / 1e6);
    }
    RUN(0, 0, true, "stores only, aligned");
    RUN(0, 2, true, "stores only, +2");
    RUN(1, 0, false, "dma only, aligned");
    RUN(1, 2, false, "dma only, +2");
    RUN(1, 0, true, "dma + stores, aligned");
    RUN(1, 2, true, "dma + stores, +2");
    RUN(2, 2, false, "dword loads only, +2");
    RUN(2, 2, true, "dword loads + stores, +2");
    RUN(3, 2, false, "x4 loads + ds_write, +2");
    RUN(3, 2, true, "x4 loads + ds_write + stores, +2");
    return 0;
}
