// enc_skeleton2.hip -- microbenchmark (not product code): the encode's memory traffic shape with
// no arithmetic, second series.  Question: is the row-store cost the bytes, the junction lines or
// the number of (partly empty) store instructions?  A 1,430-byte row is 89.4 16-byte blocks: one
// wave storing it whole issues a full 1 KiB instruction and a 26-lane one.  "Packed" stores give
// each wave-instruction 64 consecutive blocks of the plane's concatenated rows (as the DMA loads
// already do), so a plane of 20 rows is 28 instructions instead of 40.
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 -o scripts/enc_skeleton2 scripts/enc_skeleton2.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr uint32_t SC = 1430, CS = 100 * SC, SLEN = 5 * CS + 48, NOBJ = 1024, NST = 5;
constexpr uint32_t OBJ = 4u << 20;
constexpr uint32_t NB = (SC + 15) / 16;  // 90 blocks per row, the last one overlapping

// P planes per store batch (rows of P consecutive planes form one piece per chunk);
// NPART partner rows per plane; PACK: packed store instructions; LPACK: packed loads.
template <int P, int NPART, bool PACK, bool LPACK, int NW = 6>
__global__ void __launch_bounds__(768) skel(const uint8_t *in, uint8_t *out, uint32_t *sink) {
    extern __shared__ uint32_t lds[];
    const uint32_t lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t job = blockIdx.x, obj = job / NST, st = job % NST;
    const uint8_t *src = in + (size_t)obj * OBJ + (size_t)st * 7 * CS;
    const uint32_t src_len = st + 1 < NST ? 7 * CS : OBJ - (NST - 1) * 7 * CS;
    uint8_t *dst = out + (size_t)obj * 20 * SLEN + (size_t)st * CS;
    const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(src), 0, (int)src_len, 0x00020000);
    const __amdgpu_buffer_rsrc_t wb = __builtin_amdgcn_make_buffer_rsrc(dst, 0, (int)(19 * SLEN + CS), 0x00020000);
    u32x4 acc = {0, 0, 0, 0};
    const u32x4 v = {lane, wv, 7u, 9u};
    constexpr uint32_t NLOAD = 7 + NPART;
    constexpr uint32_t PL = P * SC;                 // piece bytes per chunk
    constexpr uint32_t PB = (PL + 15) / 16;         // blocks per piece (last one overlapping)
    for (uint32_t z = 0; z < 100; z++) {
        const uint32_t z0 = z / 10, s = z % 10;
        auto row_off = [&](uint32_t r) -> uint32_t {
            return r < 7 ? r * CS + z * SC : (z0 < 7 ? z0 : 0) * CS + ((r - 7) * 10 + s) * SC;
        };
        if (LPACK) {
            constexpr uint32_t NI = (NLOAD * NB + 63) / 64;
            for (uint32_t i = wv; i < NI; i += NW) {
                const uint32_t b = 64 * i + lane, r = b / NB, k = b - r * NB;
                const uint32_t o = r < NLOAD ? row_off(r) + (k * 16 + 16 <= SC ? k * 16 : SC - 16) : 0x80000000u;
                acc ^= __builtin_amdgcn_raw_buffer_load_b128(rb, (int)o, 0, 0);
            }
        } else {
            for (uint32_t r = wv; r < NLOAD; r += NW) {
                const uint32_t off = row_off(r);
#pragma unroll
                for (uint32_t k = 0; k < 2; k++) {
                    const uint32_t bk = k * 64 + lane;
                    const uint32_t o = bk < NB ? (bk * 16 + 16 <= SC ? bk * 16 : SC - 16) : 0x80000000u;
                    acc ^= __builtin_amdgcn_raw_buffer_load_b128(rb, (int)o, (int)off, 0);
                }
            }
        }
        __syncthreads();
        if ((z + 1) % P == 0) {
            const uint32_t zb = z + 1 - P;
            if (PACK) {
                constexpr uint32_t NI = (20 * PB + 63) / 64;
                for (uint32_t i = wv; i < NI; i += NW) {
                    const uint32_t b = 64 * i + lane, c = b / PB, k = b - c * PB;
                    const uint32_t o = c < 20 ? c * SLEN + zb * SC + (k * 16 + 16 <= PL ? k * 16 : PL - 16) : 0x80000000u;
                    __builtin_amdgcn_raw_buffer_store_b128(v, wb, (int)o, 0, 2);
                }
            } else {
                constexpr uint32_t PI = (PB + 63) / 64;
                for (uint32_t c = wv; c < 20; c += NW) {
                    const uint32_t base = c * SLEN + zb * SC;
#pragma unroll
                    for (uint32_t k = 0; k < PI; k++) {
                        const uint32_t bk = k * 64 + lane;
                        const uint32_t o = bk < PB ? (bk * 16 + 16 <= PL ? bk * 16 : PL - 16) : 0x80000000u;
                        __builtin_amdgcn_raw_buffer_store_b128(v, wb, (int)o, (int)base, 2);
                    }
                }
            }
        }
    }
    if (acc.x == 0x12345678u && acc.y == 3u) sink[0] = acc.z + lds[threadIdx.x];
}

template <typename F>
float timeit(F f, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    f();
    float best = 1e9;
    for (int k = 0; k < 3; k++) {
        CK(hipEventRecord(e0, 0));
        for (int r = 0; r < reps; r++) f();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        CK(hipGetLastError());
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms / reps < best) best = ms / reps;
    }
    return best;
}

template <int P, int NPART, bool PACK, bool LPACK, int NW = 6>
void run(const char *name, uint8_t *din, uint8_t *dout, uint32_t *sink, size_t lds) {
    auto fn = skel<P, NPART, PACK, LPACK, NW>;
    CK(hipFuncSetAttribute(reinterpret_cast<const void *>(fn), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    const float t = timeit([&] { hipLaunchKernelGGL(fn, dim3(NOBJ * NST), dim3(NW * 64), lds, 0, din, dout, sink); }, 10);
    const double alg = (double)NOBJ * OBJ + (double)NOBJ * 20 * SLEN;
    printf("%-52s %8.3f ms  %7.1f GB/s alg  frac %.3f\n", name, t, alg / t / 1e6, alg / t / 1e6 / 8000.0);
}

int main() {
    const size_t in_b = (size_t)NOBJ * OBJ, out_b = (size_t)NOBJ * 20 * SLEN;
    uint8_t *din, *dout;
    uint32_t *sink;
    CK(hipMalloc(&din, in_b + (1 << 20)));
    CK(hipMalloc(&dout, out_b + (1 << 20)));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(din, 0x5a, in_b));
    const size_t L2 = 80 * 1024, L1 = 150 * 1024;
    run<1, 9, false, true>("P1 part9 lpack, row stores (current kernel)", din, dout, sink, L2);
    run<1, 9, true, true>("P1 part9 lpack, packed stores", din, dout, sink, L2);
    run<1, 0, false, true>("P1 part0 lpack, row stores", din, dout, sink, L2);
    run<1, 0, true, true>("P1 part0 lpack, packed stores", din, dout, sink, L2);
    run<2, 9, true, true>("P2 part9 lpack, packed stores", din, dout, sink, L2);
    run<2, 0, true, true>("P2 part0 lpack, packed stores", din, dout, sink, L2);
    run<10, 0, true, true>("P10 part0 lpack, packed stores", din, dout, sink, L2);
    run<1, 9, true, true, 12>("P1 part9 lpack packed, 12 waves 1 WG/CU", din, dout, sink, L1);
    run<1, 0, true, true, 12>("P1 part0 lpack packed, 12 waves 1 WG/CU", din, dout, sink, L1);
    run<1, 9, false, false>("P1 part9 row loads, row stores", din, dout, sink, L2);
    run<1, 9, true, false>("P1 part9 row loads, packed stores", din, dout, sink, L2);
    return 0;
}
