// enc_skeleton3.hip -- microbenchmark (not product code), third series: the encode's memory shape
// with no arithmetic, through LDS-DMA as enc_dma_kernel loads.  Questions: (1) per-row DMA
// instructions (2 per 1,430-byte row) against the kernel's packed ones (64 consecutive blocks of
// the plane's concatenated rows); (2) two planes per step: rows of planes s, s+1 loaded / stored as
// one 2,860-byte piece (contiguous) or as two row pieces issued together (split).
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 -o scripts/enc_skeleton3 scripts/enc_skeleton3.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr uint32_t SC = 1430, CS = 100 * SC, SLEN = 5 * CS + 48, NOBJ = 1024, NST = 5;
constexpr uint32_t OBJ = 4u << 20;
constexpr uint32_t NB = (SC + 15) / 16;  // 90

__device__ __forceinline__ u32x4 rsrc(const void *p, uint32_t nrec) {
    const uint64_t a = reinterpret_cast<uint64_t>(p);
    u32x4 r;
    r.x = __builtin_amdgcn_readfirstlane((uint32_t)a);
    r.y = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32) & 0xffffu);
    r.z = __builtin_amdgcn_readfirstlane(nrec);
    r.w = 0x00020000u;
    return r;
}
__device__ __forceinline__ void dma16(u32x4 rs, uint32_t voff, uint32_t soff, uint32_t lds) {
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
        "buffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
        : "=&s"(keep) : "v"(voff), "s"(rs), "s"(lds), "s"(soff) : "memory");
}

// LMODE: 0 packed (kernel), 1 per-row, 2 two-plane contiguous pieces, 3 two-plane split rows
// SMODE: 0 per-row each plane, 2 two-plane contiguous pieces, 3 two-plane split rows,
//        4 split rows: every wave stores its own 256-byte column segment of every row (dword per
//          lane, the compute layout's words; no staging)
template <int LMODE, int SMODE, int NW = 6>
__global__ void __launch_bounds__(NW * 64) skel(const uint8_t *in, uint8_t *out, uint32_t *sink) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const uint32_t lds0 = __builtin_amdgcn_groupstaticsize();
    const uint32_t lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t job = blockIdx.x, obj = job / NST, st = job % NST;
    const uint8_t *src = in + (size_t)obj * OBJ + (size_t)st * 7 * CS;
    const uint32_t src_len = st + 1 < NST ? 7 * CS : OBJ - (NST - 1) * 7 * CS;
    uint8_t *dst = out + (size_t)obj * 20 * SLEN + (size_t)st * CS;
    const u32x4 rs = rsrc(src, src_len);
    const __amdgpu_buffer_rsrc_t wb = __builtin_amdgcn_make_buffer_rsrc(dst, 0, (int)(19 * SLEN + CS), 0x00020000);
    const u32x4 v = {lane, wv, 7u, 9u};
    constexpr bool TWO = LMODE >= 2 || SMODE == 2 || SMODE == 3;
    constexpr uint32_t STEP = TWO ? 2 : 1;
    constexpr uint32_t SLOT = 16 * 2 * 1440 + 1024;
    for (uint32_t z = 0; z < 100; z += STEP) {
        const uint32_t z0 = z / 10, s = z % 10;
        const uint32_t slot = ((z / STEP) & 1) * SLOT;
        auto row_off = [&](uint32_t r, uint32_t zz) -> uint32_t {
            return r < 7 ? r * CS + zz * SC : (z0 < 7 ? z0 : 0) * CS + ((r - 7) * 10 + zz % 10) * SC;
        };
        // ---- loads (16 rows per plane) ----
        if (LMODE == 0) {  // packed: 16 rows x 90 blocks = 23 instructions per plane
            for (uint32_t p = 0; p < STEP; p++) {
                for (uint32_t i = wv; i < 23; i += NW) {
                    const uint32_t b = 64 * i + lane, r = b / NB, k = b - r * NB;
                    if (r < 16) dma16(rs, row_off(r, z + p) + (k * 16 + 16 <= SC ? k * 16 : SC - 16), 0,
                                      __builtin_amdgcn_readfirstlane(lds0 + slot + p * 16 * 1440 + 1024 * i));
                }
            }
        } else if (LMODE == 1 || LMODE == 3) {  // per row: 2 instructions
            for (uint32_t p = 0; p < STEP; p++) {
                for (uint32_t r = wv; r < 16; r += NW) {
#pragma unroll
                    for (uint32_t k = 0; k < 2; k++) {
                        const uint32_t bk = 64 * k + lane;
                        if (bk < NB) dma16(rs, (bk * 16 + 16 <= SC ? bk * 16 : SC - 16), row_off(r, z + p),
                                           __builtin_amdgcn_readfirstlane(lds0 + slot + (p * 16 + r) * 1440 + 1024 * k));
                    }
                }
            }
        } else {  // two-plane pieces: 2,860 bytes = 179 blocks, 3 instructions
            for (uint32_t r = wv; r < 16; r += NW) {
#pragma unroll
                for (uint32_t k = 0; k < 3; k++) {
                    const uint32_t bk = 64 * k + lane;
                    if (bk < 179) dma16(rs, (bk * 16 + 16 <= 2 * SC ? bk * 16 : 2 * SC - 16), row_off(r, z),
                                        __builtin_amdgcn_readfirstlane(lds0 + slot + r * 2880 + 1024 * k));
                }
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        // ---- stores (20 chunks) ----
        if (SMODE == 4) {  // each wave: its 64 words of each of the 20 rows (a lane's 4 columns)
            const uint32_t col = (wv * 64 + lane) * 4;
            for (uint32_t c = 0; c < 20; c++) {
                const uint32_t base = c * SLEN + z * SC;
                __builtin_amdgcn_raw_buffer_store_b32(v.x, wb, (int)(col + 4 <= SC ? col : 0x80000000u), (int)base, 2);
            }
        } else if (SMODE == 0 || SMODE == 3) {
            for (uint32_t c = wv; c < 20; c += NW) {
                for (uint32_t p = 0; p < STEP; p++) {
                    const uint32_t base = c * SLEN + (z + p) * SC;
#pragma unroll
                    for (uint32_t k = 0; k < 2; k++) {
                        const uint32_t bk = 64 * k + lane;
                        const uint32_t o = bk < NB ? (bk * 16 + 16 <= SC ? bk * 16 : SC - 16) : 0x80000000u;
                        __builtin_amdgcn_raw_buffer_store_b128(v, wb, (int)o, (int)base, 2);
                    }
                }
            }
        } else {
            for (uint32_t c = wv; c < 20; c += NW) {
                const uint32_t base = c * SLEN + z * SC;
#pragma unroll
                for (uint32_t k = 0; k < 3; k++) {
                    const uint32_t bk = 64 * k + lane;
                    const uint32_t o = bk < 179 ? (bk * 16 + 16 <= 2 * SC ? bk * 16 : 2 * SC - 16) : 0x80000000u;
                    __builtin_amdgcn_raw_buffer_store_b128(v, wb, (int)o, (int)base, 2);
                }
            }
        }
    }
    if (lds[threadIdx.x] == 0x12345678u) sink[0] = 1;
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

template <int LMODE, int SMODE, int NW = 6>
void run(const char *name, uint8_t *din, uint8_t *dout, uint32_t *sink, size_t lds) {
    auto fn = skel<LMODE, SMODE, NW>;
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
    // LDS: two slots of 2 planes x 16 rows; 2 WG/CU need <= 80 KB: use one-plane slots then
    const size_t L1p = 2 * (16 * 1440 + 1024), L2p = 2 * (16 * 2 * 1440 + 1024);
    run<0, 0>("L packed, S row (kernel shape)", din, dout, sink, L1p);
    run<1, 0>("L row, S row", din, dout, sink, L1p);
    run<1, 3>("L row, S two-plane split", din, dout, sink, L2p);
    run<3, 3>("L two-plane split, S two-plane split", din, dout, sink, L2p);
    run<2, 2>("L two-plane piece, S two-plane piece", din, dout, sink, L2p);
    run<2, 3>("L two-plane piece, S two-plane split", din, dout, sink, L2p);
    run<3, 2>("L two-plane split, S two-plane piece", din, dout, sink, L2p);
    run<0, 0, 12>("L packed, S row, 12 waves", din, dout, sink, L2p + 8192);
    run<3, 3, 12>("L split2, S split2, 12 waves", din, dout, sink, L2p + 8192);
    run<2, 2, 12>("L piece2, S piece2, 12 waves", din, dout, sink, L2p + 8192);
    run<0, 0>("L packed, S row (kernel shape) again", din, dout, sink, L1p);
    run<0, 4>("L packed, S split words (no staging)", din, dout, sink, L1p);
    run<0, 4, 12>("L packed, S split words, 12 waves", din, dout, sink, L2p + 8192);
    run<0, 0>("L packed, S row (kernel shape) 3rd", din, dout, sink, L1p);
    return 0;
}
