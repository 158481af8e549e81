// enc_skeleton.hip -- microbenchmark (not product code): the encode's exact memory traffic shape
// (1024 x 4 MiB objects, 5 stripes each, sub-chunk 1,430 B, 20 slices of 715,048 B per object)
// with no arithmetic, to find which traversal shape the HBM rewards before building it.
//
// Per stripe (one workgroup of 6 waves, 80 KB of LDS requested so two are resident per CU, as in
// enc_dma_kernel): 100 planes; per plane 7 own rows + NPART partner rows are loaded (16 B per
// lane, summed into a sink), and every P planes the 20 chunks' rows of those P planes are stored
// as one contiguous piece of P x 1,430 B per chunk.  BAR: an s_barrier per plane.
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 -o scripts/enc_skeleton scripts/enc_skeleton.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr uint32_t SC = 1430, CS = 100 * SC, SLEN = 5 * CS + 48, NOBJ = 1024, NST = 5;
constexpr uint32_t OBJ = 4u << 20;

template <int P, int NPART, bool BAR, int AUX, bool LINE, int LP = 1, int NW = 6>
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
    constexpr uint32_t NLOAD = 7 + NPART;               // rows per plane
    constexpr uint32_t PIECE = P * SC;                  // bytes per chunk per store batch
    constexpr uint32_t PI = (PIECE + 1023) / 1024;      // 1 KiB instructions per piece
    for (uint32_t z = 0; z < 100; z++) {
        const uint32_t z0 = z / 10, s = z % 10;
        // loads: row r of this plane, 2 instructions per row (1 KiB + rest); LP planes at once
        // as one LP x 1,430 B piece per row
        if (z % LP == 0) {
            constexpr uint32_t LPIECE = LP * SC, LI = (LPIECE + 1023) / 1024;
            for (uint32_t r = wv; r < NLOAD; r += NW) {
                uint32_t off;
                if (r < 7) off = r * CS + z * SC;
                else off = (z0 < 7 ? z0 : 0) * CS + ((r - 7) * 10 + s) * SC;
#pragma unroll
                for (uint32_t k = 0; k < LI; k++) {
                    const uint32_t o = k * 1024 + lane * 16;
                    acc ^= __builtin_amdgcn_raw_buffer_load_b128(rb, (int)(o < LPIECE ? o : 0x80000000u), (int)off, AUX);
                }
            }
        }
        if (BAR) __syncthreads();
        if ((z + 1) % P == 0) {
            const uint32_t zb = z + 1 - P;
            for (uint32_t c = wv; c < 20; c += NW) {
                uint32_t base = c * SLEN + zb * SC;
                uint32_t len = PIECE;
                if (LINE) {  // stores on the 128-byte line grid (wrong bytes: timing only)
                    base &= ~127u;
                    len = (PIECE + 127) & ~127u;
                }
#pragma unroll
                for (uint32_t k = 0; k < PI; k++) {
                    const uint32_t o = k * 1024 + lane * 16;
                    __builtin_amdgcn_raw_buffer_store_b128(v, wb, (int)(o < len ? o : 0x80000000u), (int)base, 2);
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

template <int P, int NPART, bool BAR, int AUX, bool LINE, int LP = 1, int NW = 6>
void run(const char *name, uint8_t *din, uint8_t *dout, uint32_t *sink, size_t lds) {
    auto fn = skel<P, NPART, BAR, AUX, LINE, LP, NW>;
    CK(hipFuncSetAttribute(reinterpret_cast<const void *>(fn), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    const float t = timeit([&] { hipLaunchKernelGGL(fn, dim3(NOBJ * NST), dim3(NW * 64), lds, 0, din, dout, sink); }, 10);
    const double alg = (double)NOBJ * OBJ + (double)NOBJ * 20 * SLEN;
    printf("%-60s %8.3f ms  %7.1f GB/s alg  frac %.3f\n", name, t, alg / t / 1e6, alg / t / 1e6 / 8000.0);
}

int main() {
    const size_t in_b = (size_t)NOBJ * OBJ, out_b = (size_t)NOBJ * 20 * SLEN;
    uint8_t *din, *dout;
    uint32_t *sink;
    CK(hipMalloc(&din, in_b + (1 << 20)));
    CK(hipMalloc(&dout, out_b + (1 << 20)));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(din, 0x5a, in_b));
    const size_t L2 = 80 * 1024, L3 = 52 * 1024;
    const size_t L1 = 150 * 1024;
    run<1, 9, true, 0, false>("P1 part9 bar (current shape)", din, dout, sink, L2);
    run<2, 9, true, 0, false>("P2 part9 bar", din, dout, sink, L2);
    run<2, 9, true, 0, false, 2>("P2 LP2 part9 bar", din, dout, sink, L2);
    run<2, 9, true, 0, false, 2, 12>("P2 LP2 part9 bar, 12 waves 1 WG/CU", din, dout, sink, L1);
    run<2, 9, true, 0, false, 2, 6>("P2 LP2 part9 bar, 6 waves 1 WG/CU", din, dout, sink, L1);
    run<1, 9, true, 0, false, 1, 12>("P1 part9 bar, 12 waves 1 WG/CU", din, dout, sink, L1);
    run<2, 0, true, 0, false, 2>("P2 LP2 part0 bar", din, dout, sink, L2);
    run<4, 9, true, 0, false, 2>("P4 LP2 part9 bar", din, dout, sink, L2);
    run<2, 9, true, 2, false, 2>("P2 LP2 part9 bar nt loads", din, dout, sink, L2);
    run<2, 9, false, 0, false, 2>("P2 LP2 part9 nobar", din, dout, sink, L2);
    run<1, 0, true, 0, false>("P1 part0 bar (reads once)", din, dout, sink, L2);
    run<1, 9, false, 0, false>("P1 part9 nobar", din, dout, sink, L2);
    run<1, 9, true, 0, true>("P1 part9 bar line-grid stores", din, dout, sink, L2);
    run<5, 0, true, 0, false>("P5 part0 bar", din, dout, sink, L2);
    run<10, 0, true, 0, false>("P10 part0 bar", din, dout, sink, L2);
    run<10, 9, true, 0, false>("P10 part9 bar", din, dout, sink, L2);
    run<10, 0, false, 0, false>("P10 part0 nobar", din, dout, sink, L2);
    run<10, 0, true, 0, true>("P10 part0 bar line-grid", din, dout, sink, L2);
    run<1, 0, true, 0, false, 1, 12>("P1 part0 bar 12 waves 1 WG/CU", din, dout, sink, L1);
    run<10, 0, true, 0, false, 1, 12>("P10 part0 bar 12 waves 1 WG/CU", din, dout, sink, L1);
    return 0;
}
