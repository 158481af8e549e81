// vmem_bench8.hip -- encode output pattern: whole rows vs line-exact junctions (not product code).
// Each stripe writes its 20 rotated chunks plane by plane (one 1,430-byte row per chunk per step),
// as enc_dma_kernel does.  Variants per row store:
//   ROW   : [A, A + sc) from 16-byte blocks relative to A (today's shape: the junction line with the
//           next row is written by two instructions one step apart);
//   LINE  : the aligned lines [R(A), R(A + sc)) -- the head junction line written whole, with the
//           previous row's tail (what a carry buffer supplies), the tail line left to the next row;
//   DEFER : the previous row's tail [R(A), A) and then [A, R(A + sc)): both halves of a junction
//           line written back to back by one wave;
//   PAD   : rows padded to 1,536 B (every line whole -- control).
// WPG waves per workgroup; wave w of a stripe's workgroup stores the rows r = w mod WPG of each
// step (chunk assignment rotating with the step, as the flush table does).
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 -o scripts/vmem_bench8 scripts/vmem_bench8.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t xcd_tile(uint32_t b, uint32_t nb) {
    const uint32_t full = nb & ~7u;
    if (b >= full) return b;
    return (b & 7u) * (full >> 3) + (b >> 3);
}

enum { ROW = 0, LINE = 1, DEFER = 2, PAD = 3 };

template <int MODE, int WPG, bool NT, uint32_t SC = (MODE == PAD ? 1536u : 1430u), uint32_t SX = (MODE == PAD ? 128u : 48u)>
__global__ void __launch_bounds__(64 * WPG) encw(uint8_t *out, uint32_t nst) {
    constexpr uint32_t sc = SC, cs = 100 * sc, slen = 5 * cs + SX;
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t job = xcd_tile(blockIdx.x, gridDim.x);
    if (job >= nst) return;
    const uint32_t obj = job / 5, s = job - obj * 5;
    const uint64_t base = (uint64_t)obj * 20 * slen;  // out is 4 KiB aligned: addresses mod 128 are real
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out + base, 0, (int)(20 * slen), 0x00020000);
    const uint32_t rot = (s * 7) % 20;
    for (uint32_t z = 0; z < 100; z++) {
        for (uint32_t r = wv; r < 20; r += WPG) {
            const uint32_t rr = (r + z) % 20;  // which chunk this wave stores rotates with the step
            uint32_t sl = rr + rot;
            sl = sl >= 20 ? sl - 20 : sl;
            const uint32_t A = sl * slen + s * cs + z * sc;  // offset from base (base % 128 == 0)
            const u32x4 v = u32x4{z, rr, lane, 0};
            if (MODE == ROW || MODE == PAD) {  // PAD: ROW stores of padded rows
                for (uint32_t k = 0; k < 2; k++) {
                    const uint32_t b = k * 1024 + lane * 16;
                    const uint32_t o = b + 16 <= sc ? b : (b < sc + 15 ? sc - 16 : 0x80000000u);
                    if (o != 0x80000000u) __builtin_amdgcn_raw_buffer_store_b128(v, rs, (int)o, (int)A, NT ? 2 : 0);
                }
            } else {
                const uint32_t R0 = A & ~127u, R1 = z == 99 ? (A + sc + 15) & ~15u : (A + sc) & ~127u;
                uint32_t from = R0;
                if (MODE == DEFER && z > 0) {  // previous tail (16-B blocks from R0 to A), then the row
                    const uint32_t o = R0 + lane * 16;
                    if (o < A) __builtin_amdgcn_raw_buffer_store_b128(v, rs, (int)o, 0, NT ? 2 : 0);
                    from = A & ~15u;
                } else if (z == 0) {
                    from = A & ~15u;
                }
                for (uint32_t k = 0; k < 2; k++) {
                    const uint32_t o = from + k * 1024 + lane * 16;
                    if (o < R1) __builtin_amdgcn_raw_buffer_store_b128(v, rs, (int)o, 0, NT ? 2 : 0);
                }
            }
        }
    }
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
    const uint32_t nobj = 1024, nst = nobj * 5;
    uint8_t *d;
    CK(hipMalloc(&d, (size_t)nobj * 20 * (5 * 166400 + 4096) + 4096));
    const double B = (double)nobj * 20 * (5 * 143000 + 48);
    auto rep = [&](const char *name, float t, double b) { printf("%-44s %8.3f ms  %7.1f GB/s\n", name, t, b / t / 1e6); };
#define RUN(M, W, NT, name, bytes) \
    rep(name, timeit([&] { hipLaunchKernelGGL((encw<M, W, NT>), dim3(nst), dim3(64 * W), 0, 0, d, nst); }, 5), bytes)
    RUN(ROW, 1, false, "ROW   1 wave/stripe", B);
    RUN(LINE, 1, false, "LINE  1 wave/stripe", B);
    RUN(DEFER, 1, false, "DEFER 1 wave/stripe", B);
    RUN(PAD, 1, false, "PAD   1 wave/stripe", B * 1536 / 1430);
    RUN(ROW, 6, false, "ROW   6 waves/stripe", B);
    RUN(LINE, 6, false, "LINE  6 waves/stripe", B);
    RUN(DEFER, 6, false, "DEFER 6 waves/stripe", B);
    RUN(PAD, 6, false, "PAD   6 waves/stripe", B * 1536 / 1430);
    RUN(ROW, 6, true, "ROW   6 waves/stripe nt", B);
    RUN(LINE, 6, true, "LINE  6 waves/stripe nt", B);
    RUN(DEFER, 6, true, "DEFER 6 waves/stripe nt", B);
    // geometry probes: which property makes PAD fast
#define RUNG(M, SC, SX, name) \
    rep(name, timeit([&] { hipLaunchKernelGGL((encw<M, 6, false, SC, SX>), dim3(nst), dim3(384), 0, 0, d, nst); }, 5), \
        (double)nobj * 20 * (5 * 100.0 * SC + SX))
    RUNG(ROW, 1408, 128, "ROW  sc 1408 (11 lines), slices aligned");
    RUNG(LINE, 1408, 48, "LINE sc 1408, slice tail 48 B");
    RUNG(ROW, 1408, 48, "ROW  sc 1408, slice tail 48 B");
    RUNG(LINE, 1440, 128, "LINE sc 1440, slices aligned");
    RUNG(ROW, 1440, 128, "ROW  sc 1440, slices aligned");
    RUNG(ROW, 1430, 8, "ROW  sc 1430, slices aligned");
    RUNG(LINE, 1430, 8, "LINE sc 1430, slices aligned");
    RUNG(LINE, 1536, 48, "LINE sc 1536, slice tail 48 B");
    RUNG(ROW, 1472, 128, "ROW  sc 1472 (rows at 0/64 mod 128)");
    RUNG(LINE, 1472, 128, "LINE sc 1472");
    RUNG(ROW, 1344, 128, "ROW  sc 1344 (10.5 lines)");
    return 0;
}
