// hbm_probe.hip -- measurement only (libtecprobe.so, loaded by bench.py; not part of libtapeec).
//
// The box's own ceiling for the encode's byte mix, measured in the same process just before the
// timed region (two box types ran the same binary at 0.41 and 0.48 of the 8 TB/s
// spec, with identical reported clocks, so the bench line carries what THIS box's HBM does with
// the encode's exact traffic).  The mix is the encode's algorithmic bytes of one step: the batch's
// object bytes read once and its slice bytes written once (4.29 GB in, 14.64 GB out for 1024 x
// 4 MiB), with no compute, no barriers and no re-reads:
//   shape 0 ("blocks"): every workgroup streams a contiguous input range and a contiguous output
//                       range in whole 1 KiB wave-blocks (16 B per lane, nt stores);
//   shape 1 ("rows"):   the same, but the output walks 1,430-byte rows from a 2-aligned start, two
//                       store instructions per row -- the slices' sub-chunk rows, as the encode
//                       kernel writes them;
//   shape 2 ("rows, aligned interior"): the same rows, their 16-byte-aligned interior as aligned
//                       16-byte pieces and the partial head / tail as 2-byte stores (measurement).
// A kernel can at best reach the "blocks" figure; "rows" is what the slices' row shape alone costs.
#include <hip/hip_runtime.h>
#include <cstdint>

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int ROWS>  // 0 blocks, 1 rows (16-B pieces from the 2-aligned row start), 2 rows with
                    // 16-B-aligned interior pieces and 2-byte stores for the partial head / tail
__global__ void __launch_bounds__(256) mix_kernel(const uint8_t *in, uint64_t in_per_wg, uint8_t *out,
                                                  uint64_t out_per_wg, uint32_t *sink) {
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint8_t *src = in + (uint64_t)blockIdx.x * in_per_wg;
    uint8_t *dst = out + (uint64_t)blockIdx.x * out_per_wg;
    const __amdgpu_buffer_rsrc_t rb =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(src), 0, (int)in_per_wg, 0x00020000);
    const __amdgpu_buffer_rsrc_t wb = __builtin_amdgcn_make_buffer_rsrc(dst, 0, (int)out_per_wg, 0x00020000);
    const uint32_t nin = (uint32_t)(in_per_wg / 1024);
    const uint32_t nout = (uint32_t)(ROWS == 5 ? out_per_wg / 1408 : ROWS ? (out_per_wg - 2) / 1430 : out_per_wg / 1024);
    const uint32_t iters = (nin + 3) / 4;
    u32x4 acc = {0, 0, 0, 0};
    const u32x4 v = {lane, wv, 7u, 9u};
    for (uint32_t it = 0; it < iters; it++) {
        const uint32_t blk = it * 4 + wv;
        if (blk < nin) acc ^= __builtin_amdgcn_raw_buffer_load_b128(rb, (int)(blk * 1024 + lane * 16), 0, 0);
        // this iteration's share of the output, in proportion (reads : writes as in the encode)
        const uint32_t w0 = (uint32_t)((uint64_t)it * nout / iters), w1 = (uint32_t)((uint64_t)(it + 1) * nout / iters);
        for (uint32_t b = w0 + wv; b < w1; b += 4) {
            if constexpr (ROWS == 2) {
                const uint32_t a0 = 2 + b * 1430u, e0 = a0 + 1430u, A = (a0 + 15u) & ~15u, E = e0 & ~15u;
                const uint32_t n16 = (E - A) >> 4;
                __builtin_amdgcn_raw_buffer_store_b128(v, wb, (int)(lane < n16 ? A + lane * 16u : 0x80000000u), 0, 2);
                __builtin_amdgcn_raw_buffer_store_b128(v, wb, (int)(lane + 64u < n16 ? A + (lane + 64u) * 16u : 0x80000000u), 0, 2);
                const uint32_t nh = (A - a0) >> 1, nt = (e0 - E) >> 1;
                const uint32_t o2 = lane < nh ? a0 + 2u * lane : (lane >= 8 && lane - 8u < nt ? E + 2u * (lane - 8u) : 0x80000000u);
                __builtin_amdgcn_raw_buffer_store_b16((uint16_t)lane, wb, (int)o2, 0, 2);
            } else if constexpr (ROWS == 1 || ROWS == 3) {  // 3: the same with the default (write-back) policy
                constexpr int aux = ROWS == 1 ? 2 : 0;
                const uint32_t base = 2 + b * 1430u;
                __builtin_amdgcn_raw_buffer_store_b128(v, wb, (int)(lane * 16), (int)base, aux);
                const uint32_t o1 = lane < 25 ? 1024u + 16u * lane : (lane == 25 ? 1430u - 16u : 0x80000000u);
                __builtin_amdgcn_raw_buffer_store_b128(v, wb, (int)o1, (int)base, aux);
            } else if constexpr (ROWS == 5) {  // whole-line rows: 1,408 B (11 lines) from 128-B-aligned starts, 64 + 24 lanes
                const uint32_t base = b * 1408u;
                __builtin_amdgcn_raw_buffer_store_b128(v, wb, (int)(lane * 16), (int)base, 2);
                __builtin_amdgcn_raw_buffer_store_b128(v, wb, (int)(lane < 24 ? 1024u + 16u * lane : 0x80000000u), (int)base, 2);
            } else if constexpr (ROWS == 4) {  // nt interior, write-back for the two pieces in the junction lines
                const uint32_t base = 2 + b * 1430u;
                const uint32_t o1 = lane < 25 ? 1024u + 16u * lane : (lane == 25 ? 1430u - 16u : 0x80000000u);
                // pieces inside the row's partial first / last 128-B line (shared with the neighbour row)
                const uint32_t ab = (uint32_t)(reinterpret_cast<uintptr_t>(dst) & 127u) + base, ae = ab + 1430u;
                const uint32_t first_end = (ab & 127u) ? (ab + 127u) & ~127u : ab, last_beg = (ae & 127u) ? ae & ~127u : ae;
                const uint32_t p0 = ab + lane * 16u, p1 = ab + o1;
                const bool j0 = p0 < first_end || p0 + 16u > last_beg, j1 = o1 != 0x80000000u && (p1 < first_end || p1 + 16u > last_beg);
                __builtin_amdgcn_raw_buffer_store_b128(v, wb, (int)(j0 ? 0x80000000u : lane * 16), (int)base, 2);
                __builtin_amdgcn_raw_buffer_store_b128(v, wb, (int)(j0 ? 0u : 0x80000000u), (int)base, 0);
                __builtin_amdgcn_raw_buffer_store_b128(v, wb, (int)(j1 ? 0x80000000u : o1), (int)base, 2);
                __builtin_amdgcn_raw_buffer_store_b128(v, wb, (int)(j1 ? o1 : 0x80000000u), (int)base, 0);
            } else {
                __builtin_amdgcn_raw_buffer_store_b128(v, wb, (int)(b * 1024 + lane * 16), 0, 2);
            }
        }
    }
    if (acc.x == 0x12345678u && acc.y == 3u) sink[0] = acc.z;  // keeps the loads; never true for the bench input
}

uint32_t *g_sink = nullptr;

}  // namespace

// Average ms per launch of the mix over `reps` launches (after one untimed launch), on `stream`.
// in/out: device buffers of >= in_bytes / out_bytes; out is overwritten with junk.  `wgs`
// workgroups of 256 threads split both ranges evenly (per-workgroup ranges under 2 GiB).
// Returns 0, or a HIP error code.
extern "C" int tec_probe_encode_mix(const void *in, uint64_t in_bytes, void *out, uint64_t out_bytes, int shape,
                                    int wgs, int reps, void *stream, float *ms_out) {
    if (!in || !out || wgs <= 0 || reps <= 0 || !ms_out) return (int)hipErrorInvalidValue;
    hipStream_t s = (hipStream_t)stream;
    if (!g_sink) {
        hipError_t e = hipMalloc(&g_sink, 64);
        if (e != hipSuccess) return (int)e;
    }
    const uint64_t ipw = (in_bytes / (uint64_t)wgs) & ~(uint64_t)1023;
    const uint64_t opw = shape == 5 ? (out_bytes / (uint64_t)wgs) & ~(uint64_t)127
                         : shape ? (out_bytes / (uint64_t)wgs) & ~(uint64_t)15 : (out_bytes / (uint64_t)wgs) & ~(uint64_t)1023;
    if (ipw >= (1ull << 31) || opw >= (1ull << 31)) return (int)hipErrorInvalidValue;
    auto launch = [&] {
        if (shape == 5)
            hipLaunchKernelGGL(mix_kernel<5>, dim3(wgs), dim3(256), 0, s, (const uint8_t *)in, ipw, (uint8_t *)out,
                               opw, g_sink);
        else if (shape == 4)
            hipLaunchKernelGGL(mix_kernel<4>, dim3(wgs), dim3(256), 0, s, (const uint8_t *)in, ipw, (uint8_t *)out,
                               opw, g_sink);
        else if (shape == 3)
            hipLaunchKernelGGL(mix_kernel<3>, dim3(wgs), dim3(256), 0, s, (const uint8_t *)in, ipw, (uint8_t *)out,
                               opw, g_sink);
        else if (shape == 2)
            hipLaunchKernelGGL(mix_kernel<2>, dim3(wgs), dim3(256), 0, s, (const uint8_t *)in, ipw, (uint8_t *)out,
                               opw, g_sink);
        else if (shape)
            hipLaunchKernelGGL(mix_kernel<1>, dim3(wgs), dim3(256), 0, s, (const uint8_t *)in, ipw, (uint8_t *)out,
                               opw, g_sink);
        else
            hipLaunchKernelGGL(mix_kernel<0>, dim3(wgs), dim3(256), 0, s, (const uint8_t *)in, ipw, (uint8_t *)out,
                               opw, g_sink);
    };
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return (int)hipErrorUnknown;
    launch();
    (void)hipEventRecord(e0, s);
    for (int r = 0; r < reps; r++) launch();
    (void)hipEventRecord(e1, s);
    hipError_t e = hipEventSynchronize(e1);
    if (e == hipSuccess) e = hipGetLastError();
    float ms = 0;
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    *ms_out = ms / (float)reps;
    return (int)e;
}
