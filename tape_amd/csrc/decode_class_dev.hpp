// decode_class_dev.hpp -- device side of the decode class kernels (dec_class.hpp explains the
// classes; the kernel bodies are generated at build time into build/gen/dec_class_<id>.hip).
//
// A workgroup owns one stripe's row segment: G waves x 64 lanes x 4 columns, each lane one 4-byte
// word of every plane (as decode_stage.hip and the hipRTC pattern kernels), words kept in load
// order and stored straight back to their data chunk.  What is run-time here is only what the
// survivor set decides: the slices of the known nodes, the physical plane of each canonical
// plane digit, the data chunk of each canonical data node, and the decoding matrix (v_perm tables,
// scalar-loaded from the pattern).
#pragma once
#include "kernels.hpp"
#include "gf_dev.hpp"
#include "dev_io.hpp"

namespace tec {
namespace dcls {

typedef uint32_t u32;
typedef uint8_t u8;
typedef uint64_t u64;

struct DecClassArgs {
    const GpeJob *jobs;
    const GpePattern *patterns;  // the pattern store (or the call's arena copy); jobs name entries
    u8 *scratch;                 // njobs x wgs_per_stripe tiles of nscratch rows
    u64 in_stride;               // slice length
    u64 out_stride;              // chunk size
    u32 njobs, sc, wps, wgs_per_stripe, n, nscratch;
    u32 out_full;                // a job whose out_len reaches this writes every output row whole
};

// host registry entry of one class (decode_class.hip)
struct DecClassEntry {
    const void *fn[2] = {nullptr, nullptr};  // G = 1, 2
    uint32_t nslots = 0, nscratch = 0, nring = 0;  // nring: the per-call kernel's ring rows per step
};

__device__ __forceinline__ u32 pft3(u32 a, u32 b) { return a ^ xt(a ^ b); }  // 3a ^ 2b (PFT, A3)

// G waves of columns per workgroup (one 4-byte word per lane); W waves share those columns and
// split each step's work (the per-call kernel: W = 4, all values in LDS, a barrier per step)
template <int G, int W = 1>
struct CTile {
    typedef const __attribute__((address_space(4))) GpePattern cPat;
    typedef const __attribute__((address_space(4))) PermTab cTab;
    static constexpr u32 RS = G * 256u;  // LDS / scratch row stride (G waves x 64 lanes x 4 B)
    u8 *lds8;
    cPat *pat;
    u32 lane, col_local, vcol, sc, olen, rot, n, in_stride, out_stride, wv;
    bool full;
    __amdgpu_buffer_rsrc_t rs_in, rs_out, rs_scr;

    __device__ __forceinline__ CTile(const DecClassArgs &a, u8 *lds) {
        lds8 = lds;
        lane = threadIdx.x & 63u;
        const u32 t = threadIdx.x % (G * 64u);  // this thread's column word within the workgroup's
        wv = __builtin_amdgcn_readfirstlane(threadIdx.x / (G * 64u));  // which of the W sharing waves
        col_local = t * 4u;
        const u32 tile = xcd_tile(blockIdx.x, gridDim.x);
        const u32 job = tile / a.wgs_per_stripe, seg = tile - job * a.wgs_per_stripe;
        typedef const __attribute__((address_space(4))) GpeJob cJob;
        cJob &J = *(cJob *)(uintptr_t)(a.jobs + job);
        pat = (cPat *)(uintptr_t)(a.patterns + J.pattern);
        sc = a.sc;
        n = a.n;
        rot = J.rot;
        in_stride = (u32)a.in_stride;
        out_stride = (u32)a.out_stride;
        u32 w = seg * G * 64u + t;
        if (w >= a.wps) w = a.wps - 1;  // words past the stripe alias the last (same values, same bytes)
        const u32 col = w * 4u;
        vcol = col + 4u > a.sc ? a.sc - 4u : col;  // the row's last 4 bytes for a word past the sub-chunk
        rs_in = __builtin_amdgcn_make_buffer_rsrc((void *)J.in, 0, (int)(u32)(a.n * a.in_stride), 0x00020000);
        olen = (u32)J.out_len;
        full = olen >= a.out_full;  // every output row inside the job's output share (not a last stripe)
        rs_out = __builtin_amdgcn_make_buffer_rsrc((void *)J.out, 0, (int)olen, 0x00020000);
        const u32 nscr = a.nscratch ? a.nscratch : 1u;
        rs_scr = __builtin_amdgcn_make_buffer_rsrc(a.scratch + (u64)tile * nscr * RS, 0, (int)(nscr * RS), 0x00020000);
    }
    // the W sharing waves' LDS hand-off between steps (LDS only: loads in flight keep flying)
    __device__ __forceinline__ void sync() const { lds_barrier(); }
    // the pattern's known / erased node ids (ascending), scalar loads
    __device__ __forceinline__ u32 K(int i) const { return pat->known[i]; }
    __device__ __forceinline__ u32 E(int i) const { return pat->erased[i]; }
    // slice byte offset of node `node` in the stripe's (rotated) input
    __device__ __forceinline__ u32 kbase(u32 node) const {
        const u32 s = node + rot;
        return (s >= n ? s - n : s) * in_stride;
    }
    // a known row's own words (read once: non-temporal) and a partner row's
    __device__ __forceinline__ u32 ld_own(u32 base, u32 off) const {
        return __builtin_amdgcn_raw_buffer_load_b32(rs_in, (int)vcol, (int)(base + off), 2);
    }
    __device__ __forceinline__ u32 ld(u32 base, u32 off) const {
        return __builtin_amdgcn_raw_buffer_load_b32(rs_in, (int)vcol, (int)(base + off), 0);
    }
    template <int AUX>
    __device__ __forceinline__ u32 ld_aux(u32 base, u32 off) const {
        return __builtin_amdgcn_raw_buffer_load_b32(rs_in, (int)vcol, (int)(base + off), AUX);
    }
    __device__ __forceinline__ u32 lds_ld(u32 row) const { return *reinterpret_cast<const u32 *>(lds8 + row * RS + col_local); }
    __device__ __forceinline__ void lds_st(u32 row, u32 v) const { *reinterpret_cast<u32 *>(lds8 + row * RS + col_local) = v; }
    template <int AUX = 0>
    __device__ __forceinline__ u32 scr_ld(u32 row) const {
        return __builtin_amdgcn_raw_buffer_load_b32(rs_scr, (int)col_local, (int)(row * RS), AUX);
    }
    __device__ __forceinline__ void scr_st(u32 row, u32 v) const {
        __builtin_amdgcn_raw_buffer_store_b32(v, rs_scr, (int)col_local, (int)(row * RS), 0);
    }
    // output base of column-0 node `node`: its data chunk, or for a parity node an offset past
    // every stripe's output range, so the buffer range check drops its stores
    __device__ __forceinline__ u32 out_base(u32 node) const { return node < kData ? node * out_stride : kDropBase; }
    static constexpr u32 kData = 7, kDropBase = 0x80000000u;
    // one decoded word to data chunk offset `ob` at plane offset `po`, where it was loaded; a
    // word across the end of the stripe's output share is written byte by byte
    __device__ __forceinline__ void out_st(u32 ob, u32 po, u32 v) const {
        if (ob == kDropBase) return;  // uniform: a column-0 parity node's row is not output
        out_st_oob(ob, po, v);
    }
    // the same without the uniform skip: a dropped row's store goes past the buffer's range and
    // the range check discards it (measurement variant, gen_dec_class TEC_GEN_DROP_BRANCH=0)
    __device__ __forceinline__ void out_st_oob(u32 ob, u32 po, u32 v) const {
        const u32 o = ob + po + vcol;
        if (full) {  // uniform: every data row of the stripe lies inside its output share
            __builtin_amdgcn_raw_buffer_store_b32(v, rs_out, (int)o, 0, 2);
        } else if (o + 4u > olen && o < olen) {
#pragma unroll
            for (u32 k = 0; k < 4u; k++) __builtin_amdgcn_raw_buffer_store_b8((u8)(v >> (8u * k)), rs_out, (int)(o + k), 0, 0);
        } else {
            __builtin_amdgcn_raw_buffer_store_b32(v, rs_out, (int)o, 0, 2);
        }
    }
    // The matrix of one erased row: the pattern pointer is laundered each time so the row's table
    // loads are issued where they are used, not hoisted over the straight-line program (the
    // 13 x 7 tables of 5 dwords are 455 SGPRs: hoisted, they spill).
    __device__ __forceinline__ cTab (*mat() const)[kGpeMaxKnown] {
        u64 p = (u64)(uintptr_t)pat;
        asm volatile("; mat" : "+s"(p));
        return ((cPat *)(uintptr_t)p)->D;
    }
    // the 2-bit-field tables of one erased row (laundered as mat())
    typedef const __attribute__((address_space(4))) u32 cU32;
    __device__ __forceinline__ cU32 (*mat4() const)[kClsMaxK][4] {
        u64 p = (u64)(uintptr_t)pat;
        asm volatile("; mat4" : "+s"(p));  // a fresh value per call: the loads are not hoisted
        return ((cPat *)(uintptr_t)p)->D4;
    }
    __device__ __forceinline__ static u32 mul2(u32 acc, cU32 (*D)[kClsMaxK][4], int e, int j, const Sel4 &x, const Sel4 &y) {
        cU32 *p = D[e][j], *q = D[e][j + 1];
        return perm4_mul2_acc(acc, x, p[0], p[1], p[2], p[3], y, q[0], q[1], q[2], q[3]);
    }
    __device__ __forceinline__ static u32 mul1(u32 acc, cU32 (*D)[kClsMaxK][4], int e, int j, const Sel4 &x) {
        cU32 *p = D[e][j];
        return perm4_mul_acc(acc, x, p[0], p[1], p[2], p[3]);
    }
    __device__ __forceinline__ static u32 mul2(u32 acc, cTab (*D)[kGpeMaxKnown], int e, int j, const Sel &x, const Sel &y) {
        cTab &p = D[e][j], &q = D[e][j + 1];
        return perm_mul2_acc(acc, x, p.t[0], p.t[1], p.t[2], p.t[3], p.t[4], y, q.t[0], q.t[1], q.t[2], q.t[3], q.t[4]);
    }
    __device__ __forceinline__ static u32 mul1(u32 acc, cTab (*D)[kGpeMaxKnown], int e, int j, const Sel &x) {
        cTab &p = D[e][j];
        return perm_mul_acc(acc, x, p.t[0], p.t[1], p.t[2], p.t[3], p.t[4]);
    }
};

}  // namespace dcls
}  // namespace tec
