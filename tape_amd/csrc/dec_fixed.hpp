// dec_fixed.hpp -- device helpers of the per-pattern decode kernels (ClayCoder::decode,
// lib/slicer/src/clay.rs:106-122, inside Slicer::decode's per-stripe loop, slicer.rs:333-361;
// q = 10, t = 2 profiles).
//
// decode_stage.hip runs any erasure pattern from a program held in memory: each step's 48 control
// words are read out of a VGPR with v_readlane, every load slot is issued whether the step uses it
// or not, and each MDS product is a 6-VALU v_perm table product.  A per-pattern kernel is that
// same program (ClayHost::dec_prog, value by value) written out as straight-line code by the host
// (dec_rtc.hpp dec_fixed_source) and compiled at run time with hipRTC:
//   * only the loads a step uses are issued, at constant offsets, and no control words exist;
//   * the decoding matrix is folded: xtime multiples of each uncoupled U and v_bitop3 XOR
//     selections (~2 VALU per product instead of 6);
//   * LDS slot / staging rows and scratch rows are constants.
// This header is everything the generated source includes, so it depends on nothing but the
// compiler's builtins (hipRTC predefines the HIP keywords and thread indices it uses).
#pragma once
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#endif

#define TEC_DFI __device__ inline __attribute__((always_inline))

namespace tec {
namespace dfix {

typedef unsigned int u32;
typedef unsigned char u8;
typedef unsigned long long u64;

struct Job {  // layout of kernels.hpp GpeJob
    const u8 *in;
    u8 *out;
    u64 in_len, out_len;
    u32 rot, pattern;
};
struct Args {
    const Job *jobs;
    u8 *scratch;       // njobs x wgs_per_stripe tiles of the pattern's scratch rows
    u64 in_stride;     // slice length
    u64 out_stride;    // chunk size
    u32 njobs, sc, wps, wgs_per_stripe, n, nscratch;
};

TEC_DFI u32 xor3(u32 a, u32 b, u32 c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }
// x * 2 for four packed bytes over 0x11D (gf_dev.hpp xt)
TEC_DFI u32 xt(u32 x) {
    const u32 hb = (x >> 7) & 0x01010101u;
    return ((x & 0x7f7f7f7fu) << 1) ^ __builtin_amdgcn_perm(0u, 0x00001d00u, hb);
}
TEC_DFI u32 pft3(u32 a, u32 b) { return a ^ xt(a ^ b); }  // 3a ^ 2b: U from (C, C_partner), C from (U, U_partner)
// c * x for a constant c given as its 3/3/2-bit v_perm tables (gf.hpp PermTab): ~9 VALU where an
// xtime chain of c = 0xf4 (the type-1 coefficient) is ~37
TEC_DFI u32 mulk(u32 x, u32 t0, u32 t1, u32 t2, u32 t3, u32 t4) {
    return xor3(__builtin_amdgcn_perm(t1, t0, x & 0x07070707u), __builtin_amdgcn_perm(t3, t2, (x >> 3) & 0x07070707u),
                __builtin_amdgcn_perm(t4, t4, (x >> 6) & 0x03030303u));
}

// A lane's 8 columns (8-byte lanes, WB = 8): two dwords, every operation byte-wise per dword.
struct V2 {
    u32 x, y;
};
TEC_DFI V2 operator^(V2 a, V2 b) { return V2{a.x ^ b.x, a.y ^ b.y}; }
TEC_DFI V2 xor3(V2 a, V2 b, V2 c) { return V2{xor3(a.x, b.x, c.x), xor3(a.y, b.y, c.y)}; }
TEC_DFI V2 xt(V2 a) { return V2{xt(a.x), xt(a.y)}; }
TEC_DFI V2 pft3(V2 a, V2 b) { return a ^ xt(a ^ b); }
TEC_DFI V2 mulk(V2 x, u32 t0, u32 t1, u32 t2, u32 t3, u32 t4) {
    return V2{mulk(x.x, t0, t1, t2, t3, t4), mulk(x.y, t0, t1, t2, t3, t4)};
}

// Lane value type and its memory forms per lane width.
template <int WB> struct Lane;
template <> struct Lane<4> {
    typedef u32 V;
    static TEC_DFI V zero() { return 0u; }
    static TEC_DFI V ld(__amdgpu_buffer_rsrc_t r, u32 vo, u32 so) { return __builtin_amdgcn_raw_buffer_load_b32(r, (int)vo, (int)so, 0); }
    template <int AUX> static TEC_DFI void st(V v, __amdgpu_buffer_rsrc_t r, u32 vo, u32 so) { __builtin_amdgcn_raw_buffer_store_b32(v, r, (int)vo, (int)so, AUX); }
    // bytes [s, 4) then [0, s): the tail lane's columns from a load s bytes early
    static TEC_DFI V rot(V v, u32 s) { return __builtin_amdgcn_alignbyte(v, v, s); }
    static TEC_DFI V unrot(V v, u32 s) { return __builtin_amdgcn_alignbyte(v, v, (4u - s) & 3u); }
    static TEC_DFI u32 byte(V v, u32 k) { return v >> (8u * k); }
};
template <> struct Lane<8> {
    typedef V2 V;
    typedef u32 u32x2 __attribute__((ext_vector_type(2)));
    static TEC_DFI V zero() { return V2{0u, 0u}; }
    static TEC_DFI V ld(__amdgpu_buffer_rsrc_t r, u32 vo, u32 so) {
        const u32x2 t = __builtin_amdgcn_raw_buffer_load_b64(r, (int)vo, (int)so, 0);
        return V2{t.x, t.y};
    }
    template <int AUX> static TEC_DFI void st(V v, __amdgpu_buffer_rsrc_t r, u32 vo, u32 so) {
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{v.x, v.y}, r, (int)vo, (int)so, AUX);
    }
    // rotate the 8 bytes right by s (even, < 8): byte i <- byte (i + s) mod 8
    static TEC_DFI V rot(V v, u32 s) {
        const bool sw = s >= 4u;
        const u32 a = sw ? v.y : v.x, b = sw ? v.x : v.y, t = s & 3u;
        return V2{__builtin_amdgcn_alignbyte(b, a, t), __builtin_amdgcn_alignbyte(a, b, t)};
    }
    static TEC_DFI V unrot(V v, u32 s) { return rot(v, (8u - s) & 7u); }
    static TEC_DFI u32 byte(V v, u32 k) { return (k < 4u ? v.x : v.y) >> (8u * (k & 3u)); }
};

// Per-lane state of a workgroup's tile: one stripe's row segment, G waves x 64 lanes x WB columns.
template <int G, int WB = 4> struct Tile {
    typedef typename Lane<WB>::V V;
    static constexpr u32 RS = G * 64u * WB;  // LDS row stride
    u8 *lds8;
    u32 wv, lane, col_local, vcol, vsh, sc, seg0, lseg, nb, tail, olen;
    bool wide_tail;
    u32 out_stride;
    __amdgpu_buffer_rsrc_t rs_in, rs_out, rs_scr;
    u32 nbase[20];  // slice byte offset of internal node i (rotated)

    TEC_DFI Tile(const Args &a, u8 *lds) {
        lds8 = lds;
        wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        lane = threadIdx.x & 63u;
        col_local = threadIdx.x * (u32)WB;
        const u32 nbk = gridDim.x, b = blockIdx.x, full = nbk & ~7u;  // XCD-contiguous tiles (dev_io.hpp xcd_tile)
        const u32 tile = b >= full ? b : (b & 7u) * (full >> 3) + (b >> 3);
        const u32 job = tile / a.wgs_per_stripe, seg = tile - job * a.wgs_per_stripe;
        const Job &J = a.jobs[job];
        sc = a.sc;
        out_stride = (u32)a.out_stride;
        seg0 = seg * RS;
        lseg = a.sc - seg0 < RS ? a.sc - seg0 : RS;
        u32 w = seg * G * 64u + threadIdx.x;
        if (w >= a.wps) w = a.wps - 1;
        const u32 col = w * (u32)WB;
        // the word's high part is past the sub-chunk: load the row's last WB bytes instead
        const bool tailw = col + WB > a.sc;
        vcol = tailw ? a.sc - WB : col;
        vsh = col - vcol;
        rs_in = __builtin_amdgcn_make_buffer_rsrc((void *)J.in, 0, (int)(u32)(a.n * a.in_stride), 0x00020000);
        rs_out = __builtin_amdgcn_make_buffer_rsrc((void *)J.out, 0, (int)(u32)J.out_len, 0x00020000);
        const u32 nscr = a.nscratch ? a.nscratch : 1u;
        rs_scr = __builtin_amdgcn_make_buffer_rsrc(a.scratch + (u64)tile * nscr * RS, 0, (int)(nscr * RS), 0x00020000);
        for (u32 i = 0; i < 20u; i++) {
            const u32 s = i + J.rot;
            nbase[i] = (s >= a.n ? s - a.n : s) * (u32)a.in_stride;
        }
        nb = lseg >> 4;
        tail = lseg & 15u;
        wide_tail = tail != 0 && nb > 0;
        olen = (u32)J.out_len;
    }
    TEC_DFI V ld(u32 node, u32 plane) const { return Lane<WB>::ld(rs_in, vcol, nbase[node] + plane * sc); }
    // direct output (TEC_DFIX_RAW) stores every word back at the column it was loaded from and the
    // arithmetic is byte-wise, so words stay in load order; staged rows need column order
#ifdef TEC_DFIX_RAW
    TEC_DFI V rot(V v) const { return v; }
#else
    TEC_DFI V rot(V v) const { return Lane<WB>::rot(v, vsh); }
#endif
    TEC_DFI V lds_ld(u32 row) const { return *reinterpret_cast<const V *>(lds8 + row * RS + col_local); }
    TEC_DFI void lds_st(u32 row, V v) const { *reinterpret_cast<V *>(lds8 + row * RS + col_local) = v; }
    TEC_DFI V scr_ld(u32 row) const { return Lane<WB>::ld(rs_scr, col_local, row * RS); }
    TEC_DFI void scr_st(u32 row, V v) const { Lane<WB>::template st<0>(v, rs_scr, col_local, row * RS); }
    // one decoded word straight to data chunk x at plane z: every lane stores its word where it
    // loaded it (vcol: a tail lane's columns overlap its neighbour's, same values); a word across
    // the stripe's output share is written byte by byte (the range check drops whole dwords)
    TEC_DFI void out_st(u32 x, u32 z, V v) const {
        const u32 o = x * out_stride + z * sc + vcol;
#ifdef TEC_DFIX_RAW
        const V w = v;
#else
        const V w = Lane<WB>::unrot(v, vsh);
#endif
        if (o + (u32)WB > olen && o < olen) {
            for (u32 k = 0; k < (u32)WB; k++) __builtin_amdgcn_raw_buffer_store_b8((u8)Lane<WB>::byte(w, k), rs_out, (int)(o + k), 0, 0);
        } else {
            Lane<WB>::template st<2>(w, rs_out, o, 0);
        }
    }
    TEC_DFI void barrier() const { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

    // this wave's share [wv n / G, (wv + 1) n / G) of the step's n staged rows -> data chunk x
    // at plane z, item r = x | z << 8 (a uniform loop; the items are scalar-loaded after the
    // barrier), each row whole by one wave, trimmed at the stripe's output share
    TEC_DFI void flush(u32 row0, const unsigned short *items, u32 n) const {
        typedef u32 u32x4 __attribute__((ext_vector_type(4)));
        constexpr u32 kDrop = 0x80000000u;
        const u32 r_end = ((wv + 1) * n) / G;
#pragma unroll 1
        for (u32 i = (wv * n) / G; i < r_end; i++) {
            const u32 it = items[i];
            const u8 *r = lds8 + (row0 + i) * RS;
            const u32 off = (it & 0xffu) * out_stride + (it >> 8) * sc + seg0;
#pragma unroll
            for (u32 h = 0; h < (RS > 1024u ? 2u : 1u); h++) {
                const u32 b = lane + h * 64u;
                const u32 vo = b < nb ? b * 16u : ((wide_tail && b == nb) ? lseg - 16u : kDrop), lo = vo == kDrop ? 0u : vo;
                const u32x4 v = *reinterpret_cast<const u32x4 *>(r + lo);
                if (vo == kDrop || off + vo + 16u <= olen) {
                    __builtin_amdgcn_raw_buffer_store_b128(v, rs_out, (int)vo, (int)off, 2);
                } else {  // bytes past out_len fail the range check
#pragma unroll 1
                    for (u32 k = 0; k < 16u; k++)
                        __builtin_amdgcn_raw_buffer_store_b8((u8)(v[k >> 2] >> (8u * (k & 3u))), rs_out, (int)(vo + k), (int)off, 0);
                }
            }
            if (!wide_tail) {
                const u32 lt = nb * 16u + lane * 2u, vot = lane < (tail >> 1) ? lt : kDrop;
                const unsigned short v = *reinterpret_cast<const unsigned short *>(r + lt);
                if (vot == kDrop || off + vot + 2u <= olen)
                    __builtin_amdgcn_raw_buffer_store_b16(v, rs_out, (int)vot, (int)off, 0);
                else
                    __builtin_amdgcn_raw_buffer_store_b8((u8)v, rs_out, (int)vot, (int)off, 0);
            }
        }
    }
};

}  // namespace dfix
}  // namespace tec
