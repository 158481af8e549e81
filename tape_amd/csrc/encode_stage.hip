// encode_stage.hip -- Clay layered encode for the q = 10, t = 2 profiles (n = 20, d = k + 9):
// the production profile (20,7,16) (lib/core/src/encoding.rs:236-239) and the reference test
// profile (20,10,19).  Replaces ClayCoder::encode -> clay_codes::ClayCode::encode
// (lib/slicer/src/clay.rs:99-104) inside Slicer::encode's per-stripe loop (slicer.rs:268-286),
// fused with the rotation scatter `distribute_chunks` (slicer.rs:60-71).
//
// Algebra (encode = decode_layered with the parity nodes erased):
//   plane z = 10*z0 + z1; nodes (x, y), y = 0 for nodes 0..9, y = 1 for nodes 10..19; data
//   nodes are x < K in column 0.  Column-0 couplings join planes of equal z1, column-1
//   couplings join planes of equal z0 (a "row" of planes).  Planes with z0 < K are decode
//   level 1, z0 >= K level 2 (their column-0 partners are level-1 parity of the same z1).
//
// Work decomposition (MI355X):
//   * compute: a workgroup owns one stripe's row segment (G <= 6 waves x 64 lanes x 4 columns,
//     the whole 1,430-byte row for 1 MB stripes) and walks the 100 planes in decode order; a
//     lane owns one 4-column word of every plane, so every coupling partner is either an input,
//     a value this lane parked earlier, or (level 2) a level-1 output re-read from HBM.
//   * store: HBM writes reach streaming rate only when each 128-byte line is written whole by
//     ONE wave (scripts/vmem_bench5-7: a row split between two waves 3.0 TB/s, whole rows by one
//     wave 4.8 TB/s, streaming 5.8).  So every value is first staged in LDS at its column
//     position (aligned ds_write_b32), and after a workgroup barrier the finished rows are
//     written out one whole row per wave (aligned ds_read_b128 -> 16 B per lane, contiguous
//     wave stores; a row's 2-aligned start costs nothing, vmem_bench6 T4).
//   * column-1 pairs (U of plane (z0, j) meets U of (z0, s)) are parked in LDS "slot rows" of
//     the same layout; when the pair finishes, the burst row C(10+s, (z0, j)) is written back
//     into its slot row in place and flushed from there -- no copy.
//   * level-2 column-0 pairs park their U in a per-stripe global scratch (same lane, same
//     address: program order), 30 rows per stripe.
// Coefficients (generator, PFT) are constexpr: each GF product is a fixed XOR selection of
// xtime multiples, or a 2-bit v_perm lookup with SGPR tables for one-off heavy constants.
#include "kernels.hpp"
#include "gf_dev.hpp"
#include "dev_io.hpp"

namespace tec {
namespace stage {

constexpr int kQ = 10;
constexpr int kMaxG = 6;           // waves (64-word column groups) per workgroup
constexpr int kStageRows = 22;     // staging rows: node r's row of this plane + 2 level-2 extras
constexpr int kScratchRows = 30;   // level-2 parked U rows per stripe segment

template <int K>
struct Consts {
    uint8_t G[20][K];   // systematic generator (rows >= K used)
    uint8_t Gt[kQ][K];  // column-0 parity rows pre-scaled for level-1 type-1 recovery: t_u * G
};

template <int K>
constexpr Consts<K> make_consts() {
    Consts<K> rc{};
    const Mat g = rs_generator(K, 20);
    for (int r = 0; r < 20; r++)
        for (int x = 0; x < K; x++) rc.G[r][x] = g.v[r][x];
    for (int r = K; r < kQ; r++)
        for (int x = 0; x < K; x++) rc.Gt[r][x] = gf_mul(kPft.t_u[1], g.v[r][x]);
    return rc;
}

// The pairwise transform of this field (A3: RS(2,2) parity [[3,2],[2,3]]) is orientation-free:
// uncoupling (U = 3C + 2C') and re-coupling (C = 3U + 2U') are both  a -> a ^ 2(a ^ b).
static_assert(kPft.u_c[0] == 3 && kPft.u_c[1] == 3 && kPft.u_p[0] == 2 && kPft.u_p[1] == 2, "PFT uncouple");
static_assert(kPft.c_u[0] == 3 && kPft.c_u[1] == 3 && kPft.c_p[0] == 2 && kPft.c_p[1] == 2, "PFT couple");
__device__ __forceinline__ uint32_t pft3(uint32_t a, uint32_t b) { return a ^ xt(a ^ b); }

// Column-1 pair (i, j), i < j, of a row: U(10+j, (z0, i)) is parked at plane i and consumed at
// plane j, where the finished C(10+j, (z0, i)) is written back into the same slot row and
// flushed.  So a slot consumed at plane j is reusable from plane j + 1 on: interval colouring
// with that rule needs 29 slots (max over p of (p+1)(10-p) - 1).
struct PairSlots {
    uint8_t slot[kQ][kQ];
    int nslots;
};
constexpr PairSlots make_pair_slots() {
    PairSlots ps{};
    int busy_until[64];
    for (int i = 0; i < 64; i++) busy_until[i] = -1;  // step at which the slot is last read
    for (int p = 0; p < kQ; p++) {
        for (int j = p + 1; j < kQ; j++) {
            int sl = 0;
            while (busy_until[sl] >= p) sl++;
            busy_until[sl] = j;
            ps.slot[p][j] = (uint8_t)sl;
            if (sl + 1 > ps.nslots) ps.nslots = sl + 1;
        }
    }
    return ps;
}
constexpr PairSlots kSlots = make_pair_slots();
static_assert(kSlots.nslots == 29, "row pairs need 29 slots");
constexpr int kSlotRows = 29;
constexpr int kLdsRows = kStageRows + kSlotRows;



// Flush schedule: for each step type (0 = level 1; 1 + i0 = level-2 plane row z0 = K + i0) and
// plane s, the rows that are final after the step, in ascending node order (a column-1 burst in
// ascending plane order), split into contiguous per-wave shares for G waves.  Item = LDS row
// (0..21 staging, 22 + slot) | node << 8 | target z0 << 16 (0xff: this step's z0) | target s << 24.
constexpr int kMaxItems = 32;
template <int G>
struct FlushTab {
    static constexpr int kCap = (kMaxItems + G - 1) / G;  // items per wave
    struct W {
        uint32_t n;
        uint32_t item[kCap];
    } w[4][kQ][G];
};
constexpr uint32_t fitem(int lds, int node, int z0, int s) {
    return (uint32_t)lds | ((uint32_t)node << 8) | ((uint32_t)(z0 & 0xff) << 16) | ((uint32_t)s << 24);
}
template <int K, int G>
constexpr FlushTab<G> make_flush_tab() {
    FlushTab<G> t{};
    constexpr int NP0 = kQ - K;
    for (int type = 0; type < (NP0 ? 4 : 1); type++) {
        const int i0 = type - 1;
        for (int s = 0; s < kQ; s++) {
            uint32_t items[kMaxItems] = {};
            int n = 0;
            for (int r = 0; r < 20; r++) {
                if (r < K) {
                    items[n++] = fitem(r, r, -1, s);
                } else if (r < kQ) {
                    const int ri = r - K;
                    if (type == 0 || ri <= i0) items[n++] = fitem(r, r, -1, s);  // level 1 / red / finished pair
                } else {
                    const int j = r - kQ;
                    if (j < s) items[n++] = fitem(r, r, -1, s);
                    if (j == s) {
                        for (int jj = 0; jj < s; jj++) items[n++] = fitem(kStageRows + kSlots.slot[jj][s], r, -1, jj);
                        items[n++] = fitem(r, r, -1, s);
                    }
                }
            }
            for (int i = 0; i < i0; i++) items[n++] = fitem(20 + i, K + i0, K + i, s);  // C(K+i0, (K+i, s))
            for (int w = 0; w < G; w++) {
                const int b = w * n / G, e = (w + 1) * n / G;
                t.w[type][s][w].n = (uint32_t)(e - b);
                for (int i = b; i < e; i++) t.w[type][s][w].item[i - b] = items[i];
            }
        }
    }
    return t;
}
template <int K, int G>
struct FlushHolder {
    static __constant__ FlushTab<G> tab;
};
template <int K, int G>
__constant__ FlushTab<G> FlushHolder<K, G>::tab = make_flush_tab<K, G>();

// Column-1 LDS byte offsets of step s, pair index j (row * RS): rd = the row holding
// U(10+s, (z0, j)) when j < s (any row otherwise); wr = where the step's j value goes: the burst
// C(10+s, (z0, j)) in place (j < s), the parked U(10+j, (z0, s)) (j > s), or node 10+s's
// staging row again (j == s).
template <int G>
struct Col1Off {
    uint32_t rd[kQ][kQ], wr[kQ][kQ];
};
template <int G>
constexpr Col1Off<G> make_col1_off() {
    Col1Off<G> t{};
    for (int s = 0; s < kQ; s++)
        for (int j = 0; j < kQ; j++) {
            const int row = j < s ? kStageRows + kSlots.slot[j][s] : (j > s ? kStageRows + kSlots.slot[s][j] : kQ + s);
            t.rd[s][j] = t.wr[s][j] = (uint32_t)row * G * 256u;
        }
    return t;
}
template <int G>
struct Col1Holder {
    static __constant__ Col1Off<G> tab;
};
template <int G>
__constant__ Col1Off<G> Col1Holder<G>::tab = make_col1_off<G>();

#ifndef TEC_STAGE_ST_AUX
#define TEC_STAGE_ST_AUX 2  // cache policy of the slice stores (gfx950: 2 = nt, 16 = sc1): nt measured 2 % faster
#endif
#ifndef TEC_STAGE_PRIO
#define TEC_STAGE_PRIO 1  // wave priority during a step's compute (s_setprio), 0 = off
#endif
#ifndef TEC_STAGE_OWN_AUX
#define TEC_STAGE_OWN_AUX 0  // cache policy of the level-1 own-row loads
#endif
#ifndef TEC_STAGE_PART_AUX
#define TEC_STAGE_PART_AUX 0  // cache policy of the level-1 partner-row loads
#endif
#ifndef TEC_STAGE_PF
#define TEC_STAGE_PF 1  // planes of load lookahead (1 or 2)
#endif
#ifndef TEC_STAGE_WAVES_PER_EU
#define TEC_STAGE_WAVES_PER_EU 3
#endif

#ifndef TEC_STAGE_ABLATE
#define TEC_STAGE_ABLATE 0  // timing builds only (scripts/kbench.hip): bit0 no flush stores,
#endif                      // bit1 no barriers, bit2 trivial MDS, bit3 no global loads
template <int AUX = 0>
__device__ __forceinline__ uint32_t gload(__amdgpu_buffer_rsrc_t rs, uint32_t vo, uint32_t so) {
    if constexpr (TEC_STAGE_ABLATE & 8) return vo * 0x9e3779b1u ^ so;
    return __builtin_amdgcn_raw_buffer_load_b32(rs, (int)vo, (int)so, AUX);
}
__device__ __forceinline__ void step_barrier() {
    if constexpr (!(TEC_STAGE_ABLATE & 2)) lds_barrier();
}
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

inline size_t lds_bytes(uint32_t g) { return (size_t)kLdsRows * g * 256u; }

// acc[r] ^= sum_x coef(r, x) * u[x] for the 20-K parity rows, coefficients folded at compile
// time: per input the xtime multiples 2^i u[x], then every row XORs the multiples its
// coefficient selects, two at a time (v_bitop3 xor3), a leftover single carried to the next
// input so each row costs ~ceil(terms / 2) instructions.
template <int K, bool SCALED>
__device__ __forceinline__ void mds_rows(const uint32_t *u, uint32_t *acc) {
    constexpr Consts<K> RC = make_consts<K>();
    constexpr int NR = 20 - K;
    uint32_t pend[NR];
    bool hp[NR];  // compile-time after unrolling
#pragma unroll
    for (int r = 0; r < NR; r++) { acc[r] = 0; hp[r] = false; pend[r] = 0; }
#pragma unroll
    for (int x = 0; x < K; x++) {
        if constexpr (TEC_STAGE_ABLATE & 4) {
#pragma unroll
            for (int r = 0; r < NR; r++) acc[r] ^= u[x] + r;
            continue;
        }
        const Mult<7> mu(u[x]);
#pragma unroll
        for (int r = 0; r < NR; r++) {
            const uint8_t c = (K + r < kQ && SCALED) ? RC.Gt[K + r][x] : RC.G[K + r][x];
#pragma unroll
            for (int i = 0; i < 8; i++) {
                if (!(c >> i & 1)) continue;
                if (hp[r]) {
                    acc[r] = xor3(acc[r], pend[r], mu.m[i]);
                    hp[r] = false;
                } else {
                    pend[r] = mu.m[i];
                    hp[r] = true;
                }
            }
        }
    }
#pragma unroll
    for (int r = 0; r < NR; r++)
        if (hp[r]) acc[r] ^= pend[r];
}

// MASKED: the stripe's data end is not dword aligned (only an object's last stripe, when its
// length is not a multiple of 4): words are masked per lane instead of relying on the range check.
// G: waves per workgroup = 64-word column groups of the row segment (compile-time row stride).
template <int K, int G, bool MASKED>
__global__ void __launch_bounds__(G * 64, TEC_STAGE_WAVES_PER_EU) enc_stage_kernel(EncArgs a) {
    constexpr int NP0 = kQ - K;  // column-0 parity nodes
    static_assert(NP0 == 0 || NP0 == 3, "fast encode covers k = 7 and k = 10");
    constexpr uint32_t RS = G * 256u;  // LDS row stride (bytes)
    constexpr int CAP = FlushTab<G>::kCap;
    const FlushTab<G> &FT = FlushHolder<K, G>::tab;
    const Col1Off<G> &C1 = Col1Holder<G>::tab;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    uint8_t *const lds8 = reinterpret_cast<uint8_t *>(lds);  // rows [0, 22) staging, then 29 slot rows

    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t col_local = threadIdx.x * 4u;  // column within the segment

    const uint32_t tile = xcd_tile(blockIdx.x, gridDim.x);
    const uint32_t job = tile / a.wgs_per_stripe, seg = tile - job * a.wgs_per_stripe;
    const EncJob J = a.jobs[job];
    const uint32_t cs = a.cs, sc = a.sc, slen = a.slice_len, wps = a.words_per_stripe;
    const uint32_t seg0 = seg * RS;               // first column of the segment
    const uint32_t lseg = min(RS, sc - seg0);     // columns of the segment
    // Word of this lane (lanes past the stripe's last word redo it; their LDS columns lie past
    // the segment and are never flushed).  When sc = 2 mod 4 the last word's high half belongs to
    // the next sub-chunk: it lands past `lseg` in LDS too.
    uint32_t w = seg * G * 64u + threadIdx.x;
    if (w >= wps) w = wps - 1;
    const uint32_t col = w * 4u;
    // Buffer resources (32-bit offsets).  The input resource starts at J.src rounded down to 4
    // bytes and ends exactly at the stripe's last data byte, so the range check returns the zero
    // padding of Slicer::encode (slicer.rs:276-283) for every dword past the data.
    const uint32_t src_len = (uint32_t)J.src_len;
    const uint32_t src_al = (uint32_t)reinterpret_cast<uintptr_t>(J.src) & 3u;
    const int src_range = (int)(MASKED ? (src_len + src_al + 3u) & ~3u : src_len + src_al);
    const __amdgpu_buffer_rsrc_t rs_src =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(J.src - src_al), 0, src_range, 0x00020000);
    // output range = the object's n slices as seen from this stripe's base (< 2^31, host-checked)
    const uint32_t dst_range = a.n * slen - J.dst_skew;
    const __amdgpu_buffer_rsrc_t rs_dst = __builtin_amdgcn_make_buffer_rsrc(J.dst, 0, (int)dst_range, 0x00020000);
    // level-2 parking: kScratchRows rows of this segment, lane-private columns
    uint8_t *const scr = a.scratch + (size_t)tile * kScratchRows * RS;
    const __amdgpu_buffer_rsrc_t rs_scr =
        __builtin_amdgcn_make_buffer_rsrc(scr, 0, (int)(kScratchRows * RS), 0x00020000);
    // slice byte offset of node i in lane i (read back with v_readlane for uniform nodes)
    uint32_t sl_lane = lane + J.rot;
    sl_lane = (sl_lane >= 20u ? sl_lane - 20u : sl_lane) * slen;
    auto slice_off = [&](uint32_t node) -> uint32_t { return __builtin_amdgcn_readlane(sl_lane, node); };
    // per-lane load offsets: own rows x*cs + col, partner rows 10*x*sc + col
    uint32_t vo_own[K], vo_part[kQ];
#pragma unroll
    for (int x = 0; x < K; x++) vo_own[x] = col + (uint32_t)x * cs;
#pragma unroll
    for (int x = 0; x < kQ; x++) vo_part[x] = col + (uint32_t)x * kQ * sc;
    auto ld_pair = [&](__amdgpu_buffer_rsrc_t rs, uint32_t o) -> uint32_t {
        const uint32_t lo = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(o & ~3u), 0, 0);
        const uint32_t hi = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)((o & ~3u) + 4u), 0, 0);
        return __builtin_amdgcn_alignbyte(hi, lo, o & 3u);
    };
    auto keep_mask = [&](uint32_t off) -> uint32_t {  // MASKED: bytes of the word below src_len
        const int rem = (int)src_len - (int)off;
        return rem >= 4 ? 0xffffffffu : (rem <= 0 ? 0u : (1u << (8 * rem)) - 1u);
    };
    // staging row r at this lane's column (compile-time offset)
    auto stage = [&](int r, uint32_t v) { *reinterpret_cast<uint32_t *>(lds8 + r * RS + col_local) = v; };
    // Words load as ONE dword at their (2-aligned) address.  The range check zeroes a dword that
    // straddles the end of the resource, so the single word of the stripe that straddles the
    // data end would read as 0: its row ("end row", node ex, plane ez) is fetched once here with
    // aligned pairs (+ byte mask) and substituted wherever that row is used.
    const uint32_t last = src_len ? src_len - 1u : 0u;
    const uint32_t ex = src_len ? last / cs : 0xffffu, ez = src_len ? (last - ex * cs) / sc : 0xffffu;
    uint32_t fixw = 0;
    if (src_len) {
        const uint32_t off = ex * cs + ez * sc + col;
        fixw = ld_pair(rs_src, src_al + off);
        if constexpr (MASKED) fixw &= keep_mask(off);
    }
    // level-2 park index of U(K+r, (z0, *)): (7,1) -> 0, (7,2) -> 1, (8,2) -> 2   [K = 7]
    auto pidx = [](uint32_t z0, int r) -> uint32_t { return z0 == (uint32_t)K ? (uint32_t)r - 1u : 2u; };

    // Loads of plane (z0, s).  own[x] = C(x, (z0, s)) for the data nodes; part[x] = the
    // column-0 partner C(z0, (x, s)): an input chunk at level 1 (z0 < K); at level 2 a level-1
    // parity row re-read from HBM (x < K) or a U this lane parked in scratch (K <= x < z0).
    uint32_t own[K], part[kQ];    // plane t + 1
    uint32_t own2[K], part2[kQ];  // plane t + 2 (TEC_STAGE_PF == 2)
    auto load_own_to = [&](uint32_t(&o)[K], uint32_t z0, uint32_t s) {
        const uint32_t so = src_al + (z0 * kQ + s) * sc;
#pragma unroll
        for (int x = 0; x < K; x++) o[x] = gload<TEC_STAGE_OWN_AUX>(rs_src, vo_own[x], so);
    };
    auto load_part_to = [&](uint32_t(&part)[kQ], uint32_t z0, uint32_t s) {
        if (z0 < (uint32_t)K) {
            const uint32_t so = src_al + z0 * cs + s * sc;
#pragma unroll
            for (int x = 0; x < kQ; x++) part[x] = gload<TEC_STAGE_PART_AUX>(rs_src, vo_part[x], so);
        } else {
            // level-1 outputs of other waves: written before the level-1 -> level-2 drain
            // (vmcnt(0) + barrier); nt loads skip this CU's L1
            const uint32_t so = slice_off(z0) + s * sc;
#pragma unroll
            for (int x = 0; x < K; x++) part[x] = gload<2>(rs_dst, vo_part[x], so);
#pragma unroll
            for (int i = 0; i < NP0; i++) {
                // U(z0, (K+i, s)) parked at plane (K+i, s) with r = z0 - K
                const uint32_t so2 = (uint32_t)(K + i) < z0 ? (pidx((uint32_t)(K + i), (int)z0 - K) * kQ + s) * RS : 0x80000000u;
                part[K + i] = gload(rs_scr, col_local, so2);
            }
        }
    };
    // Column 1 of plane (z0, s): u1[j] = U(10+j, (z0, s)).  Red node (j == s): C = U.  Pair
    // (10+j at (z0, s)) <-> (10+s at (z0, j)): for j < s the partner U was parked at plane
    // (z0, j); both C's are final now (the burst one in place in its slot row).  For j > s this
    // plane's half is parked.  Branch-free: every LDS row comes from the per-step table.
    auto col1 = [&](const uint32_t *u1, uint32_t s) {
        uint32_t pu[kQ];
#pragma unroll
        for (int j = 0; j < kQ; j++) pu[j] = *reinterpret_cast<const uint32_t *>(lds8 + C1.rd[s][j] + col_local);
#pragma unroll
        for (int j = 0; j < kQ; j++) {
            const bool lt = (uint32_t)j < s;          // pair finishes now (else: red, or park)
            const uint32_t tt = xt(u1[j] ^ pu[j]);
            stage(kQ + j, lt ? u1[j] ^ tt : u1[j]);  // C(10+j, (z0, s)); rows j > s are not flushed
            *reinterpret_cast<uint32_t *>(lds8 + C1.wr[s][j] + col_local) = lt ? pu[j] ^ tt : u1[j];
        }
    };
    // Write the rows the step finished: this wave's share of the step's items; per row, 16 B
    // per lane from LDS (aligned) to the slice (whole row by this wave).  With G = 6 all the
    // wave's rows are read into registers first; then the workgroup barrier that frees the LDS
    // rows for the next step (B1), then the stores -- a wave held up by a full store queue no
    // longer holds the others.
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    // Branch-free row copy: every lane reads its LDS bytes unconditionally (past the row: junk
    // from the next row, or 0 past the allocation) and a lane with nothing to write stores at an
    // out-of-range offset, which the buffer range check drops.
    // A row's last partial block (lseg % 16 bytes) is covered by one more lane storing the row's
    // LAST 16 bytes (overlapping bytes rewritten with the same values; its LDS read is the only
    // unaligned one) -- no separate narrow store per row.  Rows shorter than 16 bytes fall back
    // to 16-bit stores.
    const uint32_t nb = lseg >> 4, tail = lseg & 15u;
    constexpr uint32_t kDrop = 0x80000000u;
    const bool wide_tail = tail != 0 && nb > 0;
    auto blk_off = [&](uint32_t b) -> uint32_t {  // byte offset of lane block b, kDrop if none
        return b < nb ? b * 16u : ((wide_tail && b == nb) ? lseg - 16u : kDrop);
    };
    const uint32_t vo0 = blk_off(lane), vo1 = blk_off(lane + 64u);
    const uint32_t lo0 = vo0 == kDrop ? 0u : vo0, lo1 = vo1 == kDrop ? 0u : vo1;  // LDS offsets
    const uint32_t vot = (!wide_tail && lane < (tail >> 1)) ? nb * 16u + lane * 2u : kDrop;
    const uint32_t lt_off = nb * 16u + lane * 2u;  // 16-bit tail LDS offset (short rows only)
    auto item_off = [&](uint32_t it, uint32_t z0) -> uint32_t {
        const uint32_t node = (it >> 8) & 0xffu, tz0 = (it >> 16) & 0xffu, ts = it >> 24;
        const uint32_t plane = (tz0 == 0xffu ? z0 : tz0) * kQ + ts;
        return slice_off(node) + plane * sc + seg0;  // uniform
    };
    auto st128 = [&](u32x4 v, uint32_t vo, uint32_t off) {
        if constexpr (TEC_STAGE_ABLATE & 1) {
            if (v.x == 0x12345678u) __builtin_amdgcn_raw_buffer_store_b32(v.y, rs_dst, (int)vo, (int)off, 0);
        } else {
            __builtin_amdgcn_raw_buffer_store_b128(v, rs_dst, (int)vo, (int)off, TEC_STAGE_ST_AUX);
        }
    };
    auto st16 = [&](uint32_t v, uint32_t off) {
        if constexpr (!(TEC_STAGE_ABLATE & 1)) __builtin_amdgcn_raw_buffer_store_b16((uint16_t)v, rs_dst, (int)vot, (int)off, 0);
    };
    auto rd128 = [&](const uint8_t *row, uint32_t o) -> u32x4 { return *reinterpret_cast<const u32x4 *>(row + o); };
    auto flush = [&](const typename FlushTab<G>::W &F, uint32_t z0) {
        const uint32_t n = F.n;
        if constexpr (CAP <= 6) {
            u32x4 d0[CAP], d1[CAP];
            uint32_t dt[CAP];
#pragma unroll
            for (int q = 0; q < CAP; q++) {
                if ((uint32_t)q < n) {
                    const uint8_t *row = lds8 + (F.item[q] & 0xffu) * RS;
                    d0[q] = rd128(row, lo0);
                    if (RS > 1024u) d1[q] = rd128(row, lo1);
                    if (!wide_tail) dt[q] = *reinterpret_cast<const uint16_t *>(row + lt_off);
                }
            }
            step_barrier();  // B1
#pragma unroll
            for (int q = 0; q < CAP; q++) {
                if ((uint32_t)q < n) {
                    const uint32_t off = item_off(F.item[q], z0);
                    st128(d0[q], vo0, off);
                    if (RS > 1024u) st128(d1[q], vo1, off);
                    if (!wide_tail) st16(dt[q], off);
                }
            }
        } else {  // small workgroups (short rows): row by row
            for (uint32_t q = 0; q < n; q++) {
                const uint8_t *row = lds8 + (F.item[q] & 0xffu) * RS;
                const uint32_t off = item_off(F.item[q], z0);
                st128(rd128(row, lo0), vo0, off);
                if (RS > 1024u) st128(rd128(row, lo1), vo1, off);
                if (!wide_tail) st16(*reinterpret_cast<const uint16_t *>(row + lt_off), off);
            }
            step_barrier();  // B1
        }
    };

    // Planes in decode order.  Loads of the next plane (own and partners) are issued before this
    // one is computed, except across the level-1 -> level-2 boundary, where the partners are
    // level-1 rows other waves stored: there every wave drains its stores (vmcnt(0)) and the
    // workgroup syncs first.
    // With TEC_STAGE_PF == 2 the loads run two planes ahead; the partner loads of (K, 0) and
    // (K, 1) then wait for the boundary drain.
    load_own_to(own, 0, 0);
    load_part_to(part, 0, 0);
    if constexpr (TEC_STAGE_PF == 2) {
        load_own_to(own2, 0, 1);
        load_part_to(part2, 0, 1);
    }
    for (uint32_t z0 = 0; z0 < (uint32_t)kQ; z0++) {
#pragma unroll 2
        for (uint32_t s = 0; s < (uint32_t)kQ; s++) {
            const uint32_t z = z0 * kQ + s;
            uint32_t cown[K], cpart[kQ];
#pragma unroll
            for (int x = 0; x < K; x++) cown[x] = own[x];
#pragma unroll
            for (int x = 0; x < kQ; x++) cpart[x] = part[x];
            if constexpr (TEC_STAGE_PF == 2) {
#pragma unroll
                for (int x = 0; x < K; x++) own[x] = own2[x];
#pragma unroll
                for (int x = 0; x < kQ; x++) part[x] = part2[x];
            }
            if (z == ez) {  // end-row substitution (see fixw)
#pragma unroll
                for (int x = 0; x < K; x++) cown[x] = (uint32_t)x == ex ? fixw : cown[x];
            }
            if (z0 == ex && z0 < (uint32_t)K && s == ez % kQ) {
#pragma unroll
                for (int x = 0; x < kQ; x++) cpart[x] = (uint32_t)x == ez / kQ ? fixw : cpart[x];
            }
            const bool boundary = NP0 > 0 && z0 + 1 == (uint32_t)K && s + 1 == (uint32_t)kQ;
            if (z + TEC_STAGE_PF < (uint32_t)(kQ * kQ)) {
                const uint32_t t2 = z + TEC_STAGE_PF, nz0 = t2 / kQ, ns = t2 - nz0 * kQ;
                // partners of level-2 planes are level-1 rows: only after the boundary drain
                const bool after_drain = NP0 == 0 || nz0 < (uint32_t)K || z0 >= (uint32_t)K;
                if constexpr (TEC_STAGE_PF == 2) {
                    load_own_to(own2, nz0, ns);
                    if (after_drain) load_part_to(part2, nz0, ns);
                } else {
                    load_own_to(own, nz0, ns);
                    if (after_drain) load_part_to(part, nz0, ns);
                }
            }
            if (z0 < (uint32_t)K) {
                // ---- level 1: data partners are inputs; column-0 parity by type-1 recovery ----
                if constexpr (TEC_STAGE_PRIO) __builtin_amdgcn_s_setprio(TEC_STAGE_PRIO);
                uint32_t u[K];
#pragma unroll
                for (int x = 0; x < K; x++) {
                    stage(x, cown[x]);  // systematic chunk
                    u[x] = (uint32_t)x == z0 ? cown[x] : pft3(cown[x], cpart[x]);
                }
                uint32_t acc[20 - K];
                mds_rows<K, true>(u, acc);
#pragma unroll
                for (int r = K; r < kQ; r++) stage(r, acc[r - K] ^ mulc(kPft.t_p[1], cpart[r]));
                col1(acc + NP0, s);
                if constexpr (TEC_STAGE_PRIO) __builtin_amdgcn_s_setprio(0);
                step_barrier();  // B2: the step's rows are staged
                flush(FT.w[0][s][wv], z0);
                if (boundary) {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    __syncthreads();
                    load_part_to(part, (uint32_t)K, 0);
                    if constexpr (TEC_STAGE_PF == 2) load_part_to(part2, (uint32_t)K, 1);
                }
            } else if constexpr (NP0 > 0) {
                // ---- level 2: data partners are the level-1 column-0 parity C(z0, (x, s)) ----
                if constexpr (TEC_STAGE_PRIO) __builtin_amdgcn_s_setprio(TEC_STAGE_PRIO);
                uint32_t u[K];
#pragma unroll
                for (int x = 0; x < K; x++) {
                    stage(x, cown[x]);
                    u[x] = pft3(cown[x], cpart[x]);  // x < K <= z0
                }
                uint32_t acc[20 - K];
                mds_rows<K, false>(u, acc);
                // column-0 parity K+r at plane (z0, s): red when K+r == z0 (C = U); paired with
                // (z0, (K+r, s)) otherwise, finished at the later of the two planes: the earlier
                // one parks its U in scratch, the later one loaded it as cpart[K + i].
                const int i0 = (int)z0 - K;
#pragma unroll
                for (int i = 0; i < NP0; i++) {
                    if (i >= i0) break;
                    const uint32_t us = cpart[K + i];  // U(K+i0, (K+i, s)), parked
                    const uint32_t up = acc[i];        // U(K+i, (K+i0, s))
                    const uint32_t tt = xt(us ^ up);
                    stage(20 + i, us ^ tt);  // C(K+i0, (K+i, s))
                    stage(K + i, up ^ tt);   // C(K+i, (z0, s))
                }
#pragma unroll
                for (int r = 0; r < NP0; r++) {
                    if (r == i0) stage(K + r, acc[r]);  // red: C = U
                    if (r > i0)
                        __builtin_amdgcn_raw_buffer_store_b32(acc[r], rs_scr, (int)col_local,
                                                              (int)((pidx(z0, r) * kQ + s) * RS), 0);
                }
                col1(acc + NP0, s);
                if constexpr (TEC_STAGE_PRIO) __builtin_amdgcn_s_setprio(0);
                step_barrier();
                flush(FT.w[1 + i0][s][wv], z0);
            }
        }
    }
}

}  // namespace stage

// Metadata suffix (metadata.rs:22-64): the 48-byte record into each of an object's n slices.
__global__ void meta_kernel(const MetaJob *__restrict__ jobs, uint32_t njobs, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t per = n * 6u;
    if (i >= njobs * per) return;
    const uint32_t j = i / per, r = i - j * per, sl = r / 6u, wd = r - sl * 6u;
    uint8_t *p = jobs[j].dst + (uint64_t)sl * jobs[j].slice_len + 8u * wd;
    const uint64_t v = jobs[j].words[wd];
    if ((reinterpret_cast<uintptr_t>(p) & 7u) == 0) {
        *reinterpret_cast<uint64_t *>(p) = v;
    } else {
        for (int b = 0; b < 8; b++) p[b] = (uint8_t)(v >> (8 * b));
    }
}

hipError_t launch_meta(const MetaJob *jobs, uint32_t njobs, uint32_t n, hipStream_t s) {
    if (!njobs) return hipSuccess;
    const uint32_t total = njobs * n * 6u;
    hipLaunchKernelGGL(meta_kernel, dim3((total + 255) / 256), dim3(256), 0, s, jobs, njobs, n);
    return hipGetLastError();
}

// Batched gather (te_recover_batch_device's lost-slice assembly): job j copies `valid` bytes
// from src and zero-fills up to `len` at dst; 8-byte granules when src and dst are 8-aligned.
// kGatherSplit workgroups per job, so one launch replaces a memcpy per chunk.
constexpr uint32_t kGatherSplit = 8;
__global__ void __launch_bounds__(256) gather_kernel(const CopyJob *__restrict__ jobs) {
    const CopyJob J = jobs[blockIdx.x / kGatherSplit];
    const uint32_t part = blockIdx.x % kGatherSplit;
    const uint64_t len = J.len, valid = J.valid < J.len ? J.valid : J.len;
    const bool wide = ((reinterpret_cast<uintptr_t>(J.src) | reinterpret_cast<uintptr_t>(J.dst)) & 7u) == 0;
    if (wide) {
        const uint64_t words = len / 8u, per = (words + kGatherSplit - 1) / kGatherSplit;
        const uint64_t w0 = part * per, w1 = w0 + per < words ? w0 + per : words;
        const uint64_t *src = reinterpret_cast<const uint64_t *>(J.src);
        uint64_t *dst = reinterpret_cast<uint64_t *>(J.dst);
        for (uint64_t w = w0 + threadIdx.x; w < w1; w += 256u) {
            const uint64_t b = w * 8u;
            uint64_t v = 0;
            if (b + 8u <= valid) {
                v = src[w];
            } else if (b < valid) {
                for (uint32_t k = 0; k < (uint32_t)(valid - b); k++) v |= (uint64_t)J.src[b + k] << (8 * k);
            }
            dst[w] = v;
        }
        if (part == kGatherSplit - 1)
            for (uint64_t b = words * 8u + threadIdx.x; b < len; b += 256u) J.dst[b] = b < valid ? J.src[b] : 0;
    } else {
        const uint64_t per = (len + kGatherSplit - 1) / kGatherSplit;
        const uint64_t b0 = part * per, b1 = b0 + per < len ? b0 + per : len;
        for (uint64_t b = b0 + threadIdx.x; b < b1; b += 256u) J.dst[b] = b < valid ? J.src[b] : 0;
    }
}

hipError_t launch_gather(const CopyJob *jobs, uint32_t njobs, hipStream_t s) {
    if (!njobs) return hipSuccess;
    if ((uint64_t)njobs * kGatherSplit > 0x7fffffffull) return hipErrorInvalidValue;
    hipLaunchKernelGGL(gather_kernel, dim3(njobs * kGatherSplit), dim3(256), 0, s, jobs);
    return hipGetLastError();
}

bool encode_rows_supported(int n, int k, int d) { return n == 20 && d == k + 9 && (k == 7 || k == 10); }

// waves per workgroup: every column group of the stripe when they fit (kMaxG), or at most
// a.groups_per_wg when the caller set it (small batches: more, shorter workgroups per stripe)
static uint32_t stage_g(const EncArgs &a) {
    uint32_t g = a.groups_per_stripe < (uint32_t)stage::kMaxG ? a.groups_per_stripe : (uint32_t)stage::kMaxG;
    if (a.groups_per_wg && a.groups_per_wg < g) g = a.groups_per_wg;
    return g;
}

size_t encode_rows_scratch_bytes(const EncArgs &a) {
    const uint32_t g = stage_g(a);
    const uint32_t wgs = (a.groups_per_stripe + g - 1) / g;
    return (size_t)a.njobs * wgs * stage::kScratchRows * g * 256u;
}

template <int K, int G, bool MASKED>
hipError_t launch_stage_g(const EncArgs &a, uint64_t blocks, hipStream_t s) {
    const size_t lds = stage::lds_bytes(G);
    hipError_t e = ensure_dyn_lds(reinterpret_cast<const void *>(stage::enc_stage_kernel<K, G, MASKED>), lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((stage::enc_stage_kernel<K, G, MASKED>), dim3((uint32_t)blocks), dim3(G * 64), lds, s, a);
    return hipGetLastError();
}

template <int K, bool MASKED>
hipError_t launch_stage(EncArgs a, hipStream_t s) {
    if (a.njobs == 0) return hipSuccess;
    const uint32_t g = stage_g(a);
    a.groups_per_wg = g;
    a.wgs_per_stripe = (a.groups_per_stripe + g - 1) / g;
    a.stripes_per_wg = 1;
    const uint64_t blocks = (uint64_t)a.njobs * a.wgs_per_stripe;
    if (blocks > 0x7fffffffull || !a.scratch) return hipErrorInvalidValue;
    switch (g) {
        case 1: return launch_stage_g<K, 1, MASKED>(a, blocks, s);
        case 2: return launch_stage_g<K, 2, MASKED>(a, blocks, s);
        case 3: return launch_stage_g<K, 3, MASKED>(a, blocks, s);
        case 4: return launch_stage_g<K, 4, MASKED>(a, blocks, s);
        case 5: return launch_stage_g<K, 5, MASKED>(a, blocks, s);
        default: return launch_stage_g<K, 6, MASKED>(a, blocks, s);
    }
}

hipError_t launch_encode_rows(int k, bool masked, const EncArgs &a, hipStream_t s) {
    switch (k * 2 + (masked ? 1 : 0)) {
        case 14: return launch_stage<7, false>(a, s);
        case 15: return launch_stage<7, true>(a, s);
        case 20: return launch_stage<10, false>(a, s);
        case 21: return launch_stage<10, true>(a, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace tec
