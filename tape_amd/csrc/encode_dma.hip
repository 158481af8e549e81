// encode_dma.hip -- Clay(20,7,16) layered encode of 1 MB stripes (sub-chunk 1,281..1,440 bytes),
// row by row per plane.  Replaces ClayCoder::encode -> clay_codes::ClayCode::encode
// (lib/slicer/src/clay.rs:99-104) in Slicer::encode's stripe loop (slicer.rs:268-286), fused
// with distribute_chunks' rotation (slicer.rs:60-71): the production hot path.  Same algebra and
// plane order as encode_stage.hip; what differs is how bytes
// move (a row-of-planes variant that stores 14,300-byte pieces measured slower as a skeleton at
// one workgroup per CU, profiles/r04_enc_skeleton4.txt):
//   * inputs arrive by LDS-DMA (buffer_load_dwordx4 ... lds, 1 KiB per wave-instruction, from
//     2-aligned addresses -- scripts/ldsdma_probe.hip) into a two-slot ring of plane images,
//     one plane ahead, issued by a dedicated loader wave: 23 wave-instructions per plane;
//   * the compute lanes (4 byte-columns each) read their words from the image (ds_read_b32);
//   * column-1 pairs are parked in VGPRs (25 slots, compile-time indices via a switch on the
//     plane digit), not in LDS; level-2 column-0 pairs park their U in the output slice at the
//     place the pair's final C overwrites later, and are read back by the same DMA as the
//     level-1 parity rows -- no scratch buffer;
//   * systematic rows are written from the ring image (no staging copy);
//   * the compute waves issue no loads, so the compiler inserts no vmcnt waits for them: the
//     loader waits for its DMA explicitly before the barrier that hands the plane over.
// LDS: 2 x 23,552 B ring + 24 x 1,440 B staging = 81,664 B -> two workgroups (14 waves) per CU.
#include "kernels.hpp"
#include "gf_dev.hpp"
#include "dev_io.hpp"
#include "enc_common.hpp"

namespace tec {
namespace dma {

using enc::kQ;
using enc::pft3;
constexpr int K = 7;
constexpr int G = 6;                       // waves; lane word w covers columns 4w..4w+3
constexpr uint32_t RB = 90;                // 16-byte blocks per image / staging row
constexpr uint32_t RW = RB * 16;           // 1,440: row stride
constexpr uint32_t kOwnBlk = 7 * RB;       // 7 own rows, then 9 partner rows; the pieces that
constexpr uint32_t kPartBlk = 9 * RB;      // overhang a region run with those lanes masked off
constexpr uint32_t kPartBase = kOwnBlk * 16;
constexpr uint32_t kSlotBytes = (kOwnBlk + kPartBlk) * 16;
constexpr uint32_t kRing = 2;              // ring slots (planes in flight)
constexpr uint32_t kStageBase = kRing * kSlotBytes;
constexpr uint32_t kStageRows = 24;
constexpr uint32_t kLdsBytes = kStageBase + kStageRows * RW;
static_assert(kLdsBytes <= 81920 - 1024, "two workgroups per CU, with a margin");
constexpr int kOwnInstr = 10, kPartInstr = 13, kDmaInstr = kOwnInstr + kPartInstr;
constexpr int kWaves = G + 1;              // six compute waves and a loader wave that issues every DMA
// compute waves keep at most this many stores in flight before B1, so every slice row a
// later DMA reads back (level-2 partners, >= 8 steps later) has landed: <= 3 steps of stores
constexpr int kCap = 5;  // flush rows per wave per step
#ifndef TEC_DMA_STORELAG
#define TEC_DMA_STORELAG 30
#endif
constexpr int kStoreLag = TEC_DMA_STORELAG;
static_assert(kStoreLag <= 3 * 2 * kCap && kStoreLag < 64, "stores older than 3 steps must have landed");
constexpr uint32_t kDrop = 0x80000000u;    // offset past every resource: the range check drops it
#ifndef TEC_DMA_JX
#define TEC_DMA_JX 0  // 1: measurement only, junction-line pricing (writes wrong bytes)
#endif
#ifndef TEC_DMA_ST_AUX
#define TEC_DMA_ST_AUX 2
#endif
constexpr int kStAux = TEC_DMA_ST_AUX;     // slice stores: nt
// DMA issue shape (measurement variants): 0 = packed (7 own rows in 10 instructions, 9 partner rows
// in 13); 1 = one instruction pair per row, each input row's SECOND touch (own row read after it
// was a partner, or partner after own, or a red row's only touch) non-temporal and its first touch
// default policy, so the rows a later plane re-reads are the ones the caches keep; 2 = per row,
// every row default policy
#ifndef TEC_DMA_ROWPOL
#define TEC_DMA_ROWPOL 1
#endif
#ifndef TEC_DMA_L2NT
#define TEC_DMA_L2NT 1  // level-2 partner rows (parity read back from the slices) non-temporal
#endif
// (r01-r03 timing variants of this kernel -- direct stores, DMA orders, priorities, ablations,
// occupancy probes -- live in the measurement copy scripts/kbench_encode_dma.hip)

// Staging rows (per plane).
constexpr int kRowC0 = 0;   // 0..2: node 7+r at this plane (level 1 parity; level 2 red / pair / park)
constexpr int kRowX = 3;    // 3..4: level 2, C(z0, (7+i, s)) of the pair finished now
constexpr int kRowC1 = 5;   // 5..14: C(10+j, (z0, s)) for j <= s
constexpr int kRowB = 15;   // 15..23: burst C(10+s, (z0, j)) for j < s

// Column-1 pair (p, j), p < j, of a row of planes: U(10+j, (z0, p)) parked at step p and read at
// step j.  Reads precede writes within a step, so a slot read at step j is free again at step j:
// interval colouring needs max_p (p+1)(9-p) = 25 slots.
struct PairSlots {
    uint8_t slot[kQ][kQ];
    int n;
};
constexpr PairSlots make_slots() {
    PairSlots ps{};
    int busy[32];
    for (int i = 0; i < 32; i++) busy[i] = -1;
    for (int p = 0; p < kQ; p++)
        for (int j = p + 1; j < kQ; j++) {
            int sl = 0;
            while (busy[sl] > p) sl++;
            busy[sl] = j;
            ps.slot[p][j] = (uint8_t)sl;
            if (sl + 1 > ps.n) ps.n = sl + 1;
        }
    return ps;
}
constexpr PairSlots kSl = make_slots();
static_assert(kSl.n == 25, "row pairs need 25 slots");
constexpr int kSlots = 25;

// Flush schedule: per step type (0 = level 1, 1 + i0 = level-2 row 7 + i0) and plane digit s,
// the rows the step finishes, split into contiguous per-wave shares.  Item = source (0x80 | x:
// ring own row x; else staging row) | node << 8 | target z0 << 16 (0xff: this step's) |
// target s << 24 (0xff: this step's).
struct FlushTab {
    struct W {
        uint32_t n;
        uint32_t item[kCap];
    } w[4][kQ][G];
    uint32_t extra;  // the one item the last plane (31 rows) leaves for a flush after the loop
};
constexpr uint32_t fitem(int src, int node, int z0, int s) {
    return (uint32_t)src | ((uint32_t)node << 8) | ((uint32_t)(z0 & 0xff) << 16) | ((uint32_t)(s & 0xff) << 24);
}
constexpr FlushTab make_flush_tab() {
    FlushTab t{};
    for (int type = 0; type < 4; type++) {
        const int i0 = type - 1;
        for (int s = 0; s < kQ; s++) {
            uint32_t items[40] = {};
            int n = 0;
            for (int x = 0; x < K; x++) items[n++] = fitem(0x80 | x, x, -1, -1);           // systematic
            for (int r = 0; r < 3; r++) items[n++] = fitem(kRowC0 + r, K + r, -1, -1);     // nodes 7..9
            for (int i = 0; i < i0; i++) items[n++] = fitem(kRowX + i, K + i0, K + i, -1);  // C(z0, (7+i, s))
            for (int j = 0; j <= s; j++) items[n++] = fitem(kRowC1 + j, kQ + j, -1, -1);
            for (int j = 0; j < s; j++) items[n++] = fitem(kRowB + j, kQ + s, -1, j);
            if (n > G * kCap) t.extra = items[--n];  // only plane 99 (type 3, s = 9)
            for (int w = 0; w < G; w++) {
                const int b = w * n / G, e = (w + 1) * n / G;
                t.w[type][s][w].n = (uint32_t)(e - b);
                for (int i = b; i < e; i++) t.w[type][s][w].item[i - b] = items[i];
            }
        }
    }
    return t;
}
constexpr FlushTab kFlushC = make_flush_tab();
constexpr bool flush_ok() {
    for (int t = 0; t < 4; t++)
        for (int s = 0; s < kQ; s++)
            for (int w = 0; w < G; w++)
                if (kFlushC.w[t][s][w].n < 1 || kFlushC.w[t][s][w].n > (uint32_t)kCap) return false;
    return true;
}
static_assert(flush_ok(), "every wave flushes 1..kCap rows per step (>= 2 stores: the vmcnt(2) wait)");
static_assert(kFlushC.extra != 0 && (kFlushC.extra & 0x80u) == 0, "the left-over item is a staging row");
__constant__ FlushTab kFlush = kFlushC;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x4 rsrc(const void *p, uint32_t nrec) {
    const uint64_t a = reinterpret_cast<uint64_t>(p);
    u32x4 r;
    r.x = __builtin_amdgcn_readfirstlane((uint32_t)a);
    r.y = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32) & 0xffffu);
    r.z = __builtin_amdgcn_readfirstlane(nrec);
    r.w = 0x00020000u;
    return r;
}

// One LDS-DMA piece: lane l's 16 bytes at (voff + soff) of the resource land at LDS
// lds + 16 l.  Inline asm on purpose (see the header): the compiler neither counts it nor
// orders LDS reads behind it; the kernel waits with explicit vmcnt + barrier.
// cache policy of a second-touch (or only-touch) DMA row (TEC_DMA_ROWPOL 1) / a level-2 partner
#ifndef TEC_DMA_NT_SEL
#define TEC_DMA_NT_SEL 0
#endif
#if TEC_DMA_NT_SEL == 1
#define TEC_DMA_NT_POL "sc0 nt"
#elif TEC_DMA_NT_SEL == 2
#define TEC_DMA_NT_POL "sc1 nt"
#elif TEC_DMA_NT_SEL == 3
#define TEC_DMA_NT_POL "sc0 sc1 nt"
#else
#define TEC_DMA_NT_POL "nt"
#endif
template <bool NT>
__device__ __forceinline__ void dma16(u32x4 rs, uint32_t voff, uint32_t soff, uint32_t lds) {
    uint32_t keep;
    if constexpr (NT)
        asm volatile(
            "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
            "buffer_load_dwordx4 %1, %2, %4 offen " TEC_DMA_NT_POL " lds\n\ts_mov_b32 m0, %0"
            : "=&s"(keep) : "v"(voff), "s"(rs), "s"(lds), "s"(soff) : "memory");
    else
        asm volatile(
            "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
            "buffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
            : "=&s"(keep) : "v"(voff), "s"(rs), "s"(lds), "s"(soff) : "memory");
}

__device__ __forceinline__ uint32_t lds32(const uint8_t *p) { return *reinterpret_cast<const uint32_t *>(p); }
__device__ __forceinline__ void st32(uint8_t *p, uint32_t v) { *reinterpret_cast<uint32_t *>(p) = v; }

// Column 1 of plane (z0, S): u1[j] = U(10+j, (z0, S)).  j < S: the pair with U(10+S, (z0, j))
// parked at step j finishes (both C's staged); j == S: red, C = U; j > S: park.
template <int S, class Out>
__device__ __forceinline__ void col1(const uint32_t *u1, uint32_t (&sl)[kSlots], Out &&out) {
#pragma unroll
    for (int j = 0; j < S; j++) {
        const uint32_t pu = sl[kSl.slot[j][S]];
        const uint32_t tt = xt(u1[j] ^ pu);
        out(kRowC1 + j, u1[j] ^ tt);  // C(10+j, (z0, S))
        out(kRowB + j, pu ^ tt);      // C(10+S, (z0, j))
    }
    out(kRowC1 + S, u1[S]);
#pragma unroll
    for (int j = S + 1; j < kQ; j++) sl[kSl.slot[S][j]] = u1[j];
}

// MASKED: the stripe's data end is not dword aligned (an object's last stripe only).
template <bool MASKED>
__global__ void __launch_bounds__(kWaves * 64, 4) enc_dma_kernel(EncArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    uint8_t *const lds8 = reinterpret_cast<uint8_t *>(lds);
    const uint32_t lds0 = __builtin_amdgcn_groupstaticsize();  // LDS address of the dynamic array
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;

    const uint32_t tile = xcd_tile(blockIdx.x, gridDim.x);
    const uint32_t split = a.z0_split ? a.z0_split : 1u;
    const uint32_t job = tile / split, part = tile - job * split;
    const uint32_t z0b = a.z0_count ? a.z0_first + part * a.z0_count : 0u;
    const uint32_t z0e = a.z0_count ? min(z0b + a.z0_count, a.z0_limit ? a.z0_limit : (uint32_t)kQ) : (uint32_t)kQ;
    const uint32_t zb = z0b * kQ, ze = z0e * kQ;  // this workgroup's planes [zb, ze)
    const EncJob J = a.jobs[job];
    const uint32_t cs = a.cs, sc = a.sc, slen = a.slice_len;
    // lane word: columns 4w..4w+3 of every row; words past the 1,440-column image alias the
    // last one (same inputs, same values, same staging address)
    const uint32_t w = threadIdx.x < RB * 4u ? threadIdx.x : RB * 4u - 1u;
    const uint32_t colw = w * 4u;

    // Input resource: from J.src rounded down to 4 bytes to the stripe's last data byte, so the
    // range check supplies Slicer::encode's zero padding (slicer.rs:276-283).
    const uint32_t src_len = (uint32_t)J.src_len;
    const uint32_t src_al = (uint32_t)reinterpret_cast<uintptr_t>(J.src) & 3u;
    const uint32_t src_range = MASKED ? (src_len + src_al + 3u) & ~3u : src_len + src_al;
    const u32x4 rs_src = rsrc(J.src - src_al, src_range);
    const __amdgpu_buffer_rsrc_t rb_src =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(J.src - src_al), 0, (int)src_range, 0x00020000);
    const uint32_t dst_range = a.n * slen - J.dst_skew;  // < 2^31, host-checked
    const u32x4 rs_dst = rsrc(J.dst, dst_range);
    const __amdgpu_buffer_rsrc_t rb_dst = __builtin_amdgcn_make_buffer_rsrc(J.dst, 0, (int)dst_range, 0x00020000);
#if TEC_DMA_JX
    // (measurement) the destination base's line offset, and a resource from the line it starts in
    const uint32_t jx_base = (uint32_t)(reinterpret_cast<uintptr_t>(J.dst) & 127u);
    const __amdgpu_buffer_rsrc_t rb_jx =
        __builtin_amdgcn_make_buffer_rsrc(J.dst - jx_base, 0, (int)(dst_range + jx_base), 0x00020000);
#endif
    const uint32_t store_mask = J.store_mask;  // chunks to write (internal nodes)
    uint32_t sl_lane = lane + J.rot;
    sl_lane = (sl_lane >= 20u ? sl_lane - 20u : sl_lane) * slen;
    auto slice_off = [&](uint32_t node) -> uint32_t { return __builtin_amdgcn_readlane(sl_lane, node); };

    // The one word of the stripe that straddles the data end reads short through the range check
    // (it is checked per dword of the load): fetched here with aligned pairs (+ byte mask) and
    // substituted where its row is used.
    const uint32_t last = src_len ? src_len - 1u : 0u;
    const uint32_t ex = src_len ? last / cs : 0xffffu, ez = src_len ? (last - ex * cs) / sc : 0xffffu;
    uint32_t fixw = 0;
    if (src_len) {
        const uint32_t off = ex * cs + ez * sc + colw, o = src_al + off;
        const uint32_t lo = __builtin_amdgcn_raw_buffer_load_b32(rb_src, (int)(o & ~3u), 0, 0);
        const uint32_t hi = __builtin_amdgcn_raw_buffer_load_b32(rb_src, (int)((o & ~3u) + 4u), 0, 0);
        fixw = __builtin_amdgcn_alignbyte(hi, lo, o & 3u);
        if constexpr (MASKED) {
            const int rem = (int)src_len - (int)off;
            fixw &= rem >= 4 ? 0xffffffffu : (rem <= 0 ? 0u : (1u << (8 * rem)) - 1u);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::"v"(fixw) : "memory");

    // DMA pieces of the loader wave: instruction i of the 23 per plane (0..9 own rows, 10..22
    // partner rows).  dvo = per-lane source offset (partner: for x = p; +10 sc when the piece's
    // partner row index p >= z0 skips the red node).
    uint32_t dvo[kDmaInstr];
#pragma unroll
    for (int i = 0; i < kDmaInstr; i++) {
        dvo[i] = kDrop;
        if (i < kOwnInstr) {
            const uint32_t b = 64u * i + lane, x = b / RB, j = b - x * RB;
            if (b < (uint32_t)K * RB) dvo[i] = x * cs + 16u * j;
        } else {
            const uint32_t b = 64u * (i - kOwnInstr) + lane, p = b / RB, j = b - p * RB;
            if (b < 9u * RB) dvo[i] = p * kQ * sc + 16u * j;  // 16 j < 10 sc: p >= z0 <=> dvo >= 10 sc z0
        }
    }
    // DMA of plane tp into ring slot `slot`: own rows from the input; partner rows C(z0, (x, s)),
    // x != z0: the input chunk z0 at level 1, node z0's slice at level 2 (level-1 parity rows
    // and parked U, written >= 8 steps earlier -- complete by the vmcnt waits below; nt loads
    // skip this CU's L1).
    // per-row pieces (TEC_DMA_ROWPOL): lane l's block l of the row (first instruction) and block
    // 64 + l (second, lanes < RB - 64)
    const uint32_t rvo0 = 16u * lane, rvo1 = lane < RB - 64u ? 16u * (64u + lane) : kDrop;
    auto issue_rows = [&](uint32_t tp, uint32_t slot) {
        const uint32_t nz0 = tp / kQ, ns = tp - nz0 * kQ;
        const bool lvl2 = nz0 >= (uint32_t)K;
        const uint32_t so_own = src_al + tp * sc;
        const uint32_t so_pbase = lvl2 ? slice_off(nz0) + ns * sc : src_al + nz0 * cs + ns * sc;
        auto piece = [&](bool from_dst, bool nt, uint32_t so, uint32_t ld) {
            so = __builtin_amdgcn_readfirstlane(so);
            ld = __builtin_amdgcn_readfirstlane(lds0 + ld);
            const u32x4 rs = from_dst ? rs_dst : rs_src;
            if (nt) dma16<true>(rs, rvo0, so, ld);
            else dma16<false>(rs, rvo0, so, ld);
            if (rvo1 != kDrop) {
                if (nt) dma16<true>(rs, rvo1, so, ld + 1024u);
                else dma16<false>(rs, rvo1, so, ld + 1024u);
            }
        };
#pragma unroll
        for (int x = 0; x < K; x++)  // own rows: a second touch unless its partner read is still ahead
            piece(false, TEC_DMA_ROWPOL == 1 && (lvl2 || (uint32_t)x <= nz0), so_own + x * cs, slot + x * RW);
#pragma unroll
        for (int p = 0; p < 9; p++) {
            const uint32_t x = (uint32_t)p + ((uint32_t)p >= nz0 ? 1u : 0u);
            // level 2 reads node z0's rows 7.. only for the pairs z0 finishes (x < z0): rows 8, 9 of
            // row 7 and row 9 of row 8 are never used (30 of the stripe's 270 read-backs)
            if (lvl2 && x >= (uint32_t)K && x > nz0) continue;
            piece(lvl2, TEC_DMA_ROWPOL == 1 && (lvl2 ? TEC_DMA_L2NT != 0 : x < nz0), so_pbase + x * kQ * sc,
                  slot + kPartBase + p * RW);
        }
    };
    auto issue_dma = [&](uint32_t tp, uint32_t slot) {
        if constexpr (TEC_DMA_ROWPOL != 0) {
            issue_rows(tp, slot);
            return;
        }
        const uint32_t nz0 = tp / kQ, ns = tp - nz0 * kQ;
        const uint32_t so_own = __builtin_amdgcn_readfirstlane(src_al + tp * sc);
        const bool lvl2 = nz0 >= (uint32_t)K;
        const uint32_t so_part = __builtin_amdgcn_readfirstlane(lvl2 ? slice_off(nz0) + ns * sc : src_al + nz0 * cs + ns * sc);
        const uint32_t skip = kQ * sc, skip_from = skip * nz0;
#pragma unroll
        for (int i = 0; i < kDmaInstr; i++) {
            // lanes past the region's last block are masked off (an LDS-DMA lane that is merely
            // range-dropped still writes zeros to its LDS destination)
            if (dvo[i] == kDrop) continue;
            if (i < kOwnInstr) {
                dma16<false>(rs_src, dvo[i], so_own, __builtin_amdgcn_readfirstlane(lds0 + slot + 1024u * i));
            } else {
                const uint32_t vo = dvo[i] + (dvo[i] >= skip_from ? skip : 0u);
                const uint32_t ld = __builtin_amdgcn_readfirstlane(lds0 + slot + kPartBase + 1024u * (i - kOwnInstr));
                if (lvl2) dma16<true>(rs_dst, vo, so_part, ld);
                else dma16<false>(rs_src, vo, so_part, ld);
            }
        }
    };

    // flush: lane block offsets of a row (16 B per lane; the row's last partial block is one more
    // lane storing the row's LAST 16 bytes -- overlap rewritten with the same bytes)
    const uint32_t nb = sc >> 4, tail = sc & 15u;
    auto blk_off = [&](uint32_t b) -> uint32_t {
        return b < nb ? b * 16u : ((tail != 0 && b == nb) ? sc - 16u : kDrop);
    };
    const uint32_t vo0 = blk_off(lane), vo1 = blk_off(lane + 64u);
    const uint32_t lo0 = vo0 == kDrop ? 0u : vo0, lo1 = vo1 == kDrop ? 0u : vo1;

    uint32_t sl[kSlots];
#pragma unroll
    for (int i = 0; i < kSlots; i++) sl[i] = 0;

    if (wv == (uint32_t)G) {
        // the loader: every plane's DMA, two planes ahead of the compute; the barriers mirror
        // the compute waves' B2 / B1 (the ring slot of plane z is free after B1 of z)
        issue_dma(zb, 0);  // zb is even: plane z uses ring slot z & 1
        issue_dma(zb + 1u, kSlotBytes);
        if (zb != 0)  // a level-2 start (split launch) issues fewer rows per plane: wait for both
            asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        else if constexpr (TEC_DMA_ROWPOL != 0)
            asm volatile("s_waitcnt vmcnt(32)\n\ts_barrier" ::: "memory");  // plane 0 landed (16 rows x 2)
        else
            asm volatile("s_waitcnt vmcnt(23)\n\ts_barrier" ::: "memory");  // plane 0 landed
        // the same number of iterations as the compute waves' plane loop: two barriers each
        for (uint32_t z = zb; z < ze; z++) {
            lds_barrier();                                  // B2
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // plane z + 1 landed
            lds_barrier();                                  // B1
            if (z + 2u < ze) issue_dma(z + 2u, (z & 1u) * kSlotBytes);
        }
        return;
    }
    asm volatile("s_barrier" ::: "memory");

    uint8_t *const stg = lds8 + kStageBase + colw;
    for (uint32_t z0 = z0b; z0 < z0e; z0++) {
        const bool lvl2 = z0 >= (uint32_t)K;
        const uint32_t type = lvl2 ? z0 - (K - 1) : 0u;
        for (uint32_t s = 0; s < (uint32_t)kQ; s++) {
            const uint32_t z = z0 * kQ + s;
            const uint32_t slot = (z & 1u) * kSlotBytes;
            const uint8_t *img = lds8 + slot + colw;
            // an output row of this step: staging row `r` (the flush table's numbering)
            auto out = [&](int r, uint32_t v) { st32(stg + r * RW, v); };
            // ---- compute ----
            uint32_t own[K], part[kQ];
#pragma unroll
            for (int x = 0; x < K; x++) own[x] = lds32(img + x * RW);
            if (z == ez) {  // end-row substitution, also patched into the image the flush copies
                own[ex] = fixw;
                st32(lds8 + slot + ex * RW + colw, fixw);
            }
            uint32_t acc[20 - K];
            if (!lvl2) {
#pragma unroll
                for (int x = 0; x < kQ; x++)
                    part[x] = lds32(img + kPartBase + x * RW - ((uint32_t)x > z0 ? RW : 0u));
                if (z0 == ex && s == ez % kQ) part[ez / kQ] = fixw;
                uint32_t u[K];
#pragma unroll
                for (int x = 0; x < K; x++) u[x] = (uint32_t)x == z0 ? own[x] : pft3(own[x], part[x]);
                enc::mds7_slp<true>(u, acc);
#pragma unroll
                for (int r = 0; r < 3; r++)
                    out(kRowC0 + r, acc[r] ^ mulc(kPft.t_p[1], part[K + r]));
            } else {
#pragma unroll
                for (int x = 0; x < 9; x++) part[x] = lds32(img + kPartBase + x * RW);
                uint32_t u[K];
#pragma unroll
                for (int x = 0; x < K; x++) u[x] = pft3(own[x], part[x]);
                enc::mds7_slp<false>(u, acc);
                const uint32_t i0 = z0 - K;
#pragma unroll
                for (int r = 0; r < 3; r++) {
                    // r < i0: pair with U(z0, (7+r, s)) parked in the slice; r == i0: red;
                    // r > i0: park U(7+r, (z0, s)) (staged like an output row)
                    if (r < 2) {
                        const uint32_t us = part[K + r], up = acc[r];
                        const uint32_t tt = xt(us ^ up);
                        // C(z0, (7+r, s)): a row only for r < i0 (staged unconditionally, flushed
                        // only then)
                        out(kRowX + r, us ^ tt);
                        out(kRowC0 + r, (uint32_t)r < i0 ? up ^ tt : up);  // C / U(7+r, (z0, s))
                    } else {
                        out(kRowC0 + r, acc[r]);
                    }
                }
            }
            switch (s) {
                case 0: col1<0>(acc + 3, sl, out); break;
                case 1: col1<1>(acc + 3, sl, out); break;
                case 2: col1<2>(acc + 3, sl, out); break;
                case 3: col1<3>(acc + 3, sl, out); break;
                case 4: col1<4>(acc + 3, sl, out); break;
                case 5: col1<5>(acc + 3, sl, out); break;
                case 6: col1<6>(acc + 3, sl, out); break;
                case 7: col1<7>(acc + 3, sl, out); break;
                case 8: col1<8>(acc + 3, sl, out); break;
                default: col1<9>(acc + 3, sl, out); break;
            }
            lds_barrier();  // B2: the plane's rows are staged
            // ---- flush: this wave's share, read now, stored after B1 ----
            const FlushTab::W &F = kFlush.w[type][s][wv];
            const uint32_t n = F.n;
            u32x4 d0[kCap], d1[kCap];
            uint32_t dst[kCap];
#pragma unroll
            for (int q = 0; q < kCap; q++) {
                if ((uint32_t)q < n) {
                    const uint32_t it = F.item[q];
                    const uint32_t src = it & 0xffu;
                    const uint8_t *row = (src & 0x80u) ? lds8 + slot + (src & 0x7fu) * RW : lds8 + kStageBase + src * RW;
                    d0[q] = *reinterpret_cast<const u32x4 *>(row + lo0);
                    d1[q] = *reinterpret_cast<const u32x4 *>(row + lo1);
                    const uint32_t node = (it >> 8) & 0xffu, tz0 = (it >> 16) & 0xffu, ts = it >> 24;
                    dst[q] = slice_off(node) + ((tz0 == 0xffu ? z0 : tz0) * kQ + (ts == 0xffu ? s : ts)) * sc;
                    if (!((store_mask >> node) & 1u)) dst[q] = kDrop;  // a chunk the caller does not keep
                }
            }
            // B1: the next plane's DMA has landed and every wave is done reading this slot and the
            // staging rows; the compute waves issue no loads, so they only bound their stores in
            // flight (see kStoreLag)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kStoreLag) : "memory");
            lds_barrier();
#pragma unroll
            for (int q = 0; q < kCap; q++) {
                if ((uint32_t)q < n) {
#if TEC_DMA_JX
                    // measurement only (wrong bytes): the row's stores as whole 128-B lines, every
                    // junction line once -- the write pattern of line-exact stores, to price them
                    const uint32_t ab = jx_base + dst[q], first = (ab + 127u) & ~127u;
                    const uint32_t o0 = first + 16u * lane - jx_base, o1 = first + 16u * (64u + lane) - jx_base;
                    const uint32_t lim = ((ab + (uint32_t)sc + 127u) & ~127u) - jx_base;
                    __builtin_amdgcn_raw_buffer_store_b128(d0[q], rb_jx, (int)(dst[q] == kDrop ? kDrop : o0), 0, kStAux);
                    __builtin_amdgcn_raw_buffer_store_b128(d1[q], rb_jx, (int)(dst[q] == kDrop || o1 >= lim ? kDrop : o1), 0, kStAux);
#else
                    __builtin_amdgcn_raw_buffer_store_b128(d0[q], rb_dst, (int)vo0, (int)dst[q], kStAux);
                    __builtin_amdgcn_raw_buffer_store_b128(d1[q], rb_dst, (int)vo1, (int)dst[q], kStAux);
#endif
                }
            }
        }
    }
    // the last plane's left-over row (its staging row is untouched since the last compute)
    if (wv == 0 && z0e == (uint32_t)kQ) {
        const uint32_t it = kFlush.extra, src = it & 0xffu;
        const uint8_t *row = lds8 + kStageBase + src * RW;
        const u32x4 e0 = *reinterpret_cast<const u32x4 *>(row + lo0);
        const u32x4 e1 = *reinterpret_cast<const u32x4 *>(row + lo1);
        const uint32_t node = (it >> 8) & 0xffu, tz0 = (it >> 16) & 0xffu, ts = it >> 24;
        const uint32_t d = ((store_mask >> node) & 1u)
                               ? slice_off(node) + ((tz0 == 0xffu ? kQ - 1u : tz0) * kQ + (ts == 0xffu ? kQ - 1u : ts)) * sc
                               : kDrop;
        __builtin_amdgcn_raw_buffer_store_b128(e0, rb_dst, (int)vo0, (int)d, kStAux);
        __builtin_amdgcn_raw_buffer_store_b128(e1, rb_dst, (int)vo1, (int)d, kStAux);
    }
}

}  // namespace dma

bool encode_dma_supported(int n, int k, uint32_t sc) { return n == 20 && k == 7 && sc > 1280u && sc <= 1440u && sc % 2 == 0; }

hipError_t launch_encode_dma(bool masked, const EncArgs &a, hipStream_t s) {
    if (a.njobs == 0) return hipSuccess;
    if (!encode_dma_supported((int)a.n, 7, a.sc) || a.njobs > 0x7fffffffu) return hipErrorInvalidValue;
    const void *fn = masked ? reinterpret_cast<const void *>(dma::enc_dma_kernel<true>)
                            : reinterpret_cast<const void *>(dma::enc_dma_kernel<false>);
#ifndef TEC_DMA_LDS_PAD
#define TEC_DMA_LDS_PAD 0  // measurement: extra dynamic LDS (e.g. 40960 -> one workgroup per CU)
#endif
    const size_t lds = dma::kLdsBytes + TEC_DMA_LDS_PAD;
    hipError_t e = ensure_dyn_lds(fn, lds);
    if (e != hipSuccess) return e;
    // a plane range must start on an even plane (ring slot parity) and stay within the 100 planes
    // every part non-empty and within the 10 rows (a shorter last part when z0_limit cuts it)
    if (a.z0_count) {
        const uint32_t lim = a.z0_limit ? a.z0_limit : 10u;
        if (a.z0_split == 0 || lim > 10u || a.z0_first + (a.z0_split - 1u) * a.z0_count >= lim) return hipErrorInvalidValue;
    }
    const uint64_t grid = (uint64_t)a.njobs * (a.z0_count ? a.z0_split : 1u);
    if (grid > 0x7fffffffu) return hipErrorInvalidValue;
    if (masked)
        hipLaunchKernelGGL(dma::enc_dma_kernel<true>, dim3((uint32_t)grid), dim3(dma::kWaves * 64), lds, s, a);
    else
        hipLaunchKernelGGL(dma::enc_dma_kernel<false>, dim3((uint32_t)grid), dim3(dma::kWaves * 64), lds, s, a);
    return hipGetLastError();
}

}  // namespace tec
