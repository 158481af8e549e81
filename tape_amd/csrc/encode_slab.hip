// encode_slab.hip -- Clay layered encode for the q = 10, t = 2 profiles (n = 20, d = k + 9),
// i.e. the production profile (20,7,16) (lib/core/src/encoding.rs:236-239) and the reference
// test profile (20,10,19).  Replaces ClayCoder::encode -> clay_codes::ClayCode::encode
// (lib/slicer/src/clay.rs:99-104) inside Slicer::encode's per-stripe loop (slicer.rs:268-286),
// fused with the rotation scatter `distribute_chunks` (slicer.rs:60-71).
//
// Algebra (encode = decode_layered with the parity nodes erased):
//   plane z = 10*z0 + z1; nodes (x, y), y = 0 for nodes 0..9, y = 1 for nodes 10..19; data
//   nodes are x < K in column 0.  Column-0 couplings join planes of equal z1 (a "slab"),
//   column-1 couplings join planes of equal z0 (a "row").  Planes with z0 < K are decode
//   level 1, z0 >= K level 2 (their column-0 partners are level-1 parity of the same slab).
//
// Work decomposition (MI355X): a wave owns 64 consecutive 4-column words (one per lane) of one
// stripe and walks ALL 100 planes of them in decode order (z0 = 0..9, z1 = 0..9), so no value
// ever crosses waves: column-0 partners are inputs or the wave's own earlier level-1 outputs
// (re-read: same thread, same address), column-1 pairs and level-2 column-0 pairs wait in a
// thread-private LDS slot table until their second half is computed.  A workgroup is the
// G = ceil(sc / 256) waves covering a stripe's columns (6 for 1 MB stripes), walking the planes
// in lockstep, so every plane step writes complete 1,430-byte sub-chunk rows of all 20 slices
// at once -- HBM takes row-complete bursts at ~2x the rate of the 256-byte pieces a
// column-split-in-time order produces (scripts/vmem_bench2.hip).
// Coefficients (generator, PFT) are constexpr: each GF product is a fixed XOR selection of
// xtime multiples, or a 2-bit v_perm lookup with SGPR tables for one-off heavy constants.
#include "kernels.hpp"
#include "gf_dev.hpp"
#include "dev_io.hpp"

namespace tec {

constexpr int kQ = 10;

template <int K>
struct SlabConst {
    uint8_t G[20][K];   // systematic generator (rows >= K used)
    uint8_t Gt[kQ][K];  // column-0 parity rows pre-scaled for level-1 type-1 recovery: t_u * G
};

template <int K>
constexpr SlabConst<K> make_slab_const() {
    SlabConst<K> rc{};
    const Mat g = rs_generator(K, 20);
    for (int r = 0; r < 20; r++)
        for (int x = 0; x < K; x++) rc.G[r][x] = g.v[r][x];
    for (int r = K; r < kQ; r++)
        for (int x = 0; x < K; x++) rc.Gt[r][x] = gf_mul(kPft.t_u[1], g.v[r][x]);
    return rc;
}

// The pairwise transform of this field (A3: RS(2,2) parity [[3,2],[2,3]]) is orientation-free:
// uncoupling (U = 3C + 2C') and re-coupling (C = 3U + 2U') are both  a -> a ^ 2(a ^ b), so a
// pair costs ONE doubling: a' = a ^ t, b' = b ^ t with t = xt(a ^ b).
static_assert(kPft.u_c[0] == 3 && kPft.u_c[1] == 3 && kPft.u_p[0] == 2 && kPft.u_p[1] == 2, "PFT uncouple");
static_assert(kPft.c_u[0] == 3 && kPft.c_u[1] == 3 && kPft.c_p[0] == 2 && kPft.c_p[1] == 2, "PFT couple");
__device__ __forceinline__ uint32_t pft3(uint32_t a, uint32_t b) { return a ^ xt(a ^ b); }

// Column-1 pairs within a row: U(10+j, (z0, i)) is computed at plane (z0, i) and consumed at
// plane (z0, j), i < j.  Slots are assigned by greedy interval colouring in plane order
// (consume before allocate): 25 slots, the maximum number simultaneously pending.
struct PairSlots {
    uint8_t slot[kQ][kQ];
    int nslots;
};
constexpr PairSlots make_pair_slots() {
    PairSlots ps{};
    bool used[kQ * kQ] = {};
    for (int p = 0; p < kQ; p++) {
        for (int i = 0; i < p; i++) used[ps.slot[i][p]] = false;
        for (int j = p + 1; j < kQ; j++) {
            int sl = 0;
            while (used[sl]) sl++;
            used[sl] = true;
            ps.slot[p][j] = (uint8_t)sl;
            if (sl + 1 > ps.nslots) ps.nslots = sl + 1;
        }
    }
    return ps;
}
constexpr PairSlots kPairSlots = make_pair_slots();
static_assert(kPairSlots.nslots == 25, "row pairs need 25 slots");
constexpr int kEncSlots = 25;

#ifndef TEC_ENC_WAVES_PER_EU
#define TEC_ENC_WAVES_PER_EU 5
#endif
#ifndef TEC_ENC_PREFETCH
#define TEC_ENC_PREFETCH 1  // next plane's loads issued before this plane's compute: 1 own, 2 all
#endif
#ifndef TEC_ENC_LOCKSTEP
#define TEC_ENC_LOCKSTEP 0  // s_barrier every N planes (0: none): the workgroup's waves write rows together
#endif
constexpr uint32_t kEncMaxGroupsPerWg = 8;  // column groups per workgroup (10 MB stripes: 56 groups)
#ifndef TEC_ENC_STRIPES_PER_WG
#define TEC_ENC_STRIPES_PER_WG 2  // 2 x 6 waves for 1 MB stripes: 3 waves on each SIMD
#endif
constexpr uint32_t kEncMaxWavesPerWg = 16;

#ifndef TEC_ENC_DRIFT
#define TEC_ENC_DRIFT 0  // >0: a wave starts plane t only when every wave of its workgroup has
                         // finished plane t - DRIFT (LDS progress words, no s_barrier)
#endif
inline size_t enc_lds_bytes(uint32_t waves) { return (size_t)waves * kEncSlots * 64 * 4 + kEncMaxWavesPerWg * 4; }

// MODE (ablation builds only, scripts/kbench.hip): bit0 = drop global stores, bit1 = replace
// GF arithmetic by plain XOR, bit2 = skip the LDS slot table.  Production uses MODE 0.
// MASKED: the stripe's data end is not dword aligned (only an object's last stripe, when its
// length is not a multiple of 4): words are masked per lane instead of relying on the range check.
template <int K, int MODE = 0, bool MASKED = false>
__global__ void __launch_bounds__(kEncMaxWavesPerWg * 64, TEC_ENC_WAVES_PER_EU) enc_slab_kernel(EncArgs a) {
    constexpr SlabConst<K> RC = make_slab_const<K>();
    constexpr int NP0 = kQ - K;  // column-0 parity nodes
    static_assert(NP0 == 0 || NP0 == 3, "fast encode covers k = 7 and k = 10");
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];

    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform
    const int lane = threadIdx.x & 63;
    uint32_t *const slots = lds + wv * (kEncSlots * 64) + lane;      // thread-private, stride 64
    volatile uint32_t *const progress = lds + (blockDim.x >> 6) * (kEncSlots * 64);  // [wave]
    if constexpr (TEC_ENC_DRIFT > 0) {
        if (lane == 0) progress[wv] = 0;
        __syncthreads();
    }
    // workgroup = groups [gb, gb + blockDim/64) of one stripe; every base address is uniform
    const uint32_t tile = xcd_tile(blockIdx.x, gridDim.x);
    const uint32_t sub = (uint32_t)wv / a.groups_per_wg, gl = (uint32_t)wv - sub * a.groups_per_wg;
    uint32_t job, g;
    if (a.stripes_per_wg > 1) {  // several whole stripes per workgroup (balanced over the SIMDs)
        job = tile * a.stripes_per_wg + sub;
        g = gl;
    } else {
        job = tile / a.wgs_per_stripe;
        g = (tile - job * a.wgs_per_stripe) * a.groups_per_wg + gl;
    }
    // Surplus waves (a short last workgroup, or groups past the stripe's last word) leave: a
    // second wave on the same words would race with the values parked in the output (level 2).
    // Lanes past the last word inside a live wave duplicate it in lockstep, which is benign.
    if (job >= a.njobs || g * 64u >= a.words_per_stripe) {
        if constexpr (TEC_ENC_DRIFT > 0) {
            if (lane == 0) progress[wv] = 0xffffu;
        }
        return;
    }
    const EncJob J = a.jobs[job];
    const uint32_t cs = a.cs, sc = a.sc, slen = a.slice_len, wps = a.words_per_stripe;
    // Word of this lane (a wave past the last group redoes the stripe's last word).  When
    // sc = 2 mod 4 the last word has 2 columns: its lane stores the high half at an
    // out-of-range offset, which the range check drops.
    uint32_t w = g * 64u + (uint32_t)lane;
    if (w >= wps) w = wps - 1;
    const uint32_t col = w * 4u;
    const uint32_t hi_skip = col + 4u > sc ? 0x80000000u : 0u;
    const bool tail_wave = (sc & 3u) != 0 && g + 1 >= a.groups_per_stripe;  // uniform
    // Buffer resources (32-bit offsets).  The input resource starts at J.src rounded down to 4
    // bytes and ends exactly at the stripe's last data byte, so the range check returns the zero
    // padding of Slicer::encode (slicer.rs:276-283) for every dword past the data.  A word is two
    // aligned dwords + one v_alignbyte (uniform shift): no branch on the load path.
    const uint32_t src_len = (uint32_t)J.src_len;
    const uint32_t src_al = (uint32_t)reinterpret_cast<uintptr_t>(J.src) & 3u;
    // (gfx950 zeroes a dword that straddles num_records entirely, so the MASKED variant rounds
    // the range up to the dword holding the last data byte -- same page, always readable --
    // and clears the bytes past the data per lane.)
    const __amdgpu_buffer_rsrc_t rs_src = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t *>(J.src - src_al), 0, (int)(MASKED ? (src_len + src_al + 3u) & ~3u : src_len + src_al),
        0x00020000);
    // output range = the object's n slices as seen from this stripe's base (< 2^31, host-checked),
    // so an offset with bit 31 set is out of range and its store is dropped
    const uint32_t dst_al = (uint32_t)reinterpret_cast<uintptr_t>(J.dst) & 3u;
    const uint32_t dst_range = a.n * slen - J.dst_skew;
    const __amdgpu_buffer_rsrc_t rs_dst = __builtin_amdgcn_make_buffer_rsrc(J.dst, 0, (int)dst_range, 0x00020000);
    auto slice_of = [&](int r) -> uint32_t {
        uint32_t sl = (uint32_t)r + J.rot;
        return sl >= 20u ? sl - 20u : sl;
    };
    auto out_st = [&](int r, uint32_t z, uint32_t v) {
        if constexpr (MODE & 1) {
            if (v == 0x12345678u) __builtin_amdgcn_raw_buffer_store_b32(v, rs_dst, (int)col, 0, 0);  // keep v live
            return;
        }
        // uniform part of the address in soffset (the range check covers voffset + soffset).
        // Planes at 2 mod 4 store two aligned halves: a single unaligned dword store is legal
        // but measured slower (it splits into partial-dword writes).
        const uint32_t off = slice_of(r) * slen + z * sc;  // uniform
        const uint32_t al = (dst_al + off) & 3u;           // uniform
        if (al == 0 && !tail_wave) {
            __builtin_amdgcn_raw_buffer_store_b32(v, rs_dst, (int)col, (int)off, 0);
        } else if (!(al & 1u)) {
            __builtin_amdgcn_raw_buffer_store_b16((uint16_t)v, rs_dst, (int)col, (int)off, 0);
            __builtin_amdgcn_raw_buffer_store_b16((uint16_t)(v >> 16), rs_dst, (int)((col + 2u) | hi_skip), (int)off, 0);
        } else {
            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)v, rs_dst, (int)col, (int)off, 0);
            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(v >> 8), rs_dst, (int)(col + 1u), (int)off, 0);
            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(v >> 16), rs_dst, (int)((col + 2u) | hi_skip), (int)off, 0);
            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(v >> 24), rs_dst, (int)((col + 3u) | hi_skip), (int)off, 0);
        }
    };
    // aligned-pair word load at byte offset o of resource rs (o counted from its aligned base)
    auto ld_pair = [&](__amdgpu_buffer_rsrc_t rs, uint32_t o) -> uint32_t {
        const uint32_t lo = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(o & ~3u), 0, 0);
        const uint32_t hi = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)((o & ~3u) + 4u), 0, 0);
        return __builtin_amdgcn_alignbyte(hi, lo, o & 3u);
    };
    auto keep_mask = [&](uint32_t off) -> uint32_t {  // MASKED: bytes of the word below src_len
        const int rem = (int)src_len - (int)off;
        return rem >= 4 ? 0xffffffffu : (rem <= 0 ? 0u : (1u << (8 * rem)) - 1u);
    };
    auto slot = [&](int i) -> uint32_t & { return slots[i * 64]; };
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

    // Loads of plane (z0, s).  own[x] = C(x, (z0, s)) for the data nodes; part[x] = the
    // column-0 partner C(z0, (x, s)): an input chunk at level 1 (z0 < K), at level 2 the
    // level-1 parity this lane stored a row earlier or more (same thread, same address).
    uint32_t own[K], part[kQ];
    auto load_own = [&](uint32_t z0, uint32_t s) {
        const uint32_t z = z0 * kQ + s;
#pragma unroll
        for (int x = 0; x < K; x++)
            own[x] = __builtin_amdgcn_raw_buffer_load_b32(rs_src, (int)col, (int)(src_al + (uint32_t)x * cs + z * sc), 0);
    };
    auto load_part = [&](uint32_t z0, uint32_t s) {
        const bool lvl1 = z0 < (uint32_t)K;  // uniform
        const __amdgpu_buffer_rsrc_t rs_p = __builtin_amdgcn_make_buffer_rsrc(
            lvl1 ? const_cast<uint8_t *>(J.src - src_al) : J.dst, 0,
            (int)(lvl1 ? (MASKED ? (src_len + src_al + 3u) & ~3u : src_len + src_al) : dst_range), 0x00020000);
        const uint32_t pbase = lvl1 ? src_al + z0 * cs : slice_of((int)z0) * slen;
#pragma unroll
        for (int x = 0; x < kQ; x++) {
            // x >= K: level 1 needs C(z0, (x, s)) (type-1 recovery of column-0 parity); level 2
            // re-reads the U(z0, (K+i, s)) parked at i = x - K < z0 - K (see level 2 below)
            uint32_t so = pbase + ((uint32_t)x * kQ + s) * sc;
            if (x >= K && !lvl1 && (uint32_t)x >= z0) so = 0x80000000u;
            part[x] = __builtin_amdgcn_raw_buffer_load_b32(rs_p, (int)col, (int)so, 0);
        }
    };
    auto mds = [&](const uint32_t *u, uint32_t *acc, bool scaled) {
#pragma unroll
        for (int r = 0; r < 20 - K; r++) acc[r] = 0;
#pragma unroll
        for (int x = 0; x < K; x++) {
            if constexpr (MODE & 2) {
#pragma unroll
                for (int r = K; r < 20; r++) acc[r - K] ^= u[x] + r;
            } else {
                const Mult<7> mu(u[x]);
#pragma unroll
                for (int r = K; r < 20; r++) acc[r - K] ^= mu.mul(r < kQ && scaled ? RC.Gt[r][x] : RC.G[r][x]);
            }
        }
    };
    // Column 1 of plane (z0, s): u1[j] = U(10+j, (z0, s)).  Red node (j == s): C = U.  Pair
    // (10+j at (z0, s)) <-> (10+s at (z0, j)): for j < s the partner U was parked at plane
    // (z0, j) and both C's are written now; for j > s this plane's half is parked.
    auto col1 = [&](const uint32_t *u1, uint32_t z0, uint32_t s) {
        const uint32_t z = z0 * kQ + s;
#pragma unroll
        for (int j = 0; j < kQ; j++) {
            if ((uint32_t)j == s) {
                out_st(kQ + j, z, u1[j]);
            } else if ((uint32_t)j < s) {
                // slot index: compile-time j, run-time s -> small uniform table walk
                uint32_t si = 0;
#pragma unroll
                for (int q = 0; q < kQ; q++)
                    if ((uint32_t)q == s) si = kPairSlots.slot[j][q];
                const uint32_t pu = (MODE & 4) ? u1[(j + 1) % kQ] : slot((int)si);  // U(10+s, (z0, j))
                const uint32_t tt = xt(u1[j] ^ pu);
                out_st(kQ + j, z, u1[j] ^ tt);
                out_st(kQ + (int)s, z0 * kQ + (uint32_t)j, pu ^ tt);
            } else {
                uint32_t si = 0;
#pragma unroll
                for (int q = 0; q < kQ; q++)
                    if ((uint32_t)q == s) si = kPairSlots.slot[q][j];
                if constexpr (!(MODE & 4)) slot((int)si) = u1[j];
            }
        }
    };

    // Planes in decode order; loads of the next plane are issued before this one is computed.
    load_own(0, 0);
    if constexpr (TEC_ENC_PREFETCH == 2) load_part(0, 0);
    for (uint32_t z0 = 0; z0 < (uint32_t)kQ; z0++) {
        for (uint32_t s = 0; s < (uint32_t)kQ; s++) {
            const uint32_t z = z0 * kQ + s;
            uint32_t cown[K], cpart[kQ];
            if constexpr (TEC_ENC_PREFETCH != 2) load_part(z0, s);
            // end-row substitution (uniform conditions; see fixw)
            const bool own_end = z == ez, part_end = z0 == ex && z0 < (uint32_t)K && s == ez % kQ;
#pragma unroll
            for (int x = 0; x < K; x++) cown[x] = (own_end && (uint32_t)x == ex) ? fixw : own[x];
#pragma unroll
            for (int x = 0; x < kQ; x++) cpart[x] = (part_end && (uint32_t)x == ez / kQ) ? fixw : part[x];
            if (z + 1 < (uint32_t)(kQ * kQ)) {
                const uint32_t nz0 = s + 1 < (uint32_t)kQ ? z0 : z0 + 1, ns = s + 1 < (uint32_t)kQ ? s + 1 : 0;
                load_own(nz0, ns);
                if constexpr (TEC_ENC_PREFETCH == 2) load_part(nz0, ns);
            }
            if (z0 < (uint32_t)K) {
                // ---- level 1: data partners are inputs; column-0 parity by type-1 recovery ----
                uint32_t u[K];
#pragma unroll
                for (int x = 0; x < K; x++) {
                    out_st(x, z, cown[x]);  // systematic chunk -> its rotated slice
                    u[x] = (uint32_t)x == z0 ? cown[x] : pft3(cown[x], cpart[x]);
                }
                uint32_t acc[20 - K];
                mds(u, acc, true);
                // column-0 parity (x = r >= K, not red at level 1): type-1 with partner C(z0, (r, s))
#pragma unroll
                for (int r = K; r < kQ; r++) out_st(r, z, acc[r - K] ^ mulc(kPft.t_p[1], cpart[r]));
                col1(acc + NP0, z0, s);
            } else if constexpr (NP0 > 0) {
                // ---- level 2: data partners are the level-1 column-0 parity C(z0, (x, s)) ----
                uint32_t u[K];
#pragma unroll
                for (int x = 0; x < K; x++) {
                    out_st(x, z, cown[x]);
                    u[x] = pft3(cown[x], cpart[x]);  // x < K <= z0
                }
                uint32_t acc[20 - K];
                mds(u, acc, false);
                // column-0 parity K+r at plane (z0, s): red when K+r == z0 (C = U); otherwise
                // paired with (z0, (K+r, s)) -- both erased -- and finished at the later of the
                // two planes.  The earlier plane parks its U in the output slot of that C (it
                // is overwritten when finished); the later plane's loads fetched it as
                // cpart[K + i] (same thread, same address: program order).
                const int i0 = (int)z0 - K;
#pragma unroll
                for (int i = 0; i < NP0; i++) {
                    if (i >= i0) break;
                    const uint32_t us = cpart[K + i];             // U(K+i0, (K+i, s)), parked
                    const uint32_t up = acc[i];                   // U(K+i, (K+i0, s))
                    const uint32_t tt = xt(us ^ up);
                    out_st(K + i0, (uint32_t)(K + i) * kQ + s, us ^ tt);
                    out_st(K + i, z, up ^ tt);
                }
#pragma unroll
                for (int r = 0; r < NP0; r++) {
                    if (r == i0) out_st(K + r, z, acc[r]);  // red: C = U
                    if (r > i0) out_st(K + r, z, acc[r]);   // park U(K+r, (z0, s))
                }
                col1(acc + NP0, z0, s);
            }
            if constexpr (TEC_ENC_LOCKSTEP > 0)
                if ((z + 1) % TEC_ENC_LOCKSTEP == 0) __builtin_amdgcn_s_barrier();
            if constexpr (TEC_ENC_DRIFT > 0) {
                // publish "plane z done", then hold while any wave is DRIFT or more planes behind
                if (lane == 0) progress[wv] = z + 1;
                const uint32_t nw = blockDim.x >> 6;
                if (z + 1 >= (uint32_t)TEC_ENC_DRIFT) {
                    for (;;) {
                        uint32_t mn = 0xffffffffu;
                        for (uint32_t q = 0; q < nw; q++) mn = min(mn, progress[q]);
                        mn = __builtin_amdgcn_readfirstlane(mn);
                        if (mn + TEC_ENC_DRIFT >= z + 1) break;
                        __builtin_amdgcn_s_sleep(1);
                    }
                }
            }
        }
    }
}

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

bool encode_rows_supported(int n, int k, int d) { return n == 20 && d == k + 9 && (k == 7 || k == 10); }

template <int K, int MODE, bool MASKED>
hipError_t launch_enc_mode(EncArgs a, hipStream_t s) {
    if (a.njobs == 0) return hipSuccess;
    a.groups_per_wg = a.groups_per_stripe < kEncMaxGroupsPerWg ? a.groups_per_stripe : kEncMaxGroupsPerWg;
    a.wgs_per_stripe = (a.groups_per_stripe + a.groups_per_wg - 1) / a.groups_per_wg;
    a.stripes_per_wg = 1;
    if (a.wgs_per_stripe == 1)
        while (a.stripes_per_wg < TEC_ENC_STRIPES_PER_WG && (a.stripes_per_wg + 1) * a.groups_per_wg <= kEncMaxWavesPerWg)
            a.stripes_per_wg++;
    const uint64_t blocks = a.stripes_per_wg > 1 ? (a.njobs + a.stripes_per_wg - 1) / a.stripes_per_wg
                                                 : (uint64_t)a.njobs * a.wgs_per_stripe;
    const uint32_t waves = a.groups_per_wg * a.stripes_per_wg;
    if (blocks > 0x7fffffffull) return hipErrorInvalidValue;
    const size_t lds = enc_lds_bytes(waves);
    static size_t lds_set = 0;  // per instantiation: raise the dynamic-LDS cap once
    if (lds > lds_set) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(enc_slab_kernel<K, MODE, MASKED>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        lds_set = lds;
    }
    hipLaunchKernelGGL((enc_slab_kernel<K, MODE, MASKED>), dim3((uint32_t)blocks), dim3(waves * 64), lds,
                       s, a);
    return hipGetLastError();
}

hipError_t launch_encode_rows(int k, bool masked, const EncArgs &a, hipStream_t s) {
    switch (k * 2 + (masked ? 1 : 0)) {
        case 14: return launch_enc_mode<7, 0, false>(a, s);
        case 15: return launch_enc_mode<7, 0, true>(a, s);
        case 20: return launch_enc_mode<10, 0, false>(a, s);
        case 21: return launch_enc_mode<10, 0, true>(a, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_meta(const MetaJob *jobs, uint32_t njobs, uint32_t n, hipStream_t s) {
    if (!njobs) return hipSuccess;
    const uint32_t total = njobs * n * 6u;
    hipLaunchKernelGGL(meta_kernel, dim3((total + 255) / 256), dim3(256), 0, s, jobs, njobs, n);
    return hipGetLastError();
}

}  // namespace tec
