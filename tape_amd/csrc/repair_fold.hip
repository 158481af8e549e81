// repair_fold.hip -- single-chunk Clay repair with the decoding matrix folded at compile time,
// for the helper sets ClayCoder::minimum_to_repair (repair.rs:53-70 -> clay_codes) picks in
// Clay(20,7,16): the lost node's 9 column-mates plus the first 7 available nodes of the other
// column.  With all 19 others available (a healthy cluster) those are the other column's nodes
// 0..6; with one of them down (a peer outage, the node's fallback across peer maps,
// network/node/src/features/spool/repair.rs:228-267) they are 0..7 without it.  The erasure
// pattern is then fixed by the lost column y_l and the other column's known set K (7 of 10
// positions, the other 3 aloof); the kernel is instantiated per (y_l, K) for those 2 x 8 sets
// with the MDS decoding matrix D = G_E inv(G_K) as constants.  Other helper sets run the
// table-driven kernel (repair_stage.hip); results are identical.
//
// Algebra (Ceph repair_one_lost_chunk): the beta = 10 repair planes are the
// planes whose y_l digit is x_l; index them by their other digit w (= the row of each helper's
// repair data).  For known node j of the other column at plane w:
//   w == j             red, U = C
//   w in K, w != j     partner = known node w at plane j: the pair is uncoupled from both C's
//   w aloof            partner = aloof node w at plane j: U = a_c C + a_p U_aloof(w, j)
// so the planes w in K go first (they also yield the aloof U's the aloof planes consume).  Per
// plane the MDS solve gives the 10 column nodes' U: the lost node is red (its C at the plane = U)
// and each column-mate m's helper C and solved U give the lost chunk at the plane whose y_l digit
// is x_m.  Every plane thus finishes 10 lost-chunk planes (y_l digit 0..9, other digit w).
//
// Work decomposition (MI355X): a workgroup owns one stripe's row segment (G <= 6 waves x 64 lanes
// x 4 columns), a lane one 4-column word.  The lane loads each helper row it needs exactly once
// (the 7 x 7 known block up front, the column-mates one plane ahead): 160 dword loads per word,
// the algorithmic read volume.  The MDS is xtime multiples + v_bitop3 XOR selections (no tables,
// no scalar loads); the 10 rows a plane finishes are staged in LDS (double-buffered, one barrier
// per plane) and stored whole by one wave each.
#include "kernels.hpp"
#include "enc_common.hpp"
#include "dev_io.hpp"

#ifndef TEC_RFOLD_WPE
#define TEC_RFOLD_WPE 4  // 128 VGPRs (52 B/lane spill): 0.567 ms vs 0.63 at 141 VGPRs (1024 x 4 MiB)
#endif
#ifndef TEC_RFOLD_DIRECT
#ifndef TEC_RFOLD_AP_FOLD
#define TEC_RFOLD_AP_FOLD 1  // aloof planes' U with one constant product (0: two, measurement)
#endif
static_assert(tec::kPft.a_p[0] == (tec::kPft.a_c[0] ^ 1), "a_p = a_c ^ 1 (PFT [[3,2],[2,3]])");
#define TEC_RFOLD_DIRECT 1  // 1: each finished word stored straight to the lost chunk (no staging, no barrier)
#endif
#ifndef TEC_RFOLD_MAXG
#define TEC_RFOLD_MAXG 2  // waves per workgroup at most (direct: 2 measured best; 0.592 -> 0.572 ms, one down 0.590 -> 0.549)
#endif
#ifndef TEC_RFOLD_ST_AUX
#define TEC_RFOLD_ST_AUX 2  // cache policy of the lost-chunk row stores (nt)
#endif

namespace tec {
namespace rfold {

constexpr int kQ = 10, kK = 7, kA = kQ - kK;  // known / aloof nodes of the other column
constexpr int kMaxG = TEC_RFOLD_MAXG;
constexpr uint32_t kStageRows = TEC_RFOLD_DIRECT ? 0u : 2u * kQ;  // LDS rows before the aloof-U rows

// The other column's known set K as a 10-bit mask of positions; its members ascending (kn) and
// the aloof rest (al).
struct KSet {
    int kn[kK], al[kA];
};
constexpr KSet make_kset(uint32_t km) {
    KSet s{};
    int a = 0, b = 0;
    for (int x = 0; x < kQ; x++) {
        if ((km >> x) & 1u) {
            if (a < kK) s.kn[a] = x;
            a++;
        } else {
            if (b < kA) s.al[b] = x;
            b++;
        }
    }
    return s;
}
constexpr int popc10(uint32_t km) {
    int c = 0;
    for (int x = 0; x < kQ; x++) c += (km >> x) & 1u;
    return c;
}

// The instantiated known sets: minimum_to_repair's choice with every other node available
// (0..6), and with other-column node p < 7 unavailable ({0..7} \ {p}).
constexpr uint32_t kFoldSets[8] = {0x07fu, 0x0feu, 0x0fdu, 0x0fbu, 0x0f7u, 0x0efu, 0x0dfu, 0x0bfu};

// D rows: the 10 column nodes (x = 0..9), then the 3 aloof nodes of the other column (al order);
// columns: the known nodes of the other column (kn order).
struct Fold {
    uint8_t D[kQ + kA][kK];
};

constexpr Fold make_fold(int yl, uint32_t km) {
    const Mat g = rs_generator(kK, 2 * kQ);
    const int yo = 1 - yl;
    const KSet ks = make_kset(km);
    Mat gk{};
    gk.rows = gk.cols = kK;
    for (int j = 0; j < kK; j++)
        for (int c = 0; c < kK; c++) gk.v[j][c] = g.v[yo * kQ + ks.kn[j]][c];
    mat_invert(gk);
    Fold f{};
    for (int e = 0; e < kQ + kA; e++) {
        const int node = e < kQ ? yl * kQ + e : yo * kQ + ks.al[e - kQ];
        for (int j = 0; j < kK; j++) {
            uint8_t acc = 0;
            for (int l = 0; l < kK; l++) acc ^= gf_mul(g.v[node][l], gk.v[l][j]);
            f.D[e][j] = acc;
        }
    }
    return f;
}

// PFT relations this kernel hard-wires (A3): uncoupling is pft3; the lost node's C at
// a swapped plane is 2^-1 (U_m + 3 C_m) from column-mate m; an aloof partner gives
// U = 3^-1 (C + 2 U_aloof).  Orientation-free for [[3,2],[2,3]].
static_assert(kPft.l_u[0] == kPft.l_u[1] && kPft.l_c[0] == kPft.l_c[1], "PFT lost-map orientation");
static_assert(kPft.l_u[0] == gf_inv(2) && kPft.l_c[0] == gf_mul(3, gf_inv(2)), "PFT lost-map");
static_assert(kPft.a_c[0] == kPft.a_c[1] && kPft.a_p[0] == kPft.a_p[1], "PFT aloof orientation");

// x / 2 for four packed bytes: shift down, and where the low bit was set add 2^-1 = 0x8e
__device__ __forceinline__ uint32_t half(uint32_t x) {
    const uint32_t lb = x & 0x01010101u;
    const uint32_t red = __builtin_amdgcn_perm(0u, 0x00008e00u, lb);
    return ((x >> 1) & 0x7f7f7f7fu) ^ red;
}
// lost node's C at the mate's swapped plane: 2^-1 (U_m ^ C_m ^ 2 C_m)
__device__ __forceinline__ uint32_t lost_c(uint32_t cm, uint32_t um) { return half(enc::xor3(um, cm, xt(cm))); }

// acc[r] = sum_j D[r][j] u[j] for rows [0, NR) (NR = 13 with the aloof rows, 10 without)
template <int YL, uint32_t KM, int NR>
__device__ __forceinline__ void mds(const uint32_t *u, uint32_t *acc) {
    constexpr Fold F = make_fold(YL, KM);
    uint32_t pend[NR];
    bool hp[NR];
#pragma unroll
    for (int r = 0; r < NR; r++) { acc[r] = 0; hp[r] = false; pend[r] = 0; }
#pragma unroll
    for (int j = 0; j < kK; j++) {
        const Mult<7> mu(u[j]);
#pragma unroll
        for (int r = 0; r < NR; r++) {
            const uint8_t c = F.D[r][j];
#pragma unroll
            for (int i = 0; i < 8; i++) {
                if (!(c >> i & 1)) continue;
                if (hp[r]) {
                    acc[r] = enc::xor3(acc[r], pend[r], mu.m[i]);
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

template <int YL, int G, uint32_t KM>
__device__ __forceinline__ void rep_fold_body(const RepArgs &a) {
    constexpr int YO = 1 - YL;
    static_assert(popc10(KM) == kK, "seven known nodes in the other column");
    constexpr KSet KS = make_kset(KM);
    constexpr uint32_t RS = G * 256u;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    uint8_t *const lds8 = reinterpret_cast<uint8_t *>(lds);  // 2 x 10 staging rows, 21 aloof-U rows
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t col_local = threadIdx.x * 4u;

    const uint32_t tile = xcd_tile(blockIdx.x, gridDim.x);
    const uint32_t job = tile / a.wgs_per_stripe, seg = tile - job * a.wgs_per_stripe;
    typedef const __attribute__((address_space(4))) RepJob cRepJob;
    cRepJob &J = *(cRepJob *)(uintptr_t)(a.jobs + job);
    const uint32_t sc = a.sc, wps = a.words_per_stripe, xl = J.aux & 0xffu;
    const uint32_t seg0 = seg * RS, lseg = min(RS, sc - seg0);
    uint32_t w = seg * G * 64u + threadIdx.x;
    if (w >= wps) w = wps - 1;
    const uint32_t col = w * 4u;
    // A word whose high half lies past the sub-chunk (sc = 2 mod 4, last word) loads the dword 2
    // bytes earlier (the last helper row may end its buffer).  Everything below is byte-parallel
    // (XOR, xtime, halving), so the lane computes on the unrotated dword and rotates only the
    // results it stages.
    const bool tailw = col + 4u > sc;
    const uint32_t vcol = tailw ? col - 2u : col, vsh = tailw ? 2u : 0u;
    // Helper rows are read with global loads off the node's base pointer (SGPR pair) and a 32-bit
    // lane offset; nodes without helper data (the lost node, aloof nodes) carry a copy of another
    // helper's pointer (host-side), so every load is in bounds and needs no branch.
    auto load_h = [&](uint32_t node, uint32_t ri) -> uint32_t {  // helper C of `node` at repair row ri
        const g_u8 *base = (const g_u8 *)J.helper[node];
        return *(const g_u32 *)(base + (ri * sc + vcol));
    };
    const __amdgpu_buffer_rsrc_t rs_out = __builtin_amdgcn_make_buffer_rsrc(J.out, 0, (int)a.cs, 0x00020000);

    // flush geometry: a row segment of lseg bytes as 16-byte blocks (lanes) + a 2-byte tail
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const uint32_t nb = lseg >> 4, tail = lseg & 15u;
    constexpr uint32_t kDrop = 0x80000000u;
    const bool wide_tail = tail != 0 && nb > 0;
    auto blk_off = [&](uint32_t b) -> uint32_t {
        return b < nb ? b * 16u : ((wide_tail && b == nb) ? lseg - 16u : kDrop);
    };
    const uint32_t vo0 = blk_off(lane), vo1 = blk_off(lane + 64u);
    const uint32_t lo0 = vo0 == kDrop ? 0u : vo0, lo1 = vo1 == kDrop ? 0u : vo1;
    const uint32_t vot = (!wide_tail && lane < (tail >> 1)) ? nb * 16u + lane * 2u : kDrop;
    const uint32_t lt_off = nb * 16u + lane * 2u;
    const uint32_t r_beg = (wv * kQ) / G, r_end = ((wv + 1) * kQ) / G;

    // the 10 lost-chunk planes plane p finishes: staged in buffer p & 1, stored whole per row
    // the staging buffer alternates with the STEP, not the plane: with a plane of the known set
    // missing, two consecutive steps can have planes of equal parity (a shared buffer would be
    // refilled while other waves still store it)
    auto finish = [&](uint32_t p, uint32_t step, const uint32_t *acc, const uint32_t *ccm) {
        if constexpr (TEC_RFOLD_DIRECT != 0) {  // each word back where the lane loads (vcol)
#pragma unroll
            for (int x = 0; x < kQ; x++) {
                const uint32_t v = (uint32_t)x == xl ? acc[x] : lost_c(ccm[x], acc[x]);
                const uint32_t plane = YL == 0 ? (uint32_t)x * kQ + p : p * kQ + (uint32_t)x;
                __builtin_amdgcn_raw_buffer_store_b32(v, rs_out, (int)vcol, (int)(plane * sc), TEC_RFOLD_ST_AUX);
            }
            return;
        }
        uint8_t *const stg = lds8 + (step & 1u) * kQ * RS;
#pragma unroll
        for (int x = 0; x < kQ; x++) {
            const uint32_t v = (uint32_t)x == xl ? acc[x] : lost_c(ccm[x], acc[x]);
            *reinterpret_cast<uint32_t *>(stg + x * RS + col_local) = __builtin_amdgcn_alignbyte(v, v, vsh);
        }
        lds_barrier();  // staged; buffer (step + 1) & 1 was flushed before this barrier
        for (uint32_t r = r_beg; r < r_end; r++) {
            const uint8_t *row = stg + r * RS;
            const uint32_t plane = YL == 0 ? r * kQ + p : p * kQ + r;
            const uint32_t off = plane * sc + seg0;
            __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const u32x4 *>(row + lo0), rs_out, (int)vo0, (int)off, TEC_RFOLD_ST_AUX);
            if (RS > 1024u)
                __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const u32x4 *>(row + lo1), rs_out, (int)vo1, (int)off, TEC_RFOLD_ST_AUX);
            if (!wide_tail)
                __builtin_amdgcn_raw_buffer_store_b16(*reinterpret_cast<const uint16_t *>(row + lt_off), rs_out, (int)vot, (int)off, 0);
        }
    };
    // lane-private LDS rows after the staging buffers: aloof node al[i]'s U at plane kn[j]
    auto ua_at = [&](uint32_t i, uint32_t j) {
        return reinterpret_cast<uint32_t *>(lds8 + (kStageRows + i * kK + j) * RS + col_local);
    };

    // Loads of plane p, issued one plane ahead and unconditionally (a branch around a load makes
    // the compiler wait for it inside the branch): the known nodes' C; each one's partner C --
    // known node p at plane kn[j], the helper row another plane loads as its own, so the re-read
    // is an L2 hit; at kn[j] == p it is the node's own C and pft3(C, C) = C (red); for aloof p
    // the value is unused; and the column-mates' C (unused for the lost node).
    uint32_t own[kK], part[kK], cm[kQ];
    auto load_plane = [&](uint32_t p) {
#pragma unroll
        for (int j = 0; j < kK; j++) {
            own[j] = load_h(YO * kQ + KS.kn[j], p);
            part[j] = load_h(YO * kQ + p, (uint32_t)KS.kn[j]);
        }
#pragma unroll
        for (int x = 0; x < kQ; x++) cm[x] = load_h(YL * kQ + x, p);
    };
    load_plane((uint32_t)KS.kn[0]);
    // Both plane loops are unrolled (no loop-carried register copies, whose moves would wait for
    // the in-flight loads and, vmcnt being in order, for the plane's stores), with a scheduling
    // barrier per plane so the compiler does not hoist every plane's loads to the top.
#pragma unroll
    for (int jp = 0; jp < kK; jp++) {  // known planes: every known partner is a helper
        const uint32_t p = (uint32_t)KS.kn[jp];
        __builtin_amdgcn_sched_barrier(0);
        uint32_t u[kK], ccm[kQ], acc[kQ + kA];
#pragma unroll
        for (int j = 0; j < kK; j++) u[j] = enc::pft3(own[j], part[j]);
#pragma unroll
        for (int x = 0; x < kQ; x++) ccm[x] = cm[x];
        load_plane(jp + 1 < kK ? (uint32_t)KS.kn[jp + 1] : (uint32_t)KS.al[0]);
        mds<YL, KM, kQ + kA>(u, acc);
#pragma unroll
        for (int i = 0; i < kA; i++) *ua_at(i, jp) = acc[kQ + i];
        finish(p, (uint32_t)jp, acc, ccm);
    }
#pragma unroll
    for (int ip = 0; ip < kA; ip++) {  // aloof planes: partner aloof node p, U from the known planes
        const uint32_t p = (uint32_t)KS.al[ip];
        __builtin_amdgcn_sched_barrier(0);
        uint32_t u[kK], ccm[kQ], acc[kQ];
#pragma unroll
        for (int j = 0; j < kK; j++) {
#if TEC_RFOLD_AP_FOLD
            // a_c C ^ a_p U with a_p = a_c ^ 1: one table product, a_c (C ^ U) ^ U
            const uint32_t ua = *ua_at(ip, j);
            u[j] = mulc(kPft.a_c[0], own[j] ^ ua) ^ ua;
#else
            u[j] = mulc(kPft.a_c[0], own[j]) ^ mulc(kPft.a_p[0], *ua_at(ip, j));
#endif
        }
#pragma unroll
        for (int x = 0; x < kQ; x++) ccm[x] = cm[x];
        if (ip + 1 < kA) load_plane((uint32_t)KS.al[ip + 1]);
        mds<YL, KM, kQ>(u, acc);
        finish(p, (uint32_t)(kK + ip), acc, ccm);
    }
}

// One launch for every folded stripe of a batch: the job's kernel index (lost column * 8 + set,
// RepJob::aux >> 8) selects the body; uniform per workgroup, so no divergence (a launch per index
// ran 0.79 ms against 0.57 for the two launches of the all-available case, 1024 x 4 MiB).
template <int G>
__global__ void __launch_bounds__(G * 64, TEC_RFOLD_WPE) rep_fold_kernel(RepArgs a) {
    const uint32_t job = xcd_tile(blockIdx.x, gridDim.x) / a.wgs_per_stripe;
    const uint32_t fold = __builtin_amdgcn_readfirstlane(a.jobs[job].aux >> 8);
    switch (fold) {
        case 0: rep_fold_body<0, G, kFoldSets[0]>(a); break;
        case 1: rep_fold_body<0, G, kFoldSets[1]>(a); break;
        case 2: rep_fold_body<0, G, kFoldSets[2]>(a); break;
        case 3: rep_fold_body<0, G, kFoldSets[3]>(a); break;
        case 4: rep_fold_body<0, G, kFoldSets[4]>(a); break;
        case 5: rep_fold_body<0, G, kFoldSets[5]>(a); break;
        case 6: rep_fold_body<0, G, kFoldSets[6]>(a); break;
        case 7: rep_fold_body<0, G, kFoldSets[7]>(a); break;
        case 8: rep_fold_body<1, G, kFoldSets[0]>(a); break;
        case 9: rep_fold_body<1, G, kFoldSets[1]>(a); break;
        case 10: rep_fold_body<1, G, kFoldSets[2]>(a); break;
        case 11: rep_fold_body<1, G, kFoldSets[3]>(a); break;
        case 12: rep_fold_body<1, G, kFoldSets[4]>(a); break;
        case 13: rep_fold_body<1, G, kFoldSets[5]>(a); break;
        case 14: rep_fold_body<1, G, kFoldSets[6]>(a); break;
        default: rep_fold_body<1, G, kFoldSets[7]>(a); break;
    }
}

}  // namespace rfold

// The helper sets of kFoldSets: returns the kernel index (lost column y_l) * 8 + set index for
// such a pattern, else -1.
int repair_fold_column(uint32_t q, uint32_t t, uint32_t k, uint32_t beta, uint32_t sc, uint32_t lost,
                       uint64_t erased_mask, uint64_t aloof_mask) {
    using namespace rfold;
    if (q != (uint32_t)kQ || t != 2 || k != (uint32_t)kK || beta != (uint32_t)kQ || sc < 8 || lost >= 2u * kQ) return -1;
    const uint32_t yl = lost / kQ, yo = 1 - yl;
    const uint64_t col = ((1ull << kQ) - 1ull) << (yl * kQ);
    for (int i = 0; i < 8; i++) {
        const uint64_t alf = (uint64_t)(~kFoldSets[i] & 0x3ffu) << (yo * kQ);
        if (aloof_mask == alf && erased_mask == (col | alf)) return (int)yl * 8 + i;
    }
    return -1;
}

template <int G>
static hipError_t launch_fold_g(const RepArgs &a, uint64_t blocks, hipStream_t s) {
    const size_t lds = (size_t)(rfold::kStageRows + rfold::kA * rfold::kK) * G * 256u;
    hipLaunchKernelGGL((rfold::rep_fold_kernel<G>), dim3((uint32_t)blocks), dim3(G * 64), lds, s, a);
    return hipGetLastError();
}

template <int G>
static hipError_t fold_dispatch(uint32_t g, const RepArgs &a, uint64_t blocks, hipStream_t s) {
    if constexpr (G > 1)
        if (g < (uint32_t)G) return fold_dispatch<G - 1>(g, a, blocks, s);
    return launch_fold_g<G>(a, blocks, s);
}

hipError_t launch_repair_fold(RepArgs a, hipStream_t s) {
    if (a.njobs == 0) return hipSuccess;
    if (a.sc < 8) return hipErrorInvalidValue;
    const uint32_t groups = (a.words_per_stripe + 63) / 64;
    const uint32_t g = groups < (uint32_t)rfold::kMaxG ? groups : (uint32_t)rfold::kMaxG;
    a.wgs_per_stripe = (groups + g - 1) / g;
    const uint64_t blocks = (uint64_t)a.njobs * a.wgs_per_stripe;
    if (blocks > 0x7fffffffull) return hipErrorInvalidValue;
    // waves per workgroup (g <= kMaxG; small sub-chunks use fewer): only 1..kMaxG are built
    return fold_dispatch<rfold::kMaxG>(g, a, blocks, s);
}

}  // namespace tec
