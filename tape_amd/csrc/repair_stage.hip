// repair_stage.hip -- bandwidth-optimal repair of one lost chunk (Ceph repair_one_lost_chunk
// restated) for q = 10 profiles: ClayCoder::repair (lib/slicer/src/repair.rs:
// 75-88) inside Slicer::repair's per-stripe loop (repair.rs:337-363).
//
// Algebra: only the beta = alpha / q repair planes (z_{y_lost} = x_lost) are decoded.  Erased =
// the lost node's whole column (lost + q-1 column-mates) plus the aloof nodes (not helpers);
// known = the remaining helpers.  Per repair plane: uncouple the known helpers (partner a helper:
// both C's read; partner aloof: its U from an earlier level), MDS-solve the erased U (the
// pattern's decoding matrix as v_perm tables, scalar-loaded), then the lost node is red (C = U)
// and each column-mate's helper C and solved U give the lost chunk at the mate's swapped plane.
//
// Work decomposition (MI355X), as the encode (encode_stage.hip): a workgroup owns one stripe's
// row segment (G <= 6 waves x 64 lanes x 4 columns) and walks the repair planes in level order;
// loads are one dword per lane down each helper's sub-chunk rows (coalesced, 256 B per wave
// instruction); the 10 lost-chunk rows each plane finishes are staged in LDS and written whole
// by one wave each (HBM lines whole per wave); aloof U's stay in lane-private LDS rows.
#include "kernels.hpp"
#include "gf_dev.hpp"
#include "dev_io.hpp"

#ifndef TEC_REP_PRIO
#define TEC_REP_PRIO 0  // wave priority during a plane's compute (s_setprio), 0 = off
#endif
#ifndef TEC_REP_ST_AUX
#define TEC_REP_ST_AUX 2  // cache policy of the lost-chunk row stores (2 = nt: ~1 % faster)
#endif

namespace tec {
namespace rstage {

#ifndef TEC_REP_DIRECT
#define TEC_REP_DIRECT 1  // each finished word stored straight to the lost chunk (no staging, no barrier)
#endif
#ifndef TEC_REP_MAXG
#define TEC_REP_MAXG 2  // waves per workgroup at most (6 with staging)
#endif

constexpr int kQ = 10;        // q of the supported profiles (beta = 10 repair planes)
constexpr int kMaxG = TEC_REP_MAXG;
constexpr int kOutRows = TEC_REP_DIRECT ? 0 : kQ;  // staging: lost (red) + q-1 column-mates per plane
constexpr int kMaxAloof = 4;
constexpr int kLdsRows = kOutRows + kMaxAloof * kQ;

inline size_t lds_bytes(uint32_t g) { return (size_t)kLdsRows * g * 256u; }

template <int MAXE, int MAXK, int G>
__global__ void __launch_bounds__(G * 64, 3) rep_stage_kernel(RepArgs a) {
    constexpr uint32_t RS = G * 256u;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    uint8_t *const lds8 = reinterpret_cast<uint8_t *>(lds);  // rows [0, 10) staging, then aloof U rows
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t col_local = threadIdx.x * 4u;

    const uint32_t tile = xcd_tile(blockIdx.x, gridDim.x);
    const uint32_t job = tile / a.wgs_per_stripe, seg = tile - job * a.wgs_per_stripe;
    typedef const __attribute__((address_space(4))) RepJob cRepJob;
    typedef const __attribute__((address_space(4))) RepPattern cRepPattern;
    cRepJob &J = *(cRepJob *)(uintptr_t)(a.jobs + job);
    cRepPattern &PT = *(cRepPattern *)(uintptr_t)(a.patterns + J.pattern);
    const uint32_t sc = a.sc, beta = PT.beta, wps = a.words_per_stripe;
    const uint32_t seg0 = seg * RS, lseg = min(RS, sc - seg0);
    uint32_t w = seg * G * 64u + threadIdx.x;
    if (w >= wps) w = wps - 1;
    const uint32_t col = w * 4u;
    // A word whose high half lies past the sub-chunk (sc = 2 mod 4, last word) would straddle the
    // end of the last helper row: it loads the dword 2 bytes earlier; staged rows need its bytes
    // rotated into column order, direct stores put it back where it was loaded (the arithmetic
    // is byte-wise).
    const bool tailw = col + 4u > sc;
    const uint32_t vcol = tailw ? col - 2u : col, vsh = tailw ? 2u : 0u;
    const uint32_t ner = PT.nerased, nkn = PT.nknown;
    const __amdgpu_buffer_rsrc_t rs_out = __builtin_amdgcn_make_buffer_rsrc(J.out, 0, (int)a.cs, 0x00020000);
    auto load_h = [&](uint32_t node, uint32_t ri) -> uint32_t {  // helper C of `node` at repair row ri
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc((void *)J.helper[node], 0, J.helper[node] ? (int)(beta * sc) : 0, 0x00020000);
        const uint32_t v = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)vcol, (int)(ri * sc), 0);
        return TEC_REP_DIRECT ? v : __builtin_amdgcn_alignbyte(v, v, vsh);
    };
    typedef const __attribute__((address_space(4))) uint32_t cU32;
    cU32 *oplane_p = nullptr;  // the plane's staging row -> lost-chunk plane map (direct), scalar-loaded
    auto stage = [&](uint32_t r, uint32_t v) {
        if constexpr (TEC_REP_DIRECT != 0)
            __builtin_amdgcn_raw_buffer_store_b32(v, rs_out, (int)vcol, (int)(oplane_p[r] * sc), TEC_REP_ST_AUX);
        else
            *reinterpret_cast<uint32_t *>(lds8 + r * RS + col_local) = v;
    };

    // flush: staging row r -> lost-chunk plane (r == 0: z; else the column-mate's swapped plane)
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
    const uint32_t r_beg = (wv * kOutRows) / G, r_end = ((wv + 1) * kOutRows) / G;

    // uniform control data through the constant address space (scalar loads)
    typedef const __attribute__((address_space(4))) RepProg cRepProg;
    typedef const __attribute__((address_space(4))) PermTab cPermTab;
    cRepProg &PR = *(cRepProg *)(uintptr_t)(a.progs + J.pattern);
    cPermTab(*D)[kGpeMaxKnown] = (cPermTab(*)[kGpeMaxKnown])(uintptr_t)(&PT.D[0][0]);
    // every load of a plane: the known helpers' C, their helper partners' C and the column-mates'
    // C; issued one plane ahead
    uint32_t cv[MAXK], pv[MAXK], mcv[MAXE];
    auto load_plane = [&](uint32_t pi) {
        const auto &S = PR.step[pi];
        const uint32_t ri = S.ri;
#pragma unroll
        for (int j = 0; j < MAXK; j++) {
            cv[j] = pv[j] = 0;
            if ((uint32_t)j < nkn) {
                cv[j] = load_h(PR.knode0[j], ri);
                const uint32_t kk = S.kkind[j];
                if (kk == 1 || kk == 2) pv[j] = load_h(S.knode[j], S.krow[j]);
            }
        }
#pragma unroll
        for (int e = 0; e < MAXE; e++) {
            mcv[e] = 0;
            if ((uint32_t)e < ner && PR.ekind[e] >= 2) mcv[e] = load_h(PR.enode[e], ri);
        }
    };
    load_plane(0);
    for (uint32_t pi = 0; pi < (uint32_t)kQ; pi++) {
        const auto &S = PR.step[pi];
        const uint32_t ri = S.ri;
        uint32_t ccv[MAXK], cpv[MAXK], cmcv[MAXE];
#pragma unroll
        for (int j = 0; j < MAXK; j++) ccv[j] = cv[j], cpv[j] = pv[j];
#pragma unroll
        for (int e = 0; e < MAXE; e++) cmcv[e] = mcv[e];
        if (pi + 1 < (uint32_t)kQ) load_plane(pi + 1);
        if constexpr (TEC_REP_PRIO) __builtin_amdgcn_s_setprio(TEC_REP_PRIO);
        uint32_t acc[MAXE];
#pragma unroll
        for (int e = 0; e < MAXE; e++) acc[e] = 0;
#pragma unroll
        for (int j = 0; j < MAXK; j++) {
            if ((uint32_t)j >= nkn) continue;
            const uint32_t c = ccv[j], kk = S.kkind[j];
            uint32_t u = c;
            if (kk == 1) u = mulc(kPft.u_c[0], c) ^ mulc(kPft.u_p[0], cpv[j]);
            if (kk == 2) u = mulc(kPft.u_c[1], c) ^ mulc(kPft.u_p[1], cpv[j]);
            if (kk >= 3) {
                const uint32_t pu = *reinterpret_cast<const uint32_t *>(lds8 + (kOutRows + S.krow[j]) * RS + col_local);
                u = kk == 4 ? (mulc(kPft.a_c[1], c) ^ mulc(kPft.a_p[1], pu)) : (mulc(kPft.a_c[0], c) ^ mulc(kPft.a_p[0], pu));
            }
            const Sel s(u);
#pragma unroll
            for (int e = 0; e < MAXE; e++)
                if ((uint32_t)e < ner) acc[e] = perm_mul_acc(acc[e], s, D[e][j].t[0], D[e][j].t[1], D[e][j].t[2], D[e][j].t[3], D[e][j].t[4]);
        }
        if constexpr (TEC_REP_DIRECT == 0) lds_barrier();  // B1: the previous plane's rows have been read out of staging
        oplane_p = S.oplane;
#pragma unroll
        for (int e = 0; e < MAXE; e++) {
            if ((uint32_t)e >= ner) continue;
            const uint32_t kind = PR.ekind[e], row = PR.erow[e];
            if (kind == 0) {
                *reinterpret_cast<uint32_t *>(lds8 + (kOutRows + row * kQ + ri) * RS + col_local) = acc[e];
            } else if (kind == 1) {
                stage(0, acc[e]);  // the lost node is red in every repair plane: C = U
            } else {
                // column-mate: its helper C and solved U give the lost node's C at the swapped plane
                const uint32_t v = kind == 3 ? (mulc(kPft.l_c[1], cmcv[e]) ^ mulc(kPft.l_u[1], acc[e]))
                                             : (mulc(kPft.l_c[0], cmcv[e]) ^ mulc(kPft.l_u[0], acc[e]));
                stage(row, v);
            }
        }
        if constexpr (TEC_REP_PRIO) __builtin_amdgcn_s_setprio(0);
        if constexpr (TEC_REP_DIRECT != 0) continue;
        lds_barrier();  // B2: the plane's rows are staged
        for (uint32_t r = r_beg; r < r_end; r++) {
            const uint8_t *row = lds8 + r * RS;
            const uint32_t off = S.oplane[r] * sc + seg0;
            __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const u32x4 *>(row + lo0), rs_out, (int)vo0, (int)off, TEC_REP_ST_AUX);
            if (RS > 1024u)
                __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const u32x4 *>(row + lo1), rs_out, (int)vo1, (int)off, TEC_REP_ST_AUX);
            if (!wide_tail)
                __builtin_amdgcn_raw_buffer_store_b16(*reinterpret_cast<const uint16_t *>(row + lt_off), rs_out, (int)vot, (int)off, 0);
        }
    }
}

}  // namespace rstage

bool repair_stage_supported(uint32_t q, uint32_t beta, uint32_t sc, uint32_t nerased, uint32_t nknown, uint64_t aloof_mask) {
    return q == (uint32_t)rstage::kQ && beta == (uint32_t)rstage::kQ && sc >= 8 && nerased <= 13 && nknown <= 10 &&
           __builtin_popcountll(aloof_mask) <= rstage::kMaxAloof;
}

template <int G>
static hipError_t launch_rep_stage_g(const RepArgs &a, uint64_t blocks, hipStream_t s) {
    const size_t lds = rstage::lds_bytes(G);
    hipError_t e = ensure_dyn_lds(reinterpret_cast<const void *>(rstage::rep_stage_kernel<13, 10, G>), lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((rstage::rep_stage_kernel<13, 10, G>), dim3((uint32_t)blocks), dim3(G * 64), lds, s, a);
    return hipGetLastError();
}

template <int G>
static hipError_t rep_stage_dispatch(uint32_t g, const RepArgs &a, uint64_t blocks, hipStream_t s) {
    if constexpr (G > 1)
        if (g < (uint32_t)G) return rep_stage_dispatch<G - 1>(g, a, blocks, s);
    return launch_rep_stage_g<G>(a, blocks, s);
}

hipError_t launch_repair_stage(RepArgs a, hipStream_t s) {
    if (a.njobs == 0) return hipSuccess;
    const uint32_t groups = (a.words_per_stripe + 63) / 64;
    const uint32_t g = groups < (uint32_t)rstage::kMaxG ? groups : (uint32_t)rstage::kMaxG;
    a.wgs_per_stripe = (groups + g - 1) / g;
    const uint64_t blocks = (uint64_t)a.njobs * a.wgs_per_stripe;
    if (blocks > 0x7fffffffull) return hipErrorInvalidValue;
    return rep_stage_dispatch<rstage::kMaxG>(g, a, blocks, s);  // only 1..kMaxG waves are built
}

}  // namespace tec
