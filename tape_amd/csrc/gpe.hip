// gpe.hip -- generic layered Clay engine for arbitrary erasure patterns.
//
// Covers ClayCoder::decode (lib/slicer/src/clay.rs:106-122 -> clay_codes decode, the per-stripe
// loop of Slicer::decode slicer.rs:333-361), encode for profiles outside the q=10,t=2 fast path,
// and ClayCoder::repair (lib/slicer/src/repair.rs:75-88, per-stripe loop :337-363).
//
// A block owns kGpeWords 4-column words of one stripe for ALL planes; 32 plane-threads per word
// walk the planes of each decode level (intersection score order, host-sorted).  Per plane:
// uncouple the known nodes (pairwise transform with the coupling partner, which is either an
// input chunk or a C recovered at a lower level, held in LDS), multiply by the pattern's MDS
// decoding matrix (v_perm tables, scalar-loaded), then after a barrier re-couple the erased
// nodes (copy / type-1 / pair), keeping recovered C and U in LDS for later levels.
#include "kernels.hpp"
#include "gf_dev.hpp"
#include "dev_io.hpp"

namespace tec {

__device__ __forceinline__ uint32_t popc64(uint64_t v) { return (uint32_t)__popcll(v); }

template <int MAXE>
__global__ void __launch_bounds__(kGpeWords * kGpePlaneThreads) gpe_kernel(GpeArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const uint32_t job = blockIdx.x / a.groups_per_stripe;
    const uint32_t grp = blockIdx.x - job * a.groups_per_stripe;
    const uint32_t wi = threadIdx.x % kGpeWords, pt = threadIdx.x / kGpeWords;
    uint32_t w = a.word_base + grp * kGpeWords + wi;
    if (w >= a.word_end) w = a.word_end - 1;
    const GpeJob J = a.jobs[job];
    const GpePattern &PT = a.patterns[J.pattern];
    const WordPos wp = word_pos(w, a.sc);
    const uint32_t alpha = a.alpha, q = a.q, t = a.t, sc = a.sc;
    const uint32_t ner = PT.nerased, nkn = PT.nknown;
    const uint64_t emask = PT.erased_mask;

    uint32_t *const Ur = lds;                                     // [e][z][wi]
    uint32_t *const Cr = lds + (size_t)ner * alpha * kGpeWords;   // [e][z][wi]
    uint8_t *const dig = reinterpret_cast<uint8_t *>(lds + (size_t)2 * ner * alpha * kGpeWords);
    for (uint32_t i = threadIdx.x; i < alpha * t; i += blockDim.x) {
        const uint32_t z = i / t, y = i - z * t;
        dig[i] = (uint8_t)((z / a.qpow[t - 1 - y]) % q);
    }
    lds_barrier();

    auto ext_of = [&](uint32_t node) -> int {
        return node < a.k ? (int)node : (node < a.k + a.nu ? -1 : (int)(node - a.nu));
    };
    auto load_in = [&](uint32_t node, uint32_t z) -> uint32_t {
        const int e = ext_of(node);
        if (e < 0) return 0u;
        uint32_t side = (uint32_t)e;
        if (a.in_rotated) { side += J.rot; side = side >= a.n ? side - a.n : side; }
        return ld_word(J.in, (uint64_t)side * a.in_stride + (uint64_t)z * sc + wp.c, J.in_len, wp.nc);
    };
    auto store_out = [&](uint32_t node, uint32_t z, uint32_t v) {
        const int e = ext_of(node);
        if (e < 0) return;
        uint32_t side = (uint32_t)e;
        if (a.out_rotated) { side += J.rot; side = side >= a.n ? side - a.n : side; }
        st_word_trim(J.out, (uint64_t)side * a.out_stride + (uint64_t)z * sc + wp.c, J.out_len, v, wp.nc);
    };
    auto slot = [&](uint32_t *base, uint32_t e, uint32_t z) -> uint32_t & {
        return base[((size_t)e * alpha + z) * kGpeWords + wi];
    };
    auto eidx = [&](uint32_t node) -> uint32_t { return popc64(emask & ((1ull << node) - 1ull)); };

    const uint16_t *planes = a.plane_pool + PT.planes_off;
    for (uint32_t L = 0; L < PT.nlevels; L++) {
        const uint32_t ls = PT.level_start[L], le = PT.level_start[L + 1];
        // ---- phase A: uncouple known nodes, MDS-solve the erased uncoupled values ----
        for (uint32_t pi = ls + pt; pi < le; pi += kGpePlaneThreads) {
            const uint32_t z = planes[pi];
            uint32_t acc[MAXE];
#pragma unroll
            for (int e = 0; e < MAXE; e++) acc[e] = 0;
            for (uint32_t j = 0; j < nkn; j++) {
                const uint32_t node = PT.known[j];
                const uint32_t x = node % q, y = node / q;
                const uint32_t c = load_in(node, z);
                if ((a.out_mask >> node) & 1ull) store_out(node, z, c);
                const uint32_t zy = dig[z * t + y];
                uint32_t u;
                if (zy == x) {
                    u = c;
                } else {
                    const uint32_t sw = y * q + zy;
                    const uint32_t zsw = z + (x - zy) * a.qpow[t - 1 - y];
                    const uint32_t p = ((emask >> sw) & 1ull) ? slot(Cr, eidx(sw), zsw) : load_in(sw, zsw);
                    u = (x > zy) ? (mulc(kPft.u_c[1], c) ^ mulc(kPft.u_p[1], p))
                                 : (mulc(kPft.u_c[0], c) ^ mulc(kPft.u_p[0], p));
                }
                const Sel s(u);
#pragma unroll
                for (int e = 0; e < MAXE; e++)
                    if ((uint32_t)e < ner) acc[e] = perm_mul_acc(acc[e], s, PT.D[e][j].t[0], PT.D[e][j].t[1], PT.D[e][j].t[2], PT.D[e][j].t[3], PT.D[e][j].t[4]);
            }
#pragma unroll
            for (int e = 0; e < MAXE; e++)
                if ((uint32_t)e < ner) slot(Ur, e, z) = acc[e];
        }
        lds_barrier();
        // ---- phase B: re-couple the erased nodes of this level ----
        for (uint32_t pi = ls + pt; pi < le; pi += kGpePlaneThreads) {
            const uint32_t z = planes[pi];
            for (uint32_t e = 0; e < ner; e++) {
                const uint32_t node = PT.erased[e];
                const uint32_t x = node % q, y = node / q;
                const uint32_t u = slot(Ur, e, z);
                const uint32_t zy = dig[z * t + y];
                uint32_t cval;
                if (zy == x) {
                    cval = u;
                } else {
                    const uint32_t sw = y * q + zy;
                    const uint32_t zsw = z + (x - zy) * a.qpow[t - 1 - y];
                    const bool hi = x > zy;
                    if (!((emask >> sw) & 1ull)) {
                        const uint32_t p = load_in(sw, zsw);
                        cval = hi ? (mulc(kPft.t_u[1], u) ^ mulc(kPft.t_p[1], p))
                                  : (mulc(kPft.t_u[0], u) ^ mulc(kPft.t_p[0], p));
                    } else {
                        const uint32_t pu = slot(Ur, eidx(sw), zsw);
                        cval = hi ? (mulc(kPft.c_u[1], u) ^ mulc(kPft.c_p[1], pu))
                                  : (mulc(kPft.c_u[0], u) ^ mulc(kPft.c_p[0], pu));
                    }
                }
                slot(Cr, e, z) = cval;
                if ((a.out_mask >> node) & 1ull) store_out(node, z, cval);
            }
        }
        lds_barrier();
    }
}

// ------------------------------------------------------------------------------------------
// Bandwidth-optimal repair of one lost chunk from d helpers x beta sub-chunks (Ceph
// repair_one_lost_chunk): only the beta repair planes are processed, in order of their
// intersection score with the erased set (lost column + aloof nodes).
// ------------------------------------------------------------------------------------------
template <int MAXE>
__global__ void __launch_bounds__(kGpeWords * kGpePlaneThreads) repair_kernel(RepArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const uint32_t job = blockIdx.x / a.groups_per_stripe;
    const uint32_t grp = blockIdx.x - job * a.groups_per_stripe;
    const uint32_t wi = threadIdx.x % kGpeWords, pt = threadIdx.x / kGpeWords;
    uint32_t w = grp * kGpeWords + wi;
    if (w >= a.words_per_stripe) w = a.words_per_stripe - 1;
    const RepJob &J = a.jobs[job];
    const RepPattern &PT = a.patterns[J.pattern];
    const WordPos wp = word_pos(w, a.sc);
    const uint32_t alpha = a.alpha, q = a.q, t = a.t, sc = a.sc, beta = PT.beta;
    const uint32_t ner = PT.nerased, nkn = PT.nknown;
    const uint64_t emask = PT.erased_mask, amask = PT.aloof_mask;
    const uint32_t lost = PT.lost, xl = lost % q, yl = lost / q;
    uint8_t *const outp = J.out;

    uint32_t *const Ur = lds;  // [e][repair plane index][wi]
    uint8_t *const dig = reinterpret_cast<uint8_t *>(lds + (size_t)ner * beta * kGpeWords);
    for (uint32_t i = threadIdx.x; i < alpha * t; i += blockDim.x) {
        const uint32_t z = i / t, y = i - z * t;
        dig[i] = (uint8_t)((z / a.qpow[t - 1 - y]) % q);
    }
    lds_barrier();

    const uint16_t *pind = a.plane_ind + (size_t)J.pattern * alpha;
    auto load_h = [&](uint32_t node, uint32_t ri) -> uint32_t {
        const uint8_t *h = J.helper[node];
        if (!h) return 0u;  // shortened (nu) node
        return ld_word(h, (uint64_t)ri * sc + wp.c, ~0ull, wp.nc);
    };
    auto slot = [&](uint32_t e, uint32_t ri) -> uint32_t & {
        return Ur[((size_t)e * beta + ri) * kGpeWords + wi];
    };
    auto eidx = [&](uint32_t node) -> uint32_t { return popc64(emask & ((1ull << node) - 1ull)); };

    const uint16_t *planes = a.plane_pool + PT.planes_off;
    for (uint32_t L = 0; L < PT.nlevels; L++) {
        const uint32_t ls = PT.level_start[L], le = PT.level_start[L + 1];
        for (uint32_t pi = ls + pt; pi < le; pi += kGpePlaneThreads) {
            const uint32_t z = planes[pi];
            const uint32_t ri = pind[z];
            uint32_t acc[MAXE];
#pragma unroll
            for (int e = 0; e < MAXE; e++) acc[e] = 0;
            for (uint32_t j = 0; j < nkn; j++) {
                const uint32_t node = PT.known[j];
                const uint32_t x = node % q, y = node / q;
                const uint32_t c = load_h(node, ri);
                const uint32_t zy = dig[z * t + y];
                uint32_t u;
                if (zy == x) {
                    u = c;
                } else {
                    const uint32_t sw = y * q + zy;
                    const uint32_t zsw = z + (x - zy) * a.qpow[t - 1 - y];
                    const uint32_t rsw = pind[zsw];
                    const bool hi = x > zy;
                    if ((amask >> sw) & 1ull) {
                        const uint32_t pu = slot(eidx(sw), rsw);
                        u = hi ? (mulc(kPft.a_c[1], c) ^ mulc(kPft.a_p[1], pu))
                               : (mulc(kPft.a_c[0], c) ^ mulc(kPft.a_p[0], pu));
                    } else {
                        const uint32_t p = load_h(sw, rsw);
                        u = hi ? (mulc(kPft.u_c[1], c) ^ mulc(kPft.u_p[1], p))
                               : (mulc(kPft.u_c[0], c) ^ mulc(kPft.u_p[0], p));
                    }
                }
                const Sel s(u);
#pragma unroll
                for (int e = 0; e < MAXE; e++)
                    if ((uint32_t)e < ner) acc[e] = perm_mul_acc(acc[e], s, PT.D[e][j].t[0], PT.D[e][j].t[1], PT.D[e][j].t[2], PT.D[e][j].t[3], PT.D[e][j].t[4]);
            }
#pragma unroll
            for (int e = 0; e < MAXE; e++) {
                if ((uint32_t)e >= ner) continue;
                const uint32_t node = PT.erased[e];
                slot(e, ri) = acc[e];
                if (node == lost) {
                    // the lost node is red in every repair plane: C = U
                    st_word(outp + (uint64_t)z * sc + wp.c, acc[e], wp.nc);
                } else if (!((amask >> node) & 1ull)) {
                    // column-mate: its helper C and uncoupled U give the lost node's C at z_sw
                    const uint32_t x = node % q;
                    const uint32_t zsw = z + (x - xl) * a.qpow[t - 1 - yl];
                    const uint32_t c = load_h(node, ri);
                    const uint32_t v = (x > xl) ? (mulc(kPft.l_c[1], c) ^ mulc(kPft.l_u[1], acc[e]))
                                                : (mulc(kPft.l_c[0], c) ^ mulc(kPft.l_u[0], acc[e]));
                    st_word(outp + (uint64_t)zsw * sc + wp.c, v, wp.nc);
                }
            }
        }
        lds_barrier();
    }
}

template <int E>
static hipError_t launch_gpe_t(const GpeArgs &a, hipStream_t s) {
    const size_t lds = (size_t)2 * E * a.alpha * kGpeWords * 4 + a.alpha * a.t + 16;
    if (lds > 64 * 1024) {
        hipError_t e = ensure_dyn_lds(reinterpret_cast<const void *>(gpe_kernel<E>), lds);
        if (e != hipSuccess) return e;
    }
    const uint64_t blocks = (uint64_t)a.njobs * a.groups_per_stripe;
    hipLaunchKernelGGL(gpe_kernel<E>, dim3((uint32_t)blocks), dim3(kGpeWords * kGpePlaneThreads), lds, s, a);
    return hipGetLastError();
}

template <int E>
static hipError_t launch_rep_t(const RepArgs &a, hipStream_t s) {
    const size_t lds = (size_t)E * (a.alpha / a.q) * kGpeWords * 4 + a.alpha * a.t + 16;
    if (lds > 64 * 1024) {
        hipError_t e = ensure_dyn_lds(reinterpret_cast<const void *>(repair_kernel<E>), lds);
        if (e != hipSuccess) return e;
    }
    const uint64_t blocks = (uint64_t)a.njobs * a.groups_per_stripe;
    hipLaunchKernelGGL(repair_kernel<E>, dim3((uint32_t)blocks), dim3(kGpeWords * kGpePlaneThreads), lds, s, a);
    return hipGetLastError();
}

hipError_t launch_gpe(const GpeArgs &a, uint32_t max_erased, hipStream_t s) {
    if (a.njobs == 0) return hipSuccess;
    if (max_erased <= 4) return launch_gpe_t<4>(a, s);
    if (max_erased <= 8) return launch_gpe_t<8>(a, s);
    if (max_erased <= 13) return launch_gpe_t<13>(a, s);
    if (max_erased <= kGpeMaxErased) return launch_gpe_t<kGpeMaxErased>(a, s);
    return hipErrorInvalidValue;
}

hipError_t launch_repair(const RepArgs &a, uint32_t max_erased, hipStream_t s) {
    if (a.njobs == 0) return hipSuccess;
    if (max_erased <= 4) return launch_rep_t<4>(a, s);
    if (max_erased <= 8) return launch_rep_t<8>(a, s);
    if (max_erased <= 13) return launch_rep_t<13>(a, s);
    if (max_erased <= kGpeMaxErased) return launch_rep_t<kGpeMaxErased>(a, s);
    return hipErrorInvalidValue;
}

}  // namespace tec
