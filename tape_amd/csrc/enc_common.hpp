// enc_common.hpp -- pieces shared by the q = 10, t = 2 Clay encode kernels (encode_stage.hip,
// encode_dma.hip): compile-time coefficient tables and the xtime-selection MDS.
#pragma once
#include "gf_dev.hpp"

namespace tec {
namespace enc {

constexpr int kQ = 10;

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
// The fast kernels hard-wire this: another PFT would need the generic kernel.
static_assert(kPft.u_c[0] == 3 && kPft.u_c[1] == 3 && kPft.u_p[0] == 2 && kPft.u_p[1] == 2, "PFT uncouple");
static_assert(kPft.c_u[0] == 3 && kPft.c_u[1] == 3 && kPft.c_p[0] == 2 && kPft.c_p[1] == 2, "PFT couple");
__device__ __forceinline__ uint32_t pft3(uint32_t a, uint32_t b) { return a ^ xt(a ^ b); }

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// acc[r] = sum_x coef(r, x) * u[x] for the 20-K parity rows, coefficients folded at compile
// time: per input the xtime multiples 2^i u[x], then every row XORs the multiples its
// coefficient selects, two at a time (v_bitop3 xor3), a leftover single carried to the next
// input so each row costs ~ceil(terms / 2) instructions.  SCALED: column-0 parity rows use Gt.
template <int K, bool SCALED, bool TRIVIAL = false>
__device__ __forceinline__ void mds_rows(const uint32_t *u, uint32_t *acc) {
    constexpr Consts<K> RC = make_consts<K>();
    constexpr int NR = 20 - K;
    uint32_t pend[NR];
    bool hp[NR];  // compile-time after unrolling
#pragma unroll
    for (int r = 0; r < NR; r++) { acc[r] = 0; hp[r] = false; pend[r] = 0; }
#pragma unroll
    for (int x = 0; x < K; x++) {
        if constexpr (TRIVIAL) {  // timing builds only
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

// ---- Clay(20,7,16): the MDS as a shared-XOR program (scripts/gen_mds_slp.py) ----
// The generator's columns repeat their coefficients (most values twice), so the 13 rows share
// many XORs of multiples: 105 / 85 XOR3-equivalent instructions per plane word (scaled / plain)
// against ~189 / ~173 row by row.
constexpr int kSlpMaxOps = 160;
constexpr int kSlpSlots = 160;
struct SlpOp {
    uint8_t kind, dst, a, b, c;  // 0: multiples of input dst; 1: mov; 2: xor; 3: xor3
};
struct SlpProg {
    int n;
    SlpOp op[kSlpMaxOps];
    uint8_t out[13];
};
#include "mds_slp.inc"

// The program must compute exactly G (or Gt) of rs_generator(7, 20): evaluated over bit masks
// of the 56 multiples (signal 8x + i = 2^i u_x); every value is defined before it is read.
constexpr bool slp_ok(const SlpProg &P, bool scaled) {
    const Consts<7> RC = make_consts<7>();
    uint64_t sig[kSlpSlots] = {};
    bool def[kSlpSlots] = {};
    for (int i = 0; i < P.n; i++) {
        const SlpOp &o = P.op[i];
        if (o.kind == 0) {
            if (o.dst >= 7) return false;
            for (int j = 0; j < 8; j++) {
                sig[8 * o.dst + j] = 1ull << (8 * o.dst + j);
                def[8 * o.dst + j] = true;
            }
            continue;
        }
        if (o.kind > 3 || o.dst < 56 || o.dst >= kSlpSlots) return false;
        const uint8_t s[3] = {o.a, o.b, o.c};
        uint64_t v = 0;
        for (int j = 0; j < o.kind && j < 3; j++) {
            if (s[j] >= kSlpSlots || !def[s[j]]) return false;
            v ^= sig[s[j]];
        }
        sig[o.dst] = v;
        def[o.dst] = true;
    }
    for (int r = 0; r < 13; r++) {
        uint64_t want = 0;
        for (int x = 0; x < 7; x++) {
            const uint8_t c = (7 + r < kQ && scaled) ? RC.Gt[7 + r][x] : RC.G[7 + r][x];
            for (int i = 0; i < 8; i++)
                if (c >> i & 1) want ^= 1ull << (8 * x + i);
        }
        if (P.out[r] >= kSlpSlots || !def[P.out[r]] || sig[P.out[r]] != want) return false;
    }
    return true;
}
static_assert(slp_ok(kSlpScaled, true), "mds_slp.inc: kSlpScaled != t_u-scaled rs_generator(7, 20)");
static_assert(slp_ok(kSlpPlain, false), "mds_slp.inc: kSlpPlain != rs_generator(7, 20)");

// (a << S) & M ^ r for the multiples below, as one v_bitop3 after the shift.
template <int S>
__device__ __forceinline__ uint32_t shl_and_xor(uint32_t a, uint32_t m, uint32_t r) {
    return ((a << S) & m) ^ r;
}

// m[i] = 2^i u, i = 0..7, in 29 VALU instead of 7 xtimes (35): 2u and 4u share one selector of
// u's top two bits per byte (the reduction of the bits shifted out is a 4-entry v_perm table),
// likewise 8u / 16u from 4u and 32u / 64u from 16u; 128u is one xtime of 64u.
__device__ __forceinline__ void mult8(uint32_t u, uint32_t *m) {
    // reduction bytes for the top two bits b7 b6 (selector value 2 b7 + b6)
    // tables and masks in SGPRs (gfx9 VOP3 takes no literal; left to itself the compiler keeps
    // the tables in VGPRs, which the register budget cannot spare)
    uint32_t kR1, kR2, kM1, kM2;
    asm("s_mov_b32 %0, 0x1d1d0000" : "=s"(kR1));  // 2u: b7 * 0x1d
    asm("s_mov_b32 %0, 0x273a1d00" : "=s"(kR2));  // 4u: b7 * 0x3a ^ b6 * 0x1d
    asm("s_mov_b32 %0, 0xfefefefe" : "=s"(kM1));
    asm("s_mov_b32 %0, 0xfcfcfcfc" : "=s"(kM2));
    m[0] = u;
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const uint32_t b = m[2 * k];
        const uint32_t sel = (b >> 6) & 0x03030303u;
        m[2 * k + 1] = shl_and_xor<1>(b, kM1, __builtin_amdgcn_perm(0u, kR1, sel));
        m[2 * k + 2] = shl_and_xor<2>(b, kM2, __builtin_amdgcn_perm(0u, kR2, sel));
    }
    m[7] = xt(m[6]);
}

#ifndef TEC_MULT8
#define TEC_MULT8 0  // 1: shared-selector multiples (29 VALU per input; +registers: spills at 128)
#endif

// acc[r] = parity row 7 + r of the plane (scaled: rows 7..9 by t_u, as mds_rows<7, true>)
template <bool SCALED>
__device__ __forceinline__ void mds7_slp(const uint32_t *u, uint32_t *acc) {
    constexpr SlpProg P = SCALED ? kSlpScaled : kSlpPlain;
    uint32_t sig[kSlpSlots];
#pragma unroll
    for (int i = 0; i < P.n; i++) {
        const SlpOp &o = P.op[i];
        if (o.kind == 0) {
            // keep the generator's order (its accumulator schedule bounds the live values; the
            // machine scheduler would hoist every input's multiples and spill)
            if (i) __builtin_amdgcn_sched_barrier(0);
            if constexpr (TEC_MULT8) {
                mult8(u[o.dst], sig + 8 * o.dst);
            } else {
                const Mult<7> mu(u[o.dst]);
#pragma unroll
                for (int q = 0; q < 8; q++) sig[8 * o.dst + q] = mu.m[q];
            }
        }
        else if (o.kind == 1)
            sig[o.dst] = sig[o.a];
        else if (o.kind == 2)
            sig[o.dst] = sig[o.a] ^ sig[o.b];
        else
            sig[o.dst] = xor3(sig[o.a], sig[o.b], sig[o.c]);
    }
#pragma unroll
    for (int r = 0; r < 13; r++) acc[r] = sig[P.out[r]];
}

}  // namespace enc
}  // namespace tec
