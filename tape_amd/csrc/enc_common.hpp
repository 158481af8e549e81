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

}  // namespace enc
}  // namespace tec
