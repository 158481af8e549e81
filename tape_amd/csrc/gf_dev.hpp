// gf_dev.hpp -- packed GF(2^8) arithmetic on gfx950 VALU (4 byte-columns per 32-bit lane).
//
// Two multiply forms, chosen at compile time per use site:
//   * xtime "multiples": x, 2x, 4x, ... are built with 6 VALU ops per doubling and a
//     compile-time coefficient becomes a straight XOR selection (v_xor3_b32 after isel).  Used
//     where one input feeds many products (the per-plane MDS) or for tiny constants (2, 3).
//   * 2-bit v_perm_b32 tables: mul(c, x) = XOR_i perm(T_i, T_i, (x >> 2i) & 0x03030303), with the
//     four table dwords in SGPRs (compile-time constants, or s_load'ed for run-time matrices).
//     Used for single-use products by "heavy" constants and for run-time (decode) matrices.
// No MFMA: this is byte-wise finite-field arithmetic, not a float contraction.
#pragma once
#include <hip/hip_runtime.h>
#include "gf.hpp"

namespace tec {

// x * 2 for four packed bytes: ((x & 0x7f..) << 1) ^ (0x1d where the byte's top bit was set)
__device__ __forceinline__ uint32_t xt(uint32_t x) {
    const uint32_t hb = (x >> 7) & 0x01010101u;
    const uint32_t red = __builtin_amdgcn_perm(0u, 0x00001d00u, hb);
    return ((x & 0x7f7f7f7fu) << 1) ^ red;
}

constexpr int msb8(uint8_t c) {
    int m = -1;
    for (int i = 0; i < 8; i++)
        if (c >> i & 1) m = i;
    return m;
}

// Multiples m[i] = x * 2^i for i <= top.
template <int TOP>
struct Mult {
    uint32_t m[TOP + 1];
    __device__ __forceinline__ explicit Mult(uint32_t x) {
        m[0] = x;
#pragma unroll
        for (int i = 1; i <= TOP; i++) m[i] = xt(m[i - 1]);
    }
    // c * x for a coefficient that folds to a constant after unrolling
    __device__ __forceinline__ uint32_t mul(uint8_t c) const {
        uint32_t r = 0;
#pragma unroll
        for (int i = 0; i <= TOP; i++)
            if (c >> i & 1) r ^= m[i];
        return r;
    }
};

struct Sel {
    uint32_t s0, s1, s2, s3;
    __device__ __forceinline__ Sel() {}
    __device__ __forceinline__ explicit Sel(uint32_t x)
        : s0(x & 0x03030303u), s1((x >> 2) & 0x03030303u), s2((x >> 4) & 0x03030303u),
          s3((x >> 6) & 0x03030303u) {}
};

__device__ __forceinline__ uint32_t perm_mul(const Sel &s, uint32_t t0, uint32_t t1, uint32_t t2,
                                             uint32_t t3) {
    const uint32_t a = __builtin_amdgcn_perm(t0, t0, s.s0);
    const uint32_t b = __builtin_amdgcn_perm(t1, t1, s.s1);
    const uint32_t c = __builtin_amdgcn_perm(t2, t2, s.s2);
    const uint32_t d = __builtin_amdgcn_perm(t3, t3, s.s3);
    return a ^ b ^ c ^ d;
}

// acc ^ c * x in six VALU: four v_perm and two v_bitop3 XOR3 (the backend does not form XOR3
// from the plain expression, which costs four v_xor_b32)
__device__ __forceinline__ uint32_t perm_mul_acc(uint32_t acc, const Sel &s, uint32_t t0, uint32_t t1, uint32_t t2,
                                                 uint32_t t3) {
    const uint32_t a = __builtin_amdgcn_perm(t0, t0, s.s0);
    const uint32_t b = __builtin_amdgcn_perm(t1, t1, s.s1);
    const uint32_t c = __builtin_amdgcn_perm(t2, t2, s.s2);
    const uint32_t d = __builtin_amdgcn_perm(t3, t3, s.s3);
    return __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_bitop3_b32(acc, a, b, 0x96), c, d, 0x96);
}

__device__ __forceinline__ uint32_t perm_mul(const Sel &s, const PermTab &t) {
    return perm_mul(s, t.t[0], t.t[1], t.t[2], t.t[3]);
}

// c * x for a compile-time-foldable constant used once.
__device__ __forceinline__ uint32_t mulc(uint8_t c, uint32_t x) {
    if (c == 0) return 0;
    if (c == 1) return x;
    if (msb8(c) <= 1) {  // 2 or 3
        const uint32_t x2 = xt(x);
        return (c & 1) ? (x2 ^ x) : x2;
    }
    const PermTab t = perm_tab(c);
    return perm_mul(Sel(x), t);
}

}  // namespace tec
