// gf_dev.hpp -- packed GF(2^8) arithmetic on gfx950 VALU (4 byte-columns per 32-bit lane).
//
// Two multiply forms, chosen at compile time per use site:
//   * xtime "multiples": x, 2x, 4x, ... are built with 6 VALU ops per doubling and a
//     compile-time coefficient becomes a straight XOR selection (v_xor3_b32 after isel).  Used
//     where one input feeds many products (the per-plane MDS) or for tiny constants (2, 3).
//   * v_perm_b32 tables over the byte's 3-, 3- and 2-bit fields: mul(c, x) = XOR of three perms,
//     with the five table dwords in SGPRs (compile-time constants, or s_load'ed for run-time matrices).
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

// Byte fields of four packed bytes, as v_perm selectors: bits [0,3), [3,6) (one 8-entry table
// pair each) and [6,8) (a 4-entry table).
struct Sel {
    uint32_t s0, s1, s2;
    __device__ __forceinline__ Sel() {}
    __device__ __forceinline__ explicit Sel(uint32_t x)
        : s0(x & 0x07070707u), s1((x >> 3) & 0x07070707u), s2((x >> 6) & 0x03030303u) {}
};

__device__ __forceinline__ uint32_t gf_xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

__device__ __forceinline__ uint32_t perm_mul(const Sel &s, uint32_t t0, uint32_t t1, uint32_t t2, uint32_t t3,
                                             uint32_t t4) {
    return gf_xor3(__builtin_amdgcn_perm(t1, t0, s.s0), __builtin_amdgcn_perm(t3, t2, s.s1),
                   __builtin_amdgcn_perm(t4, t4, s.s2));
}

// acc ^ c * x in five VALU: three v_perm and two XOR (v_bitop3 for the three-input one: the
// backend does not form XOR3 from the plain expression)
__device__ __forceinline__ uint32_t perm_mul_acc(uint32_t acc, const Sel &s, uint32_t t0, uint32_t t1, uint32_t t2,
                                                 uint32_t t3, uint32_t t4) {
    const uint32_t a = __builtin_amdgcn_perm(t1, t0, s.s0);
    const uint32_t b = __builtin_amdgcn_perm(t3, t2, s.s1);
    const uint32_t c = __builtin_amdgcn_perm(t4, t4, s.s2);
    return gf_xor3(acc, a, b) ^ c;
}

// acc ^ c * x ^ d * y in nine VALU (six v_perm, three XOR3)
__device__ __forceinline__ uint32_t perm_mul2_acc(uint32_t acc, const Sel &sx, uint32_t c0, uint32_t c1, uint32_t c2,
                                                  uint32_t c3, uint32_t c4, const Sel &sy, uint32_t d0, uint32_t d1,
                                                  uint32_t d2, uint32_t d3, uint32_t d4) {
    const uint32_t a = __builtin_amdgcn_perm(c1, c0, sx.s0);
    const uint32_t b = __builtin_amdgcn_perm(c3, c2, sx.s1);
    const uint32_t c = __builtin_amdgcn_perm(c4, c4, sx.s2);
    const uint32_t d = __builtin_amdgcn_perm(d1, d0, sy.s0);
    const uint32_t e = __builtin_amdgcn_perm(d3, d2, sy.s1);
    const uint32_t f = __builtin_amdgcn_perm(d4, d4, sy.s2);
    return gf_xor3(gf_xor3(acc, a, b), gf_xor3(c, d, e), f);
}

// 2-bit fields of four packed bytes (PermTab4 tables)
struct Sel4 {
    uint32_t s0, s1, s2, s3;
    __device__ __forceinline__ Sel4() {}
    __device__ __forceinline__ explicit Sel4(uint32_t x)
        : s0(x & 0x03030303u), s1((x >> 2) & 0x03030303u), s2((x >> 4) & 0x03030303u), s3((x >> 6) & 0x03030303u) {}
};

// acc ^ c * x ^ d * y with 2-bit tables: eight v_perm (each reading one table dword twice, so the
// tables stay in SGPRs with no move) and four XOR3
__device__ __forceinline__ uint32_t perm4_mul2_acc(uint32_t acc, const Sel4 &x, uint32_t c0, uint32_t c1, uint32_t c2,
                                                   uint32_t c3, const Sel4 &y, uint32_t d0, uint32_t d1, uint32_t d2,
                                                   uint32_t d3) {
    const uint32_t a = __builtin_amdgcn_perm(c0, c0, x.s0), b = __builtin_amdgcn_perm(c1, c1, x.s1);
    const uint32_t c = __builtin_amdgcn_perm(c2, c2, x.s2), d = __builtin_amdgcn_perm(c3, c3, x.s3);
    const uint32_t e = __builtin_amdgcn_perm(d0, d0, y.s0), f = __builtin_amdgcn_perm(d1, d1, y.s1);
    const uint32_t g = __builtin_amdgcn_perm(d2, d2, y.s2), h = __builtin_amdgcn_perm(d3, d3, y.s3);
    return gf_xor3(gf_xor3(gf_xor3(acc, a, b), c, d), gf_xor3(e, f, g), h);
}
__device__ __forceinline__ uint32_t perm4_mul_acc(uint32_t acc, const Sel4 &x, uint32_t c0, uint32_t c1, uint32_t c2,
                                                  uint32_t c3) {
    const uint32_t a = __builtin_amdgcn_perm(c0, c0, x.s0), b = __builtin_amdgcn_perm(c1, c1, x.s1);
    const uint32_t c = __builtin_amdgcn_perm(c2, c2, x.s2), d = __builtin_amdgcn_perm(c3, c3, x.s3);
    return gf_xor3(gf_xor3(acc, a, b), c, d);
}

__device__ __forceinline__ uint32_t perm_mul(const Sel &s, const PermTab &t) {
    return perm_mul(s, t.t[0], t.t[1], t.t[2], t.t[3], t.t[4]);
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
