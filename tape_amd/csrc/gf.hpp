// gf.hpp -- GF(2^8) arithmetic and the Clay coefficient algebra, usable at compile time.
//
// Field: GF(2^8) with polynomial 0x11D and generator 2, the `galois_8` field of
// reed-solomon-erasure 6.0.0 (Cargo.lock:5374-5385), which clay-codes 0.1.1 builds its
// per-plane MDS code and pairwise transform on.
//
// Everything here is constexpr so the encode kernels can fold generator coefficients into
// straight-line XOR selections at compile time, and the host builds the same tables at run
// time for arbitrary erasure patterns.
#pragma once
#include <stdint.h>
#include <stddef.h>

namespace tec {

struct GfTables {
    uint8_t exp[512];
    uint8_t log[256];
};

constexpr GfTables make_gf_tables() {
    GfTables t{};
    unsigned x = 1;
    for (int i = 0; i < 255; i++) {
        t.exp[i] = (uint8_t)x;
        t.log[x] = (uint8_t)i;
        x <<= 1;
        if (x & 0x100) x ^= 0x11D;
    }
    for (int i = 255; i < 512; i++) t.exp[i] = t.exp[i - 255];
    t.log[0] = 0;
    return t;
}

inline constexpr GfTables kGf = make_gf_tables();

constexpr uint8_t gf_mul(uint8_t a, uint8_t b) {
    return (a == 0 || b == 0) ? 0 : kGf.exp[kGf.log[a] + kGf.log[b]];
}
constexpr uint8_t gf_inv(uint8_t a) { return kGf.exp[255 - kGf.log[a]]; }
// galois_8::exp(a, n) with 0^0 = 1
constexpr uint8_t gf_pow(uint8_t a, int n) {
    if (n == 0) return 1;
    if (a == 0) return 0;
    return kGf.exp[(kGf.log[a] * n) % 255];
}

constexpr int kMaxNodes = 32;  // internal Clay nodes (q*t) the engine supports

struct Mat {
    int rows = 0, cols = 0;
    uint8_t v[kMaxNodes][kMaxNodes] = {};
};

// Gauss-Jordan inverse over GF(2^8); returns false if singular.
constexpr bool mat_invert(Mat &m) {
    const int r = m.rows;
    uint8_t aug[kMaxNodes][2 * kMaxNodes] = {};
    for (int i = 0; i < r; i++)
        for (int j = 0; j < 2 * r; j++) aug[i][j] = j < r ? m.v[i][j] : (uint8_t)(j - r == i);
    for (int c = 0; c < r; c++) {
        int piv = -1;
        for (int i = c; i < r; i++)
            if (aug[i][c]) { piv = i; break; }
        if (piv < 0) return false;
        if (piv != c)
            for (int j = 0; j < 2 * r; j++) { uint8_t t = aug[c][j]; aug[c][j] = aug[piv][j]; aug[piv][j] = t; }
        const uint8_t iv = gf_inv(aug[c][c]);
        for (int j = 0; j < 2 * r; j++) aug[c][j] = gf_mul(aug[c][j], iv);
        for (int i = 0; i < r; i++) {
            if (i == c || aug[i][c] == 0) continue;
            const uint8_t f = aug[i][c];
            for (int j = 0; j < 2 * r; j++) aug[i][j] ^= gf_mul(f, aug[c][j]);
        }
    }
    for (int i = 0; i < r; i++)
        for (int j = 0; j < r; j++) m.v[i][j] = aug[i][r + j];
    return true;
}

// Systematic generator of reed-solomon-erasure `build_matrix(data, total)`:
// G = V * inv(V[0..data)), V[r][c] = r^c.  total x data.
constexpr Mat rs_generator(int data, int total) {
    Mat top{};
    top.rows = top.cols = data;
    for (int r = 0; r < data; r++)
        for (int c = 0; c < data; c++) top.v[r][c] = gf_pow((uint8_t)r, c);
    mat_invert(top);
    Mat g{};
    g.rows = total;
    g.cols = data;
    for (int r = 0; r < total; r++)
        for (int c = 0; c < data; c++) {
            uint8_t acc = 0;
            for (int j = 0; j < data; j++) acc ^= gf_mul(gf_pow((uint8_t)r, j), top.v[j][c]);
            g.v[r][c] = acc;
        }
    return g;
}

// Pairwise coupling transform (PFT): [C_hi, C_lo, U_hi, U_lo] is a codeword of the systematic
// RS(2,2) code (A3).  All four 2-term relations the layered code needs, as coefficient pairs:
//   U_self  = u_c * C_self + u_p * C_partner           (uncoupling; A4 orientation resolved)
//   C_self  = t_u * U_self + t_p * C_partner           (type-1 recovery)
//   C_self  = c_u * U_self + c_p * U_partner           (both erased)
// indexed by orientation o = 1 if self is the "hi" (larger x) member of the pair, else 0.
struct Pft {
    uint8_t u_c[2], u_p[2];
    uint8_t t_u[2], t_p[2];
    uint8_t c_u[2], c_p[2];
    // repair-specific: U_self from C_self and U_partner (partner aloof)
    uint8_t a_c[2], a_p[2];
    // repair: C_partner from C_self and U_self (partner = lost node)
    uint8_t l_c[2], l_u[2];
};

// Solve the [4,2] codeword: given values at positions a,b, coefficients producing position w.
constexpr void pft_coef(const Mat &g4, int a, int b, int w, uint8_t &ca, uint8_t &cb) {
    Mat s{};
    s.rows = s.cols = 2;
    s.v[0][0] = g4.v[a][0]; s.v[0][1] = g4.v[a][1];
    s.v[1][0] = g4.v[b][0]; s.v[1][1] = g4.v[b][1];
    mat_invert(s);
    ca = gf_mul(g4.v[w][0], s.v[0][0]) ^ gf_mul(g4.v[w][1], s.v[1][0]);
    cb = gf_mul(g4.v[w][0], s.v[0][1]) ^ gf_mul(g4.v[w][1], s.v[1][1]);
}

constexpr Pft make_pft() {
    const Mat g4 = rs_generator(2, 4);
    Pft p{};
    for (int o = 0; o < 2; o++) {
        // self = hi (o==1): self C at 0, partner C at 1, self U at 2, partner U at 3.
        // self = lo (o==0): Ceph swaps (0<->1, 2<->3): self C at 1, partner C at 0, ...
        const int sc = o ? 0 : 1, pc = o ? 1 : 0, su = o ? 2 : 3, pu = o ? 3 : 2;
        pft_coef(g4, sc, pc, su, p.u_c[o], p.u_p[o]);
        pft_coef(g4, su, pc, sc, p.t_u[o], p.t_p[o]);
        pft_coef(g4, su, pu, sc, p.c_u[o], p.c_p[o]);
        pft_coef(g4, sc, pu, su, p.a_c[o], p.a_p[o]);
        pft_coef(g4, sc, su, pc, p.l_c[o], p.l_u[o]);
    }
    return p;
}

inline constexpr Pft kPft = make_pft();

// v_perm tables for multiplication by a runtime constant, over the byte's bit fields [0,3),
// [3,6), [6,8): v_perm_b32 picks one of 8 bytes of a register pair per byte lane, so a 3-bit
// field is one perm.  t[0..1] = c*j for j < 8 (low dword j < 4), t[2..3] = c*(j << 3),
// t[4] = c*(j << 6) for j < 4.
struct PermTab {
    uint32_t t[5];
};
// 2-bit fields: t[f] byte j = c * (j << 2f), j < 4 -- one dword per field, so a v_perm selects
// from the same register twice (gfx9 reads one SGPR per VALU instruction: no v_mov needed)
struct PermTab4 {
    uint32_t t[4];
};

constexpr PermTab4 perm_tab4(uint8_t c) {
    PermTab4 r{};
    for (int f = 0; f < 4; f++)
        for (int j = 0; j < 4; j++) r.t[f] |= (uint32_t)gf_mul(c, (uint8_t)(j << (2 * f))) << (8 * j);
    return r;
}
constexpr PermTab perm_tab(uint8_t c) {
    PermTab r{};
    constexpr int sh[3] = {0, 3, 6}, n[3] = {8, 8, 4};
    int w = 0;
    for (int f = 0; f < 3; f++)
        for (int j0 = 0; j0 < n[f]; j0 += 4, w++)
            for (int j = 0; j < 4; j++) r.t[w] |= (uint32_t)gf_mul(c, (uint8_t)((j0 + j) << sh[f])) << (8 * j);
    return r;
}

}  // namespace tec
