// rs16.hpp -- GF(2^16) Reed-Solomon in the Leopard construction (the algorithm of
// reed-solomon-simd 3.1.0, behind lib/slicer/src/outer.rs OuterCoder and
// lib/slicer/src/reed_solomon.rs ReedSolomonCoder): host-side tables and the
// per-column transform the GPU kernels (rs16.hip) run, used on the host only to derive the
// decoding matrix (a setup step per erasure pattern, like the Clay D tables).
//
//   * field GF(2^16), LFSR polynomial 0x1002D, logarithms in the Cantor basis (LCH);
//   * skew factors of the basis drive the additive FFT (Lin-Chung-Han, FOCS 2014);
//   * high rate (next_pow2(m) <= next_pow2(k)): IFFT each chunk of c = next_pow2(m) originals at
//     skew offset pos + c, XOR-fold, one FFT at offset 0; low rate: one IFFT of the originals
//     (c = next_pow2(k), offset 0), one FFT per chunk of c recovery shards at offset pos + c.
#pragma once
#include <stdint.h>
#include <string.h>
#include <vector>

namespace tec {
namespace rs16 {

constexpr int kBits = 16;
constexpr uint32_t kOrder = 65536, kModulus = 65535, kPoly = 0x1002D;

struct Tables {
    std::vector<uint16_t> exp, log, skew;
    Tables() : exp(kOrder), log(kOrder), skew(kModulus) {
        static const uint16_t cantor[kBits] = {0x0001, 0xACCA, 0x3C0E, 0x163E, 0xC582, 0xED2E, 0x914C, 0x4012,
                                               0x6C98, 0x10D8, 0x6A72, 0xB900, 0xFDB8, 0xFB34, 0xFF38, 0x991E};
        uint32_t st = 1;
        for (uint32_t i = 0; i < kModulus; i++) {
            exp[st] = (uint16_t)i;
            st <<= 1;
            if (st >= kOrder) st ^= kPoly;
        }
        exp[0] = kModulus;
        log[0] = 0;
        for (int i = 0; i < kBits; i++)
            for (uint32_t j = 0, w = 1u << i; j < w; j++) log[j + w] = log[j] ^ cantor[i];
        for (uint32_t i = 0; i < kOrder; i++) log[i] = exp[log[i]];
        for (uint32_t i = 0; i < kOrder; i++) exp[log[i]] = (uint16_t)i;
        exp[kModulus] = exp[0];
        uint16_t t[kBits - 1];
        for (int i = 1; i < kBits; i++) t[i - 1] = (uint16_t)(1u << i);
        for (int m = 0; m < kBits - 1; m++) {
            skew[(1u << m) - 1] = 0;
            for (int i = m; i < kBits - 1; i++) {
                const uint32_t s = 1u << (i + 1);
                for (uint32_t j = (1u << m) - 1; j < s; j += 1u << (m + 1)) skew[j + s] = skew[j] ^ t[i];
            }
            t[m] = (uint16_t)(kModulus - log[mul(t[m], log[t[m] ^ 1])]);
            for (int i = m + 1; i < kBits - 1; i++) t[i] = mul(t[i], add(log[t[i] ^ 1], t[m]));
        }
        for (uint32_t i = 0; i < kModulus; i++) skew[i] = log[skew[i]];
    }
    static uint16_t add(uint16_t x, uint16_t y) {  // x + y mod 65535 (65535 == 0)
        const uint32_t s = (uint32_t)x + y;
        return (uint16_t)(s + (s >> kBits));
    }
    uint16_t mul(uint16_t x, uint16_t log_m) const { return x ? exp[add(log[x], log_m)] : 0; }
    uint16_t gmul(uint16_t a, uint16_t b) const { return (a && b) ? exp[add(log[a], log[b])] : 0; }
    uint16_t inv(uint16_t a) const { return exp[(kModulus - log[a]) % kModulus]; }
};

inline const Tables &tables() {
    static const Tables t;
    return t;
}

inline uint32_t next_pow2(uint32_t x) {
    uint32_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

// rate::use_high_rate: 1 high, 0 low, -1 unsupported shard counts
inline int use_high_rate(uint32_t k, uint32_t m) {
    if (k == 0 || m == 0 || k > kOrder || m > kOrder) return -1;
    const uint32_t kp = next_pow2(k), mp = next_pow2(m);
    if ((uint64_t)(kp < mp ? kp : mp) + (k > m ? k : m) > kOrder) return -1;
    return mp <= kp ? 1 : 0;
}

// the transform size c and the column's work length
inline uint32_t chunk(uint32_t k, uint32_t m) { return use_high_rate(k, m) ? next_pow2(m) : next_pow2(k); }
inline uint32_t work_len(uint32_t k, uint32_t m) {
    const uint32_t c = chunk(k, m);
    return use_high_rate(k, m) ? 2 * c : ((m + c - 1) / c) * c;
}
// one past the largest skew index the transforms of a (k, m) encode touch
inline uint32_t skew_span(uint32_t k, uint32_t m) {
    const uint32_t c = chunk(k, m);
    const uint32_t top = use_high_rate(k, m) ? ((k + c - 1) / c) * c : ((m + c - 1) / c) * c;
    return top + 2 * c + 1;
}

// ---- one column on the host (decode setup) ----
inline void fft(const Tables &T, uint16_t *w, uint32_t size, uint32_t trunc, uint32_t delta) {
    auto b2 = [&](uint16_t &x, uint16_t &y, uint16_t lm) {
        if (lm != kModulus) x ^= T.mul(y, lm);
        y ^= x;
    };
    uint32_t dist4 = size, dist = size >> 2;
    for (; dist; dist4 = dist, dist >>= 2)
        for (uint32_t r = 0; r < trunc; r += dist4) {
            const uint32_t b = r + dist + delta - 1;
            const uint16_t m01 = T.skew[b], m02 = T.skew[b + dist], m23 = T.skew[b + 2 * dist];
            for (uint32_t i = r; i < r + dist; i++) {
                b2(w[i], w[i + 2 * dist], m02);
                b2(w[i + dist], w[i + 3 * dist], m02);
                b2(w[i], w[i + dist], m01);
                b2(w[i + 2 * dist], w[i + 3 * dist], m23);
            }
        }
    if (dist4 == 2)
        for (uint32_t r = 0; r < trunc; r += 2) b2(w[r], w[r + 1], T.skew[r + delta]);
}
inline void ifft(const Tables &T, uint16_t *w, uint32_t size, uint32_t trunc, uint32_t delta) {
    auto b2 = [&](uint16_t &x, uint16_t &y, uint16_t lm) {
        y ^= x;
        if (lm != kModulus) x ^= T.mul(y, lm);
    };
    uint32_t dist = 1, dist4 = 4;
    for (; dist4 <= size; dist = dist4, dist4 <<= 2)
        for (uint32_t r = 0; r < trunc; r += dist4) {
            const uint32_t b = r + dist + delta - 1;
            const uint16_t m01 = T.skew[b], m02 = T.skew[b + dist], m23 = T.skew[b + 2 * dist];
            for (uint32_t i = r; i < r + dist; i++) {
                b2(w[i], w[i + dist], m01);
                b2(w[i + 2 * dist], w[i + 3 * dist], m23);
                b2(w[i], w[i + 2 * dist], m02);
                b2(w[i + dist], w[i + 3 * dist], m02);
            }
        }
    if (dist < size) {
        const uint16_t lm = T.skew[dist + delta - 1];
        for (uint32_t i = 0; i < dist; i++) b2(w[i], w[i + dist], lm);
    }
}

// recovery values of one column (k originals -> m recovery)
inline void encode_column(uint32_t k, uint32_t m, const uint16_t *orig, uint16_t *rec) {
    const Tables &T = tables();
    const uint32_t c = chunk(k, m);
    std::vector<uint16_t> w(work_len(k, m), 0);
    if (use_high_rate(k, m)) {
        for (uint32_t s = 0; s < k; s += c) {
            uint16_t *t = w.data() + (s ? c : 0);
            memset(t, 0, c * sizeof(uint16_t));
            const uint32_t n = k - s < c ? k - s : c;
            memcpy(t, orig + s, n * sizeof(uint16_t));
            ifft(T, t, c, n, s + c);
            if (s)
                for (uint32_t i = 0; i < c; i++) w[i] ^= t[i];
        }
        fft(T, w.data(), c, m, 0);
    } else {
        memcpy(w.data(), orig, k * sizeof(uint16_t));
        ifft(T, w.data(), c, k, 0);
        for (uint32_t s = c; s < m; s += c) memcpy(w.data() + s, w.data(), c * sizeof(uint16_t));
        for (uint32_t s = 0; s < m; s += c) fft(T, w.data() + s, c, m - s < c ? m - s : c, s + c);
    }
    memcpy(rec, w.data(), m * sizeof(uint16_t));
}

// Decoding matrix for a set of received shards: rows[i] (original i = 0..k-1 restored from the
// k received shard ids `recv`, originals 0..k-1, recovery k..k+m-1).  out[i*k + r] multiplies
// received shard r.  false if the received rows are singular (never for an MDS code).
inline bool decode_matrix(uint32_t k, uint32_t m, const std::vector<uint32_t> &recv, std::vector<uint16_t> &out) {
    const Tables &T = tables();
    std::vector<uint16_t> G((size_t)(k + m) * k, 0), o(k), r(m);
    for (uint32_t i = 0; i < k; i++) G[(size_t)i * k + i] = 1;
    for (uint32_t c = 0; c < k; c++) {
        std::fill(o.begin(), o.end(), 0);
        o[c] = 1;
        encode_column(k, m, o.data(), r.data());
        for (uint32_t j = 0; j < m; j++) G[(size_t)(k + j) * k + c] = r[j];
    }
    std::vector<uint16_t> A((size_t)k * 2 * k, 0);
    for (uint32_t i = 0; i < k; i++)
        for (uint32_t c = 0; c < 2 * k; c++)
            A[(size_t)i * 2 * k + c] = c < k ? G[(size_t)recv[i] * k + c] : (uint16_t)(c - k == i);
    for (uint32_t c = 0; c < k; c++) {
        uint32_t p = c;
        while (p < k && !A[(size_t)p * 2 * k + c]) p++;
        if (p == k) return false;
        if (p != c)
            for (uint32_t j = 0; j < 2 * k; j++) std::swap(A[(size_t)c * 2 * k + j], A[(size_t)p * 2 * k + j]);
        const uint16_t iv = T.inv(A[(size_t)c * 2 * k + c]);
        for (uint32_t j = 0; j < 2 * k; j++) A[(size_t)c * 2 * k + j] = T.gmul(A[(size_t)c * 2 * k + j], iv);
        for (uint32_t i = 0; i < k; i++) {
            const uint16_t f = A[(size_t)i * 2 * k + c];
            if (i == c || !f) continue;
            for (uint32_t j = 0; j < 2 * k; j++) A[(size_t)i * 2 * k + j] ^= T.gmul(f, A[(size_t)c * 2 * k + j]);
        }
    }
    out.assign((size_t)k * k, 0);
    for (uint32_t i = 0; i < k; i++)
        for (uint32_t j = 0; j < k; j++) out[(size_t)i * k + j] = A[(size_t)i * 2 * k + k + j];
    return true;
}

// The encode as a matrix: recovery j = sum_i E[j*k + i] * original i.  The transforms are linear
// over GF(2^16) (every step is x ^= y * const), so column i is the encode of the unit vector e_i.
inline void encode_matrix(uint32_t k, uint32_t m, std::vector<uint16_t> &E) {
    std::vector<uint16_t> o(k), r(m);
    E.assign((size_t)m * k, 0);
    for (uint32_t i = 0; i < k; i++) {
        std::fill(o.begin(), o.end(), 0);
        o[i] = 1;
        encode_column(k, m, o.data(), r.data());
        for (uint32_t j = 0; j < m; j++) E[(size_t)j * k + i] = r[j];
    }
}

// Lookup image of a rows x k matrix M for rs16_matrix_kernel (kernels.hpp Rs16MatArgs), G = the
// 4-row groups: per input r and nibble position q a block of G x 64 u16 holding, for n < 16, the
// products M[row][r] * (n << 4q) -- groups 2h and 2h + 1 (8 rows) as 16 entries of 8 u16 at h * 128
// + n * 8, and for odd G the last group as 16 entries of 4 u16 at (G / 2) * 128 + n * 4.  Zero past
// the last row.
// tv (rows = 8 h + 1, kernels.hpp rs16_mat_tailv): the last row is not in the blocks (h x 128
// u16 per (r, q)); after them, per input r 16 u32 constants K[r][b] = M[rows - 1][r] * (1 << b),
// the product in both halves (the product is linear over GF(2): x * c = XOR of K[b] over the set
// bits b of x; the kernel applies it to two elements at once).
// tail_bytes (kernels.hpp rs16_mat_tail_bytes, odd G only): the last group's entry size, 2 / 4 / 8 B
// for 1 / 2 / 3-4 rows (16 entries of tail_bytes at (G / 2) * 128 u16); the block of (r, q) is
// (G / 2) * 128 + 8 * tail_bytes u16.
inline std::vector<uint16_t> mat_image(uint32_t k, uint32_t rows, const uint16_t *M, bool tv = false,
                                       uint32_t tail_bytes = 8) {
    const Tables &T = tables();
    tv = tv && rows % 8 == 1 && rows > 1;
    const uint32_t G = (rows + 3) / 4, NP = G / 2;
    const uint32_t TBu = (G % 2 && !tv) ? tail_bytes / 2 : 0;  // u16 per tail entry
    const uint32_t BQ = NP * 128 + 16 * TBu;                   // u16 per (r, q) block
    std::vector<uint16_t> img((size_t)k * 4 * BQ + (tv ? (size_t)k * 32 : 0), 0);
    if (tv) {
        uint16_t *kt = img.data() + (size_t)k * 4 * BQ;
        for (uint32_t r = 0; r < k; r++)
            for (uint32_t b = 0; b < 16; b++)
                kt[((size_t)r * 16 + b) * 2] = kt[((size_t)r * 16 + b) * 2 + 1] =
                    T.gmul((uint16_t)(1u << b), M[(size_t)(rows - 1) * k + r]);
    }
    for (uint32_t r = 0; r < k; r++)
        for (uint32_t q = 0; q < 4; q++) {
            uint16_t *blk = img.data() + ((size_t)r * 4 + q) * BQ;
            for (uint32_t row = 0; row < (tv ? rows - 1 : rows); row++) {
                const uint32_t g = row / 4, j = row % 4;
                const uint16_t c = M[(size_t)row * k + r];
                for (uint32_t n = 0; n < 16; n++) {
                    const size_t at = g < 2 * NP ? (g / 2) * 128 + n * 8 + (g % 2) * 4 + j : NP * 128 + n * TBu + j;
                    blk[at] = T.gmul((uint16_t)(n << (4 * q)), c);
                }
            }
        }
    return img;
}

}  // namespace rs16
}  // namespace tec
