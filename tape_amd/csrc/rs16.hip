// rs16.hip -- GF(2^16) Reed-Solomon (Leopard construction, the algorithm of reed-solomon-simd
// 3.1.0) on the device: OuterCoder encode / decode (lib/slicer/src/outer.rs:70-197).
//
// Shard layout (the crate's): every 64-byte block holds 32 field elements, element i = byte i |
// byte 32 + i << 8.  A thread owns one element column -- the same element of every shard -- and
// runs the whole transform of rs16.hpp on it: its work vector lives in LDS (work[i] at
// i * blockDim + tid), the butterflies' multipliers are the skew factors of the LCH basis, and a
// product x * exp(log_m) is four 16-entry nibble tables per multiplier, staged in LDS
// (x = n0 | n1 << 4 | n2 << 8 | n3 << 12 -> T[n0] ^ T[16 + n1] ^ T[32 + n2] ^ T[48 + n3]; the table
// of log_m = 65535, the basis' "zero", is all zeros, which makes the butterfly a plain XOR).
// Decode applies the host-derived k x k decoding matrix the same way, one table per coefficient.
// A first kernel: correct for every shard count the crate supports within the LDS budget.
#include <algorithm>
#include "kernels.hpp"

namespace tec {
namespace rs16k {

constexpr uint32_t kRs16DecLds = 48 * 1024;  // decoding tables staged in LDS up to this size
#ifndef TEC_RS16_REG
#define TEC_RS16_REG 1  // low rate, chunk <= 32: rs16_encode_low_kernel (work vector in VGPRs)
#endif
#ifndef TEC_RS16_UNROLL
#define TEC_RS16_UNROLL 1  // butterfly groups in flight per thread in the transforms' inner loops
#endif

__device__ __forceinline__ uint32_t mulx(uint32_t x, const uint16_t *T) {
    return T[x & 15u] ^ T[16u + ((x >> 4) & 15u)] ^ T[32u + ((x >> 8) & 15u)] ^ T[48u + (x >> 12)];
}

struct Col {  // one thread's work vector in LDS
    uint16_t *w;
    uint32_t bt;
    __device__ uint32_t ld(uint32_t i) const { return w[i * bt]; }
    __device__ void st(uint32_t i, uint32_t v) const { w[i * bt] = (uint16_t)v; }
};

// FFT / IFFT of work[pos .. pos + size) (rs16.hpp restated on LDS columns).  A radix-4 group's
// four values stay in registers across its four butterflies (4 LDS loads + 4 stores per group
// instead of 8 + 8).
__device__ void fft(const Col &c, const uint16_t *lut, uint32_t pos, uint32_t size, uint32_t trunc, uint32_t delta) {
    uint32_t dist4 = size, dist = size >> 2;
    for (; dist; dist4 = dist, dist >>= 2)
        for (uint32_t r = 0; r < trunc; r += dist4) {
            const uint32_t b = r + dist + delta - 1;
            const uint16_t *t0 = lut + b * 64u, *t1 = lut + (b + dist) * 64u, *t2 = lut + (b + 2 * dist) * 64u;
#pragma unroll TEC_RS16_UNROLL
            for (uint32_t i = r; i < r + dist; i++) {
                const uint32_t p = pos + i;
                uint32_t x0 = c.ld(p), x1 = c.ld(p + dist), x2 = c.ld(p + 2 * dist), x3 = c.ld(p + 3 * dist);
                x0 ^= mulx(x2, t1);  // (i, i + 2 dist)
                x2 ^= x0;
                x1 ^= mulx(x3, t1);  // (i + dist, i + 3 dist)
                x3 ^= x1;
                x0 ^= mulx(x1, t0);  // (i, i + dist)
                x1 ^= x0;
                x2 ^= mulx(x3, t2);  // (i + 2 dist, i + 3 dist)
                x3 ^= x2;
                c.st(p, x0);
                c.st(p + dist, x1);
                c.st(p + 2 * dist, x2);
                c.st(p + 3 * dist, x3);
            }
        }
    if (dist4 == 2)
        for (uint32_t r = 0; r < trunc; r += 2) {
            uint32_t x = c.ld(pos + r), y = c.ld(pos + r + 1);
            x ^= mulx(y, lut + (r + delta) * 64u);
            y ^= x;
            c.st(pos + r, x);
            c.st(pos + r + 1, y);
        }
}

__device__ void ifft(const Col &c, const uint16_t *lut, uint32_t pos, uint32_t size, uint32_t trunc, uint32_t delta) {
    uint32_t dist = 1, dist4 = 4;
    for (; dist4 <= size; dist = dist4, dist4 <<= 2)
        for (uint32_t r = 0; r < trunc; r += dist4) {
            const uint32_t b = r + dist + delta - 1;
            const uint16_t *t0 = lut + b * 64u, *t1 = lut + (b + dist) * 64u, *t2 = lut + (b + 2 * dist) * 64u;
#pragma unroll TEC_RS16_UNROLL
            for (uint32_t i = r; i < r + dist; i++) {
                const uint32_t p = pos + i;
                uint32_t x0 = c.ld(p), x1 = c.ld(p + dist), x2 = c.ld(p + 2 * dist), x3 = c.ld(p + 3 * dist);
                x1 ^= x0;  // (i, i + dist)
                x0 ^= mulx(x1, t0);
                x3 ^= x2;  // (i + 2 dist, i + 3 dist)
                x2 ^= mulx(x3, t2);
                x2 ^= x0;  // (i, i + 2 dist)
                x0 ^= mulx(x2, t1);
                x3 ^= x1;  // (i + dist, i + 3 dist)
                x1 ^= mulx(x3, t1);
                c.st(p, x0);
                c.st(p + dist, x1);
                c.st(p + 2 * dist, x2);
                c.st(p + 3 * dist, x3);
            }
        }
    if (dist < size)
        for (uint32_t i = 0; i < dist; i++) {
            uint32_t x = c.ld(i + pos), y = c.ld(i + dist + pos);
            y ^= x;
            x ^= mulx(y, lut + (dist + delta - 1) * 64u);
            c.st(i + pos, x);
            c.st(i + dist + pos, y);
        }
}

__device__ __forceinline__ uint32_t ld_elem(const uint8_t *shard, uint32_t e) {
    const uint32_t o = (e >> 5) * 64u + (e & 31u);
    return (uint32_t)shard[o] | ((uint32_t)shard[o + 32u] << 8);
}
__device__ __forceinline__ void st_elem(uint8_t *shard, uint32_t e, uint32_t v) {
    const uint32_t o = (e >> 5) * 64u + (e & 31u);
    shard[o] = (uint8_t)v;
    shard[o + 32u] = (uint8_t)(v >> 8);
}

#ifndef TEC_RS16_WPE
#define TEC_RS16_WPE 6  // waves per SIMD the encode is compiled for: 6 -> 3.94 ms, 5 -> 4.75, 8 (spills) -> 4.19
#endif
__global__ void __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(TEC_RS16_WPE))) rs16_encode_kernel(Rs16EncArgs a) {  // grid.y = segments
    extern __shared__ __attribute__((aligned(16))) uint16_t lds16[];
    uint16_t *lut = lds16;                     // span x 64 entries
    uint16_t *work = lds16 + a.span * 64u;     // work_len x blockDim
    for (uint32_t t = threadIdx.x; t < a.span * 32u; t += blockDim.x)
        reinterpret_cast<uint32_t *>(lut)[t] = reinterpret_cast<const uint32_t *>(a.lut)[t];
    __syncthreads();
    const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= a.elems) return;  // no barrier below
    a.in += (uint64_t)blockIdx.y * a.seg_in;
    a.out += (uint64_t)blockIdx.y * a.seg_out;
    const Col c{work + threadIdx.x, blockDim.x};
    const uint32_t k = a.k, m = a.m, cs = a.c;
    for (uint32_t i = 0; i < (a.one_chunk ? cs : a.work_len); i++) c.st(i, 0);
    if (a.high) {
        // chunks of c originals: the first at work[0..c), each further one at work[c..2c),
        // transformed at its own skew offset and XOR-folded into the first
        for (uint32_t s = 0; s < k; s += cs) {
            const uint32_t pos = s ? cs : 0u, n = k - s < cs ? k - s : cs;
            for (uint32_t j = 0; j < cs; j++)
                c.st(pos + j, j < n ? ld_elem(a.in + (uint64_t)(s + j) * a.in_stride, e) : 0u);
            ifft(c, lut, pos, cs, n, s + cs);
            if (s)
                for (uint32_t j = 0; j < cs; j++) c.st(j, c.ld(j) ^ c.ld(cs + j));
        }
        fft(c, lut, 0, cs, m, 0);
    } else if (a.one_chunk) {
        // low rate, chunk <= 32: one chunk of work in LDS; the IFFT result is kept in registers
        // (two elements per VGPR) and restored before each chunk's FFT, which is then written out
        for (uint32_t j = 0; j < k; j++) c.st(j, ld_elem(a.in + (uint64_t)j * a.in_stride, e));
        ifft(c, lut, 0, cs, k, 0);
        uint32_t keep[16];
#pragma unroll
        for (uint32_t q = 0; q < 16u; q++) keep[q] = 2 * q < cs ? c.ld(2 * q) | c.ld(2 * q + 1) << 16 : 0u;
        for (uint32_t s = 0; s < m; s += cs) {
            if (s) {
#pragma unroll
                for (uint32_t q = 0; q < 16u; q++)
                    if (2 * q < cs) {
                        c.st(2 * q, keep[q] & 0xffffu);
                        c.st(2 * q + 1, keep[q] >> 16);
                    }
            }
            const uint32_t n = m - s < cs ? m - s : cs;
            fft(c, lut, 0, cs, n, s + cs);
            for (uint32_t j = 0; j < n; j++) st_elem(a.out + (uint64_t)(s + j) * a.out_stride, e, c.ld(j));
        }
        return;
    } else {
        for (uint32_t j = 0; j < k; j++) c.st(j, ld_elem(a.in + (uint64_t)j * a.in_stride, e));
        ifft(c, lut, 0, cs, k, 0);
        for (uint32_t s = cs; s < m; s += cs)
            for (uint32_t j = 0; j < cs; j++) c.st(s + j, c.ld(j));
        for (uint32_t s = 0; s < m; s += cs) fft(c, lut, s, cs, m - s < cs ? m - s : cs, s + cs);
    }
    for (uint32_t j = 0; j < m; j++) st_elem(a.out + (uint64_t)j * a.out_stride, e, c.ld(j));
}

// ---- low rate, chunk C <= 32: the work vector in registers ----
// The kernel above keeps a thread's work vector in LDS, so every butterfly group adds 4 loads and 4
// stores to the 4 table lookups of each product: 6 LDS accesses per product on a kernel whose
// bound is the LDS pipe (r04/r05: OuterCoder(17, 50) at 3.94 ms, 0.107 of HBM).  With C fixed at
// compile time the transforms unroll completely, every work index is a constant and the vector
// lives in VGPRs (C values + C kept IFFT values); a product is then its 4 conflict-free lookups
// (one multiplier's 16-entry nibble table is 8 dwords in 8 banks).  The truncation tests (r <
// trunc) and the chunk offsets are uniform branches on kernel arguments.
// Tables are addressed by LDS byte offset (uint32_t) rather than through the extern array, so a
// lookup is a bit-field extract plus one shift-add of the multiplier's (uniform) table offset.
typedef __attribute__((address_space(3))) const uint16_t lds_u16;
__device__ __forceinline__ uint32_t lds_ld16(uint32_t a) { return *reinterpret_cast<lds_u16 *>((size_t)a); }
// v_bfe_u32 by hand: the compiler rewrites a field extract followed by << 1 as a shift and a mask
// (3 VALU per lookup with the add); extract + v_lshl_add_u32 is 2
__device__ __forceinline__ uint32_t nib(uint32_t x, int q) {
    uint32_t n;
    asm("v_bfe_u32 %0, %1, %2, 4" : "=v"(n) : "v"(x), "i"(4 * q));
    return n;
}
__device__ __forceinline__ uint32_t mulx_a(uint32_t x, uint32_t tb) {  // tb: the table's byte offset
    const uint32_t t0 = lds_ld16((nib(x, 0) << 1) + tb);
    const uint32_t t1 = lds_ld16((nib(x, 1) << 1) + (tb + 32u));
    const uint32_t t2 = lds_ld16((nib(x, 2) << 1) + (tb + 64u));
    const uint32_t t3 = lds_ld16((nib(x, 3) << 1) + (tb + 96u));
    return t0 ^ t1 ^ t2 ^ t3;
}

template <int DIST, int DIST4, int C>
__device__ __forceinline__ void ifft_layer_r(uint32_t (&w)[C], uint32_t lut, uint32_t trunc, uint32_t delta) {
#pragma unroll
    for (int r = 0; r < C; r += DIST4) {
        if ((uint32_t)r >= trunc) continue;  // (not break: a run-time exit leaves the loop rolled)
        const uint32_t b = r + DIST + delta - 1;
        const uint32_t t0 = lut + b * 128u, t1 = t0 + DIST * 128u, t2 = t0 + 2 * DIST * 128u;
#pragma unroll
        for (int i = r; i < r + DIST; i++) {
            uint32_t &x0 = w[i], &x1 = w[i + DIST], &x2 = w[i + 2 * DIST], &x3 = w[i + 3 * DIST];
            x1 ^= x0;
            x0 ^= mulx_a(x1, t0);
            x3 ^= x2;
            x2 ^= mulx_a(x3, t2);
            x2 ^= x0;
            x0 ^= mulx_a(x2, t1);
            x3 ^= x1;
            x1 ^= mulx_a(x3, t1);
        }
    }
}
template <int DIST, int C>
__device__ __forceinline__ void ifft_r(uint32_t (&w)[C], uint32_t lut, uint32_t trunc, uint32_t delta) {
    if constexpr (DIST * 4 <= C) {
        ifft_layer_r<DIST, DIST * 4, C>(w, lut, trunc, delta);
        ifft_r<DIST * 4, C>(w, lut, trunc, delta);
    } else if constexpr (DIST < C) {
        const uint32_t t = lut + (DIST + delta - 1) * 128u;
#pragma unroll
        for (int i = 0; i < DIST; i++) {
            w[i + DIST] ^= w[i];
            w[i] ^= mulx_a(w[i + DIST], t);
        }
    }
}
template <int DIST4, int C>
__device__ __forceinline__ void fft_r(uint32_t (&w)[C], uint32_t lut, uint32_t trunc, uint32_t delta) {
    constexpr int DIST = DIST4 / 4;
    if constexpr (DIST >= 1) {
#pragma unroll
        for (int r = 0; r < C; r += DIST4) {
            if ((uint32_t)r >= trunc) continue;
            const uint32_t b = r + DIST + delta - 1;
            const uint32_t t0 = lut + b * 128u, t1 = t0 + DIST * 128u, t2 = t0 + 2 * DIST * 128u;
#pragma unroll
            for (int i = r; i < r + DIST; i++) {
                uint32_t &x0 = w[i], &x1 = w[i + DIST], &x2 = w[i + 2 * DIST], &x3 = w[i + 3 * DIST];
                x0 ^= mulx_a(x2, t1);
                x2 ^= x0;
                x1 ^= mulx_a(x3, t1);
                x3 ^= x1;
                x0 ^= mulx_a(x1, t0);
                x1 ^= x0;
                x2 ^= mulx_a(x3, t2);
                x3 ^= x2;
            }
        }
        fft_r<DIST, C>(w, lut, trunc, delta);
    } else if constexpr (DIST4 == 2) {
#pragma unroll
        for (int r = 0; r < C; r += 2) {
            if ((uint32_t)r >= trunc) continue;
            w[r] ^= mulx_a(w[r + 1], lut + (r + delta) * 128u);
            w[r + 1] ^= w[r];
        }
    }
}

#ifndef TEC_RS16_LOW_WPE
#define TEC_RS16_LOW_WPE 4
#endif
template <int C>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(TEC_RS16_LOW_WPE)))
rs16_encode_low_kernel(Rs16EncArgs a) {  // grid.y = segments
    extern __shared__ __attribute__((aligned(16))) uint16_t lds16[];
    for (uint32_t t = threadIdx.x; t < a.span * 32u; t += blockDim.x)
        reinterpret_cast<uint32_t *>(lds16)[t] = reinterpret_cast<const uint32_t *>(a.lut)[t];
    __syncthreads();
    const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= a.elems) return;  // no barrier below
    const uint32_t lut = (uint32_t)(size_t)(lds_u16 *)lds16;
    const uint8_t *in = a.in + (uint64_t)blockIdx.y * a.seg_in;
    uint8_t *out = a.out + (uint64_t)blockIdx.y * a.seg_out;
    const uint32_t k = a.k, m = a.m;
    uint32_t w[C], keep[C];
    // every load issued before the first use: the shards past k re-read shard k - 1 (same lines,
    // cache hits) and are zeroed after, instead of a branch and a wait per shard
#pragma unroll
    for (int j = 0; j < C; j++) w[j] = ld_elem(in + (uint64_t)((uint32_t)j < k ? (uint32_t)j : k - 1u) * a.in_stride, e);
#pragma unroll
    for (int j = 0; j < C; j++) w[j] = (uint32_t)j < k ? w[j] : 0u;
    ifft_r<1, C>(w, lut, k, 0);
#pragma unroll
    for (int j = 0; j < C; j++) keep[j] = w[j];
#pragma unroll 1
    for (uint32_t s = 0; s < m; s += C) {
        if (s) {
#pragma unroll
            for (int j = 0; j < C; j++) w[j] = keep[j];
        }
        const uint32_t n = m - s < (uint32_t)C ? m - s : (uint32_t)C;
        fft_r<C, C>(w, lut, n, s + C);
#pragma unroll
        for (int j = 0; j < C; j++)
            if ((uint32_t)j < n) st_elem(out + (uint64_t)(s + j) * a.out_stride, e, w[j]);
    }
}

// ---- matrix apply: out[i] = sum_r M[i][r] * in[r] (encode: M = the encode matrix; decode: the
// decoding matrix's missing rows) ----
// The FFT encode's products each have their own multiplier and input, so each costs 4 ds_read_u16
// (2 LDS cycles each) and ~14 VALU.  As a matrix the products of one input share their nibble
// indices across every output row: the image packs 4 rows' table entries into 8 bytes, so one
// ds_read_b64 (2 cycles, conflict-free: a 16-entry x 8 B table is 32 dwords in distinct banks)
// serves 4 products, and the nibble extraction is paid once per input instead of once per
// product.  OuterCoder(17, 50): 17 x 36 products per column (vs ~190 in the transforms) at 0.5
// LDS cycles and ~1.3 VALU each.  A thread owns two adjacent elements (their low bytes adjacent:
// 16-bit loads and stores); the image is staged once per block and the blocks loop over the
// (segment, column-tile) space.
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) const u32x2 lds_u32x2;
typedef __attribute__((address_space(3))) const u32x4 lds_u32x4;

// One input's products: the image block of (r, q) holds G / 2 pairs of row groups as 16-entry
// tables of 16 B (8 rows per ds_read_b128: 4 LDS cycles, conflict-free -- 16 distinct entries
// fill the 64 banks once) and, for odd G, the last group as a 16-entry table of 8 B
// (ds_read_b64).  Not 8-byte reads throughout: the compiler pairs those into ds_read2_b64, which
// costs 8 cycles for the two instead of 4.  The four nibble tables' entries of a group are XORed
// together before the accumulator (bitop3: 2 VALU per dword).
// three-input XOR (v_bitop3_b32 0x96): the compiler leaves XOR chains as 2-input v_xor_b32
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t d;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}

// One input's products for the thread's E elements (element e's 16 bits at bit sh + 16 e of w).
// TV: no tail group in the image (rows = 8 NP + 1; mat_tail computes the last row).  TB: the tail
// group's entry bytes (kernels.hpp rs16_mat_tail_bytes): 2 = one row (ds_read_u16, 1 LDS cycle
// instead of the 8-byte read's 2), 4 = two rows (ds_read_b32), 8 = three or four.
typedef __attribute__((address_space(3))) const uint16_t lds_u16;
typedef __attribute__((address_space(3))) const uint32_t lds_u32;
template <int G, int TB, bool TV>
constexpr int mat_block_bytes() { return (G / 2) * 256 + ((G % 2 && !TV) ? 16 * TB : 0); }
template <int G, int E, bool TV, int TB>
__device__ __forceinline__ void mat_input(uint32_t (&acc)[E][2 * G], const uint8_t *blk, uint32_t w, int sh) {
    constexpr int NP = G / 2, BQ = mat_block_bytes<G, TB, TV>();  // BQ: bytes per (r, q) block
    uint32_t n[E][4];
#pragma unroll
    for (int e = 0; e < E; e++)
#pragma unroll
        for (int q = 0; q < 4; q++) n[e][q] = nib(w, (sh + 16 * e) / 4 + q);
#pragma unroll
    for (int h = 0; h < NP; h++) {
        u32x4 v[E][4];
#pragma unroll
        for (int e = 0; e < E; e++)
#pragma unroll
            for (int q = 0; q < 4; q++) v[e][q] = *(lds_u32x4 *)(blk + (n[e][q] << 4) + (q * BQ + h * 256));
#pragma unroll
        for (int e = 0; e < E; e++)
#pragma unroll
            for (int d = 0; d < 4; d++)
                acc[e][4 * h + d] = xor3(xor3(acc[e][4 * h + d], v[e][0][d], v[e][1][d]), v[e][2][d], v[e][3][d]);
    }
    if constexpr (G % 2 && !TV && TB == 8) {  // tail group: entries of 8 B at NP * 256 within each nibble block
        u32x2 v[E][4];
#pragma unroll
        for (int e = 0; e < E; e++)
#pragma unroll
            for (int q = 0; q < 4; q++) v[e][q] = *(lds_u32x2 *)(blk + (n[e][q] << 3) + (q * BQ + NP * 256));
#pragma unroll
        for (int e = 0; e < E; e++)
#pragma unroll
            for (int d = 0; d < 2; d++)
                acc[e][4 * NP + d] = xor3(xor3(acc[e][4 * NP + d], v[e][0][d], v[e][1][d]), v[e][2][d], v[e][3][d]);
    } else if constexpr (G % 2 && !TV) {  // 2- or 4-byte entries: rows 8 NP (+ 1) in acc[e][4 NP]
        uint32_t v[E][4];
#pragma unroll
        for (int e = 0; e < E; e++)
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const uint8_t *at = blk + n[e][q] * TB + (q * BQ + NP * 256);
                if constexpr (TB == 2) v[e][q] = *(lds_u16 *)at;
                else v[e][q] = *(lds_u32 *)at;
            }
#pragma unroll
        for (int e = 0; e < E; e++)
            acc[e][4 * NP] = xor3(xor3(acc[e][4 * NP], v[e][0], v[e][1]), v[e][2], v[e][3]);
    }
}

// t ^ (m & c) (v_bitop3_b32, LUT over src0 = 0xf0, src1 = 0xcc, src2 = 0xaa)
__device__ __forceinline__ uint32_t xor_and(uint32_t t, uint32_t m, uint32_t c) {
    uint32_t d;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x78" : "=v"(d) : "v"(t), "v"(m), "s"(c));
    return d;
}
// The lone last row of rows = 8 h + 1 on the VALU: x * c = XOR over the set bits b of x of K[b] =
// c * 2^b (16 constants per input, scalar loads).  E = 2: both elements at once -- bit b of each
// half spread over its half by a packed shift pair (v_pk_lshlrev_b16 / v_pk_ashrrev_i16), K[b]
// in both halves: 3 VALU per bit for two products, against the tail group's 8 LDS cycles (4-row
// entries of which 1 row is used) in the LDS-bound kernel.  Products accumulate in t (element e
// in half e; E = 1: the low half).
typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(4))) const uint32_t const_u32;  // constant space: scalar loads
template <int E>
__device__ __forceinline__ uint32_t mat_tail(uint32_t t, uint32_t w, int sh, const_u32 *K) {
#pragma unroll
    for (int b = 0; b < 16; b++) {
        uint32_t m;
        if constexpr (E == 2) {
            s16x2 x = __builtin_bit_cast(s16x2, w);
            if (b != 15) x = (s16x2)(x << (short)(15 - b));
            m = __builtin_bit_cast(uint32_t, (s16x2)(x >> (short)15));
        } else {
            m = (uint32_t)__builtin_amdgcn_sbfe((int)w, sh + b, 1);
        }
        t = xor_and(t, m, K[b]);
    }
    return t;
}

#ifndef TEC_RS16_MAT_E
#define TEC_RS16_MAT_E 2     // elements per thread: 2 (16-bit loads / stores) or 1 (byte ones, fewer VGPRs)
#endif
#ifndef TEC_RS16_MAT_BT
#define TEC_RS16_MAT_BT 512  // threads per block (2 blocks per CU at OuterCoder(17, 50)'s 78 KB image)
#endif
#ifndef TEC_RS16_MAT_TVPOS
#define TEC_RS16_MAT_TVPOS 1  // where the VALU tail row runs: 1 = before the table reads, 0 = per input beside them
#endif
#ifndef TEC_RS16_MAT_WPE
#define TEC_RS16_MAT_WPE 4   // waves per SIMD the registers are budgeted for
#endif
constexpr int kMatE = TEC_RS16_MAT_E, kMatBT = TEC_RS16_MAT_BT;

template <int G, int KB, bool PTRS, bool TV, int TB>  // KB: input slots (k <= KB); TV: rows = 8 (G / 2) + 1, mat_tail; TB: tail entry bytes
__global__ void __launch_bounds__(kMatBT) __attribute__((amdgpu_waves_per_eu(TEC_RS16_MAT_WPE)))
rs16_matrix_kernel(Rs16MatArgs a) {
    constexpr int E = kMatE, NP = G / 2, BQ = mat_block_bytes<G, TB, TV>();
    extern __shared__ __attribute__((aligned(16))) uint16_t lds16[];
    {
        const uint32_t n16 = a.k * (uint32_t)BQ / 4u;  // 16-byte units of the image (4 blocks per input)
        for (uint32_t t = threadIdx.x; t < n16; t += blockDim.x)
            reinterpret_cast<uint4 *>(lds16)[t] = reinterpret_cast<const uint4 *>(a.tab)[t];
    }
    __syncthreads();
    const uint8_t *tab = reinterpret_cast<const uint8_t *>(lds16);
    const uint32_t units = a.elems / E, tps = (units + blockDim.x - 1) / blockDim.x;
    const uint32_t ntiles = a.segments * tps;
    for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {  // no barrier in the loop
        // k and the strides re-read opaquely per tile: loop-invariant, the per-input and per-row
        // offsets derived from them were hoisted out of the tile loop (~100 scalars, 324 SGPRs
        // spilled to VGPR lanes); a few scalar ops per tile instead
        uint32_t k = a.k, rstride = a.rstride;
        uint64_t in_stride = a.in_stride, out_stride = a.out_stride;
        const uint32_t *ktab = a.ktab;
        asm volatile("" : "+s"(k), "+s"(rstride), "+s"(in_stride), "+s"(out_stride), "+s"(ktab));
        const uint32_t seg = tile / tps, u = (tile - seg * tps) * blockDim.x + threadIdx.x;
        if (u >= units) continue;
        const uint32_t e0 = E * u, eo = (e0 >> 5) * 64u + (e0 & 31u);
        auto inp = [&](uint32_t r) -> const uint8_t * {
            if constexpr (PTRS) return a.ptr[seg * (k + a.rows) + r] + eo;
            else return a.in + (uint64_t)seg * a.seg_in + (uint64_t)r * in_stride + eo;
        };
        uint32_t acc[E][2 * G];
#pragma unroll
        for (int e = 0; e < E; e++)
#pragma unroll
            for (int i = 0; i < 2 * G; i++) acc[e][i] = 0;
        // every input loaded up front (KB >= k slots, indices past k - 1 clamped), 32 bits of
        // elements per VGPR (E = 2: both elements of one input, one v_perm; E = 1: two inputs), and
        // all of them pinned here by an empty asm: otherwise the compiler sinks each load into the
        // run-time-guarded block that uses it and waits for it there, one HBM latency per input (a
        // rolling prefetch in a loop fared no better: its waits came out as vmcnt(0)).  One wait
        // per tile; the other waves on the CU cover it.
        constexpr int NW = E == 2 ? KB : KB / 2;
        uint32_t P[NW];
#pragma unroll
        for (int j = 0; j < KB; j++) {
            const uint8_t *s = inp((uint32_t)j < k ? (uint32_t)j : k - 1u);
            if constexpr (E == 2) {
                const uint32_t lo = *reinterpret_cast<const uint16_t *>(s), hi = *reinterpret_cast<const uint16_t *>(s + 32);
                P[j] = __builtin_amdgcn_perm(hi, lo, 0x05010400u);  // [lo.b0, hi.b0, lo.b1, hi.b1]
            } else {
                const uint32_t x = (uint32_t)s[0] | (uint32_t)s[32] << 8;
                P[j >> 1] = (j & 1) ? P[j >> 1] | x << 16 : x;
            }
        }
#pragma unroll
        for (int j = 0; j < NW; j++) asm volatile("" ::"v"(P[j]));
        // TV: the tail products first, in their own pass (TEC_RS16_MAT_TVPOS 1): their scalar
        // loads share lgkmcnt with the LDS reads and return out of order, so each use waits for
        // lgkmcnt(0) -- interleaved with the table reads (0) that drains the wave's LDS queue per input
        uint32_t tv = 0;
        if constexpr (TV && TEC_RS16_MAT_TVPOS == 1) {
#pragma unroll
            for (int r = 0; r < KB; r++)
                if ((uint32_t)r < k) tv = mat_tail<E>(tv, E == 2 ? P[r] : P[r >> 1], E == 2 ? 0 : 16 * (r & 1), (const_u32 *)ktab + r * 16);
        }
#pragma unroll
        for (int r = 0; r < KB; r++)
            if ((uint32_t)r < k) {
                const uint32_t w = E == 2 ? P[r] : P[r >> 1];
                const int sh = E == 2 ? 0 : 16 * (r & 1);
                mat_input<G, E, TV, TB>(acc, tab + r * rstride, w, sh);
                if constexpr (TV && TEC_RS16_MAT_TVPOS == 0) tv = mat_tail<E>(tv, w, sh, (const_u32 *)ktab + r * 16);
            }
        if constexpr (TV) {
            acc[0][4 * NP] = tv & 0xffffu;
            if constexpr (E == 2) acc[E - 1][4 * NP] = tv >> 16;
        }
#pragma unroll
        for (int i = 0; i < 4 * G; i++) {
            if ((uint32_t)i >= a.rows) continue;
            uint8_t *o;
            if constexpr (PTRS) o = const_cast<uint8_t *>(a.ptr[seg * (k + a.rows) + k + i]) + eo;
            else o = a.out + (uint64_t)seg * a.seg_out + (uint64_t)i * out_stride + eo;
            const uint32_t v0 = (acc[0][i >> 1] >> (16 * (i & 1))) & 0xffffu;
            if constexpr (E == 2) {
                const uint32_t v1 = (acc[E - 1][i >> 1] >> (16 * (i & 1))) & 0xffffu;
                *reinterpret_cast<uint16_t *>(o) = (uint16_t)((v0 & 0xffu) | (v1 & 0xffu) << 8);
                *reinterpret_cast<uint16_t *>(o + 32) = (uint16_t)((v0 >> 8) | (v1 & 0xff00u));
            } else {
                o[0] = (uint8_t)v0;
                o[32] = (uint8_t)(v0 >> 8);
            }
        }
    }
}

template <int G, int KB, bool TV, int TB>
hipError_t launch_mat_gkt(Rs16MatArgs a, uint32_t grid, size_t lds, hipStream_t s) {
    a.rstride = 4u * (uint32_t)mat_block_bytes<G, TB, TV>();
    if ((size_t)a.k * a.rstride != lds) return hipErrorInvalidValue;  // host image and kernel layout agree
    a.ktab = TV ? reinterpret_cast<const uint32_t *>(reinterpret_cast<const uint8_t *>(a.tab) + lds) : nullptr;
    const void *fn = a.ptrs ? reinterpret_cast<const void *>(rs16_matrix_kernel<G, KB, true, TV, TB>)
                            : reinterpret_cast<const void *>(rs16_matrix_kernel<G, KB, false, TV, TB>);
    if (const hipError_t e = ensure_dyn_lds(fn, lds); e != hipSuccess) return e;
    if (a.ptrs) hipLaunchKernelGGL((rs16_matrix_kernel<G, KB, true, TV, TB>), dim3(grid), dim3(kMatBT), lds, s, a);
    else hipLaunchKernelGGL((rs16_matrix_kernel<G, KB, false, TV, TB>), dim3(grid), dim3(kMatBT), lds, s, a);
    return hipGetLastError();
}
template <int G, int KB>
hipError_t launch_mat_gk(const Rs16MatArgs &a, uint32_t grid, size_t lds, hipStream_t s) {
    if constexpr (G % 2 == 1) {
        if constexpr (TEC_RS16_MAT_TV && G > 1)
            if (rs16_mat_tailv(a.rows)) return launch_mat_gkt<G, KB, true, 8>(a, grid, lds, s);
        switch (rs16_mat_tail_bytes(a.rows)) {
            case 2: return launch_mat_gkt<G, KB, false, 2>(a, grid, lds, s);
            case 4: return launch_mat_gkt<G, KB, false, 4>(a, grid, lds, s);
            default: break;
        }
    }
    return launch_mat_gkt<G, KB, false, 8>(a, grid, lds, s);
}
template <int G>
hipError_t launch_mat_g(const Rs16MatArgs &a, uint32_t grid, size_t lds, hipStream_t s) {
    if constexpr (G <= (int)kRs16MatMaxG) {
        if ((a.rows + 3) / 4 > (uint32_t)G) return launch_mat_g<G + 1>(a, grid, lds, s);
        if (a.k <= 16) return launch_mat_gk<G, 16>(a, grid, lds, s);
        if (a.k <= 32) return launch_mat_gk<G, 32>(a, grid, lds, s);
    }
    return hipErrorInvalidValue;
}

// Restore the missing originals: out[i] = sum_r D[i][r] * received[r] (nibble tables per
// coefficient, staged in LDS).  REG (k <= 32): a thread loads its element of each received shard
// once into registers and computes every missing output from them (the first kernel re-read the
// k received elements for each of the nmiss outputs).
// TLDS: the tables staged in LDS (<= kRs16DecLds), else read from L2.  A compile-time choice, so the
// lookups are ds_read_u16 with 32-bit addresses: a run-time select between the two pointers made
// every lookup a flat load with 64-bit address arithmetic (r04: 1,225 flat loads and 4,577 VALU per
// wave per segment, 16 VALU per product)
template <int KB, bool TLDS>  // KB: k rounded up to 4 (<= 32), 0 = any k, elements re-read per output
__global__ void __launch_bounds__(512) rs16_decode_kernel(Rs16DecArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint16_t lds16[];
    const uint32_t ntab = a.nmiss * a.k;
    if constexpr (TLDS) {
        for (uint32_t t = threadIdx.x; t < ntab * 32u; t += blockDim.x)
            reinterpret_cast<uint32_t *>(lds16)[t] = reinterpret_cast<const uint32_t *>(a.lut)[t];
        __syncthreads();
    }
    const uint16_t *tab;
    if constexpr (TLDS) tab = lds16; else tab = a.lut;
    const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= a.elems) return;
    const uint32_t pb = blockIdx.y * (a.k + a.nmiss);
    auto recv = [&](uint32_t r) { return a.ptr[pb + r]; };
    auto outp = [&](uint32_t i) { return const_cast<uint8_t *>(a.ptr[pb + a.k + i]); };
    if constexpr (KB > 0) {
        // two adjacent elements per thread (their low bytes adjacent, their high bytes 32 B on:
        // 16-bit loads and stores instead of byte ones).  Per received element its four lookup
        // offsets into a coefficient's 64-entry table, one byte each (byte q = 32 q + 2 * nibble
        // q), built once: a lookup is then one add with a byte select plus the ds_read (the r02
        // kernel re-derived each nibble index per output).  KB = k rounded up to 4: the products
        // run branch-free (a branch per product kept each product's four reads waiting alone);
        // the r >= k ones read entry 0 (= 0) of table k - 1
        const uint32_t e0 = 2u * e;
        if (e0 >= a.elems) return;
        const uint32_t eo = (e0 >> 5) * 64u + (e0 & 31u);  // e0 even: 2-byte aligned
        auto spread = [](uint32_t x) {
            return ((x & 0xfu) << 1) | ((x & 0xf0u) << 5) | ((x & 0xf00u) << 9) | ((x & 0xf000u) << 13) | 0x60402000u;
        };
        uint32_t off0[KB], off1[KB];
#pragma unroll
        for (uint32_t r = 0; r < (uint32_t)KB; r++) {
            uint32_t lo = 0, hi = 0;
            if (r < a.k) {
                lo = *reinterpret_cast<const uint16_t *>(recv(r) + eo);
                hi = *reinterpret_cast<const uint16_t *>(recv(r) + eo + 32u);
            }
            off0[r] = spread((lo & 0xffu) | (hi & 0xffu) << 8);
            off1[r] = spread((lo >> 8) | (hi & 0xff00u));
        }
#pragma unroll 1
        for (uint32_t i = 0; i < a.nmiss; i++) {
            const uint8_t *ti = reinterpret_cast<const uint8_t *>(tab) + i * a.k * 128u;
#pragma unroll
            for (uint32_t r = 0; r < (uint32_t)KB; r++) asm volatile("" : "+v"(off0[r]), "+v"(off1[r]));  // packed
            uint32_t acc0 = 0, acc1 = 0;
            auto look = [](const uint8_t *tr, uint32_t o) {
                return *reinterpret_cast<const uint16_t *>(tr + (o & 0xffu)) ^
                       *reinterpret_cast<const uint16_t *>(tr + ((o >> 8) & 0xffu)) ^
                       *reinterpret_cast<const uint16_t *>(tr + ((o >> 16) & 0xffu)) ^
                       *reinterpret_cast<const uint16_t *>(tr + (o >> 24));
            };
#pragma unroll
            for (uint32_t r = 0; r < (uint32_t)KB; r++) {
                const uint8_t *tr = ti + (r < a.k ? r : a.k - 1u) * 128u;
                acc0 ^= look(tr, off0[r]);
                acc1 ^= look(tr, off1[r]);
            }
            uint8_t *o = outp(i) + eo;
            *reinterpret_cast<uint16_t *>(o) = (uint16_t)((acc0 & 0xffu) | (acc1 & 0xffu) << 8);
            *reinterpret_cast<uint16_t *>(o + 32u) = (uint16_t)((acc0 >> 8) | (acc1 & 0xff00u));
        }
    } else {
        for (uint32_t i = 0; i < a.nmiss; i++) {
            uint32_t acc = 0;
            for (uint32_t r = 0; r < a.k; r++) acc ^= mulx(ld_elem(recv(r), e), tab + (i * a.k + r) * 64u);
            st_elem(outp(i), e, acc);
        }
    }
}

// k <= 32: the KB = ceil(k / 4) * 4 instance; larger k: elements re-read per output
template <int KB>
hipError_t launch_dec_kb(const Rs16DecArgs &a, dim3 grid, dim3 block, size_t lds, hipStream_t s) {  // grid.y = segments
    if constexpr (KB <= 32) {
        if (a.k > (uint32_t)KB) return launch_dec_kb<KB + 4>(a, grid, block, lds, s);
        if (lds) hipLaunchKernelGGL((rs16_decode_kernel<KB, true>), grid, block, lds, s, a);
        else hipLaunchKernelGGL((rs16_decode_kernel<KB, false>), grid, block, 0, s, a);
    } else {
        if (lds) hipLaunchKernelGGL((rs16_decode_kernel<0, true>), grid, block, lds, s, a);
        else hipLaunchKernelGGL((rs16_decode_kernel<0, false>), grid, block, 0, s, a);
    }
    return hipGetLastError();
}

}  // namespace rs16k


// Block size of the encode: the nibble tables (span x 128 B) are staged once per block and every
// thread keeps work_len u16 in LDS, so larger blocks amortise the tables; pick the size that
// keeps the most waves per CU within its 160 KB of LDS (128 threads, 32.5 KB, for OuterCoder(17,
// 50) left 8 waves per CU; 512 threads, 80.5 KB, leave 16; with one chunk of work per thread,
// 1024 threads, 80.5 KB, leave 32).
static uint32_t rs16_enc_threads(const Rs16EncArgs &a, size_t *lds_out) {
    uint32_t best_t = 128, best_w = 0;
    size_t best_lds = 0;
    const uint32_t per = a.one_chunk ? a.c : a.work_len;  // u16 of work per thread
    for (uint32_t t = 128; t <= 1024; t *= 2) {
        const size_t lds = (size_t)a.span * 128u + (size_t)per * t * 2u;
        if (lds > 160 * 1024) break;
        // whole blocks fit within the LDS and within the waves per SIMD the kernel's registers allow
        const uint32_t blocks = std::min((uint32_t)((160 * 1024) / lds), 4u * TEC_RS16_WPE / (t / 64u));
        const uint32_t waves = blocks * (t / 64u);
        if (waves > best_w) { best_w = waves; best_t = t; best_lds = lds; }
    }
    *lds_out = best_lds;
    return best_w ? best_t : 0;
}

hipError_t launch_rs16_encode(const Rs16EncArgs &a, uint32_t segments, hipStream_t s) {
    if (a.elems == 0 || segments == 0) return hipSuccess;
#if TEC_RS16_REG
    if (a.one_chunk && a.c >= 1 && a.c <= 32) {
        if (segments > 65535) return hipErrorInvalidValue;
        const size_t lds = (size_t)a.span * 128u;
        const dim3 grid((a.elems + 255) / 256, segments);
        const void *fn = nullptr;
        switch (a.c) {
        case 1: fn = reinterpret_cast<const void *>(rs16k::rs16_encode_low_kernel<1>); break;
        case 2: fn = reinterpret_cast<const void *>(rs16k::rs16_encode_low_kernel<2>); break;
        case 4: fn = reinterpret_cast<const void *>(rs16k::rs16_encode_low_kernel<4>); break;
        case 8: fn = reinterpret_cast<const void *>(rs16k::rs16_encode_low_kernel<8>); break;
        case 16: fn = reinterpret_cast<const void *>(rs16k::rs16_encode_low_kernel<16>); break;
        case 32: fn = reinterpret_cast<const void *>(rs16k::rs16_encode_low_kernel<32>); break;
        default: return hipErrorInvalidValue;
        }
        const hipError_t e = ensure_dyn_lds(fn, lds);
        if (e != hipSuccess) return e;
        switch (a.c) {
        case 1: hipLaunchKernelGGL(rs16k::rs16_encode_low_kernel<1>, grid, dim3(256), lds, s, a); break;
        case 2: hipLaunchKernelGGL(rs16k::rs16_encode_low_kernel<2>, grid, dim3(256), lds, s, a); break;
        case 4: hipLaunchKernelGGL(rs16k::rs16_encode_low_kernel<4>, grid, dim3(256), lds, s, a); break;
        case 8: hipLaunchKernelGGL(rs16k::rs16_encode_low_kernel<8>, grid, dim3(256), lds, s, a); break;
        case 16: hipLaunchKernelGGL(rs16k::rs16_encode_low_kernel<16>, grid, dim3(256), lds, s, a); break;
        default: hipLaunchKernelGGL(rs16k::rs16_encode_low_kernel<32>, grid, dim3(256), lds, s, a); break;
        }
        return hipGetLastError();
    }
#endif
    size_t lds = 0;
    const uint32_t t = rs16_enc_threads(a, &lds);
    if (!t || segments > 65535) return hipErrorInvalidValue;
    const hipError_t e = ensure_dyn_lds(reinterpret_cast<const void *>(rs16k::rs16_encode_kernel), lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(rs16k::rs16_encode_kernel, dim3((uint32_t)((a.elems + t - 1) / t), segments), dim3(t), lds, s, a);
    return hipGetLastError();
}

hipError_t launch_rs16_matrix(const Rs16MatArgs &a, hipStream_t s) {
    if (a.elems == 0 || a.segments == 0) return hipSuccess;
    if (!rs16_mat_supported(a.k, a.rows) || a.elems % 2) return hipErrorInvalidValue;
    if (a.ptrs && (uint64_t)a.segments * (a.k + a.rows) > kRs16DecPtrs) return hipErrorInvalidValue;
    const uint64_t tiles = (uint64_t)a.segments * ((a.elems / rs16k::kMatE + rs16k::kMatBT - 1) / rs16k::kMatBT);
    if (tiles > 0xffffffffull) return hipErrorInvalidValue;
    // a resident grid (2 blocks per CU at the largest image) looping over the tiles: the image is
    // staged once per block, not once per 1,024 columns
    const uint32_t grid = (uint32_t)std::min<uint64_t>(tiles, 2048);
    return rs16k::launch_mat_g<1>(a, grid, rs16_mat_bytes(a.k, a.rows), s);
}

hipError_t launch_rs16_decode(const Rs16DecArgs &a, uint32_t segments, hipStream_t s) {
    if (a.elems == 0 || a.nmiss == 0 || segments == 0) return hipSuccess;
    if ((uint64_t)segments * (a.k + a.nmiss) > kRs16DecPtrs || segments > 65535) return hipErrorInvalidValue;
    const size_t tab = (size_t)a.nmiss * a.k * 128u, lds = tab <= rs16k::kRs16DecLds ? tab : 0;
    if (a.k > kRs16MaxK || a.nmiss > kRs16MaxK) return hipErrorInvalidValue;
    // 512-thread blocks: the tables (<= 48 KB) are staged once per 8 waves, not per 2; k <= 32:
    // two elements per thread (elems is a multiple of 32: 64-byte shard blocks)
    if (a.k <= 32 && a.elems % 2) return hipErrorInvalidValue;
    const uint64_t threads = a.k <= 32 ? a.elems / 2 : a.elems;
    const dim3 grid((uint32_t)((threads + 511) / 512), segments), block(512);
    return rs16k::launch_dec_kb<4>(a, grid, block, lds, s);
}

}  // namespace tec
