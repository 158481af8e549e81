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
    size_t lds = 0;
    const uint32_t t = rs16_enc_threads(a, &lds);
    if (!t || segments > 65535) return hipErrorInvalidValue;
    const hipError_t e = ensure_dyn_lds(reinterpret_cast<const void *>(rs16k::rs16_encode_kernel), lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(rs16k::rs16_encode_kernel, dim3((uint32_t)((a.elems + t - 1) / t), segments), dim3(t), lds, s, a);
    return hipGetLastError();
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
