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
#include "kernels.hpp"

namespace tec {
namespace rs16k {

constexpr uint32_t kRs16DecLds = 48 * 1024;  // decoding tables staged in LDS up to this size

__device__ __forceinline__ uint32_t mulx(uint32_t x, const uint16_t *T) {
    return T[x & 15u] ^ T[16u + ((x >> 4) & 15u)] ^ T[32u + ((x >> 8) & 15u)] ^ T[48u + (x >> 12)];
}

struct Col {  // one thread's work vector in LDS
    uint16_t *w;
    uint32_t bt;
    __device__ uint32_t ld(uint32_t i) const { return w[i * bt]; }
    __device__ void st(uint32_t i, uint32_t v) const { w[i * bt] = (uint16_t)v; }
};

// FFT / IFFT of work[pos .. pos + size) (rs16.hpp restated on LDS columns)
__device__ void fft(const Col &c, const uint16_t *lut, uint32_t pos, uint32_t size, uint32_t trunc, uint32_t delta) {
    auto b2 = [&](uint32_t ix, uint32_t iy, uint32_t s) {
        uint32_t x = c.ld(pos + ix), y = c.ld(pos + iy);
        x ^= mulx(y, lut + s * 64u);
        y ^= x;
        c.st(pos + ix, x);
        c.st(pos + iy, y);
    };
    uint32_t dist4 = size, dist = size >> 2;
    for (; dist; dist4 = dist, dist >>= 2)
        for (uint32_t r = 0; r < trunc; r += dist4) {
            const uint32_t b = r + dist + delta - 1;
            for (uint32_t i = r; i < r + dist; i++) {
                b2(i, i + 2 * dist, b + dist);
                b2(i + dist, i + 3 * dist, b + dist);
                b2(i, i + dist, b);
                b2(i + 2 * dist, i + 3 * dist, b + 2 * dist);
            }
        }
    if (dist4 == 2)
        for (uint32_t r = 0; r < trunc; r += 2) b2(r, r + 1, r + delta);
}

__device__ void ifft(const Col &c, const uint16_t *lut, uint32_t pos, uint32_t size, uint32_t trunc, uint32_t delta) {
    auto b2 = [&](uint32_t ix, uint32_t iy, uint32_t s) {
        uint32_t x = c.ld(pos + ix), y = c.ld(pos + iy);
        y ^= x;
        x ^= mulx(y, lut + s * 64u);
        c.st(pos + ix, x);
        c.st(pos + iy, y);
    };
    uint32_t dist = 1, dist4 = 4;
    for (; dist4 <= size; dist = dist4, dist4 <<= 2)
        for (uint32_t r = 0; r < trunc; r += dist4) {
            const uint32_t b = r + dist + delta - 1;
            for (uint32_t i = r; i < r + dist; i++) {
                b2(i, i + dist, b);
                b2(i + 2 * dist, i + 3 * dist, b + 2 * dist);
                b2(i, i + 2 * dist, b + dist);
                b2(i + dist, i + 3 * dist, b + dist);
            }
        }
    if (dist < size)
        for (uint32_t i = 0; i < dist; i++) b2(i, i + dist, dist + delta - 1);
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

__global__ void __launch_bounds__(128) rs16_encode_kernel(Rs16EncArgs a) {  // grid.y = segments
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
    for (uint32_t i = 0; i < a.work_len; i++) c.st(i, 0);
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
// coefficient, staged in LDS).
__global__ void __launch_bounds__(128) rs16_decode_kernel(Rs16DecArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint16_t lds16[];
    const uint32_t ntab = a.nmiss * a.k;
    const bool in_lds = ntab * 128u <= kRs16DecLds;  // else the tables are read from L2
    if (in_lds) {
        for (uint32_t t = threadIdx.x; t < ntab * 32u; t += blockDim.x)
            reinterpret_cast<uint32_t *>(lds16)[t] = reinterpret_cast<const uint32_t *>(a.lut)[t];
        __syncthreads();
    }
    const uint16_t *tab = in_lds ? lds16 : a.lut;
    const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= a.elems) return;
    for (uint32_t i = 0; i < a.nmiss; i++) {
        uint32_t acc = 0;
        for (uint32_t r = 0; r < a.k; r++) acc ^= mulx(ld_elem(a.recv[r], e), tab + (i * a.k + r) * 64u);
        st_elem(a.out[i], e, acc);
    }
}

}  // namespace rs16k

static uint32_t rs16_blocks(uint64_t elems) { return (uint32_t)((elems + 127) / 128); }

hipError_t launch_rs16_encode(const Rs16EncArgs &a, uint32_t segments, hipStream_t s) {
    if (a.elems == 0 || segments == 0) return hipSuccess;
    const size_t lds = (size_t)a.span * 128u + (size_t)a.work_len * 128u * 2u;
    if (lds > 64 * 1024 || segments > 65535) return hipErrorInvalidValue;
    hipLaunchKernelGGL(rs16k::rs16_encode_kernel, dim3(rs16_blocks(a.elems), segments), dim3(128), lds, s, a);
    return hipGetLastError();
}

hipError_t launch_rs16_decode(const Rs16DecArgs &a, hipStream_t s) {
    if (a.elems == 0 || a.nmiss == 0) return hipSuccess;
    const size_t tab = (size_t)a.nmiss * a.k * 128u, lds = tab <= rs16k::kRs16DecLds ? tab : 0;
    if (a.k > kRs16MaxK || a.nmiss > kRs16MaxK) return hipErrorInvalidValue;
    hipLaunchKernelGGL(rs16k::rs16_decode_kernel, dim3(rs16_blocks(a.elems)), dim3(128), lds, s, a);
    return hipGetLastError();
}

}  // namespace tec
