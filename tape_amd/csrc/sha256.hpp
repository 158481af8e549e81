// sha256.hpp -- SHA-256 (FIPS 180-4) compression and the merkle hashes of lib/crypto, shared by
// the commitment kernels (commit.hip) and the host entry points (engine.cpp).
//
// hash_leaf(data)   = SHA-256("LEAF" || data)                        lib/crypto/src/merkle/tree.rs:53-56
// hash_pair(l, r)   = SHA-256("LEFT" || l || "RIGHT" || r)           tree.rs:58-62
// (`hashv` hashes the concatenation of its parts, lib/crypto/src/hash.rs:91-98.)
// Plain C operators throughout: on gfx950 the rotates become v_alignbit_b32, the three-input
// logic v_bitop3_b32 and the three-term adds v_add3_u32.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tec {
namespace sha {

__host__ __device__ constexpr uint32_t kK(int i) {
    constexpr uint32_t k[64] = {
        0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
        0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
        0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
        0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
        0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
        0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
        0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
        0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};
    return k[i];
}
constexpr uint32_t kH0[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                             0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
constexpr uint32_t kLeafWord = 0x4c454146u;  // "LEAF" as a big-endian message word

__host__ __device__ __forceinline__ uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
// three-way XOR: one v_bitop3_b32 on gfx950 (the backend forms it for Ch/Maj but not here)
__host__ __device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
    return a ^ b ^ c;
#endif
}
__host__ __device__ __forceinline__ uint32_t bswap(uint32_t x) {
    return (x >> 24) | ((x >> 8) & 0xff00u) | ((x << 8) & 0xff0000u) | (x << 24);
}

// One 64-byte block (16 big-endian words, consumed) into the state.
__host__ __device__ __forceinline__ void compress(uint32_t st[8], uint32_t w[16]) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
    for (int i = 0; i < 64; i++) {
        if (i >= 16) {
            const uint32_t w15 = w[(i + 1) & 15], w2 = w[(i + 14) & 15];
            const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
            const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
            w[i & 15] = w[i & 15] + s0 + w[(i + 9) & 15] + s1;
        }
        const uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
        const uint32_t ch = (e & f) ^ (~e & g);
        const uint32_t t1 = h + S1 + ch + kK(i) + w[i & 15];
        const uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
        const uint32_t mj = (a & b) | (c & (a | b));
        h = g; g = f; f = e; e = d + t1;
        d = c; c = b; b = a; a = t1 + S0 + mj;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

__host__ __device__ __forceinline__ void init(uint32_t st[8]) {
#pragma unroll
    for (int i = 0; i < 8; i++) st[i] = kH0[i];
}

// Streaming SHA-256 over byte parts (host side and the per-object tree work on the device).
struct Stream {
    uint32_t st[8];
    uint8_t buf[64];
    uint32_t nbuf;
    uint64_t total;
    __host__ __device__ void begin() { init(st); nbuf = 0; total = 0; }
    __host__ __device__ void block() {
        uint32_t w[16];
        for (int i = 0; i < 16; i++)
            w[i] = (uint32_t)buf[4 * i] << 24 | (uint32_t)buf[4 * i + 1] << 16 | (uint32_t)buf[4 * i + 2] << 8 | buf[4 * i + 3];
        compress(st, w);
        nbuf = 0;
    }
    __host__ __device__ void update(const uint8_t *p, uint64_t n) {
        total += n;
        while (n) {
            const uint32_t take = (uint32_t)((64u - nbuf) < n ? (64u - nbuf) : n);
            for (uint32_t i = 0; i < take; i++) buf[nbuf + i] = p[i];
            nbuf += take; p += take; n -= take;
            if (nbuf == 64) block();
        }
    }
    __host__ __device__ void finish(uint8_t out[32]) {
        const uint64_t bits = total * 8;
        buf[nbuf++] = 0x80;
        if (nbuf > 56) {
            while (nbuf < 64) buf[nbuf++] = 0;
            block();
        }
        while (nbuf < 56) buf[nbuf++] = 0;
        for (int i = 0; i < 8; i++) buf[56 + i] = (uint8_t)(bits >> (56 - 8 * i));
        block();
        for (int i = 0; i < 8; i++) {
            out[4 * i] = (uint8_t)(st[i] >> 24); out[4 * i + 1] = (uint8_t)(st[i] >> 16);
            out[4 * i + 2] = (uint8_t)(st[i] >> 8); out[4 * i + 3] = (uint8_t)st[i];
        }
    }
};

__host__ __device__ inline void hash_leaf(const uint8_t *data, uint64_t len, uint8_t out[32]) {
    Stream s;
    s.begin();
    const uint8_t label[4] = {'L', 'E', 'A', 'F'};
    s.update(label, 4);
    s.update(data, len);
    s.finish(out);
}

__host__ __device__ inline void hash_pair(const uint8_t l[32], const uint8_t r[32], uint8_t out[32]) {
    Stream s;
    s.begin();
    const uint8_t left[4] = {'L', 'E', 'F', 'T'}, right[5] = {'R', 'I', 'G', 'H', 'T'};
    s.update(left, 4);
    s.update(l, 32);
    s.update(right, 5);
    s.update(r, 32);
    s.finish(out);
}

// EMPTY_ROOTS[h] (tree.rs:15-48): hash_leaf([]) paired with itself h times (tree.rs:832-841).
__host__ __device__ inline void empty_root(uint32_t height, uint8_t out[32]) {
    hash_leaf(nullptr, 0, out);
    for (uint32_t i = 0; i < height; i++) {
        uint8_t t[32];
        hash_pair(out, out, t);
        for (int j = 0; j < 32; j++) out[j] = t[j];
    }
}

}  // namespace sha
}  // namespace tec
