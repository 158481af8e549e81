// dev_io.hpp -- sub-chunk word access for the Clay kernels.
//
// A "word" is 4 byte-columns of one sub-chunk (cols c..c+3).  Sub-chunks are sc bytes with
// sc = chunk_size/alpha, always even but only 2-aligned (sc = 1,430 for 1 MB stripes), so a
// word sits at an address that is 0 or 2 mod 4.  Aligned words move as one dword; the others as
// two 16-bit halves (never an unaligned dword).  When sc = 2 mod 4 the last word of a
// sub-chunk carries only 2 columns, so alignment stays uniform across a wave.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tec {

struct WordPos {
    uint32_t c;   // first column
    uint32_t nc;  // columns in this word: 4 (or 2 when sc == 2)
};

__device__ __forceinline__ WordPos word_pos(uint32_t w, uint32_t sc) {
    WordPos p;
    p.c = w * 4u;
    p.nc = p.c + 4u <= sc ? 4u : sc - p.c;
    return p;
}

// Load a word from base+off where only [0, len) of base is valid (zero-padding beyond).
__device__ __forceinline__ uint32_t ld_word(const uint8_t *__restrict__ base, uint64_t off,
                                            uint64_t len, uint32_t nc) {
    const uint8_t *p = base + off;
    const uintptr_t al = reinterpret_cast<uintptr_t>(p) & 3u;
    if (off + nc <= len && (al & 1u) == 0) {
        if (nc == 4) {
            if (al == 0) return *reinterpret_cast<const uint32_t *>(p);
            const uint32_t lo = *reinterpret_cast<const uint16_t *>(p);
            const uint32_t hi = *reinterpret_cast<const uint16_t *>(p + 2);
            return lo | (hi << 16);
        }
        return *reinterpret_cast<const uint16_t *>(p);
    }
    // tail of the valid region (zero padding beyond len) or an odd caller offset: bytes
    uint32_t v = 0;
    for (uint32_t i = 0; i < nc; i++)
        if (off + i < len) v |= (uint32_t)p[i] << (8 * i);
    return v;
}

__device__ __forceinline__ void st_word(uint8_t *__restrict__ p, uint32_t v, uint32_t nc) {
    const uintptr_t al = reinterpret_cast<uintptr_t>(p) & 3u;
    if (al == 0 && nc == 4) {
        *reinterpret_cast<uint32_t *>(p) = v;
    } else if ((al & 1u) == 0) {
        *reinterpret_cast<uint16_t *>(p) = (uint16_t)v;
        if (nc == 4) *reinterpret_cast<uint16_t *>(p + 2) = (uint16_t)(v >> 16);
    } else {
        for (uint32_t i = 0; i < nc; i++) p[i] = (uint8_t)(v >> (8 * i));
    }
}

// Store only the bytes of the word that fall below `limit` (byte offset bound of the output).
__device__ __forceinline__ void st_word_trim(uint8_t *__restrict__ base, uint64_t off, uint64_t limit,
                                             uint32_t v, uint32_t nc) {
    if (off + nc <= limit) {
        st_word(base + off, v, nc);
        return;
    }
    for (uint32_t i = 0; i < nc; i++)
        if (off + i < limit) base[off + i] = (uint8_t)(v >> (8 * i));
}

// Wave-uniform access: `ub` (uniform base, SGPR) + the lane's 32-bit column offset.  `al` is the
// uniform alignment of ub (ub & 3): 0 -> one dword, 2 -> two 16-bit halves, odd -> bytes.
#define TEC_GLOBAL __attribute__((address_space(1)))
typedef TEC_GLOBAL uint8_t g_u8;
typedef TEC_GLOBAL uint16_t g_u16;
typedef TEC_GLOBAL uint32_t g_u32;

__device__ __forceinline__ uint32_t ld_u(const uint8_t *ub_, uint32_t col, uint32_t al) {
    const g_u8 *ub = (const g_u8 *)ub_;
    if (al == 0) return *(const g_u32 *)(ub + col);
    if (al == 2) {
        const uint32_t lo = *(const g_u16 *)(ub + col);
        const uint32_t hi = *(const g_u16 *)(ub + col + 2);
        return lo | (hi << 16);
    }
    const g_u8 *p = ub + col;
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

__device__ __forceinline__ void st_u(uint8_t *ub_, uint32_t col, uint32_t al, uint32_t v) {
    g_u8 *ub = (g_u8 *)ub_;
    if (al == 0) {
        *(g_u32 *)(ub + col) = v;
    } else if (al == 2) {
        *(g_u16 *)(ub + col) = (uint16_t)v;
        *(g_u16 *)(ub + col + 2) = (uint16_t)(v >> 16);
    } else {
        g_u8 *p = ub + col;
        p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
    }
}

// Workgroup barrier for LDS-only hand-offs: waits for this wave's LDS operations, not for its
// global loads/stores (a __syncthreads() is a full fence and would drain vmcnt every plane).
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// XCD-aware block remap: blocks b and b+8 share an XCD (round-robin dispatch), so give each
// XCD a contiguous run of tiles; speed only, never correctness.
__device__ __forceinline__ uint32_t xcd_tile(uint32_t b, uint32_t nb) {
    const uint32_t full = nb & ~7u;
    if (b >= full) return b;
    return (b & 7u) * (full >> 3) + (b >> 3);
}

}  // namespace tec
