// dev_io.hpp -- sub-chunk word access for the Clay kernels.
//
// A "word" is 4 byte-columns of one sub-chunk (cols c..c+3).  Sub-chunks are sc bytes with
// sc = chunk_size/alpha, always even but only 2-aligned (sc = 1,430 for 1 MB stripes), so a
// word sits at an address that is 0 or 2 mod 4.  Aligned words move as one dword; the others as
// two 16-bit halves (never an unaligned dword).  The last word of a sub-chunk is shifted back
// to end at sc (it overlaps its neighbour; both lanes write identical bytes).  When sc == 2 a
// word carries only 2 columns.
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
    p.nc = sc >= 4 ? 4u : sc;
    const uint32_t c = w * 4u;
    p.c = c + p.nc <= sc ? c : sc - p.nc;
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

// XCD-aware block remap: blocks b and b+8 share an XCD (round-robin dispatch), so give each
// XCD a contiguous run of tiles; speed only, never correctness.
__device__ __forceinline__ uint32_t xcd_tile(uint32_t b, uint32_t nb) {
    const uint32_t full = nb & ~7u;
    if (b >= full) return b;
    return (b & 7u) * (full >> 3) + (b >> 3);
}

}  // namespace tec
