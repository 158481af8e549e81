// encode_r10.hip -- Clay(20,7,16) layered encode of 1 MB stripes, output in row-of-planes pieces:
// the production hot path of Slicer::encode (lib/slicer/src/slicer.rs:268-286 ->
// ClayCoder::encode, clay.rs:99-104; every object of 1 MB < L <= 100 MB has 1,000,000-byte
// stripes, sub-chunk 1,430 B), fused with distribute_chunks' rotation (slicer.rs:60-71).  Same
// algebra and plane order as encode_dma.hip; what differs is the
// shape of the stores.
//
// Why: the output is 77 % of the bytes.  Written as 1,430-byte rows (one per node and plane) every
// row boundary splits a 128-byte line between two stores issued a plane apart, and the encode's
// byte mix ran at 0.51-0.55 of HBM peak in load/store skeletons of that shape, against 0.63 with
// each node's ten consecutive planes (a "row" z0 of the plane grid, 14,300 contiguous bytes)
// stored as one piece (profiles/r03_enc_skeleton3.txt, r04_enc_skeleton4.txt).  Here one
// workgroup owns one stripe and walks it row by row:
//   * a loader wave DMAs each plane's 16 input rows (7 own, 9 partner) into a two-slot LDS ring,
//     two planes ahead, as encode_dma.hip does; odd planes are fetched from 2 bytes before the row
//     so every lane word sits on the absolute 4-byte grid of the slices;
//   * the six compute waves keep every output word of the row in VGPRs: 13 parity nodes x 10
//     planes (+ the level-2 pieces that finish a parked pair), column-1 pairs parked in place;
//   * at the row's end the words go through LDS (a transposition area of 7 pieces) and each
//     (node, row) leaves as one 14,300-byte piece, stored by one wave (14 x 1 KiB stores);
//   * the loader copies the 7 systematic pieces of the row straight from the object to the slices
//     (global -> global, 14,300 bytes each) while the row's planes stream through the ring.
// Level-2 rows read back rows of nodes 7..9 written by earlier rows' flushes: at the row boundaries
// 6|7, 7|8, 8|9 the loader issues the next row's first planes only after those stores have landed.
// One workgroup per CU (146 KB of LDS, <= 256 VGPRs); falls back to encode_dma.hip for stripes it
// does not cover (unaligned objects, a data end inside a dword, chunk filters).
#include "kernels.hpp"
#include "gf_dev.hpp"
#include "dev_io.hpp"
#include "enc_common.hpp"

namespace tec {
namespace r10 {

using enc::kQ;
using enc::pft3;
constexpr int K = 7;
constexpr int G = 6;                         // compute waves; the seventh wave is the loader
constexpr int kWaves = G + 1;
constexpr uint32_t SC = 1430, CS = 143000, PIECE = 10 * SC;
constexpr uint32_t RB = 90, RW = RB * 16;    // 16-byte blocks per image row, image row stride
constexpr uint32_t kPartBase = 7 * RW;       // 7 own rows, then 9 partner rows
constexpr uint32_t kSlot = 16 * RW;          // one plane image
constexpr uint32_t kTP = 14336;              // transposition area: stride per piece
constexpr int kTPieces = 7;                  // pieces per transposition batch
constexpr uint32_t kTBase = 2 * kSlot;
constexpr uint32_t kLds = kTBase + kTPieces * kTP;  // 146,432 B
static_assert(kLds <= 160 * 1024, "one workgroup per CU");
constexpr uint32_t kWords = 358;             // lane words per row (4 columns each)
constexpr uint32_t kFull = PIECE / 16;       // 893 whole 16-byte blocks of a piece, then 12 bytes
constexpr uint32_t kDrop = 0x80000000u;      // offset past every resource: the range check drops it
constexpr int kOwnInstr = 10, kPartInstr = 13, kDmaInstr = kOwnInstr + kPartInstr;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));

__device__ __forceinline__ u32x4 rsrc(const void *p, uint32_t nrec) {
    const uint64_t a = reinterpret_cast<uint64_t>(p);
    u32x4 r;
    r.x = __builtin_amdgcn_readfirstlane((uint32_t)a);
    r.y = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32) & 0xffffu);
    r.z = __builtin_amdgcn_readfirstlane(nrec);
    r.w = 0x00020000u;
    return r;
}

// One LDS-DMA piece (lane l's 16 bytes at voff + soff land at LDS lds + 16 l); inline asm so the
// compiler neither counts nor orders it: the loader waits with explicit vmcnt + barrier.
__device__ __forceinline__ void dma16(u32x4 rs, uint32_t voff, uint32_t soff, uint32_t lds) {
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
        "buffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
        : "=&s"(keep) : "v"(voff), "s"(rs), "s"(lds), "s"(soff) : "memory");
}

__device__ __forceinline__ uint32_t lds32(const uint8_t *p) { return *reinterpret_cast<const uint32_t *>(p); }
// m ? a : b for a wave-uniform all-ones / all-zeros mask, as one v_bfi_b32
__device__ __forceinline__ uint32_t bsel(uint32_t m, uint32_t a, uint32_t b) {
    m = __builtin_amdgcn_readfirstlane(m);
    return __builtin_amdgcn_bitop3_b32(m, a, b, 0xca);
}

// Barrier counts at a row's end, identical in the compute waves and the loader: two per
// transposition batch; then, before a level-2 row, one after the stores landed and one after the
// next row's first plane landed.
__device__ __forceinline__ int row_pieces(uint32_t z0) { return 13 + (z0 > (uint32_t)K ? (int)(z0 - K) : 0); }
__device__ __forceinline__ int row_batches(uint32_t z0) { return (row_pieces(z0) + kTPieces - 1) / kTPieces; }
__device__ __forceinline__ bool read_back_next(uint32_t z0) { return z0 + 1 >= (uint32_t)K && z0 + 1 < (uint32_t)kQ; }

// The lane's word v of plane s of the piece in transposition slot `slot` (piece bytes at
// kTBase + slot * kTP).  Odd planes start at 2 mod 4, so the word straddling planes s-1 | s of a
// piece takes its low half from word 357 of the even plane and its high half from word 0 of the
// odd one.
struct TPut {
    uint32_t addr;       // LDS address of kTBase + 4 * (lane word)
    uint32_t keep_even;  // nonzero: the lane writes its whole word on even planes (not word 357)
    uint32_t keep_odd;   // nonzero: ... on odd planes (not word 0)
    // One asm block, so the compiler sees no divergent control flow (branches here made it spill
    // the row's words): the lanes with the flag write the dword; the others, with exec flipped,
    // write their half (even plane: the low half; odd plane: the high half at + 2).
    template <int S>
    __device__ __forceinline__ void put(uint32_t slot, uint32_t v) const {
        constexpr int off = S * (int)SC - (S & 1) * 2;
        const uint32_t a = addr + slot * kTP;
        uint64_t save;
        if constexpr (S & 1)
            asm volatile(
                "s_mov_b64 %0, exec\n\tv_cmpx_ne_u32_e32 0, %1\n\t"
                "ds_write_b32 %2, %3 offset:%4\n\ts_xor_b64 exec, exec, %0\n\t"
                "ds_write_b16_d16_hi %2, %3 offset:%5\n\ts_mov_b64 exec, %0"
                : "=&s"(save) : "v"(keep_odd), "v"(a), "v"(v), "i"(off), "i"(off + 2) : "memory", "vcc");
        else
            asm volatile(
                "s_mov_b64 %0, exec\n\tv_cmpx_ne_u32_e32 0, %1\n\t"
                "ds_write_b32 %2, %3 offset:%4\n\ts_xor_b64 exec, exec, %0\n\t"
                "ds_write_b16 %2, %3 offset:%4\n\ts_mov_b64 exec, %0"
                : "=&s"(save) : "v"(keep_even), "v"(a), "v"(v), "i"(off) : "memory", "vcc");
    }
};

// One plane (z0, S) of a row.  Column-1 outputs stay in registers for the whole row: o[j][s] is
// node 10 + j at plane (z0, s), pairs parked in place.  Column-0 parity (nodes 7..9, row z0) and,
// at level 2, node z0's pieces finished by this row (rows 7..z0-1) are final when computed and go
// straight to transposition slots 0..2 and 3..4.
template <int S>
__device__ __forceinline__ void plane(const uint8_t *img, uint32_t z0, uint32_t (&o)[kQ][kQ], const TPut &T) {
    const bool lvl2 = z0 >= (uint32_t)K;
    uint32_t own[K], p9[9];
#pragma unroll
    for (int i = 0; i < K; i++) own[i] = lds32(img + i * RW);
#pragma unroll
    for (int i = 0; i < 9; i++) p9[i] = lds32(img + kPartBase + i * RW);
    // partner of data node i at plane (z0, S): node z0 at plane (i, S) -- the image's partner rows
    // skip plane z0 (level 1: the red node's own row); level 2: node z0's level-1 rows 0..6
    // (bit selects on wave-uniform masks: as ?: the compiler branched around the transforms, and
    // the branchy row body spilled)
    uint32_t u[K];
#pragma unroll
    for (int i = 0; i < K; i++) {
        const uint32_t mp = (lvl2 || (uint32_t)i < z0) ? ~0u : 0u, mr = (!lvl2 && (uint32_t)i == z0) ? ~0u : 0u;
        const uint32_t pp = bsel(mp, p9[i], p9[i > 0 ? i - 1 : 0]);
        u[i] = bsel(mr, own[i], pft3(own[i], pp));
    }
    uint32_t acc[20 - K];
    enc::mds7_slp<false>(u, acc);
    // column-0 parity (computed on either side of a uniform branch; the stores after it, so the
    // row body keeps one basic block per plane).  Level 1: node 7+r's C from its U and its
    // partner's known C (node z0 at plane (7+r, S)).  Level 2, i0 = z0 - 7: r < i0 pairs with
    // U(z0, (7+r, S)) parked by row 7+r (both C's final: node 7+r here, node z0's plane (7+r, S)
    // to slot 3+r); r == i0 is red; r > i0 parks U(7+r, (z0, S)) in its own place (finished by
    // row 7+r).  Slots 3, 4 take a word on every plane: where no pair finishes there, the row end
    // overwrites them with column-1 pieces.
    // Both levels' values are computed and one is selected: any branch in the row body (even a
    // uniform one) made the register allocator spill the row's column-1 words.
    uint32_t c0[3], xv[2];
    const uint32_t m2 = lvl2 ? ~0u : 0u, i0 = z0 - K;
#pragma unroll
    for (int r = 0; r < 3; r++) {
        const uint32_t l1 = mulc(kPft.t_u[1], acc[r]) ^ mulc(kPft.t_p[1], p9[6 + r]);
        uint32_t l2 = acc[r];
        if (r < 2) {
            const uint32_t us = p9[7 + r], tt = xt(us ^ acc[r]);
            l2 = bsel((uint32_t)r < i0 ? ~0u : 0u, acc[r] ^ tt, acc[r]);
            xv[r] = us ^ tt;
        }
        c0[r] = bsel(m2, l2, l1);
    }
#pragma unroll
    for (int r = 0; r < 3; r++) T.put<S>(r, c0[r]);
    T.put<S>(3, xv[0]);
    T.put<S>(4, xv[1]);
    // column 1 (nodes 10..19) within the row: pair (j, S), j < S, finishes now with U(10+S, (z0, j))
    // parked at step j in o[S][j]; j > S parks U(10+j, (z0, S)) in o[j][S]
#pragma unroll
    for (int j = 0; j < S; j++) {
        const uint32_t pu = o[S][j], u1 = acc[3 + j];
        const uint32_t tt = xt(u1 ^ pu);
        o[j][S] = u1 ^ tt;
        o[S][j] = pu ^ tt;
    }
    o[S][S] = acc[3 + S];
#pragma unroll
    for (int j = S + 1; j < kQ; j++) o[j][S] = acc[3 + j];
}

__global__ void __launch_bounds__(kWaves * 64, 1) enc_r10_kernel(EncArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    uint8_t *const lds8 = reinterpret_cast<uint8_t *>(lds);
    const uint32_t lds0 = __builtin_amdgcn_groupstaticsize();
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    const EncJob J = a.jobs[xcd_tile(blockIdx.x, gridDim.x)];
    const uint32_t slen = a.slice_len;
    // input: the stripe's data bytes (4-aligned, whole dwords: host-checked); the range check
    // supplies Slicer::encode's zero padding past them (slicer.rs:276-283)
    const uint32_t src_len = (uint32_t)J.src_len;
    const u32x4 rs_src = rsrc(J.src, src_len);
    const __amdgpu_buffer_rsrc_t rb_src =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(J.src), 0, (int)src_len, 0x00020000);
    const uint32_t dst_range = a.n * slen - J.dst_skew;  // < 2^31, host-checked
    const u32x4 rs_dst = rsrc(J.dst, dst_range);
    const __amdgpu_buffer_rsrc_t rb_dst = __builtin_amdgcn_make_buffer_rsrc(J.dst, 0, (int)dst_range, 0x00020000);
    uint32_t sl_lane = lane + J.rot;
    sl_lane = (sl_lane >= 20u ? sl_lane - 20u : sl_lane) * slen;
    auto slice_off = [&](uint32_t node) -> uint32_t { return __builtin_amdgcn_readlane(sl_lane, node); };

    // one 14,300-byte piece at piece offset `so` of resource rb from `dofs` of the slices: 14
    // store slots of 64 lanes x 16 bytes, the last block (12 bytes) as one dwordx3
    auto piece_off = [&](uint32_t i) -> uint32_t {
        const uint32_t b = 64u * i + lane;
        return b < kFull ? 16u * b : kDrop;
    };
    const uint32_t tail_off = (lane == kFull - 64u * 13u) ? 16u * kFull : kDrop;  // lane 61 of slot 13

    if (wv == (uint32_t)G) {
        // ---------------- loader ----------------
        uint32_t dvo[kDmaInstr];
#pragma unroll
        for (int i = 0; i < kDmaInstr; i++) {
            dvo[i] = kDrop;
            if (i < kOwnInstr) {
                const uint32_t b = 64u * i + lane, x = b / RB, j = b - x * RB;
                if (b < (uint32_t)K * RB) dvo[i] = x * CS + 16u * j;
            } else {
                const uint32_t b = 64u * (i - kOwnInstr) + lane, p = b / RB, j = b - p * RB;
                if (b < 9u * RB) dvo[i] = p * kQ * SC + 16u * j;
            }
        }
        // plane tp into ring slot (tp & 1): own rows from the input, partner rows node z0 at
        // planes (p, s), p != z0 -- the input chunk at level 1, node z0's slice at level 2;
        // odd planes from 2 bytes before each row (the absolute 4-byte grid)
        auto issue = [&](uint32_t tp) {
            const uint32_t nz0 = tp / kQ, ns = tp - nz0 * kQ, sh = (tp & 1u) * 2u;
            const uint32_t slot = (tp & 1u) * kSlot;
            const bool lvl2 = nz0 >= (uint32_t)K;
            const uint32_t so_own = __builtin_amdgcn_readfirstlane(tp * SC - sh);
            const uint32_t so_part = __builtin_amdgcn_readfirstlane(lvl2 ? slice_off(nz0) + ns * SC - sh
                                                                         : nz0 * CS + ns * SC - sh);
            const uint32_t skip_from = kQ * SC * nz0;
#pragma unroll
            for (int i = 0; i < kDmaInstr; i++) {
                // lanes past the region's last block are masked off (a range-dropped LDS-DMA lane
                // still writes zeros to its LDS destination)
                if (dvo[i] == kDrop) continue;
                if (i < kOwnInstr) {
                    dma16(rs_src, dvo[i], so_own, __builtin_amdgcn_readfirstlane(lds0 + slot + 1024u * i));
                } else {
                    const uint32_t vo = dvo[i] + (dvo[i] >= skip_from ? kQ * SC : 0u);
                    const uint32_t ld = __builtin_amdgcn_readfirstlane(lds0 + slot + kPartBase + 1024u * (i - kOwnInstr));
                    if (lvl2) dma16(rs_dst, vo, so_part, ld);
                    else dma16(rs_src, vo, so_part, ld);
                }
            }
        };
        issue(0);
        issue(1);
        asm volatile("s_waitcnt vmcnt(23)\n\ts_barrier" ::: "memory");  // plane 0 landed
#pragma unroll 1
        for (uint32_t z0 = 0; z0 < (uint32_t)kQ; z0++) {
            const bool hold = read_back_next(z0);  // next row reads this row's stores back
#pragma unroll 1
            for (uint32_t s = 0; s < (uint32_t)kQ; s++) {
                const uint32_t z = z0 * kQ + s;
                if (s < (uint32_t)K) {
                    // systematic piece (node s, row z0): object bytes to the slice as they are
                    const uint32_t so = s * CS + z0 * PIECE, dofs = slice_off(s) + z0 * PIECE;
                    u32x4 v[14];
#pragma unroll
                    for (int i = 0; i < 14; i++)
                        v[i] = __builtin_amdgcn_raw_buffer_load_b128(rb_src, (int)(i < 13 ? piece_off(i) : min(piece_off(i), 16u * kFull)), (int)so, 0);
#pragma unroll
                    for (int i = 0; i < 14; i++)
                        __builtin_amdgcn_raw_buffer_store_b128(v[i], rb_dst, (int)piece_off(i), (int)dofs, 2);
                    const u32x3 t3 = {v[13].x, v[13].y, v[13].z};
                    __builtin_amdgcn_raw_buffer_store_b96(t3, rb_dst, (int)tail_off, (int)dofs, 2);
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // plane z + 1 landed
                lds_barrier();                                      // B1 of plane z
                if (z + 2u < (uint32_t)(kQ * kQ) && !(hold && s >= 8u)) issue(z + 2u);
            }
            for (int b = 0; b < 2 * row_batches(z0); b++) lds_barrier();
            if (hold) {
                lds_barrier();  // the compute waves' stores of row z0 have landed
                issue((z0 + 1u) * kQ);
                issue((z0 + 1u) * kQ + 1u);
                asm volatile("s_waitcnt vmcnt(23)" ::: "memory");
                lds_barrier();  // plane (z0 + 1, 0) landed
            }
        }
        return;
    }

    // ---------------- compute waves ----------------
    asm volatile("s_barrier" ::: "memory");
    const uint32_t w = threadIdx.x < kWords ? threadIdx.x : kWords - 1u;  // words past the row alias the last
    TPut T;
    T.addr = lds0 + kTBase + 4u * w;
    T.keep_even = w != kWords - 1u;
    T.keep_odd = threadIdx.x != 0u;
    uint32_t o[kQ][kQ];
#pragma unroll 1
    for (uint32_t z0 = 0; z0 < (uint32_t)kQ; z0++) {
        const uint8_t *img0 = lds8 + 4u * w, *img1 = lds8 + kSlot + 4u * w;
#define R10_PLANE(S)                                  \
        plane<S>((S) & 1 ? img1 : img0, z0, o, T);    \
        lds_barrier();
        R10_PLANE(0) R10_PLANE(1) R10_PLANE(2) R10_PLANE(3) R10_PLANE(4)
        R10_PLANE(5) R10_PLANE(6) R10_PLANE(7) R10_PLANE(8) R10_PLANE(9)
#undef R10_PLANE
        // ---- row end: the pieces leave through the transposition area, 7 per batch ----
        // slots 0..2: nodes 7..9 (written during the row); 3..pre-1: node z0's rows 7.. (level 2);
        // then the column-1 pieces c = 0..9 (node 10 + c) in order
        const uint32_t pre = 3u + (z0 > (uint32_t)K ? z0 - K : 0u);
        const uint32_t first = kTPieces - pre;  // column-1 pieces in batch 0
        const int nb = row_batches(z0);
        for (int b = 0; b < nb; b++) {
#pragma unroll
            for (int c = 0; c < kQ; c++) {
                const uint32_t cb = (uint32_t)c < first ? 0u : 1u + ((uint32_t)c - first) / kTPieces;
                const uint32_t slot = (uint32_t)c < first ? pre + c : ((uint32_t)c - first) % kTPieces;
                if (cb != (uint32_t)b) continue;
                T.put<0>(slot, o[c][0]); T.put<1>(slot, o[c][1]); T.put<2>(slot, o[c][2]);
                T.put<3>(slot, o[c][3]); T.put<4>(slot, o[c][4]); T.put<5>(slot, o[c][5]);
                T.put<6>(slot, o[c][6]); T.put<7>(slot, o[c][7]); T.put<8>(slot, o[c][8]);
                T.put<9>(slot, o[c][9]);
            }
            lds_barrier();
            // store: the batch's pieces, piece 7b + q by wave (7b + q) % 6: 14 slots of 1 KiB + the
            // 12-byte tail each
            const uint32_t nq = min((uint32_t)kTPieces, (uint32_t)row_pieces(z0) - (uint32_t)(kTPieces * b));
            for (uint32_t q = 0; q < nq; q++) {
                if ((kTPieces * (uint32_t)b + q) % G != wv) continue;
                uint32_t node, row;
                if (b == 0 && q < 3u) {
                    node = K + q, row = z0;
                } else if (b == 0 && q < pre) {
                    node = z0, row = K + q - 3u;
                } else {
                    const uint32_t c = b == 0 ? q - pre : first + kTPieces * (b - 1) + q;
                    node = kQ + c, row = z0;
                }
                const uint32_t dofs = slice_off(node) + row * PIECE;
                const uint8_t *t = lds8 + kTBase + q * kTP;
#pragma unroll
                for (int i = 0; i < 14; i++) {
                    const uint32_t po = piece_off(i);
                    const u32x4 d = *reinterpret_cast<const u32x4 *>(t + (po == kDrop ? 16u * kFull : po));
                    __builtin_amdgcn_raw_buffer_store_b128(d, rb_dst, (int)po, (int)dofs, 2);
                    if (i == 13) {
                        const u32x3 t3 = {d.x, d.y, d.z};
                        __builtin_amdgcn_raw_buffer_store_b96(t3, rb_dst, (int)tail_off, (int)dofs, 2);
                    }
                }
            }
            lds_barrier();
        }
        if (read_back_next(z0)) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this row's pieces have landed
            lds_barrier();
            lds_barrier();  // the loader: the next row's first plane has landed
        }
    }
}

}  // namespace r10

bool encode_r10_supported(int n, int k, uint32_t sc) { return n == 20 && k == 7 && sc == r10::SC; }

hipError_t launch_encode_r10(const EncArgs &a, hipStream_t s) {
    if (a.njobs == 0) return hipSuccess;
    if (!encode_r10_supported((int)a.n, 7, a.sc) || a.njobs > 0x7fffffffu) return hipErrorInvalidValue;
    hipError_t e = ensure_dyn_lds(reinterpret_cast<const void *>(r10::enc_r10_kernel), r10::kLds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(r10::enc_r10_kernel, dim3(a.njobs), dim3(r10::kWaves * 64), r10::kLds, s, a);
    return hipGetLastError();
}

}  // namespace tec
