// encode_rows.hip -- Clay layered encode for the q = 10, t = 2 profiles (n = 20, d = k + 9),
// i.e. the production profile (20,7,16) (lib/core/src/encoding.rs:236-239) and the reference
// test profile (20,10,19).  Replaces ClayCoder::encode -> clay_codes::ClayCode::encode
// (lib/slicer/src/clay.rs:99-104) inside Slicer::encode's per-stripe loop (slicer.rs:268-286),
// fused with the rotation scatter `distribute_chunks` (slicer.rs:60-71).
//
// Algebra (encode = decode_layered with the parity nodes erased):
//   plane z = (z0, z1), nodes (x, y) with y = 0 for nodes 0..9 and y = 1 for nodes 10..19.
//   Data nodes are x < K in column 0.  Column-0 couplings join planes of equal z1 ("slab"),
//   column-1 couplings join planes of equal z0 ("row").  Planes with z0 < K form decode level 1,
//   z0 >= K level 2 (they need the level-1 parity C of column 0 as coupling partners).
//
// Work decomposition (MI355X): a workgroup = 10 waves, wave r owns row z0 = r for 64
// consecutive 4-column words (lanes).  Loads/stores of a wave are 256 contiguous bytes of one
// sub-chunk.  Everything a row needs stays in its wave; cross-row values go through LDS:
//   X  level-1 column-0 parity C, consumed by the level-2 rows (partners),
//   Y  level-2 column-0 uncoupled values (pairs between level-2 rows),
//   P  per-row pending column-1 uncoupled values (pairs inside the row), 25 reusable slots.
// LDS layout is [entry][lane] (dword per lane) so every access is bank-conflict free.
// Coefficients (generator, PFT) are constexpr: each GF product is a fixed XOR selection of
// xtime multiples, or a 2-bit v_perm lookup with SGPR tables for one-off heavy constants.
#include "kernels.hpp"
#include "gf_dev.hpp"
#include "dev_io.hpp"

namespace tec {

constexpr int kQ = 10;

template <int K>
struct RowConst {
    uint8_t G[20][K];   // systematic generator (rows >= K used)
    uint8_t Gt[kQ][K];  // column-0 parity rows pre-scaled for type-1 recovery: t_u * G
    int nslots;
};

struct SlotTab {
    int8_t s[kQ][kQ];   // pending slot of entry (a, b), a > b: U(node 10+a, plane (z0, b))
    int nslots;
};

constexpr SlotTab make_slots() {
    SlotTab t{};
    int owner_a[kQ * kQ] = {}, owner_b[kQ * kQ] = {};
    bool used[kQ * kQ] = {};
    int nslots = 0;
    for (int p = 0; p < kQ; p++) {
        // entries (p, b) are read at plane p, before this plane's writes (j-loop order) -> free
        for (int sidx = 0; sidx < kQ * kQ; sidx++)
            if (used[sidx] && owner_a[sidx] == p) used[sidx] = false;
        for (int j = p + 1; j < kQ; j++) {
            int sidx = 0;
            while (used[sidx]) sidx++;
            used[sidx] = true;
            owner_a[sidx] = j;
            owner_b[sidx] = p;
            t.s[j][p] = (int8_t)sidx;
            if (sidx + 1 > nslots) nslots = sidx + 1;
        }
    }
    (void)owner_b;
    t.nslots = nslots;
    return t;
}

inline constexpr SlotTab kSlotsHost = make_slots();
__constant__ SlotTab kSlots = make_slots();

template <int K>
constexpr RowConst<K> make_row_const() {
    RowConst<K> rc{};
    const Mat g = rs_generator(K, 20);
    for (int r = 0; r < 20; r++)
        for (int x = 0; x < K; x++) rc.G[r][x] = g.v[r][x];
    for (int r = K; r < kQ; r++)
        for (int x = 0; x < K; x++) rc.Gt[r][x] = gf_mul(kPft.t_u[1], g.v[r][x]);
    rc.nslots = kSlotsHost.nslots;
    return rc;
}

template <int K>
struct RowLds {
    static constexpr int NP0 = kQ - K;
    static constexpr int NX = NP0 * K * kQ;
    static constexpr int NY = NP0 * NP0 * kQ;
    static constexpr int NS = kSlotsHost.nslots;
    static constexpr int ENTRIES = NX + NY + kQ * NS;
};

template <int K>
__global__ void __launch_bounds__(640, 1) enc_rows_kernel(EncArgs a) {
    constexpr RowConst<K> RC = make_row_const<K>();
    using L = RowLds<K>;
    constexpr int NP0 = L::NP0;
    __shared__ uint32_t lds[L::ENTRIES * 64];
    uint32_t *const X = lds;
    uint32_t *const Y = lds + L::NX * 64;
    uint32_t *const P = lds + (L::NX + L::NY) * 64;

    const int row = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const uint32_t tile = xcd_tile(blockIdx.x, gridDim.x);
    uint64_t gw = (uint64_t)tile * 64u + lane;
    if (gw >= a.total_words) gw = a.total_words - 1;  // tail lanes redo the last word
    const uint32_t job = (uint32_t)(gw / a.words_per_stripe);
    const uint32_t w = (uint32_t)(gw - (uint64_t)job * a.words_per_stripe);
    const EncJob J = a.jobs[job];
    const WordPos wp = word_pos(w, a.sc);
    const uint32_t cs = a.cs, sc = a.sc, slen = a.slice_len;

    auto out_ptr = [&](int r, uint32_t z) -> uint8_t * {
        uint32_t sl = (uint32_t)r + J.rot;
        sl = sl >= 20u ? sl - 20u : sl;
        return J.dst + (uint64_t)sl * slen + (uint64_t)z * sc + wp.c;
    };
    auto in_word = [&](int x, uint32_t z) -> uint32_t {
        return ld_word(J.src, (uint64_t)x * cs + (uint64_t)z * sc + wp.c, J.src_len, wp.nc);
    };
    auto lref = [&](uint32_t *base, int e) -> uint32_t & { return base[e * 64 + lane]; };

    // Column-1 coupled values from the plane's uncoupled values acc[kQ-K .. 19-K]:
    // red node (j == z1) is copied; pairs (j, z1) <-> (z1, j) inside the row are resolved when
    // the second member is computed, the first waits in a pending LDS slot.
    auto col1 = [&](const uint32_t *acc, int z1) {
        const uint32_t z = (uint32_t)(row * kQ + z1);
#pragma unroll
        for (int j = 0; j < kQ; j++) {
            const uint32_t uj = acc[kQ + j - K];
            if (j == z1) {
                st_word(out_ptr(kQ + j, z), uj, wp.nc);
            } else if (j < z1) {
                const uint32_t pend = lref(P, row * L::NS + kSlots.s[z1][j]);  // U(10+z1, (z0, j))
                // C(10+j, (z0,z1)): self x=j < partner x=z1 -> orientation lo
                const uint32_t c1 = mulc(kPft.c_u[0], uj) ^ mulc(kPft.c_p[0], pend);
                // C(10+z1, (z0,j)): self x=z1 > partner x=j -> orientation hi
                const uint32_t c2 = mulc(kPft.c_u[1], pend) ^ mulc(kPft.c_p[1], uj);
                st_word(out_ptr(kQ + j, z), c1, wp.nc);
                st_word(out_ptr(kQ + z1, (uint32_t)(row * kQ + j)), c2, wp.nc);
            } else {
                lref(P, row * L::NS + kSlots.s[j][z1]) = uj;
            }
        }
    };

    if (row < K) {
        // ---------------- decode level 1: planes (z0 < K, z1) ----------------
        for (int z1 = 0; z1 < kQ; z1++) {
            const uint32_t z = (uint32_t)(row * kQ + z1);
            uint32_t u[K];
#pragma unroll
            for (int x = 0; x < K; x++) {
                const uint32_t own = in_word(x, z);
                st_word(out_ptr(x, z), own, wp.nc);  // systematic chunk -> its rotated slice
                if (x == row) {
                    u[x] = own;
                } else {
                    const uint32_t p = in_word(row, (uint32_t)(x * kQ + z1));  // C(z0, (x, z1))
                    u[x] = (x > row) ? (mulc(kPft.u_c[1], own) ^ mulc(kPft.u_p[1], p))
                                     : (mulc(kPft.u_c[0], own) ^ mulc(kPft.u_p[0], p));
                }
            }
            uint32_t acc[20 - K];
#pragma unroll
            for (int r = 0; r < 20 - K; r++) acc[r] = 0;
#pragma unroll
            for (int x = 0; x < K; x++) {
                const Mult<7> mu(u[x]);
#pragma unroll
                for (int r = K; r < 20; r++) acc[r - K] ^= mu.mul(r < kQ ? RC.Gt[r][x] : RC.G[r][x]);
            }
            // column-0 parity (x = r >= K, not red since z0 < K): type-1 from C(z0, (r, z1))
#pragma unroll
            for (int r = K; r < kQ; r++) {
                const uint32_t p = in_word(row, (uint32_t)(r * kQ + z1));
                const uint32_t cval = acc[r - K] ^ mulc(kPft.t_p[1], p);
                st_word(out_ptr(r, z), cval, wp.nc);
                lref(X, ((r - K) * K + row) * kQ + z1) = cval;
            }
            col1(acc, z1);
        }
    }
    if constexpr (K < kQ) {
        __syncthreads();
        if (row >= K) {
            // ---------------- decode level 2: planes (z0 >= K, z1) ----------------
            for (int z1 = 0; z1 < kQ; z1++) {
                const uint32_t z = (uint32_t)(row * kQ + z1);
                uint32_t u[K];
#pragma unroll
                for (int x = 0; x < K; x++) {
                    const uint32_t own = in_word(x, z);
                    st_word(out_ptr(x, z), own, wp.nc);
                    const uint32_t p = lref(X, ((row - K) * K + x) * kQ + z1);  // C(z0, (x, z1))
                    u[x] = mulc(kPft.u_c[0], own) ^ mulc(kPft.u_p[0], p);       // x < K <= z0
                }
                uint32_t acc[20 - K];
#pragma unroll
                for (int r = 0; r < 20 - K; r++) acc[r] = 0;
#pragma unroll
                for (int x = 0; x < K; x++) {
                    const Mult<7> mu(u[x]);
#pragma unroll
                    for (int r = K; r < 20; r++) acc[r - K] ^= mu.mul(RC.G[r][x]);
                }
#pragma unroll
                for (int r = K; r < kQ; r++) {
                    if (r == row) st_word(out_ptr(r, z), acc[r - K], wp.nc);  // red: C = U
                    else lref(Y, ((row - K) * NP0 + (r - K)) * kQ + z1) = acc[r - K];
                }
                col1(acc, z1);
            }
        }
        __syncthreads();
        if (row >= K) {
            // column-0 pairs between level-2 rows: (r, (z0,z1)) <-> (z0, (r,z1))
            for (int z1 = 0; z1 < kQ; z1++) {
#pragma unroll
                for (int r = K; r < kQ; r++) {
                    if (r == row) continue;
                    const uint32_t us = lref(Y, ((row - K) * NP0 + (r - K)) * kQ + z1);
                    const uint32_t up = lref(Y, ((r - K) * NP0 + (row - K)) * kQ + z1);
                    const uint32_t cval = (r > row) ? (mulc(kPft.c_u[1], us) ^ mulc(kPft.c_p[1], up))
                                                    : (mulc(kPft.c_u[0], us) ^ mulc(kPft.c_p[0], up));
                    st_word(out_ptr(r, (uint32_t)(row * kQ + z1)), cval, wp.nc);
                }
            }
        }
    }
}

__global__ void meta_kernel(const MetaJob *__restrict__ jobs, uint32_t njobs, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t per = n * 6u;
    if (i >= njobs * per) return;
    const uint32_t j = i / per, r = i - j * per, sl = r / 6u, wd = r - sl * 6u;
    uint8_t *p = jobs[j].dst + (uint64_t)sl * jobs[j].slice_len + 8u * wd;
    const uint64_t v = jobs[j].words[wd];
    if ((reinterpret_cast<uintptr_t>(p) & 7u) == 0) {
        *reinterpret_cast<uint64_t *>(p) = v;
    } else {
        for (int b = 0; b < 8; b++) p[b] = (uint8_t)(v >> (8 * b));
    }
}

bool encode_rows_supported(int n, int k, int d) { return n == 20 && d == k + 9 && (k == 7 || k == 10); }

hipError_t launch_encode_rows(int k, const EncArgs &a, hipStream_t s) {
    if (a.total_words == 0) return hipSuccess;
    const uint64_t blocks = (a.total_words + 63) / 64;
    if (blocks > 0x7fffffffull) return hipErrorInvalidValue;
    const dim3 grid((uint32_t)blocks), block(640);
    switch (k) {
        case 7: hipLaunchKernelGGL(enc_rows_kernel<7>, grid, block, 0, s, a); break;
        case 10: hipLaunchKernelGGL(enc_rows_kernel<10>, grid, block, 0, s, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_meta(const MetaJob *jobs, uint32_t njobs, uint32_t n, hipStream_t s) {
    if (!njobs) return hipSuccess;
    const uint32_t total = njobs * n * 6u;
    hipLaunchKernelGGL(meta_kernel, dim3((total + 255) / 256), dim3(256), 0, s, jobs, njobs, n);
    return hipGetLastError();
}

}  // namespace tec
