// encode_slab.hip -- Clay layered encode for the q = 10, t = 2 profiles (n = 20, d = k + 9),
// i.e. the production profile (20,7,16) (lib/core/src/encoding.rs:236-239) and the reference
// test profile (20,10,19).  Replaces ClayCoder::encode -> clay_codes::ClayCode::encode
// (lib/slicer/src/clay.rs:99-104) inside Slicer::encode's per-stripe loop (slicer.rs:268-286),
// fused with the rotation scatter `distribute_chunks` (slicer.rs:60-71).
//
// Algebra (encode = decode_layered with the parity nodes erased):
//   plane z = (z0, z1); nodes (x, y), y = 0 for nodes 0..9, y = 1 for nodes 10..19; data nodes
//   are x < K in column 0.  Column-0 couplings join planes of equal z1 (a "slab"), column-1
//   couplings join planes of equal z0.  Planes with z0 < K are decode level 1, z0 >= K level 2
//   (their column-0 coupling partners are level-1 parity C of the same slab).
//
// Work decomposition (MI355X): a workgroup = 10 waves; wave s owns slab z1 = s for 64
// consecutive 4-column words (one word per lane), and walks z0 = 0..9 in decode order, so every
// column-0 dependency stays in the wave's registers (the level-1 parity C it later needs, the
// level-2 pair values).  Column-1 pairs (node 10+j at (z0,s)) <-> (node 10+s at (z0,j)) cross
// slabs: each plane-row z0 the ten waves publish their ten column-1 uncoupled values into a
// double-buffered LDS tile [slab][node][lane] (51 KB) and read their nine partners after one
// barrier.  All waves do identical work every step (no idle level phases), the LDS budget
// admits 3 workgroups per CU, loads/stores of a wave are 256 contiguous bytes of one sub-chunk.
// Coefficients (generator, PFT) are constexpr: each GF product is a fixed XOR selection of
// xtime multiples, or a 2-bit v_perm lookup with SGPR tables for one-off heavy constants.
#include "kernels.hpp"
#include "gf_dev.hpp"
#include "dev_io.hpp"

namespace tec {

constexpr int kQ = 10;

template <int K>
struct SlabConst {
    uint8_t G[20][K];   // systematic generator (rows >= K used)
    uint8_t Gt[kQ][K];  // column-0 parity rows pre-scaled for level-1 type-1 recovery: t_u * G
};

template <int K>
constexpr SlabConst<K> make_slab_const() {
    SlabConst<K> rc{};
    const Mat g = rs_generator(K, 20);
    for (int r = 0; r < 20; r++)
        for (int x = 0; x < K; x++) rc.G[r][x] = g.v[r][x];
    for (int r = K; r < kQ; r++)
        for (int x = 0; x < K; x++) rc.Gt[r][x] = gf_mul(kPft.t_u[1], g.v[r][x]);
    return rc;
}

// MODE (ablation builds only, scripts/kbench.hip): bit0 = drop global stores, bit1 = replace
// GF arithmetic by plain XOR, bit2 = skip the column-1 LDS exchange.  Production uses MODE 0.
// MASKED: the stripe's data end is not dword aligned (only an object's last stripe, when its
// length is not a multiple of 4): words are masked per lane instead of relying on the range check.
template <int K, int MODE = 0, bool MASKED = false>
__global__ void __launch_bounds__(640, 4) enc_slab_kernel(EncArgs a) {
    constexpr SlabConst<K> RC = make_slab_const<K>();
    constexpr int NP0 = kQ - K;              // column-0 parity nodes
    constexpr int NX = NP0 > 0 ? NP0 : 1;
    __shared__ uint32_t E[2 * kQ * kQ * 64];  // [buf][slab][node j][lane]
    // thread-private carried values: XL[slab][r][x][lane] = level-1 column-0 parity C(K+r, (x, s)),
    // YL[slab][i][r][lane] = level-2 U(K+r, (K+i, s)); dynamic indices cost nothing in LDS
    __shared__ uint32_t XL[kQ * NX * K * 64];
    __shared__ uint32_t YL[kQ * NX * NX * 64];

    const int slab = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform
    const int lane = threadIdx.x & 63;
    // a workgroup never straddles stripes: the job (and every base address) is uniform, so
    // addressing is SGPR base + per-lane 32-bit column offset
    const uint32_t tile = xcd_tile(blockIdx.x, gridDim.x);
    const uint32_t job = tile / a.groups_per_stripe;
    const uint32_t grp = tile - job * a.groups_per_stripe;
    uint32_t w = grp * 64u + (uint32_t)lane;
    if (w >= a.words_per_stripe) w = a.words_per_stripe - 1;  // tail lanes redo the last word
    const EncJob J = a.jobs[job];
    const uint32_t col = w * 4u;
    const uint32_t cs = a.cs, sc = a.sc, slen = a.slice_len;
    // Buffer resources from wave-uniform values (32-bit offsets).  The input resource starts at
    // J.src rounded down to 4 bytes and ends exactly at the stripe's last data byte, so the
    // hardware range check returns the zero padding of Slicer::encode (slicer.rs:276-283) for every
    // dword past the data.  Each word is two aligned dwords + one v_alignbyte (uniform shift):
    // no branch on the load path, so no s_waitcnt is forced next to a load.
    const uint32_t src_len = (uint32_t)J.src_len;
    const uint32_t src_al = (uint32_t)reinterpret_cast<uintptr_t>(J.src) & 3u;
    // (gfx950 zeroes a dword that straddles num_records entirely, so the MASKED variant rounds
    // the range up to the dword holding the last data byte -- same page, always readable --
    // and clears the bytes past the data per lane.)
    const __amdgpu_buffer_rsrc_t rs_src = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t *>(J.src - src_al), 0, (int)(MASKED ? (src_len + src_al + 3u) & ~3u : src_len + src_al),
        0x00020000);
    // output range = the object's n slices as seen from this stripe's base (< 2^31, host-checked),
    // so an offset with bit 31 set is out of range and its store is dropped
    const __amdgpu_buffer_rsrc_t rs_dst =
        __builtin_amdgcn_make_buffer_rsrc(J.dst, 0, (int)(a.n * slen - J.dst_skew), 0x00020000);
    const uint32_t dst_al = (uint32_t)reinterpret_cast<uintptr_t>(J.dst) & 3u;

    // When sc = 2 mod 4 the last word of a sub-chunk has 2 columns: lanes holding it (only in the
    // stripe's last workgroup) store their high half at an out-of-range offset, which the buffer
    // range check drops.  Its loads read 2 bytes past the sub-chunk: harmless column garbage.
    const bool tail_wave = (sc & 3u) != 0 && grp + 1 == a.groups_per_stripe;  // uniform
    const bool tail_lane = col + 4u > sc;
    const uint32_t hi_skip = tail_lane ? 0x80000000u : 0u;
    auto out_st = [&](int r, uint32_t z, uint32_t v) {
        if constexpr (MODE & 1) {
            if (v == 0x12345678u) __builtin_amdgcn_raw_buffer_store_b32(v, rs_dst, (int)col, 0, 0);  // keep v live
            return;
        }
        uint32_t sl = (uint32_t)r + J.rot;
        sl = sl >= 20u ? sl - 20u : sl;
        const uint32_t off = sl * slen + z * sc;             // uniform
        const uint32_t al = (dst_al + off) & 3u;              // uniform
        const int vo = (int)(off + col);
        if (al == 0 && !tail_wave) {
            __builtin_amdgcn_raw_buffer_store_b32(v, rs_dst, vo, 0, 0);
        } else if (!(al & 1u)) {
            __builtin_amdgcn_raw_buffer_store_b16((uint16_t)v, rs_dst, vo, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b16((uint16_t)(v >> 16), rs_dst, (int)((uint32_t)(vo + 2) | hi_skip), 0, 0);
        } else {
            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)v, rs_dst, vo, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(v >> 8), rs_dst, vo + 1, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(v >> 16), rs_dst, (int)((uint32_t)(vo + 2) | hi_skip), 0, 0);
            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(v >> 24), rs_dst, (int)((uint32_t)(vo + 3) | hi_skip), 0, 0);
        }
    };
    auto in_word = [&](int x, uint32_t z) -> uint32_t {
        const uint32_t off = (uint32_t)x * cs + z * sc;       // uniform
        const uint32_t o = src_al + off + col;                // from the aligned base
        const uint32_t lo = __builtin_amdgcn_raw_buffer_load_b32(rs_src, (int)(o & ~3u), 0, 0);
        const uint32_t hi = __builtin_amdgcn_raw_buffer_load_b32(rs_src, (int)((o & ~3u) + 4u), 0, 0);
        uint32_t v = __builtin_amdgcn_alignbyte(hi, lo, o & 3u);
        if constexpr (MASKED) {
            const int rem = (int)src_len - (int)(off + col);
            const uint32_t keep = rem >= 4 ? 0xffffffffu : (rem <= 0 ? 0u : (1u << (8 * rem)) - 1u);
            v &= keep;
        }
        return v;
    };

    // Column-1: publish this plane's ten uncoupled values, then couple each with its partner
    // U(10+s, (z0, j)) published by slab j.  Red node (j == s): C = U.
    auto col1 = [&](const uint32_t *u1, int z0) {
        uint32_t *const buf = E + (z0 & 1) * (kQ * kQ * 64);
        if constexpr (!(MODE & 4)) {
#pragma unroll
            for (int j = 0; j < kQ; j++) buf[(slab * kQ + j) * 64 + lane] = u1[j];
            lds_barrier();
        }
        const uint32_t z = (uint32_t)(z0 * kQ + slab);
#pragma unroll
        for (int j = 0; j < kQ; j++) {
            uint32_t cval = u1[j];
            if (j != slab) {
                const uint32_t pu = (MODE & 4) ? u1[(j + 1) % kQ] : buf[(j * kQ + slab) * 64 + lane];
                cval = (j > slab) ? (mulc(kPft.c_u[1], u1[j]) ^ mulc(kPft.c_p[1], pu))
                                  : (mulc(kPft.c_u[0], u1[j]) ^ mulc(kPft.c_p[0], pu));
            }
            out_st(kQ + j, z, cval);
        }
    };

    auto xl = [&](int r, int x) -> uint32_t & { return XL[((slab * NX + r) * K + x) * 64 + lane]; };
    auto yl = [&](int i, int r) -> uint32_t & { return YL[((slab * NX + i) * NX + r) * 64 + lane]; };

    // ---------------- decode levels 1 (z0 < K) and 2 (z0 >= K), one plane per step ----------------
    // Loads of plane z0+1 are issued (unconditionally: every address is valid, out-of-range
    // ones read 0 without memory traffic) before plane z0 is computed, so the wait for them lands
    // a full plane of ALU work later.  No branch separates a load from its alignbyte.
    uint32_t own[K], part[kQ];
    auto load_plane = [&](int z0) {
        const uint32_t z = (uint32_t)(z0 * kQ + slab);
#pragma unroll
        for (int x = 0; x < K; x++) own[x] = in_word(x, z);
#pragma unroll
        for (int x = 0; x < kQ; x++) part[x] = in_word(z0, (uint32_t)(x * kQ + slab));  // C(z0,(x,s))
    };
    load_plane(0);
    for (int z0 = 0; z0 < kQ; z0++) {
        const uint32_t z = (uint32_t)(z0 * kQ + slab);
        uint32_t cown[K], cpart[kQ];
#pragma unroll
        for (int x = 0; x < K; x++) cown[x] = own[x];
#pragma unroll
        for (int x = 0; x < kQ; x++) cpart[x] = part[x];
        load_plane(z0 + 1 < kQ ? z0 + 1 : z0);
        if (z0 < K) {
            // ---- level 1: data partners are inputs; column-0 parity by type-1 recovery ----
            uint32_t u[K];
#pragma unroll
            for (int x = 0; x < K; x++) {
                out_st(x, z, cown[x]);  // systematic chunk -> its rotated slice
                if (x == z0) u[x] = cown[x];
                else u[x] = (x > z0) ? (mulc(kPft.u_c[1], cown[x]) ^ mulc(kPft.u_p[1], cpart[x]))
                                     : (mulc(kPft.u_c[0], cown[x]) ^ mulc(kPft.u_p[0], cpart[x]));
            }
            uint32_t acc[20 - K];
#pragma unroll
            for (int r = 0; r < 20 - K; r++) acc[r] = 0;
#pragma unroll
            for (int x = 0; x < K; x++) {
                if constexpr (MODE & 2) {
#pragma unroll
                    for (int r = K; r < 20; r++) acc[r - K] ^= u[x] + r;
                } else {
                    const Mult<7> mu(u[x]);
#pragma unroll
                    for (int r = K; r < 20; r++) acc[r - K] ^= mu.mul(r < kQ ? RC.Gt[r][x] : RC.G[r][x]);
                }
            }
            // column-0 parity (x = r >= K, not red at level 1): type-1 with partner C(z0, (r, s))
#pragma unroll
            for (int r = K; r < kQ; r++) {
                const uint32_t cval = acc[r - K] ^ mulc(kPft.t_p[1], cpart[r]);
                out_st(r, z, cval);
                xl(r - K, z0) = cval;
            }
            col1(acc + NP0, z0);
        } else if constexpr (NP0 > 0) {
            // ---- level 2: data partners are the level-1 column-0 parity C (registers) ----
            uint32_t u[K];
#pragma unroll
            for (int x = 0; x < K; x++) {
                out_st(x, z, cown[x]);
                const uint32_t p = xl(z0 - K, x);  // C(z0, (x, s)) from level 1
                u[x] = mulc(kPft.u_c[0], cown[x]) ^ mulc(kPft.u_p[0], p);  // x < K <= z0
            }
            uint32_t acc[20 - K];
#pragma unroll
            for (int r = 0; r < 20 - K; r++) acc[r] = 0;
#pragma unroll
            for (int x = 0; x < K; x++) {
                if constexpr (MODE & 2) {
#pragma unroll
                    for (int r = K; r < 20; r++) acc[r - K] ^= u[x] + r;
                } else {
                    const Mult<7> mu(u[x]);
#pragma unroll
                    for (int r = K; r < 20; r++) acc[r - K] ^= mu.mul(RC.G[r][x]);
                }
            }
#pragma unroll
            for (int r = K; r < kQ; r++)
                if (r == z0) out_st(r, z, acc[r - K]);  // red: C = U
#pragma unroll
            for (int r = 0; r < NP0; r++) yl(z0 - K, r) = acc[r];
            col1(acc + NP0, z0);
        }
    }
    if constexpr (NP0 > 0) {
        // column-0 pairs among level-2 planes: (K+r, (K+i, s)) <-> (K+i, (K+r, s))
#pragma unroll
        for (int i = 0; i < NP0; i++)
#pragma unroll
            for (int r = 0; r < NP0; r++) {
                if (r == i) continue;
                const uint32_t us = yl(i, r), up = yl(r, i);
                const uint32_t cval = (r > i) ? (mulc(kPft.c_u[1], us) ^ mulc(kPft.c_p[1], up))
                                              : (mulc(kPft.c_u[0], us) ^ mulc(kPft.c_p[0], up));
                out_st(K + r, (uint32_t)((K + i) * kQ + slab), cval);
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

hipError_t launch_encode_rows(int k, bool masked, const EncArgs &a, hipStream_t s) {
    if (a.njobs == 0) return hipSuccess;
    const uint64_t blocks = (uint64_t)a.njobs * a.groups_per_stripe;
    if (blocks > 0x7fffffffull) return hipErrorInvalidValue;
    const dim3 grid((uint32_t)blocks), block(640);
    switch (k * 2 + (masked ? 1 : 0)) {
        case 14: hipLaunchKernelGGL((enc_slab_kernel<7, 0, false>), grid, block, 0, s, a); break;
        case 15: hipLaunchKernelGGL((enc_slab_kernel<7, 0, true>), grid, block, 0, s, a); break;
        case 20: hipLaunchKernelGGL((enc_slab_kernel<10, 0, false>), grid, block, 0, s, a); break;
        case 21: hipLaunchKernelGGL((enc_slab_kernel<10, 0, true>), grid, block, 0, s, a); break;
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
