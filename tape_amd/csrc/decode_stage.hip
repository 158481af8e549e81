// decode_stage.hip -- layered Clay decode for q = 10, t = 2 profiles (n = 20): ClayCoder::decode
// (lib/slicer/src/clay.rs:106-122 -> clay_codes decode) inside Slicer::decode's per-stripe loop
// (slicer.rs:333-361), any erasure pattern of at most n - k nodes.
//
// The host compiles each erasure pattern into a 100-step program (ClayHost::dec_prog): planes row
// by row, and per plane which known node uncouples against what (an input row, or a C recovered
// earlier), which erased U's the MDS solve must produce, and what becomes of them (a data row
// written out, a type-1 C, or a pair's U parked for the pair's later plane).  The kernel follows it:
//   * a workgroup owns one stripe's row segment (G <= 6 waves x 64 lanes x 4 columns); a lane
//     owns one 4-column word of every plane, so every parked value is lane-private: an LDS slot
//     when its consumer is in the same row, a per-stripe global scratch row otherwise;
//   * loads are one dword per lane down each slice row (coalesced), one plane ahead; the MDS
//     solve uses the pattern's decoding matrix as v_perm tables (scalar-loaded);
//   * recovered and copied data rows are staged in LDS and written whole by one wave each.
#include "kernels.hpp"
#include "gf_dev.hpp"
#include "dev_io.hpp"

namespace tec {
namespace dstage {

// measurement-only ablations (never in a shipped build): bit 0 no scratch loads, bit 1 no MDS
// products, bit 2 no flush stores, bit 3 no input loads, bit 4 no barrier and no flush
#ifndef TEC_DEC_ABLATE
#define TEC_DEC_ABLATE 0
#endif
#ifndef TEC_DEC_PRIO
#define TEC_DEC_PRIO 0  // wave priority during a step's compute (s_setprio), 0 = off
#endif
#ifndef TEC_DEC_ST_AUX
#define TEC_DEC_ST_AUX 2  // cache policy of the output row stores (2 = nt: ~1 % faster)
#endif
#ifndef TEC_DEC_COND_LD
#define TEC_DEC_COND_LD 0  // 1: issue only the loads a step uses (uniform branches); 0: every slot, range-dropped
#endif
#ifndef TEC_DEC_DIRECT
#define TEC_DEC_DIRECT 1  // 1: decoded words stored straight to the data chunks (no staging rows, no barrier)
#endif
#ifndef TEC_DEC_WPE
#define TEC_DEC_WPE 4  // waves per SIMD the register budget is cut for
#endif
#ifndef TEC_DEC_MAXG
#define TEC_DEC_MAXG 2  // waves per workgroup at most (direct output: 2 measured best, 6 -> 2: 7.48 -> 5.95 ms)
#endif
#ifndef TEC_DEC_LATE_LD
#define TEC_DEC_LATE_LD 1  // 1: a step's loads for the next step issued after its own are consumed (r04: random 5.47 vs 5.52-5.55 ms, recover 3.89 vs 3.94-3.96; 115 VGPRs instead of 127); 0: at the step's start
#endif
#ifndef TEC_DEC_OWN_AUX
#define TEC_DEC_OWN_AUX 2  // known rows' own loads non-temporal (r05 A/B: random 5.41-5.44 vs 5.49-5.53 ms, recover neutral; partner loads nt: neutral / worse)
#endif
#ifndef TEC_DEC_PART_AUX
#define TEC_DEC_PART_AUX 0
#endif
#ifndef TEC_DEC_WPL
#define TEC_DEC_WPL 1  // words per lane: each lane decodes WPL words (columns 4w.. of WPL row segments) with one step's control
#endif
#ifndef TEC_DEC_WPE_WIDE
#define TEC_DEC_WPE_WIDE 2  // waves per SIMD the register budget is cut for when WPL > 1
#endif
#ifndef TEC_DEC_TAB_LDS
#define TEC_DEC_TAB_LDS 0  // 1: v_perm tables staged in LDS (broadcast reads; r04 A/B: random 5.52 vs 5.51 ms, recover 4.12 vs 3.93); 0: scalar-loaded
#endif
constexpr int kMaxG = TEC_DEC_MAXG;
constexpr int kWpl = TEC_DEC_WPL;
static_assert(kWpl >= 1 && kWpl <= 2 && (kWpl == 1 || TEC_DEC_DIRECT), "WPL > 1 needs direct output");
constexpr uint32_t kTabDw = 8;  // LDS dwords per v_perm table (5 used; 32-byte aligned for one b128 + one b32 read)
__host__ __device__ constexpr uint32_t tab_lds_bytes(int nk) { return TEC_DEC_TAB_LDS ? (uint32_t)(2 * kRepQ - nk) * nk * kTabDw * 4u : 0u; }
constexpr uint32_t kMaxLdsRows = 64;  // 2 x staging + zero + trash + slots (G = 6: 96 KB)

// PFT of the supported profiles: U = 3 C ^ 2 Cp = C ^ xt(C ^ Cp), and the inverse has the same
// form (C = 3 U ^ 2 Up); type-1 C = t_u (U ^ Cp) ^ Cp.
__device__ __forceinline__ uint32_t pft3(uint32_t a, uint32_t b) { return a ^ xt(a ^ b); }
static_assert(kPft.u_c[0] == 3 && kPft.u_p[0] == 2 && kPft.c_u[0] == 3 && kPft.c_p[0] == 2 &&
              kPft.u_c[1] == 3 && kPft.u_p[1] == 2 && kPft.c_u[1] == 3 && kPft.c_p[1] == 2, "PFT");
static_assert(kPft.t_u[0] == kPft.t_u[1] && kPft.t_p[0] == kPft.t_p[1] && (kPft.t_u[0] ^ kPft.t_p[0]) == 1,
              "type-1 C = t (U ^ Cp) ^ Cp");

template <int NK, int G, int WPL = kWpl>
__global__ void __launch_bounds__(G * 64, WPL > 1 ? TEC_DEC_WPE_WIDE : TEC_DEC_WPE) dec_stage_kernel(DecArgs a) {
    constexpr int NE = 2 * kRepQ - NK;  // padded patterns: every other node erased
    // a lane owns WPL words: word k of lane t is column group (seg * WPL + k) * G * 64 + t, so each
    // load instruction still reads G * 256 contiguous bytes; LDS slot rows and scratch rows hold
    // the WPL word groups side by side (RSW bytes each)
    constexpr uint32_t RSW = G * 256u, RS = RSW * WPL;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    uint8_t *const lds8 = reinterpret_cast<uint8_t *>(lds);
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t col_local = threadIdx.x * 4u;

    const uint32_t tile = xcd_tile(blockIdx.x, gridDim.x);
    const uint32_t job = tile / a.wgs_per_stripe, seg = tile - job * a.wgs_per_stripe;
    typedef const __attribute__((address_space(4))) GpeJob cJob;
    typedef const __attribute__((address_space(4))) DecProgHdr cHdr;
    typedef const __attribute__((address_space(4))) uint32_t cU32;
    cJob &J = *(cJob *)(uintptr_t)(a.jobs + job);
    cHdr &H = *(cHdr *)(uintptr_t)(a.hdrs + J.pattern);
    const DecStepP *prog = a.steps + ((cU32 *)(uintptr_t)a.step_off)[J.pattern];
    const uint32_t sc = a.sc, wps = a.words_per_stripe;
    const uint32_t seg0 = seg * RS, lseg = min(RS, sc - seg0);
    // a word whose high half lies past the sub-chunk (sc = 2 mod 4) loads the dword 2 bytes
    // earlier and rotates: the last row of the last slice may end the buffer
    uint32_t vcol[WPL], vsh[WPL];
#pragma unroll
    for (int k = 0; k < WPL; k++) {
        uint32_t w = (seg * WPL + k) * G * 64u + threadIdx.x;
        if (w >= wps) w = wps - 1;  // words past the stripe alias the last (same values, same bytes)
        const uint32_t col = w * 4u;
        const bool tailw = col + 4u > sc;
        vcol[k] = tailw ? col - 2u : col;
        vsh[k] = tailw ? 2u : 0u;
    }
    const uint32_t in_range = (uint32_t)(a.n * a.in_stride);  // host-checked < 2^31
    const __amdgpu_buffer_rsrc_t rs_in = __builtin_amdgcn_make_buffer_rsrc((void *)J.in, 0, (int)in_range, 0x00020000);
    // data chunk x at out + x * out_stride, trimmed to the stripe's share of the object
    const __amdgpu_buffer_rsrc_t rs_out = __builtin_amdgcn_make_buffer_rsrc((void *)J.out, 0, (int)(uint32_t)J.out_len, 0x00020000);
    uint8_t *const scr = a.scratch + (size_t)tile * a.nscratch_max * RS;
    const __amdgpu_buffer_rsrc_t rs_scr = __builtin_amdgcn_make_buffer_rsrc(scr, 0, (int)(a.nscratch_max * RS), 0x00020000);
    // input slice byte offset of internal node i (= shard i, nu = 0) in lane i, rotated
    uint32_t sl_lane = lane + J.rot;
    sl_lane = (sl_lane >= a.n ? sl_lane - a.n : sl_lane) * (uint32_t)a.in_stride;
    uint32_t kbase[NK];  // the known nodes' slices
#pragma unroll
    for (int j = 0; j < NK; j++) kbase[j] = __builtin_amdgcn_readlane(sl_lane, H.knode[j]);
    // raw input word (the tail-word rotation is applied where the value is consumed, so a load
    // inside a branch has no use inside it)
    // cache policy of the known rows' own loads / partner loads (measurement variants)
    auto ldraw = [&](uint32_t so, int k) -> uint32_t {
        if (TEC_DEC_ABLATE & 8) return so;
        return __builtin_amdgcn_raw_buffer_load_b32(rs_in, (int)vcol[k], (int)so, TEC_DEC_OWN_AUX);
    };
    auto ldopt = [&](uint32_t so, int k) -> uint32_t {
        if (TEC_DEC_ABLATE & 8) return so;
        return (TEC_DEC_COND_LD && so == 0x80000000u)
                   ? 0u
                   : __builtin_amdgcn_raw_buffer_load_b32(rs_in, (int)vcol[k], (int)so, TEC_DEC_PART_AUX);
    };
    // staged rows need each word's bytes in column order (the tail lane's load rotated); direct
    // output stores every word back where it was loaded, and all the arithmetic is byte-wise, so
    // the loaded order is kept throughout
    auto rot = [&](uint32_t v, int k) { return TEC_DEC_DIRECT ? v : __builtin_amdgcn_alignbyte(v, v, vsh[k]); };
    // LDS rows: two staging buffers of max_out rows (a step stages into buffer st & 1, so one
    // barrier per step suffices), a zero row, a trash row, then the lane-private slots
    const uint32_t mo = TEC_DEC_DIRECT ? 0u : H.max_out, zrow = 2u * mo, trow = zrow + 1u, srow0 = zrow + 2u;
    auto lds_at = [&](uint32_t off, int k) -> uint32_t * {
        return reinterpret_cast<uint32_t *>(lds8 + off + (uint32_t)k * RSW + col_local);
    };
#pragma unroll
    for (int k = 0; k < WPL; k++) *lds_at(zrow * RS, k) = 0u;  // lane-private: read back only by this lane
    // flush: staging row i -> data chunk x at the item's plane, the whole row by one wave
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const uint32_t nb = lseg >> 4, tail = lseg & 15u;
    constexpr uint32_t kDrop = 0x80000000u;
    const bool wide_tail = tail != 0 && nb > 0;
    auto blk_off = [&](uint32_t b) -> uint32_t {
        return b < nb ? b * 16u : ((wide_tail && b == nb) ? lseg - 16u : kDrop);
    };
    // the stripe's output share ends at out_len, possibly inside a data row (the last chunk's
    // padding, or the next stripe's share): a block across that end is written byte by byte
    const uint32_t olen = (uint32_t)J.out_len;
    auto flush16 = [&](const uint8_t *row, uint32_t b, uint32_t off) {  // block b of the row
        const uint32_t vo = blk_off(b), lo = vo == kDrop ? 0u : vo;
        const u32x4 v = *reinterpret_cast<const u32x4 *>(row + lo);
        if (vo == kDrop || off + vo + 16u <= olen) {
            __builtin_amdgcn_raw_buffer_store_b128(v, rs_out, (int)vo, (int)off, TEC_DEC_ST_AUX);
        } else {
#pragma unroll
            for (uint32_t b = 0; b < 16u; b++)  // bytes past out_len fail the range check
                __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(v[b >> 2] >> (8u * (b & 3u))), rs_out, (int)(vo + b), (int)off, 0);
        }
    };

    // Step control words in VGPRs: a step's 48 words in lanes 0..47 of one VGPR, loaded two
    // steps ahead (vmcnt waits are in order).  Every per-word quantity (load offsets, LDS row
    // offsets, scratch offsets) is derived for all words at once in vector code and read out with
    // v_readlane, so the step needs no per-field scalar decoding or branches.  The decoding matrix
    // (NE x NK v_perm tables, 1.5 KB per pattern) is scalar-loaded per erased row: its loads
    // depend on nothing and stay in the scalar cache.
    typedef const __attribute__((address_space(4))) PermTab cPermTab;
    cPermTab(*D)[kGpeMaxKnown] = (cPermTab(*)[kGpeMaxKnown])(uintptr_t)(&a.patterns[J.pattern].D[0][0]);
    // TEC_DEC_TAB_LDS: the NE x NK tables copied once into LDS after the rows (kTabDw dwords each);
    // a product then reads its table with one broadcast b128 + b32 LDS read into VGPRs, so the
    // v_perm needs no v_mov of an SGPR table half (the scalar-loaded form pays 2 per product:
    // gfx9 VALU reads one SGPR per instruction) and the step waits on no scalar load
    const uint32_t tab_dw = (a.lds_rows * RS) >> 2;
    if constexpr (TEC_DEC_TAB_LDS != 0) {
        const uint32_t *Dw = reinterpret_cast<const uint32_t *>(&a.patterns[J.pattern].D[0][0]);
        for (uint32_t i = threadIdx.x; i < (uint32_t)(NE * NK * 5); i += G * 64u) {
            const uint32_t e = i / (NK * 5), r = i - e * (NK * 5), j = r / 5u, t = r - j * 5u;
            lds[tab_dw + (e * NK + j) * kTabDw + t] = Dw[(e * kGpeMaxKnown + j) * 5u + t];
        }
        __syncthreads();
    }
    // one 32-bit lane offset into a buffer over the pattern's steps (a per-lane 64-bit pointer
    // held two more VGPRs across the loop and spilled with the LDS tables)
    const __amdgpu_buffer_rsrc_t rs_prog = __builtin_amdgcn_make_buffer_rsrc((void *)prog, 0, (int)((H.nsteps + 2) * sizeof(DecStepP)), 0x00020000);
    const uint32_t progl = (lane < kDpWords ? lane : 0u) * 4u;
    auto ldw = [&](uint32_t st) -> uint32_t {
        return __builtin_amdgcn_raw_buffer_load_b32(rs_prog, (int)progl, (int)(st * (uint32_t)sizeof(DecStepP)), 0);
    };
    auto W = [](uint32_t v, int i) -> uint32_t { return __builtin_amdgcn_readlane(v, i); };
    const bool kd_l = lane >= kDpKd && lane < kDpKd + NK, ed_l = lane >= kDpEd && lane < kDpEd + NE;
    // input offset of the partner load word x describes (known input partner, type-1 partner)
    auto vec_in = [&](uint32_t x) -> uint32_t {
        const uint32_t k = x >> 28;
        const bool on = (kd_l && k == kKnInput) || (ed_l && k == kErType1);
        uint32_t sl_l = lane + J.rot;  // sl_lane, recomputed (not held across the loop)
        sl_l = (sl_l >= a.n ? sl_l - a.n : sl_l) * (uint32_t)a.in_stride;
        const uint32_t sl = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((x & 0xffu) << 2), (int)sl_l);
        return on ? sl + ((x >> 8) & 0xffu) * sc : kDrop;
    };
    // a consumed location (known partner C, pair partner U): scratch offset or kDrop ...
    auto consumed = [&](uint32_t x, uint32_t ty) {
        const uint32_t k = x >> 28;
        return ((kd_l && k == kKnLoc) || (ed_l && k == kErFinish)) && ((x >> 8) & 3u) == ty;
    };
    auto vec_scr = [&](uint32_t x) -> uint32_t { return consumed(x, kLocScratch) ? (x & 0xffu) * RS : kDrop; };
    // ... and its LDS row (the zero row unless a slot)
    auto vec_slot = [&](uint32_t x) -> uint32_t { return (consumed(x, kLocSlot) ? srow0 + (x & 0xffu) : zrow) * RS; };
    // a produced value's 10-bit location -> LDS row offset (trash row for none / scratch)
    auto dst_lds = [&](uint32_t f, uint32_t sbase) -> uint32_t {
        const uint32_t ty = (f >> 8) & 3u, ix = f & 0xffu;
        const uint32_t row = (f & 0x3ffu) == kLoc10None ? trow
                             : ty == kLocStage    ? (TEC_DEC_DIRECT ? trow : sbase + ix)
                             : ty == kLocSlot     ? srow0 + ix
                                                  : trow;
        return row * RS;
    };
    auto dst_scr = [&](uint32_t f) -> uint32_t {
        return ((f & 0x3ffu) != kLoc10None && ((f >> 8) & 3u) == kLocScratch) ? (f & 0xffu) * RS : kDrop;
    };

    // direct mode: a staged destination's data chunk and plane (the step's flush item), as the
    // row's byte offset in the stripe's output, or kDrop
    auto vec_out = [&](uint32_t f, uint32_t w) -> uint32_t {
        const uint32_t ix = f & 0xffu;
        const uint32_t iw = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((kDpOut + (ix >> 1)) << 2), (int)w);
        const uint32_t it = (iw >> (16u * (ix & 1u))) & 0xffffu;
        const bool st = (f & 0x3ffu) != kLoc10None && ((f >> 8) & 3u) == kLocStage;
        return st ? (it & 0xffu) * (uint32_t)a.out_stride + (it >> 8) * sc : kDrop;
    };
    // one decoded word (in the lane's load order) to its row at `off` (uniform), at the lane's
    // load column vcol; a row across the stripe's output share is written byte by byte there
    auto put_out = [&](uint32_t off, uint32_t wv_, int k) {
        if (off == kDrop) return;
        if (off + sc <= olen) {
            __builtin_amdgcn_raw_buffer_store_b32(wv_, rs_out, (int)vcol[k], (int)off, TEC_DEC_ST_AUX);
        } else {
#pragma unroll
            for (uint32_t b = 0; b < 4u; b++)  // bytes past out_len fail the range check
                __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(wv_ >> (8u * b)), rs_out, (int)(vcol[k] + b), (int)off, 0);
        }
    };

    uint32_t own[WPL][NK], part[WPL][NK], tkp[WPL][NE];
    auto load_known = [&](uint32_t x) {
        const uint32_t zs = (W(x, kDpHdr) & 0xffu) * sc;
        const uint32_t vin = vec_in(x);
#pragma unroll
        for (int j = 0; j < NK; j++) {
            const uint32_t so = W(vin, kDpKd + j);
#pragma unroll
            for (int k = 0; k < WPL; k++) {
                own[k][j] = ldraw(kbase[j] + zs, k);
                part[k][j] = ldopt(so, k);
            }
        }
    };
    auto load_tkp = [&](uint32_t x) {
        const uint32_t vin = vec_in(x);
#pragma unroll
        for (int e = 0; e < NE; e++) {
            const uint32_t so = W(vin, kDpEd + e);
#pragma unroll
            for (int k = 0; k < WPL; k++) tkp[k][e] = ldopt(so, k);
        }
    };
    auto load_step = [&](uint32_t x) {
        load_known(x);
        load_tkp(x);
    };
    // scratch loads of a step, issued after the previous step's scratch stores (lane-private
    // addresses: program order within the lane is the only ordering needed)
    uint32_t ksc[WPL][NK], esc[WPL][NE];
    auto load_scr = [&](uint32_t x) {
        const uint32_t vs = vec_scr(x);
        if (TEC_DEC_ABLATE & 1) {
            for (int k = 0; k < WPL; k++) {
                for (int j = 0; j < NK; j++) ksc[k][j] = 0;
                for (int e = 0; e < NE; e++) esc[k][e] = 0;
            }
            return;
        }
        auto ld = [&](uint32_t so, int k) -> uint32_t {
            return (TEC_DEC_COND_LD && so == 0x80000000u)
                       ? 0u
                       : __builtin_amdgcn_raw_buffer_load_b32(rs_scr, (int)(col_local + (uint32_t)k * RSW), (int)so, 0);
        };
#pragma unroll
        for (int j = 0; j < NK; j++) {
            const uint32_t so = W(vs, kDpKd + j);
#pragma unroll
            for (int k = 0; k < WPL; k++) ksc[k][j] = ld(so, k);
        }
#pragma unroll
        for (int e = 0; e < NE; e++) {
            const uint32_t so = W(vs, kDpEd + e);
#pragma unroll
            for (int k = 0; k < WPL; k++) esc[k][e] = ld(so, k);
        }
    };

    const uint32_t nsteps = H.nsteps;
    uint32_t w_cur = ldw(0), w_nxt = ldw(1);  // steps nsteps, nsteps + 1 are blank
    load_step(w_cur);
    load_scr(w_cur);
    for (uint32_t st = 0; st < nsteps; st++) {
        const uint32_t w_nn = ldw(st + 2);
        uint32_t cown[WPL][NK], cpart[WPL][NK], ctkp[WPL][NE];
#pragma unroll
        for (int k = 0; k < WPL; k++) {
#pragma unroll
            for (int j = 0; j < NK; j++) cown[k][j] = rot(own[k][j], k), cpart[k][j] = rot(part[k][j], k);
#pragma unroll
            for (int e = 0; e < NE; e++) ctkp[k][e] = rot(tkp[k][e], k);
        }
        if constexpr (!TEC_DEC_LATE_LD) load_step(w_nxt);  // blank step: every partner load dropped
        if constexpr (TEC_DEC_PRIO) __builtin_amdgcn_s_setprio(TEC_DEC_PRIO);
        // ---- uncouple the known nodes: dropped loads read 0, a non-slot partner reads the zero
        // row, a red node masks the PFT term ----
        const uint32_t vsl = vec_slot(w_cur);
        Sel sel[WPL][NK];
#pragma unroll
        for (int j = 0; j < NK; j++) {
            const uint32_t mred = (W(w_cur, kDpKd + j) >> 28) == kKnRed ? 0u : ~0u;
            const uint32_t sl_off = W(vsl, kDpKd + j);
#pragma unroll
            for (int k = 0; k < WPL; k++) {
                const uint32_t p = cpart[k][j] ^ ksc[k][j] ^ *lds_at(sl_off, k);
                sel[k][j] = Sel(cown[k][j] ^ (xt(cown[k][j] ^ p) & mred));
            }
        }
        // known data rows: copies (staging is double-buffered, so any time in the step)
        const uint32_t sbase = (st & 1u) * mo;
        {
            if (TEC_DEC_DIRECT) {
                const uint32_t ok = vec_out(w_cur >> 16, w_cur);
#pragma unroll
                for (int j = 0; j < NK; j++) {
                    const uint32_t o = W(ok, kDpKd + j);
#pragma unroll
                    for (int k = 0; k < WPL; k++) put_out(o, cown[k][j], k);
                }
            } else {
                const uint32_t lk = dst_lds(w_cur >> 16, sbase);
#pragma unroll
                for (int j = 0; j < NK; j++) *lds_at(W(lk, kDpKd + j), 0) = cown[0][j];
            }
        }
        // TEC_DEC_LATE_LD: the next step's known-row loads once this step's are consumed (no second
        // register set for them), its type-1 partner loads after the writes below
        if constexpr (TEC_DEC_LATE_LD != 0) load_known(w_nxt);
        // pair partners' U (read before this step's writes: a location may be rewritten from its
        // consumer step on)
        uint32_t pu[WPL][NE];
#pragma unroll
        for (int e = 0; e < NE; e++) {
            const uint32_t sl_off = W(vsl, kDpEd + e);
#pragma unroll
            for (int k = 0; k < WPL; k++) pu[k][e] = esc[k][e] ^ *lds_at(sl_off, k);
        }
        // ---- MDS-solve the erased U's the program needs ----
        uint32_t acc[WPL][NE];
#pragma unroll
        for (int e = 0; e < NE; e++) {
#pragma unroll
            for (int k = 0; k < WPL; k++) acc[k][e] = 0;
            if ((W(w_cur, kDpEd + e) >> 28) == kErSkip) continue;
            if (TEC_DEC_ABLATE & 2) {
#pragma unroll
                for (int k = 0; k < WPL; k++)
#pragma unroll
                    for (int j = 0; j < NK; j++) acc[k][e] ^= sel[k][j].s0 + e;
                continue;
            }
            // known inputs in pairs: 3 perms and 1.5 XOR3 per product, plus a v_mov per 3-bit perm
            // when both table halves are SGPRs (one SGPR operand per VALU instruction on gfx9; the
            // tables in LDS instead, one broadcast ds_read_b128 per product, measured 30 % slower);
            // the WPL words of a lane share each table
            if constexpr (TEC_DEC_TAB_LDS != 0) {
                const uint32_t *tr = lds + tab_dw + (uint32_t)e * NK * kTabDw;
                auto tq = [&](int j) { return *reinterpret_cast<const u32x4 *>(tr + j * kTabDw); };
#pragma unroll
                for (int j = 0; j + 1 < NK; j += 2) {
                    const u32x4 p = tq(j), q = tq(j + 1);
                    const uint32_t p4 = tr[j * kTabDw + 4], q4 = tr[(j + 1) * kTabDw + 4];
#pragma unroll
                    for (int k = 0; k < WPL; k++)
                        acc[k][e] = perm_mul2_acc(acc[k][e], sel[k][j], p.x, p.y, p.z, p.w, p4, sel[k][j + 1], q.x, q.y,
                                                  q.z, q.w, q4);
                }
                if (NK & 1) {
                    const u32x4 p = tq(NK - 1);
                    const uint32_t p4 = tr[(NK - 1) * kTabDw + 4];
#pragma unroll
                    for (int k = 0; k < WPL; k++) acc[k][e] = perm_mul_acc(acc[k][e], sel[k][NK - 1], p.x, p.y, p.z, p.w, p4);
                }
                continue;
            }
#pragma unroll
            for (int j = 0; j + 1 < NK; j += 2)
#pragma unroll
                for (int k = 0; k < WPL; k++)
                    acc[k][e] = perm_mul2_acc(acc[k][e], sel[k][j], D[e][j].t[0], D[e][j].t[1], D[e][j].t[2], D[e][j].t[3],
                                              D[e][j].t[4], sel[k][j + 1], D[e][j + 1].t[0], D[e][j + 1].t[1],
                                              D[e][j + 1].t[2], D[e][j + 1].t[3], D[e][j + 1].t[4]);
            if (NK & 1)
#pragma unroll
                for (int k = 0; k < WPL; k++)
                    acc[k][e] = perm_mul_acc(acc[k][e], sel[k][NK - 1], D[e][NK - 1].t[0], D[e][NK - 1].t[1],
                                             D[e][NK - 1].t[2], D[e][NK - 1].t[3], D[e][NK - 1].t[4]);
        }
        // ---- writes: lane A of a word is its general destination (known: kout; erased: the
        // park location; eo: ed0), B and C the staging-only ed1 / epd ----
        const uint32_t fa = kd_l ? (w_cur >> 16) : ed_l ? (((w_cur >> 28) == kErPark) ? w_cur : kLoc10None) : w_cur;
        const uint32_t la = dst_lds(fa, sbase), sa = dst_scr(fa);
        const uint32_t lb = dst_lds(w_cur >> 10, sbase), lc = dst_lds(w_cur >> 20, sbase);
        // direct mode: staged destinations as output rows (A: ed0 of eo words; B: ed1; C: epd)
        const uint32_t oa = TEC_DEC_DIRECT ? vec_out(w_cur, w_cur) : kDrop;
        const uint32_t ob = TEC_DEC_DIRECT ? vec_out(w_cur >> 10, w_cur) : kDrop;
        const uint32_t oc = TEC_DEC_DIRECT ? vec_out(w_cur >> 20, w_cur) : kDrop;
        auto put_a = [&](int i, uint32_t v, int k) {
            *lds_at(W(la, i), k) = v;
            const uint32_t so = W(sa, i);
            if (so != kDrop)
                __builtin_amdgcn_raw_buffer_store_b32(v, rs_scr, (int)(col_local + (uint32_t)k * RSW), (int)so, 0);
        };
#pragma unroll
        for (int e = 0; e < NE; e++) {
            const uint32_t ek = W(w_cur, kDpEd + e) >> 28;
            if (ek == kErRed) {
#pragma unroll
                for (int k = 0; k < WPL; k++) {
                    *lds_at(W(la, kDpEo + e), k) = acc[k][e];
                    if (TEC_DEC_DIRECT) put_out(W(oa, kDpEo + e), acc[k][e], k);
                }
            } else if (ek == kErType1) {
#pragma unroll
                for (int k = 0; k < WPL; k++) {
                    const uint32_t c = mulc(kPft.t_u[0], acc[k][e] ^ ctkp[k][e]) ^ ctkp[k][e];
                    put_a(kDpEo + e, c, k);
                    *lds_at(W(lb, kDpEo + e), k) = c;
                    if (TEC_DEC_DIRECT) put_out(W(oa, kDpEo + e), c, k), put_out(W(ob, kDpEo + e), c, k);
                }
            } else if (ek == kErPark) {
#pragma unroll
                for (int k = 0; k < WPL; k++) put_a(kDpEd + e, acc[k][e], k);
            } else if (ek == kErFinish) {
#pragma unroll
                for (int k = 0; k < WPL; k++) {
                    const uint32_t c0 = pft3(acc[k][e], pu[k][e]), c1 = pft3(pu[k][e], acc[k][e]);
                    *lds_at(W(la, kDpEo + e), k) = c0;
                    *lds_at(W(lc, kDpEo + e), k) = c1;
                    if (TEC_DEC_DIRECT) put_out(W(oa, kDpEo + e), c0, k), put_out(W(oc, kDpEo + e), c1, k);
                }
            }
        }
        if constexpr (TEC_DEC_LATE_LD != 0) load_tkp(w_nxt);
        load_scr(w_nxt);
        if constexpr (TEC_DEC_PRIO) __builtin_amdgcn_s_setprio(0);
        // the step's rows are staged (and the step before last's flushed); ablation bit 4: timing only
        if constexpr (TEC_DEC_DIRECT != 0 || (TEC_DEC_ABLATE & 16) != 0) {  // nothing staged: no barrier, no flush
            w_cur = w_nxt;
            w_nxt = w_nn;
            continue;
        }
        lds_barrier();
        const uint32_t no = W(w_cur, kDpHdr) >> 8;
        const uint32_t r_beg = (wv * no) / G, r_end = ((wv + 1) * no) / G;
        for (uint32_t r = r_beg; r < r_end && !(TEC_DEC_ABLATE & 4); r++) {
            const uint8_t *row = lds8 + (sbase + r) * RS;
            const uint32_t it = ((uint32_t)__builtin_amdgcn_readlane(w_cur, kDpOut + (r >> 1)) >> (16u * (r & 1u))) & 0xffffu;
            const uint32_t off = (it & 0xffu) * (uint32_t)a.out_stride + (it >> 8) * sc + seg0;
            flush16(row, lane, off);
            if (RS > 1024u) flush16(row, lane + 64u, off);
            if (!wide_tail) {
                const uint32_t lt_off = nb * 16u + lane * 2u, vot = lane < (tail >> 1) ? lt_off : kDrop;
                const uint16_t v = *reinterpret_cast<const uint16_t *>(row + lt_off);
                if (vot == kDrop || off + vot + 2u <= olen) {
                    __builtin_amdgcn_raw_buffer_store_b16(v, rs_out, (int)vot, (int)off, 0);
                } else {
                    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)v, rs_out, (int)vot, (int)off, 0);
                }
            }
        }
        w_cur = w_nxt;
        w_nxt = w_nn;
    }
}

}  // namespace dstage

uint32_t decode_stage_rows(uint32_t nslots, uint32_t max_out) { return (TEC_DEC_DIRECT ? 0u : 2 * max_out) + 2 + nslots; }
bool decode_stage_fits(uint32_t nslots, uint32_t max_out) { return decode_stage_rows(nslots, max_out) <= dstage::kMaxLdsRows; }
bool decode_stage_k(int k) { return k >= 7 && k <= 10; }

uint32_t decode_stage_g(uint32_t words_per_stripe, uint32_t gmax) {
    const uint32_t groups = (words_per_stripe + 63) / 64;
    const uint32_t cap = gmax && gmax < (uint32_t)dstage::kMaxG ? gmax : (uint32_t)dstage::kMaxG;
    return groups < cap ? groups : cap;
}

// workgroups per stripe: groups of 64 words, g * WPL of them per workgroup
static uint32_t decode_stage_wgs(uint32_t words_per_stripe, uint32_t gmax) {
    const uint32_t groups = (words_per_stripe + 63) / 64, g = decode_stage_g(words_per_stripe, gmax);
    return (groups + g * dstage::kWpl - 1) / (g * dstage::kWpl);
}

size_t decode_stage_scratch_bytes(const DecArgs &a) {
    const uint32_t g = decode_stage_g(a.words_per_stripe, a.gmax), wgs = decode_stage_wgs(a.words_per_stripe, a.gmax);
    return (size_t)a.njobs * wgs * (a.nscratch_max ? a.nscratch_max : 1) * g * 256u * dstage::kWpl;
}

template <int NK, int G>
static hipError_t launch_dec_g(const DecArgs &a, uint64_t blocks, hipStream_t s) {
    const size_t lds = (size_t)a.lds_rows * G * 256u * dstage::kWpl + dstage::tab_lds_bytes(NK);
    hipError_t e = ensure_dyn_lds(reinterpret_cast<const void *>(dstage::dec_stage_kernel<NK, G>), lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((dstage::dec_stage_kernel<NK, G>), dim3((uint32_t)blocks), dim3(G * 64), lds, s, a);
    return hipGetLastError();
}

// waves per workgroup g <= kMaxG: only 1..kMaxG are built (unreachable bodies)
template <int NK, int G = dstage::kMaxG>
static hipError_t launch_dec_k(const DecArgs &a, uint32_t g, uint64_t blocks, hipStream_t s) {
    if constexpr (G > 1)
        if (g < (uint32_t)G) return launch_dec_k<NK, G - 1>(a, g, blocks, s);
    return launch_dec_g<NK, G>(a, blocks, s);
}

hipError_t launch_decode_stage(DecArgs a, hipStream_t s) {
    if (a.njobs == 0) return hipSuccess;
    if (a.lds_rows == 0 || a.lds_rows > dstage::kMaxLdsRows || a.sc < 8 || !a.scratch || a.n != 2u * kRepQ ||
        !decode_stage_k((int)a.nk))
        return hipErrorInvalidValue;
    const uint32_t g = decode_stage_g(a.words_per_stripe, a.gmax);
    a.wgs_per_stripe = decode_stage_wgs(a.words_per_stripe, a.gmax);
    const uint64_t blocks = (uint64_t)a.njobs * a.wgs_per_stripe;
    if (blocks > 0x7fffffffull) return hipErrorInvalidValue;
    switch (a.nk) {
        case 7: return launch_dec_k<7>(a, g, blocks, s);
        case 8: return launch_dec_k<8>(a, g, blocks, s);
        case 9: return launch_dec_k<9>(a, g, blocks, s);
        default: return launch_dec_k<10>(a, g, blocks, s);
    }
}

}  // namespace tec
