// kernels.hpp -- device job descriptors and launcher declarations shared by host and HIP code.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include "gf.hpp"
#include "dec_fixed.hpp"

namespace tec {

// Measurement knobs (kernel variants, JIT geometry, forced windows) are read from the environment
// only when TEC_DEBUG_KNOBS=1 is also set: a stray variable in a production process changes nothing.
inline const char *tec_knob(const char *name) {
    const char *on = getenv("TEC_DEBUG_KNOBS");
    if (!on || on[0] != '1' || on[1] != 0) return nullptr;
    return getenv(name);
}

// Raise `fn`'s dynamic-LDS limit to `bytes` on the CURRENT device.  Launchers call it before every
// launch that needs more than 64 KiB; it calls hipFuncSetAttribute once per (device, kernel) and
// larger size, under a lock (launchers run on several host threads, one handle per GPU).
hipError_t ensure_dyn_lds(const void *fn, size_t bytes);

// One stripe of one object for the encode kernels (Slicer::encode, slicer.rs:237-296).
struct EncJob {
    const uint8_t *src;   // first byte of the stripe in the object
    uint8_t *dst;         // object's slice-0 base + stripe*chunk_size
    uint64_t src_len;     // valid bytes of the stripe (rest is zero padding)
    uint32_t rot;         // rotation offset (stripe*7) % n, 0 for identity mapping
    uint32_t dst_skew;    // stripe*chunk_size: dst - (object's slice-0 base)
    uint32_t store_mask;  // internal nodes whose chunk is written (encode_dma.hip; others write all)
    uint32_t pad_;
};

struct EncArgs {
    const EncJob *jobs;
    uint32_t njobs;
    uint32_t groups_per_stripe;  // ceil(words_per_stripe / 64): 64-word column groups per stripe
    uint32_t words_per_stripe;
    uint32_t groups_per_wg;      // column groups one workgroup walks (all of them when they fit)
    uint32_t wgs_per_stripe;     // ceil(groups_per_stripe / groups_per_wg)
    uint32_t stripes_per_wg;     // whole stripes per workgroup when wgs_per_stripe == 1
    uint32_t cs;           // chunk size
    uint32_t sc;           // sub-chunk size
    uint32_t slice_len;
    uint32_t n;
    uint8_t *scratch;      // level-2 parking, encode_rows_scratch_bytes() bytes
    // encode_dma.hip: rows of planes z0 = z0_first + part * z0_count .. + z0_count, part < z0_split
    // (z0_split workgroups per stripe); z0_count 0 = all ten.  The level-1 rows (z0 < 7) are
    // independent of each other, so a small call runs them on 7 workgroups per stripe and the
    // level-2 rows (7..9, a chain) in a second launch.
    uint32_t z0_first, z0_count, z0_split;
    uint32_t z0_limit;     // a part's rows end at min(its start + z0_count, z0_limit) (0: no bound)
};

// Metadata suffix writer: one 48-byte record per object, copied to its n slices.
struct MetaJob {
    uint8_t *dst;          // object's slice-0 base + num_stripes*chunk_size
    uint64_t slice_len;    // stride between the object's slices
    uint64_t words[6];
};

// ---- generic layered engine (decode / generic encode) ----
constexpr int kGpeMaxErased = 20;
constexpr int kGpeMaxKnown = 20;

// Erasure pattern of one stripe: which internal nodes are erased, the per-plane MDS decoder
// (as v_perm tables) and the planes grouped by intersection score (decode order).
struct GpePattern {
    uint64_t erased_mask;
    uint32_t nknown, nerased, nlevels, alpha;
    uint8_t known[kGpeMaxKnown];
    uint8_t erased[kGpeMaxErased];
    uint32_t level_start[16];          // planes of level L: planes[level_start[L] .. level_start[L+1])
    uint32_t planes_off;               // offset (in uint16) of this pattern's plane list in the plane pool
    uint32_t pad_;
    PermTab D[kGpeMaxErased][kGpeMaxKnown];  // U_erased[e] = sum_j D[e][j] * U_known[j]
    // the same matrix as 2-bit-field tables (perm_tab4) for patterns of at most kClsMaxE x kClsMaxK
    // (the decode class kernels: each v_perm reads one table dword twice, so no table move)
    uint32_t D4[13][7][4];
};
constexpr int kClsMaxE = 13, kClsMaxK = 7;

struct GpeJob {
    const uint8_t *in;     // node-strided input base
    uint8_t *out;          // node-strided output base
    uint64_t in_len;       // valid input bytes from `in` (zero beyond)
    uint64_t out_len;      // output bytes kept from `out` (trim beyond)
    uint32_t rot;          // rotation offset for the rotated side
    uint32_t pattern;      // index into the pattern array
};

struct GpeArgs {
    const GpeJob *jobs;
    const GpePattern *patterns;
    const uint16_t *plane_pool;
    uint32_t njobs;
    uint32_t word_base, word_end;  // words [word_base, word_end) of each stripe are processed
    uint32_t groups_per_stripe;  // ceil((word_end - word_base) / kGpeWords)
    uint32_t cs, sc, q, t, k, nu, n, alpha;
    uint64_t in_stride, out_stride;  // bytes between consecutive nodes on each side
    uint32_t in_rotated, out_rotated;
    uint64_t out_mask;               // internal nodes whose C is written to `out`
    uint32_t qpow[16];               // q^i
};

// ---- repair engine ----
struct RepPattern {
    uint64_t erased_mask, aloof_mask;
    uint32_t nknown, nerased, nlevels, beta;
    uint32_t lost;                     // internal lost node
    uint32_t pad_;
    uint8_t known[kGpeMaxKnown];
    uint8_t erased[kGpeMaxErased];
    uint32_t level_start[16];          // over the repair-plane list
    uint32_t planes_off;               // plane pool offset: beta repair planes in decode order
    uint32_t pad2_;
    PermTab D[kGpeMaxErased][kGpeMaxKnown];
};

struct RepJob {
    const uint8_t *helper[kMaxNodes];  // per internal node: this stripe's beta sub-chunks (or null)
    uint8_t *out;                      // lost chunk destination (chunk_size bytes)
    uint32_t pattern;
    uint32_t aux;                      // repair_fold.hip: x of the lost node | kernel index << 8
};

// Staged repair kernel (repair_stage.hip): per pattern, the uniform control data of every
// repair plane, host-resolved so the kernel does no index arithmetic (q = beta = 10 profiles).
constexpr int kRepQ = 10;
struct RepProg {                   // 32-bit fields: scalar loads have no sub-dword form on gfx950
    uint32_t ekind[kGpeMaxErased];  // erased e: 0 aloof, 1 lost, 2 column-mate x < x_lost, 3 mate x > x_lost
    uint32_t erow[kGpeMaxErased];   // aloof index (kind 0) / staging row (kinds 1-3)
    uint32_t enode[kGpeMaxErased];  // erased node id
    uint32_t knode0[kGpeMaxKnown];  // known node id
    struct Step {
        uint32_t z, ri;                   // plane, its repair row
        uint32_t kkind[kGpeMaxKnown];     // known j: 0 red, 1/2 helper partner (x < / > z_y), 3/4 aloof partner
        uint32_t knode[kGpeMaxKnown];     // partner node (kinds 1, 2)
        uint32_t krow[kGpeMaxKnown];      // partner repair row (1, 2) or aloof LDS row ai * 10 + r (3, 4)
        uint32_t oplane[kRepQ];           // staging row -> lost-chunk plane
    } step[kRepQ];
};

// Staged decode kernel (decode_stage.hip): a host-compiled program per erasure pattern for
// q = 10, t = 2 profiles.  Planes run row by row (rows = one plane digit, "outer"); every value a
// later plane needs is parked in a lane-private LDS slot (consumer in the same row) or in a
// per-stripe global scratch row (later row).  Location codes: 0xffffffff none, else
// type << 24 | index with type 0 staging row, 1 LDS slot, 2 scratch row.
constexpr int kDecMaxK = 10, kDecMaxE = 13, kDecMaxOut = 16;
constexpr int kDecMaxOutProg = 32;  // DecStep items: the packed (table-kernel) form holds kDecMaxOut
constexpr uint32_t kLocNone = 0xffffffffu;
enum : uint32_t { kLocStage = 0, kLocSlot = 1, kLocScratch = 2 };
enum : uint32_t { kKnRed = 0, kKnInput = 1, kKnLoc = 2, kKnPark = 3, kKnInputU = 4 };                       // known j kinds
enum : uint32_t { kErSkip = 0, kErRed = 1, kErType1 = 2, kErPark = 3, kErFinish = 4, kErType1U = 5 };  // erased e kinds
// kKnPark / kErType1U (generated class kernels and hipRTC pattern kernels, dec_prog_fuse_type1): the type-1 step
// parks its known partner's U = pft3(Cp, C) instead of C, and stores the partner's row out if it is
// an output, so the partner's own step reads U from the location and never loads its own row.
// kKnInputU (dec_prog fuse_pairs): of two known nodes coupled within one row of planes, the first
// step parks the second's U = pft3(Cp, C) in an LDS slot (kpark) and stores its row out (kpout);
// the second step is kKnPark and loads neither row.
struct DecStep {
    uint32_t z;                    // plane
    uint32_t nout;                 // flush items (item i = staging row i)
    uint32_t out[kDecMaxOutProg];  // data chunk x | plane << 8
    uint32_t kk[kDecMaxK];         // known j kind
    uint32_t kp[kDecMaxK];         // kKnInput: partner node | plane << 8; kKnLoc: partner C location
    uint32_t kout[kDecMaxK];       // staging row of the known node's C (data nodes), or none
    uint32_t kpark[kDecMaxK];      // kKnInputU: location of the partner's U; kpout: its row's output
    uint32_t kpout[kDecMaxK];
    uint32_t ek[kDecMaxE];         // erased e kind
    uint32_t ep[kDecMaxE];         // type-1: partner node | plane << 8; park: U location; finish: partner U location
    uint32_t ed0[kDecMaxE], ed1[kDecMaxE];  // destinations of C (red / type-1 / finish)
    uint32_t epd[kDecMaxE];        // finish: destination of the partner's C
};
// The form the kernel reads (ClayHost::dec_pack): 48 dwords per step, lanes 0..47 of one VGPR.
//   kd[j] = kind << 28 | kout << 16 | src        eo[e] = ed0 | ed1 << 10 | epd << 20
//   ed[e] = kind << 28 | src                     out:  flush items, 16 bits each (x | plane << 8)
//   src: node | plane << 8 (kKnInput, kErType1), else a 10-bit location;
//   10-bit location: type << 8 | index, 0x3ff none.
constexpr uint32_t kLoc10None = 0x3ffu;
enum : uint32_t { kDpHdr = 0, kDpKd = 1, kDpEd = kDpKd + kDecMaxK, kDpEo = kDpEd + kDecMaxE,
                  kDpOut = kDpEo + kDecMaxE, kDpWords = 48 };
struct DecStepP {
    uint32_t w[kDpWords];          // hdr = z | nout << 8
};
static_assert(kDpOut + kDecMaxOut / 2 <= kDpWords, "packed step");
struct DecProgHdr {
    uint32_t nsteps, nslots, nscratch, max_out;
    uint32_t knode[kDecMaxK];      // known node ids (input slices)
};

struct RepArgs {
    const RepJob *jobs;
    const RepPattern *patterns;
    const uint16_t *plane_pool;       // repair planes per pattern (decode order)
    const uint16_t *plane_ind;        // per pattern: alpha entries, plane -> index in helper buffer
    uint32_t njobs, words_per_stripe, groups_per_stripe;
    uint32_t cs, sc, q, t, alpha;
    uint32_t qpow[16];
    uint32_t wgs_per_stripe;          // staged kernel: workgroups per stripe row
    const RepProg *progs;             // staged kernel: per pattern
};

constexpr int kGpeWords = 4;     // words (4 columns each) per GPE block
constexpr int kGpePlaneThreads = 32;

struct DecArgs {
    const GpeJob *jobs;            // in = object's slice 0 + stripe*cs, out = object + stripe*S
    const GpePattern *patterns;    // D tables
    const DecProgHdr *hdrs;        // per pattern
    const DecStepP *steps;         // per pattern: 100 steps + 2 blank, at step_off[pattern]
    const uint32_t *step_off;
    uint8_t *scratch;              // per workgroup tile: nscratch_max rows
    uint32_t njobs, words_per_stripe, wgs_per_stripe;
    uint32_t cs, sc, n, nk, lds_rows, nscratch_max;  // lds_rows: max over patterns of slots + staging rows
    uint64_t in_stride, out_stride;
    uint32_t gmax;  // waves per workgroup at most (0: the build's TEC_DEC_MAXG); 1 for small calls
};
hipError_t launch_decode_stage(DecArgs a, hipStream_t s);
size_t decode_stage_scratch_bytes(const DecArgs &a);
uint32_t decode_stage_rows(uint32_t nslots, uint32_t max_out);  // LDS rows of a program
bool decode_stage_fits(uint32_t nslots, uint32_t max_out);
uint32_t decode_stage_g(uint32_t words_per_stripe, uint32_t gmax = 0);  // waves per workgroup

// Per-pattern decode kernels compiled at run time (dec_rtc.cpp, dec_fixed.hpp), per handle.
using dfix_args = dfix::Args;
static_assert(sizeof(dfix::Job) == sizeof(GpeJob) && offsetof(dfix::Job, rot) == offsetof(GpeJob, rot), "dfix::Job");
struct DecJitKernel {
    hipFunction_t fn;
    size_t lds;          // dynamic LDS bytes
    uint32_t nscratch;   // scratch rows per tile
    uint32_t wb;         // columns per lane (4 or 8)
};
struct DecJit;
struct ClayHost;
DecJit *dec_jit_new(int device);
void dec_jit_free(DecJit *j);
void dec_jit_set(DecJit *j, int mode, uint64_t min_stripes);  // mode 0 off, 1 async, 2 sync
void dec_jit_counts(DecJit *j, uint32_t timeout_ms, uint32_t *ready, uint32_t *pending, uint32_t *failed);
// A status reader keeps `j` alive across dec_jit_counts: hold it while the handle's lock still
// guards `j`, unhold after.  dec_jit_free wakes held waiters and waits for them to leave.
void dec_jit_hold(DecJit *j);
void dec_jit_unhold(DecJit *j);
// The pattern's kernel for G waves of wb-column lanes if built; counts `stripes` toward building it.
const DecJitKernel *dec_jit_get(DecJit *j, const ClayHost &h, const GpePattern &P, int orient, int G, int wb, uint64_t stripes);
// Tile geometry of a pattern kernel for sub-chunk sc: lanes of wb columns, wps words per row,
// G waves per workgroup, wgs workgroups per stripe.
struct DecJitGeom { uint32_t wb, wps, G, wgs; };
DecJitGeom dec_jit_geom(uint32_t sc);
hipError_t launch_dec_fixed(const DecJitKernel &k, const dfix_args &a, uint32_t G, hipStream_t s);
bool decode_stage_k(int k);  // a staged-decode kernel is compiled for this k (n = 20)

// Decode class kernels (decode_class.hip, dec_class.hpp): one ahead-of-time kernel per class of
// 7-of-20 survivor sets of Clay(20,7,16), run-time node / plane relabelling and decoding matrix.
bool dec_class_info(int id, uint32_t *nslots, uint32_t *nscratch);  // false: no such kernel
uint32_t dec_class_wgs(uint32_t sc, uint32_t G);
size_t dec_class_scratch_bytes(int id, uint32_t njobs, uint32_t sc, uint32_t G);
hipError_t launch_dec_class(int id, const GpeJob *jobs, const GpePattern *patterns, uint32_t njobs, uint32_t sc,
                            uint64_t in_stride, uint64_t out_stride, uint32_t n, uint8_t *scratch, uint32_t G,
                            hipStream_t s);

// ---- slice commitments (commit.hip) ----
constexpr int kCommitMaxLeaves = 64;
struct CommitArgs {
    const uint8_t *slices;     // object o's slice i at slices + o * obj_stride + i * slice_len
    uint64_t obj_stride, slice_len;  // slice_len % 4 == 0
    uint32_t n, nobj, height;
    uint8_t *leaf;             // nobj * n * 32
    uint8_t *root;             // nobj * 32, or null (no tree)
    uint8_t *proof;            // nobj * n * height * 32, or null
};
hipError_t launch_commit(const CommitArgs &a, hipStream_t s);

hipError_t launch_encode_rows(int k, bool masked, const EncArgs &a, hipStream_t s);
// encode_dma.hip: Clay(20,7,16), 1,280 < sub-chunk <= 1,440 bytes (the 1 MB stripes), no scratch
bool encode_dma_supported(int n, int k, uint32_t sc);
hipError_t launch_encode_dma(bool masked, const EncArgs &a, hipStream_t s);
hipError_t launch_meta(const MetaJob *jobs, uint32_t njobs, uint32_t n, hipStream_t s);
struct CopyJob {
    const uint8_t *src;
    uint8_t *dst;
    uint64_t len;          // bytes written at dst
    uint64_t valid;        // bytes copied from src; the rest of len is zero-filled
};
hipError_t launch_gather(const CopyJob *jobs, uint32_t njobs, hipStream_t s);
hipError_t launch_gpe(const GpeArgs &a, uint32_t max_erased, hipStream_t s);

// ---- GF(2^16) Leopard RS (rs16.hip) ----
constexpr uint32_t kRs16MaxK = 64;  // decode: received shards per matrix row
struct Rs16EncArgs {
    const uint8_t *in;          // original shard j at in + seg * seg_in + j * in_stride
    uint8_t *out;               // recovery shard j at out + seg * seg_out + j * out_stride
    uint64_t in_stride, out_stride, seg_in, seg_out;
    const uint16_t *lut;        // span x 64 nibble-table entries: multiplier = skew[s]
    uint32_t k, m, c, high, work_len, span, elems;  // elems: field elements per shard (bytes / 2)
    uint32_t one_chunk;         // low rate, c <= 32: one chunk of work in LDS, the IFFT kept in registers
};
constexpr uint32_t kRs16DecPtrs = 256;  // shard pointers per decode launch (kernel arguments)
struct Rs16DecArgs {
    // per segment g (grid.y): its k received shards at ptr[g * (k + nmiss) + r], then its nmiss
    // restored originals -- kernel arguments, so a call uploads nothing
    const uint8_t *ptr[kRs16DecPtrs];
    const uint16_t *lut;            // nmiss x k nibble tables (decoding-matrix coefficients)
    uint32_t k, nmiss, elems;
};
// GF(2^16) matrix apply (rs16.hip rs16_matrix_kernel), the encode and the decode both:
// out[i] = sum_r M[i][r] * in[r] for i < rows, r < k.  `tab` is M's packed lookup image
// (rs16::mat_image): per input r, nibble q and group g of 4 rows, 16 entries of 4 u16 -- entry n
// holds M[4g + j][r] * (n << 4q) for j = 0..3 -- so one 8-byte LDS read serves 4 rows' products.
constexpr uint32_t kRs16MatMaxG = 16;          // rows <= 64
constexpr uint32_t kRs16MatLds = 80 * 1024;    // image bytes (k * G * 512) staged per block: 2 blocks per CU
struct Rs16MatArgs {
    const uint8_t *in;   // ptrs == 0: input r of segment g at in + g * seg_in + r * in_stride,
    uint8_t *out;        //            output i at out + g * seg_out + i * out_stride
    uint64_t in_stride, out_stride, seg_in, seg_out;
    const uint8_t *ptr[kRs16DecPtrs];  // ptrs == 1: segment g's k inputs then rows outputs at ptr[g * (k + rows) + j]
    const uint16_t *tab;
    const uint32_t *ktab;  // set by the launcher: rs16_mat_tailv's constants (after the staged image)
    uint32_t k, rows, elems, segments, ptrs;
    uint32_t rstride;  // set by the launcher: image bytes per input (a run-time value, so the kernel's
                       // per-input bases stay one scalar each instead of 4k folded constants)
};
// TEC_RS16_MAT_TV=1 (off by default: measured slower): for rows = 8 h + 1 (OuterCoder(17, 50):
// 33 encode rows, 17 decode rows) the last row is computed bit-serially on the VALU from 16
// per-input constants instead of an 8-byte table read per nibble (which serves 4 rows for the 1
// needed), so the LDS array moves only whole 8-row entries.  r05 on the GPU: encode 1.67 ms
// against 1.58, decode 1.36 against 1.20 -- the VALU (~70 % busy) cannot take 3 more
// instructions per bit of every input.
#ifndef TEC_RS16_MAT_TV
#define TEC_RS16_MAT_TV 0
#endif
inline bool rs16_mat_tailv(uint32_t rows) { return TEC_RS16_MAT_TV && rows % 8 == 1 && rows > 1; }
// The odd last 4-row group (G = ceil(rows / 4) odd) holds rows - 8 (G / 2) rows: its nibble
// entries are 2 B for one row (ds_read_u16), 4 B for two (ds_read_b32), else 8 B (ds_read_b64) --
// TEC_RS16_MAT_NARROW=0: 8 B always.  The LDS array bounds the kernel, and an 8-byte
// read serving one row's products was a quarter used.
#ifndef TEC_RS16_MAT_NARROW
#define TEC_RS16_MAT_NARROW 1
#endif
inline uint32_t rs16_mat_tail_bytes(uint32_t rows) {
    const uint32_t G = (rows + 3) / 4;
    if (!(G & 1) || rs16_mat_tailv(rows)) return 0;
    const uint32_t t = rows - 8 * (G / 2);
    return !TEC_RS16_MAT_NARROW || t > 2 ? 8u : 2u * t;
}
// bytes of one (input, nibble position) block: G / 2 pair tables of 256 B, then the tail table
inline uint32_t rs16_mat_block_bytes(uint32_t rows) { return ((rows + 3) / 4 / 2) * 256u + 16u * rs16_mat_tail_bytes(rows); }
inline size_t rs16_mat_bytes(uint32_t k, uint32_t rows) {  // the LDS-staged part of the image
    return (size_t)k * 4u * rs16_mat_block_bytes(rows);
}
inline size_t rs16_mat_image_bytes(uint32_t k, uint32_t rows) {  // + the tail row's constants (k x 16 u32)
    return rs16_mat_bytes(k, rows) + (rs16_mat_tailv(rows) ? (size_t)k * 64u : 0u);
}
inline bool rs16_mat_supported(uint32_t k, uint32_t rows) {
    return k >= 1 && k <= 32 && rows >= 1 && (rows + 3) / 4 <= kRs16MatMaxG && rs16_mat_bytes(k, rows) <= kRs16MatLds;
}
hipError_t launch_rs16_matrix(const Rs16MatArgs &a, hipStream_t s);
hipError_t launch_rs16_encode(const Rs16EncArgs &a, uint32_t segments, hipStream_t s);
hipError_t launch_rs16_decode(const Rs16DecArgs &a, uint32_t segments, hipStream_t s);
hipError_t launch_repair(const RepArgs &a, uint32_t max_erased, hipStream_t s);
hipError_t launch_repair_stage(RepArgs a, hipStream_t s);
// repair_fold.hip: Clay(20,7,16) with minimum_to_repair's helper set when at most one of the
// other column's first 7 nodes is unavailable (the decoding matrix folded per lost column and
// known set); repair_fold_column() -> kernel index 0..15 for such a pattern, else -1.  One launch
// serves every index: RepJob::aux = x_lost | index << 8.
int repair_fold_column(uint32_t q, uint32_t t, uint32_t k, uint32_t beta, uint32_t sc, uint32_t lost,
                       uint64_t erased_mask, uint64_t aloof_mask);
hipError_t launch_repair_fold(RepArgs a, hipStream_t s);
bool repair_stage_supported(uint32_t q, uint32_t beta, uint32_t sc, uint32_t nerased, uint32_t nknown, uint64_t aloof_mask);
bool encode_rows_supported(int n, int k, int d);
size_t encode_rows_scratch_bytes(const EncArgs &a);  // a.njobs, a.groups_per_stripe set

}  // namespace tec
