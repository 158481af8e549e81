/*
 * tape_ec.h -- C ABI of the MI355X-native Tapedrive erasure-coding engine (libtapeec.so).
 *
 * Drop-in boundary for the reference hot path `lib/slicer` (crate tape-slicer).  Every entry
 * point below replaces one Rust item of lib/slicer's public surface (lib/slicer/src/lib.rs:15-27);
 * the file:line it replaces is cited next to it.  The Rust binding a maintainer would add
 * (an `extern "C"` block behind `ClayCoder`/`Slicer`) is shown in INTEGRATION.md.
 *
 * Conventions (mirroring the reference):
 *   - plain pointers + sizes, caller-allocated outputs, int status (0 = ok), no exceptions;
 *   - status codes map 1:1 onto EncodeError / DecodeError / RepairError
 *     (lib/slicer/src/errors.rs:5-37) plus engine errors;
 *   - all GF(2^8) compute runs on the GPU (gfx950).  With no HIP device the compute entry
 *     points return TE_ERR_NO_DEVICE: there is NO CPU fallback in this library.
 *   - host-only entry points (geometry, metadata, rotation maps, repair planning, helper-side
 *     gather) are pure integer bookkeeping and work without a GPU, as in the reference.
 *   - thread safety: a te_clay may be used from several threads; calls on one te_clay are
 *     serialised internally.  The GPU context is a process-wide singleton.
 */
#ifndef TAPE_EC_H
#define TAPE_EC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TE_META_SIZE 48      /* SliceMetadata::SIZE          lib/slicer/src/metadata.rs:44 */
#define TE_ROTATION_STEP 7   /* ROTATION_STEP                lib/slicer/src/slicer.rs:21   */
#define TE_GROUP_SIZE 20     /* GROUP_SIZE                   lib/core/src/erasure.rs:5     */
#define TE_ENCODING_CLAY 2   /* EncodingType::Clay           lib/core/src/encoding.rs:25   */
#define TE_CLAY_DEFAULT_PARAMS 0x100714ull /* ClayParams::DEFAULT (20,7,16) encoding.rs:236-239 */

typedef enum te_status {
    TE_OK = 0,
    /* EncodeError  errors.rs:5-11 */
    TE_ERR_TOO_MUCH_DATA = 1,
    TE_ERR_EMPTY_INPUT = 2,
    /* DecodeError  errors.rs:13-23 */
    TE_ERR_NOT_ENOUGH_SLICES = 3,
    TE_ERR_BAD_ENCODING = 4,
    TE_ERR_INVALID_LAYOUT = 5,
    /* RepairError  errors.rs:25-37 */
    TE_ERR_NOT_ENOUGH_HELPERS = 6,
    TE_ERR_INVALID_SLICE = 7,
    TE_ERR_CLAY = 8,
    TE_ERR_MISSING_HELPER = 9,
    /* MerkleError (lib/crypto/src/merkle/tree.rs:360-366) */
    TE_ERR_MERKLE_TREE_FULL = 10,
    TE_ERR_MERKLE_INVALID_PROOF = 11,
    TE_ERR_MERKLE_INVALID_INDEX = 12,
    TE_ERR_MERKLE_PROOF_LENGTH = 13,
    /* engine */
    TE_ERR_INVALID_ARG = 20,
    TE_ERR_NO_DEVICE = 21,
    TE_ERR_HIP = 22,
    TE_ERR_UNSUPPORTED = 23,
    TE_ERR_OUT_OF_MEMORY = 24,
    TE_ERR_BUFFER_TOO_SMALL = 25
} te_status;

const char *te_strerror(int status);
/* Number of usable gfx950 devices (0 on a CPU-only host).  Does not create a context. */
int te_device_count(void);
/* Make `device` the calling thread's current HIP device (hipSetDevice).  Handles do not depend on
 * it: a te_clay runs on the device it is bound to (te_clay_bind_device). */
int te_set_device(int device);
/* Detail of the last TE_ERR_HIP/OOM/NO_DEVICE on the calling thread (HIP error string). */
const char *te_last_error_detail(void);
/* Kernel timing (diagnostics for benchmarks): while enabled, every device batch call records a
 * HIP event pair on its stream around its kernel launches (after descriptor upload).
 * te_kernel_time_ms synchronises on the recorded events, returns their summed elapsed time and
 * count, and clears them.  Off by default; no effect on results. */
int te_kernel_timing(int enable);
int te_kernel_time_ms(double *total_ms, uint32_t *count);
/* Library build identification string. */
const char *te_version(void);

/* ------------------------------------------------------------------------------------------
 * ClayCoder                                                     lib/slicer/src/clay.rs:13-122
 * ------------------------------------------------------------------------------------------ */
typedef struct te_clay te_clay;
typedef struct te_clay_info {
    uint32_t n, k, m, d;     /* ErasureCoder::{n,k,m}, ClayCoder::d()   coder.rs:16-25, clay.rs:43-45 */
    uint32_t q, t, nu;       /* Clay layout: q = d-k+1, t = (n+nu)/q                                */
    uint32_t alpha, beta;    /* ClayCoder::alpha()/beta()                clay.rs:48-57              */
} te_clay_info;

/* ClayCoder::new(n, k, d)  clay.rs:24-34.  The reference panics on invalid params; this returns
 * TE_ERR_INVALID_ARG.  Profiles whose layout the GPU engine does not cover return
 * TE_ERR_UNSUPPORTED. */
int te_clay_new(uint32_t n, uint32_t k, uint32_t d, te_clay **out);
/* ClayCoder::from_params(ClayParams)  clay.rs:37-39 (packed n | k<<8 | d<<16, encoding.rs:193-197) */
int te_clay_from_params(uint64_t packed_params, te_clay **out);
void te_clay_free(te_clay *c);
/* Device binding (SURVEY 8b device-mask context; one SDK process may drive several GPUs): a handle
 * is bound to the device that was current on the creating thread; every allocation and launch it
 * makes runs on that device whatever the calling thread's current device is (the thread's device
 * is restored on return).  Re-binding drains and frees the handle's device state first. */
int te_clay_bind_device(te_clay *c, int device);
int te_clay_device(const te_clay *c);
/* Per-pattern decode kernels (no reference counterpart; an engine knob).  A hot erasure pattern
 * of a q = 10, t = 2 profile gets a kernel with its plane program and decoding matrix compiled
 * in (hipRTC, ~25 s of host time, off the caller's thread in mode 1); until then, and for every
 * other pattern, the table-driven kernel decodes it.  Clay(20,7,16) survivor sets run their
 * ahead-of-time class kernels instead, which time at or below the pattern kernels, unless this
 * function has been called on the handle.  mode: 0 off, 1 async (default; env
 * TEC_DEC_JIT=off|sync|async), 2 sync (compile in the decoding call).  A pattern is built once
 * `min_stripes` of its stripes have been decoded on the handle (default 1024, env
 * TEC_DEC_JIT_MIN). */
int te_clay_set_decode_jit(te_clay *c, int mode, uint64_t min_stripes);
/* Pattern kernels ready / compiling / failed on the handle, after waiting up to `timeout_ms` for
 * compiles in flight to finish. */
int te_clay_decode_jit_status(te_clay *c, uint32_t timeout_ms, uint32_t *ready, uint32_t *pending, uint32_t *failed);
/* Most distinct stripe patterns the handle's device-resident decode store holds (default and
 * maximum 16,384, ~26 KB of device memory and as much host memory each; the store grows by
 * doubling from 256 as patterns arrive).  A call with more distinct patterns than this uploads
 * them with the call. */
int te_clay_set_decode_store_cap(te_clay *c, uint32_t max_patterns);
/* The handle's device-resident decode pattern store (diagnostics): slots allocated (it grows by
 * doubling from 256 up to the cap) and filled, how often a full store was
 * emptied, how often it grew, and how many calls had more distinct stripe patterns than it holds
 * (those upload their patterns with the call instead). */
int te_clay_decode_store_stats(te_clay *c, uint32_t *capacity, uint32_t *used, uint64_t *clears, uint64_t *grows,
                               uint64_t *arena_calls);
int te_clay_get_info(const te_clay *c, te_clay_info *out);
/* ClayCoder::chunk_size_for  clay.rs:61-73 */
size_t te_clay_chunk_size_for(const te_clay *c, size_t input_len);
/* ClayCoder::track_chunk_size  clay.rs:81-84 */
size_t te_clay_track_chunk_size(const te_clay *c, size_t stripe_size, size_t blob_len);
/* ErasureCoder::encode for ClayCoder  clay.rs:99-104.  chunks: n*chunk_size bytes, chunk i at
 * i*chunk_size.  Empty input -> TE_ERR_EMPTY_INPUT.  (GPU) */
int te_clay_encode(te_clay *c, const uint8_t *data, size_t len, uint8_t *chunks, size_t cap,
                   size_t *chunk_size);
/* ErasureCoder::decode for ClayCoder  clay.rs:106-122.  chunks[i] == NULL marks chunk i missing.
 * out: k*chunk_size bytes (padded data; the Slicer trims).  (GPU) */
int te_clay_decode(te_clay *c, const uint8_t *const *chunks, size_t chunk_size, uint8_t *out,
                   size_t cap);
/* ClayCoder::plan_repair  repair.rs:53-70: helpers_out gets d shard ids (ascending),
 * sub_chunks_out gets beta plane indices (ascending).  Host only. */
int te_clay_plan_repair(const te_clay *c, uint32_t lost, const uint32_t *available, size_t navail,
                        uint32_t *helpers_out, uint32_t *sub_chunks_out);
/* ClayCoder::repair  repair.rs:75-88: helper_data[j] = beta*sub_chunk bytes of helpers[j].
 * out = chunk_size bytes.  (GPU) */
int te_clay_repair(te_clay *c, uint32_t lost, const uint32_t *helpers,
                   const uint8_t *const *helper_data, size_t nhelpers, size_t chunk_size,
                   uint8_t *out);

/* ------------------------------------------------------------------------------------------
 * Slicer<ClayCoder>                          lib/slicer/src/{adaptive,slicer,metadata}.rs
 * ------------------------------------------------------------------------------------------ */
size_t te_pick_stripe_size(size_t blob_len);                      /* adaptive.rs:31-39 */
size_t te_num_stripes(size_t blob_len, size_t stripe_size);       /* adaptive.rs:43-49 */
uint32_t te_shard_to_slice(int rotated, uint32_t n, uint32_t stripe, uint32_t shard); /* slicer.rs:34-42 */
uint32_t te_slice_to_shard(int rotated, uint32_t n, uint32_t stripe, uint32_t slice); /* slicer.rs:46-54 */

typedef struct te_slice_metadata {   /* SliceMetadata, 48-byte LE suffix   metadata.rs:22-37 */
    uint64_t version, blob_len, stripe_size, encoding, params, chunk_index;
} te_slice_metadata;
/* SliceMetadata::to_bytes  metadata.rs:66-69 */
void te_slice_metadata_to_bytes(const te_slice_metadata *m, uint8_t out[TE_META_SIZE]);
/* SliceMetadata::from_slice  metadata.rs:72-87 (rejects stripe sizes not in STRIPE_SIZES) */
int te_slice_metadata_from_slice(const uint8_t *slice, size_t len, te_slice_metadata *out);

typedef struct te_slicer_cfg {       /* Slicer fields   slicer.rs:124-132 */
    int rotated;                     /* MappingStrategy::Rotated if non-zero */
    uint64_t encoding, params;       /* EncodingProfile written to the metadata suffix */
    uint64_t chunk_index;            /* ChunkNumber salt */
} te_slicer_cfg;
typedef struct te_geometry {
    uint64_t stripe_size, num_stripes, chunk_size, sub_chunk_size, slice_len;
} te_geometry;
/* Slicer::encode geometry (pick_stripe_size + chunk_size_for + metadata) slicer.rs:237-262 */
int te_slicer_geometry(const te_clay *c, size_t blob_len, te_geometry *out);
/* Slicer::encode  slicer.rs:237-296 (+ encode_empty_blob :368-387).  slices: n*slice_len
 * bytes, slice i at i*slice_len.  (GPU) */
int te_slicer_encode(te_clay *c, const te_slicer_cfg *cfg, const uint8_t *data, size_t len,
                     uint8_t *slices, size_t cap);
/* Slicer::decode  slicer.rs:298-364.  slices[i] == NULL marks slice i missing; all present
 * slices are slice_len bytes.  (GPU) */
int te_slicer_decode(te_clay *c, const te_slicer_cfg *cfg, const uint8_t *const *slices,
                     size_t slice_len, uint8_t *out, size_t cap, size_t *out_len);

/* ------------------------------------------------------------------------------------------
 * Repair                                                       lib/slicer/src/repair.rs
 * ------------------------------------------------------------------------------------------ */
typedef struct te_repair_plan te_repair_plan;
typedef struct te_repair_plan_info {  /* RepairPlan  repair.rs:16-28 */
    uint32_t lost, num_stripes, d, beta;
    uint64_t chunk_size, sub_chunk_size;
} te_repair_plan_info;
/* Slicer::repair_plan_from_params  repair.rs:137-201 (host only) */
int te_repair_plan_from_params(const te_clay *c, int rotated, uint32_t lost,
                               const uint32_t *available, size_t navail, uint64_t blob_len,
                               uint64_t stripe_size, te_repair_plan **out);
/* Slicer::repair_plan  repair.rs:208-281 (layout from a reference slice; host only) */
int te_repair_plan_from_slice(const te_clay *c, int rotated, uint32_t lost,
                              const uint32_t *available, size_t navail,
                              const uint8_t *reference, size_t ref_len, te_repair_plan **out);
void te_repair_plan_free(te_repair_plan *p);
int te_repair_plan_get_info(const te_repair_plan *p, te_repair_plan_info *out);
/* StripeRepair/HelperPlan  repair.rs:30-47: helper_slices/helper_shards get d entries,
 * sub_chunks gets d*beta entries (helper-major). */
int te_repair_plan_stripe(const te_repair_plan *p, uint32_t stripe, uint32_t *lost_shard,
                          uint32_t *helper_slices, uint32_t *helper_shards, uint32_t *sub_chunks);
/* Bytes helper `slice` contributes under the plan. */
size_t te_extract_repair_data_size(const te_repair_plan *p, uint32_t helper_slice);
/* extract_repair_data  repair.rs:97-130 (helper-side gather; host only) */
int te_extract_repair_data(const te_repair_plan *p, const uint8_t *slice, size_t slice_len,
                           uint32_t helper_slice, uint8_t *out, size_t cap, size_t *out_len);
/* per_helper_reqs (network/node/src/features/spool/repair.rs:468-491) for one helper: the
 * RepairRequest (network/protocol/src/api/types.rs:75-85) the repairing node sends helper slice
 * `helper_slice` -- one StripeSubChunkRequest {stripe, sub_chunks} per stripe the helper serves,
 * in plan order; stripe k at stripes[k], its beta sub-chunk indices at sub_chunks[k*beta].
 * *count = the number of stripes (arrays NULL: count only). */
int te_repair_plan_helper_request(const te_repair_plan *p, uint32_t helper_slice, uint32_t *stripes,
                                  uint32_t *sub_chunks, size_t cap_stripes, size_t *count);
/* The helper node's extract_repair_data (network/node/src/features/spool/repair.rs:496-553):
 * serve a RepairRequest from the stored slice alone -- geometry from its metadata suffix and the
 * coder's alpha; stripe i's nsub[i] sub-chunk indices are consecutive in sub_chunks; output is
 * every requested sub-chunk in request order.  Layout errors return TE_ERR_INVALID_LAYOUT with
 * the reference's message in te_last_error_detail().  Host only. */
int te_serve_repair_request(te_clay *c, const uint8_t *slice, size_t slice_len, const uint32_t *stripes,
                            const uint32_t *nsub, const uint32_t *sub_chunks, size_t nstripes, uint8_t *out,
                            size_t cap, size_t *out_len);
/* Slicer::repair  repair.rs:324-367: helper_data/helper_lens indexed by SLICE id (n entries,
 * NULL = not provided).  out = num_stripes*chunk_size + 48 bytes.  (GPU) */
int te_slicer_repair(te_clay *c, const te_repair_plan *p, const uint8_t *const *helper_data,
                     const size_t *helper_lens, const uint8_t metadata[TE_META_SIZE],
                     uint8_t *out, size_t cap);

/* ------------------------------------------------------------------------------------------
 * Device-resident batch API (new; the batching seam of sdk/src/stream/write.rs:332-362 and
 * network/node/src/features/spool/repair.rs:94-226).  All pointers are DEVICE pointers;
 * descriptors are host arrays; work is enqueued on `hip_stream` (NULL = default stream) and
 * the call returns without synchronising.
 * ------------------------------------------------------------------------------------------ */
typedef struct te_object {
    uint64_t data_off;    /* object bytes at d_data + data_off */
    uint64_t blob_len;
    uint64_t out_off;     /* n slices at d_out + out_off, slice i at + i*slice_len */
    uint64_t chunk_index;
} te_object;
/* Batched Slicer::encode of nobj objects (each object's geometry from its blob_len). */
int te_encode_batch_device(te_clay *c, const te_slicer_cfg *cfg, const uint8_t *d_data,
                           const te_object *objs, size_t nobj, uint8_t *d_out, void *hip_stream);

/* Batched Slicer::encode HOST -> HOST: the shape of the sdk stream writer's encode stage
 * (sdk/src/stream/write.rs:332-362: object bytes in, n slices per object out).  Offsets in
 * `objs` are relative to h_data / h_out.  Objects are pipelined through the device in windows
 * of at most `window_bytes` (input + output; 0 = 128 MiB) over three streams, so the H2D copy of
 * one window, the kernels of the next and the D2H copy of a third overlap.  h_data/h_out
 * should be pinned (hipHostMalloc / hipHostRegister) for full PCIe rate.  Synchronous. */
int te_encode_batch_host(te_clay *c, const te_slicer_cfg *cfg, const uint8_t *h_data,
                         const te_object *objs, size_t nobj, uint8_t *h_out, size_t window_bytes);
/* The same over several handles (typically one per device): objects are split into contiguous
 * ranges by bytes, one host thread per handle, each running te_encode_batch_host on its range.
 * The first error (by handle order) is returned.  Synchronous. */
int te_encode_batch_host_multi(te_clay *const *coders, size_t ncoders, const te_slicer_cfg *cfg,
                               const uint8_t *h_data, const te_object *objs, size_t nobj, uint8_t *h_out,
                               size_t window_bytes);
/* Host only: the split te_encode_batch_host_multi uses.  cuts[0..nparts] (nparts + 1 entries):
 * part p encodes objects [cuts[p], cuts[p+1]); contiguous, covering, by about equal input bytes
 * (blob_len + 1 per object).  Parts may be empty when nobj < nparts. */
int te_balance_object_ranges(const te_object *objs, size_t nobj, size_t nparts, size_t *cuts);
/* te_encode_batch_host plus the slice commitments of BlobEncoder::encode_with_proofs
 * (sdk/src/codec/encoder.rs:220-260; the stream writer's per-chunk step, sdk/src/stream/write.rs:
 * 332-362): per object o, leaf hashes hash_leaf(slice i) at h_leaf_hashes + (o*n + i)*32, the
 * root root_from_leaf_hashes::<height> at h_roots + o*32 and, if h_proofs is not NULL, proof i
 * (create_proof_from_leaf_hashes::<height>) at h_proofs + ((o*n + i)*height + level)*32.
 * Hashed on the device from the slices in HBM while they are copied out: objects go through the
 * device in groups of at most `window_bytes` (input + output; 0 = 4 GiB; three groups resident),
 * each copied in windows of <= 128 MiB, and one leaf launch hashes a whole group (its time is
 * one slice's SHA-256 whatever the group size, so groups are large).  The handle keeps the three
 * group buffers allocated between calls (te_clay_free frees them).  Requires
 * n <= 2^height, height <= 32 and slice_len % 4 == 0 (every Clay profile with even alpha).
 * Synchronous; objects keep their order. */
int te_encode_commit_batch_host(te_clay *c, const te_slicer_cfg *cfg, const uint8_t *h_data,
                                const te_object *objs, size_t nobj, uint8_t *h_out, uint32_t height,
                                uint8_t *h_leaf_hashes, uint8_t *h_roots, uint8_t *h_proofs,
                                size_t window_bytes);

/* Ordered, asynchronous window submission: the stream writer's encode stage
 * (sdk/src/stream/write.rs:332-362 keeps up to min(cores, 4) chunk encodes in flight and hands them
 * on in order through FuturesOrdered) as one GPU pipeline per handle.
 *   te_stream_writer_new: over ncoders device-bound handles (one per GPU); window t goes to handle
 *     (t - 1) mod ncoders.  Consecutive windows share a hashing group of at most group_bytes
 *     (input + output; 0 = 8 GiB), hashed once it holds half of that (one leaf launch costs one
 *     slice's SHA-256, ~29 ms, whatever the group size), three groups resident per handle.  The
 *     writer owns its device buffers and runs on the handles' own streams; the handles must
 *     outlive it and must not be re-bound to another device meanwhile.
 *   te_stream_submit: enqueue one window -- te_encode_commit_batch_host's outputs for its objects
 *     (slices at h_out + out_off, leaf hashes, roots, proofs if h_proofs is not NULL) -- and return
 *     its ticket (1, 2, ... in submission order) without waiting for the device: window t+1's
 *     encode overlaps window t's hashing and copies.  Every host buffer of the window must stay
 *     valid (pinned for full overlap) until te_stream_wait has returned for its ticket.
 *   te_stream_wait: complete every window up to `ticket`, in submission order (a window whose
 *     hashing group is still open has it hashed now); returns the first failure among the
 *     windows it completes (TE_OK if none).
 *   te_stream_writer_free: waits for every window, then frees the writer. */
typedef struct te_stream_writer te_stream_writer;
int te_stream_writer_new(te_clay *const *coders, size_t ncoders, const te_slicer_cfg *cfg, uint32_t height,
                         size_t group_bytes, te_stream_writer **out);
int te_stream_submit(te_stream_writer *w, const uint8_t *h_data, const te_object *objs, size_t nobj, uint8_t *h_out,
                     uint8_t *h_leaf_hashes, uint8_t *h_roots, uint8_t *h_proofs, uint64_t *ticket);
int te_stream_wait(te_stream_writer *w, uint64_t ticket);
void te_stream_writer_free(te_stream_writer *w);

/* Who computes the leaf hashes of te_encode_commit_batch_host / te_stream_submit.  SHA-256 is
 * sequential within a slice, so the device hashes one slice per lane (~24 MB/s per lane, one leaf
 * launch ~ one slice's hash time): it wins for groups of many short slices (batches of 4 MiB
 * objects).  The SDK's stream shape -- 64 MiB chunks (MAX_TRACK_SIZE, sdk/src/stream/manifest.rs:22),
 * <= 4 encodes in flight (sdk/src/stream/write.rs:54-57), 9.7 MB slices -- is hashed faster by
 * host cores, as the SDK does (sdk/src/codec/encoder.rs:220-234): the slices are hashed from the
 * host output buffer by a worker pool (x86 SHA extensions when present) as soon as their D2H copy
 * has landed.  TE_HASH_AUTO picks per window (stream writer) or per group (one-shot call) from the
 * slice count, slice length and pool size; the results are identical either way. */
#define TE_HASH_AUTO 0
#define TE_HASH_DEVICE 1
#define TE_HASH_HOST 2
int te_set_commit_hashing(int mode);  /* process default (writers copy it when created) */
int te_stream_writer_set_hashing(te_stream_writer *w, int mode);
/* Host hashing pool size (0 = default: min(16, CPUs in this process's affinity mask)); waits
 * until the pool is idle. */
int te_set_host_hash_threads(int threads);
int te_host_hash_threads(void);
int te_host_sha_extensions(void);     /* 1 if the host SHA-256 uses the CPU's SHA extensions */
double te_host_hash_rate(void);       /* one pool thread's leaf-hash rate, bytes/s (measured at start) */
/* Slices one pool task hashes together, interleaved round by round (1..4): the lane count whose
 * measured per-thread rate is best on this host (a lone SHA-256 chain leaves the CPU's SHA unit
 * idle between dependent rounds). */
int te_host_hash_lanes(void);

/* Page-locked host memory for the host <-> device entry points (te_encode_*_host, te_stream_submit,
 * the per-call te_slicer_* / te_clay_* calls): copies from it run at full PCIe rate and need no
 * driver staging.  The callers of lib/slicer pass pageable Vec<u8>s (sdk/src/track/write.rs:273-308,
 * network/node/src/features/spool/repair.rs:312-339); a binding fills buffers from here instead
 * (rust/tape-slicer-gpu PinnedBuf), or pins an existing allocation in place with te_host_register.
 * Portable: pinned for every device.  Need a HIP device (TE_ERR_NO_DEVICE otherwise). */
int te_host_alloc(size_t bytes, void **out);
void te_host_free(void *p);
int te_host_register(void *p, size_t bytes);
int te_host_unregister(void *p);

typedef struct te_decode_object {
    uint64_t slices_off;  /* slice i at d_slices + slices_off + i*slice_len */
    uint64_t slice_len;
    uint32_t avail_mask;  /* bit i set = slice i present */
    uint32_t pad_;
    uint64_t out_off;     /* blob bytes written at d_out + out_off */
} te_decode_object;
/* Batched Slicer::decode.  Metadata is read on the host from `h_meta` (nobj*48 bytes: one
 * suffix per object, as the caller already holds them); no device->host sync is needed. */
int te_decode_batch_device(te_clay *c, const te_slicer_cfg *cfg, const uint8_t *d_slices,
                           const te_decode_object *objs, const uint8_t *h_meta, size_t nobj,
                           uint8_t *d_out, void *hip_stream);

typedef struct te_repair_object {
    const te_repair_plan *plan;
    uint64_t helper_off[TE_GROUP_SIZE]; /* extract_repair_data output of slice i at d_helpers+off */
    uint64_t out_off;                   /* num_stripes*chunk_size + 48 bytes at d_out + out_off */
    uint8_t metadata[TE_META_SIZE];
} te_repair_object;
/* Batched Slicer::repair of nobj lost slices (each with its own plan). */
int te_repair_batch_device(te_clay *c, const uint8_t *d_helpers, const te_repair_object *objs,
                           size_t nobj, uint8_t *d_out, void *hip_stream);

typedef struct te_recover_object {
    uint64_t slices_off;  /* peer slice i at d_slices + slices_off + i*slice_len (if in avail_mask) */
    uint64_t slice_len;
    uint32_t avail_mask;  /* bit i set = slice i present (>= k of them) */
    uint32_t lost;        /* slice index to rebuild */
    uint64_t out_off;     /* the rebuilt slice (slice_len bytes) at d_out + out_off */
} te_recover_object;
/* Batched node recover, network/node/src/features/spool/recover.rs:411-442 `reconstruct`
 * (SURVEY §8f-2): Slicer::decode from the peer slices, Slicer::encode of the object with the
 * peers' chunk_index, keep slice `lost`.  h_meta: one 48-byte suffix per object (host). */
int te_recover_batch_device(te_clay *c, const te_slicer_cfg *cfg, const uint8_t *d_slices,
                            const te_recover_object *objs, const uint8_t *h_meta, size_t nobj,
                            uint8_t *d_out, void *hip_stream);

/* ------------------------------------------------------------------------------------------
 * Slice commitments: BlobEncoder::encode_with_proofs' step after encode
 * (sdk/src/codec/encoder.rs:226-234) -- hash_leaf per slice, the merkle root and a proof per
 * slice -- from lib/crypto/src/merkle/tree.rs.  Hashes are 32-byte SHA-256 digests.
 * ------------------------------------------------------------------------------------------ */
#define TE_HASH_SIZE 32
#define TE_SLICE_TREE_HEIGHT 5          /* SLICE_TREE_HEIGHT      lib/core/src/erasure.rs:9  */
#define TE_MAX_MERKLE_TREE_HEIGHT 32    /* MAX_MERKLE_TREE_HEIGHT tree.rs:6                  */
#define TE_COMMIT_MAX_LEAVES 64         /* leaves per object in te_commit_batch_device       */

/* hash_leaf (tree.rs:53-56): SHA-256("LEAF" || data).  Host. */
int te_hash_leaf(const uint8_t *data, size_t len, uint8_t out[TE_HASH_SIZE]);
/* hash_leaf of `count` messages of `len` bytes each at data + i*len (an object's slices, as
 * encoder.rs:226-229 hashes them one by one) into out + i*32, `lanes` (1..4; 0 = te_host_hash_lanes)
 * of them interleaved on the calling thread.  Host. */
int te_hash_leaves(const uint8_t *data, size_t len, size_t count, uint32_t lanes, uint8_t *out);
/* hash_pair (tree.rs:58-62): SHA-256("LEFT" || left || "RIGHT" || right).  Host. */
int te_hash_pair(const uint8_t left[TE_HASH_SIZE], const uint8_t right[TE_HASH_SIZE], uint8_t out[TE_HASH_SIZE]);
/* empty_subtree_root / EMPTY_ROOTS[height] (tree.rs:15-48, 64-68), height < 32.  Host. */
int te_empty_subtree_root(uint32_t height, uint8_t out[TE_HASH_SIZE]);
/* root_from_leaf_hashes::<height> (tree.rs:344-350): count <= 2^height (else TREE_FULL). */
int te_merkle_root_from_leaf_hashes(const uint8_t *hashes, size_t count, uint32_t height, uint8_t out[TE_HASH_SIZE]);
/* create_proof_from_leaf_hashes::<height> (tree.rs:353-358, 397-455): `height` hashes. */
int te_merkle_proof_from_leaf_hashes(const uint8_t *hashes, size_t count, size_t index, uint32_t height,
                                     uint8_t *proof_out);
/* verify_proof (tree.rs:462-481) over a pre-hashed leaf: 1 valid, 0 not valid. */
int te_merkle_verify_leaf_hash(const uint8_t leaf_hash[TE_HASH_SIZE], const uint8_t root[TE_HASH_SIZE],
                               const uint8_t *proof, size_t proof_len, uint64_t index, uint32_t height);
/* Batched commitments on the device (DEVICE pointers, enqueued on hip_stream): object o's n
 * slices at d_slices + o*obj_stride + i*slice_len (slice_len % 4 == 0, n <= 64) ->
 * leaf hashes d_leaf_hashes[(o*n + i)*32], roots d_roots[o*32] (NULL: leaves only), proofs
 * d_proofs[((o*n + i)*height + level)*32] (NULL: none). */
int te_commit_batch_device(const uint8_t *d_slices, uint64_t obj_stride, uint64_t slice_len, uint32_t n,
                           size_t nobj, uint32_t height, uint8_t *d_leaf_hashes, uint8_t *d_roots,
                           uint8_t *d_proofs, void *hip_stream);

/* ------------------------------------------------------------------------------------------
 * OuterCoder (lib/slicer/src/outer.rs:19-197): single-level Reed-Solomon over
 * GF(2^16) in the Leopard construction of reed-solomon-simd 3.1.0 (parity unpinned: the crate
 * is not in the container).  n chunks, any k reconstruct; chunks 0..k-1 are the
 * data (systematic), k..n-1 the crate's recovery shards.  Chunk bytes are 64-byte aligned
 * (outer.rs:74-80), at most TE_OUTER_MAX_CHUNK_BYTES.
 * ------------------------------------------------------------------------------------------ */
#define TE_OUTER_MAX_CHUNK_BYTES (4u * 1024u * 1024u)  /* MAX_CHUNK_BYTES  outer.rs:12 */
/* chunk size for `len` data bytes: ceil(len / k) rounded up to 64, 64 for empty data. */
size_t te_outer_chunk_bytes(uint32_t k, size_t len);
/* OuterCoder::encode (outer.rs:70-118): out = n chunks of *chunk_bytes (data zero-padded to
 * k * chunk_bytes, then the n - k recovery chunks, computed on the GPU).  TE_ERR_TOO_MUCH_DATA
 * past the chunk limit; TE_ERR_UNSUPPORTED for shard counts the codec does not support. */
int te_outer_encode(uint32_t k, uint32_t n, const uint8_t *data, size_t len, uint8_t *out, size_t cap,
                    size_t *chunk_bytes);
/* OuterCoder::decode (outer.rs:126-197): chunks[i] for i < n (NULL = missing), all chunk_bytes
 * long; out = the k data chunks (k * chunk_bytes, data padding included).  Missing data chunks
 * are restored on the GPU from k received chunks.  TE_ERR_NOT_ENOUGH_SLICES below k chunks. */
int te_outer_decode(uint32_t k, uint32_t n, const uint8_t *const *chunks, size_t chunk_bytes, uint8_t *out,
                    size_t cap);
/* Batched device form of the encode (DEVICE pointers): `segments` segments, segment g's k
 * original shards at d_in + g*seg_in (shard j at + j*chunk_bytes), its m = n - k recovery shards
 * to d_out + g*seg_out (shard j at + j*chunk_bytes).  Runs on hip_stream and waits for it. */
int te_outer_encode_device(uint32_t k, uint32_t m, const uint8_t *d_in, uint64_t chunk_bytes, uint32_t segments,
                           uint64_t seg_in, uint8_t *d_out, uint64_t seg_out, void *hip_stream);
/* Device form of the decode (outer.rs:126-197) for snapshot reads: d_chunks = n DEVICE pointers
 * (host array; NULL = missing), each chunk_bytes long; d_out = the k data chunks (DEVICE,
 * k * chunk_bytes).  Received data chunks are copied, missing ones restored from the first k
 * received chunks on the GPU.  Enqueued on hip_stream; returns without waiting (the d_chunks
 * array is read before it returns).  The decoding tables are cached per erasure pattern. */
int te_outer_decode_device(uint32_t k, uint32_t n, const uint8_t *const *d_chunks, uint64_t chunk_bytes,
                           uint8_t *d_out, void *hip_stream);
/* The same for `segments` segments in one call (a snapshot read): segment g's chunk i at
 * d_chunks[g * n + i] (host array of DEVICE pointers, NULL = missing), its k data chunks to
 * d_out + g * seg_out.  Segments sharing an erasure pattern share launches (up to 256 shard
 * pointers each).  seg_out >= k * chunk_bytes when segments > 1 (TE_ERR_INVALID_ARG otherwise).
 * Every segment is validated before anything is enqueued.  Enqueued on hip_stream; returns
 * without waiting. */
int te_outer_decode_device_batch(uint32_t k, uint32_t n, const uint8_t *const *d_chunks, uint32_t segments,
                                 uint64_t chunk_bytes, uint8_t *d_out, uint64_t seg_out, void *hip_stream);

#ifdef __cplusplus
}
#endif
#endif /* TAPE_EC_H */
