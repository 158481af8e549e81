// engine.cpp -- libtapeec.so: the C ABI (include/tape_ec.h) over the gfx950 Clay engines.
//
// Host side of the drop-in for lib/slicer: Slicer striping/padding/rotation/metadata
// (slicer.rs, adaptive.rs, metadata.rs), repair planning (repair.rs), descriptor building and
// launch orchestration.  All GF arithmetic and hashing runs in the HIP kernels (encode_dma.hip,
// encode_stage.hip, decode_stage.hip + the per-pattern kernels of dec_rtc.cpp, repair_fold.hip,
// repair_stage.hip, gpe.hip, commit.hip, rs16.hip); there is no CPU compute fallback -- without a
// device the compute calls fail with TE_ERR_NO_DEVICE.
#include <hip/hip_runtime.h>
#include <string.h>
#include <stdio.h>
#include <stdlib.h>
#include <deque>
#include <map>
#include <unordered_map>
#include <mutex>
#include <vector>
#include <algorithm>
#include <functional>
#include <thread>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include "../../include/tape_ec.h"
#include "kernels.hpp"
#include "sha256.hpp"
#include <array>
#include "clay_host.hpp"
#include "rs16.hpp"
#include "host_hash.hpp"
#include "copy_pool.hpp"
#include "dec_class.hpp"

using namespace tec;

namespace {

constexpr size_t kStripeSizes[3] = {100000, 1000000, 10000000};  // adaptive.rs:15-19

thread_local char g_last_error[256] = "";
// TEC_ENCODE_KERNEL=stage selects the previous 1 MB-stripe encode kernel (measurement only)
const bool g_no_dma_encode = [] {
    const char *e = tec_knob("TEC_ENCODE_KERNEL");
    return e && strcmp(e, "stage") == 0;
}();

// Small per-call encodes (te_slicer_encode / te_clay_encode): a call of at most TEC_ENC_SMALL 1 MB
// stripes may run the staged kernel with one wave per workgroup (six workgroups per stripe).
// Measured slower (r05 trace of --mode percall: 438 us per 4 MiB object against 296 us for the
// LDS-DMA kernel -- a lone stripe is bound by the 100-plane chain's latency, not its work per
// step), so it is off (0); measurement only.
// Per-call encodes of at most this many 1 MB stripes run the LDS-DMA kernel split in two launches:
// the seven level-1 plane rows of a stripe on seven workgroups, then the level-2 chain on one --
// a lone stripe is latency-bound by its 100-plane chain (296 us per 4 MiB object).  Measurement
// option TEC_DEBUG_KNOBS=1 TEC_ENC_SPLIT=n (0: never).
const uint32_t g_enc_split = [] {
    const char *e = tec_knob("TEC_ENC_SPLIT");
    return e ? (uint32_t)atoi(e) : 512u;
}();
// Measurement option TEC_DEBUG_KNOBS=1 TEC_ENC_SPLIT_BATCH=1: every call split that way (the seven
// level-1 workgroups of a stripe run side by side on one XCD, so a row one of them reads as its
// own and another as a partner is read twice at about the same time).
const uint32_t g_enc_split_batch = [] {  // 0 off, else the level-1 rows per workgroup (1..7)
    const char *e = tec_knob("TEC_ENC_SPLIT_BATCH");
    const int v = e ? atoi(e) : 0;
    return (uint32_t)(v < 0 ? 0 : v > 7 ? 7 : v);
}();
const uint32_t g_enc_small = [] {
    const char *e = tec_knob("TEC_ENC_SMALL");
    return e ? (uint32_t)atoi(e) : 0u;
}();

// TEC_REPAIR_KERNEL=stage keeps the folded repair kernel off (measurement / cross-check only)
const bool g_no_fold_repair = [] {
    const char *e = tec_knob("TEC_REPAIR_KERNEL");
    return e && strcmp(e, "stage") == 0;
}();

int hip_status(hipError_t e) {
    if (e == hipSuccess) return TE_OK;
    snprintf(g_last_error, sizeof(g_last_error), "%s (%d)", hipGetErrorString(e), (int)e);
    if (e == hipErrorOutOfMemory) return TE_ERR_OUT_OF_MEMORY;
    if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return TE_ERR_NO_DEVICE;
    return TE_ERR_HIP;
}

#define TE_HIP(expr)                              \
    do {                                          \
        hipError_t e_ = (expr);                   \
        if (e_ != hipSuccess) return hip_status(e_); \
    } while (0)

// Wait for the work queued on s so far by sleeping on a blocking-sync event, not spinning in
// hipStreamSynchronize: a caller that waits while the host hashing pool runs must not take one of
// the process's CPUs (the GPU's host share is a 16-CPU quota on the pool this runs on).
int sync_sleep(hipStream_t s) {
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventBlockingSync) != hipSuccess)
        return hip_status(hipStreamSynchronize(s));
    hipError_t r = hipEventRecord(e, s);
    if (r == hipSuccess) r = hipEventSynchronize(e);
    (void)hipEventDestroy(e);
    return hip_status(r);
}

int g_device_count = -1;
std::mutex g_dev_mu;

int device_count() {
    std::lock_guard<std::mutex> lk(g_dev_mu);
    if (g_device_count < 0) {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
        g_device_count = n;
    }
    return g_device_count;
}

// Runs the enclosed calls on a handle's device, whatever the calling thread's current device
// is, and restores the thread's device afterwards.
struct DeviceGuard {
    int prev = -1;
    hipError_t err = hipSuccess;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) err = hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

// Measurement option (TEC_DEBUG_KNOBS=1 TEC_VMM_BUFS=1): buffers of >= 64 MiB through the virtual
// memory API -- physical memory created at the recommended granularity and mapped into a fresh
// address range -- instead of hipMalloc (to test whether a slowdown follows the page placement of
// re-allocated buffers, DESIGN §4.4's open item).
static bool vmm_bufs() {
    static const bool v = [] {
        const char *s = tec_knob("TEC_VMM_BUFS");
        return s && s[0] == '1';
    }();
    return v;
}

// The last launches that read a shared device resource, one event per stream: each
// call re-records its own stream's event, so a clear / free waits for the readers on EVERY stream
// that used the resource, not only the most recent one.  Bounded: past kMax streams the events are
// drained on the host and their slots reused (a process rarely reads one handle from > 16 streams).
struct ReaderEvents {
    struct E {
        hipStream_t s = nullptr;
        hipEvent_t ev = nullptr;
        bool pending = false;
    };
    static constexpr size_t kMax = 16;
    std::vector<E> v;
    bool any() const {
        for (const E &e : v)
            if (e.pending) return true;
        return false;
    }
    // after the launches on `s` that read the resource
    hipError_t record(hipStream_t s) {
        E *slot = nullptr;
        for (E &e : v)
            if (e.s == s) slot = &e;
        if (!slot) {
            if (v.size() >= kMax) {
                if (hipError_t r = sync(); r != hipSuccess) return r;
                slot = &v[0];
                slot->s = s;
            } else {
                E e;
                e.s = s;
                if (hipError_t r = hipEventCreateWithFlags(&e.ev, hipEventDisableTiming); r != hipSuccess) return r;
                v.push_back(e);
                slot = &v.back();
            }
        }
        hipError_t r = hipEventRecord(slot->ev, s);
        if (r == hipSuccess) slot->pending = true;
        return r;
    }
    // stream `s` waits (on the device) for every reader on the other streams
    hipError_t wait(hipStream_t s) const {
        for (const E &e : v)
            if (e.pending && e.s != s)
                if (hipError_t r = hipStreamWaitEvent(s, e.ev, 0); r != hipSuccess) return r;
        return hipSuccess;
    }
    // the host waits for every reader (before the resource is freed)
    hipError_t sync() {
        for (E &e : v)
            if (e.pending) {
                if (hipError_t r = hipEventSynchronize(e.ev); r != hipSuccess) return r;
                e.pending = false;
            }
        return hipSuccess;
    }
    void destroy() {
        for (E &e : v)
            if (e.ev) (void)hipEventDestroy(e.ev);
        v.clear();
    }
};

// One copy pool per device, so per-call copies of handles on different GPUs do not queue behind
// one another.  Three workers plus the calling thread.
static tec::CopyPool &copy_pool(int device) {
    static std::mutex mu;
    static tec::CopyPool *pools[65] = {};
    const int slot = device < 0 || device >= 64 ? 64 : device;
    std::lock_guard<std::mutex> g(mu);
    if (!pools[slot]) pools[slot] = new tec::CopyPool(std::max(0, std::min(3, hh::default_threads() - 1)));
    return *pools[slot];
}

struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    hipMemGenericAllocationHandle_t vh{};  // VMM allocation (vmm_bufs), else hipMalloc
    bool vmm = false;
    hipError_t free_() {
        if (!p) return hipSuccess;
        hipError_t e = hipSuccess;
        if (vmm) {
            (void)hipDeviceSynchronize();
            e = hipMemUnmap(p, cap);
            if (e == hipSuccess) e = hipMemRelease(vh);
            if (e == hipSuccess) e = hipMemAddressFree(p, cap);
        } else {
            e = hipFree(p);
        }
        p = nullptr;
        cap = 0;
        vmm = false;
        return e;
    }
    hipError_t alloc_vmm(size_t n) {
        int dev = 0;
        hipError_t e = hipGetDevice(&dev);
        if (e != hipSuccess) return e;
        hipMemAllocationProp prop{};
        prop.type = hipMemAllocationTypePinned;
        prop.location.type = hipMemLocationTypeDevice;
        prop.location.id = dev;
        size_t g = 0;
        if ((e = hipMemGetAllocationGranularity(&g, &prop, hipMemAllocationGranularityRecommended)) != hipSuccess) return e;
        if (g == 0) g = (size_t)2 << 20;
        const size_t sz = (n + g - 1) / g * g;
        void *va = nullptr;
        if ((e = hipMemAddressReserve(&va, sz, g, nullptr, 0)) != hipSuccess) return e;
        hipMemGenericAllocationHandle_t h{};
        if ((e = hipMemCreate(&h, sz, &prop, 0)) != hipSuccess) {
            (void)hipMemAddressFree(va, sz);
            return e;
        }
        if ((e = hipMemMap(va, sz, 0, h, 0)) != hipSuccess) {
            (void)hipMemRelease(h);
            (void)hipMemAddressFree(va, sz);
            return e;
        }
        hipMemAccessDesc ad{};
        ad.location = prop.location;
        ad.flags = hipMemAccessFlagsProtReadWrite;
        if ((e = hipMemSetAccess(va, sz, &ad, 1)) != hipSuccess) {
            (void)hipMemUnmap(va, sz);
            (void)hipMemRelease(h);
            (void)hipMemAddressFree(va, sz);
            return e;
        }
        p = va;
        cap = sz;
        vh = h;
        vmm = true;
        return hipSuccess;
    }
    hipError_t ensure(size_t n) {
        if (n <= cap) return hipSuccess;
        if (p) {
            hipError_t e = free_();
            if (e != hipSuccess) return e;
        }
        if (vmm_bufs() && n >= ((size_t)64 << 20)) return alloc_vmm(n);
        // large buffers in whole 2 MiB units (the device's large-page size)
        size_t want = std::max<size_t>(n, 4096);
        const size_t unit = want >= ((size_t)64 << 20) ? ((size_t)2 << 20) : 4096;
        want = (want + unit - 1) & ~(unit - 1);
        hipError_t e = hipMalloc(&p, want);
        if (e != hipSuccess) { p = nullptr; return e; }
        cap = want;
        return hipSuccess;
    }
    template <class T> T *as() const { return reinterpret_cast<T *>(p); }
    void release() { (void)free_(); }
};

struct HostBuf {  // pinned staging (descriptor uploads, the per-call entry points' host side)
    void *p = nullptr;
    size_t cap = 0;
    uint8_t *u8() const { return static_cast<uint8_t *>(p); }
    hipError_t ensure(size_t n) {
        if (n <= cap) return hipSuccess;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        size_t want = std::max<size_t>(n, 4096);
        hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
        if (e != hipSuccess) { p = nullptr; return e; }
        cap = want;
        return hipSuccess;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
    }
};

// A descriptor arena: host image assembled per call, uploaded (only if changed) to a device
// mirror on the caller's stream.  An event guards the pinned staging against reuse while a
// previous upload may still be pending.
struct Arena {
    std::vector<uint8_t> img, last;
    HostBuf stage;
    DevBuf dev;
    DevBuf scratch;  // kernel workspace (encode level-2 parking), ordered like `dev`
    hipEvent_t ev = nullptr;
    bool ev_pending = false;
    hipStream_t last_stream = nullptr;
    hipEvent_t done = nullptr;  // recorded after the launches that read `dev`
    bool done_pending = false;

    size_t put(const void *src, size_t bytes, size_t align = 16) {
        size_t off = (img.size() + align - 1) & ~(align - 1);
        img.resize(off + bytes);
        if (bytes) memcpy(img.data() + off, src, bytes);
        return off;
    }
    int upload(hipStream_t s) {
        if (!ev) TE_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        if (!done) TE_HIP(hipEventCreateWithFlags(&done, hipEventDisableTiming));
        if (img == last && dev.p && dev.cap >= img.size()) return TE_OK;
        // device mirror may still be read by launches on another stream
        if (done_pending && last_stream != s) TE_HIP(hipStreamWaitEvent(s, done, 0));
        if (ev_pending) TE_HIP(hipEventSynchronize(ev));
        ev_pending = false;
        if (img.size() > dev.cap) {
            // old mirror may still be referenced by queued kernels: drain before freeing
            if (done_pending) TE_HIP(hipEventSynchronize(done));
            TE_HIP(dev.ensure(img.size()));
        }
        TE_HIP(stage.ensure(img.size()));
        memcpy(stage.p, img.data(), img.size());
        TE_HIP(hipMemcpyAsync(dev.p, stage.p, img.size(), hipMemcpyHostToDevice, s));
        TE_HIP(hipEventRecord(ev, s));
        ev_pending = true;
        last = img;
        return TE_OK;
    }
    int mark_done(hipStream_t s) {
        TE_HIP(hipEventRecord(done, s));
        done_pending = true;
        last_stream = s;
        return TE_OK;
    }
    template <class T> const T *at(size_t off) const { return reinterpret_cast<const T *>(dev.as<uint8_t>() + off); }
    // workspace of at least `bytes` for launches about to be enqueued on stream s
    int workspace(size_t bytes, hipStream_t s, uint8_t **out) {
        if (bytes > scratch.cap) {
            if (done_pending) TE_HIP(hipEventSynchronize(done));  // queued kernels may still use it
            TE_HIP(scratch.ensure(bytes));
        } else if (done_pending && last_stream != s) {
            TE_HIP(hipStreamWaitEvent(s, done, 0));
        }
        *out = scratch.as<uint8_t>();
        return TE_OK;
    }
    void release() {
        dev.release();
        scratch.release();
        stage.release();
        if (ev) (void)hipEventDestroy(ev);
        if (done) (void)hipEventDestroy(done);
        ev = done = nullptr;
    }
};

// Kernel timing (te_kernel_timing): event pairs around each batch call's kernel launches.
struct KTimeState {
    std::mutex mu;
    bool enabled = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> pairs;
} g_ktime;

struct KTimer {
    hipEvent_t a = nullptr, b = nullptr;
    hipStream_t s;
    explicit KTimer(hipStream_t st) : s(st) {
        std::lock_guard<std::mutex> g(g_ktime.mu);
        if (!g_ktime.enabled) return;
        if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess || hipEventRecord(a, s) != hipSuccess) {
            a = b = nullptr;
        }
    }
    ~KTimer() {
        if (a) (void)hipEventDestroy(a);
        if (b) (void)hipEventDestroy(b);
    }
    void stop() {
        if (!a) return;
        std::lock_guard<std::mutex> g(g_ktime.mu);
        if (hipEventRecord(b, s) == hipSuccess) g_ktime.pairs.push_back({a, b});
        a = b = nullptr;
    }
};

void put_u64(uint8_t *p, uint64_t v) {
    for (int i = 0; i < 8; i++) p[i] = (uint8_t)(v >> (8 * i));
}
uint64_t get_u64(const uint8_t *p) {
    uint64_t v = 0;
    for (int i = 0; i < 8; i++) v |= (uint64_t)p[i] << (8 * i);
    return v;
}

bool valid_stripe(uint64_t s) { return s == kStripeSizes[0] || s == kStripeSizes[1] || s == kStripeSizes[2]; }

}  // namespace

// ------------------------------------------------------------------------------------------
struct te_clay {
    ClayHost h;
    bool fast_encode = false;
    std::mutex mu;
    int device = 0;                // every allocation and launch of this handle runs on it
    hipStream_t stream = nullptr;  // for the synchronous host-buffer entry points
    Arena enc, dec, rep, rec;
    DevBuf io_in, io_out;          // staging for host-buffer entry points
    HostBuf hio_in, hio_out;       // their page-locked host side (te_slicer_repair's gather / scatter)
    // te_recover_batch_device workspaces (decoded objects, re-encoded slices); `rec_done` is
    // recorded after the last launch that reads them, on `rec_stream`
    DevBuf rec_blob, rec_slices;
    hipEvent_t rec_done = nullptr;
    bool rec_pending = false;
    hipStream_t rec_stream = nullptr;
    // te_encode_batch_host pipeline: kPipe slots, each with its own stream, descriptor arena
    // and device window buffers, so window w+1's H2D overlaps window w's kernel and D2H.
    static constexpr int kPipe = 3;  // a fourth slot measured slower
    // Compiled decode patterns (layered pattern + staged plane program), by padded erasure mask:
    // building them is host work per distinct pattern (matrix inversion, program, colouring).
    struct DecCache {
        GpePattern P;
        std::vector<uint16_t> planes;  // P's plane list (P.planes_off is set per call)
        bool staged = false;           // a plane program exists for the staged kernel
        DecProgHdr H{};
        std::vector<DecStepP> steps;   // packed program + 2 blank steps
        int orient = 0;                // the program's row orientation (ClayHost::dec_prog)
    };
    // Device-resident store of staged decode patterns (GpePattern, DecProgHdr, program) by
    // cache key: a pattern is uploaded once and serves later calls in place.  Random survivor
    // sets make nearly every stripe a pattern of its own, and re-uploading ~26 KB per stripe per
    // call cost more host time than the kernel takes.  Slots are handed out in order; a full store
    // is emptied after its last reader (`used`) has finished.
    // The store grows by doubling from kMin slots (each slot ~26 KB of device memory: 102 steps
    // of DecStepP plus its GpePattern and header; kCap slots = ~430 MB; te_clay_set_decode_store_cap
    // lowers the cap) once its last reader is done.  New slots are filled with stream-ordered copies from the call's descriptor upload
    // (decode_enqueue), never with a host-blocking copy; a call on another stream waits for the
    // last fill (`written`) before reading.
    struct DecStore {
        // 16,384: a batch of 2,048 x 4 MiB reads with random survivor sets has ~10,000 distinct
        // stripe patterns; at 8,192 every such call overflowed to per-call uploads and recompiles
        static constexpr uint32_t kCap = 16384, kMin = 256;
        uint32_t max_cap = kCap;
        static constexpr uint32_t kSteps = kRepQ * kRepQ + 2;  // 100 planes + 2 blank steps
        DevBuf pats, hdrs, steps, soff;
        uint32_t cap = 0;
        std::unordered_map<uint64_t, uint32_t> slot;
        uint32_t n = 0;
        ReaderEvents readers;             // the last launches that read the store, per stream
        hipEvent_t written = nullptr;
        bool written_pending = false;
        hipStream_t written_stream = nullptr;
        uint64_t clears = 0, grows = 0, arena_calls = 0;  // te_clay_decode_store_stats
    } dstore;
    // per-pattern decode kernels built at run time (dec_rtc.cpp); created on first decode
    DecJit *jit = nullptr;
    int jit_mode = -1;                 // te_clay_set_decode_jit; -1 = the environment's default
    uint64_t jit_min = 0;
    std::unordered_map<uint64_t, DecCache> dec_cache;
    // Compiled repair patterns by (lost shard, helper shards...): the layered pattern with its
    // plane lists, the staged kernel's program, and the folded kernel index (-1: none).  Host work
    // per distinct helper set (matrix inversion, programs) is done once per handle.
    struct RepCache {
        RepPattern P;
        std::vector<uint16_t> pool, pind;
        RepProg prog{};
        bool prog_ok = false;
        int fold = -1;
    };
    struct RepKey {  // (lost shard, helper shard set): rep_pattern depends on the set only
        uint64_t helpers;
        uint32_t lost;
        bool operator==(const RepKey &o) const { return helpers == o.helpers && lost == o.lost; }
    };
    struct RepKeyHash {
        size_t operator()(const RepKey &k) const {
            return (size_t)((k.helpers ^ ((uint64_t)k.lost << 56)) * 0x9E3779B97F4A7C15ull >> 7);
        }
    };
    std::unordered_map<RepKey, RepCache, RepKeyHash> rep_cache;  // node-based: entries stay put
    struct Slot {
        hipStream_t s = nullptr;
        Arena arena;
        DevBuf in, out;
        DevBuf commit;  // te_encode_commit_batch_host: the window's leaf hashes, roots, proofs
    } pipe[kPipe];
    // encode + commit pipeline streams on disjoint CU sets (commit_streams): hashing on a few
    // CUs, slot streams (copies, encodes) on the rest
    hipStream_t cm_ss[2] = {}, cm_hs = nullptr;
    bool cm_tried = false;
    // decode class kernels run side by side (decode_enqueue): side streams forked from and joined
    // back into the call's stream with events, so their work is ordered like the call's
    static constexpr int kClsSide = 7;
    hipStream_t cls_s[kClsSide] = {};
    hipEvent_t cls_fork = nullptr, cls_join[kClsSide] = {};
};

// Drain and free everything a handle holds on its device (on that device).
static void release_device_state(te_clay *c) {
    if (device_count() <= 0) return;
    DeviceGuard dg(c->device);
    if (dg.err != hipSuccess) return;
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->rec_done) (void)hipEventSynchronize(c->rec_done);
    for (auto &sl : c->pipe)
        if (sl.s) (void)hipStreamSynchronize(sl.s);
    for (hipStream_t &cs : c->cls_s)
        if (cs) (void)hipStreamSynchronize(cs), (void)hipStreamDestroy(cs), cs = nullptr;
    if (c->cls_fork) (void)hipEventDestroy(c->cls_fork), c->cls_fork = nullptr;
    for (hipEvent_t &pe : c->cls_join)
        if (pe) (void)hipEventDestroy(pe), pe = nullptr;
    c->enc.release();
    c->dec.release();
    c->rep.release();
    c->rec.release();
    c->io_in.release();
    c->io_out.release();
    c->hio_in.release();
    c->hio_out.release();
    c->rec_blob.release();
    c->rec_slices.release();
    for (DevBuf *b : {&c->dstore.pats, &c->dstore.hdrs, &c->dstore.steps, &c->dstore.soff}) b->release();
    c->dstore.slot.clear();
    c->dstore.n = 0;
    c->dstore.readers.destroy();
    if (c->dstore.written) (void)hipEventDestroy(c->dstore.written);
    c->dstore.written = nullptr;
    c->dstore.written_pending = false;
    c->dstore.written_stream = nullptr;
    c->dstore.cap = 0;
    if (c->rec_done) (void)hipEventDestroy(c->rec_done);
    c->rec_done = nullptr;
    dec_jit_free(c->jit);  // joins compiles in flight; every stream is drained above
    c->jit = nullptr;
    c->rec_pending = false;
    if (c->stream) (void)hipStreamDestroy(c->stream);
    c->stream = nullptr;
    for (hipStream_t *ps : {&c->cm_ss[0], &c->cm_ss[1], &c->cm_hs}) {
        if (*ps) (void)hipStreamSynchronize(*ps), (void)hipStreamDestroy(*ps);
        *ps = nullptr;
    }
    c->cm_tried = false;
    for (auto &sl : c->pipe) {
        sl.arena.release();
        sl.in.release();
        sl.out.release();
        sl.commit.release();
        if (sl.s) (void)hipStreamDestroy(sl.s);
        sl.s = nullptr;
    }
}

struct te_repair_plan {
    uint32_t lost = 0, ns = 0, d = 0, beta = 0, n = 0;
    uint64_t cs = 0, sc = 0;
    std::vector<uint32_t> lost_shard;   // [ns]
    std::vector<uint32_t> helper_slice; // [ns*d]
    std::vector<uint32_t> helper_shard; // [ns*d]
    std::vector<uint32_t> sub_chunks;   // [ns*d*beta]
};

namespace tec {
hipError_t ensure_dyn_lds(const void *fn, size_t bytes) {
    static std::mutex mu;
    static std::map<std::pair<int, const void *>, size_t> done;  // (device, kernel) -> limit set
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> lk(mu);
    size_t &cur = done[{dev, fn}];
    if (bytes <= cur) return hipSuccess;
    e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e == hipSuccess) cur = bytes;
    return e;
}
}  // namespace tec

extern "C" {

const char *te_strerror(int s) {
    switch (s) {
        case TE_OK: return "ok";
        case TE_ERR_TOO_MUCH_DATA: return "too much data to encode in a single stripe/coder configuration";
        case TE_ERR_EMPTY_INPUT: return "empty input data";
        case TE_ERR_NOT_ENOUGH_SLICES: return "not enough slices to reconstruct (need at least DATA_SLICES)";
        case TE_ERR_BAD_ENCODING: return "invalid padding in recovered data";
        case TE_ERR_INVALID_LAYOUT: return "invalid layout or inconsistent slices";
        case TE_ERR_NOT_ENOUGH_HELPERS: return "not enough helpers";
        case TE_ERR_INVALID_SLICE: return "invalid slice index";
        case TE_ERR_CLAY: return "clay error";
        case TE_ERR_MISSING_HELPER: return "missing helper data";
        case TE_ERR_MERKLE_TREE_FULL: return "merkle tree full";
        case TE_ERR_MERKLE_INVALID_PROOF: return "invalid merkle proof";
        case TE_ERR_MERKLE_INVALID_INDEX: return "invalid merkle leaf index";
        case TE_ERR_MERKLE_PROOF_LENGTH: return "merkle proof length differs from the tree height";
        case TE_ERR_INVALID_ARG: return "invalid argument";
        case TE_ERR_NO_DEVICE: return "no gfx950 HIP device available (libtapeec has no CPU fallback)";
        case TE_ERR_HIP: return "HIP runtime error";
        case TE_ERR_UNSUPPORTED: return "profile/layout not supported by the GPU engine";
        case TE_ERR_OUT_OF_MEMORY: return "out of device memory";
        case TE_ERR_BUFFER_TOO_SMALL: return "output buffer too small";
    }
    return "unknown status";
}

int te_device_count(void) { return device_count(); }

const char *te_last_error_detail(void) { return g_last_error; }


int te_set_device(int device) {
    if (device < 0 || device >= device_count()) return TE_ERR_NO_DEVICE;
    TE_HIP(hipSetDevice(device));
    return TE_OK;
}

const char *te_version(void) { return "tapeec 0.1.0 (gfx950)"; }

int te_kernel_timing(int enable) {
    std::lock_guard<std::mutex> g(g_ktime.mu);
    g_ktime.enabled = enable != 0;
    return TE_OK;
}

int te_kernel_time_ms(double *total_ms, uint32_t *count) {
    if (!total_ms) return TE_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> g(g_ktime.mu);
    double tot = 0;
    for (auto &p : g_ktime.pairs) {
        TE_HIP(hipEventSynchronize(p.second));
        float ms = 0;
        TE_HIP(hipEventElapsedTime(&ms, p.first, p.second));
        tot += ms;
        (void)hipEventDestroy(p.first);
        (void)hipEventDestroy(p.second);
    }
    if (count) *count = (uint32_t)g_ktime.pairs.size();
    g_ktime.pairs.clear();
    *total_ms = tot;
    return TE_OK;
}

// ------------------------------------------------------------------------------------------
int te_clay_new(uint32_t n, uint32_t k, uint32_t d, te_clay **out) {
    if (!out) return TE_ERR_INVALID_ARG;
    *out = nullptr;
    if (n > TE_GROUP_SIZE) return TE_ERR_INVALID_ARG;
    te_clay *c = new (std::nothrow) te_clay();
    if (!c) return TE_ERR_OUT_OF_MEMORY;
    const int r = c->h.init((int)n, (int)k, (int)d);
    if (r) {
        delete c;
        return r == -1 ? TE_ERR_INVALID_ARG : TE_ERR_UNSUPPORTED;
    }
    c->fast_encode = encode_rows_supported((int)n, (int)k, (int)d);
    if (device_count() > 0) {  // bound to the creating thread's current device (te_clay_bind_device)
        int dev = 0;
        if (hipGetDevice(&dev) == hipSuccess) c->device = dev;
    }
    *out = c;
    return TE_OK;
}

int te_clay_bind_device(te_clay *c, int device) {
    if (!c) return TE_ERR_INVALID_ARG;
    if (device < 0 || device >= device_count()) return TE_ERR_NO_DEVICE;
    std::lock_guard<std::mutex> lk(c->mu);
    if (device == c->device) return TE_OK;
    release_device_state(c);  // buffers and streams live on the old device
    c->device = device;
    return TE_OK;
}

int te_clay_device(const te_clay *c) { return c ? c->device : -1; }

int te_clay_set_decode_jit(te_clay *c, int mode, uint64_t min_stripes) {
    if (!c || mode < 0 || mode > 2) return TE_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(c->mu);
    c->jit_mode = mode;
    c->jit_min = min_stripes;
    if (c->jit) dec_jit_set(c->jit, mode, min_stripes);
    return TE_OK;
}

int te_clay_set_decode_store_cap(te_clay *c, uint32_t max_patterns) {
    if (!c || max_patterns < 1 || max_patterns > te_clay::DecStore::kCap) return TE_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(c->mu);
    te_clay::DecStore &S = c->dstore;
    if (S.cap > max_patterns) {  // shrink: the store is re-allocated at the next decode
        (void)S.readers.sync();
        for (DevBuf *b : {&S.pats, &S.hdrs, &S.steps, &S.soff}) b->release();
        S.cap = 0;
        S.slot.clear();
        S.n = 0;
    }
    S.max_cap = max_patterns;
    return TE_OK;
}

int te_clay_decode_store_stats(te_clay *c, uint32_t *capacity, uint32_t *used, uint64_t *clears, uint64_t *grows,
                               uint64_t *arena_calls) {
    if (!c) return TE_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(c->mu);
    if (capacity) *capacity = c->dstore.cap;
    if (used) *used = c->dstore.n;
    if (clears) *clears = c->dstore.clears;
    if (grows) *grows = c->dstore.grows;
    if (arena_calls) *arena_calls = c->dstore.arena_calls;
    return TE_OK;
}

int te_clay_decode_jit_status(te_clay *c, uint32_t timeout_ms, uint32_t *ready, uint32_t *pending, uint32_t *failed) {
    if (!c) return TE_ERR_INVALID_ARG;
    DecJit *j;
    {
        std::lock_guard<std::mutex> lk(c->mu);
        j = c->jit;
        if (j) dec_jit_hold(j);  // dec_jit_free (te_clay_free / bind_device, under c->mu) waits for it
    }
    uint32_t r = 0, p = 0, f = 0;
    if (j) {
        dec_jit_counts(j, timeout_ms, &r, &p, &f);
        dec_jit_unhold(j);
    }
    if (ready) *ready = r;
    if (pending) *pending = p;
    if (failed) *failed = f;
    return TE_OK;
}

int te_clay_from_params(uint64_t p, te_clay **out) {
    return te_clay_new((uint32_t)(p & 0xFF), (uint32_t)((p >> 8) & 0xFF), (uint32_t)((p >> 16) & 0xFF), out);
}

void te_clay_free(te_clay *c) {
    if (!c) return;
    release_device_state(c);
    delete c;
}

int te_clay_get_info(const te_clay *c, te_clay_info *o) {
    if (!c || !o) return TE_ERR_INVALID_ARG;
    const ClayHost &h = c->h;
    o->n = h.n; o->k = h.k; o->m = h.m; o->d = h.d;
    o->q = h.q; o->t = h.t; o->nu = h.nu; o->alpha = h.alpha; o->beta = h.beta;
    return TE_OK;
}

size_t te_clay_chunk_size_for(const te_clay *c, size_t len) { return c ? c->h.chunk_size_for(len) : 0; }

size_t te_clay_track_chunk_size(const te_clay *c, size_t stripe, size_t blob_len) {
    return c ? c->h.chunk_size_for(std::min(stripe, blob_len)) : 0;
}

// ------------------------------------------------------------------------------------------
size_t te_pick_stripe_size(size_t blob_len) {
    if (blob_len <= 1000000) return kStripeSizes[0];
    if (blob_len <= 100000000) return kStripeSizes[1];
    return kStripeSizes[2];
}

size_t te_num_stripes(size_t blob_len, size_t stripe) {
    if (blob_len == 0) return 1;
    if (stripe == 0) return 0;
    return (blob_len + stripe - 1) / stripe;
}

uint32_t te_shard_to_slice(int rotated, uint32_t n, uint32_t stripe, uint32_t shard) {
    if (!rotated || n == 0) return shard;
    const uint32_t off = (uint32_t)(((uint64_t)stripe * TE_ROTATION_STEP) % n);
    return (shard + off) % n;
}

uint32_t te_slice_to_shard(int rotated, uint32_t n, uint32_t stripe, uint32_t slice) {
    if (!rotated || n == 0) return slice;
    const uint32_t off = (uint32_t)(((uint64_t)stripe * TE_ROTATION_STEP) % n);
    return (slice + n - off) % n;
}

void te_slice_metadata_to_bytes(const te_slice_metadata *m, uint8_t out[TE_META_SIZE]) {
    put_u64(out, m->version);
    put_u64(out + 8, m->blob_len);
    put_u64(out + 16, m->stripe_size);
    put_u64(out + 24, m->encoding);
    put_u64(out + 32, m->params);
    put_u64(out + 40, m->chunk_index);
}

int te_slice_metadata_from_slice(const uint8_t *slice, size_t len, te_slice_metadata *out) {
    if (!slice || !out || len < TE_META_SIZE) return TE_ERR_INVALID_LAYOUT;
    const uint8_t *p = slice + len - TE_META_SIZE;
    out->version = get_u64(p);
    out->blob_len = get_u64(p + 8);
    out->stripe_size = get_u64(p + 16);
    out->encoding = get_u64(p + 24);
    out->params = get_u64(p + 32);
    out->chunk_index = get_u64(p + 40);
    if (!valid_stripe(out->stripe_size)) return TE_ERR_INVALID_LAYOUT;
    return TE_OK;
}

int te_slicer_geometry(const te_clay *c, size_t blob_len, te_geometry *g) {
    if (!c || !g) return TE_ERR_INVALID_ARG;
    const size_t S = te_pick_stripe_size(blob_len);
    const size_t ns = te_num_stripes(blob_len, S);
    const size_t eff = blob_len == 0 ? S : std::min(blob_len, S);
    const size_t cs = c->h.chunk_size_for(eff);
    g->stripe_size = S;
    g->num_stripes = ns;
    g->chunk_size = cs;
    g->sub_chunk_size = cs / (size_t)c->h.alpha;
    g->slice_len = ns * cs + TE_META_SIZE;
    return TE_OK;
}

}  // extern "C"

// ------------------------------------------------------------------------------------------
// Encode
// ------------------------------------------------------------------------------------------
namespace {

struct GeomKey {
    uint64_t cs, slice_len;
    bool masked;  // stripe data end not dword aligned -> masked kernel variant
    bool odd;     // stripe data at an odd address: the fast kernels load 4 bytes at 2-aligned
                  // addresses only (an odd-address dword near the data end reads short through
                  // the range check), so such stripes take the generic byte-exact kernel
    bool operator<(const GeomKey &o) const {
        if (cs != o.cs) return cs < o.cs;
        if (slice_len != o.slice_len) return slice_len < o.slice_len;
        if (odd != o.odd) return odd < o.odd;
        return masked < o.masked;
    }
};

int ensure_stream(te_clay *c) {
    if (device_count() <= 0) return TE_ERR_NO_DEVICE;
    if (!c->stream) TE_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    return TE_OK;
}

// Enqueue the encode of a batch.  raw = ClayCoder::encode semantics (no slicing/rotation/meta,
// slices are the n chunks of one padded input).
// keep(obj, stripe): which stripes to encode and which of their chunks to write -- a mask of
// internal nodes, 0 = skip the stripe (all stripes, all chunks when empty).  With a selector no
// metadata suffix is written (te_recover_batch_device writes its own).  The mask is a store
// filter of the LDS-DMA kernel (it must include the column-0 parity nodes, which that kernel
// reads back); the other kernels write every chunk.
using StripeSel = std::function<uint32_t(size_t, size_t)>;

int encode_enqueue(te_clay *c, const te_slicer_cfg *cfg, const uint8_t *d_data, const te_object *objs,
                   size_t nobj, uint8_t *d_out, hipStream_t s, bool raw, Arena *arena = nullptr,
                   const StripeSel &keep = StripeSel(), bool per_call = false) {
    const ClayHost &h = c->h;
    const int n = h.n;
    const int rotated = cfg ? cfg->rotated : 0;
    std::map<GeomKey, std::vector<EncJob>> groups;
    std::vector<MetaJob> metas;

    for (size_t i = 0; i < nobj; i++) {
        const te_object &o = objs[i];
        size_t S, ns, cs, slice_len;
        if (raw) {
            if (o.blob_len == 0) return TE_ERR_EMPTY_INPUT;
            cs = h.chunk_size_for(o.blob_len);
            S = cs * h.k;
            ns = 1;
            slice_len = cs;
        } else {
            te_geometry g;
            te_slicer_geometry(c, o.blob_len, &g);
            S = g.stripe_size; ns = g.num_stripes; cs = g.chunk_size; slice_len = g.slice_len;
        }
        if (cs % (size_t)h.alpha || slice_len > 0xffffffffull || cs > 0xffffffffull) return TE_ERR_TOO_MUCH_DATA;
        for (size_t st = 0; st < ns; st++) {
            const uint32_t store = keep ? keep(i, st) : ~0u;
            if (!store) continue;
            EncJob j{};
            j.store_mask = store;
            const uint64_t start = (uint64_t)st * S;
            j.src = d_data + o.data_off + start;
            j.src_len = o.blob_len == 0 ? 0 : std::min<uint64_t>(S, o.blob_len - start);
            j.dst = d_out + o.out_off + st * cs;
            j.rot = rotated ? (uint32_t)((st * TE_ROTATION_STEP) % n) : 0u;
            j.dst_skew = (uint32_t)(st * cs);
            const bool masked = ((reinterpret_cast<uintptr_t>(j.src) & 3u) + j.src_len) % 4 != 0;
            const bool odd = (reinterpret_cast<uintptr_t>(j.src) & 1u) != 0;
            groups[GeomKey{cs, slice_len, masked, odd}].push_back(j);
        }
        if (!raw && !keep) {
            MetaJob m{};
            m.dst = d_out + o.out_off + ns * cs;
            m.slice_len = slice_len;
            m.words[0] = 0;
            m.words[1] = o.blob_len;
            m.words[2] = S;
            m.words[3] = cfg ? cfg->encoding : TE_ENCODING_CLAY;
            m.words[4] = cfg ? cfg->params : TE_CLAY_DEFAULT_PARAMS;
            m.words[5] = o.chunk_index;
            metas.push_back(m);
        }
    }
    // descriptor image
    Arena &A = arena ? *arena : c->enc;
    A.img.clear();
    struct Launch { GeomKey key; size_t off, count; };
    std::vector<Launch> launches;
    for (auto &kv : groups) launches.push_back({kv.first, A.put(kv.second.data(), kv.second.size() * sizeof(EncJob)), kv.second.size()});
    const size_t meta_off = A.put(metas.data(), metas.size() * sizeof(MetaJob));
    // generic-engine pattern (parity erased) for profiles outside the fast path
    size_t pat_off = 0, pool_off = 0;
    GpePattern pat{};
    std::vector<uint16_t> pool;
    std::vector<GpeJob> gjobs;
    std::vector<size_t> gjob_off;
    {
        uint64_t mask = 0;
        for (int i = h.k + h.nu; i < h.qt; i++) mask |= 1ull << i;
        if (!h.gpe_pattern(mask, pat, pool)) return TE_ERR_UNSUPPORTED;
        pat_off = A.put(&pat, sizeof(pat));
        pool_off = A.put(pool.data(), pool.size() * sizeof(uint16_t));
        for (auto &kv : groups) {
            std::vector<GpeJob> gj;
            for (const EncJob &e : kv.second) {
                GpeJob g{};
                g.in = e.src; g.out = e.dst; g.in_len = e.src_len; g.out_len = ~0ull; g.rot = e.rot; g.pattern = 0;
                gj.push_back(g);
            }
            gjob_off.push_back(A.put(gj.data(), gj.size() * sizeof(GpeJob)));
        }
    }
    int r = A.upload(s);
    if (r) return r;
    // one workspace for every fast-path launch of the call (they run in stream order)
    auto fast_path = [&](const Launch &L) {
        return c->fast_encode && !L.key.odd && (uint64_t)n * L.key.slice_len < 0x7fffffffull;
    };
    size_t total_stripes = 0;
    for (const Launch &L : launches) total_stripes += L.count;
    // a small per-call encode (every chunk kept): the staged kernel with one wave per workgroup
    const bool small = per_call && !keep && total_stripes <= g_enc_small;
    auto dma_path = [&](const Launch &L) {
        return fast_path(L) && encode_dma_supported(n, h.k, (uint32_t)(L.key.cs / h.alpha)) && !g_no_dma_encode &&
               !small;
    };
    size_t scratch_bytes = 0;
    for (const Launch &L : launches) {
        if (!fast_path(L) || dma_path(L)) continue;
        const uint32_t wps = ((uint32_t)(L.key.cs / h.alpha) + 3) / 4;
        EncArgs a{};
        a.njobs = (uint32_t)L.count;
        a.groups_per_stripe = (wps + 63) / 64;
        a.groups_per_wg = small ? 1u : 0u;
        scratch_bytes = std::max(scratch_bytes, encode_rows_scratch_bytes(a));
    }
    uint8_t *scratch = nullptr;
    if (scratch_bytes) {
        r = A.workspace(scratch_bytes, s, &scratch);
        if (r) return r;
    }
    KTimer kt(s);
    if (!metas.empty()) TE_HIP(launch_meta(A.at<MetaJob>(meta_off), (uint32_t)metas.size(), (uint32_t)n, s));
    auto gpe_args = [&](size_t gi, const Launch &L, uint32_t word_base, uint32_t word_end) {
        const uint32_t cs = (uint32_t)L.key.cs, sc = cs / (uint32_t)h.alpha;
        (void)sc;
        GpeArgs a{};
        a.jobs = A.at<GpeJob>(gjob_off[gi]);
        a.patterns = A.at<GpePattern>(pat_off);
        a.plane_pool = A.at<uint16_t>(pool_off);
        a.njobs = (uint32_t)L.count;
        a.word_base = word_base;
        a.word_end = word_end;
        a.groups_per_stripe = (word_end - word_base + kGpeWords - 1) / kGpeWords;
        a.cs = cs; a.sc = cs / (uint32_t)h.alpha; a.q = h.q; a.t = h.t; a.k = h.k; a.nu = h.nu; a.n = n;
        a.alpha = h.alpha;
        a.in_stride = cs; a.out_stride = L.key.slice_len;
        a.in_rotated = 0; a.out_rotated = 1;
        a.out_mask = 0;
        for (int i = 0; i < h.qt; i++)
            if (h.int_to_ext(i) >= 0) a.out_mask |= 1ull << i;
        for (int i = 0; i < 16; i++) a.qpow[i] = h.qpow[i];
        return a;
    };
    size_t gi = 0;
    std::vector<std::pair<bool, EncArgs>> level2;  // split launches' level-2 halves, enqueued last
    for (const Launch &L : launches) {
        const uint32_t cs = (uint32_t)L.key.cs, sc = cs / (uint32_t)h.alpha;
        const uint32_t wps = (sc + 3) / 4;   // words incl. a 2-column tail when sc % 4 == 2
        const uint32_t full = sc / 4;        // full 4-column words
        // fast kernel addresses an object's slices with 31-bit buffer offsets
        if (dma_path(L)) {  // the 1 MB-stripe kernel (encode_dma.hip)
            EncArgs a{};
            a.jobs = A.at<EncJob>(L.off);
            a.njobs = (uint32_t)L.count;
            a.cs = cs;
            a.sc = sc;
            a.slice_len = (uint32_t)L.key.slice_len;
            a.n = (uint32_t)n;
            if ((per_call && total_stripes <= g_enc_split) || g_enc_split_batch) {
                // level-1 rows z0 = 0..6: one workgroup each (or g_enc_split_batch rows each)
                const uint32_t per = per_call ? 1u : g_enc_split_batch;
                a.z0_first = 0; a.z0_count = per; a.z0_split = (7 + per - 1) / per; a.z0_limit = 7;
                TE_HIP(launch_encode_dma(L.key.masked, a, s));
                a.z0_limit = 0;
                a.z0_first = 7; a.z0_count = 3; a.z0_split = 1;   // level 2 reads their parity back:
                level2.push_back({L.key.masked, a});              // after every level-1 launch
            } else {
                TE_HIP(launch_encode_dma(L.key.masked, a, s));
            }
        } else if (fast_path(L)) {
            (void)full;
            EncArgs a{};
            a.jobs = A.at<EncJob>(L.off);
            a.njobs = (uint32_t)L.count;
            a.groups_per_stripe = (wps + 63) / 64;
            a.groups_per_wg = small ? 1u : 0u;
            a.words_per_stripe = wps;
            a.cs = cs;
            a.sc = sc;
            a.slice_len = (uint32_t)L.key.slice_len;
            a.n = (uint32_t)n;
            a.scratch = scratch;
            TE_HIP(launch_encode_rows(h.k, L.key.masked, a, s));
        } else {
            TE_HIP(launch_gpe(gpe_args(gi, L, 0, wps), (uint32_t)pat.nerased, s));
        }
        gi++;
    }
    for (const auto &l2 : level2) TE_HIP(launch_encode_dma(l2.first, l2.second, s));
    kt.stop();
    return A.mark_done(s);
}

}  // namespace

// ------------------------------------------------------------------------------------------
// Decode
// ------------------------------------------------------------------------------------------
namespace {

struct DecItem {          // one object, host-validated
    uint64_t in_base;     // offset in d_slices of slice 0
    uint64_t slice_len, blob_len, stripe, ns, cs, out_off;
    uint32_t avail;
    int32_t lost = -1;    // >= 0: output = that slice's chunks at out_off + stripe * cs (node recover)
};

// Validate one object like Slicer::decode (slicer.rs:298-331, validate_layout :79-105).
int decode_validate(const te_clay *c, const uint8_t *meta48, uint64_t slice_len, uint32_t avail, DecItem &it) {
    const ClayHost &h = c->h;
    const int na = __builtin_popcount(avail & ((h.n >= 32) ? 0xffffffffu : ((1u << h.n) - 1u)));
    if (na == 0) return TE_ERR_NOT_ENOUGH_SLICES;
    te_slice_metadata m;
    int r = te_slice_metadata_from_slice(meta48, TE_META_SIZE, &m);
    if (r) return r;
    const uint32_t pk = (uint32_t)((m.params >> 8) & 0xFF);  // profile k  slicer.rs:308-311
    if ((uint32_t)na < pk) return TE_ERR_NOT_ENOUGH_SLICES;
    it.blob_len = m.blob_len;
    it.stripe = m.stripe_size;
    it.slice_len = slice_len;
    it.avail = avail;
    if (m.blob_len == 0) { it.ns = 0; it.cs = 0; return TE_OK; }
    it.ns = (m.blob_len + m.stripe_size - 1) / m.stripe_size;
    const uint64_t total = slice_len >= TE_META_SIZE ? slice_len - TE_META_SIZE : 0;
    if (total == 0 || total % it.ns) return TE_ERR_INVALID_LAYOUT;
    it.cs = total / it.ns;
    if (na < h.k) return TE_ERR_NOT_ENOUGH_SLICES;  // ClayCoder::decode clay.rs:107-109
    if (it.cs % (uint64_t)h.alpha) return TE_ERR_BAD_ENCODING;
    // take <= decoded stripe size (slicer.rs:351-357)
    const uint64_t last_take = m.blob_len - (it.ns - 1) * m.stripe_size;
    if (std::max<uint64_t>(it.ns > 1 ? m.stripe_size : 0, last_take) > it.cs * (uint64_t)h.k) return TE_ERR_INVALID_LAYOUT;
    return TE_OK;
}

// The compiled form of one padded erasure pattern, built once per handle (caller holds c->mu).
// Compile one padded erasure pattern (host only, thread-safe: pure ClayHost work).  out_node >= 0:
// the program outputs that internal node's chunk (ClayHost::dec_prog).
bool compile_pattern(const ClayHost &h, uint64_t emask, int out_node, te_clay::DecCache &d) {
    const int n = h.n;
    if (!h.gpe_pattern(emask, d.P, d.planes)) return false;
    d.P.planes_off = 0;
    // node recover of Clay(20,7,16): the lost node first among its column's erased nodes, the
    // order the recover class kernels assume (dec_class.hpp); every program below follows it
    if (out_node >= 0 && dec_class_of(h, d.P) >= 0) dec_class_lost_first(d.P, out_node);
    // staged kernel (decode_stage.hip): compiled per k with every other node erased (padded
    // patterns); of the two row orientations, two workgroups per CU first (2 x 53 x 1536 B <=
    // 160 KB), then fewer scratch rows
    if (decode_stage_k(h.k) && d.P.nknown == (uint32_t)h.k && d.P.nerased == (uint32_t)(n - h.k)) {
        DecProgHdr best{};
        std::vector<DecStep> best_steps;
        bool found = false;
        auto cost = [](const DecProgHdr &x) {
            return (decode_stage_rows(x.nslots, x.max_out) > 53 ? 1u << 20 : 0u) + x.nscratch;
        };
        static const int force = [] {  // TEC_DEC_ORIENT=0/1: one row orientation only (measurement)
            const char *e = tec_knob("TEC_DEC_ORIENT");
            return e ? atoi(e) : -1;
        }();
        for (int orient = 0; orient < 2; orient++) {
            if (force >= 0 && orient != force) continue;
            DecProgHdr H;
            std::vector<DecStep> st;
            if (!h.dec_prog(d.P, orient, H, st, out_node) || !decode_stage_fits(H.nslots, H.max_out)) continue;
            if (!found || cost(H) < cost(best)) { best = H; best_steps.swap(st); found = true; d.orient = orient; }
        }
        bool ok = found;
        for (const DecStep &S : best_steps) {
            d.steps.emplace_back();
            ok = ok && ClayHost::dec_pack(S, d.steps.back());
        }
        d.steps.resize(d.steps.size() + 2);  // blank steps: the kernel reads two steps ahead
        d.staged = ok && d.steps.size() == te_clay::DecStore::kSteps;
        d.H = best;
    }
    return true;
}

inline uint64_t dec_key(uint64_t emask, int out_node) { return emask | (uint64_t)(out_node + 1) << 48; }

// The compiled form of one padded erasure pattern, built once per handle (caller holds c->mu).
const te_clay::DecCache *dec_pattern(te_clay *c, uint64_t emask, int out_node = -1) {
    const uint64_t key = dec_key(emask, out_node);
    auto f = c->dec_cache.find(key);
    if (f != c->dec_cache.end()) return &f->second;
    te_clay::DecCache d;
    if (!compile_pattern(c->h, emask, out_node, d)) return nullptr;
    return &c->dec_cache.emplace(key, std::move(d)).first->second;
}

// Compile the patterns of `keys` missing from the cache, on up to 16 host threads (random
// survivor sets bring one new pattern per stripe: ~150 us of host work each).
void dec_precompile(te_clay *c, const std::vector<std::pair<uint64_t, int>> &keys) {
    std::vector<std::pair<uint64_t, int>> todo;
    for (const auto &k : keys)
        if (!c->dec_cache.count(dec_key(k.first, k.second))) todo.push_back(k);
    if (todo.size() < 8) return;  // dec_pattern compiles the few inline
    std::vector<te_clay::DecCache> out(todo.size());
    std::vector<char> ok(todo.size(), 0);
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const size_t nth = std::min<size_t>({16, (size_t)hw, (todo.size() + 7) / 8});
    std::atomic<size_t> next{0};
    auto work = [&] {
        for (size_t i; (i = next.fetch_add(1)) < todo.size();)
            ok[i] = compile_pattern(c->h, todo[i].first, todo[i].second, out[i]);
    };
    std::vector<std::thread> th;
    for (size_t t = 1; t < nth; t++) th.emplace_back(work);
    work();
    for (auto &t : th) t.join();
    for (size_t i = 0; i < todo.size(); i++)
        if (ok[i]) c->dec_cache.emplace(dec_key(todo[i].first, todo[i].second), std::move(out[i]));
}

// Slots of the device-resident pattern store (te_clay::DecStore) for the staged patterns of one
// call.  The patterns not there yet are appended to U (host images of their store entries) for
// decode_enqueue to upload with the call's descriptors and copy into their slots on the call's
// stream.  false: more distinct patterns than the store holds (the call then uploads its patterns
// through the arena).
struct StoreFill {
    uint32_t n0 = 0;                  // first new slot
    bool wait_used = false;           // new slots overwrite slots earlier launches may still read
    std::vector<GpePattern> pats;
    std::vector<DecProgHdr> hdrs;
    std::vector<DecStepP> steps;
    std::vector<uint32_t> soff;       // slot -> step offset, when the store was (re)allocated
};
bool dec_store_slots(te_clay *c, const std::vector<const te_clay::DecCache *> &cached, const std::vector<uint64_t> &keys,
                     std::vector<uint32_t> &slot_of, StoreFill &U, int &rc) {
    te_clay::DecStore &S = c->dstore;
    constexpr uint32_t kSteps = te_clay::DecStore::kSteps;
    rc = TE_OK;
    const uint32_t cap_max = S.max_cap;
    if (keys.size() > cap_max) {
        S.arena_calls++;
        return false;
    }
    if (!S.written && (rc = hip_status(hipEventCreateWithFlags(&S.written, hipEventDisableTiming)))) return false;
    size_t fresh = 0;
    for (uint64_t k : keys) fresh += S.slot.count(k) == 0;
    if (S.n + fresh > S.cap) {
        // grow (doubling, up to kCap) when the call's patterns do not fit, else empty the full
        // store; either way the old contents go once their last reader is done
        const uint32_t need = (uint32_t)std::min<size_t>(cap_max, std::max<size_t>(keys.size(), (size_t)S.n + fresh));
        if (S.cap < cap_max && need > S.cap) {
            uint32_t cap = std::min(te_clay::DecStore::kMin, cap_max);
            while (cap < need) cap *= 2;
            cap = std::min(cap, cap_max);
            // the buffers are freed: every launch that read them must be done (rare: <= 6 times)
            if ((rc = hip_status(S.readers.sync()))) return false;
            S.pats.release();
            S.hdrs.release();
            S.steps.release();
            S.soff.release();
            if ((rc = hip_status(S.pats.ensure((size_t)cap * sizeof(GpePattern))))) return false;
            if ((rc = hip_status(S.hdrs.ensure((size_t)cap * sizeof(DecProgHdr))))) return false;
            if ((rc = hip_status(S.steps.ensure((size_t)cap * kSteps * sizeof(DecStepP))))) return false;
            if ((rc = hip_status(S.soff.ensure((size_t)cap * sizeof(uint32_t))))) return false;
            S.cap = cap;
            U.soff.resize(cap);
            for (uint32_t i = 0; i < cap; i++) U.soff[i] = i * kSteps;
            S.grows++;
        } else {
            U.wait_used = S.readers.any();  // the fill waits (on the device) for the last reader on every stream
            S.clears++;
        }
        S.slot.clear();
        S.n = 0;
    }
    slot_of.assign(keys.size(), 0);
    U.n0 = S.n;
    for (size_t i = 0; i < keys.size(); i++) {
        auto f = S.slot.find(keys[i]);
        if (f != S.slot.end()) {
            slot_of[i] = f->second;
            continue;
        }
        const uint32_t sl = S.n++;
        S.slot.emplace(keys[i], sl);
        slot_of[i] = sl;
        U.pats.push_back(cached[i]->P);
        U.hdrs.push_back(cached[i]->H);
        U.steps.insert(U.steps.end(), cached[i]->steps.begin(), cached[i]->steps.end());
    }
    return true;
}

// A decode call of at most this many stripes is a per-call decode: one wave per workgroup.
constexpr size_t kDecSmallStripes = 64;

// Items with lost >= 0 (node recover) need the staged kernel: TE_ERR_UNSUPPORTED, before anything
// is enqueued, when a pattern has no plane program (the caller then decodes and re-encodes).
int decode_enqueue(te_clay *c, const te_slicer_cfg *cfg, const uint8_t *d_slices, const DecItem *items,
                   size_t nitems, uint8_t *d_out, hipStream_t s, bool raw) {
    const ClayHost &h = c->h;
    const int n = h.n;
    const int rotated = (cfg && !raw) ? cfg->rotated : 0;
    // compiled programs kept on the host: <= ~430 MB (26 KB per pattern, as many as the device
    // store's cap; 77,520 masks exist for k = 7, x 20 outputs for node recover)
    if (c->dec_cache.size() > std::max<size_t>(c->dstore.max_cap, nitems)) c->dec_cache.clear();
    {
        std::vector<std::pair<uint64_t, int>> keys;
        std::unordered_map<uint64_t, char> seen;
        for (size_t i = 0; i < nitems; i++) {
            const DecItem &it = items[i];
            for (uint64_t st = 0; st < it.ns; st++) {
                uint64_t emask = 0;
                for (int sh = 0; sh < n; sh++) {
                    const uint32_t sl = te_shard_to_slice(rotated, (uint32_t)n, (uint32_t)st, (uint32_t)sh);
                    if (!((it.avail >> sl) & 1u)) emask |= 1ull << h.ext_to_int(sh);
                }
                emask = h.pad_erasures(emask);
                const int onode = it.lost >= 0 ? h.ext_to_int((int)te_slice_to_shard(rotated, (uint32_t)n, (uint32_t)st,
                                                                                      (uint32_t)it.lost)) : -1;
                if (seen.emplace(dec_key(emask, onode), 1).second) keys.push_back({emask, onode});
            }
        }
        dec_precompile(c, keys);
    }
    std::unordered_map<uint64_t, uint32_t> pat_index;  // erased mask (| output node << 48) -> pattern id
    std::vector<uint64_t> pat_keys;                    // by pattern id
    bool fused = false;
    std::vector<GpePattern> pats;  // the generic kernel's per-call copies (built only for it)
    std::vector<const te_clay::DecCache *> cached;
    std::vector<uint16_t> pool;
    std::map<uint64_t, std::vector<GpeJob>> groups;  // by chunk size
    std::map<uint64_t, uint64_t> group_in_stride;
    uint32_t max_er = 0;
    for (size_t i = 0; i < nitems; i++) {
        const DecItem &it = items[i];
        for (uint64_t st = 0; st < it.ns; st++) {
            uint64_t emask = 0;
            for (int sh = 0; sh < n; sh++) {
                const uint32_t sl = te_shard_to_slice(rotated, (uint32_t)n, (uint32_t)st, (uint32_t)sh);
                if (!((it.avail >> sl) & 1u)) emask |= 1ull << h.ext_to_int(sh);
            }
            emask = h.pad_erasures(emask);
            const int onode = it.lost >= 0 ? h.ext_to_int((int)te_slice_to_shard(rotated, (uint32_t)n, (uint32_t)st,
                                                                                  (uint32_t)it.lost)) : -1;
            fused = fused || onode >= 0;
            const uint64_t pkey = emask | (uint64_t)(onode + 1) << 48;
            auto f = pat_index.find(pkey);
            uint32_t pid;
            if (f == pat_index.end()) {
                const te_clay::DecCache *dc = dec_pattern(c, emask, onode);
                if (!dc) return TE_ERR_BAD_ENCODING;
                pid = (uint32_t)cached.size();
                cached.push_back(dc);
                pat_index[pkey] = pid;
                pat_keys.push_back(pkey);
                max_er = std::max(max_er, dc->P.nerased);
            } else {
                pid = f->second;
            }
            GpeJob g{};
            g.in = d_slices + it.in_base + st * it.cs;
            g.in_len = ~0ull;
            if (onode >= 0) {  // the lost slice's chunk of this stripe, whole
                g.out = d_out + it.out_off + st * it.cs;
                g.out_len = it.cs;
            } else {
                g.out = d_out + it.out_off + st * (raw ? 0 : it.stripe);
                g.out_len = raw ? it.cs * (uint64_t)h.k : (st + 1 == it.ns ? it.blob_len - st * it.stripe : it.stripe);
            }
            g.rot = rotated ? (uint32_t)((st * TE_ROTATION_STEP) % n) : 0u;
            g.pattern = pid;
            auto key = (it.cs << 32) ^ it.slice_len;
            groups[key].push_back(g);
            group_in_stride[key] = it.slice_len;
        }
    }
    if (groups.empty()) return TE_OK;
    // staged kernel (decode_stage.hip) when every pattern compiles to a plane program; of the two
    // row orientations the one with fewer scratch rows
    uint32_t lds_rows = 0, nscr_max = 0;
    bool staged = true;
    for (size_t i = 0; i < cached.size() && staged; i++) {
        const te_clay::DecCache &dc = *cached[i];
        staged = dc.staged;
        if (!staged) break;
        lds_rows = std::max(lds_rows, decode_stage_rows(dc.H.nslots, dc.H.max_out));
        nscr_max = std::max(nscr_max, dc.H.nscratch);
    }
    lds_rows = std::max(lds_rows, 1u);
    // the staged kernel addresses a stripe's slices and its output share with 31-bit offsets
    auto staged_group = [&](uint64_t key) {
        const uint64_t cs = key >> 32, sc = cs / (uint64_t)h.alpha;
        return staged && sc >= 8 && (uint64_t)n * group_in_stride[key] < 0x7fffffffull &&
               cs * (uint64_t)h.k < 0x7fffffffull;
    };
    if (fused)
        for (auto &kv : groups)
            if (!staged_group(kv.first)) return TE_ERR_UNSUPPORTED;
    // patterns with a per-pattern kernel built (dec_rtc.cpp) leave their group for a launch of
    // their own; every staged stripe counts toward building its pattern's kernel
    struct Fixed { uint64_t key; const DecJitKernel *k; std::vector<GpeJob> jobs; size_t off = 0; };
    constexpr uint64_t kJitMinStripes = 512;  // two workgroups per CU
    // a caller that lowered the build threshold (te_clay_set_decode_jit, tests) lowers the floor too
    const uint64_t jit_floor = c->jit_mode >= 0 ? std::min<uint64_t>(kJitMinStripes, c->jit_min) : kJitMinStripes;
    std::vector<Fixed> fixed;
    static const bool class_on = [] {
        const char *e = tec_knob("TEC_DEC_CLASS");
        return !(e && e[0] == '0');
    }();
    if (staged && !fused) {  // (pattern kernels write data chunks; recover's outputs are other nodes)
        if (!c->jit) {
            c->jit = dec_jit_new(c->device);
            if (c->jit_mode >= 0) dec_jit_set(c->jit, c->jit_mode, c->jit_min);
        }
        for (auto &kv : groups) {
            if (!staged_group(kv.first)) continue;
            const uint32_t sc = (uint32_t)((kv.first >> 32) / (uint64_t)h.alpha);
            const DecJitGeom geo = dec_jit_geom(sc);
            std::vector<uint64_t> cnt(cached.size(), 0);
            for (const GpeJob &g : kv.second) cnt[g.pattern]++;
            std::vector<int> fx(cached.size(), -1);
            for (size_t p = 0; p < cached.size(); p++) {
                // a pattern kernel gets a launch of its own: only worth it for a group that fills
                // the GPU; smaller groups stay in the shared table-driven launch (recover's
                // windows hold ~64 stripes per pattern: 80 small launches per step ran 29.3 ms
                // against 14.5 for the shared one).  Such groups do not count toward building a
                // kernel either: it could never be launched for them.
                if (cnt[p] < std::max<uint64_t>(1, jit_floor)) continue;
                // a survivor set with a class kernel runs it: after the load fusions the class
                // kernels time at or below the hipRTC pattern kernels (4.26 vs 4.36-4.39 ms, worst
                // case, same box) with no 25 s compile; a caller that asked for the pattern kernels
                // (te_clay_set_decode_jit) still gets them
                if (c->jit_mode < 0 && class_on && dec_class_of(h, cached[p]->P) >= 0) continue;
                const DecJitKernel *k = dec_jit_get(c->jit, h, cached[p]->P, cached[p]->orient, (int)geo.G, (int)geo.wb, cnt[p]);
                if (!k) continue;
                fx[p] = (int)fixed.size();
                fixed.push_back(Fixed{kv.first, k, {}});
            }
            std::vector<GpeJob> rest;
            for (const GpeJob &g : kv.second) {
                if (fx[g.pattern] >= 0) fixed[fx[g.pattern]].jobs.push_back(g);
                else rest.push_back(g);
            }
            kv.second.swap(rest);
        }
    }
    // decode class kernels (decode_class.hip, dec_class.hpp): the remaining stripes of every
    // Clay(20,7,16) survivor set run the ahead-of-time kernel of the set's class -- the program's
    // control compiled in, the set's slices, planes and decoding matrix read at run time.
    // Measurement option TEC_DEBUG_KNOBS=1 TEC_DEC_CLASS=0: the table-driven kernel instead.
    struct ClassGrp { uint64_t key; int id; std::vector<GpeJob> jobs; size_t off = 0; };
    std::vector<ClassGrp> cls;
    bool cls_small = false;  // the class stripes fit one round of per-call workgroups
    // measurement option TEC_DEC_CLASS_SMALL=1 (off by default: per call 64 MiB, kernel 0.596 ms
    // on the per-call class kernels against 0.472 on the one table-driven launch)
    static const bool small_dec_cls = [] {
        const char *e = tec_knob("TEC_DEC_CLASS_SMALL");
        return e && e[0] == '1';
    }();
    // streams the class groups of a call run on, side by side (TEC_DEC_CLASS_STREAMS)
    static const int class_streams = [] {
        const char *e = tec_knob("TEC_DEC_CLASS_STREAMS");
        const int v = e ? atoi(e) : 4;  // the process's hardware queues (GPU_MAX_HW_QUEUES default)
        return std::max(1, std::min(v, 1 + te_clay::kClsSide));
    }();
    if (staged && class_on) {
        std::vector<int> cid(cached.size(), -1);
        for (size_t p = 0; p < cached.size(); p++) {
            const int onode = (int)(pat_keys[p] >> 48) - 1;  // >= 0: node recover's output node
            const int id = dec_class_of(h, cached[p]->P, onode);
            cid[p] = id >= 0 && dec_class_info(id, nullptr, nullptr) ? id : -1;
        }
        for (auto &kv : groups) {
            if (!staged_group(kv.first)) continue;
            int at[kDecClasses];
            std::fill(at, at + kDecClasses, -1);
            std::vector<GpeJob> rest;
            for (const GpeJob &g : kv.second) {
                const int id = cid[g.pattern];
                if (id < 0) {
                    rest.push_back(g);
                    continue;
                }
                if (at[id] < 0) {
                    at[id] = (int)cls.size();
                    cls.push_back(ClassGrp{kv.first, id, {}});
                }
                cls[(size_t)at[id]].jobs.push_back(g);
            }
            kv.second.swap(rest);
        }
        // a call that does not fill the GPU is bound by one stripe's 100-step chain per launch:
        // with more class groups than streams some launches would run after others, so such a
        // call runs on the table-driven kernel in one launch (per call 64 MiB: 3.67 ms as
        // classes against 3.00, r06)
        // (per-call decodes of <= 64 stripes run the classes' one-wave kernels, whose input loads
        // lead by four steps: their chains are short enough to run a few one after another)
        // (TEC_DEC_CLASS_SMALL=1: a call whose class stripes fit one round of per-call workgroups
        // -- G = 1, 4 compute waves and a loader wave per 64-column group, <= 2 per CU by LDS --
        // runs them on the per-call kernels instead; measured slower for 64 MiB per call)
        size_t ncls = 0, nall = 0, small_wgs = 0;
        for (const ClassGrp &cg : cls) {
            ncls += cg.jobs.size();
            const uint64_t sc = (cg.key >> 32) / (uint64_t)h.alpha;
            small_wgs += cg.jobs.size() * (size_t)((sc / 4 + 63) / 64);
        }
        for (auto &kv : groups) nall += kv.second.size();
        cls_small = small_dec_cls && !cls.empty() && small_wgs <= 512;
        if (!cls_small && cls.size() > (size_t)class_streams && ncls < 1024 && ncls + nall > kDecSmallStripes) {
            for (ClassGrp &cg : cls) groups[cg.key].insert(groups[cg.key].end(), cg.jobs.begin(), cg.jobs.end());
            cls.clear();
        }
    }
    // staged patterns live in the device store (uploaded once per handle), the jobs name slots;
    // otherwise (generic kernel, or more patterns than the store holds) they go in the arena
    std::vector<uint32_t> slot_of;
    StoreFill fill;
    bool in_store = false;
    bool every_group_staged = staged;  // the generic kernel reads per-call patterns (plane lists)
    for (auto &kv : groups) every_group_staged = every_group_staged && (kv.second.empty() || staged_group(kv.first));
    if (every_group_staged) {
        int rs = TE_OK;
        in_store = dec_store_slots(c, cached, pat_keys, slot_of, fill, rs);
        if (rs) return rs;
        if (in_store) {
            for (auto &kv : groups)
                for (GpeJob &g : kv.second) g.pattern = slot_of[g.pattern];
            for (ClassGrp &cg : cls)
                for (GpeJob &g : cg.jobs) g.pattern = slot_of[g.pattern];
        }
    }
    std::vector<DecProgHdr> dhdrs;
    std::vector<DecStepP> dsteps;
    std::vector<uint32_t> dstep_off;
    if (staged && !in_store) {
        for (size_t i = 0; i < cached.size(); i++) {
            dhdrs.push_back(cached[i]->H);
            dstep_off.push_back((uint32_t)dsteps.size());
            dsteps.insert(dsteps.end(), cached[i]->steps.begin(), cached[i]->steps.end());
        }
    }
    if (!in_store)
        for (const te_clay::DecCache *dc : cached) {
            pats.push_back(dc->P);
            pats.back().planes_off = (uint32_t)pool.size();
            pool.insert(pool.end(), dc->planes.begin(), dc->planes.end());
        }
    Arena &A = c->dec;
    A.img.clear();
    const size_t pat_off = in_store ? 0 : A.put(pats.data(), pats.size() * sizeof(GpePattern));
    const size_t pool_off = A.put(pool.data(), pool.size() * sizeof(uint16_t));
    size_t hdr_off = 0, step_off = 0, soff_off = 0;
    if (staged && !in_store) {
        hdr_off = A.put(dhdrs.data(), dhdrs.size() * sizeof(DecProgHdr));
        step_off = A.put(dsteps.data(), dsteps.size() * sizeof(DecStepP), 64);
        soff_off = A.put(dstep_off.data(), dstep_off.size() * sizeof(uint32_t));
    }
    std::vector<std::pair<uint64_t, size_t>> offs;
    for (auto &kv : groups)
        if (!kv.second.empty()) offs.push_back({kv.first, A.put(kv.second.data(), kv.second.size() * sizeof(GpeJob))});
    for (Fixed &f : fixed) f.off = A.put(f.jobs.data(), f.jobs.size() * sizeof(GpeJob));
    for (ClassGrp &cg : cls) cg.off = A.put(cg.jobs.data(), cg.jobs.size() * sizeof(GpeJob));
    // new store entries ride in the same upload, then move to their slots on this stream
    size_t fp_off = 0, fh_off = 0, fs_off = 0, fo_off = 0;
    if (in_store && !fill.pats.empty()) {
        fp_off = A.put(fill.pats.data(), fill.pats.size() * sizeof(GpePattern));
        fh_off = A.put(fill.hdrs.data(), fill.hdrs.size() * sizeof(DecProgHdr));
        fs_off = A.put(fill.steps.data(), fill.steps.size() * sizeof(DecStepP), 64);
    }
    if (in_store && !fill.soff.empty()) fo_off = A.put(fill.soff.data(), fill.soff.size() * sizeof(uint32_t));
    int r = A.upload(s);
    if (r) return r;
    if (in_store) {
        te_clay::DecStore &S = c->dstore;
        if (fill.wait_used) TE_HIP(S.readers.wait(s));
        // entries another stream filled and nobody on this stream has waited for yet
        if (S.written_pending && S.written_stream != s) TE_HIP(hipStreamWaitEvent(s, S.written, 0));
        const bool any = !fill.pats.empty() || !fill.soff.empty();
        if (!fill.pats.empty()) {
            const size_t np = fill.pats.size();
            TE_HIP(hipMemcpyAsync(S.pats.as<GpePattern>() + fill.n0, A.at<GpePattern>(fp_off), np * sizeof(GpePattern),
                                  hipMemcpyDeviceToDevice, s));
            TE_HIP(hipMemcpyAsync(S.hdrs.as<DecProgHdr>() + fill.n0, A.at<DecProgHdr>(fh_off), np * sizeof(DecProgHdr),
                                  hipMemcpyDeviceToDevice, s));
            TE_HIP(hipMemcpyAsync(S.steps.as<DecStepP>() + (size_t)fill.n0 * te_clay::DecStore::kSteps,
                                  A.at<DecStepP>(fs_off), fill.steps.size() * sizeof(DecStepP), hipMemcpyDeviceToDevice, s));
        }
        if (!fill.soff.empty())
            TE_HIP(hipMemcpyAsync(S.soff.p, A.at<uint32_t>(fo_off), fill.soff.size() * sizeof(uint32_t),
                                  hipMemcpyDeviceToDevice, s));
        if (any) {
            TE_HIP(hipEventRecord(S.written, s));
            S.written_pending = true;
            S.written_stream = s;
        }
    }
    // a small call (a per-call decode: a few stripes on a 256-CU chip) runs one wave per
    // workgroup, so each stripe's 100-step chain is split over more workgroups with less work per
    // step.  Measurement option TEC_DEBUG_KNOBS=1 TEC_DEC_SMALL=n: the stripe bound (0: never).
    static const size_t dec_small_max = [] {
        const char *e = tec_knob("TEC_DEC_SMALL");
        return e ? (size_t)atoi(e) : kDecSmallStripes;
    }();
    size_t call_stripes = 0;
    for (auto &o : offs) call_stripes += groups[o.first].size();
    for (const ClassGrp &cg : cls) call_stripes += cg.jobs.size();
    static const uint32_t class_g_big = [] {  // measurement option TEC_DEC_CLASS_G (1 or 2)
        const char *e = tec_knob("TEC_DEC_CLASS_G");
        return e && atoi(e) == 1 ? 1u : 2u;
    }();
    const uint32_t class_g = call_stripes <= dec_small_max || (cls_small && small_dec_cls) ? 1u : class_g_big;
    const bool small_dec = call_stripes <= dec_small_max;
    auto dec_args = [&](const std::pair<uint64_t, size_t> &o) {
        const uint64_t cs = o.first >> 32;
        const uint32_t sc = (uint32_t)(cs / (uint64_t)h.alpha);
        DecArgs a{};
        a.jobs = A.at<GpeJob>(o.second);
        if (in_store) {
            a.patterns = c->dstore.pats.as<GpePattern>();
            a.hdrs = c->dstore.hdrs.as<DecProgHdr>();
            a.steps = c->dstore.steps.as<DecStepP>();
            a.step_off = c->dstore.soff.as<uint32_t>();
        } else {
            a.patterns = A.at<GpePattern>(pat_off);
            a.hdrs = A.at<DecProgHdr>(hdr_off);
            a.steps = A.at<DecStepP>(step_off);
            a.step_off = A.at<uint32_t>(soff_off);
        }
        a.njobs = (uint32_t)groups[o.first].size();
        a.words_per_stripe = (sc + 3) / 4;
        a.cs = (uint32_t)cs; a.sc = sc; a.n = (uint32_t)n; a.nk = (uint32_t)h.k;
        a.lds_rows = lds_rows;
        a.nscratch_max = nscr_max;
        a.in_stride = group_in_stride[o.first];
        a.out_stride = cs;
        a.gmax = small_dec ? 1u : 0u;
        return a;
    };
    auto fixed_args = [&](const Fixed &f, uint8_t *scratch) {
        const uint64_t cs = f.key >> 32;
        dfix_args a{};
        a.jobs = reinterpret_cast<const dfix::Job *>(A.at<GpeJob>(f.off));
        a.scratch = scratch;
        a.in_stride = group_in_stride[f.key];
        a.out_stride = cs;
        a.njobs = (uint32_t)f.jobs.size();
        a.sc = (uint32_t)(cs / (uint64_t)h.alpha);
        const DecJitGeom geo = dec_jit_geom(a.sc);  // the geometry the kernel was built for
        a.wps = geo.wps;
        a.wgs_per_stripe = geo.wgs;
        a.n = (uint32_t)n;
        a.nscratch = f.k->nscratch;
        return a;
    };
    size_t scratch_bytes = 0;
    for (auto &o : offs)
        if (staged_group(o.first)) scratch_bytes = std::max(scratch_bytes, decode_stage_scratch_bytes(dec_args(o)));
    for (const Fixed &f : fixed) {
        const dfix_args a = fixed_args(f, nullptr);
        const DecJitGeom geo = dec_jit_geom(a.sc);
        const size_t b = (size_t)a.njobs * a.wgs_per_stripe * std::max(a.nscratch, 1u) * geo.G * 64u * geo.wb;
        scratch_bytes = std::max(scratch_bytes, b);
    }
    // the class launches may run side by side: each its own scratch range, after the others'
    size_t cls_bytes = 0;
    for (const ClassGrp &cg : cls) {
        const uint32_t sc = (uint32_t)((cg.key >> 32) / (uint64_t)h.alpha);
        cls_bytes += dec_class_scratch_bytes(cg.id, (uint32_t)cg.jobs.size(), sc, class_g);
    }
    const size_t cls_off = (scratch_bytes + 255) & ~(size_t)255;
    if (cls_bytes) scratch_bytes = cls_off + cls_bytes;
    uint8_t *scratch = nullptr;
    if (scratch_bytes) {
        r = A.workspace(scratch_bytes, s, &scratch);
        if (r) return r;
    }
    uint8_t *const cls_scratch = scratch ? scratch + cls_off : nullptr;
    KTimer kt(s);
    for (const Fixed &f : fixed) {
        const dfix_args a = fixed_args(f, scratch);
        TE_HIP(launch_dec_fixed(*f.k, a, dec_jit_geom(a.sc).G, s));
    }
    if (!cls.empty()) {
        // the class groups side by side on up to 1 + kClsSide streams, largest first, each with
        // its own scratch range: one class's launch has a 100-step chain as its floor whatever
        // its size, so groups one after another leave the GPU idle at every tail
        const int ns = std::min<int>(class_streams, (int)cls.size());
        std::vector<size_t> order(cls.size());
        for (size_t i = 0; i < order.size(); i++) order[i] = i;
        std::stable_sort(order.begin(), order.end(), [&](size_t x, size_t y) { return cls[x].jobs.size() > cls[y].jobs.size(); });
        hipStream_t ss[1 + te_clay::kClsSide] = {s};
        if (ns > 1) {
            if (!c->cls_fork) TE_HIP(hipEventCreateWithFlags(&c->cls_fork, hipEventDisableTiming));
            TE_HIP(hipEventRecord(c->cls_fork, s));
            for (int i = 1; i < ns; i++) {
                if (!c->cls_s[i - 1]) TE_HIP(hipStreamCreateWithFlags(&c->cls_s[i - 1], hipStreamNonBlocking));
                if (!c->cls_join[i - 1]) TE_HIP(hipEventCreateWithFlags(&c->cls_join[i - 1], hipEventDisableTiming));
                TE_HIP(hipStreamWaitEvent(c->cls_s[i - 1], c->cls_fork, 0));
                ss[i] = c->cls_s[i - 1];
            }
        }
        const GpePattern *pp = in_store ? c->dstore.pats.as<GpePattern>() : A.at<GpePattern>(pat_off);
        size_t scr_at = 0;
        for (size_t k = 0; k < order.size(); k++) {
            const ClassGrp &cg = cls[order[k]];
            const uint64_t cs = cg.key >> 32;
            const uint32_t sc = (uint32_t)(cs / (uint64_t)h.alpha);
            TE_HIP(launch_dec_class(cg.id, A.at<GpeJob>(cg.off), pp, (uint32_t)cg.jobs.size(), sc, group_in_stride[cg.key],
                                    cs, (uint32_t)n, cls_scratch + scr_at, class_g, ss[k % (size_t)ns]));
            scr_at += dec_class_scratch_bytes(cg.id, (uint32_t)cg.jobs.size(), sc, class_g);
        }
        for (int i = 1; i < ns; i++) {
            TE_HIP(hipEventRecord(c->cls_join[i - 1], ss[i]));
            TE_HIP(hipStreamWaitEvent(s, c->cls_join[i - 1], 0));
        }
    }
    for (auto &o : offs) {
        if (staged_group(o.first)) {
            DecArgs a = dec_args(o);
            a.scratch = scratch;
            TE_HIP(launch_decode_stage(a, s));
            continue;
        }
        const uint64_t cs = o.first >> 32;
        const uint32_t sc = (uint32_t)(cs / (uint64_t)h.alpha);
        const uint32_t wps = sc >= 4 ? (sc + 3) / 4 : 1;
        GpeArgs a{};
        a.jobs = A.at<GpeJob>(o.second);
        a.patterns = A.at<GpePattern>(pat_off);
        a.plane_pool = A.at<uint16_t>(pool_off);
        a.njobs = (uint32_t)groups[o.first].size();
        a.word_base = 0;
        a.word_end = wps;
        a.groups_per_stripe = (wps + kGpeWords - 1) / kGpeWords;
        a.cs = (uint32_t)cs; a.sc = sc; a.q = h.q; a.t = h.t; a.k = h.k; a.nu = h.nu; a.n = n; a.alpha = h.alpha;
        a.in_stride = group_in_stride[o.first];
        a.out_stride = cs;
        a.in_rotated = rotated ? 1u : 0u;
        a.out_rotated = 0;
        a.out_mask = (h.k >= 64) ? ~0ull : ((1ull << h.k) - 1ull);
        for (int i = 0; i < 16; i++) a.qpow[i] = h.qpow[i];
        TE_HIP(launch_gpe(a, max_er, s));
    }
    kt.stop();
    if (in_store) TE_HIP(c->dstore.readers.record(s));  // a later call that empties the store waits for these launches
    return A.mark_done(s);
}

// ------------------------------------------------------------------------------------------
// Repair
// ------------------------------------------------------------------------------------------
struct RepItem {
    const te_repair_plan *plan;
    const uint64_t *helper_off;  // [n] offsets into d_helpers by slice id (UINT64_MAX = absent)
    uint64_t out_off;
    const uint8_t *meta;         // 48 bytes or null (raw)
};

int repair_enqueue(te_clay *c, const uint8_t *d_helpers, const RepItem *items, size_t nitems, uint8_t *d_out,
                   hipStream_t s) {
    const ClayHost &h = c->h;
    using RepKey = te_clay::RepKey;
    std::unordered_map<RepKey, uint32_t, te_clay::RepKeyHash> pat_index;  // -> pattern id of this call
    std::vector<RepPattern> pats;
    std::vector<const te_clay::RepCache *> cached;  // entries stay put: the map is trimmed only here
    if (c->rep_cache.size() > 4096) c->rep_cache.clear();
    std::vector<uint16_t> pool, pind;
    // jobs by (chunk size, folded kernel or not), in first-seen order; usually one chunk size
    struct Group { uint64_t cs; std::vector<RepJob> jobs[2]; };
    std::vector<Group> groups;
    std::vector<MetaJob> metas;
    uint32_t max_er = 0;
    uint64_t run[64];
    RepKey last_key{~0ull, ~0u};
    uint32_t last_pid = 0;
    for (size_t i = 0; i < nitems; i++) {
        const te_repair_plan *p = items[i].plan;
        if (p->n > 64) return TE_ERR_INVALID_ARG;
        std::fill(run, run + p->n, 0ull);
        Group *grp = nullptr;
        for (Group &g : groups)
            if (g.cs == p->cs) grp = &g;
        if (!grp) {
            groups.push_back(Group{p->cs, {}});
            grp = &groups.back();
            grp->jobs[0].reserve(nitems * p->ns);
        }
        const uint32_t sc = (uint32_t)(p->cs / (uint64_t)h.alpha);
        for (uint32_t st = 0; st < p->ns; st++) {
            const uint32_t *hsh = p->helper_shard.data() + (size_t)st * p->d;
            RepKey key{0, p->lost_shard[st]};
            for (uint32_t j = 0; j < p->d; j++) key.helpers |= 1ull << hsh[j];
            uint32_t pid;
            auto f = key == last_key ? pat_index.end() : pat_index.find(key);
            if (key == last_key) {
                pid = last_pid;
            } else if (f == pat_index.end()) {
                auto cf = c->rep_cache.find(key);
                if (cf == c->rep_cache.end()) {
                    te_clay::RepCache rc;
                    const std::vector<int> hs(hsh, hsh + p->d);
                    if (!h.rep_pattern((int)p->lost_shard[st], hs, rc.P, rc.pool, rc.pind)) return TE_ERR_CLAY;
                    if (h.nu == 0 && h.n == 2 * h.q && !g_no_fold_repair)
                        rc.fold = repair_fold_column(h.q, h.t, h.k, rc.P.beta, 8, rc.P.lost, rc.P.erased_mask,
                                                     rc.P.aloof_mask);
                    rc.prog_ok = repair_stage_supported(h.q, rc.P.beta, 8, rc.P.nerased, rc.P.nknown, rc.P.aloof_mask) &&
                                 h.rep_prog(rc.P, rc.pool.data(), rc.pind.data(), rc.prog);
                    cf = c->rep_cache.emplace(key, std::move(rc)).first;
                }
                const te_clay::RepCache &rc = cf->second;
                pid = (uint32_t)pats.size();
                pats.push_back(rc.P);
                pats.back().planes_off = (uint32_t)pool.size();
                pool.insert(pool.end(), rc.pool.begin(), rc.pool.end());
                pind.insert(pind.end(), rc.pind.begin(), rc.pind.end());
                cached.push_back(&rc);
                pat_index[key] = pid;
                max_er = std::max(max_er, rc.P.nerased);
            } else {
                pid = f->second;
            }
            last_key = key;
            last_pid = pid;
            RepJob j{};
            const uint8_t *any = nullptr;
            for (uint32_t hj = 0; hj < p->d; hj++) {
                const uint32_t sl = p->helper_slice[st * p->d + hj];
                const uint64_t off = items[i].helper_off[sl];
                if (off == ~0ull) return TE_ERR_MISSING_HELPER;
                any = j.helper[h.ext_to_int((int)hsh[hj])] = d_helpers + off + run[sl];
                run[sl] += (uint64_t)p->beta * p->sc;
            }
            j.out = d_out + items[i].out_off + (uint64_t)st * p->cs;
            j.pattern = pid;
            // stripes whose pattern is one of the folded kernel's helper sets of Clay(20,7,16) (all
            // 19 others available, or one of the other column's first 7 down) go to that kernel,
            // the rest to the staged / generic kernel
            const int fc = sc >= 8 ? cached[pid]->fold : -1;
            if (fc >= 0) {  // the folded kernel loads every node unconditionally (repair_fold.hip)
                j.aux = pats[pid].lost % (uint32_t)h.q | (uint32_t)fc << 8;
                for (int nd = 0; nd < h.qt; nd++)
                    if (!j.helper[nd]) j.helper[nd] = any;
            }
            grp->jobs[fc >= 0 ? 0 : 1].push_back(j);
        }
        if (items[i].meta) {
            MetaJob m{};
            m.dst = d_out + items[i].out_off + (uint64_t)p->ns * p->cs;
            m.slice_len = 0;
            for (int w = 0; w < 6; w++) m.words[w] = get_u64(items[i].meta + 8 * w);
            metas.push_back(m);
        }
    }
    // staged kernel when every pattern outside the folded kernel has a plane program
    std::vector<RepProg> progs(pats.size());
    bool staged = true;
    for (size_t i = 0; i < pats.size(); i++) {
        progs[i] = cached[i]->prog;
        if (cached[i]->fold < 0) staged = staged && cached[i]->prog_ok;
    }
    Arena &A = c->rep;
    A.img.clear();
    const size_t pat_off = A.put(pats.data(), pats.size() * sizeof(RepPattern));
    const size_t prog_off = staged ? A.put(progs.data(), progs.size() * sizeof(RepProg)) : 0;
    const size_t pool_off = A.put(pool.data(), pool.size() * sizeof(uint16_t));
    const size_t pind_off = A.put(pind.data(), pind.size() * sizeof(uint16_t));
    const size_t meta_off = A.put(metas.data(), metas.size() * sizeof(MetaJob));
    // one launch per chunk size for the folded kernel (every helper set), one for the others
    struct Launch { uint64_t cs; int fold; size_t off, njobs; };
    std::vector<Launch> offs;
    for (Group &g : groups)
        for (int f = 0; f < 2; f++)
            if (!g.jobs[f].empty())
                offs.push_back({g.cs, f == 0 ? 0 : -1, A.put(g.jobs[f].data(), g.jobs[f].size() * sizeof(RepJob)),
                                g.jobs[f].size()});
    int r = A.upload(s);
    if (r) return r;
    KTimer kt(s);
    if (!metas.empty()) TE_HIP(launch_meta(A.at<MetaJob>(meta_off), (uint32_t)metas.size(), 1u, s));
    for (auto &o : offs) {
        const uint64_t cs = o.cs;
        const uint32_t sc = (uint32_t)(cs / (uint64_t)h.alpha);
        const uint32_t wps = sc >= 4 ? (sc + 3) / 4 : 1;
        RepArgs a{};
        a.jobs = A.at<RepJob>(o.off);
        a.patterns = A.at<RepPattern>(pat_off);
        a.plane_pool = A.at<uint16_t>(pool_off);
        a.plane_ind = A.at<uint16_t>(pind_off);
        a.njobs = (uint32_t)o.njobs;
        a.words_per_stripe = wps;
        a.groups_per_stripe = (wps + kGpeWords - 1) / kGpeWords;
        a.cs = (uint32_t)cs; a.sc = sc; a.q = h.q; a.t = h.t; a.alpha = h.alpha;
        for (int i = 0; i < 16; i++) a.qpow[i] = h.qpow[i];
        if (o.fold >= 0) {
            TE_HIP(launch_repair_fold(a, s));
        } else if (staged && sc >= 8) {  // staged kernel: coalesced loads, whole-row stores
            a.progs = A.at<RepProg>(prog_off);
            TE_HIP(launch_repair_stage(a, s));
        } else {
            TE_HIP(launch_repair(a, max_er, s));
        }
    }
    kt.stop();
    return A.mark_done(s);
}

// ClayCoder::plan_repair maps every minimum_to_repair failure to RepairError::Clay(e.to_string())
// (repair.rs:59-62); the detail text goes to te_last_error_detail().
int clay_plan_error(int r, int lost_shard, size_t navail, int d) {
    if (r == -1)
        snprintf(g_last_error, sizeof(g_last_error), "minimum_to_repair: need %d helpers, %zu available (lost shard %d)",
                 d, navail, lost_shard);
    else
        snprintf(g_last_error, sizeof(g_last_error),
                 "minimum_to_repair: a column-mate of lost shard %d is not available", lost_shard);
    return TE_ERR_CLAY;
}

int build_plan(const te_clay *c, int rotated, uint32_t lost, const uint32_t *avail, size_t navail, uint64_t ns,
               uint64_t cs, te_repair_plan **out) {
    const ClayHost &h = c->h;
    if (lost >= (uint32_t)h.n) return TE_ERR_INVALID_SLICE;
    if (cs % (uint64_t)h.alpha) return TE_ERR_INVALID_LAYOUT;
    te_repair_plan *p = new (std::nothrow) te_repair_plan();
    if (!p) return TE_ERR_OUT_OF_MEMORY;
    p->lost = lost; p->ns = (uint32_t)ns; p->d = (uint32_t)h.d; p->beta = (uint32_t)h.beta; p->n = (uint32_t)h.n;
    p->cs = cs; p->sc = cs / (uint64_t)h.alpha;
    for (uint64_t st = 0; st < ns; st++) {
        const int ls = (int)te_slice_to_shard(rotated, (uint32_t)h.n, (uint32_t)st, lost);
        std::vector<int> av;
        for (size_t i = 0; i < navail; i++) {
            if (avail[i] >= (uint32_t)h.n) { delete p; return TE_ERR_INVALID_SLICE; }
            av.push_back((int)te_slice_to_shard(rotated, (uint32_t)h.n, (uint32_t)st, avail[i]));
        }
        std::vector<int> hs;
        const int r = h.min_to_repair(ls, av, hs);
        if (r) { delete p; return clay_plan_error(r, ls, navail, h.d); }
        const std::vector<int> planes = h.repair_planes(ls);
        p->lost_shard.push_back((uint32_t)ls);
        for (int sh : hs) {
            p->helper_shard.push_back((uint32_t)sh);
            p->helper_slice.push_back(te_shard_to_slice(rotated, (uint32_t)h.n, (uint32_t)st, (uint32_t)sh));
            for (int z : planes) p->sub_chunks.push_back((uint32_t)z);
        }
    }
    *out = p;
    return TE_OK;
}

}  // namespace

// Host -> host encode pipeline (te_encode_batch_host), optionally with the slice commitments of
// BlobEncoder::encode_with_proofs (sdk/src/codec/encoder.rs:220-260): per object the n leaf hashes,
// the root and n proofs, computed on the device from the window's slices before they leave HBM.
struct CommitOut {
    uint8_t *leaf, *root, *proof;  // host: nobj * n * 32, nobj * 32, nobj * n * height * 32 (or null)
    uint32_t height;
};

// Host <-> device copy runs of a window: consecutive objects contiguous on the host move with one DMA.
struct CopyRun { uint64_t host, dev, len; };

// Device layout of objects [a, b) placed from offsets (din, dout) of a slot's buffers: the encode
// descriptors (`local`, offsets relative to the buffers) and the H2D / D2H copy runs.
static void window_layout(const te_object *objs, const std::vector<uint64_t> &out_bytes, size_t a, size_t b,
                          uint64_t din, uint64_t dout, std::vector<te_object> &local, std::vector<CopyRun> &hin,
                          std::vector<CopyRun> &hout) {
    auto add_run = [](std::vector<CopyRun> &v, uint64_t host, uint64_t dev, uint64_t len) {
        if (!len) return;
        if (!v.empty() && v.back().host + v.back().len == host && v.back().dev + v.back().len == dev)
            v.back().len += len;
        else
            v.push_back({host, dev, len});
    };
    local.clear();
    hin.clear();
    hout.clear();
    for (size_t o = a; o < b; o++) {
        local.push_back(te_object{din, objs[o].blob_len, dout, objs[o].chunk_index});
        add_run(hin, objs[o].data_off, din, objs[o].blob_len);
        add_run(hout, objs[o].out_off, dout, out_bytes[o]);
        din += (objs[o].blob_len + 15) & ~15ull;  // device copies 16-byte aligned
        dout += out_bytes[o];
    }
}

static int copy_runs(const std::vector<CopyRun> &runs, uint8_t *dev, const uint8_t *host, hipMemcpyKind kind,
                     hipStream_t s) {
    for (const CopyRun &r : runs) {
        const bool h2d = kind == hipMemcpyHostToDevice;
        void *dst = h2d ? (void *)(dev + r.dev) : (void *)(host + r.host);
        const void *src = h2d ? (const void *)(host + r.host) : (const void *)(dev + r.dev);
        TE_HIP(hipMemcpyAsync(dst, src, r.len, kind, s));
    }
    return TE_OK;
}

static int encode_host_impl(te_clay *c, const te_slicer_cfg *cfg, const uint8_t *h_data, const te_object *objs,
                            size_t nobj, uint8_t *h_out, size_t window_bytes) {
    if (!c || !cfg || (!objs && nobj) || (nobj && (!h_data || !h_out))) return TE_ERR_INVALID_ARG;
    if (device_count() <= 0) return TE_ERR_NO_DEVICE;
    // default window 128 MiB (1024 x 4 MiB pinned: 14.1 GiB/s against 12.6 at 1 GiB -- smaller
    // windows overlap the H2D, kernels and D2H more finely; 64 MiB varied 11.1-14.3, below that the
    // per-window launches cost more; a fourth slot measured slower)
    if (window_bytes == 0) window_bytes = (size_t)128 << 20;
    const uint32_t n = (uint32_t)c->h.n;
    std::vector<uint64_t> out_bytes(nobj);
    for (size_t i = 0; i < nobj; i++) {
        te_geometry g;
        te_slicer_geometry(c, objs[i].blob_len, &g);
        out_bytes[i] = (uint64_t)n * g.slice_len;
    }
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard dg(c->device);
    TE_HIP(dg.err);
    // three slot streams: the handle's two pipe streams and its own stream -- the same three the
    // commit pipeline uses (commit_streams), so with the caller's stream a process holds four
    // streams for its four hardware queues (GPU_MAX_HW_QUEUES) whichever host paths it runs
    if (int r0 = ensure_stream(c)) return r0;
    for (int k = 0; k < 2; k++)
        if (!c->pipe[k].s) TE_HIP(hipStreamCreateWithFlags(&c->pipe[k].s, hipStreamNonBlocking));
    auto slot_stream = [&](size_t k) { return k < 2 ? c->pipe[k].s : c->stream; };
    int rc = TE_OK;
    size_t i = 0, w = 0;
    std::vector<te_object> local;
    std::vector<CopyRun> hin, hout;
    while (i < nobj && rc == TE_OK) {
        // window [i, j): at least one object, in + out bytes within window_bytes
        size_t j = i;
        uint64_t in_sz = 0, out_sz = 0;
        while (j < nobj && (j == i || in_sz + out_sz + objs[j].blob_len + out_bytes[j] <= window_bytes)) {
            in_sz += (objs[j].blob_len + 15) & ~15ull;  // device copies 16-byte aligned
            out_sz += out_bytes[j];
            j++;
        }
        te_clay::Slot &sl = c->pipe[w % te_clay::kPipe];
        const hipStream_t ss = slot_stream(w % te_clay::kPipe);
        if ((rc = hip_status(sl.in.ensure(in_sz + 16))) || (rc = hip_status(sl.out.ensure(out_sz)))) break;
        window_layout(objs, out_bytes, i, j, 0, 0, local, hin, hout);
        if ((rc = copy_runs(hin, sl.in.as<uint8_t>(), h_data, hipMemcpyHostToDevice, ss))) break;
        rc = encode_enqueue(c, cfg, sl.in.as<uint8_t>(), local.data(), local.size(), sl.out.as<uint8_t>(), ss,
                            false, &sl.arena);
        if (rc) break;
        if ((rc = copy_runs(hout, sl.out.as<uint8_t>(), h_out, hipMemcpyDeviceToHost, ss))) break;
        i = j;
        w++;
    }
    for (size_t k = 0; k < te_clay::kPipe; k++) {
        const int r2 = hip_status(hipStreamSynchronize(slot_stream(k)));
        if (rc == TE_OK) rc = r2;
    }
    return rc;
}

// te_encode_commit_batch_host / te_stream_submit: encode + commitments, host -> host.  The leaf
// kernel's time per launch is one slice stream's SHA-256 (~27-30 ms for a 715 KB slice, DESIGN
// §4.4) whatever the number of objects, so hashing must not sit between a window's encode and its
// D2H copy (hashing each window on its slot stream: 9.6-10.5 GiB/s).  Objects go through the
// device in GROUPS of at most `group_bytes` (input + output); a group's slices stay in one of three
// resident group buffers until hashed.  Each group is encoded in copy windows of <= 128 MiB that
// rotate over two slot streams (H2D of the window into the slot's input buffer, encode into the
// group buffer, D2H of its slices: copies stay in stream order behind kernels and overlap across
// slots).  The hash stream hashes a whole group at once (one leaf/tree launch per run of equal
// slice lengths, then the D2H of leaf hashes, roots and proofs) after every slot stream has passed
// the group's last window.  A group buffer is refilled once its hashing is done.  Every ordering
// is a GPU-side event wait, so the host enqueues a group without blocking: consecutive calls on a
// CommitPipe (te_stream_submit's windows) overlap one window's encode with the previous one's
// hashing and copies.

// One device's pipeline state.  The one-shot entry point points it at the handle's slot streams,
// buffers and arenas (c->pipe, c->stream); a stream writer owns its own (te_stream_writer).
struct CommitPipe {
    static constexpr int R = te_clay::kPipe;  // resident group buffers
    // copy windows rotate over two slot streams: with the hashing stream and the caller's stream
    // that is four streams for four hardware queues (three slots: 9.5 against 12.0 GiB/s on one
    // box, 1024 x 4 MiB, in a process that had used its current stream, as bench.py has)
    static constexpr int S = 2;
    hipStream_t ss[S] = {}, hs = nullptr;
    DevBuf *in[S] = {};
    Arena *arena[S] = {};
    DevBuf *gout[R] = {}, *gcom[R] = {};
    // per slot stream "encoded its latest window" and "copied it out", per group buffer "hashed"
    // (which implies copied out); a stream wait binds to the record current when enqueued
    hipEvent_t ev_enc[S] = {}, ev_slot[S] = {}, ev_hashed[R] = {};
    bool slot_used[S] = {}, hashed_pending[R] = {};
    bool grow_ok = false;  // buffers may grow (after draining their users); else pre-sized
    size_t w = 0, groups = 0;

    int make_events() {
        for (hipEvent_t *e : {ev_enc, ev_slot})
            for (int k = 0; k < S; k++)
                if (!e[k]) TE_HIP(hipEventCreateWithFlags(&e[k], hipEventDisableTiming));
        for (int r = 0; r < R; r++)
            if (!ev_hashed[r]) TE_HIP(hipEventCreateWithFlags(&ev_hashed[r], hipEventDisableTiming));
        return TE_OK;
    }
    void destroy_events() {
        for (hipEvent_t *e : {ev_enc, ev_slot})
            for (int k = 0; k < S; k++)
                if (e[k]) (void)hipEventDestroy(e[k]), e[k] = nullptr;
        for (int r = 0; r < R; r++)
            if (ev_hashed[r]) (void)hipEventDestroy(ev_hashed[r]), ev_hashed[r] = nullptr;
    }
};

// One call's (or one submitted window's) objects and their commitment outputs.
struct CommitBatch {
    const uint8_t *h_data = nullptr;
    const te_object *objs = nullptr;
    size_t nobj = 0;
    uint8_t *h_out = nullptr;
    CommitOut co{};
    uint32_t n = 0;
    std::vector<uint64_t> out_bytes, slice_len;
    uint64_t leaf_b = 0, proof_b = 0;
    uint64_t in_bytes(size_t o) const { return (objs[o].blob_len + 15) & ~15ull; }  // device copies 16-byte aligned
};

static int commit_prepare(const te_clay *c, CommitBatch &B) {
    B.n = (uint32_t)c->h.n;
    B.out_bytes.assign(B.nobj, 0);
    B.slice_len.assign(B.nobj, 0);
    for (size_t i = 0; i < B.nobj; i++) {
        te_geometry g;
        te_slicer_geometry(c, B.objs[i].blob_len, &g);
        B.slice_len[i] = g.slice_len;
        B.out_bytes[i] = (uint64_t)B.n * g.slice_len;
        if (g.slice_len % 4) return TE_ERR_INVALID_ARG;  // the leaf kernel reads dwords
        // encode_enqueue's per-object check, made before a window touches a shared group
        if (g.chunk_size % (size_t)c->h.alpha || g.slice_len > 0xffffffffull || g.chunk_size > 0xffffffffull)
            return TE_ERR_TOO_MUCH_DATA;
    }
    B.leaf_b = (uint64_t)B.n * TE_HASH_SIZE;
    B.proof_b = B.co.proof ? B.leaf_b * B.co.height : 0;
    return TE_OK;
}

// Groups [gcut[x], gcut[x+1]) of about equal size (a small last group would be hashed after the
// previous one), and each group's copy windows.
struct CommitPlan {
    std::vector<size_t> gcut{0};
    std::vector<std::vector<size_t>> wcut;  // per group: window boundaries, first = group start
    uint64_t max_win_in = 16, max_group_out = 0, max_group_obj = 0;
};
static void commit_plan(const CommitBatch &B, uint64_t group_bytes, uint64_t copy_bytes, CommitPlan &P) {
    uint64_t total = 0;
    for (size_t o = 0; o < B.nobj; o++) total += B.objs[o].blob_len + B.out_bytes[o];
    const uint64_t target = total / std::max<uint64_t>(1, (total + group_bytes - 1) / group_bytes);
    for (size_t i = 0; i < B.nobj;) {
        size_t j = i;
        uint64_t gsz = 0, gout = 0;
        while (j < B.nobj && (j == i || (gsz < target && gsz + B.objs[j].blob_len + B.out_bytes[j] <= group_bytes))) {
            gsz += B.objs[j].blob_len + B.out_bytes[j];
            gout += B.out_bytes[j];
            j++;
        }
        std::vector<size_t> wc{i};
        for (size_t a = i; a < j;) {
            size_t b = a;
            uint64_t win = 0, win_in = 0;
            while (b < j && (b == a || win + B.objs[b].blob_len + B.out_bytes[b] <= copy_bytes)) {
                win += B.objs[b].blob_len + B.out_bytes[b];
                win_in += B.in_bytes(b);
                b++;
            }
            P.max_win_in = std::max(P.max_win_in, win_in + 16);
            wc.push_back(b);
            a = b;
        }
        P.wcut.push_back(std::move(wc));
        P.max_group_out = std::max(P.max_group_out, gout);
        P.max_group_obj = std::max<uint64_t>(P.max_group_obj, j - i);
        P.gcut.push_back(j);
        i = j;
    }
}

// One object's slices copied out in row pieces (host-hashed groups, pinned host output): piece p
// is bytes [beg[p], beg[p+1]) of every slice, landed once ev[p] has completed.  The host hashing
// tasks follow the pieces as they land instead of waiting for the whole window's D2H.
//
// The piece events come from a per-device pool and are waited for by polling (hipEventQuery with
// short sleeps), not by blocking-sync waits: with one blocking-sync event created, waited for by
// interrupt and destroyed per piece (ten per 64 MiB chunk), the SDK-shape stream slowed to
// 7.1 GiB/s (chunk latency 33.6 ms, against 15-16 ms in a fresh process) once the process had run
// the earlier copy-inclusive legs -- and ran 11.6 GiB/s in that same state with no pieces
// (r05, gpurun_out/r5h).  Polling costs a worker a few microseconds per check and no interrupt.
class EventPool {
  public:
    static EventPool &get(int device) {
        static std::mutex mu;
        static std::map<int, EventPool *> pools;
        std::lock_guard<std::mutex> g(mu);
        EventPool *&p = pools[device];
        if (!p) p = new EventPool();  // never destroyed (events outlive static destructors' order)
        return *p;
    }
    hipError_t acquire(hipEvent_t &e) {
        {
            std::lock_guard<std::mutex> g(m_);
            if (!free_.empty()) {
                e = free_.back();
                free_.pop_back();
                return hipSuccess;
            }
        }
        return hipEventCreateWithFlags(&e, hipEventDisableTiming);
    }
    void release(hipEvent_t e) {
        std::lock_guard<std::mutex> g(m_);
        if (free_.size() < 4096) free_.push_back(e);
        else (void)hipEventDestroy(e);
    }

  private:
    std::mutex m_;
    std::vector<hipEvent_t> free_;
};

// Wait for an event by polling: a short spin, then sleeps of 20 us (hashing workers waiting for
// the next row piece of their slices).
static hipError_t event_wait_poll(hipEvent_t e) {
    for (int i = 0;; i++) {
        const hipError_t r = hipEventQuery(e);
        if (r != hipErrorNotReady) return r;
        if (i < 16) std::this_thread::yield();
        else std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
}

struct PieceEvents {
    int device = 0;
    std::vector<hipEvent_t> ev;
    std::vector<uint64_t> beg;
    ~PieceEvents() {
        EventPool &pool = EventPool::get(device);
        for (hipEvent_t e : ev) pool.release(e);
    }
};

// Row pieces of kPiece bytes per slice (measurement option TEC_DEBUG_KNOBS=1 TEC_D2H_PIECE=bytes,
// 0 = one copy per window as before; TEC_D2H_ROWS=1 copies each piece slice by slice instead of
// one 2-D copy).  Objects whose slices are shorter than two pieces are copied whole.
static uint64_t d2h_piece_bytes() {
    static const uint64_t v = [] {
        const char *s = tec_knob("TEC_D2H_PIECE");
        return s ? (uint64_t)strtoull(s, nullptr, 10) : (uint64_t)1 << 20;
    }();
    return v;
}
static bool d2h_rows() {
    static const bool v = [] {
        const char *s = tec_knob("TEC_D2H_ROWS");
        return s && s[0] == '1';
    }();
    return v;
}

// Page-locked (te_host_alloc / te_host_register / hipHostMalloc): row-piece copies of pageable
// memory would each go through the driver's staging.
static bool host_pinned(const void *p) {
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

// Copy object o's n slices (slice_len bytes each, at dev / host) out in row pieces on stream s.
static int copy_out_pieces(uint8_t *host, const uint8_t *dev, uint64_t slice_len, uint32_t n, int device,
                           hipStream_t s, std::shared_ptr<PieceEvents> &out) {
    const uint64_t piece = d2h_piece_bytes();
    auto pe = std::make_shared<PieceEvents>();
    pe->device = device;
    for (uint64_t off = 0; off < slice_len;) {
        const uint64_t w = std::min(piece, slice_len - off);
        if (d2h_rows()) {
            for (uint32_t i = 0; i < n; i++)
                TE_HIP(hipMemcpyAsync(host + i * slice_len + off, dev + i * slice_len + off, w, hipMemcpyDeviceToHost, s));
        } else {
            TE_HIP(hipMemcpy2DAsync(host + off, slice_len, dev + off, slice_len, w, n, hipMemcpyDeviceToHost, s));
        }
        hipEvent_t e = nullptr;
        TE_HIP(EventPool::get(device).acquire(e));
        pe->ev.push_back(e);
        pe->beg.push_back(off);
        TE_HIP(hipEventRecord(e, s));
        off += w;
    }
    pe->beg.push_back(slice_len);
    out = std::move(pe);
    return TE_OK;
}

// A group's commitment outputs on the device: leaf hashes of row q at q * leaf_b, roots after
// `rows_cap` rows of leaves, proofs after the roots (rows = objects, in group order).
struct GroupSeg {
    CommitOut co;            // the host outputs of the segment's window
    size_t obj0 = 0;         // first object of the segment in its window (host output index)
    uint64_t row0 = 0, cnt = 0, gout_off = 0;
    std::vector<uint64_t> slice_len, out_bytes;
    const uint8_t *h_out = nullptr;  // the window's host slices (host-hashed groups read them)
    std::vector<uint64_t> h_off;     // per object: its slices at h_out + h_off
    std::vector<std::shared_ptr<PieceEvents>> pieces;  // per object: row pieces, or null (copied whole)
};
struct OpenGroup {
    bool open = false;
    size_t r = 0;                 // group buffer
    uint64_t out_off = 0, rows = 0, rows_cap = 0, bytes = 0;
    bool slots_used[CommitPipe::S] = {};
    std::vector<GroupSeg> segs;
};

// Open a group in the next group buffer: its previous group must be hashed (and copied out)
// before the slot streams write into it.  need_out / need_rows: what the first segment needs
// (a buffer grows only after the work queued on it has drained).
static int group_open(CommitPipe &P, OpenGroup &G, uint64_t need_out, uint64_t need_rows, uint64_t row_b) {
    constexpr int S = CommitPipe::S;
    const size_t r = P.groups % CommitPipe::R;
    if (P.gout[r]->cap < need_out || P.gcom[r]->cap < need_rows * row_b) {
        if (!P.grow_ok) return TE_ERR_INVALID_ARG;
        if (P.hashed_pending[r]) TE_HIP(hipEventSynchronize(P.ev_hashed[r]));
        TE_HIP(P.gout[r]->ensure(need_out));
        TE_HIP(P.gcom[r]->ensure(need_rows * row_b));
    }
    if (P.hashed_pending[r])
        for (int k = 0; k < S; k++) TE_HIP(hipStreamWaitEvent(P.ss[k], P.ev_hashed[r], 0));
    G.open = true;
    G.r = r;
    G.out_off = G.rows = G.bytes = 0;
    G.rows_cap = row_b ? P.gcom[r]->cap / row_b : 0;
    for (int k = 0; k < S; k++) G.slots_used[k] = false;
    G.segs.clear();
    return TE_OK;
}

// Encode group x of plan L into the open group (after its earlier segments): H2D, encode and D2H
// of the slices per copy window, rotating over the slot streams.  `last`: the caller's final group
// -- its encodes run ahead of the copies (one D2H per two encodes on a slot, the rest after the
// group's last encode), so its hashing, the only exposed one, starts about halfway through the
// group's copies.  `pieces` (a host-hashed group with pinned output): each large object's slices
// are copied out in row pieces with an event per piece (copy_out_pieces).
static int group_add(te_clay *c, const te_slicer_cfg *cfg, CommitPipe &P, OpenGroup &G, const CommitBatch &B,
                     const CommitPlan &L, size_t x, bool last, bool pieces = false) {
    if (last) pieces = false;
    constexpr int S = CommitPipe::S;
    const size_t i = L.gcut[x], j = L.gcut[x + 1];
    const std::vector<size_t> &wc = L.wcut[x];
    uint64_t win_in_max = 16;
    for (size_t y = 0; y + 1 < wc.size(); y++) {
        uint64_t win_in = 16;
        for (size_t o = wc[y]; o < wc[y + 1]; o++) win_in += B.in_bytes(o);
        win_in_max = std::max(win_in_max, win_in);
    }
    for (int k = 0; k < S; k++)
        if (P.in[k]->cap < win_in_max) {
            if (!P.grow_ok) return TE_ERR_INVALID_ARG;
            TE_HIP(hipStreamSynchronize(P.ss[k]));
            TE_HIP(P.in[k]->ensure(win_in_max));
        }
    GroupSeg seg;
    seg.co = B.co;
    seg.obj0 = i;
    seg.row0 = G.rows;
    seg.cnt = j - i;
    seg.gout_off = G.out_off;
    uint8_t *gout = P.gout[G.r]->as<uint8_t>();
    std::deque<std::vector<CopyRun>> pend[S];
    int encs[S] = {};
    uint64_t dout = G.out_off;
    std::vector<te_object> local;
    std::vector<CopyRun> hin, hout;
    int rc = TE_OK;
    for (size_t y = 0; y + 1 < wc.size() && !rc; y++) {
        const size_t a = wc[y], b = wc[y + 1];
        const int k = (int)(P.w % S);
        window_layout(B.objs, B.out_bytes, a, b, 0, dout, local, hin, hout);
        if ((rc = copy_runs(hin, P.in[k]->as<uint8_t>(), B.h_data, hipMemcpyHostToDevice, P.ss[k]))) break;
        if ((rc = encode_enqueue(c, cfg, P.in[k]->as<uint8_t>(), local.data(), local.size(), gout, P.ss[k], false,
                                 P.arena[k])))
            break;
        if ((rc = hip_status(hipEventRecord(P.ev_enc[k], P.ss[k])))) break;
        if (pieces) {
            const uint64_t pb = d2h_piece_bytes();
            uint64_t od = dout;
            for (size_t o = a; o < b && !rc; o++) {
                std::shared_ptr<PieceEvents> pe;
                if (pb && B.slice_len[o] >= 2 * pb)
                    rc = copy_out_pieces(B.h_out + B.objs[o].out_off, gout + od, B.slice_len[o], B.n, c->device, P.ss[k], pe);
                else
                    rc = hip_status(hipMemcpyAsync(B.h_out + B.objs[o].out_off, gout + od, B.out_bytes[o],
                                                   hipMemcpyDeviceToHost, P.ss[k]));
                seg.pieces.push_back(std::move(pe));
                od += B.out_bytes[o];
            }
        } else {
            pend[k].push_back(hout);
        }
        if (rc) break;
        if (!pieces && (!last || ++encs[k] % 2 == 0)) {
            if ((rc = copy_runs(pend[k].front(), gout, B.h_out, hipMemcpyDeviceToHost, P.ss[k]))) break;
            pend[k].pop_front();
        }
        P.slot_used[k] = true;
        G.slots_used[k] = true;
        for (size_t o = a; o < b; o++) dout += B.out_bytes[o];
        P.w++;
    }
    for (int k = 0; k < S && !rc; k++) {
        for (; !pend[k].empty() && !rc; pend[k].pop_front())
            rc = copy_runs(pend[k].front(), gout, B.h_out, hipMemcpyDeviceToHost, P.ss[k]);
        if (!rc && G.slots_used[k]) rc = hip_status(hipEventRecord(P.ev_slot[k], P.ss[k]));
    }
    if (rc) return rc;
    seg.h_out = B.h_out;
    for (size_t o = i; o < j; o++) {
        seg.slice_len.push_back(B.slice_len[o]);
        seg.out_bytes.push_back(B.out_bytes[o]);
        seg.h_off.push_back(B.objs[o].out_off);
        G.bytes += B.objs[o].blob_len + B.out_bytes[o];
    }
    G.out_off = dout;
    G.rows += seg.cnt;
    G.segs.push_back(std::move(seg));
    return TE_OK;
}

// Hash the open group: once every slot stream has encoded its last window (the last windows' D2H
// overlaps the hashing: 11.9 -> 12.4-12.6 GiB/s, one box), one leaf/tree launch per run of equal
// slice lengths across all its segments, then the D2H of each segment's leaf hashes, roots and
// proofs into its window's host buffers.
// root_from_leaf_hashes::<height> and create_proof_from_leaf_hashes::<height> of n leaves
// (lib/crypto/src/merkle/tree.rs:344-358, 397-455) from one set of layers: odd layers padded with
// EMPTY_ROOTS[level], proof i = the sibling at each level.
static int host_tree(const uint8_t *leaf, uint32_t n, uint32_t height, uint8_t *root, uint8_t *proof) {
    if (height == 0 || height > TE_MAX_MERKLE_TREE_HEIGHT || n == 0) return TE_ERR_INVALID_ARG;
    std::vector<std::array<uint8_t, 32>> cur(n), next;
    for (uint32_t i = 0; i < n; i++) memcpy(cur[i].data(), leaf + (size_t)i * 32, 32);
    std::array<uint8_t, 32> empty;
    sha::empty_root(0, empty.data());
    for (uint32_t l = 0; l < height; l++) {
        if (cur.size() % 2) cur.push_back(empty);
        if (proof)
            for (uint32_t i = 0; i < n; i++)
                memcpy(proof + ((size_t)i * height + l) * 32, cur[(i >> l) ^ 1].data(), 32);
        next.resize(cur.size() / 2);
        for (size_t j = 0; j < next.size(); j++) sha::hash_pair(cur[2 * j].data(), cur[2 * j + 1].data(), next[j].data());
        cur.swap(next);
        std::array<uint8_t, 32> e2;
        sha::hash_pair(empty.data(), empty.data(), e2.data());
        empty = e2;
    }
    memcpy(root, cur[0].data(), 32);
    return TE_OK;
}

// Host-hashed close (host_hash.hpp):the group's slices are hashed from the host output buffers
// once their D2H copies have landed -- one pool task per te_host_hash_lanes slices of an object
// (interleaved, hh::hash_leaves), the object's root and proofs by whichever of its tasks finishes
// last.  The group buffer is free as soon as the copies are
// done.  Returns the job the window tickets wait for.
static int group_close_host(CommitPipe &P, OpenGroup &G, uint32_t n, uint32_t height, int device,
                            std::shared_ptr<hh::Job> &job) {
    constexpr int S = CommitPipe::S;
    if (!G.open) return TE_OK;
    G.open = false;
    for (int k = 0; k < S; k++)
        if (G.slots_used[k]) TE_HIP(hipStreamWaitEvent(P.hs, P.ev_slot[k], 0));
    TE_HIP(hipEventRecord(P.ev_hashed[G.r], P.hs));
    P.hashed_pending[G.r] = true;
    P.groups++;
    hipEvent_t landed = nullptr;
    TE_HIP(hipEventCreateWithFlags(&landed, hipEventDisableTiming | hipEventBlockingSync));
    if (hipError_t e = hipEventRecord(landed, P.hs); e != hipSuccess) {
        (void)hipEventDestroy(landed);
        return hip_status(e);
    }
    job = std::make_shared<hh::Job>();
    // objects copied out in row pieces hash piece by piece as the pieces land (their tasks go to
    // the workers at once and wait on the piece events); the rest once the group's copies are done
    std::vector<std::function<void()>> tasks, streamed;
    const uint32_t lanes = (uint32_t)hh::Pool::get().lanes();
    for (const GroupSeg &sg : G.segs) {
        for (size_t q = 0; q < sg.cnt; q++) {
            const uint8_t *slices = sg.h_out + sg.h_off[q];
            const uint64_t slen = sg.slice_len[q];
            uint8_t *leaf = sg.co.leaf + (sg.obj0 + q) * (uint64_t)n * TE_HASH_SIZE;
            uint8_t *root = sg.co.root + (sg.obj0 + q) * TE_HASH_SIZE;
            uint8_t *proof = sg.co.proof ? sg.co.proof + (sg.obj0 + q) * (uint64_t)n * height * TE_HASH_SIZE : nullptr;
            auto left = std::make_shared<std::atomic<uint32_t>>(n);
            std::shared_ptr<PieceEvents> pe = q < sg.pieces.size() ? sg.pieces[q] : nullptr;
            // one task per `lanes` slices of the object (LeafLanes interleaves them)
            for (uint32_t i0 = 0; i0 < n; i0 += lanes)
                (pe ? streamed : tasks).push_back([=, j = job.get()] {
                    const uint32_t L = std::min(lanes, n - i0);
                    const uint8_t *src[hh::kMaxLanes];
                    uint8_t *dst[hh::kMaxLanes];
                    for (uint32_t l = 0; l < L; l++) {
                        src[l] = slices + (uint64_t)(i0 + l) * slen;
                        dst[l] = leaf + (uint64_t)(i0 + l) * TE_HASH_SIZE;
                    }
                    int rc = TE_OK;
                    hh::LeafLanes h((int)L);
                    if (!pe) {
                        h.update(src, slen);
                    } else {
                        (void)hipSetDevice(pe->device);
                        const uint8_t *at[hh::kMaxLanes];
                        for (size_t p = 0; p < pe->ev.size() && !rc; p++) {
                            rc = hip_status(event_wait_poll(pe->ev[p]));
                            for (uint32_t l = 0; l < L; l++) at[l] = src[l] + pe->beg[p];
                            if (!rc) h.update(at, pe->beg[p + 1] - pe->beg[p]);
                        }
                    }
                    h.final(dst);
                    if (left->fetch_sub(L) == L && !rc) rc = host_tree(leaf, n, height, root, proof);
                    j->done(rc);
                });
        }
    }
    job->add((int64_t)(tasks.size() + streamed.size()));
    G.segs.clear();
    if (!streamed.empty()) hh::Pool::get().submit_after(nullptr, device, std::move(streamed));
    if (tasks.empty()) {
        (void)hipEventDestroy(landed);
        return TE_OK;
    }
    hh::Pool::get().submit_after(landed, device, std::move(tasks));
    return TE_OK;
}

static int group_close(CommitPipe &P, OpenGroup &G, uint32_t n, uint32_t height, uint64_t leaf_b, uint64_t proof_b) {
    constexpr int S = CommitPipe::S;
    if (!G.open) return TE_OK;
    G.open = false;
    for (int k = 0; k < S; k++)
        if (G.slots_used[k]) TE_HIP(hipStreamWaitEvent(P.hs, P.ev_enc[k], 0));
    uint8_t *gout = P.gout[G.r]->as<uint8_t>(), *dc = P.gcom[G.r]->as<uint8_t>();
    const uint64_t root_at = G.rows_cap * leaf_b, proof_at = root_at + G.rows_cap * TE_HASH_SIZE;
    // flatten the rows: (slice length, out bytes, slice offset) in group order
    struct Row { uint64_t slen, obytes, off; };
    std::vector<Row> rows;
    rows.reserve(G.rows);
    for (const GroupSeg &sg : G.segs) {
        uint64_t off = sg.gout_off;
        for (size_t q = 0; q < sg.cnt; q++) {
            rows.push_back({sg.slice_len[q], sg.out_bytes[q], off});
            off += sg.out_bytes[q];
        }
    }
    for (size_t o = 0; o < rows.size();) {
        size_t e = o + 1;
        while (e < rows.size() && rows[e].slen == rows[o].slen) e++;
        CommitArgs ca{};
        ca.slices = gout + rows[o].off;
        ca.obj_stride = rows[o].obytes;
        ca.slice_len = rows[o].slen;
        ca.n = n;
        ca.nobj = (uint32_t)(e - o);
        ca.height = height;
        ca.leaf = dc + o * leaf_b;
        ca.root = dc + root_at + o * TE_HASH_SIZE;
        ca.proof = proof_b ? dc + proof_at + o * proof_b : nullptr;
        TE_HIP(launch_commit(ca, P.hs));
        o = e;
    }
    for (const GroupSeg &sg : G.segs) {
        const struct { uint8_t *h; uint64_t d, len; } back[3] = {
            {sg.co.leaf + sg.obj0 * leaf_b, sg.row0 * leaf_b, sg.cnt * leaf_b},
            {sg.co.root + sg.obj0 * TE_HASH_SIZE, root_at + sg.row0 * TE_HASH_SIZE, sg.cnt * TE_HASH_SIZE},
            {sg.co.proof ? sg.co.proof + sg.obj0 * proof_b : nullptr, proof_at + sg.row0 * proof_b, sg.cnt * proof_b}};
        for (const auto &bk : back)
            if (bk.h && bk.len) TE_HIP(hipMemcpyAsync(bk.h, dc + bk.d, bk.len, hipMemcpyDeviceToHost, P.hs));
    }
    for (int k = 0; k < S; k++)
        if (G.slots_used[k]) TE_HIP(hipStreamWaitEvent(P.hs, P.ev_slot[k], 0));
    TE_HIP(hipEventRecord(P.ev_hashed[G.r], P.hs));
    P.hashed_pending[G.r] = true;
    P.groups++;
    G.segs.clear();
    return TE_OK;
}

// Who hashes a group (te_set_commit_hashing / te_stream_writer_set_hashing, TE_HASH_*).  A leaf
// launch hashes one slice per lane at ~24 MB/s per lane (715,048 B in ~29.5 ms)
// whatever the number of slices up to ~64k of them; the host pool hashes at its measured
// per-thread rate (SHA extensions: 1-2 GB/s) times its threads.
// The device wins for very many short slices (tens of thousands of small objects' slices per
// group); with the contended device rate (below) the host pool takes the 4 MiB objects' groups too
// (r05: host 12.4-12.9 GiB/s against device 7.5-12.2 for 1024 x 4 MiB, every group size and
// window size measured) and the SDK's 64 MiB chunks (~9.7 MB slices: ~0.4 s per leaf launch).
std::atomic<int> g_commit_hashing{TE_HASH_AUTO};
bool host_hash_wins(int mode, uint64_t streams, uint64_t max_slice, uint64_t slice_bytes) {
    if (mode == TE_HASH_HOST) return true;
    if (mode == TE_HASH_DEVICE) return false;
    // a leaf lane hashes its slice at ~24 MB/s alone, but a group's hashing runs beside the next
    // groups' encodes and copies, which cut that to ~8 MB/s (r05 group traces: 90-128 ms per
    // 715 KB-slice group against 29 ms alone; with 24 MB/s here the 4 GiB groups went to the device
    // and the one-shot call ran 7.5 GiB/s against 12.4 host-hashed)
    const double dev_s = (double)max_slice / 8e6 * std::max(1.0, (double)streams / 65536.0);
    const hh::Pool &pool = hh::Pool::get();
    const double host_s = (double)slice_bytes / (pool.thread_rate() * pool.threads());
    return host_s < dev_s;
}

// The bytes a group of plan L needs in a group buffer, and its commitment rows.
static void group_need(const CommitBatch &B, const CommitPlan &L, size_t x, uint64_t &out, uint64_t &rows) {
    out = 0;
    for (size_t o = L.gcut[x]; o < L.gcut[x + 1]; o++) out += B.out_bytes[o];
    rows = L.gcut[x + 1] - L.gcut[x];
}

// The streams of the encode + commit pipeline (handle locked, its device current): two slot
// streams and the hashing stream -- the handle's pipe streams and its own stream.
// Measurement option (TEC_DEBUG_KNOBS=1 TEC_COMMIT_HASH_CUS=n): hash on n CUs of their own and
// copy / encode on the rest (hipExtStreamCreateWithCUMask), so no leaf wave shares a SIMD with an
// encode wave.  Not the default: it measured within the run-to-run spread (scripts/sw_probe.py,
// DESIGN §4.4), and CU-masked streams are blocking streams (they synchronise with the null stream).
static int commit_streams(te_clay *c, hipStream_t ss[2], hipStream_t &hs) {
    int hash_cus = 0;
    if (const char *e = tec_knob("TEC_COMMIT_HASH_CUS")) hash_cus = atoi(e);
    if (hash_cus > 0 && !c->cm_tried) {
        c->cm_tried = true;
        hipDeviceProp_t prop{};
        int ncu = 0;
        if (hipGetDeviceProperties(&prop, c->device) == hipSuccess) ncu = prop.multiProcessorCount;
        if (ncu > 2 * hash_cus) {
            const uint32_t words = (uint32_t)(ncu + 31) / 32;
            std::vector<uint32_t> hm(words, 0), sm(words, 0);
            for (int i = 0; i < ncu; i++) (i < hash_cus ? hm : sm)[i / 32] |= 1u << (i % 32);
            bool ok = hipExtStreamCreateWithCUMask(&c->cm_hs, words, hm.data()) == hipSuccess;
            for (int k = 0; k < 2 && ok; k++) ok = hipExtStreamCreateWithCUMask(&c->cm_ss[k], words, sm.data()) == hipSuccess;
            if (!ok)
                for (hipStream_t *ps : {&c->cm_ss[0], &c->cm_ss[1], &c->cm_hs}) {
                    if (*ps) (void)hipStreamDestroy(*ps);
                    *ps = nullptr;
                }
            (void)hipGetLastError();
        }
    }
    if (hash_cus > 0 && c->cm_hs) {
        ss[0] = c->cm_ss[0];
        ss[1] = c->cm_ss[1];
        hs = c->cm_hs;
        return TE_OK;
    }
    for (int k = 0; k < 2; k++)
        if (!c->pipe[k].s) TE_HIP(hipStreamCreateWithFlags(&c->pipe[k].s, hipStreamNonBlocking));
    if (!c->stream) TE_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    ss[0] = c->pipe[0].s;
    ss[1] = c->pipe[1].s;
    hs = c->stream;
    return TE_OK;
}

static int encode_commit_host_impl(te_clay *c, const te_slicer_cfg *cfg, const uint8_t *h_data,
                                   const te_object *objs, size_t nobj, uint8_t *h_out, size_t group_bytes,
                                   const CommitOut &co) {
    if (!c || !cfg || (!objs && nobj) || (nobj && (!h_data || !h_out))) return TE_ERR_INVALID_ARG;
    if (device_count() <= 0) return TE_ERR_NO_DEVICE;
    if (group_bytes == 0) group_bytes = (size_t)4 << 30;
    const uint64_t copy_bytes = std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)128 << 20, group_bytes / 8));
    CommitBatch B;
    B.h_data = h_data;
    B.objs = objs;
    B.nobj = nobj;
    B.h_out = h_out;
    B.co = co;
    int rc = commit_prepare(c, B);
    if (rc) return rc;
    CommitPlan L;
    commit_plan(B, group_bytes, copy_bytes, L);
    const uint64_t commit_cap = L.max_group_obj * (B.leaf_b + TE_HASH_SIZE + B.proof_b);

    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard dg(c->device);
    TE_HIP(dg.err);
    // three streams: two slot streams and the hashing stream (a fifth stream beside the caller's
    // shared a hardware queue with a slot stream in bench.py: 9.5 against 12.1 GiB/s)
    CommitPipe P;
    static_assert(CommitPipe::S == 2, "commit_streams makes two slot streams");
    if ((rc = commit_streams(c, P.ss, P.hs))) return rc;
    for (int k = 0; k < CommitPipe::S; k++) {
        P.in[k] = &c->pipe[k].in;
        P.arena[k] = &c->pipe[k].arena;
    }
    for (int r = 0; r < CommitPipe::R; r++) {
        P.gout[r] = &c->pipe[r].out;
        P.gcom[r] = &c->pipe[r].commit;
    }
    // every buffer sized up front (the pipeline never reallocates under queued work)
    const size_t ngroups = L.gcut.size() - 1, nring = std::min<size_t>(CommitPipe::R, ngroups);
    for (int k = 0; k < CommitPipe::S && nobj; k++) TE_HIP(P.in[k]->ensure(L.max_win_in));
    for (size_t r = 0; r < nring; r++) {
        TE_HIP(P.gout[r]->ensure(L.max_group_out));
        TE_HIP(P.gcom[r]->ensure(commit_cap));
    }
    rc = P.make_events();
    const uint64_t row_b = B.leaf_b + TE_HASH_SIZE + B.proof_b;
    const bool pinned_out = host_pinned(h_out);
    OpenGroup G;
    std::vector<std::shared_ptr<hh::Job>> jobs;
    for (size_t x = 0; x < ngroups && rc == TE_OK; x++) {
        uint64_t need_out, need_rows;
        group_need(B, L, x, need_out, need_rows);
        uint64_t max_slice = 0;
        for (size_t o = L.gcut[x]; o < L.gcut[x + 1]; o++) max_slice = std::max<uint64_t>(max_slice, B.slice_len[o]);
        const bool host = host_hash_wins(g_commit_hashing.load(), need_rows * B.n, max_slice, need_out);
        static const bool trace = tec_knob("TEC_COMMIT_TRACE") != nullptr;  // measurement: the choice per group
        if (trace)
            fprintf(stderr, "[tapeec] commit group %zu/%zu: %llu objects, %llu slice bytes, %s hashing (pool %.2f GB/s x %d)\n",
                    x + 1, ngroups, (unsigned long long)need_rows, (unsigned long long)need_out, host ? "host" : "device",
                    hh::Pool::get().thread_rate() / 1e9, hh::Pool::get().threads());
        const auto t0 = std::chrono::steady_clock::now();
        rc = group_open(P, G, need_out, need_rows, row_b);
        const auto t1 = std::chrono::steady_clock::now();
        if (!rc) rc = group_add(c, cfg, P, G, B, L, x, x + 1 == ngroups && !host, host && pinned_out);
        const auto t2 = std::chrono::steady_clock::now();
        if (!rc && host) {
            jobs.emplace_back();
            rc = group_close_host(P, G, B.n, B.co.height, c->device, jobs.back());
        } else if (!rc) {
            rc = group_close(P, G, B.n, B.co.height, B.leaf_b, B.proof_b);
        }
        if (trace) {  // host time enqueueing the group (a long one is a host wait inside)
            const auto t3 = std::chrono::steady_clock::now();
            auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
            fprintf(stderr, "[tapeec]   host ms: open %.2f add %.2f close %.2f\n", ms(t0, t1), ms(t1, t2), ms(t2, t3));
        }
    }
    for (int k = 0; k < CommitPipe::S; k++) {
        const int r2 = sync_sleep(P.ss[k]);
        if (rc == TE_OK) rc = r2;
    }
    const int r2 = sync_sleep(P.hs);
    if (rc == TE_OK) rc = r2;
    for (auto &j : jobs) {  // host-hashed groups: their tasks read the output buffers
        const int r3 = j ? j->wait() : TE_OK;
        if (rc == TE_OK) rc = r3;
    }
    P.destroy_events();
    return rc;
}

// ------------------------------------------------------------------------------------------
// te_stream_writer: the ordered, asynchronous window submission of the SDK's stream writer
// (sdk/src/stream/write.rs:332-362: up to min(cores, 4) chunk encodes in flight, handed on in
// order through FuturesOrdered), over one or more device-bound handles.  Window t goes to handle
// (t - 1) mod ncoders and is enqueued there without blocking; each handle's CommitPipe persists
// across windows, so window t+1's encode overlaps window t's hashing and copies.  te_stream_wait
// completes windows in submission order.
// ------------------------------------------------------------------------------------------
struct te_stream_writer {
    struct Dev {
        te_clay *c = nullptr;
        int device = 0;
        CommitPipe P;
        hipStream_t ss[CommitPipe::S] = {}, hs = nullptr;
        DevBuf in[CommitPipe::S], gout[CommitPipe::R], gcom[CommitPipe::R];
        Arena arena[CommitPipe::S];
        // windows share a hashing group until it holds group_bytes / 2 (a leaf launch costs one
        // slice's SHA-256 whatever its size: one launch per window capped small windows at
        // 7.3-7.5 GiB/s); tickets whose last group is still open complete when it closes
        OpenGroup G;
        bool G_host = false;        // the open group is hashed on the host (host_hash.hpp)
        std::vector<uint64_t> pend;
    };
    struct Ticket {
        int dev = -1;
        hipEvent_t done = nullptr;  // its groups' device work (hashing or the copies host hashing reads)
        std::vector<std::shared_ptr<hh::Job>> jobs;  // host-hashed groups holding its objects
        int rc = TE_OK;
        bool pending = false;  // its last group is the device's open group
    };
    std::vector<std::unique_ptr<Dev>> devs;
    te_slicer_cfg cfg{};
    uint32_t height = 0;
    bool proofs = true;
    uint64_t group_bytes = 0;
    int hashing = TE_HASH_AUTO;
    std::mutex mu;
    std::mutex wait_mu;  // te_stream_wait calls complete tickets one caller at a time
    uint64_t next = 1;                   // next ticket
    std::map<uint64_t, Ticket> tickets;  // submitted, not yet waited
};

namespace {
uint64_t writer_row_bytes(const te_stream_writer &w, const te_stream_writer::Dev &d, uint64_t &leaf_b, uint64_t &proof_b) {
    leaf_b = (uint64_t)d.c->h.n * TE_HASH_SIZE;
    proof_b = leaf_b * w.height;  // proofs always computed (a window may ask for them)
    return leaf_b + TE_HASH_SIZE + proof_b;
}
// Hash the device's open group and complete the tickets waiting on it.  Called with w.mu held.
int writer_close(te_stream_writer &w, te_stream_writer::Dev &d) {
    int rc = TE_OK;
    std::shared_ptr<hh::Job> job;
    if (d.G.open) {
        uint64_t leaf_b, proof_b;
        (void)writer_row_bytes(w, d, leaf_b, proof_b);
        std::lock_guard<std::mutex> lk(d.c->mu);
        DeviceGuard dg(d.device);
        rc = hip_status(dg.err);
        if (!rc && d.G_host)
            rc = group_close_host(d.P, d.G, (uint32_t)d.c->h.n, w.height, d.device, job);
        else if (!rc)
            rc = group_close(d.P, d.G, (uint32_t)d.c->h.n, w.height, leaf_b, proof_b);
        d.G.open = false;
    }
    for (uint64_t t : d.pend) {
        auto it = w.tickets.find(t);
        if (it == w.tickets.end()) continue;
        te_stream_writer::Ticket &T = it->second;
        T.pending = false;
        if (!rc) {
            // after the group's hashing and copies (a ticket spanning several groups re-records)
            DeviceGuard dg(d.device);
            // blocking: te_stream_wait sleeps in hipEventSynchronize instead of spinning a core the
            // host hashing pool could use (the GPU's host share is 16 CPUs of time on the pool)
            if (!T.done) rc = hip_status(hipEventCreateWithFlags(&T.done, hipEventDisableTiming | hipEventBlockingSync));
            if (!rc) rc = hip_status(hipEventRecord(T.done, d.hs));
        }
        if (job) T.jobs.push_back(job);
        if (rc && !T.rc) T.rc = rc;
    }
    d.pend.clear();
    return rc;
}
int writer_drain(te_stream_writer::Dev &d) {
    DeviceGuard dg(d.device);
    TE_HIP(dg.err);
    int rc = TE_OK;
    for (int k = 0; k < CommitPipe::S; k++)
        if (d.ss[k]) {
            const int r = sync_sleep(d.ss[k]);
            if (!rc) rc = r;
        }
    if (d.hs) {
        const int r = sync_sleep(d.hs);
        if (!rc) rc = r;
    }
    return rc;
}
void writer_release(te_stream_writer::Dev &d) {
    DeviceGuard dg(d.device);
    (void)writer_drain(d);
    for (auto &b : d.in) b.release();
    for (auto &b : d.gout) b.release();
    for (auto &b : d.gcom) b.release();
    for (auto &a : d.arena) a.release();
    d.P.destroy_events();  // the streams are the handle's (released with it)
}
}  // namespace

// ------------------------------------------------------------------------------------------
// C ABI: compute entry points
// ------------------------------------------------------------------------------------------
extern "C" {

int te_encode_batch_device(te_clay *c, const te_slicer_cfg *cfg, const uint8_t *d_data, const te_object *objs,
                           size_t nobj, uint8_t *d_out, void *stream) {
    if (!c || !cfg || (!objs && nobj)) return TE_ERR_INVALID_ARG;
    if (device_count() <= 0) return TE_ERR_NO_DEVICE;
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard dg(c->device);
    TE_HIP(dg.err);
    return encode_enqueue(c, cfg, d_data, objs, nobj, d_out, (hipStream_t)stream, false);
}

int te_encode_batch_host(te_clay *c, const te_slicer_cfg *cfg, const uint8_t *h_data, const te_object *objs,
                         size_t nobj, uint8_t *h_out, size_t window_bytes) {
    return encode_host_impl(c, cfg, h_data, objs, nobj, h_out, window_bytes);
}

int te_encode_commit_batch_host(te_clay *c, const te_slicer_cfg *cfg, const uint8_t *h_data, const te_object *objs,
                                size_t nobj, uint8_t *h_out, uint32_t height, uint8_t *h_leaf_hashes,
                                uint8_t *h_roots, uint8_t *h_proofs, size_t window_bytes) {
    if (!c || !h_leaf_hashes || !h_roots || height == 0 || height > TE_MAX_MERKLE_TREE_HEIGHT)
        return TE_ERR_INVALID_ARG;
    const uint32_t n = (uint32_t)c->h.n;
    if (n > TE_COMMIT_MAX_LEAVES) return TE_ERR_INVALID_ARG;
    if (height < 64 && (uint64_t)n > (1ull << height)) return TE_ERR_MERKLE_TREE_FULL;
    const CommitOut co{h_leaf_hashes, h_roots, h_proofs, height};
    return encode_commit_host_impl(c, cfg, h_data, objs, nobj, h_out, window_bytes, co);
}
int te_stream_writer_new(te_clay *const *coders, size_t ncoders, const te_slicer_cfg *cfg, uint32_t height,
                         size_t group_bytes, te_stream_writer **out) {
    if (!out) return TE_ERR_INVALID_ARG;
    *out = nullptr;
    if (!coders || ncoders == 0 || !cfg || height == 0 || height > TE_MAX_MERKLE_TREE_HEIGHT) return TE_ERR_INVALID_ARG;
    if (device_count() <= 0) return TE_ERR_NO_DEVICE;
    for (size_t i = 0; i < ncoders; i++) {
        if (!coders[i]) return TE_ERR_INVALID_ARG;
        const uint32_t n = (uint32_t)coders[i]->h.n;
        if (n > TE_COMMIT_MAX_LEAVES) return TE_ERR_INVALID_ARG;
        if (height < 64 && (uint64_t)n > (1ull << height)) return TE_ERR_MERKLE_TREE_FULL;
    }
    auto *w = new (std::nothrow) te_stream_writer();
    if (!w) return TE_ERR_OUT_OF_MEMORY;
    w->cfg = *cfg;
    w->height = height;
    w->group_bytes = group_bytes ? group_bytes : ((size_t)8 << 30);  // see te_stream_writer_new's header note
    w->hashing = g_commit_hashing.load();
    int rc = TE_OK;
    for (size_t i = 0; i < ncoders && !rc; i++) {
        auto d = std::make_unique<te_stream_writer::Dev>();
        d->c = coders[i];
        d->device = coders[i]->device;
        DeviceGuard dg(d->device);
        if ((rc = hip_status(dg.err))) break;
        {
            // the handle's own slot and hashing streams (created if missing): the process has four
            // hardware queues, and streams of their own would put the writer's slot and hashing
            // streams on shared queues behind other streams' work (te_encode_commit_batch_host's
            // note); calls on the handle serialise with the writer's windows on them
            te_clay *c = coders[i];
            std::lock_guard<std::mutex> lk(c->mu);
            rc = commit_streams(c, d->ss, d->hs);
        }
        CommitPipe &P = d->P;
        P.hs = d->hs;
        for (int k = 0; k < CommitPipe::S; k++) {
            P.ss[k] = d->ss[k];
            P.in[k] = &d->in[k];
            P.arena[k] = &d->arena[k];
        }
        for (int r = 0; r < CommitPipe::R; r++) {
            P.gout[r] = &d->gout[r];
            P.gcom[r] = &d->gcom[r];
        }
        P.grow_ok = true;  // buffers grow on demand, after the work queued on them has drained
        if (!rc) rc = P.make_events();
        w->devs.push_back(std::move(d));
    }
    if (rc) {
        te_stream_writer_free(w);
        return rc;
    }
    *out = w;
    return TE_OK;
}

int te_stream_submit(te_stream_writer *w, const uint8_t *h_data, const te_object *objs, size_t nobj, uint8_t *h_out,
                     uint8_t *h_leaf_hashes, uint8_t *h_roots, uint8_t *h_proofs, uint64_t *ticket) {
    if (!w || !ticket || (!objs && nobj) || (nobj && (!h_data || !h_out || !h_leaf_hashes || !h_roots)))
        return TE_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> g(w->mu);
    const uint64_t t = w->next++;
    *ticket = t;
    te_stream_writer::Ticket &T = w->tickets[t];
    T.dev = (int)((t - 1) % w->devs.size());
    te_stream_writer::Dev &d = *w->devs[(size_t)T.dev];
    te_clay *c = d.c;
    CommitBatch B;
    B.h_data = h_data;
    B.objs = objs;
    B.nobj = nobj;
    B.h_out = h_out;
    B.co = CommitOut{h_leaf_hashes, h_roots, h_proofs, w->height};
    // every per-object check happens here, before the window touches the device's open group
    int rc = commit_prepare(c, B);
    auto pend_t = [&] {
        if (d.pend.empty() || d.pend.back() != t) d.pend.push_back(t);
        T.pending = true;
    };
    if (!rc && nobj == 0) {  // completes after everything queued before it
        pend_t();
        rc = writer_close(*w, d);
    } else if (!rc) {
        CommitPlan L;
        const uint64_t copy_bytes = std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)128 << 20, w->group_bytes / 8));
        commit_plan(B, w->group_bytes, copy_bytes, L);
        uint64_t leaf_b, proof_b;
        const uint64_t row_b = writer_row_bytes(*w, d, leaf_b, proof_b);
        B.leaf_b = leaf_b;
        B.proof_b = proof_b;
        // host or device hashing, per window (host_hash_wins): the SDK's 64 MiB chunks hash on the
        // host, each window a group of its own closed at once; batches of small objects share
        // device groups
        uint64_t max_slice = 0, slice_bytes = 0;
        for (size_t o = 0; o < nobj; o++) {
            max_slice = std::max<uint64_t>(max_slice, B.slice_len[o]);
            slice_bytes += B.out_bytes[o];
        }
        const bool host = host_hash_wins(w->hashing, (uint64_t)nobj * B.n, max_slice, slice_bytes);
        const bool pinned_out = host && host_pinned(h_out);
        if (d.G.open && d.G_host != host) rc = writer_close(*w, d);
        const uint64_t close_at = std::max<uint64_t>(1, w->group_bytes / 2);
        for (size_t x = 0; x + 1 < L.gcut.size() && !rc; x++) {
            uint64_t need_out, need_rows, gbytes = 0;
            group_need(B, L, x, need_out, need_rows);
            for (size_t o = L.gcut[x]; o < L.gcut[x + 1]; o++) gbytes += B.objs[o].blob_len + B.out_bytes[o];
            OpenGroup &G = d.G;
            if (G.open && (G.out_off + need_out > d.P.gout[G.r]->cap || G.rows + need_rows > G.rows_cap ||
                           G.bytes + gbytes > w->group_bytes))
                rc = writer_close(*w, d);  // earlier windows' tickets complete with it
            if (rc) break;
            pend_t();
            {
                std::lock_guard<std::mutex> lk(c->mu);
                DeviceGuard dg(d.device);
                rc = c->device != d.device ? TE_ERR_INVALID_ARG : hip_status(dg.err);  // handle re-bound under the writer
                if (!rc && !G.open) {
                    // a group buffer holds a full group's slices (group_bytes of objects + slices,
                    // ~3/4 of it slices for Clay(20, 7)) and its commitment rows; a host-hashed
                    // group holds one window
                    const uint64_t want_out = host ? need_out : std::max<uint64_t>(need_out, w->group_bytes - w->group_bytes / 4);
                    const uint64_t want_rows = host ? need_rows : std::max<uint64_t>(need_rows, 4096);
                    rc = group_open(d.P, G, want_out, want_rows, row_b);
                    d.G_host = host;
                }
                // on failure the group keeps its earlier segments (group_add adds one only on
                // success): the earlier windows still complete below
                if (!rc) rc = group_add(c, &w->cfg, d.P, G, B, L, x, false, host && pinned_out);
            }
            if (!rc && (host || G.bytes >= close_at)) rc = writer_close(*w, d);  // pending windows complete with it
        }
    }
    if (rc) {
        // only this window fails: the earlier windows of the open group are hashed and complete
        // normally; then the device is drained, since work already enqueued for this window may
        // still read or write its host buffers
        d.pend.erase(std::remove(d.pend.begin(), d.pend.end(), t), d.pend.end());
        T.pending = false;
        (void)writer_close(*w, d);
        (void)writer_drain(d);
        for (auto &j : T.jobs) (void)j->wait();
        T.jobs.clear();
        if (T.done) (void)hipEventDestroy(T.done);
        T.done = nullptr;
    }
    T.rc = rc;
    return rc;
}

int te_stream_wait(te_stream_writer *w, uint64_t ticket) {
    if (!w || ticket == 0) return TE_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> wg(w->wait_mu);
    int first = TE_OK;
    for (;;) {
        te_stream_writer::Ticket T;
        {
            std::lock_guard<std::mutex> g(w->mu);
            if (ticket >= w->next) return TE_ERR_INVALID_ARG;  // never submitted
            if (w->tickets.empty() || w->tickets.begin()->first > ticket) return first;
            if (w->tickets.begin()->second.pending) {  // its group is still open: hash it now
                te_stream_writer::Dev &d = *w->devs[(size_t)w->tickets.begin()->second.dev];
                const int r = writer_close(*w, d);
                if (r) (void)writer_drain(d);
            }
            // claimed: only this caller (wait_mu) completes it
            T = std::move(w->tickets.begin()->second);
            w->tickets.erase(w->tickets.begin());
        }
        int rc = T.rc;
        if (T.done) {
            DeviceGuard dg(w->devs[(size_t)T.dev]->device);
            const int r = hip_status(hipEventSynchronize(T.done));
            if (!rc) rc = r;
            (void)hipEventDestroy(T.done);
        }
        for (auto &j : T.jobs) {
            const int r = j->wait();
            if (!rc) rc = r;
        }
        if (!first) first = rc;
    }
}

int te_stream_writer_set_hashing(te_stream_writer *w, int mode) {
    if (!w || mode < TE_HASH_AUTO || mode > TE_HASH_HOST) return TE_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> g(w->mu);
    w->hashing = mode;
    return TE_OK;
}

int te_set_commit_hashing(int mode) {
    if (mode < TE_HASH_AUTO || mode > TE_HASH_HOST) return TE_ERR_INVALID_ARG;
    g_commit_hashing.store(mode);
    return TE_OK;
}

int te_set_host_hash_threads(int threads) {
    if (threads < 0) return TE_ERR_INVALID_ARG;
    return hh::Pool::get().set_threads(threads);
}

int te_host_hash_threads(void) { return hh::Pool::get().threads(); }

int te_host_sha_extensions(void) { return hh::have_sha_ext() ? 1 : 0; }

double te_host_hash_rate(void) { return hh::Pool::get().thread_rate(); }

int te_host_hash_lanes(void) { return hh::Pool::get().lanes(); }

int te_host_alloc(size_t bytes, void **out) {
    if (!out) return TE_ERR_INVALID_ARG;
    *out = nullptr;
    if (device_count() <= 0) return TE_ERR_NO_DEVICE;
    if (bytes == 0) bytes = 1;
    void *p = nullptr;
    const hipError_t e = hipHostMalloc(&p, bytes, hipHostMallocPortable);
    if (e != hipSuccess) return e == hipErrorOutOfMemory ? TE_ERR_OUT_OF_MEMORY : hip_status(e);
    *out = p;
    return TE_OK;
}

void te_host_free(void *p) {
    if (p) (void)hipHostFree(p);
}

int te_host_register(void *p, size_t bytes) {
    if (!p || bytes == 0) return TE_ERR_INVALID_ARG;
    if (device_count() <= 0) return TE_ERR_NO_DEVICE;
    TE_HIP(hipHostRegister(p, bytes, hipHostRegisterPortable));
    return TE_OK;
}

int te_host_unregister(void *p) {
    if (!p) return TE_ERR_INVALID_ARG;
    if (device_count() <= 0) return TE_ERR_NO_DEVICE;
    TE_HIP(hipHostUnregister(p));
    return TE_OK;
}

void te_stream_writer_free(te_stream_writer *w) {
    if (!w) return;
    if (w->next > 1) (void)te_stream_wait(w, w->next - 1);
    for (auto &d : w->devs) writer_release(*d);
    delete w;
}

int te_balance_object_ranges(const te_object *objs, size_t nobj, size_t nparts, size_t *cuts) {
    if (!cuts || nparts == 0 || (!objs && nobj)) return TE_ERR_INVALID_ARG;
    // contiguous ranges of about equal input bytes (+1 per object, so empty blobs count too):
    // cut p is the first object index after which the running byte count reaches p/nparts of the total
    uint64_t total = 0;
    for (size_t i = 0; i < nobj; i++) total += objs[i].blob_len + 1;
    for (size_t p = 0; p <= nparts; p++) cuts[p] = nobj;
    cuts[0] = 0;
    unsigned __int128 acc = 0;
    size_t part = 1;
    for (size_t i = 0; i < nobj && part < nparts; i++) {
        acc += objs[i].blob_len + 1;
        while (part < nparts && acc * nparts >= (unsigned __int128)total * part) cuts[part++] = i + 1;
    }
    return TE_OK;
}

int te_encode_batch_host_multi(te_clay *const *coders, size_t ncoders, const te_slicer_cfg *cfg, const uint8_t *h_data,
                               const te_object *objs, size_t nobj, uint8_t *h_out, size_t window_bytes) {
    if (!coders || ncoders == 0 || !cfg || (!objs && nobj)) return TE_ERR_INVALID_ARG;
    for (size_t i = 0; i < ncoders; i++)
        if (!coders[i]) return TE_ERR_INVALID_ARG;
    if (ncoders == 1 || nobj <= 1) return te_encode_batch_host(coders[0], cfg, h_data, objs, nobj, h_out, window_bytes);
    std::vector<size_t> cut(ncoders + 1);
    (void)te_balance_object_ranges(objs, nobj, ncoders, cut.data());
    std::vector<int> rc(ncoders, TE_OK);
    std::vector<std::string> why(ncoders);  // each worker's te_last_error_detail (thread-local)
    std::vector<std::thread> th;
    for (size_t p = 0; p < ncoders; p++) {
        if (cut[p + 1] <= cut[p]) continue;
        th.emplace_back([&, p] {
            rc[p] = te_encode_batch_host(coders[p], cfg, h_data, objs + cut[p], cut[p + 1] - cut[p], h_out, window_bytes);
            if (rc[p]) why[p] = g_last_error;
        });
    }
    for (auto &t : th) t.join();
    for (size_t p = 0; p < ncoders; p++)
        if (rc[p]) {  // the first failing handle's status and detail, on the calling thread
            snprintf(g_last_error, sizeof(g_last_error), "%s", why[p].c_str());
            return rc[p];
        }
    return TE_OK;
}

int te_decode_batch_device(te_clay *c, const te_slicer_cfg *cfg, const uint8_t *d_slices, const te_decode_object *objs,
                           const uint8_t *h_meta, size_t nobj, uint8_t *d_out, void *stream) {
    if (!c || !cfg || (!objs && nobj) || (!h_meta && nobj)) return TE_ERR_INVALID_ARG;
    if (device_count() <= 0) return TE_ERR_NO_DEVICE;
    std::vector<DecItem> items(nobj);
    for (size_t i = 0; i < nobj; i++) {
        int r = decode_validate(c, h_meta + i * TE_META_SIZE, objs[i].slice_len, objs[i].avail_mask, items[i]);
        if (r) return r;
        items[i].in_base = objs[i].slices_off;
        items[i].out_off = objs[i].out_off;
    }
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard dg(c->device);
    TE_HIP(dg.err);
    return decode_enqueue(c, cfg, d_slices, items.data(), items.size(), d_out, (hipStream_t)stream, false);
}

int te_repair_batch_device(te_clay *c, const uint8_t *d_helpers, const te_repair_object *objs, size_t nobj,
                           uint8_t *d_out, void *stream) {
    if (!c || (!objs && nobj)) return TE_ERR_INVALID_ARG;
    if (device_count() <= 0) return TE_ERR_NO_DEVICE;
    std::vector<RepItem> items(nobj);
    for (size_t i = 0; i < nobj; i++) {
        if (!objs[i].plan) return TE_ERR_INVALID_ARG;
        if (objs[i].plan->n != (uint32_t)c->h.n || objs[i].plan->d != (uint32_t)c->h.d) return TE_ERR_INVALID_ARG;
        items[i] = RepItem{objs[i].plan, objs[i].helper_off, objs[i].out_off, objs[i].metadata};
    }
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard dg(c->device);
    TE_HIP(dg.err);
    return repair_enqueue(c, d_helpers, items.data(), items.size(), d_out, (hipStream_t)stream);
}

// Node recover (network/node/src/features/spool/recover.rs:411-442 `reconstruct`): decode the
// object from >= k peer slices, re-encode it, keep the lost slice.  Per stripe the lost slice
// holds one shard (rotation): a data shard is a piece of the decoded object (zero-padded like
// Slicer::encode's stripe, slicer.rs:276-283), so only stripes whose lost shard is a parity
// shard are re-encoded.  Objects go through the device workspaces in windows (bounded memory);
// the workspaces are ordered against a previous call on another stream by `rec_done`.
int te_recover_batch_device(te_clay *c, const te_slicer_cfg *cfg, const uint8_t *d_slices,
                            const te_recover_object *objs, const uint8_t *h_meta, size_t nobj, uint8_t *d_out,
                            void *stream) {
    if (!c || !cfg || (!objs && nobj) || (!h_meta && nobj)) return TE_ERR_INVALID_ARG;
    if (nobj == 0) return TE_OK;
    if (device_count() <= 0) return TE_ERR_NO_DEVICE;
    const ClayHost &h = c->h;
    const uint32_t n = (uint32_t)h.n;
    const int rotated = cfg->rotated;
    std::vector<DecItem> items(nobj);
    std::vector<te_object> enc(nobj);
    std::vector<uint64_t> stripe(nobj), nstripes(nobj), chunk(nobj), meta_w(nobj * 6);
    for (size_t i = 0; i < nobj; i++) {
        if (objs[i].lost >= n) return TE_ERR_INVALID_SLICE;
        int r = decode_validate(c, h_meta + i * TE_META_SIZE, objs[i].slice_len, objs[i].avail_mask, items[i]);
        if (r) return r;
        te_slice_metadata m;
        te_slice_metadata_from_slice(h_meta + i * TE_META_SIZE, TE_META_SIZE, &m);
        te_geometry g;
        te_slicer_geometry(c, items[i].blob_len, &g);
        if (g.slice_len != objs[i].slice_len) return TE_ERR_INVALID_LAYOUT;
        items[i].in_base = objs[i].slices_off;
        enc[i] = te_object{0, items[i].blob_len, 0, m.chunk_index};
        stripe[i] = g.stripe_size;
        nstripes[i] = g.num_stripes;  // an empty blob still has one (all-zero) stripe
        chunk[i] = g.chunk_size;
        for (int w = 0; w < 6; w++) meta_w[i * 6 + w] = get_u64(h_meta + i * TE_META_SIZE + 8 * w);
    }
    // A mixed batch goes in two parts: the objects the fused path takes (a plane-program profile,
    // sub-chunks of >= 8 bytes, 31-bit slice offsets: decode_enqueue's staged_group) and the rest,
    // so one small object does not send the whole batch to the windowed decode + re-encode
    // (ADVICE r03).  Offsets are absolute, so each part is the same call on a subset.
    {
        const bool planes = h.q == kRepQ && h.t == 2 && h.nu == 0;
        std::vector<size_t> part[2];
        for (size_t i = 0; i < nobj; i++) {
            const uint64_t sc = chunk[i] / (uint64_t)h.alpha;
            const bool fz = planes && (items[i].ns == 0 || sc >= 8) && (uint64_t)n * objs[i].slice_len < 0x7fffffffull &&
                            chunk[i] * (uint64_t)h.k < 0x7fffffffull;
            part[fz ? 0 : 1].push_back(i);
        }
        if (!part[0].empty() && !part[1].empty()) {
            for (const auto &pv : part) {
                std::vector<te_recover_object> o;
                std::vector<uint8_t> m;
                for (size_t i : pv) {
                    o.push_back(objs[i]);
                    m.insert(m.end(), h_meta + i * TE_META_SIZE, h_meta + (i + 1) * TE_META_SIZE);
                }
                const int r = te_recover_batch_device(c, cfg, d_slices, o.data(), m.data(), o.size(), d_out, stream);
                if (r) return r;
            }
            return TE_OK;
        }
    }
    {
        // Fused: one staged decode whose program outputs only the lost node's chunk of every stripe,
        // straight into the lost slice -- 7 slices read, 1 written, no decoded object and no
        // re-encode (a lost parity node's C is produced by the same layered decode).  Empty blobs
        // have no stripe to decode: their one chunk is zeros.
        std::vector<DecItem> fi(items);
        std::vector<CopyJob> zeros;
        std::vector<MetaJob> metas;
        for (size_t i = 0; i < nobj; i++) {
            fi[i].lost = (int32_t)objs[i].lost;
            fi[i].out_off = objs[i].out_off;
            uint8_t *dst = d_out + objs[i].out_off;
            if (items[i].ns == 0) zeros.push_back(CopyJob{d_out, dst, chunk[i] * nstripes[i], 0});
            MetaJob m{};
            m.dst = dst + nstripes[i] * chunk[i];
            m.slice_len = 0;
            for (int k = 0; k < 6; k++) m.words[k] = meta_w[i * 6 + k];
            metas.push_back(m);
        }
        std::lock_guard<std::mutex> lk(c->mu);
        DeviceGuard dg(c->device);
        TE_HIP(dg.err);
        hipStream_t s = (hipStream_t)stream;
        const int rf = decode_enqueue(c, cfg, d_slices, fi.data(), nobj, d_out, s, false);
        if (rf != TE_ERR_UNSUPPORTED) {
            if (rf) return rf;
            Arena &A = c->rec;
            if (c->rec_pending && c->rec_stream != s) TE_HIP(hipStreamWaitEvent(s, c->rec_done, 0));
            A.img.clear();
            const size_t zoff = A.put(zeros.data(), zeros.size() * sizeof(CopyJob));
            const size_t moff = A.put(metas.data(), metas.size() * sizeof(MetaJob));
            int r = A.upload(s);
            if (r) return r;
            KTimer kt(s);
            if (!zeros.empty()) TE_HIP(launch_gather(A.at<CopyJob>(zoff), (uint32_t)zeros.size(), s));
            TE_HIP(launch_meta(A.at<MetaJob>(moff), (uint32_t)metas.size(), 1u, s));
            kt.stop();
            r = A.mark_done(s);
            if (!c->rec_done) TE_HIP(hipEventCreateWithFlags(&c->rec_done, hipEventDisableTiming));
            const int r2 = hip_status(hipEventRecord(c->rec_done, s));
            c->rec_pending = true;
            c->rec_stream = s;
            return r ? r : r2;
        }
    }
    // Otherwise (profiles without plane programs): windowed decode into the object, re-encode of
    // the parity-lost stripes, gather.
    auto is_parity = [&](size_t i, size_t st) {
        return te_slice_to_shard(rotated, n, (uint32_t)st, objs[i].lost) >= (uint32_t)h.k;
    };
    // windows: <= kWinBlob decoded bytes and <= kWinSlices re-encoded slice bytes
    uint64_t kWinBlob = 1ull << 30, kWinSlices = 3ull << 30;
    if (const char *e = tec_knob("TEC_RECOVER_WINDOW_BYTES")) {  // tests: force several windows
        const uint64_t v = strtoull(e, nullptr, 10);
        if (v) kWinBlob = kWinSlices = v;
    }
    struct Win { size_t b, e; uint64_t blob, slices; };
    std::vector<Win> wins;
    uint64_t max_blob = 16, max_slices = 16;
    for (size_t i = 0; i < nobj;) {
        Win w{i, i, 0, 0};
        while (w.e < nobj) {
            const uint64_t bb = (items[w.e].blob_len + 15) & ~15ull, sb = (uint64_t)n * objs[w.e].slice_len;
            if (w.e > w.b && (w.blob + bb > kWinBlob || w.slices + sb > kWinSlices)) break;
            w.blob += bb;
            w.slices += sb;
            w.e++;
        }
        max_blob = std::max(max_blob, w.blob + 16);
        max_slices = std::max(max_slices, w.slices + 16);
        wins.push_back(w);
        i = w.e;
    }
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard dg(c->device);
    TE_HIP(dg.err);
    hipStream_t s = (hipStream_t)stream;
    if (!c->rec_done) TE_HIP(hipEventCreateWithFlags(&c->rec_done, hipEventDisableTiming));
    if (max_blob > c->rec_blob.cap || max_slices > c->rec_slices.cap) {
        if (c->rec_pending) TE_HIP(hipEventSynchronize(c->rec_done));  // queued work may still use them
    } else if (c->rec_pending && c->rec_stream != s) {
        TE_HIP(hipStreamWaitEvent(s, c->rec_done, 0));
    }
    TE_HIP(c->rec_blob.ensure(max_blob));
    TE_HIP(c->rec_slices.ensure(max_slices));
    uint8_t *const blob = c->rec_blob.as<uint8_t>(), *const slices = c->rec_slices.as<uint8_t>();
    std::vector<CopyJob> jobs;
    std::vector<MetaJob> metas;
    std::vector<te_object> wenc;
    std::vector<uint64_t> blob_off;
    int r = TE_OK;
    for (const Win &w : wins) {
        blob_off.assign(w.e - w.b, 0);
        wenc.clear();
        uint64_t bo = 0, so = 0;
        for (size_t i = w.b; i < w.e; i++) {
            items[i].out_off = bo;
            blob_off[i - w.b] = bo;
            te_object e = enc[i];
            e.data_off = bo;
            e.out_off = so;
            wenc.push_back(e);
            bo += (items[i].blob_len + 15) & ~15ull;
            so += (uint64_t)n * objs[i].slice_len;
        }
        if ((r = decode_enqueue(c, cfg, d_slices, items.data() + w.b, w.e - w.b, blob, s, false))) break;
        bool any_parity = false;
        for (size_t i = w.b; i < w.e && !any_parity; i++)
            for (uint64_t st = 0; st < nstripes[i]; st++) any_parity = any_parity || is_parity(i, st);
        // parity-lost stripes are re-encoded writing only the lost shard's chunk (plus the
        // column-0 parity chunks the LDS-DMA kernel reads back internally)
        const uint32_t col0_parity = ((1u << h.q) - 1u) & ~((1u << h.k) - 1u);
        if (any_parity &&
            (r = encode_enqueue(c, cfg, blob, wenc.data(), wenc.size(), slices, s, false, nullptr,
                                [&](size_t o, size_t st) -> uint32_t {
                                    if (!is_parity(w.b + o, st)) return 0u;
                                    return col0_parity | (1u << te_slice_to_shard(rotated, n, (uint32_t)st,
                                                                                  objs[w.b + o].lost));
                                })))
            break;
        // assemble the lost slices: per stripe the lost shard's chunk, then the suffix
        jobs.clear();
        metas.clear();
        for (size_t i = w.b; i < w.e; i++) {
            const DecItem &it = items[i];
            const uint64_t cs = chunk[i], slen = objs[i].slice_len, ns = nstripes[i];
            uint8_t *dst = d_out + objs[i].out_off;
            for (uint64_t st = 0; st < ns; st++) {
                const uint32_t sh = te_slice_to_shard(rotated, n, (uint32_t)st, objs[i].lost);
                if (sh >= (uint32_t)h.k) {
                    jobs.push_back(CopyJob{slices + wenc[i - w.b].out_off + (uint64_t)objs[i].lost * slen + st * cs,
                                           dst + st * cs, cs, cs});
                } else {
                    // data shard sh of stripe st: object bytes [st*S + sh*cs, ...) clipped to the
                    // stripe and the object, zero beyond
                    const uint64_t start = st * stripe[i] + (uint64_t)sh * cs;
                    const uint64_t end = std::min<uint64_t>(it.blob_len, (st + 1) * stripe[i]);
                    const uint64_t valid = start < end ? std::min<uint64_t>(cs, end - start) : 0;
                    jobs.push_back(CopyJob{blob + blob_off[i - w.b] + std::min(start, it.blob_len), dst + st * cs, cs, valid});
                }
            }
            MetaJob m{};
            m.dst = dst + ns * cs;
            m.slice_len = 0;
            for (int k = 0; k < 6; k++) m.words[k] = meta_w[i * 6 + k];
            metas.push_back(m);
        }
        Arena &A = c->rec;
        A.img.clear();
        const size_t off = A.put(jobs.data(), jobs.size() * sizeof(CopyJob));
        const size_t moff = A.put(metas.data(), metas.size() * sizeof(MetaJob));
        if ((r = A.upload(s))) break;
        KTimer kt(s);
        if ((r = hip_status(launch_gather(A.at<CopyJob>(off), (uint32_t)jobs.size(), s)))) break;
        if ((r = hip_status(launch_meta(A.at<MetaJob>(moff), (uint32_t)metas.size(), 1u, s)))) break;
        kt.stop();
        if ((r = A.mark_done(s))) break;
    }
    // later calls (any stream) order against everything this one enqueued
    const int r2 = hip_status(hipEventRecord(c->rec_done, s));
    c->rec_pending = true;
    c->rec_stream = s;
    return r ? r : r2;
}

int te_slicer_encode(te_clay *c, const te_slicer_cfg *cfg, const uint8_t *data, size_t len, uint8_t *slices,
                     size_t cap) {
    if (!c || !cfg || (!data && len) || !slices) return TE_ERR_INVALID_ARG;
    te_geometry g;
    te_slicer_geometry(c, len, &g);
    const size_t total = (size_t)c->h.n * g.slice_len;
    if (cap < total) return TE_ERR_BUFFER_TOO_SMALL;
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard dg(c->device);
    TE_HIP(dg.err);
    int r = ensure_stream(c);
    if (r) return r;
    TE_HIP(c->io_in.ensure(len + 16));
    TE_HIP(c->io_out.ensure(total));
    if (len) TE_HIP(hipMemcpyAsync(c->io_in.p, data, len, hipMemcpyHostToDevice, c->stream));
    te_object o{0, len, 0, cfg->chunk_index};
    r = encode_enqueue(c, cfg, c->io_in.as<uint8_t>(), &o, 1, c->io_out.as<uint8_t>(), c->stream, false, nullptr,
                       StripeSel(), true);
    if (r) return r;
    // (copying the level-1 rows out while level 2 runs, as 2-D copies on a second stream, measured
    // slower: 0.62 against 0.50 ms pageable, 0.505 against 0.485 pinned, r05)
    TE_HIP(hipMemcpyAsync(slices, c->io_out.p, total, hipMemcpyDeviceToHost, c->stream));
    TE_HIP(hipStreamSynchronize(c->stream));
    return TE_OK;
}

int te_clay_encode(te_clay *c, const uint8_t *data, size_t len, uint8_t *chunks, size_t cap, size_t *chunk_size) {
    if (!c || (!data && len) || !chunks) return TE_ERR_INVALID_ARG;
    if (len == 0) return TE_ERR_EMPTY_INPUT;  // clay.rs:100-102
    const size_t cs = c->h.chunk_size_for(len);
    const size_t total = (size_t)c->h.n * cs;
    if (chunk_size) *chunk_size = cs;
    if (cap < total) return TE_ERR_BUFFER_TOO_SMALL;
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard dg(c->device);
    TE_HIP(dg.err);
    int r = ensure_stream(c);
    if (r) return r;
    TE_HIP(c->io_in.ensure(len + 16));
    TE_HIP(c->io_out.ensure(total));
    TE_HIP(hipMemcpyAsync(c->io_in.p, data, len, hipMemcpyHostToDevice, c->stream));
    te_object o{0, len, 0, 0};
    te_slicer_cfg cfg{0, TE_ENCODING_CLAY, TE_CLAY_DEFAULT_PARAMS, 0};
    r = encode_enqueue(c, &cfg, c->io_in.as<uint8_t>(), &o, 1, c->io_out.as<uint8_t>(), c->stream, true, nullptr,
                       StripeSel(), true);
    if (r) return r;
    TE_HIP(hipMemcpyAsync(chunks, c->io_out.p, total, hipMemcpyDeviceToHost, c->stream));
    TE_HIP(hipStreamSynchronize(c->stream));
    return TE_OK;
}

}  // extern "C"
// The given slices (n pointers, null = absent) to c->io_in at i * len, on c->stream.  Page-locked
// ones, and long ones, are copied directly; only the short pageable ones are first gathered into
// the handle's pinned staging by the device's copy pool (one pageable slice used to
// send every slice, pinned ones included, through the gather): each pageable H2D goes through the
// driver's staging at ~57 us of fixed cost (te_slicer_decode, 7 x 715 KB: 1.11 -> 0.81 ms per
// 4 MiB call, against 0.70 with pinned slices, r05).  Long ones go to the driver, whose pageable
// path outruns the 4-thread memcpy there (7 x 11.4 MB, 64 MiB object: 3.03 ms direct, 4.2-4.5
// gathered).
constexpr size_t kGatherMaxSlice = 2u << 20;
static int upload_slices(te_clay *c, const uint8_t *const *slices, size_t len) {
    const int n = c->h.n;
    const uint8_t *src[64];
    int gather = 0;
    for (int i = 0; i < n; i++) {
        src[i] = slices[i];
        if (slices[i] && len <= kGatherMaxSlice && !host_pinned(slices[i])) gather++;
    }
    if (gather) {
        TE_HIP(c->hio_in.ensure((size_t)gather * len));
        std::vector<tec::CopyPool::Seg> segs;
        for (int i = 0, g = 0; i < n; i++)
            if (slices[i] && len <= kGatherMaxSlice && !host_pinned(slices[i])) {
                src[i] = c->hio_in.u8() + (size_t)g++ * len;
                segs.push_back({const_cast<uint8_t *>(src[i]), slices[i], len});
            }
        copy_pool(c->device).run(segs);
    }
    for (int i = 0; i < n; i++)
        if (slices[i])
            TE_HIP(hipMemcpyAsync(c->io_in.as<uint8_t>() + (size_t)i * len, src[i], len, hipMemcpyHostToDevice,
                                  c->stream));
    return TE_OK;
}
extern "C" {

int te_clay_decode(te_clay *c, const uint8_t *const *chunks, size_t cs, uint8_t *out, size_t cap) {
    if (!c || !chunks || !out) return TE_ERR_INVALID_ARG;
    const ClayHost &h = c->h;
    uint32_t avail = 0;
    int na = 0;
    for (int i = 0; i < h.n; i++)
        if (chunks[i]) { avail |= 1u << i; na++; }
    if (na < h.k) return TE_ERR_NOT_ENOUGH_SLICES;  // clay.rs:107-109
    if (cs == 0 || cs % (size_t)h.alpha) return TE_ERR_BAD_ENCODING;
    if (cap < (size_t)h.k * cs) return TE_ERR_BUFFER_TOO_SMALL;
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard dg(c->device);
    TE_HIP(dg.err);
    int r = ensure_stream(c);
    if (r) return r;
    const size_t total = (size_t)h.n * cs;
    DecItem it{};
    it.in_base = 0; it.slice_len = cs; it.blob_len = (uint64_t)h.k * cs; it.stripe = it.blob_len; it.ns = 1; it.cs = cs;
    it.out_off = 0; it.avail = avail;
    // one stripe: the zero-copy per-call path of te_slicer_decode (staging read and written over PCIe)
    static const bool zc = [] { const char *e = tec_knob("TEC_DECODE_ZC"); return !(e && e[0] == '0'); }();
    if (zc) {
        TE_HIP(c->hio_in.ensure(total));
        std::vector<tec::CopyPool::Seg> segs;
        for (int i = 0; i < h.n; i++)
            if (chunks[i]) segs.push_back({c->hio_in.u8() + (size_t)i * cs, chunks[i], cs});
        copy_pool(c->device).run(segs);
        const bool out_pinned = host_pinned(out);
        if (!out_pinned) TE_HIP(c->hio_out.ensure((size_t)h.k * cs));
        uint8_t *dst = out_pinned ? out : c->hio_out.u8();
        r = decode_enqueue(c, nullptr, c->hio_in.u8(), &it, 1, dst, c->stream, true);
        if (r) return r;
        TE_HIP(hipStreamSynchronize(c->stream));
        if (!out_pinned) copy_pool(c->device).run({{out, c->hio_out.p, (size_t)h.k * cs}});
        return TE_OK;
    }
    TE_HIP(c->io_in.ensure(total));
    TE_HIP(c->io_out.ensure((size_t)h.k * cs));
    r = upload_slices(c, chunks, cs);
    if (r) return r;
    r = decode_enqueue(c, nullptr, c->io_in.as<uint8_t>(), &it, 1, c->io_out.as<uint8_t>(), c->stream, true);
    if (r) return r;
    TE_HIP(hipMemcpyAsync(out, c->io_out.p, (size_t)h.k * cs, hipMemcpyDeviceToHost, c->stream));
    TE_HIP(hipStreamSynchronize(c->stream));
    return TE_OK;
}

int te_slicer_decode(te_clay *c, const te_slicer_cfg *cfg, const uint8_t *const *slices, size_t slice_len,
                     uint8_t *out, size_t cap, size_t *out_len) {
    if (!c || !cfg || !slices) return TE_ERR_INVALID_ARG;
    const ClayHost &h = c->h;
    uint32_t avail = 0;
    int first = -1;
    for (int i = 0; i < h.n; i++)
        if (slices[i]) { avail |= 1u << i; if (first < 0) first = i; }
    if (first < 0) return TE_ERR_NOT_ENOUGH_SLICES;
    if (slice_len < TE_META_SIZE) return TE_ERR_INVALID_LAYOUT;
    DecItem it{};
    int r = decode_validate(c, slices[first] + slice_len - TE_META_SIZE, slice_len, avail, it);
    if (r) return r;
    if (out_len) *out_len = it.blob_len;
    if (it.blob_len == 0) return TE_OK;
    if (!out || cap < it.blob_len) return TE_ERR_BUFFER_TOO_SMALL;
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard dg(c->device);
    TE_HIP(dg.err);
    r = ensure_stream(c);
    if (r) return r;
    const size_t total = (size_t)h.n * slice_len;
    it.in_base = 0;
    it.out_off = 0;
    // A per-call decode (<= 64 stripes, the one-wave class kernels) reads its slices from page-
    // locked host staging and writes the object to page-locked memory over PCIe, with no H2D /
    // D2H copy around a 0.3 ms kernel whose loader wave issues its loads four steps ahead; the
    // slices are gathered into the staging by the copy pool (the repair call's scheme).
    // Measurement option TEC_DEBUG_KNOBS=1 TEC_DECODE_ZC=0: the copies instead.
    static const bool zc = [] { const char *e = tec_knob("TEC_DECODE_ZC"); return !(e && e[0] == '0'); }();
    if (zc && it.ns <= kDecSmallStripes) {
        TE_HIP(c->hio_in.ensure(total));
        std::vector<tec::CopyPool::Seg> segs;
        for (int i = 0; i < h.n; i++)
            if (slices[i]) segs.push_back({c->hio_in.u8() + (size_t)i * slice_len, slices[i], slice_len});
        copy_pool(c->device).run(segs);
        const bool out_pinned = host_pinned(out);
        if (!out_pinned) TE_HIP(c->hio_out.ensure(it.blob_len));
        uint8_t *dst = out_pinned ? out : c->hio_out.u8();
        r = decode_enqueue(c, cfg, c->hio_in.u8(), &it, 1, dst, c->stream, false);
        if (r) return r;
        TE_HIP(hipStreamSynchronize(c->stream));
        if (!out_pinned) copy_pool(c->device).run({{out, c->hio_out.p, it.blob_len}});
        return TE_OK;
    }
    TE_HIP(c->io_in.ensure(total));
    TE_HIP(c->io_out.ensure(it.blob_len));
    r = upload_slices(c, slices, slice_len);
    if (r) return r;
    r = decode_enqueue(c, cfg, c->io_in.as<uint8_t>(), &it, 1, c->io_out.as<uint8_t>(), c->stream, false);
    if (r) return r;
    TE_HIP(hipMemcpyAsync(out, c->io_out.p, it.blob_len, hipMemcpyDeviceToHost, c->stream));
    TE_HIP(hipStreamSynchronize(c->stream));
    return TE_OK;
}

// ------------------------------------------------------------------------------------------
// Repair planning (host only)
// ------------------------------------------------------------------------------------------
int te_clay_plan_repair(const te_clay *c, uint32_t lost, const uint32_t *available, size_t navail,
                        uint32_t *helpers_out, uint32_t *sub_chunks_out) {
    if (!c || (!available && navail)) return TE_ERR_INVALID_ARG;
    const ClayHost &h = c->h;
    if (lost >= (uint32_t)h.n) return TE_ERR_INVALID_SLICE;
    std::vector<int> av(available, available + navail), hs;
    const int r = h.min_to_repair((int)lost, av, hs);
    if (r) return clay_plan_error(r, (int)lost, navail, h.d);
    if (helpers_out)
        for (size_t i = 0; i < hs.size(); i++) helpers_out[i] = (uint32_t)hs[i];
    if (sub_chunks_out) {
        const std::vector<int> pl = h.repair_planes((int)lost);
        for (size_t i = 0; i < pl.size(); i++) sub_chunks_out[i] = (uint32_t)pl[i];
    }
    return TE_OK;
}

int te_repair_plan_from_params(const te_clay *c, int rotated, uint32_t lost, const uint32_t *avail, size_t navail,
                               uint64_t blob_len, uint64_t stripe, te_repair_plan **out) {
    if (!c || !out || (!avail && navail) || stripe == 0) return TE_ERR_INVALID_ARG;
    *out = nullptr;
    const uint64_t ns = blob_len == 0 ? 1 : (blob_len + stripe - 1) / stripe;
    const uint64_t cs = c->h.chunk_size_for(std::min(stripe, blob_len));  // track_chunk_size
    return build_plan(c, rotated, lost, avail, navail, ns, cs, out);
}

int te_repair_plan_from_slice(const te_clay *c, int rotated, uint32_t lost, const uint32_t *avail, size_t navail,
                              const uint8_t *ref, size_t ref_len, te_repair_plan **out) {
    if (!c || !out || !ref) return TE_ERR_INVALID_ARG;
    *out = nullptr;
    te_slice_metadata m;
    if (te_slice_metadata_from_slice(ref, ref_len, &m)) return TE_ERR_INVALID_LAYOUT;
    const uint64_t ns = m.blob_len == 0 ? 1 : (m.blob_len + m.stripe_size - 1) / m.stripe_size;
    const uint64_t total = ref_len >= TE_META_SIZE ? ref_len - TE_META_SIZE : 0;
    if (total == 0 || total % ns) return TE_ERR_INVALID_LAYOUT;
    return build_plan(c, rotated, lost, avail, navail, ns, total / ns, out);
}

void te_repair_plan_free(te_repair_plan *p) { delete p; }

int te_repair_plan_get_info(const te_repair_plan *p, te_repair_plan_info *o) {
    if (!p || !o) return TE_ERR_INVALID_ARG;
    o->lost = p->lost; o->num_stripes = p->ns; o->d = p->d; o->beta = p->beta;
    o->chunk_size = p->cs; o->sub_chunk_size = p->sc;
    return TE_OK;
}

int te_repair_plan_stripe(const te_repair_plan *p, uint32_t st, uint32_t *lost_shard, uint32_t *helper_slices,
                          uint32_t *helper_shards, uint32_t *sub_chunks) {
    if (!p || st >= p->ns) return TE_ERR_INVALID_ARG;
    if (lost_shard) *lost_shard = p->lost_shard[st];
    for (uint32_t j = 0; j < p->d; j++) {
        if (helper_slices) helper_slices[j] = p->helper_slice[st * p->d + j];
        if (helper_shards) helper_shards[j] = p->helper_shard[st * p->d + j];
        if (sub_chunks)
            for (uint32_t b = 0; b < p->beta; b++) sub_chunks[j * p->beta + b] = p->sub_chunks[(st * p->d + j) * p->beta + b];
    }
    return TE_OK;
}

size_t te_extract_repair_data_size(const te_repair_plan *p, uint32_t helper) {
    if (!p) return 0;
    size_t total = 0;
    for (uint32_t st = 0; st < p->ns; st++)
        for (uint32_t j = 0; j < p->d; j++)
            if (p->helper_slice[st * p->d + j] == helper) total += (size_t)p->beta * p->sc;
    return total;
}

int te_extract_repair_data(const te_repair_plan *p, const uint8_t *slice, size_t slice_len, uint32_t helper,
                           uint8_t *out, size_t cap, size_t *out_len) {
    if (!p || !slice) return TE_ERR_INVALID_ARG;
    const size_t need = te_extract_repair_data_size(p, helper);
    if (out_len) *out_len = need;
    if (cap < need || (!out && need)) return TE_ERR_BUFFER_TOO_SMALL;
    size_t w = 0;
    for (uint32_t st = 0; st < p->ns; st++) {
        const uint64_t co = (uint64_t)st * p->cs;
        for (uint32_t j = 0; j < p->d; j++) {
            if (p->helper_slice[st * p->d + j] != helper) continue;
            if (co + p->cs > slice_len) return TE_ERR_INVALID_LAYOUT;  // "slice too short for chunk"
            for (uint32_t b = 0; b < p->beta; b++) {
                const uint64_t z = p->sub_chunks[(st * p->d + j) * p->beta + b];
                if ((z + 1) * p->sc > p->cs) return TE_ERR_INVALID_LAYOUT;  // "sub-chunk out of bounds"
                memcpy(out + w, slice + co + z * p->sc, p->sc);
                w += p->sc;
            }
        }
    }
    return TE_OK;
}

int te_repair_plan_helper_request(const te_repair_plan *p, uint32_t helper, uint32_t *stripes, uint32_t *sub_chunks,
                                  size_t cap_stripes, size_t *count) {
    if (!p || !count) return TE_ERR_INVALID_ARG;
    size_t k = 0;
    for (uint32_t st = 0; st < p->ns; st++)
        for (uint32_t j = 0; j < p->d; j++) {
            if (p->helper_slice[st * p->d + j] != helper) continue;
            if (k < cap_stripes && stripes && sub_chunks) {
                stripes[k] = st;
                memcpy(sub_chunks + k * p->beta, &p->sub_chunks[(st * p->d + j) * p->beta], p->beta * sizeof(uint32_t));
            }
            k++;
        }
    *count = k;
    return k <= cap_stripes || (!stripes && !sub_chunks) ? TE_OK : TE_ERR_BUFFER_TOO_SMALL;
}

int te_serve_repair_request(te_clay *c, const uint8_t *slice, size_t slice_len, const uint32_t *stripes,
                            const uint32_t *nsub, const uint32_t *sub_chunks, size_t nstripes, uint8_t *out, size_t cap,
                            size_t *out_len) {
    if (!c || !slice || (nstripes && (!stripes || !nsub))) return TE_ERR_INVALID_ARG;
    auto fail = [](const char *why) {
        snprintf(g_last_error, sizeof(g_last_error), "%s", why);
        return TE_ERR_INVALID_LAYOUT;
    };
    te_slice_metadata m;
    if (slice_len < TE_META_SIZE) return fail("slice too short for metadata");
    if (te_slice_metadata_from_slice(slice, slice_len, &m) != TE_OK) return fail("parse slice metadata failed");
    if (m.blob_len && !m.stripe_size) return fail("parse slice metadata failed: zero stripe size");
    const uint64_t ns = m.blob_len == 0 ? 1 : (m.blob_len + m.stripe_size - 1) / m.stripe_size;
    const uint64_t total = slice_len - TE_META_SIZE;
    if (total == 0 || total % ns) return fail("slice layout is inconsistent");
    const uint64_t cs = total / ns, alpha = (uint64_t)c->h.alpha;
    if (cs % alpha) return fail("chunk size is not divisible by alpha");
    const uint64_t sc = cs / alpha;
    uint64_t need = 0;
    size_t at = 0;
    for (size_t i = 0; i < nstripes; i++) {
        const uint64_t c0 = (uint64_t)stripes[i] * cs;
        if (c0 + cs > total + TE_META_SIZE) return fail("slice too short for requested stripe");
        for (uint32_t b = 0; b < nsub[i]; b++, at++)
            if (!sub_chunks || ((uint64_t)sub_chunks[at] + 1) * sc > cs) return fail("sub-chunk out of bounds");
        need += (uint64_t)nsub[i] * sc;
    }
    if (out_len) *out_len = (size_t)need;
    if (cap < need || (!out && need)) return TE_ERR_BUFFER_TOO_SMALL;
    uint64_t w = 0;
    at = 0;
    for (size_t i = 0; i < nstripes; i++)
        for (uint32_t b = 0; b < nsub[i]; b++, at++) {
            memcpy(out + w, slice + (uint64_t)stripes[i] * cs + (uint64_t)sub_chunks[at] * sc, sc);
            w += sc;
        }
    return TE_OK;
}

int te_slicer_repair(te_clay *c, const te_repair_plan *p, const uint8_t *const *helper_data, const size_t *helper_lens,
                     const uint8_t metadata[TE_META_SIZE], uint8_t *out, size_t cap) {
    if (!c || !p || !helper_data || !helper_lens || !metadata || !out) return TE_ERR_INVALID_ARG;
    if (p->n != (uint32_t)c->h.n || p->d != (uint32_t)c->h.d) return TE_ERR_INVALID_ARG;
    const size_t out_bytes = (size_t)p->ns * p->cs + TE_META_SIZE;
    if (cap < out_bytes) return TE_ERR_BUFFER_TOO_SMALL;
    // per-helper byte need (Slicer::repair walks a running offset per helper: repair.rs:340-354)
    std::vector<uint64_t> need(p->n, 0), off(p->n, ~0ull);
    for (uint32_t st = 0; st < p->ns; st++)
        for (uint32_t j = 0; j < p->d; j++) need[p->helper_slice[st * p->d + j]] += (uint64_t)p->beta * p->sc;
    uint64_t total = 0;
    for (uint32_t sl = 0; sl < p->n; sl++) {
        if (!need[sl]) continue;
        if (!helper_data[sl] || helper_lens[sl] < need[sl]) return TE_ERR_MISSING_HELPER;
        off[sl] = total;
        total += (need[sl] + 15) & ~15ull;
    }
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard dg(c->device);
    TE_HIP(dg.err);
    int r = ensure_stream(c);
    if (r) return r;
    TE_HIP(c->io_in.ensure(total + 16));
    TE_HIP(c->io_out.ensure(out_bytes));
    // the d helpers' buffers gathered into page-locked staging (parallel memcpy), one H2D; the
    // repaired slice back through staging: per call two DMA copies, not d + 1 driver-staged ones
    TE_HIP(c->hio_in.ensure(total + 16));
    TE_HIP(c->hio_out.ensure(out_bytes));
    std::vector<tec::CopyPool::Seg> segs;
    for (uint32_t sl = 0; sl < p->n; sl++)
        if (need[sl]) segs.push_back({c->hio_in.u8() + off[sl], helper_data[sl], need[sl]});
    copy_pool(c->device).run(segs);
    // the kernels read the helpers from and write the slice to the pinned staging directly, over
    // PCIe, with no H2D / D2H copy: 0.131 -> 0.103 ms per 4 MiB call, 0.85 -> 0.73 ms at 64 MiB
    // (r05, scripts/gpu_percall_zc.sh; the repair kernels only read their inputs and write their
    // output once).  Measurement option TEC_DEBUG_KNOBS=1 TEC_REPAIR_ZC=0: the copies instead.
    static const bool zc = [] { const char *e = tec_knob("TEC_REPAIR_ZC"); return !(e && e[0] == '0'); }();
    RepItem it{p, off.data(), 0, metadata};
    if (zc) {
        r = repair_enqueue(c, c->hio_in.u8(), &it, 1, c->hio_out.u8(), c->stream);
        if (r) return r;
    } else {
        TE_HIP(hipMemcpyAsync(c->io_in.p, c->hio_in.p, total, hipMemcpyHostToDevice, c->stream));
        r = repair_enqueue(c, c->io_in.as<uint8_t>(), &it, 1, c->io_out.as<uint8_t>(), c->stream);
        if (r) return r;
        TE_HIP(hipMemcpyAsync(c->hio_out.p, c->io_out.p, out_bytes, hipMemcpyDeviceToHost, c->stream));
    }
    TE_HIP(hipStreamSynchronize(c->stream));  // (an event spin-wait measured no better: 0.146 vs 0.132-0.139 ms, r05)
    // (pipelining the gather with the H2D in four pieces and the scatter with the D2H in two
    // halves measured slower: 0.17 against 0.134-0.143 ms per 4 MiB call, r05)
    copy_pool(c->device).run({{out, c->hio_out.p, out_bytes}});
    return TE_OK;
}

int te_clay_repair(te_clay *c, uint32_t lost, const uint32_t *helpers, const uint8_t *const *helper_data,
                   size_t nhelpers, size_t chunk_size, uint8_t *out) {
    if (!c || !helpers || !helper_data || !out) return TE_ERR_INVALID_ARG;
    const ClayHost &h = c->h;
    if (lost >= (uint32_t)h.n) return TE_ERR_INVALID_SLICE;
    if (nhelpers != (size_t)h.d) {  // clay_codes::ClayCode::repair rejects it -> RepairError::Clay (repair.rs:85-87)
        snprintf(g_last_error, sizeof(g_last_error), "repair: need exactly d=%d helpers, got %zu", h.d, nhelpers);
        return TE_ERR_CLAY;
    }
    if (chunk_size == 0 || chunk_size % (size_t)h.alpha) return TE_ERR_INVALID_LAYOUT;
    // one-stripe, identity-mapped plan with the caller's helper set
    te_repair_plan p;
    p.lost = lost; p.ns = 1; p.d = (uint32_t)h.d; p.beta = (uint32_t)h.beta; p.n = (uint32_t)h.n;
    p.cs = chunk_size; p.sc = chunk_size / (size_t)h.alpha;
    p.lost_shard.push_back(lost);
    const std::vector<int> planes = h.repair_planes((int)lost);
    std::vector<const uint8_t *> by_slice(h.n, nullptr);
    std::vector<size_t> lens(h.n, 0);
    std::vector<int> hs;
    for (size_t j = 0; j < nhelpers; j++) {
        if (helpers[j] >= (uint32_t)h.n || helpers[j] == lost) return TE_ERR_INVALID_SLICE;
        hs.push_back((int)helpers[j]);
    }
    std::sort(hs.begin(), hs.end());
    for (size_t j = 0; j < nhelpers; j++) {
        by_slice[helpers[j]] = helper_data[j];
        lens[helpers[j]] = (size_t)h.beta * p.sc;
    }
    for (int sh : hs) {
        p.helper_shard.push_back((uint32_t)sh);
        p.helper_slice.push_back((uint32_t)sh);
        for (int z : planes) p.sub_chunks.push_back((uint32_t)z);
    }
    std::vector<uint8_t> tmp(chunk_size + TE_META_SIZE);
    uint8_t meta[TE_META_SIZE] = {0};
    int r = te_slicer_repair(c, &p, by_slice.data(), lens.data(), meta, tmp.data(), tmp.size());
    if (r) return r;
    memcpy(out, tmp.data(), chunk_size);
    return TE_OK;
}


// ---- slice commitments (lib/crypto/src/merkle/tree.rs) ----
int te_hash_leaf(const uint8_t *data, size_t len, uint8_t out[TE_HASH_SIZE]) {
    if ((!data && len) || !out) return TE_ERR_INVALID_ARG;
    hh::hash_leaf(data, len, out);
    return TE_OK;
}

int te_hash_leaves(const uint8_t *data, size_t len, size_t count, uint32_t lanes, uint8_t *out) {
    if ((!data && len && count) || (!out && count) || lanes > (uint32_t)hh::kMaxLanes) return TE_ERR_INVALID_ARG;
    if (lanes == 0) lanes = (uint32_t)hh::Pool::get().lanes();
    const uint8_t *src[hh::kMaxLanes];
    uint8_t *dst[hh::kMaxLanes];
    for (size_t i0 = 0; i0 < count; i0 += lanes) {
        const int L = (int)std::min<size_t>(lanes, count - i0);
        for (int l = 0; l < L; l++) {
            src[l] = data + (i0 + l) * len;
            dst[l] = out + (i0 + l) * TE_HASH_SIZE;
        }
        hh::hash_leaves(L, src, len, dst);
    }
    return TE_OK;
}

int te_hash_pair(const uint8_t left[TE_HASH_SIZE], const uint8_t right[TE_HASH_SIZE], uint8_t out[TE_HASH_SIZE]) {
    if (!left || !right || !out) return TE_ERR_INVALID_ARG;
    sha::hash_pair(left, right, out);
    return TE_OK;
}

int te_empty_subtree_root(uint32_t height, uint8_t out[TE_HASH_SIZE]) {
    if (height >= TE_MAX_MERKLE_TREE_HEIGHT || !out) return TE_ERR_INVALID_ARG;
    sha::empty_root(height, out);
    return TE_OK;
}

// MerkleTree::<N>::new() + add_leaf_hash per leaf (tree.rs:86-153, 344-350)
int te_merkle_root_from_leaf_hashes(const uint8_t *hashes, size_t count, uint32_t height, uint8_t out[TE_HASH_SIZE]) {
    if (height == 0 || height > TE_MAX_MERKLE_TREE_HEIGHT || (!hashes && count) || !out) return TE_ERR_INVALID_ARG;
    if (height < 64 && (uint64_t)count > (1ull << height)) return TE_ERR_MERKLE_TREE_FULL;
    std::vector<std::array<uint8_t, 32>> empty(height), filled(height);
    for (uint32_t l = 0; l < height; l++) {
        sha::empty_root(l, empty[l].data());
        filled[l] = empty[l];
    }
    std::array<uint8_t, 32> root = empty[height - 1];
    for (size_t index = 0; index < count; index++) {
        std::array<uint8_t, 32> cur, t;
        memcpy(cur.data(), hashes + index * 32, 32);
        uint64_t idx = index;
        for (uint32_t l = 0; l < height; l++) {
            if ((idx & 1) == 0) {
                filled[l] = cur;
                sha::hash_pair(cur.data(), empty[l].data(), t.data());
            } else {
                sha::hash_pair(filled[l].data(), cur.data(), t.data());
            }
            cur = t;
            idx >>= 1;
        }
        root = cur;
    }
    memcpy(out, root.data(), 32);
    return TE_OK;
}

// create_merkle_proof_hashes (tree.rs:397-455)
int te_merkle_proof_from_leaf_hashes(const uint8_t *hashes, size_t count, size_t index, uint32_t height,
                                     uint8_t *proof_out) {
    if (!proof_out) return TE_ERR_INVALID_ARG;
    if (!hashes || count == 0 || index >= count || height > TE_MAX_MERKLE_TREE_HEIGHT ||
        (height < 64 && (uint64_t)count > (1ull << height)))
        return TE_ERR_MERKLE_INVALID_PROOF;
    std::vector<std::array<uint8_t, 32>> cur(count);
    for (size_t i = 0; i < count; i++) memcpy(cur[i].data(), hashes + i * 32, 32);
    std::array<uint8_t, 32> empty;
    sha::empty_root(0, empty.data());
    size_t ci = index;
    for (uint32_t l = 0; l < height; l++) {
        if (cur.size() % 2) cur.push_back(empty);
        memcpy(proof_out + (size_t)l * 32, cur[ci ^ 1].data(), 32);
        std::vector<std::array<uint8_t, 32>> next(cur.size() / 2);
        for (size_t j = 0; j < next.size(); j++) sha::hash_pair(cur[2 * j].data(), cur[2 * j + 1].data(), next[j].data());
        cur.swap(next);
        std::array<uint8_t, 32> e2;
        sha::hash_pair(empty.data(), empty.data(), e2.data());
        empty = e2;
        ci >>= 1;
    }
    return TE_OK;
}

// verify_proof (tree.rs:462-481), leaf already hashed
int te_merkle_verify_leaf_hash(const uint8_t leaf_hash[TE_HASH_SIZE], const uint8_t root[TE_HASH_SIZE],
                               const uint8_t *proof, size_t proof_len, uint64_t index, uint32_t height) {
    if (!leaf_hash || !root || (!proof && proof_len)) return TE_ERR_INVALID_ARG;
    if (proof_len != height) return 0;
    uint8_t node[32], t[32];
    memcpy(node, leaf_hash, 32);
    uint64_t idx = index;
    for (size_t i = 0; i < proof_len; i++) {
        if ((idx & 1) == 0) sha::hash_pair(node, proof + i * 32, t);
        else sha::hash_pair(proof + i * 32, node, t);
        memcpy(node, t, 32);
        idx >>= 1;
    }
    return memcmp(node, root, 32) == 0 ? 1 : 0;
}

int te_commit_batch_device(const uint8_t *d_slices, uint64_t obj_stride, uint64_t slice_len, uint32_t n,
                           size_t nobj, uint32_t height, uint8_t *d_leaf_hashes, uint8_t *d_roots,
                           uint8_t *d_proofs, void *stream) {
    if (nobj == 0) return TE_OK;
    if (!d_slices || !d_leaf_hashes || n == 0 || n > TE_COMMIT_MAX_LEAVES || slice_len % 4 ||
        nobj > 0xffffffffull / n || ((d_roots || d_proofs) && (height == 0 || height > TE_MAX_MERKLE_TREE_HEIGHT)) ||
        (d_proofs && !d_roots))
        return TE_ERR_INVALID_ARG;
    if ((d_roots || d_proofs) && height < 64 && (uint64_t)n > (1ull << height)) return TE_ERR_MERKLE_TREE_FULL;
    if (device_count() <= 0) return TE_ERR_NO_DEVICE;
    CommitArgs a{};
    a.slices = d_slices;
    a.obj_stride = obj_stride;
    a.slice_len = slice_len;
    a.n = n;
    a.nobj = (uint32_t)nobj;
    a.height = height;
    a.leaf = d_leaf_hashes;
    a.root = d_roots;
    a.proof = d_proofs;
    hipStream_t s = (hipStream_t)stream;
    KTimer kt(s);
    TE_HIP(launch_commit(a, s));
    kt.stop();
    return TE_OK;
}


// ------------------------------------------------------------------------------------------
// OuterCoder: GF(2^16) Leopard RS (lib/slicer/src/outer.rs:19-197)
// ------------------------------------------------------------------------------------------
size_t te_outer_chunk_bytes(uint32_t k, size_t len) {  // outer.rs:74-80
    if (k == 0) return 0;
    if (len == 0) return 64;
    const size_t raw = (len + k - 1) / k;
    return (raw + 63) / 64 * 64;
}

}  // extern "C"
namespace {
int outer_encode_matrix(uint32_t k, uint32_t m, const uint8_t *d_in, uint64_t chunk_bytes, uint32_t segments,
                        uint64_t seg_in, uint8_t *d_out, uint64_t seg_out, hipStream_t s);
}
extern "C" {

int te_outer_encode_device(uint32_t k, uint32_t m, const uint8_t *d_in, uint64_t chunk_bytes, uint32_t segments,
                           uint64_t seg_in, uint8_t *d_out, uint64_t seg_out, void *stream) {
    if (k == 0 || m == 0 || !d_in || !d_out || chunk_bytes == 0 || chunk_bytes % 64 || chunk_bytes / 2 > 0xffffffffull)
        return TE_ERR_INVALID_ARG;
    if (rs16::use_high_rate(k, m) < 0) return TE_ERR_UNSUPPORTED;
    if (device_count() <= 0) return TE_ERR_NO_DEVICE;
    // the encode as a matrix product (rs16_matrix_kernel) when its lookup image fits the LDS budget:
    // OuterCoder(17, 50) 17 x 33; the transforms below otherwise
    if (rs16_mat_supported(k, m) && !tec_knob("TEC_RS16_NO_MATRIX"))
        return outer_encode_matrix(k, m, d_in, chunk_bytes, segments, seg_in, d_out, seg_out, (hipStream_t)stream);
    const rs16::Tables &T = rs16::tables();
    const uint32_t c = rs16::chunk(k, m), span = rs16::skew_span(k, m), wl = rs16::work_len(k, m);
    if ((size_t)span * 128 + (size_t)wl * 256 > 160 * 1024 || span > rs16::kModulus) return TE_ERR_UNSUPPORTED;
    // nibble tables of every skew multiplier the transforms touch (zeros for the basis' zero)
    std::vector<uint16_t> lut((size_t)span * 64, 0);
    for (uint32_t sx = 0; sx < span; sx++) {
        const uint16_t lm = T.skew[sx];
        if (lm == rs16::kModulus) continue;
        for (int q = 0; q < 4; q++)
            for (uint32_t nb = 0; nb < 16; nb++) lut[(size_t)sx * 64 + q * 16 + nb] = T.mul((uint16_t)(nb << (4 * q)), lm);
    }
    hipStream_t s = (hipStream_t)stream;
    uint16_t *d_lut = nullptr;
    TE_HIP(hipMallocAsync((void **)&d_lut, lut.size() * sizeof(uint16_t), s));
    int r = hip_status(hipMemcpyAsync(d_lut, lut.data(), lut.size() * sizeof(uint16_t), hipMemcpyHostToDevice, s));
    if (r == TE_OK) {
        Rs16EncArgs a{};
        a.in = d_in;
        a.out = d_out;
        a.in_stride = a.out_stride = chunk_bytes;
        a.seg_in = seg_in;
        a.seg_out = seg_out;
        a.lut = d_lut;
        a.k = k; a.m = m; a.c = c; a.high = (uint32_t)rs16::use_high_rate(k, m);
        a.work_len = wl; a.span = span; a.elems = (uint32_t)(chunk_bytes / 2);
        a.one_chunk = !a.high && c <= 32 && wl > c;
        KTimer kt(s);
        r = hip_status(launch_rs16_encode(a, segments, s));
        kt.stop();
    }
    const int r2 = hip_status(hipFreeAsync(d_lut, s));
    if (r == TE_OK) r = hip_status(hipStreamSynchronize(s));  // the host table must outlive the copy
    return r ? r : r2;
}

int te_outer_encode(uint32_t k, uint32_t n, const uint8_t *data, size_t len, uint8_t *out, size_t cap,
                    size_t *chunk_bytes_out) {
    if (k == 0 || k > n || (!data && len)) return TE_ERR_INVALID_ARG;
    const size_t cb = te_outer_chunk_bytes(k, len);
    if (chunk_bytes_out) *chunk_bytes_out = cb;
    if (cb > TE_OUTER_MAX_CHUNK_BYTES) return TE_ERR_TOO_MUCH_DATA;  // outer.rs:82-84
    if (!out || cap < (size_t)n * cb) return TE_ERR_BUFFER_TOO_SMALL;
    if (len) memcpy(out, data, len);
    memset(out + len, 0, (size_t)k * cb - len);
    const uint32_t m = n - k;
    if (m == 0) return TE_OK;
    if (rs16::use_high_rate(k, m) < 0) return TE_ERR_UNSUPPORTED;
    if (device_count() <= 0) return TE_ERR_NO_DEVICE;
    uint8_t *d = nullptr;
    TE_HIP(hipMalloc((void **)&d, (size_t)n * cb));
    int r = hip_status(hipMemcpy(d, out, (size_t)k * cb, hipMemcpyHostToDevice));
    if (r == TE_OK) r = te_outer_encode_device(k, m, d, cb, 1, 0, d + (size_t)k * cb, 0, nullptr);
    if (r == TE_OK) r = hip_status(hipMemcpy(out + (size_t)k * cb, d + (size_t)k * cb, (size_t)m * cb, hipMemcpyDeviceToHost));
    (void)hipFree(d);
    return r;
}

}  // extern "C"

// OuterCoder decode tables on the device, cached per (device, k, m, received set, missing set):
// a snapshot read repeats its erasure pattern for every segment, and deriving the decoding matrix
// (k unit-vector encodes and a k x 2k inversion over GF(2^16)), its nmiss x k nibble tables and
// their upload cost ~0.2 ms of host time per call (r04: 3.5 ms of the 6.8 ms step for 16
// segments).  At most kOuterLutCache patterns; the least recently used is freed once the last
// launch that read it (an event) has finished.
namespace {
constexpr size_t kOuterLutCache = 64;
struct OuterLut {
    uint16_t *d = nullptr;
    bool mat = false;      // rs16::mat_image for rs16_matrix_kernel (else per-coefficient nibble tables)
    ReaderEvents readers;  // the last launches that read the table, per stream
    uint64_t tick = 0;
};
std::mutex g_outer_mu;
std::map<std::vector<uint32_t>, OuterLut> g_outer_luts;
uint64_t g_outer_tick = 0;

int outer_lut(uint32_t k, uint32_t m, const std::vector<uint32_t> &recv, const std::vector<uint32_t> &miss, int dev,
              OuterLut *&out) {
    std::vector<uint32_t> key{(uint32_t)dev, k, m};
    key.insert(key.end(), recv.begin(), recv.end());
    key.push_back(0xffffffffu);
    key.insert(key.end(), miss.begin(), miss.end());
    auto it = g_outer_luts.find(key);
    if (it != g_outer_luts.end()) {
        it->second.tick = ++g_outer_tick;
        out = &it->second;
        return TE_OK;
    }
    const uint32_t nm = (uint32_t)miss.size();
    const bool enc = nm == 1 && miss[0] == 0xfffffffeu;  // the encode matrix (outer_enc_lut)
    const uint32_t rows = enc ? m : nm;
    std::vector<uint16_t> D;
    if (enc) rs16::encode_matrix(k, m, D);
    else if (!rs16::decode_matrix(k, m, recv, D)) return TE_ERR_INVALID_LAYOUT;
    const bool mat = rs16_mat_supported(k, rows);
    if (enc && !mat) return TE_ERR_UNSUPPORTED;
    std::vector<uint16_t> lut;
    if (mat) {  // the missing rows of D, as the matrix kernel's lookup image
        std::vector<uint16_t> Dm((size_t)rows * k);
        for (uint32_t i = 0; i < rows; i++)
            memcpy(&Dm[(size_t)i * k], &D[(size_t)(enc ? i : miss[i]) * k], k * sizeof(uint16_t));
        lut = rs16::mat_image(k, rows, Dm.data(), rs16_mat_tailv(rows), rs16_mat_tail_bytes(rows));
    } else {
        const rs16::Tables &T = rs16::tables();
        lut.assign((size_t)nm * k * 64, 0);
        for (uint32_t i = 0; i < nm; i++)
            for (uint32_t r = 0; r < k; r++) {
                const uint16_t coef = D[(size_t)miss[i] * k + r];
                if (!coef) continue;
                for (int q = 0; q < 4; q++)
                    for (uint32_t nb = 0; nb < 16; nb++)
                        lut[((size_t)i * k + r) * 64 + q * 16 + nb] = T.gmul((uint16_t)(nb << (4 * q)), coef);
            }
    }
    if (g_outer_luts.size() >= kOuterLutCache) {
        auto lru = g_outer_luts.begin();
        for (auto j = g_outer_luts.begin(); j != g_outer_luts.end(); ++j)
            if (j->second.tick < lru->second.tick) lru = j;
        DeviceGuard dg(lru->first[0]);
        (void)lru->second.readers.sync();  // every stream's last reader, then free
        lru->second.readers.destroy();
        (void)hipFree(lru->second.d);
        g_outer_luts.erase(lru);
    }
    OuterLut L;
    TE_HIP(hipMalloc((void **)&L.d, lut.size() * sizeof(uint16_t)));
    if (hipError_t e = hipMemcpy(L.d, lut.data(), lut.size() * sizeof(uint16_t), hipMemcpyHostToDevice); e != hipSuccess) {
        (void)hipFree(L.d);
        return hip_status(e);
    }
    L.mat = mat;
    L.tick = ++g_outer_tick;
    out = &(g_outer_luts[key] = L);
    return TE_OK;
}

// The encode matrix's image, cached like a decode pattern's (key: received = none, missing = the
// marker 0xfffffffe); the launch waits for its stream (te_outer_encode_device's contract).
int outer_encode_matrix(uint32_t k, uint32_t m, const uint8_t *d_in, uint64_t chunk_bytes, uint32_t segments,
                        uint64_t seg_in, uint8_t *d_out, uint64_t seg_out, hipStream_t s) {
    int dev = 0;
    TE_HIP(hipGetDevice(&dev));
    int r = TE_OK;
    {
        std::lock_guard<std::mutex> lk(g_outer_mu);
        OuterLut *L = nullptr;
        if ((r = outer_lut(k, m, {}, {0xfffffffeu}, dev, L))) return r;
        Rs16MatArgs a{};
        a.in = d_in;
        a.out = d_out;
        a.in_stride = a.out_stride = chunk_bytes;
        a.seg_in = seg_in;
        a.seg_out = seg_out;
        a.tab = L->d;
        a.k = k; a.rows = m; a.elems = (uint32_t)(chunk_bytes / 2); a.segments = segments; a.ptrs = 0;
        KTimer kt(s);
        r = hip_status(launch_rs16_matrix(a, s));
        kt.stop();
        if (r == TE_OK) r = hip_status(L->readers.record(s));
    }
    if (r == TE_OK) r = hip_status(hipStreamSynchronize(s));
    return r;
}

// Restore a group's missing chunks: `cnt` segments whose shard pointers are laid out as
// Rs16DecArgs::ptr (per segment k received, then nm outputs), through the matrix kernel when the
// pattern's table is a matrix image.
int outer_restore(const OuterLut *L, uint32_t k, uint32_t nm, const uint8_t *const *ptr, uint32_t cnt,
                  uint64_t chunk_bytes, hipStream_t s) {
    if (L->mat) {
        Rs16MatArgs a{};
        memcpy(a.ptr, ptr, (size_t)cnt * (k + nm) * sizeof(ptr[0]));
        a.tab = L->d;
        a.k = k; a.rows = nm; a.elems = (uint32_t)(chunk_bytes / 2); a.segments = cnt; a.ptrs = 1;
        KTimer kt(s);
        const int r = hip_status(launch_rs16_matrix(a, s));
        kt.stop();
        return r;
    }
    Rs16DecArgs a{};
    memcpy(a.ptr, ptr, (size_t)cnt * (k + nm) * sizeof(ptr[0]));
    a.lut = L->d;
    a.k = k; a.nmiss = nm; a.elems = (uint32_t)(chunk_bytes / 2);
    KTimer kt(s);
    const int r = hip_status(launch_rs16_decode(a, cnt, s));
    kt.stop();
    return r;
}
}  // namespace

extern "C" {

int te_outer_decode(uint32_t k, uint32_t n, const uint8_t *const *chunks, size_t chunk_bytes, uint8_t *out, size_t cap) {
    if (k == 0 || k > n || !chunks || !out) return TE_ERR_INVALID_ARG;
    std::vector<uint32_t> have;
    for (uint32_t i = 0; i < n; i++)
        if (chunks[i]) have.push_back(i);
    if (have.size() < k) return TE_ERR_NOT_ENOUGH_SLICES;   // outer.rs:127-129
    if (cap < (size_t)k * chunk_bytes) return TE_ERR_BUFFER_TOO_SMALL;
    const uint32_t m = n - k;
    std::vector<uint32_t> miss;
    for (uint32_t i = 0; i < k; i++) {
        if (chunks[i]) memcpy(out + (size_t)i * chunk_bytes, chunks[i], chunk_bytes);
        else miss.push_back(i);
    }
    if (miss.empty()) return TE_OK;
    if (m == 0) return TE_ERR_INVALID_LAYOUT;                 // outer.rs:143-152
    if (chunk_bytes == 0 || chunk_bytes % 64) return TE_ERR_INVALID_LAYOUT;  // the decoder's shard-size check
    if (rs16::use_high_rate(k, m) < 0 || k > kRs16MaxK) return TE_ERR_UNSUPPORTED;
    if (device_count() <= 0) return TE_ERR_NO_DEVICE;
    std::vector<uint32_t> recv(have.begin(), have.begin() + k);  // any k shards determine the originals
    const uint32_t nm = (uint32_t)miss.size();
    int dev = 0;
    TE_HIP(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(g_outer_mu);
    OuterLut *L = nullptr;
    int r = outer_lut(k, m, recv, miss, dev, L);
    if (r) return r;
    // device image: received shards, then restored shards
    const size_t sh = (size_t)k * chunk_bytes, rs = (size_t)nm * chunk_bytes;
    uint8_t *d = nullptr;
    TE_HIP(hipMalloc((void **)&d, sh + rs));
    std::vector<const uint8_t *> ptr(k + nm);
    for (uint32_t j = 0; j < k && r == TE_OK; j++) {
        ptr[j] = d + (size_t)j * chunk_bytes;
        r = hip_status(hipMemcpy(d + (size_t)j * chunk_bytes, chunks[recv[j]], chunk_bytes, hipMemcpyHostToDevice));
    }
    for (uint32_t i = 0; i < nm; i++) ptr[k + i] = d + sh + (size_t)i * chunk_bytes;
    if (r == TE_OK) {
        r = outer_restore(L, k, nm, ptr.data(), 1, chunk_bytes, nullptr);
        if (r == TE_OK) r = hip_status(L->readers.record(nullptr));
    }
    for (uint32_t i = 0; i < nm && r == TE_OK; i++)
        r = hip_status(hipMemcpy(out + (size_t)miss[i] * chunk_bytes, d + sh + (size_t)i * chunk_bytes, chunk_bytes,
                                 hipMemcpyDeviceToHost));
    (void)hipFree(d);
    return r;
}

}  // extern "C"

namespace {
// OuterCoder decode of `segments` segments on the device (outer.rs:126-197 per segment): segment g's
// chunk i at d_chunks[g * n + i] (NULL = missing), its k data chunks to d_out + g * seg_out.
// Received data chunks are copied; segments are grouped by erasure pattern, and each group's
// missing chunks are restored from its first k received chunks in launches of as many segments
// as fit the kernel's pointer arguments.  Enqueued on the stream, nothing uploaded but a new
// pattern's tables (cached): a snapshot read's segments queue back to back (r04: a host wait per
// segment cost 0.19 ms per 0.2 ms kernel).
int outer_decode_segs(uint32_t k, uint32_t n, const uint8_t *const *d_chunks, uint32_t segments, uint64_t chunk_bytes,
                      uint8_t *d_out, uint64_t seg_out, hipStream_t s) {
    if (k == 0 || k > n || !d_chunks || !d_out || segments == 0) return TE_ERR_INVALID_ARG;
    const uint32_t m = n - k;
    if (chunk_bytes == 0 || chunk_bytes % 64 || chunk_bytes / 2 > 0xffffffffull) return TE_ERR_INVALID_LAYOUT;
    if (segments > 1 && seg_out < (uint64_t)k * chunk_bytes) return TE_ERR_INVALID_ARG;  // segment outputs would overlap
    // validate every segment before anything is enqueued
    std::map<std::vector<uint32_t>, std::vector<uint32_t>> groups;  // recv | miss -> segments
    for (uint32_t g = 0; g < segments; g++) {
        const uint8_t *const *ch = d_chunks + (size_t)g * n;
        std::vector<uint32_t> have, miss;
        for (uint32_t i = 0; i < n; i++)
            if (ch[i]) have.push_back(i);
        if (have.size() < k) return TE_ERR_NOT_ENOUGH_SLICES;   // outer.rs:127-129
        for (uint32_t i = 0; i < k; i++)
            if (!ch[i]) miss.push_back(i);
        if (miss.empty()) continue;
        if (m == 0) return TE_ERR_INVALID_LAYOUT;  // outer.rs:143-152
        if (rs16::use_high_rate(k, m) < 0 || k > kRs16MaxK || k + miss.size() > kRs16DecPtrs) return TE_ERR_UNSUPPORTED;
        std::vector<uint32_t> key(have.begin(), have.begin() + k);  // any k shards determine the originals
        key.push_back(0xffffffffu);
        key.insert(key.end(), miss.begin(), miss.end());
        groups[key].push_back(g);
    }
    if (device_count() <= 0) return TE_ERR_NO_DEVICE;
    int r = TE_OK;
    for (uint32_t g = 0; g < segments && r == TE_OK; g++)
        for (uint32_t i = 0; i < k && r == TE_OK; i++)
            if (const uint8_t *c = d_chunks[(size_t)g * n + i])
                r = hip_status(hipMemcpyAsync(d_out + g * seg_out + (size_t)i * chunk_bytes, c, chunk_bytes,
                                              hipMemcpyDeviceToDevice, s));
    if (r != TE_OK || groups.empty()) return r;
    int dev = 0;
    TE_HIP(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(g_outer_mu);
    for (const auto &gr : groups) {
        const auto sep = std::find(gr.first.begin(), gr.first.end(), 0xffffffffu);
        const std::vector<uint32_t> recv(gr.first.begin(), sep), miss(sep + 1, gr.first.end());
        const uint32_t nm = (uint32_t)miss.size(), per = k + nm, fit = kRs16DecPtrs / per;
        OuterLut *L = nullptr;
        if ((r = outer_lut(k, m, recv, miss, dev, L))) return r;
        for (size_t g0 = 0; g0 < gr.second.size(); g0 += fit) {
            const uint32_t cnt = (uint32_t)std::min<size_t>(fit, gr.second.size() - g0);
            const uint8_t *ptr[kRs16DecPtrs];
            for (uint32_t q = 0; q < cnt; q++) {
                const uint32_t g = gr.second[g0 + q];
                for (uint32_t j = 0; j < k; j++) ptr[q * per + j] = d_chunks[(size_t)g * n + recv[j]];
                for (uint32_t i = 0; i < nm; i++) ptr[q * per + k + i] = d_out + g * seg_out + (size_t)miss[i] * chunk_bytes;
            }
            if ((r = outer_restore(L, k, nm, ptr, cnt, chunk_bytes, s))) return r;
        }
        if ((r = hip_status(L->readers.record(s)))) return r;
    }
    return r;
}
}  // namespace

extern "C" {

int te_outer_decode_device(uint32_t k, uint32_t n, const uint8_t *const *d_chunks, uint64_t chunk_bytes,
                           uint8_t *d_out, void *stream) {
    return outer_decode_segs(k, n, d_chunks, 1, chunk_bytes, d_out, 0, (hipStream_t)stream);
}

int te_outer_decode_device_batch(uint32_t k, uint32_t n, const uint8_t *const *d_chunks, uint32_t segments,
                                 uint64_t chunk_bytes, uint8_t *d_out, uint64_t seg_out, void *stream) {
    return outer_decode_segs(k, n, d_chunks, segments, chunk_bytes, d_out, seg_out, (hipStream_t)stream);
}

}  // extern "C"
