// dec_rtc.cpp -- per-pattern decode kernels compiled at run time (hipRTC), cached per handle.
//
// A pattern's kernel (dec_fixed.hpp, source from dec_rtc.hpp dec_fixed_source) takes ~25 s of
// host compile, so it is built only for hot patterns: once a (pattern, G) pair has decoded
// `min_stripes` stripes on the handle (mode async: on a worker thread, the table-driven
// decode_stage kernel serving the pattern until the module is loaded; mode sync: in the calling
// thread, for tests).  Nothing here runs on the CPU in place of the GPU: a failed compile leaves
// the pattern on the table-driven kernel.
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include "kernels.hpp"
#include "clay_host.hpp"
#include "dec_rtc.hpp"

namespace tec {

namespace {
const char kDecFixedHeader[] =
#include "dec_fixed_src.inc"
    ;
constexpr size_t kMaxKernels = 64;  // compiled patterns kept per handle
constexpr int kMaxCompiles = 4;     // concurrent compiles per handle

struct Entry {
    std::atomic<int> state{0};  // 0 not started, 1 compiling, 2 ready, -1 failed
    uint64_t seen = 0;          // stripes decoded with this pattern and G
    hipModule_t mod = nullptr;
    DecJitKernel k{};
    std::string err;
};
}  // namespace

struct DecJit {
    std::mutex mu;
    std::condition_variable cv;
    int mode = 1;                 // 0 off, 1 async, 2 sync
    uint64_t min_stripes = 1024;  // ~1 GB of 1 MB stripes before a pattern is compiled
    int device = 0;
    int running = 0;              // compiles in flight
    int holders = 0;              // status readers inside dec_jit_counts (dec_jit_hold)
    bool closing = false;         // dec_jit_free: queued compiles give up, waiters return
    std::map<uint64_t, std::unique_ptr<Entry>> ents;
    std::vector<std::thread> threads;
};

DecJit *dec_jit_new(int device) {
    DecJit *j = new DecJit();
    j->device = device;
    if (const char *e = tec_knob("TEC_DEC_JIT")) {
        j->mode = !strcmp(e, "off") || !strcmp(e, "0") ? 0 : !strcmp(e, "sync") ? 2 : 1;
    }
    if (const char *e = tec_knob("TEC_DEC_JIT_MIN")) j->min_stripes = strtoull(e, nullptr, 10);
    return j;
}

// Joins the compile threads and unloads the modules; the caller has drained every stream that
// may run them, on the handle's device.
void dec_jit_free(DecJit *j) {
    if (!j) return;
    {
        std::unique_lock<std::mutex> g(j->mu);
        j->closing = true;  // queued compiles give up without compiling
        j->cv.notify_all();
        j->cv.wait(g, [&] { return j->holders == 0; });
    }
    for (auto &t : j->threads) t.join();  // at most kMaxCompiles were compiling
    for (auto &kv : j->ents)
        if (kv.second->mod) (void)hipModuleUnload(kv.second->mod);
    delete j;
}

void dec_jit_set(DecJit *j, int mode, uint64_t min_stripes) {
    std::lock_guard<std::mutex> g(j->mu);
    j->mode = mode;
    j->min_stripes = min_stripes;
}

void dec_jit_hold(DecJit *j) {
    std::lock_guard<std::mutex> g(j->mu);
    j->holders++;
}

void dec_jit_unhold(DecJit *j) {
    std::lock_guard<std::mutex> g(j->mu);
    j->holders--;
    j->cv.notify_all();
}

void dec_jit_counts(DecJit *j, uint32_t timeout_ms, uint32_t *ready, uint32_t *pending, uint32_t *failed) {
    std::unique_lock<std::mutex> g(j->mu);
    auto busy = [&] {
        for (auto &kv : j->ents)
            if (kv.second->state.load() == 1) return true;
        return false;
    };
    if (timeout_ms)
        j->cv.wait_for(g, std::chrono::milliseconds(timeout_ms), [&] { return j->closing || !busy(); });
    uint32_t r = 0, p = 0, f = 0;
    for (auto &kv : j->ents) {
        const int s = kv.second->state.load();
        r += s == 2, p += s == 1, f += s == -1;
    }
    if (ready) *ready = r;
    if (pending) *pending = p;
    if (failed) *failed = f;
}

DecJitGeom dec_jit_geom(uint32_t sc) {
    // 8-column lanes (TEC_DEC_JIT_WB=8) halve the memory instructions per byte but measured the
    // same on one box (4.71-4.72 vs 4.67-4.71 ms per 1024 x 4 MiB worst-case step) and compile
    // twice as long, so 4-column lanes are the default
    static const uint32_t wb_env = [] {
        const char *e = tec_knob("TEC_DEC_JIT_WB");
        return e && !strcmp(e, "8") ? 8u : 4u;
    }();
    DecJitGeom g{};
    g.wb = sc >= 64u ? wb_env : 4u;
    g.wps = (sc + g.wb - 1) / g.wb;
    const uint32_t groups = (g.wps + 63) / 64;
    // waves per workgroup (TEC_DEC_JIT_G, measurement knob): with words kept in load order, 2
    // measured 4.79-4.82 ms against 4.94-5.03 for 6 and 4.95-4.96 for 3 (1024 x 4 MiB, 13 erasures)
    static const uint32_t g_env = [] {
        const char *e = tec_knob("TEC_DEC_JIT_G");
        const int v = e ? atoi(e) : 2;
        return (uint32_t)(v >= 1 && v <= 6 ? v : 2);
    }();
    g.G = std::min(std::min(groups, 6u), g_env);
    g.wgs = (groups + g.G - 1) / g.G;
    return g;
}

static void compile(DecJit *j, Entry *E, std::string src, size_t lds, uint32_t nscratch, uint32_t wb, bool queued) {
    if (queued) {  // a worker: at most kMaxCompiles compile at once
        std::unique_lock<std::mutex> g(j->mu);
        j->cv.wait(g, [&] { return j->closing || j->running < kMaxCompiles; });
        if (j->closing) {  // the handle is being freed or re-bound
            E->err = "cancelled";
            E->state.store(-1);
            j->cv.notify_all();
            return;
        }
        j->running++;
    }
    std::string err;
    hiprtcProgram prog = nullptr;
    const char *hdrs[] = {kDecFixedHeader};
    const char *names[] = {"dec_fixed.hpp"};
    hipModule_t mod = nullptr;
    hipFunction_t fn = nullptr;
    if (hiprtcCreateProgram(&prog, src.c_str(), "tec_dec_fixed.hip", 1, hdrs, names) != HIPRTC_SUCCESS) {
        err = "hiprtcCreateProgram failed";
    } else {
        // TEC_DEC_JIT_SCHED (measurement): the backend scheduling strategy, e.g. max-ilp
        static const std::string sched = [] {
            const char *e = tec_knob("TEC_DEC_JIT_SCHED");
            return e ? std::string("-amdgpu-sched-strategy=") + e : std::string();
        }();
        const char *opts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17", "-mllvm", sched.c_str()};
        if (hiprtcCompileProgram(prog, sched.empty() ? 3 : 5, opts) != HIPRTC_SUCCESS) {
            size_t n = 0;
            hiprtcGetProgramLogSize(prog, &n);
            std::string log(n, '\0');
            if (n) hiprtcGetProgramLog(prog, log.data());
            err = "hipRTC: " + log.substr(0, 512);
        } else {
            size_t n = 0;
            hiprtcGetCodeSize(prog, &n);
            std::vector<char> code(n);
            hiprtcGetCode(prog, code.data());
            int cur = 0;
            (void)hipGetDevice(&cur);
            if (hipSetDevice(j->device) != hipSuccess || hipModuleLoadData(&mod, code.data()) != hipSuccess ||
                hipModuleGetFunction(&fn, mod, kDecFixedKernel) != hipSuccess)
                err = "module load failed";
            (void)hipSetDevice(cur);
        }
        hiprtcDestroyProgram(&prog);
    }
    std::lock_guard<std::mutex> g(j->mu);
    if (err.empty()) {
        E->mod = mod;
        E->k.fn = fn;
        E->k.lds = lds;
        E->k.nscratch = nscratch;
        E->k.wb = wb;
        E->state.store(2);
    } else {
        if (mod) (void)hipModuleUnload(mod);
        E->err = err;
        E->state.store(-1);
    }
    j->running--;
    j->cv.notify_all();
}

const DecJitKernel *dec_jit_get(DecJit *j, const ClayHost &h, const GpePattern &P, int orient, int G, int wb, uint64_t stripes) {
    if (!j || P.erased_mask >> 32 || G < 1 || G > 6 || (wb != 4 && wb != 8)) return nullptr;
    const uint64_t key = P.erased_mask | (uint64_t)G << 32 | (uint64_t)wb << 40;
    std::unique_lock<std::mutex> g(j->mu);
    auto f = j->ents.find(key);
    Entry *E = f == j->ents.end() ? nullptr : f->second.get();
    if (E && E->state.load() == 2) return &E->k;
    if (j->mode == 0 || (E && E->state.load() != 0)) return nullptr;
    if (!E) {
        if (j->ents.size() >= kMaxKernels) return nullptr;
        E = j->ents.emplace(key, std::make_unique<Entry>()).first->second.get();
    }
    E->seen += stripes;
    if (E->seen < j->min_stripes) return nullptr;
    // the pattern's program and matrix, as dec_pattern compiled them
    DecProgHdr H;
    std::vector<DecStep> steps;
    std::vector<int> known, erased;
    Mat Dm;
    static const bool direct = [] {  // TEC_DEC_JIT_OUT=stage: rows staged in LDS, flushed whole (measurement)
        const char *e = tec_knob("TEC_DEC_JIT_OUT");
        return !(e && !strcmp(e, "stage"));
    }();
    static const bool fuse = [] {  // TEC_DEC_JIT_FUSE=0: no type-1 / in-row pair fusion (measurement)
        const char *e = tec_knob("TEC_DEC_JIT_FUSE");
        return !(e && e[0] == '0');
    }();
    // the fused forms move output rows between steps: direct output only
    if (!h.dec_prog(P, orient, H, steps, -1, 0, direct && fuse) || !h.decoder(P.erased_mask, known, erased, Dm) ||
        known.size() != P.nknown || erased.size() != P.nerased) {
        E->state.store(-1);
        return nullptr;
    }
    uint8_t D[kGpeMaxErased][kGpeMaxKnown] = {};
    for (size_t e = 0; e < erased.size(); e++)
        for (size_t k = 0; k < known.size(); k++) D[e][k] = Dm.v[e][k];
    if (!direct) wb = 4;  // the staged form (measurement only) has 4-column lanes
    if (direct && fuse) dec_prog_fuse_type1(P, steps);
    std::string src = dec_fixed_source(P, D, H, steps, G, kPft.t_u[0], direct, wb);
    const size_t lds = dec_fixed_lds(H, G, direct, wb);
    E->state.store(1);
    if (j->mode == 2) {
        j->running++;
        g.unlock();
        compile(j, E, std::move(src), lds, H.nscratch, (uint32_t)wb, false);
        return E->state.load() == 2 ? &E->k : nullptr;
    }
    j->threads.emplace_back(compile, j, E, std::move(src), lds, H.nscratch, (uint32_t)wb, true);
    return nullptr;
}

hipError_t launch_dec_fixed(const DecJitKernel &k, const dfix_args &a, uint32_t G, hipStream_t s) {
    const uint64_t blocks = (uint64_t)a.njobs * a.wgs_per_stripe;
    if (blocks == 0) return hipSuccess;
    if (blocks > 0x7fffffffull) return hipErrorInvalidValue;
    dfix_args arg = a;
    void *params[] = {&arg};
    return hipModuleLaunchKernel(k.fn, (uint32_t)blocks, 1, 1, G * 64, 1, 1, (uint32_t)k.lds, s, params, nullptr);
}

}  // namespace tec
