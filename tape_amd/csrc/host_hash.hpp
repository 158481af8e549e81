// host_hash.hpp -- leaf hashing on host cores, for the stream shapes the device cannot hash well.
//
// The SDK's stream writer cuts a stream into MAX_TRACK_SIZE = 64 MiB chunks
// (sdk/src/stream/manifest.rs:22, write.rs:219) and keeps at most MAX_ENCODE_WORKERS = 4 chunk
// encodes in flight (write.rs:54-57, 332-362); each chunk is one encode_with_proofs, whose 20
// leaf hashes SHA-256("LEAF" || slice) are hashed on the CPU (sdk/src/codec/encoder.rs:220-234).
// SHA-256 is sequential within a message, so the device hashes one slice per lane: a 9.7 MB slice
// of a 64 MiB chunk takes ~0.4 s on one lane whatever the batch, while a host core with the SHA
// extensions hashes it in a few ms.  The writer therefore hashes a group on the device only when
// the group has enough slice streams to beat the host pool (engine.cpp `host_hash_wins`), and
// otherwise hashes the slices here, from the host output buffer, as soon as their D2H copy has
// landed.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

namespace tec {
namespace hh {

// SHA-256("LEAF" || data) (lib/crypto/src/merkle/tree.rs:53-56): x86 SHA extensions when the CPU
// has them, the portable compression (sha256.hpp) otherwise.
void hash_leaf(const uint8_t *data, size_t len, uint8_t out[32]);
// The same for L <= kMaxLanes messages of one length, interleaved round by round on one thread.
constexpr int kMaxLanes = 4;
void hash_leaves(int L, const uint8_t *const *data, size_t len, uint8_t *const *out);
// Incremental form: the messages arrive in pieces (the same length for every lane per update),
// e.g. as a window's D2H row pieces land (engine.cpp group_close_host).
struct LeafLanes {
    explicit LeafLanes(int lanes);
    void update(const uint8_t *const *data, size_t n);
    void final(uint8_t *const *out);
    int L;
    uint32_t st[kMaxLanes][8];
    uint8_t buf[kMaxLanes][64];
    size_t have = 0;   // bytes in buf
    uint64_t len = 0;  // message bytes so far ("LEAF" excluded)
};
bool have_sha_ext();

// A set of tasks whose completion a ticket waits for.
struct Job {
    std::mutex m;
    std::condition_variable cv;
    int64_t left = 0;
    int rc = 0;
    void add(int64_t n) {
        std::lock_guard<std::mutex> g(m);
        left += n;
    }
    void done(int r = 0) {
        std::lock_guard<std::mutex> g(m);
        if (r && !rc) rc = r;
        if (--left == 0) cv.notify_all();
    }
    int wait() {
        std::unique_lock<std::mutex> g(m);
        cv.wait(g, [&] { return left <= 0; });
        return rc;
    }
};

// Worker pool: `threads` hashing workers plus one gate thread that waits (in submission order)
// for the device event a batch of tasks depends on and then releases the batch to the workers.
class Pool {
  public:
    static Pool &get();
    // default: min(16, CPUs this process may run on) -- 16 is a GPU's host share on the pool
    // this runs on; te_set_host_hash_threads changes it (idle pool only)
    int threads() const { return nthreads_; }
    // one thread's SHA-256 rate (bytes/s) at lanes() interleaved messages, measured once on this
    // host at startup; lane_rate(L) the rate measured at L lanes
    double thread_rate() const { return rate_; }
    int lanes() const { return lanes_; }
    double lane_rate(int L) const { return L >= 1 && L <= kMaxLanes ? lane_rate_[L - 1] : 0.0; }
    int set_threads(int n);
    // run `tasks` once `ev` (on `device`, may be null) has completed; the pool destroys `ev`
    void submit_after(hipEvent_t ev, int device, std::vector<std::function<void()>> tasks);
    ~Pool();

  private:
    Pool();
    void start(int n);
    void stop();
    struct Gate {
        hipEvent_t ev;
        int device;
        std::vector<std::function<void()>> tasks;
    };
    std::mutex m_;
    std::condition_variable cv_work_, cv_gate_;
    std::deque<std::function<void()>> work_;
    std::deque<Gate> gates_;
    std::vector<std::thread> workers_;
    std::thread gate_;
    bool quit_ = false;
    bool resizing_ = false;  // set_threads in progress: submit_after waits (no task may land between stop and start)
    int nthreads_ = 0;
    int busy_ = 0;
    double rate_ = 1.5e9;
    int lanes_ = 1;
    double lane_rate_[kMaxLanes] = {};
};

int default_threads();

}  // namespace hh
}  // namespace tec
