// Host memcpy fan-out of the per-call entry points (engine.cpp).  Host-only.
#pragma once
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

namespace tec {

// Host memcpy fan-out for the per-call entry points: a few persistent threads (plus the caller)
// copy a list of segments, big segments split into 64 KiB pieces.  Used to gather a call's
// scattered host buffers (Slicer::repair's d helper buffers, repair.rs:340-354) into one pinned
// staging buffer -- one H2D instead of one driver-staged copy per helper -- and to scatter the
// result back into the caller's (pageable) buffer.
//
// Every run() is its own Job (pieces, claim counter, done counter), shared with the workers by
// shared_ptr.  A worker that wakes late, or is preempted inside a job, only ever touches the job it
// picked up: it cannot see the next job's piece list being rebuilt, and its counters cannot leak
// into the next job's (a shared piece vector and done counter did both).  run()
// returns once its job's pieces are all copied; a late worker then finds no piece left to claim.
// No HIP here: tests/test_copy_pool.py builds this header into a ThreadSanitizer stress program.
class CopyPool {
  public:
    struct Seg {
        void *dst;
        const void *src;
        size_t len;
    };
    // `nworkers` persistent threads besides the caller (0: the caller copies alone).  A pool is
    // meant to live for the process: its threads are detached and never stopped.
    explicit CopyPool(int nworkers) {
        for (int i = 0; i < nworkers; i++)
            workers_.emplace_back([this] {
                uint64_t seen = 0;
                for (;;) {
                    std::shared_ptr<Job> job;
                    {
                        std::unique_lock<std::mutex> g(m_);
                        cv_.wait(g, [&] { return gen_ != seen; });
                        seen = gen_;
                        job = job_;
                    }
                    if (job) work(*job);
                }
            });
        for (auto &t : workers_) t.detach();
    }
    void run(const std::vector<Seg> &segs) {
        constexpr size_t kPiece = 64 << 10;
        auto job = std::make_shared<Job>();
        size_t total = 0;
        for (const Seg &g : segs)
            for (size_t o = 0; o < g.len; o += kPiece) {
                const size_t l = std::min(kPiece, g.len - o);
                job->pieces.push_back({static_cast<uint8_t *>(g.dst) + o, static_cast<const uint8_t *>(g.src) + o, l});
                total += l;
            }
        if (job->pieces.size() <= 1 || total < (128u << 10) || workers_.empty()) {  // not worth waking anyone
            for (const Seg &g : job->pieces) memcpy(g.dst, g.src, g.len);
            return;
        }
        std::lock_guard<std::mutex> one(call_mu_);  // one job at a time per pool
        {
            std::lock_guard<std::mutex> g(m_);
            job_ = job;
            gen_++;
        }
        cv_.notify_all();
        work(*job);
        std::unique_lock<std::mutex> g(job->m);
        job->cv.wait(g, [&] { return job->done.load() == job->pieces.size(); });
        g.unlock();
        std::lock_guard<std::mutex> g2(m_);
        if (job_ == job) job_.reset();
    }
    size_t workers() const { return workers_.size(); }

  private:
    struct Job {
        std::vector<Seg> pieces;
        std::atomic<size_t> next{0}, done{0};
        std::mutex m;
        std::condition_variable cv;
    };
    static void work(Job &job) {
        const size_t n = job.pieces.size();
        for (;;) {
            const size_t i = job.next.fetch_add(1);
            if (i >= n) return;
            memcpy(job.pieces[i].dst, job.pieces[i].src, job.pieces[i].len);
            if (job.done.fetch_add(1) + 1 == n) {
                std::lock_guard<std::mutex> g(job.m);
                job.cv.notify_all();
            }
        }
    }
    std::mutex call_mu_, m_;
    std::condition_variable cv_;
    std::shared_ptr<Job> job_;
    uint64_t gen_ = 0;
    std::vector<std::thread> workers_;
};

}  // namespace tec
