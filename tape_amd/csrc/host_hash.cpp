// host_hash.cpp -- SHA-256 leaf hashing on host cores and its worker pool (host_hash.hpp).
#include "host_hash.hpp"

#include <sched.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>

#include "sha256.hpp"

#if defined(__x86_64__)
#include <immintrin.h>
#endif

namespace tec {
namespace hh {

namespace {

alignas(16) const uint32_t kKTab[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

// Portable path: the same compression the device kernels use.
void blocks_portable(uint32_t st[8], const uint8_t *p, size_t nblocks) {
    for (size_t b = 0; b < nblocks; b++, p += 64) {
        uint32_t w[16];
        for (int i = 0; i < 16; i++)
            w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 | (uint32_t)p[4 * i + 2] << 8 | p[4 * i + 3];
        sha::compress(st, w);
    }
}

#if defined(__x86_64__)
// SHA extensions: the state as (A,B,E,F) / (C,D,G,H), two rounds per sha256rnds2, the message
// schedule four words at a time (sha256msg1 adds sigma0(W[t-15]) to W[t-16], msg2 adds sigma1).
// L independent messages of the same block count are interleaved round by round: one message's
// rounds are a chain of dependent sha256rnds2, so a lone message leaves the SHA unit idle for
// most of each instruction's latency (r04: 1.4x at L=2, 1.6x at L=4 on this container's Xeon;
// the pool measures which L is fastest on its own host, Pool::Pool).
template <int L>
__attribute__((target("sha,sse4.1,ssse3"))) void blocks_shaext(uint32_t *const *st, const uint8_t *const *src,
                                                               size_t nblocks) {
    const __m128i bswap = _mm_set_epi64x(0x0c0d0e0f08090a0bll, 0x0405060700010203ll);
    __m128i s0[L], s1[L];
    const uint8_t *p[L];
    for (int l = 0; l < L; l++) {
        __m128i t = _mm_loadu_si128(reinterpret_cast<const __m128i *>(st[l]));   // A B C D
        __m128i u = _mm_loadu_si128(reinterpret_cast<const __m128i *>(st[l] + 4));  // E F G H
        t = _mm_shuffle_epi32(t, 0xB1);                                            // C D A B
        u = _mm_shuffle_epi32(u, 0x1B);                                            // H G F E
        s0[l] = _mm_alignr_epi8(t, u, 8);                                          // A B E F
        s1[l] = _mm_blend_epi16(u, t, 0xF0);                                       // C D G H
        p[l] = src[l];
    }
    for (size_t b = 0; b < nblocks; b++) {
        __m128i save0[L], save1[L], w[L][4];
        for (int l = 0; l < L; l++) save0[l] = s0[l], save1[l] = s1[l];
#pragma GCC unroll 16
        for (int g = 0; g < 16; g++) {
            const __m128i k = _mm_load_si128(reinterpret_cast<const __m128i *>(kKTab + 4 * g));
            for (int l = 0; l < L; l++) {
                if (g < 4) {
                    w[l][g] = _mm_shuffle_epi8(_mm_loadu_si128(reinterpret_cast<const __m128i *>(p[l] + 16 * g)), bswap);
                } else {
                    __m128i x = _mm_sha256msg1_epu32(w[l][g & 3], w[l][(g + 1) & 3]);                 // W[t-16] + s0(W[t-15])
                    x = _mm_add_epi32(x, _mm_alignr_epi8(w[l][(g + 3) & 3], w[l][(g + 2) & 3], 4));  // + W[t-7]
                    w[l][g & 3] = _mm_sha256msg2_epu32(x, w[l][(g + 3) & 3]);                         // + s1(W[t-2])
                }
                __m128i m = _mm_add_epi32(w[l][g & 3], k);
                s1[l] = _mm_sha256rnds2_epu32(s1[l], s0[l], m);
                m = _mm_shuffle_epi32(m, 0x0E);
                s0[l] = _mm_sha256rnds2_epu32(s0[l], s1[l], m);
            }
        }
        for (int l = 0; l < L; l++) {
            s0[l] = _mm_add_epi32(s0[l], save0[l]);
            s1[l] = _mm_add_epi32(s1[l], save1[l]);
            p[l] += 64;
        }
    }
    for (int l = 0; l < L; l++) {
        __m128i t = _mm_shuffle_epi32(s0[l], 0x1B);  // F E B A
        __m128i u = _mm_shuffle_epi32(s1[l], 0xB1);  // D C H G
        _mm_storeu_si128(reinterpret_cast<__m128i *>(st[l]), _mm_blend_epi16(t, u, 0xF0));  // D C B A
        _mm_storeu_si128(reinterpret_cast<__m128i *>(st[l] + 4), _mm_alignr_epi8(u, t, 8));  // H G F E
    }
}
#endif

bool detect_sha_ext() {
#if defined(__x86_64__)
    __builtin_cpu_init();
    return __builtin_cpu_supports("sha") && __builtin_cpu_supports("sse4.1") && __builtin_cpu_supports("ssse3");
#else
    return false;
#endif
}
const bool g_sha_ext = detect_sha_ext();

// `nblocks` 64-byte blocks of each of `L` messages (L <= kMaxLanes)
void blocks(int L, uint32_t *const *st, const uint8_t *const *p, size_t nblocks) {
#if defined(__x86_64__)
    if (g_sha_ext) {
        switch (L) {
            case 1: return blocks_shaext<1>(st, p, nblocks);
            case 2: return blocks_shaext<2>(st, p, nblocks);
            case 3: return blocks_shaext<3>(st, p, nblocks);
            case 4: return blocks_shaext<4>(st, p, nblocks);
        }
    }
#endif
    for (int l = 0; l < L; l++) blocks_portable(st[l], p[l], nblocks);
}

}  // namespace

bool have_sha_ext() { return g_sha_ext; }

LeafLanes::LeafLanes(int lanes) : L(lanes) {
    for (int l = 0; l < L; l++) {
        sha::init(st[l]);
        memcpy(buf[l], "LEAF", 4);
    }
    have = 4;
}

// Partial blocks are assembled in buf; full blocks are read in place.
void LeafLanes::update(const uint8_t *const *data, size_t n) {
    if (n == 0) return;
    const uint8_t *p[kMaxLanes];
    uint32_t *sp[kMaxLanes];
    for (int l = 0; l < L; l++) p[l] = data[l], sp[l] = st[l];
    len += n;
    if (have) {
        const size_t m = std::min(n, 64 - have);
        for (int l = 0; l < L; l++) memcpy(buf[l] + have, p[l], m), p[l] += m;
        have += m;
        n -= m;
        if (have < 64) return;
        const uint8_t *bp[kMaxLanes];
        for (int l = 0; l < L; l++) bp[l] = buf[l];
        blocks(L, sp, bp, 1);
        have = 0;
    }
    const size_t full = n / 64;
    blocks(L, sp, p, full);
    for (int l = 0; l < L; l++) memcpy(buf[l], p[l] + full * 64, n - full * 64);
    have = n - full * 64;
}

void LeafLanes::final(uint8_t *const *out) {
    const uint64_t bits = (len + 4) * 8;
    const size_t tot = have + 1 + 8 <= 64 ? 64 : 128;
    uint8_t tail[kMaxLanes][128];
    const uint8_t *bp[kMaxLanes];
    uint32_t *sp[kMaxLanes];
    for (int l = 0; l < L; l++) {
        memcpy(tail[l], buf[l], have);
        tail[l][have] = 0x80;
        memset(tail[l] + have + 1, 0, tot - 8 - have - 1);
        for (int i = 0; i < 8; i++) tail[l][tot - 8 + i] = (uint8_t)(bits >> (56 - 8 * i));
        bp[l] = tail[l];
        sp[l] = st[l];
    }
    blocks(L, sp, bp, tot / 64);
    for (int l = 0; l < L; l++)
        for (int i = 0; i < 8; i++) {
            out[l][4 * i] = (uint8_t)(st[l][i] >> 24);
            out[l][4 * i + 1] = (uint8_t)(st[l][i] >> 16);
            out[l][4 * i + 2] = (uint8_t)(st[l][i] >> 8);
            out[l][4 * i + 3] = (uint8_t)st[l][i];
        }
}

void hash_leaves(int L, const uint8_t *const *data, size_t len, uint8_t *const *out) {
    LeafLanes h(L);
    h.update(data, len);
    h.final(out);
}

void hash_leaf(const uint8_t *data, size_t len, uint8_t out[32]) { hash_leaves(1, &data, len, &out); }

int default_threads() {
    cpu_set_t cs;
    int n = 0;
    if (sched_getaffinity(0, sizeof(cs), &cs) == 0) n = CPU_COUNT(&cs);
    if (n <= 0) n = (int)std::thread::hardware_concurrency();
    if (n <= 0) n = 1;
    return n < 16 ? n : 16;
}

Pool &Pool::get() {
    static Pool *p = new Pool();  // never destroyed: workers may outlive static destructors' order
    return *p;
}

Pool::Pool() {
    // calibrate the lane count and the per-thread rate the device / host choice uses
    // (host_hash_wins): 1 MiB per lane at L = 1..4 lanes, the L sweep repeated 4 times (clock
    // ramp, noisy neighbours) keeping each L's best; a larger L is taken only when it is >= 5%
    // faster (a task of L slices takes longer, and a window waits for its last task)
    const size_t len = (size_t)1 << 20;
    std::vector<uint8_t> buf(len * kMaxLanes, 0x5a);
    uint8_t res[kMaxLanes][32];
    const uint8_t *src[kMaxLanes];
    uint8_t *out[kMaxLanes];
    for (int l = 0; l < kMaxLanes; l++) src[l] = buf.data() + l * len, out[l] = res[l];
    hash_leaves(kMaxLanes, src, len, out);  // warm up
    double best[kMaxLanes] = {};
    for (int rep = 0; rep < 4; rep++)
        for (int L = 1; L <= kMaxLanes; L++) {
            const auto t0 = std::chrono::steady_clock::now();
            hash_leaves(L, src, len, out);
            const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            if (dt > 0) best[L - 1] = std::max(best[L - 1], (double)(L * len) / dt);
        }
    for (int L = 1; L <= kMaxLanes; L++) {
        lane_rate_[L - 1] = std::min(16e9, std::max(1e8, best[L - 1]));
        if (L == 1 || lane_rate_[L - 1] >= 1.05 * rate_) {
            rate_ = lane_rate_[L - 1];
            lanes_ = L;
        }
    }
    // measurement option (TEC_DEBUG_KNOBS=1 TEC_HOST_HASH_LANES=L, kernels.hpp tec_knob): force L
    const char *on = getenv("TEC_DEBUG_KNOBS");
    if (on && !strcmp(on, "1"))
        if (const char *v = getenv("TEC_HOST_HASH_LANES")) {
            const int L = atoi(v);
            if (L >= 1 && L <= kMaxLanes) lanes_ = L, rate_ = lane_rate_[L - 1];
        }
    start(default_threads());
}
Pool::~Pool() { stop(); }

void Pool::start(int n) {
    quit_ = false;
    nthreads_ = n;
    for (int i = 0; i < n; i++)
        workers_.emplace_back([this] {
            for (;;) {
                std::function<void()> f;
                {
                    std::unique_lock<std::mutex> g(m_);
                    cv_work_.wait(g, [&] { return quit_ || !work_.empty(); });
                    if (work_.empty()) return;
                    f = std::move(work_.front());
                    work_.pop_front();
                    busy_++;
                }
                f();
                {
                    std::lock_guard<std::mutex> g(m_);
                    busy_--;
                }
                cv_gate_.notify_all();
            }
        });
    gate_ = std::thread([this] {
        for (;;) {
            Gate gt;
            {
                std::unique_lock<std::mutex> g(m_);
                cv_gate_.wait(g, [&] { return quit_ || !gates_.empty(); });
                if (gates_.empty()) return;
                gt = std::move(gates_.front());
            }
            if (gt.ev) {
                (void)hipSetDevice(gt.device);
                (void)hipEventSynchronize(gt.ev);
                (void)hipEventDestroy(gt.ev);
            }
            {
                std::lock_guard<std::mutex> g(m_);
                gates_.pop_front();
                for (auto &f : gt.tasks) work_.push_back(std::move(f));
            }
            cv_work_.notify_all();
        }
    });
}

void Pool::stop() {
    {
        std::lock_guard<std::mutex> g(m_);
        quit_ = true;
    }
    cv_work_.notify_all();
    cv_gate_.notify_all();
    if (gate_.joinable()) gate_.join();
    for (auto &t : workers_)
        if (t.joinable()) t.join();
    workers_.clear();
}

int Pool::set_threads(int n) {
    if (n <= 0) n = default_threads();
    {
        // resize only an idle pool (the stream writers hold no queued work), and hold new
        // submissions until the new workers run: a gate released between stop() and start()
        // would queue tasks no worker takes
        std::unique_lock<std::mutex> g(m_);
        cv_gate_.wait(g, [&] { return !resizing_ && gates_.empty() && work_.empty() && busy_ == 0; });
        resizing_ = true;
    }
    stop();
    {
        std::lock_guard<std::mutex> g(m_);
        start(n);
        resizing_ = false;
    }
    cv_gate_.notify_all();
    return 0;
}

void Pool::submit_after(hipEvent_t ev, int device, std::vector<std::function<void()>> tasks) {
    {
        std::unique_lock<std::mutex> g(m_);
        cv_gate_.wait(g, [&] { return !resizing_; });
        gates_.push_back(Gate{ev, device, std::move(tasks)});
    }
    cv_gate_.notify_all();
}

}  // namespace hh
}  // namespace tec
