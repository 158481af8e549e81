// host_hash.cpp -- SHA-256 leaf hashing on host cores and its worker pool (host_hash.hpp).
#include "host_hash.hpp"

#include <sched.h>
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
__attribute__((target("sha,sse4.1,ssse3"))) void blocks_shaext(uint32_t st[8], const uint8_t *p, size_t nblocks) {
    const __m128i bswap = _mm_set_epi64x(0x0c0d0e0f08090a0bll, 0x0405060700010203ll);
    __m128i t = _mm_loadu_si128(reinterpret_cast<const __m128i *>(st));      // A B C D
    __m128i s1 = _mm_loadu_si128(reinterpret_cast<const __m128i *>(st + 4)); // E F G H
    t = _mm_shuffle_epi32(t, 0xB1);                                          // C D A B
    s1 = _mm_shuffle_epi32(s1, 0x1B);                                        // H G F E
    __m128i s0 = _mm_alignr_epi8(t, s1, 8);                                  // A B E F
    s1 = _mm_blend_epi16(s1, t, 0xF0);                                       // C D G H
    for (size_t b = 0; b < nblocks; b++, p += 64) {
        const __m128i save0 = s0, save1 = s1;
        __m128i w[4];
#pragma GCC unroll 16
        for (int g = 0; g < 16; g++) {
            if (g < 4) {
                w[g] = _mm_shuffle_epi8(_mm_loadu_si128(reinterpret_cast<const __m128i *>(p + 16 * g)), bswap);
            } else {
                __m128i x = _mm_sha256msg1_epu32(w[g & 3], w[(g + 1) & 3]);              // W[t-16] + s0(W[t-15])
                x = _mm_add_epi32(x, _mm_alignr_epi8(w[(g + 3) & 3], w[(g + 2) & 3], 4));  // + W[t-7]
                w[g & 3] = _mm_sha256msg2_epu32(x, w[(g + 3) & 3]);                        // + s1(W[t-2])
            }
            __m128i m = _mm_add_epi32(w[g & 3], _mm_load_si128(reinterpret_cast<const __m128i *>(kKTab + 4 * g)));
            s1 = _mm_sha256rnds2_epu32(s1, s0, m);
            m = _mm_shuffle_epi32(m, 0x0E);
            s0 = _mm_sha256rnds2_epu32(s0, s1, m);
        }
        s0 = _mm_add_epi32(s0, save0);
        s1 = _mm_add_epi32(s1, save1);
    }
    t = _mm_shuffle_epi32(s0, 0x1B);          // F E B A
    s1 = _mm_shuffle_epi32(s1, 0xB1);         // D C H G
    s0 = _mm_blend_epi16(t, s1, 0xF0);        // D C B A
    s1 = _mm_alignr_epi8(s1, t, 8);           // H G F E
    _mm_storeu_si128(reinterpret_cast<__m128i *>(st), s0);
    _mm_storeu_si128(reinterpret_cast<__m128i *>(st + 4), s1);
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

void blocks(uint32_t st[8], const uint8_t *p, size_t nblocks) {
#if defined(__x86_64__)
    if (g_sha_ext) return blocks_shaext(st, p, nblocks);
#endif
    blocks_portable(st, p, nblocks);
}

}  // namespace

bool have_sha_ext() { return g_sha_ext; }

void hash_leaf(const uint8_t *data, size_t len, uint8_t out[32]) {
    uint32_t st[8];
    sha::init(st);
    // "LEAF" is the first 4 message bytes: block 0 is assembled, later full blocks are read in place
    uint8_t b[128];
    memcpy(b, "LEAF", 4);
    const size_t first = len < 60 ? len : 60;
    if (first) memcpy(b + 4, data, first);
    size_t have = 4 + first, done = first;
    if (have == 64) {
        blocks(st, b, 1);
        have = 0;
        const size_t full = (len - done) / 64;
        blocks(st, data + done, full);
        done += full * 64;
        memcpy(b, data + done, len - done);
        have = len - done;
    }
    const uint64_t bits = (uint64_t)(len + 4) * 8;
    b[have++] = 0x80;
    const size_t tot = have + 8 <= 64 ? 64 : 128;
    memset(b + have, 0, tot - 8 - have);
    for (int i = 0; i < 8; i++) b[tot - 8 + i] = (uint8_t)(bits >> (56 - 8 * i));
    blocks(st, b, tot / 64);
    for (int i = 0; i < 8; i++) {
        out[4 * i] = (uint8_t)(st[i] >> 24);
        out[4 * i + 1] = (uint8_t)(st[i] >> 16);
        out[4 * i + 2] = (uint8_t)(st[i] >> 8);
        out[4 * i + 3] = (uint8_t)st[i];
    }
}

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
    // calibrate the per-thread rate the device / host choice uses (host_hash_wins): hash 4 MiB
    std::vector<uint8_t> buf((size_t)4 << 20, 0x5a);
    uint8_t out[32];
    hash_leaf(buf.data(), 4096, out);  // warm up
    const auto t0 = std::chrono::steady_clock::now();
    hash_leaf(buf.data(), buf.size(), out);
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (dt > 0) rate_ = std::min(8e9, std::max(1e8, (double)buf.size() / dt));
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
        // resize only an idle pool (the stream writers hold no queued work)
        std::unique_lock<std::mutex> g(m_);
        cv_gate_.wait(g, [&] { return gates_.empty() && work_.empty() && busy_ == 0; });
    }
    stop();
    start(n);
    return 0;
}

void Pool::submit_after(hipEvent_t ev, int device, std::vector<std::function<void()>> tasks) {
    {
        std::lock_guard<std::mutex> g(m_);
        gates_.push_back(Gate{ev, device, std::move(tasks)});
    }
    cv_gate_.notify_all();
}

}  // namespace hh
}  // namespace tec
