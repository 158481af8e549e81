// Stress program for tape_amd/csrc/copy_pool.hpp: many back-to-back run()
// calls of different sizes from several threads on one pool, every destination byte checked after
// each call.  Built with -fsanitize=thread (and separately -fsanitize=address) by
// tests/test_copy_pool.py; exits non-zero on a wrong byte, prints "ok <calls>" otherwise.
#include <cstdio>
#include <cstdlib>
#include <random>
#include "../../tape_amd/csrc/copy_pool.hpp"

int main(int argc, char **argv) {
    const int callers = argc > 1 ? atoi(argv[1]) : 2;
    const int iters = argc > 2 ? atoi(argv[2]) : 300;
    tec::CopyPool &pool = *new tec::CopyPool(3);  // as in the library: never destroyed
    std::atomic<long> bad{0}, calls{0};
    std::vector<std::thread> th;
    for (int t = 0; t < callers; t++)
        th.emplace_back([&, t] {
            std::mt19937_64 rng(0x5EED + t);
            std::vector<uint8_t> src(3u << 20), dst(3u << 20);
            for (int it = 0; it < iters; it++) {
                // 1-6 segments of 0 .. 600 KiB (some under the fan-out threshold, most above)
                const int nseg = 1 + (int)(rng() % 6);
                std::vector<tec::CopyPool::Seg> segs;
                size_t at = 0;
                const uint8_t tag = (uint8_t)(it * 7 + t);
                for (int s = 0; s < nseg; s++) {
                    const size_t len = rng() % (600u << 10);
                    if (at + len > src.size()) break;
                    for (size_t i = 0; i < len; i++) src[at + i] = (uint8_t)(tag + i * 31 + s);
                    segs.push_back({dst.data() + at, src.data() + at, len});
                    at += len;
                }
                pool.run(segs);
                calls++;
                for (const auto &g : segs)
                    if (memcmp(g.dst, g.src, g.len) != 0) bad++;
            }
        });
    for (auto &x : th) x.join();
    if (bad) {
        printf("FAIL %ld bad segments\n", bad.load());
        return 1;
    }
    printf("ok %ld\n", calls.load());
    return 0;
}
