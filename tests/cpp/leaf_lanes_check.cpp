// Host check of hh::LeafLanes (tape_amd/csrc/host_hash.cpp): SHA-256("LEAF" || slice) fed in
// arbitrary pieces -- as the stream writer's hashing tasks consume a window's D2H row pieces --
// equals the one-shot hash, for 1..4 interleaved lanes, every length around the block edges and
// random piece boundaries.  Built and run by tests/test_host_hash_pieces.py (g++, no GPU).
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <random>
#include <vector>

#include "host_hash.hpp"

using namespace tec::hh;

int main() {
    std::mt19937_64 rng(20261017);
    int bad = 0, cases = 0;
    const size_t lens[] = {0, 1, 3, 59, 60, 61, 63, 64, 65, 123, 124, 125, 127, 128, 129, 1000, 4096, 70001, 1 << 20};
    for (size_t len : lens)
        for (int L = 1; L <= kMaxLanes; L++)
            for (int rep = 0; rep < 6; rep++) {
                std::vector<std::vector<uint8_t>> msg(L, std::vector<uint8_t>(len + 1));
                for (auto &m : msg)
                    for (auto &b : m) b = (uint8_t)rng();
                const uint8_t *src[kMaxLanes];
                uint8_t want[kMaxLanes][32], got[kMaxLanes][32];
                uint8_t *w[kMaxLanes], *g[kMaxLanes];
                for (int l = 0; l < L; l++) src[l] = msg[l].data(), w[l] = want[l], g[l] = got[l];
                for (int l = 0; l < L; l++) hash_leaf(src[l], len, want[l]);
                // pieces: rep 0 = one piece, 1 = 1-byte pieces (short messages), else random cuts
                LeafLanes h(L);
                size_t off = 0;
                while (off < len) {
                    size_t n = len - off;
                    if (rep == 1) n = std::min<size_t>(n, len < 5000 ? 1 : 4093);
                    else if (rep > 1) n = std::min<size_t>(n, 1 + rng() % (rep == 5 ? 200 : 70000));
                    const uint8_t *at[kMaxLanes];
                    for (int l = 0; l < L; l++) at[l] = src[l] + off;
                    h.update(at, n);
                    off += n;
                }
                h.final(g);
                cases++;
                for (int l = 0; l < L; l++)
                    if (memcmp(want[l], got[l], 32)) {
                        bad++;
                        fprintf(stderr, "mismatch len=%zu lanes=%d rep=%d lane=%d\n", len, L, rep, l);
                    }
                // hash_leaves (one-shot, interleaved) against hash_leaf too
                hash_leaves(L, src, len, g);
                for (int l = 0; l < L; l++)
                    if (memcmp(want[l], got[l], 32)) {
                        bad++;
                        fprintf(stderr, "hash_leaves mismatch len=%zu lanes=%d lane=%d\n", len, L, l);
                    }
            }
    printf("%d cases, %d mismatches, sha extensions %d\n", cases, bad, have_sha_ext() ? 1 : 0);
    return bad ? 1 : 0;
}
