// Host check of rs16::mat_image (tape_amd/csrc/rs16.hpp), the lookup image rs16_matrix_kernel
// (rs16.hip) stages: the kernel's reads are emulated here -- per input and nibble position q the
// 8-row pair entries at h * 128 + n * 8 (+ the tail group at NP * 128 + n * 1 / 2 / 4 for odd G), or
// with the VALU tail (tv, rows = 8 h + 1) the pairs only and the per-input bit constants K[b]
// XORed over the set bits of the element -- and compared with the direct product sum_r M[i][r] *
// x[r] over GF(2^16), for random and encode matrices (rs16::encode_matrix against
// rs16::encode_column).  Built and run by tests/test_outer_image.py (g++, no GPU).
#include <stdint.h>
#include <stdio.h>

#include <random>
#include <vector>

#include "rs16.hpp"

using namespace tec::rs16;

// tail_bytes: the odd last group's entry size (2 / 4 / 8 B); narrow entries must still hold every
// row of that group, so 2 B serves one row and 4 B two
static int check(uint32_t k, uint32_t rows, const std::vector<uint16_t> &M, bool tv_req, uint32_t tail_bytes,
                 std::mt19937_64 &rng) {
    const Tables &T = tables();
    const bool tv = tv_req && rows % 8 == 1 && rows > 1;
    const std::vector<uint16_t> img = mat_image(k, rows, M.data(), tv_req, tail_bytes);
    const uint32_t G = (rows + 3) / 4, NP = G / 2;
    const uint32_t TBu = (G % 2 && !tv) ? tail_bytes / 2 : 0, BQ = NP * 128 + 16 * TBu;
    const size_t want_size = (size_t)k * 4 * BQ + (tv ? (size_t)k * 32 : 0);
    if (img.size() != want_size) {
        printf("size k=%u rows=%u tv=%d: %zu != %zu\n", k, rows, tv, img.size(), want_size);
        return 1;
    }
    const uint16_t *kt = img.data() + (size_t)k * 4 * BQ;
    int bad = 0;
    for (int col = 0; col < 64; col++) {
        std::vector<uint16_t> x(k);
        for (auto &v : x) v = col == 0 ? 0xffff : col == 1 ? 0 : (uint16_t)rng();
        std::vector<uint16_t> got(4 * G, 0);
        for (uint32_t r = 0; r < k; r++)
            for (uint32_t q = 0; q < 4; q++) {
                const uint16_t *blk = img.data() + ((size_t)r * 4 + q) * BQ;
                const uint32_t n = (x[r] >> (4 * q)) & 15;
                for (uint32_t h = 0; h < NP; h++)
                    for (uint32_t j = 0; j < 8; j++) got[8 * h + j] ^= blk[h * 128 + n * 8 + j];
                if (G % 2 && !tv)
                    for (uint32_t j = 0; j < TBu; j++) got[8 * NP + j] ^= blk[NP * 128 + n * TBu + j];
            }
        if (tv)
            for (uint32_t r = 0; r < k; r++)
                for (uint32_t b = 0; b < 16; b++)
                    if (x[r] >> b & 1) {
                        const uint16_t lo = kt[((size_t)r * 16 + b) * 2], hi = kt[((size_t)r * 16 + b) * 2 + 1];
                        if (lo != hi) bad++;  // the kernel applies K to both halves of a packed pair
                        got[8 * NP] ^= lo;
                    }
        for (uint32_t i = 0; i < 4 * G; i++) {
            uint16_t want = 0;
            if (i < rows)
                for (uint32_t r = 0; r < k; r++) want ^= T.gmul(M[(size_t)i * k + r], x[r]);
            if (got[i] != want) {
                if (bad < 5) printf("k=%u rows=%u tv=%d col=%d row %u: %04x != %04x\n", k, rows, tv, col, i, got[i], want);
                bad++;
            }
        }
    }
    return bad;
}

int main() {
    std::mt19937_64 rng(20261018);
    int bad = 0, cases = 0;
    const uint32_t ks[] = {1, 2, 5, 16, 17, 20, 31, 32};
    for (uint32_t k : ks)
        for (uint32_t rows = 1; rows <= 64; rows++) {
            if ((size_t)k * ((rows + 3) / 4) * 512 > 80 * 1024) continue;
            std::vector<uint16_t> M((size_t)rows * k);
            for (auto &v : M) v = (uint16_t)rng();
            const uint32_t G = (rows + 3) / 4, t = rows - 8 * (G / 2);
            const uint32_t narrow = (G % 2 && t <= 2) ? 2 * t : 8;  // kernels.hpp rs16_mat_tail_bytes
            for (int tv = 0; tv < 2; tv++, cases++) bad += check(k, rows, M, tv, 8, rng);
            if (narrow != 8) cases++, bad += check(k, rows, M, false, narrow, rng);
        }
    // encode matrices: column r of E = the encode of unit vector e_r
    const uint32_t shapes[][2] = {{17, 33}, {16, 48}, {20, 40}, {5, 69}, {31, 40}, {17, 9}, {3, 17}};
    for (auto &sh : shapes) {
        const uint32_t k = sh[0], m = sh[1];
        if (use_high_rate(k, m) < 0) continue;
        std::vector<uint16_t> E;
        encode_matrix(k, m, E);
        std::vector<uint16_t> o(k), rec(m);
        for (int col = 0; col < 8; col++) {
            for (auto &v : o) v = (uint16_t)rng();
            encode_column(k, m, o.data(), rec.data());
            for (uint32_t j = 0; j < m; j++) {
                uint16_t w = 0;
                for (uint32_t r = 0; r < k; r++) w ^= tables().gmul(E[(size_t)j * k + r], o[r]);
                if (w != rec[j]) bad++;
            }
        }
        if ((size_t)k * ((m + 3) / 4) * 512 <= 80 * 1024)
            for (int tv = 0; tv < 2; tv++, cases++) bad += check(k, m, E, tv, 8, rng);
        {
            const uint32_t G = (m + 3) / 4, t = m - 8 * (G / 2);
            if (G % 2 && t <= 2 && (size_t)k * ((m + 3) / 4) * 512 <= 80 * 1024) cases++, bad += check(k, m, E, false, 2 * t, rng);
        }
    }
    printf("%d cases, %d mismatches\n", cases, bad);
    return bad ? 1 : 0;
}
