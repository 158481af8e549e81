/* rs16_oracle.c -- TEST INFRASTRUCTURE ONLY (CPU restatement; never linked into libtapeec).
 *
 * Reed-Solomon over GF(2^16) as the third-party crate reed-solomon-simd 3.1.0 computes it
 * (Cargo.lock of the reference; used by lib/slicer/src/outer.rs:19-197 OuterCoder and
 * lib/slicer/src/reed_solomon.rs:17-181 ReedSolomonCoder).  The crate is absent from
 * /root/reference and there is no network, so this restates its published algorithm -- the
 * Leopard-RS construction (Lin, Chung, Han, "Novel polynomial basis and its application to
 * Reed-Solomon erasure codes", FOCS 2014; C. Taylor's leopard codec, which the crate ports):
 *   * field: GF(2^16), LFSR polynomial 0x1002D, logarithms taken in the Cantor basis below;
 *   * shard bytes: every 64-byte block holds 32 field elements, element i = byte i (low) |
 *     byte 32 + i (high) << 8;
 *   * encode: the additive FFT (LCH basis) with the skew factors of the basis; "high rate" when
 *     next_pow2(recovery) <= next_pow2(original) (chunks of originals IFFT'd and XOR-folded,
 *     one FFT), "low rate" otherwise (one IFFT of the originals, one FFT per recovery chunk).
 * PARITY UNPINNED: no reference file holds reed-solomon-simd output bytes.  What the
 * reference's tests pin (outer.rs:206-391: chunk counts and sizes, systematic data chunks,
 * decode from any k chunks incl. parity-only and mixed, errors) is checked in tests/.
 *
 * Decode here is generic linear algebra (the generator matrix of the code above, inverted on the
 * received rows): any correct MDS decoder returns the same bytes, so it needs no algorithmic
 * match with the crate's FFT decoder.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define GF_BITS 16
#define GF_ORDER 65536
#define GF_MODULUS 65535u
#define GF_POLY 0x1002Du

typedef uint16_t gfe;

static gfe g_exp[GF_ORDER], g_log[GF_ORDER], g_skew[GF_MODULUS];
static int g_ready = 0;

static const gfe kCantor[GF_BITS] = {0x0001, 0xACCA, 0x3C0E, 0x163E, 0xC582, 0xED2E, 0x914C, 0x4012,
                                     0x6C98, 0x10D8, 0x6A72, 0xB900, 0xFDB8, 0xFB34, 0xFF38, 0x991E};

static gfe add_mod(gfe x, gfe y) {
    const uint32_t s = (uint32_t)x + y;
    return (gfe)(s + (s >> GF_BITS));
}
/* x * exp(log_m) */
static gfe mul_log(gfe x, gfe log_m) { return x ? g_exp[add_mod(g_log[x], log_m)] : 0; }

static void init_tables(void) {
    if (g_ready) return;
    /* LFSR exp table, then logarithms re-expressed in the Cantor basis */
    uint32_t state = 1;
    for (uint32_t i = 0; i < GF_MODULUS; i++) {
        g_exp[state] = (gfe)i;
        state <<= 1;
        if (state >= GF_ORDER) state ^= GF_POLY;
    }
    g_exp[0] = GF_MODULUS;
    g_log[0] = 0;
    for (int i = 0; i < GF_BITS; i++) {
        const uint32_t w = 1u << i;
        for (uint32_t j = 0; j < w; j++) g_log[j + w] = g_log[j] ^ kCantor[i];
    }
    for (uint32_t i = 0; i < GF_ORDER; i++) g_log[i] = g_exp[g_log[i]];
    for (uint32_t i = 0; i < GF_ORDER; i++) g_exp[g_log[i]] = (gfe)i;
    g_exp[GF_MODULUS] = g_exp[0];
    /* skew factors of the LCH basis */
    gfe temp[GF_BITS - 1];
    for (int i = 1; i < GF_BITS; i++) temp[i - 1] = (gfe)(1u << i);
    memset(g_skew, 0, sizeof g_skew);
    for (int m = 0; m < GF_BITS - 1; m++) {
        const uint32_t step = 1u << (m + 1);
        g_skew[(1u << m) - 1] = 0;
        for (int i = m; i < GF_BITS - 1; i++) {
            const uint32_t s = 1u << (i + 1);
            for (uint32_t j = (1u << m) - 1; j < s; j += step) g_skew[j + s] = g_skew[j] ^ temp[i];
        }
        temp[m] = (gfe)(GF_MODULUS - g_log[mul_log(temp[m], g_log[temp[m] ^ 1])]);
        for (int i = m + 1; i < GF_BITS - 1; i++) {
            const gfe sum = add_mod(g_log[temp[i] ^ 1], temp[m]);
            temp[i] = mul_log(temp[i], sum);
        }
    }
    for (uint32_t i = 0; i < GF_MODULUS; i++) g_skew[i] = g_log[g_skew[i]];
    g_ready = 1;
}

/* ---- transforms over one column of field elements (work[pos .. pos + size)) ---- */
static void fft_partial(gfe *x, gfe *y, gfe log_m) { *x ^= mul_log(*y, log_m); *y ^= *x; }
static void ifft_partial(gfe *x, gfe *y, gfe log_m) { *y ^= *x; *x ^= mul_log(*y, log_m); }

static void fft2(gfe *a, gfe *b, gfe log_m) {
    if (log_m == GF_MODULUS) *b ^= *a; else fft_partial(a, b, log_m);
}
static void ifft2(gfe *a, gfe *b, gfe log_m) {
    if (log_m == GF_MODULUS) *b ^= *a; else ifft_partial(a, b, log_m);
}

static void fft(gfe *w, size_t pos, size_t size, size_t trunc, size_t skew_delta) {
    size_t dist4 = size, dist = size >> 2;
    while (dist != 0) {
        for (size_t r = 0; r < trunc; r += dist4) {
            const size_t base = r + dist + skew_delta - 1;
            const gfe m01 = g_skew[base], m02 = g_skew[base + dist], m23 = g_skew[base + 2 * dist];
            for (size_t i = r; i < r + dist; i++) {
                gfe *s0 = &w[pos + i], *s1 = s0 + dist, *s2 = s1 + dist, *s3 = s2 + dist;
                fft2(s0, s2, m02);
                fft2(s1, s3, m02);
                fft2(s0, s1, m01);
                fft2(s2, s3, m23);
            }
        }
        dist4 = dist;
        dist >>= 2;
    }
    if (dist4 == 2)
        for (size_t r = 0; r < trunc; r += 2) fft2(&w[pos + r], &w[pos + r + 1], g_skew[r + skew_delta]);
}

static void ifft(gfe *w, size_t pos, size_t size, size_t trunc, size_t skew_delta) {
    size_t dist = 1, dist4 = 4;
    while (dist4 <= size) {
        for (size_t r = 0; r < trunc; r += dist4) {
            const size_t base = r + dist + skew_delta - 1;
            const gfe m01 = g_skew[base], m02 = g_skew[base + dist], m23 = g_skew[base + 2 * dist];
            for (size_t i = r; i < r + dist; i++) {
                gfe *s0 = &w[pos + i], *s1 = s0 + dist, *s2 = s1 + dist, *s3 = s2 + dist;
                ifft2(s0, s1, m01);
                ifft2(s2, s3, m23);
                ifft2(s0, s2, m02);
                ifft2(s1, s3, m02);
            }
        }
        dist = dist4;
        dist4 <<= 2;
    }
    if (dist < size) {
        const gfe m = g_skew[dist + skew_delta - 1];
        for (size_t i = 0; i < dist; i++) ifft2(&w[pos + i], &w[pos + i + dist], m);
    }
}

static size_t next_pow2(size_t x) {
    size_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

/* rate::use_high_rate: 1 high, 0 low, -1 unsupported */
int rs16_use_high_rate(size_t k, size_t m) {
    if (k == 0 || m == 0 || k > GF_ORDER || m > GF_ORDER) return -1;
    const size_t kp = next_pow2(k), mp = next_pow2(m);
    const size_t smaller = kp < mp ? kp : mp, larger = k > m ? k : m;
    if (smaller + larger > GF_ORDER) return -1;
    return mp <= kp ? 1 : 0;
}

/* Encode one column: orig[0..k) -> rec[0..m).  work: scratch of >= rs16_work_count(k, m). */
size_t rs16_work_count(size_t k, size_t m) {
    const int hr = rs16_use_high_rate(k, m);
    if (hr < 0) return 0;
    if (hr) {
        const size_t c = next_pow2(m);
        return ((k + c - 1) / c) * c + c;  /* chunks of originals, rounded up, + the accumulator */
    }
    const size_t c = next_pow2(k);
    return ((m + c - 1) / c) * c;
}

static void encode_column(size_t k, size_t m, const gfe *orig, gfe *rec, gfe *w) {
    if (rs16_use_high_rate(k, m)) {
        const size_t c = next_pow2(m);
        /* work[0..c): the first chunk's IFFT, then every further chunk's XOR-folded in */
        memset(w, 0, c * sizeof(gfe));
        const size_t first = k < c ? k : c;
        memcpy(w, orig, first * sizeof(gfe));
        ifft(w, 0, c, first, c);
        for (size_t start = c; start < k; start += c) {
            const size_t cnt = k - start < c ? k - start : c;
            gfe *t = w + c;
            memset(t, 0, c * sizeof(gfe));
            memcpy(t, orig + start, cnt * sizeof(gfe));
            /* the chunk sits at position `start` of the transform: skew_delta = start + c (the
             * skew index does not depend on where the column is stored) */
            ifft(t, 0, c, cnt, start + c);
            for (size_t i = 0; i < c; i++) w[i] ^= t[i];
        }
        fft(w, 0, c, m, 0);
        memcpy(rec, w, m * sizeof(gfe));
    } else {
        const size_t c = next_pow2(k);
        memset(w, 0, c * sizeof(gfe));
        memcpy(w, orig, k * sizeof(gfe));
        ifft(w, 0, c, k, 0);
        for (size_t start = c; start < m; start += c) memcpy(w + start, w, c * sizeof(gfe));
        for (size_t start = 0; start < m; start += c) {
            const size_t cnt = m - start < c ? m - start : c;
            fft(w, start, c, cnt, start + c);
        }
        memcpy(rec, w, m * sizeof(gfe));
    }
}

/* shard byte layout: 64-byte blocks of 32 elements (low bytes, then high bytes) */
static gfe get_elem(const uint8_t *shard, size_t e) {
    const size_t blk = e >> 5, i = e & 31;
    return (gfe)(shard[blk * 64 + i] | (shard[blk * 64 + 32 + i] << 8));
}
static void put_elem(uint8_t *shard, size_t e, gfe v) {
    const size_t blk = e >> 5, i = e & 31;
    shard[blk * 64 + i] = (uint8_t)v;
    shard[blk * 64 + 32 + i] = (uint8_t)(v >> 8);
}

/* ReedSolomonEncoder: k original shards of `bytes` (multiple of 64) -> m recovery shards.
 * Returns 0, or -1 for an unsupported shape. */
int rs16_encode(size_t k, size_t m, size_t bytes, const uint8_t *const *orig, uint8_t *const *rec) {
    init_tables();
    if (rs16_use_high_rate(k, m) < 0 || bytes == 0 || bytes % 64) return -1;
    const size_t wc = rs16_work_count(k, m);
    gfe *w = (gfe *)malloc((wc + k + m) * sizeof(gfe));
    if (!w) return -1;
    gfe *o = w + wc, *r = o + k;
    const size_t ne = bytes / 2;
    for (size_t e = 0; e < ne; e++) {
        for (size_t j = 0; j < k; j++) o[j] = get_elem(orig[j], e);
        encode_column(k, m, o, r, w);
        for (size_t j = 0; j < m; j++) put_elem(rec[j], e, r[j]);
    }
    free(w);
    return 0;
}

/* ---- decode: generator matrix of the code above, inverted on the received shards ---- */
static gfe gmul(gfe a, gfe b) { return (a && b) ? g_exp[add_mod(g_log[a], g_log[b])] : 0; }
static gfe ginv(gfe a) { return g_exp[(GF_MODULUS - g_log[a]) % GF_MODULUS]; }

/* G[(k + m) x k]: identity on top, then the recovery rows (encode of unit vectors: linear). */
static int generator(size_t k, size_t m, gfe *G) {
    const size_t wc = rs16_work_count(k, m);
    gfe *w = (gfe *)malloc((wc + k + m) * sizeof(gfe));
    if (!w) return -1;
    gfe *o = w + wc, *r = o + k;
    memset(G, 0, (k + m) * k * sizeof(gfe));
    for (size_t i = 0; i < k; i++) G[i * k + i] = 1;
    for (size_t c = 0; c < k; c++) {
        memset(o, 0, k * sizeof(gfe));
        o[c] = 1;
        encode_column(k, m, o, r, w);
        for (size_t j = 0; j < m; j++) G[(k + j) * k + c] = r[j];
    }
    free(w);
    return 0;
}

/* ReedSolomonDecoder: shards[i] for i in 0..k+m (originals then recovery; NULL = missing).
 * Restores every missing original into out[i] (out[i] may alias nothing; present ones are
 * copied).  Returns 0, -1 unsupported shape, -2 fewer than k shards. */
int rs16_decode(size_t k, size_t m, size_t bytes, const uint8_t *const *shards, uint8_t *const *out) {
    init_tables();
    if (rs16_use_high_rate(k, m) < 0 || bytes == 0 || bytes % 64) return -1;
    size_t rows[GF_ORDER > 4096 ? 4096 : GF_ORDER];
    size_t nr = 0;
    for (size_t i = 0; i < k + m && nr < k; i++)
        if (shards[i]) rows[nr++] = i;
    if (nr < k) return -2;
    gfe *G = (gfe *)malloc((k + m) * k * sizeof(gfe));
    gfe *A = (gfe *)malloc(k * 2 * k * sizeof(gfe));
    if (!G || !A || generator(k, m, G)) { free(G); free(A); return -1; }
    /* A = [G_rows | I] -> [I | G_rows^-1] */
    for (size_t r = 0; r < k; r++)
        for (size_t c = 0; c < 2 * k; c++) A[r * 2 * k + c] = c < k ? G[rows[r] * k + c] : (gfe)(c - k == r);
    for (size_t c = 0; c < k; c++) {
        size_t p = c;
        while (p < k && !A[p * 2 * k + c]) p++;
        if (p == k) { free(G); free(A); return -1; }
        if (p != c)
            for (size_t j = 0; j < 2 * k; j++) { gfe t = A[c * 2 * k + j]; A[c * 2 * k + j] = A[p * 2 * k + j]; A[p * 2 * k + j] = t; }
        const gfe iv = ginv(A[c * 2 * k + c]);
        for (size_t j = 0; j < 2 * k; j++) A[c * 2 * k + j] = gmul(A[c * 2 * k + j], iv);
        for (size_t r = 0; r < k; r++) {
            if (r == c || !A[r * 2 * k + c]) continue;
            const gfe f = A[r * 2 * k + c];
            for (size_t j = 0; j < 2 * k; j++) A[r * 2 * k + j] ^= gmul(f, A[c * 2 * k + j]);
        }
    }
    const size_t ne = bytes / 2;
    for (size_t i = 0; i < k; i++) {
        if (shards[i]) { memcpy(out[i], shards[i], bytes); continue; }
        for (size_t e = 0; e < ne; e++) {
            gfe acc = 0;
            for (size_t r = 0; r < k; r++) acc ^= gmul(A[i * 2 * k + k + r], get_elem(shards[rows[r]], e));
            put_elem(out[i], e, acc);
        }
    }
    free(G);
    free(A);
    return 0;
}

/* table access for tests (the GPU kernels derive the same tables on the host) */
gfe rs16_exp(uint32_t i) { init_tables(); return g_exp[i]; }
gfe rs16_log(uint32_t i) { init_tables(); return g_log[i]; }
gfe rs16_skew(uint32_t i) { init_tables(); return g_skew[i]; }
