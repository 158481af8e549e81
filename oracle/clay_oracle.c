/*
 * clay_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity oracle / CPU baseline).
 *
 * Plain-C restatement of the arithmetic behind Tapedrive's `lib/slicer` hot path:
 *   - the third-party `clay-codes` 0.1.1 crate (Cargo.lock:1235-1241), restated from its
 *     published algorithm (Ceph ErasureCodeClay / Vajha et al. FAST'18), with
 *   - `reed-solomon-erasure` 6.0.0 (Cargo.lock:5374-5385) GF(2^8) + systematic Vandermonde MDS,
 *   - the Slicer layer of lib/slicer/src/{adaptive,clay,slicer,metadata,repair}.rs.
 *
 * Neither crate is present in the container; byte parity of *parity* slices with the real
 * crate is therefore UNPINNED (see DESIGN.md "Parity status").  What is pinned by the
 * reference's own tests (sizes, rotation maps, metadata layout, round trips, repair == encode,
 * helper counts, bandwidth) is reproduced in tests/test_oracle_*.py.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this file's
 * shared object, and only as the checker / reported CPU baseline.  The product library
 * (tape_amd/csrc, libtapeec.so) never links it.
 *
 * Construction assumptions:
 *   A1 GF(2^8), poly 0x11D, generator 2 (reed-solomon-erasure galois_8).
 *   A2 per-plane MDS = systematic [q*t, k+nu] code G = V * inv(V[0..k+nu)), V[r][c] = r^c.
 *   A3 pairwise transform (PFT) = systematic RS(2,2) of the same library: [C_hi,C_lo,U_hi,U_lo].
 *   A4 Ceph orientation swap (0<->1, 2<->3) when z_vec[y] > x.
 *   A5 input zero-padded to a multiple of k*alpha*2 (min one block); data chunk i contiguous.
 *   A6 repair helpers: lost node's column-mates, then ascending available ids until d;
 *      sub-chunks = planes with z_vec[y_lost] == x_lost, ascending.
 *   A7 decode pads the erasure set with the lowest parity nodes >= k+nu up to m.
 */
#include <immintrin.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>
#include <pthread.h>

#define OC_MAXQT 64
#define OC_MAXALPHA 4096

/* ---------------- GF(2^8): reed-solomon-erasure galois_8 ---------------- */
static uint8_t GF_EXP[512];
static uint8_t GF_LOG[256];
static uint8_t GF_MUL[256][256];
static int gf_ready = 0;

static void gf_init(void) {
    if (gf_ready) return;
    int x = 1;
    for (int i = 0; i < 255; i++) {
        GF_EXP[i] = (uint8_t)x;
        GF_LOG[x] = (uint8_t)i;
        x <<= 1;
        if (x & 0x100) x ^= 0x11D;
    }
    for (int i = 255; i < 512; i++) GF_EXP[i] = GF_EXP[i - 255];
    for (int a = 0; a < 256; a++)
        for (int b = 0; b < 256; b++)
            GF_MUL[a][b] = (a && b) ? GF_EXP[GF_LOG[a] + GF_LOG[b]] : 0;
    gf_ready = 1;
}
static inline uint8_t gmul(uint8_t a, uint8_t b) { return GF_MUL[a][b]; }
static inline uint8_t ginv(uint8_t a) { return GF_EXP[255 - GF_LOG[a]]; }
/* galois_8::exp(a, n): 0^0 = 1 */
static uint8_t gexp(uint8_t a, int n) {
    if (n == 0) return 1;
    if (a == 0) return 0;
    return GF_EXP[(GF_LOG[a] * n) % 255];
}

/* invert an r x r matrix in place (row-major, stride OC_MAXQT). returns 0 ok, -1 singular */
static int mat_invert(uint8_t *m, int r) {
    uint8_t aug[OC_MAXQT][2 * OC_MAXQT];
    for (int i = 0; i < r; i++)
        for (int j = 0; j < 2 * r; j++)
            aug[i][j] = j < r ? m[i * OC_MAXQT + j] : (uint8_t)(j - r == i);
    for (int c = 0; c < r; c++) {
        int piv = -1;
        for (int i = c; i < r; i++) if (aug[i][c]) { piv = i; break; }
        if (piv < 0) return -1;
        if (piv != c)
            for (int j = 0; j < 2 * r; j++) { uint8_t t = aug[c][j]; aug[c][j] = aug[piv][j]; aug[piv][j] = t; }
        uint8_t iv = ginv(aug[c][c]);
        for (int j = 0; j < 2 * r; j++) aug[c][j] = gmul(aug[c][j], iv);
        for (int i = 0; i < r; i++) {
            if (i == c || !aug[i][c]) continue;
            uint8_t f = aug[i][c];
            for (int j = 0; j < 2 * r; j++) aug[i][j] ^= gmul(f, aug[c][j]);
        }
    }
    for (int i = 0; i < r; i++)
        for (int j = 0; j < r; j++) m[i * OC_MAXQT + j] = aug[i][r + j];
    return 0;
}

/* reed-solomon-erasure build_matrix(data, total): V * inv(top(V)). out is total x data */
static int rs_build_matrix(int data, int total, uint8_t *out /* stride OC_MAXQT */) {
    uint8_t top[OC_MAXQT * OC_MAXQT];
    for (int r = 0; r < data; r++)
        for (int c = 0; c < data; c++) top[r * OC_MAXQT + c] = gexp((uint8_t)r, c);
    if (mat_invert(top, data)) return -1;
    for (int r = 0; r < total; r++)
        for (int c = 0; c < data; c++) {
            uint8_t acc = 0;
            for (int j = 0; j < data; j++) acc ^= gmul(gexp((uint8_t)r, j), top[j * OC_MAXQT + c]);
            out[r * OC_MAXQT + c] = acc;
        }
    return 0;
}

/* dst[i] ^= c * src[i]: reed-solomon-erasure's region multiply.  The reference builds that crate
 * with its `simd-accel` feature (Cargo.lock:5374-5385 resolves its optional `cc` + `libc`
 * dependencies), whose C kernel multiplies 32 bytes at a time through two 16-entry nibble tables
 * and byte shuffles; this is the same method with AVX2 (the Makefile targets x86-64-v3), so the
 * CPU baseline runs at the reference's speed class rather than a per-byte table walk. */
static void mul_add(uint8_t *dst, const uint8_t *src, uint8_t c, size_t len) {
    if (!c) return;
    size_t i = 0;
    if (c == 1) {
        for (; i + 32 <= len; i += 32) {
            const __m256i d = _mm256_loadu_si256((const __m256i *)(dst + i));
            _mm256_storeu_si256((__m256i *)(dst + i), _mm256_xor_si256(d, _mm256_loadu_si256((const __m256i *)(src + i))));
        }
        for (; i < len; i++) dst[i] ^= src[i];
        return;
    }
    const uint8_t *row = GF_MUL[c];
    uint8_t lo[16], hi[16];
    for (int v = 0; v < 16; v++) {
        lo[v] = row[v];
        hi[v] = row[v << 4];
    }
    const __m256i tlo = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)lo));
    const __m256i thi = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)hi));
    const __m256i m4 = _mm256_set1_epi8(0x0f);
    for (; i + 32 <= len; i += 32) {
        const __m256i sv = _mm256_loadu_si256((const __m256i *)(src + i));
        const __m256i pl = _mm256_shuffle_epi8(tlo, _mm256_and_si256(sv, m4));
        const __m256i ph = _mm256_shuffle_epi8(thi, _mm256_and_si256(_mm256_srli_epi64(sv, 4), m4));
        const __m256i d = _mm256_loadu_si256((const __m256i *)(dst + i));
        _mm256_storeu_si256((__m256i *)(dst + i), _mm256_xor_si256(d, _mm256_xor_si256(pl, ph)));
    }
    for (; i < len; i++) dst[i] ^= row[src[i]];
}

/* ---------------- Clay code (clay-codes 0.1.1 restated) ---------------- */
typedef struct {
    int n, k, m, d, q, t, nu, qt, alpha, beta;
    uint8_t G[OC_MAXQT * OC_MAXQT]; /* qt x (k+nu) systematic generator (A2) */
    uint8_t G4[4 * OC_MAXQT];       /* PFT generator, 4 x 2 (A3) */
} oc_clay;

static int pow_int(int a, int x) { int p = 1; while (x-- > 0) p *= a; return p; }

/* ClayCoder::new(n,k,d) -> ClayCode::new(k, m, d)   lib/slicer/src/clay.rs:24-34 */
int oc_clay_init(oc_clay *c, int n, int k, int d) {
    gf_init();
    if (!(n > k && k > 0 && d >= k + 1 && d <= n - 1)) return -1;
    memset(c, 0, sizeof(*c));
    c->n = n; c->k = k; c->m = n - k; c->d = d;
    c->q = d - k + 1;
    c->nu = (c->q - (n % c->q)) % c->q;
    c->t = (n + c->nu) / c->q;
    c->qt = c->q * c->t;
    if (c->qt > OC_MAXQT) return -2;
    long a = 1;
    for (int i = 0; i < c->t; i++) { a *= c->q; if (a > OC_MAXALPHA) return -2; }
    c->alpha = (int)a;
    c->beta = c->alpha / c->q;
    if (rs_build_matrix(k + c->nu, c->qt, c->G)) return -3;
    if (rs_build_matrix(2, 4, c->G4)) return -3;
    return 0;
}

int oc_clay_sizeof(void) { return (int)sizeof(oc_clay); }
int oc_clay_alpha(const oc_clay *c) { return c->alpha; }
int oc_clay_beta(const oc_clay *c) { return c->beta; }
int oc_clay_param(const oc_clay *c, int which) {
    switch (which) { case 0: return c->n; case 1: return c->k; case 2: return c->m; case 3: return c->d;
    case 4: return c->q; case 5: return c->t; case 6: return c->nu; case 7: return c->alpha; case 8: return c->beta; }
    return -1;
}
uint8_t oc_gf_mul(uint8_t a, uint8_t b) { gf_init(); return gmul(a, b); }
void oc_generator(const oc_clay *c, uint8_t *out) { /* qt x (k+nu), dense */
    for (int r = 0; r < c->qt; r++)
        for (int j = 0; j < c->k + c->nu; j++) out[r * (c->k + c->nu) + j] = c->G[r * OC_MAXQT + j];
}

/* ClayCoder::chunk_size_for   lib/slicer/src/clay.rs:61-73 (A5) */
size_t oc_chunk_size_for(const oc_clay *c, size_t input_len) {
    size_t min_size = (size_t)c->k * c->alpha * 2;
    size_t padded = input_len == 0 ? min_size : ((input_len + min_size - 1) / min_size) * min_size;
    if (padded < min_size) padded = min_size;
    return padded / c->k;
}

static void plane_vector(const oc_clay *c, int z, int *zv) {
    for (int i = 0; i < c->t; i++) { zv[c->t - 1 - i] = z % c->q; z /= c->q; }
}

/* Solve the [4,2] PFT codeword: positions known a,b with values (buffers) -> write position w. */
static void pft_solve(const oc_clay *c, int a, const uint8_t *va, int b, const uint8_t *vb,
                      int w, uint8_t *out, size_t len) {
    uint8_t sub[OC_MAXQT * OC_MAXQT];
    sub[0] = c->G4[a * OC_MAXQT + 0]; sub[1] = c->G4[a * OC_MAXQT + 1];
    sub[OC_MAXQT + 0] = c->G4[b * OC_MAXQT + 0]; sub[OC_MAXQT + 1] = c->G4[b * OC_MAXQT + 1];
    mat_invert(sub, 2);
    /* out = G4[w] . inv . [va; vb] */
    uint8_t ca = gmul(c->G4[w * OC_MAXQT + 0], sub[0]) ^ gmul(c->G4[w * OC_MAXQT + 1], sub[OC_MAXQT + 0]);
    uint8_t cb = gmul(c->G4[w * OC_MAXQT + 0], sub[1]) ^ gmul(c->G4[w * OC_MAXQT + 1], sub[OC_MAXQT + 1]);
    /* out may alias neither va nor vb */
    memset(out, 0, len);
    mul_add(out, va, ca, len);
    mul_add(out, vb, cb, len);
}

typedef struct {
    const oc_clay *c;
    uint8_t **C;   /* qt coupled chunks (cs bytes each) */
    uint8_t **U;   /* qt uncoupled chunks */
    int sc;        /* sub-chunk size */
    int erased[OC_MAXQT];
    uint8_t D[OC_MAXQT * OC_MAXQT]; /* per-plane MDS decode matrix: erased x known */
    int known_list[OC_MAXQT], nknown;
    int er_list[OC_MAXQT], ner;
} layered_t;

static int build_mds_decoder(layered_t *L) {
    const oc_clay *c = L->c;
    int kk = c->k + c->nu;
    L->nknown = 0; L->ner = 0;
    for (int i = 0; i < c->qt; i++) {
        if (L->erased[i]) L->er_list[L->ner++] = i;
        else if (L->nknown < kk) L->known_list[L->nknown++] = i;
    }
    if (L->nknown < kk) return -1;
    uint8_t sub[OC_MAXQT * OC_MAXQT];
    for (int r = 0; r < kk; r++)
        for (int j = 0; j < kk; j++) sub[r * OC_MAXQT + j] = c->G[L->known_list[r] * OC_MAXQT + j];
    if (mat_invert(sub, kk)) return -1;
    for (int e = 0; e < L->ner; e++)
        for (int j = 0; j < kk; j++) {
            uint8_t acc = 0;
            for (int l = 0; l < kk; l++) acc ^= gmul(c->G[L->er_list[e] * OC_MAXQT + l], sub[l * OC_MAXQT + j]);
            L->D[e * OC_MAXQT + j] = acc;
        }
    return 0;
}

/* decode_uncoupled: MDS-solve erased U's of plane z from the known U's */
static void decode_uncoupled(layered_t *L, int z) {
    int sc = L->sc, kk = L->c->k + L->c->nu;
    for (int e = 0; e < L->ner; e++) {
        uint8_t *dst = L->U[L->er_list[e]] + (size_t)z * sc;
        memset(dst, 0, sc);
        for (int j = 0; j < kk; j++) mul_add(dst, L->U[L->known_list[j]] + (size_t)z * sc, L->D[e * OC_MAXQT + j], sc);
    }
}

/* Ceph get_uncoupled_from_coupled restricted to the value needed: U(node_xy, z) */
static void uncoupled_from_coupled(layered_t *L, int x, int y, int z, const int *zv) {
    const oc_clay *c = L->c;
    int node = y * c->q + x, sw = y * c->q + zv[y];
    int zsw = z + (x - zv[y]) * pow_int(c->q, c->t - 1 - y);
    int i0 = 0, i1 = 1, i2 = 2;
    if (zv[y] > x) { i0 = 1; i1 = 0; i2 = 3; }
    pft_solve(c, i0, L->C[node] + (size_t)z * L->sc, i1, L->C[sw] + (size_t)zsw * L->sc,
              i2, L->U[node] + (size_t)z * L->sc, L->sc);
}

/* type-1: C(node,z) from U(node,z) and C(sw,z_sw) */
static void recover_type1(layered_t *L, int x, int y, int z, const int *zv) {
    const oc_clay *c = L->c;
    int node = y * c->q + x, sw = y * c->q + zv[y];
    int zsw = z + (x - zv[y]) * pow_int(c->q, c->t - 1 - y);
    int i0 = 0, i1 = 1, i2 = 2;
    if (zv[y] > x) { i0 = 1; i1 = 0; i2 = 3; }
    pft_solve(c, i1, L->C[sw] + (size_t)zsw * L->sc, i2, L->U[node] + (size_t)z * L->sc,
              i0, L->C[node] + (size_t)z * L->sc, L->sc);
}

/* both erased: C(node,z), C(sw,z_sw) from U(node,z), U(sw,z_sw) */
static void coupled_from_uncoupled(layered_t *L, int x, int y, int z, const int *zv) {
    const oc_clay *c = L->c;
    int node = y * c->q + x, sw = y * c->q + zv[y];
    int zsw = z + (x - zv[y]) * pow_int(c->q, c->t - 1 - y);
    int i0 = 0, i1 = 1, i2 = 2, i3 = 3;
    if (zv[y] > x) { i0 = 1; i1 = 0; i2 = 3; i3 = 2; }
    const uint8_t *un = L->U[node] + (size_t)z * L->sc, *us = L->U[sw] + (size_t)zsw * L->sc;
    pft_solve(c, i2, un, i3, us, i0, L->C[node] + (size_t)z * L->sc, L->sc);
    pft_solve(c, i2, un, i3, us, i1, L->C[sw] + (size_t)zsw * L->sc, L->sc);
}

/* Ceph decode_layered (A7 padding included) */
static int decode_layered(layered_t *L) {
    const oc_clay *c = L->c;
    int q = c->q, t = c->t, alpha = c->alpha;
    int ner = 0;
    for (int i = 0; i < c->qt; i++) ner += L->erased[i];
    for (int i = c->k + c->nu; ner < c->m && i < c->qt; i++)
        if (!L->erased[i]) { L->erased[i] = 1; ner++; }
    if (ner != c->m) return -1;
    if (build_mds_decoder(L)) return -1;
    int *order = (int *)malloc(sizeof(int) * alpha);
    int zv[16], max_iscore = 0;
    for (int z = 0; z < alpha; z++) {
        plane_vector(c, z, zv);
        int o = 0;
        for (int i = 0; i < c->qt; i++) if (L->erased[i] && (i % q) == zv[i / q]) o++;
        order[z] = o;
        if (o > max_iscore) max_iscore = o;
    }
    for (int is = 0; is <= max_iscore; is++) {
        for (int z = 0; z < alpha; z++) {
            if (order[z] != is) continue;
            plane_vector(c, z, zv);
            /* decode_erasures: U for every non-erased node of plane z */
            for (int x = 0; x < q; x++)
                for (int y = 0; y < t; y++) {
                    int node = q * y + x;
                    if (L->erased[node]) continue;
                    if (zv[y] == x) memcpy(L->U[node] + (size_t)z * L->sc, L->C[node] + (size_t)z * L->sc, L->sc);
                    else uncoupled_from_coupled(L, x, y, z, zv);
                }
            decode_uncoupled(L, z);
        }
        for (int z = 0; z < alpha; z++) {
            if (order[z] != is) continue;
            plane_vector(c, z, zv);
            for (int node = 0; node < c->qt; node++) {
                if (!L->erased[node]) continue;
                int x = node % q, y = node / q;
                int sw = y * q + zv[y];
                if (zv[y] != x) {
                    if (!L->erased[sw]) recover_type1(L, x, y, z, zv);
                    else if (zv[y] < x) coupled_from_uncoupled(L, x, y, z, zv);
                } else {
                    memcpy(L->C[node] + (size_t)z * L->sc, L->U[node] + (size_t)z * L->sc, L->sc);
                }
            }
        }
    }
    free(order);
    return 0;
}

static uint8_t *xcalloc(size_t n) { uint8_t *p = (uint8_t *)calloc(n ? n : 1, 1); return p; }

/* ClayCode::encode: data (len bytes) -> n chunks of cs bytes, out = n*cs (external order) */
int oc_clay_encode(const oc_clay *c, const uint8_t *data, size_t len, uint8_t *out) {
    if (len == 0) return -1; /* EncodeError::EmptyInput, clay.rs:100-102 */
    size_t cs = oc_chunk_size_for(c, len);
    layered_t L; memset(&L, 0, sizeof(L));
    L.c = c; L.sc = (int)(cs / c->alpha);
    uint8_t *Cb[OC_MAXQT], *Ub[OC_MAXQT];
    uint8_t *zero_bufs = xcalloc(cs * (c->nu ? c->nu : 1));
    for (int i = 0; i < c->qt; i++) {
        int ext = i < c->k ? i : (i < c->k + c->nu ? -1 : i - c->nu);
        Cb[i] = ext >= 0 ? out + (size_t)ext * cs : zero_bufs + (size_t)(i - c->k) * cs;
        Ub[i] = xcalloc(cs);
    }
    /* data chunks: padded input split contiguously */
    memset(out, 0, (size_t)c->k * cs);
    memcpy(out, data, len);
    for (int i = c->k + c->nu; i < c->qt; i++) L.erased[i] = 1;
    L.C = Cb; L.U = Ub;
    int r = decode_layered(&L);
    for (int i = 0; i < c->qt; i++) free(Ub[i]);
    free(zero_bufs);
    return r;
}

/* ClayCode::decode(available, erasures): chunks = n*cs buffer (external order, missing ones
 * may hold garbage), avail[i] != 0 if chunk i present. out = k*cs data. */
int oc_clay_decode(const oc_clay *c, const uint8_t *chunks, const int *avail, size_t cs, uint8_t *out) {
    int na = 0;
    for (int i = 0; i < c->n; i++) na += avail[i] != 0;
    if (na < c->k) return -1; /* DecodeError::NotEnoughSlices clay.rs:107-109 */
    if (cs % c->alpha) return -2;
    layered_t L; memset(&L, 0, sizeof(L));
    L.c = c; L.sc = (int)(cs / c->alpha);
    uint8_t *Cb[OC_MAXQT], *Ub[OC_MAXQT];
    for (int i = 0; i < c->qt; i++) {
        int ext = i < c->k ? i : (i < c->k + c->nu ? -1 : i - c->nu);
        Cb[i] = xcalloc(cs); Ub[i] = xcalloc(cs);
        if (ext >= 0 && avail[ext]) memcpy(Cb[i], chunks + (size_t)ext * cs, cs);
        if (ext >= 0 && !avail[ext]) L.erased[i] = 1;
    }
    L.C = Cb; L.U = Ub;
    int r = decode_layered(&L);
    if (!r) for (int i = 0; i < c->k; i++) memcpy(out + (size_t)i * cs, Cb[i], cs);
    for (int i = 0; i < c->qt; i++) { free(Cb[i]); free(Ub[i]); }
    return r;
}

/* get_repair_subchunks -> expanded ascending plane list (A6). returns count (beta) */
int oc_repair_subchunks(const oc_clay *c, int lost_ext, int *planes) {
    int lost = lost_ext < c->k ? lost_ext : lost_ext + c->nu;
    int y = lost / c->q, x = lost % c->q;
    int seq = pow_int(c->q, c->t - 1 - y), nseq = pow_int(c->q, y), cnt = 0;
    int index = x * seq;
    for (int s = 0; s < nseq; s++) {
        for (int j = index; j < index + seq; j++) planes[cnt++] = j;
        index += c->q * seq;
    }
    return cnt;
}

/* ClayCode::minimum_to_repair(lost, available) -> d helper ids (ascending) (A6)
 * returns number of helpers (d) or negative error. */
int oc_minimum_to_repair(const oc_clay *c, int lost_ext, const int *avail_ids, int navail, int *helpers) {
    if (lost_ext < 0 || lost_ext >= c->n) return -1;
    if (navail < c->d) return -2;
    int chosen[OC_MAXQT]; memset(chosen, 0, sizeof(chosen));
    int isavail[OC_MAXQT]; memset(isavail, 0, sizeof(isavail));
    for (int i = 0; i < navail; i++) if (avail_ids[i] >= 0 && avail_ids[i] < c->n) isavail[avail_ids[i]] = 1;
    int lost = lost_ext < c->k ? lost_ext : lost_ext + c->nu;
    int cnt = 0;
    for (int j = 0; j < c->q; j++) {
        if (j == lost % c->q) continue;
        int rep = (lost / c->q) * c->q + j;
        int ext = rep < c->k ? rep : (rep >= c->k + c->nu ? rep - c->nu : -1);
        if (ext < 0) continue;
        if (!isavail[ext]) return -3; /* column-mate required for Clay repair */
        if (!chosen[ext]) { chosen[ext] = 1; cnt++; }
    }
    /* available in ascending order (a set in Ceph) */
    for (int id = 0; id < c->n && cnt < c->d; id++)
        if (isavail[id] && !chosen[id] && id != lost_ext) { chosen[id] = 1; cnt++; }
    if (cnt != c->d) return -2;
    int h = 0;
    for (int id = 0; id < c->n; id++) if (chosen[id]) helpers[h++] = id;
    return h;
}

/* ClayCode::repair(lost, helper_data, chunk_size) -- Ceph repair/repair_one_lost_chunk.
 * helper_ids: d external ids; helper_bufs: concatenated [d][beta*sc] in helper_ids order. */
int oc_clay_repair(const oc_clay *c, int lost_ext, const int *helper_ids, int nh,
                   const uint8_t *helper_bufs, size_t cs, uint8_t *out) {
    if (nh != c->d) return -1;
    if (cs % c->alpha) return -2;
    int q = c->q, t = c->t, alpha = c->alpha, sc = (int)(cs / alpha);
    size_t rb = (size_t)c->beta * sc;
    int lost = lost_ext < c->k ? lost_ext : lost_ext + c->nu;
    const uint8_t *H[OC_MAXQT]; memset(H, 0, sizeof(H));
    uint8_t *zero_helper = xcalloc(rb);
    int aloof[OC_MAXQT]; memset(aloof, 0, sizeof(aloof));
    for (int i = 0; i < nh; i++) {
        int e = helper_ids[i];
        if (e < 0 || e >= c->n || e == lost_ext) { free(zero_helper); return -3; }
        int node = e < c->k ? e : e + c->nu;
        H[node] = helper_bufs + (size_t)i * rb;
    }
    for (int e = 0; e < c->n; e++) {
        int node = e < c->k ? e : e + c->nu;
        if (!H[node] && e != lost_ext) aloof[node] = 1;
    }
    for (int i = c->k; i < c->k + c->nu; i++) H[i] = zero_helper;
    int planes[OC_MAXALPHA];
    int nrp = oc_repair_subchunks(c, lost_ext, planes);
    int *plane_ind = (int *)malloc(sizeof(int) * alpha);
    for (int z = 0; z < alpha; z++) plane_ind[z] = -1;
    for (int i = 0; i < nrp; i++) plane_ind[planes[i]] = i;
    /* erasures: lost column + aloof */
    layered_t L; memset(&L, 0, sizeof(L));
    L.c = c; L.sc = sc;
    for (int i = 0; i < q; i++) L.erased[lost - lost % q + i] = 1;
    for (int i = 0; i < c->qt; i++) if (aloof[i]) L.erased[i] = 1;
    int ner = 0; for (int i = 0; i < c->qt; i++) ner += L.erased[i];
    if (ner > c->m) { free(plane_ind); free(zero_helper); return -4; }
    if (build_mds_decoder(&L)) { free(plane_ind); free(zero_helper); return -4; }
    uint8_t *Ub[OC_MAXQT];
    for (int i = 0; i < c->qt; i++) Ub[i] = xcalloc(cs);
    L.U = Ub;
    /* order per repair plane */
    int zv[16], maxo = 0;
    int *ord = (int *)malloc(sizeof(int) * alpha);
    for (int i = 0; i < nrp; i++) {
        int z = planes[i], o = 0;
        plane_vector(c, z, zv);
        if ((lost % q) == zv[lost / q]) o++;
        for (int nd = 0; nd < c->qt; nd++) if (aloof[nd] && (nd % q) == zv[nd / q]) o++;
        ord[i] = o; if (o > maxo) maxo = o;
    }
    uint8_t *tmp = xcalloc(sc);
    for (int o = 1; o <= maxo; o++) {
        for (int pi = 0; pi < nrp; pi++) {
            if (ord[pi] != o) continue;
            int z = planes[pi];
            plane_vector(c, z, zv);
            for (int y = 0; y < t; y++)
                for (int x = 0; x < q; x++) {
                    int node = y * q + x;
                    if (L.erased[node]) continue;
                    int zsw = z + (x - zv[y]) * pow_int(q, t - 1 - y);
                    int sw = y * q + zv[y];
                    int i0 = 0, i1 = 1, i2 = 2, i3 = 3;
                    if (zv[y] > x) { i0 = 1; i1 = 0; i2 = 3; i3 = 2; }
                    const uint8_t *cn = H[node] + (size_t)plane_ind[z] * sc;
                    uint8_t *un = Ub[node] + (size_t)z * sc;
                    if (aloof[sw]) {
                        pft_solve(c, i0, cn, i3, Ub[sw] + (size_t)zsw * sc, i2, un, sc);
                    } else if (zv[y] != x) {
                        const uint8_t *cs_ = H[sw] + (size_t)plane_ind[zsw] * sc;
                        pft_solve(c, i0, cn, i1, cs_, i2, un, sc);
                    } else {
                        memcpy(un, cn, sc);
                    }
                    (void)i1; (void)i3;
                }
            decode_uncoupled(&L, z);
            for (int node = 0; node < c->qt; node++) {
                if (!L.erased[node] || aloof[node]) continue;
                int x = node % q, y = node / q;
                int sw = y * q + zv[y];
                int zsw = z + (x - zv[y]) * pow_int(q, t - 1 - y);
                int i0 = 0, i1 = 1, i2 = 2;
                if (zv[y] > x) { i0 = 1; i1 = 0; i2 = 3; }
                if (x == zv[y]) {
                    memcpy(out + (size_t)z * sc, Ub[node] + (size_t)z * sc, sc);
                } else {
                    if (sw != lost) { free(tmp); return -5; }
                    pft_solve(c, i0, H[node] + (size_t)plane_ind[z] * sc, i2, Ub[node] + (size_t)z * sc,
                              i1, out + (size_t)zsw * sc, sc);
                }
            }
        }
    }
    free(tmp); free(ord); free(plane_ind); free(zero_helper);
    for (int i = 0; i < c->qt; i++) free(Ub[i]);
    return 0;
}

/* ---------------- Slicer layer (lib/slicer/src/{adaptive,slicer,metadata,repair}.rs) ---------------- */
#define OC_META 48
static const size_t STRIPE_SIZES[3] = {100000, 1000000, 10000000};

/* adaptive.rs:31-39 */
size_t oc_pick_stripe_size(size_t blob_len) {
    if (blob_len <= 1000000) return STRIPE_SIZES[0];
    if (blob_len <= 100000000) return STRIPE_SIZES[1];
    return STRIPE_SIZES[2];
}
/* adaptive.rs:43-49 */
size_t oc_num_stripes(size_t blob_len, size_t stripe) { return blob_len == 0 ? 1 : (blob_len + stripe - 1) / stripe; }

/* slicer.rs:34-53 */
int oc_shard_to_slice(int rotated, int n, int stripe, int shard) {
    if (!rotated) return shard;
    int off = (int)(((long)stripe * 7) % n);
    return (shard + off) % n;
}
int oc_slice_to_shard(int rotated, int n, int stripe, int slice) {
    if (!rotated) return slice;
    int off = (int)(((long)stripe * 7) % n);
    return (slice + n - off) % n;
}

static void put_u64(uint8_t *p, uint64_t v) { for (int i = 0; i < 8; i++) p[i] = (uint8_t)(v >> (8 * i)); }
static uint64_t get_u64(const uint8_t *p) { uint64_t v = 0; for (int i = 0; i < 8; i++) v |= (uint64_t)p[i] << (8 * i); return v; }

/* metadata.rs:22-64: [version][blob_len][stripe_size][encoding][params][chunk_index] */
void oc_metadata(uint8_t *out, uint64_t blob_len, uint64_t stripe, uint64_t encoding, uint64_t params, uint64_t chunk_index) {
    put_u64(out, 0); put_u64(out + 8, blob_len); put_u64(out + 16, stripe);
    put_u64(out + 24, encoding); put_u64(out + 32, params); put_u64(out + 40, chunk_index);
}

/* Slicer::encode geometry: returns slice length, fills stripe size / stripes / chunk size */
size_t oc_slicer_geometry(const oc_clay *c, size_t blob_len, size_t *stripe, size_t *ns, size_t *cs) {
    size_t S = oc_pick_stripe_size(blob_len);
    size_t n_s = oc_num_stripes(blob_len, S);
    size_t eff = blob_len == 0 ? S : (blob_len < S ? blob_len : S);
    size_t ch = oc_chunk_size_for(c, eff);
    if (stripe) *stripe = S;
    if (ns) *ns = n_s;
    if (cs) *cs = ch;
    return n_s * ch + OC_META;
}

/* Slicer<ClayCoder>::encode   slicer.rs:237-296 (+ encode_empty_blob :368-387).
 * out = n slices, each slice_len bytes, contiguous. */
int oc_slicer_encode(const oc_clay *c, int rotated, uint64_t encoding, uint64_t params, uint64_t chunk_index,
                     const uint8_t *data, size_t blob_len, uint8_t *out) {
    size_t S, ns, cs;
    size_t slice_len = oc_slicer_geometry(c, blob_len, &S, &ns, &cs);
    int n = c->n;
    uint8_t *chunks = (uint8_t *)malloc((size_t)n * cs);
    uint8_t *stripe_buf = xcalloc((size_t)c->k * cs);
    for (size_t s = 0; s < ns; s++) {
        size_t start = s * S, end = start + S < blob_len ? start + S : blob_len;
        size_t slen = blob_len == 0 ? S : end - start;
        memset(stripe_buf, 0, (size_t)c->k * cs);
        if (blob_len) memcpy(stripe_buf, data + start, slen);
        /* the coder's own chunk size for this stripe; Slicer re-encodes zero-padded to S when it
         * differs (slicer.rs:273-283) -- either way the stripe is zero-padded to k*cs bytes. */
        size_t pad_len = oc_chunk_size_for(c, slen) == cs ? slen : S;
        if (oc_clay_encode(c, stripe_buf, pad_len, chunks)) { free(chunks); free(stripe_buf); return -1; }
        for (int sh = 0; sh < n; sh++) {
            int sl = oc_shard_to_slice(rotated, n, (int)s, sh);
            memcpy(out + (size_t)sl * slice_len + s * cs, chunks + (size_t)sh * cs, cs);
        }
    }
    uint8_t meta[OC_META];
    oc_metadata(meta, blob_len, S, encoding, params, chunk_index);
    for (int sl = 0; sl < n; sl++) memcpy(out + (size_t)sl * slice_len + ns * cs, meta, OC_META);
    free(chunks); free(stripe_buf);
    return 0;
}

/* Slicer::decode  slicer.rs:298-364. slices: n * slice_len buffer; avail[i] marks present slices.
 * out must hold blob_len bytes (from metadata). returns blob_len or negative:
 * -1 NotEnoughSlices, -2 InvalidLayout, -3 BadEncoding */
long oc_slicer_decode(const oc_clay *c, int rotated, const uint8_t *slices, const int *avail,
                      size_t slice_len, uint8_t *out) {
    int n = c->n, first = -1, na = 0;
    for (int i = 0; i < n; i++) if (avail[i]) { na++; if (first < 0) first = i; }
    if (na == 0) return -1;
    if (slice_len < OC_META) return -2;
    const uint8_t *meta = slices + (size_t)first * slice_len + slice_len - OC_META;
    uint64_t blob_len = get_u64(meta + 8), S = get_u64(meta + 16), params = get_u64(meta + 32);
    if (S != 100000 && S != 1000000 && S != 10000000) return -2;
    int pk = (int)((params >> 8) & 0xFF);
    if (na < pk) return -1;
    if (blob_len == 0) return 0;
    size_t ns = (blob_len + S - 1) / S;
    size_t total = slice_len - OC_META;
    if (total == 0 || total % ns) return -2;
    size_t cs = total / ns;
    if (na < c->k) return -1;
    uint8_t *chunks = (uint8_t *)malloc((size_t)n * cs);
    uint8_t *dec = (uint8_t *)malloc((size_t)c->k * cs);
    int av[OC_MAXQT];
    size_t written = 0;
    for (size_t s = 0; s < ns; s++) {
        for (int sh = 0; sh < n; sh++) {
            int sl = oc_shard_to_slice(rotated, n, (int)s, sh);
            av[sh] = avail[sl] != 0;
            if (av[sh]) memcpy(chunks + (size_t)sh * cs, slices + (size_t)sl * slice_len + s * cs, cs);
        }
        if (oc_clay_decode(c, chunks, av, cs, dec)) { free(chunks); free(dec); return -3; }
        size_t take = (s == ns - 1) ? blob_len - written : S;
        if (take > (size_t)c->k * cs) { free(chunks); free(dec); return -2; }
        memcpy(out + written, dec, take);
        written += take;
    }
    free(chunks); free(dec);
    return (long)blob_len;
}

/* repair_plan_from_params (repair.rs:137-201): fills per stripe lost shard, helper slices,
 * helper shards and sub-chunk planes. helpers_out: ns * d slice ids; shards_out: ns*d; planes: beta.
 * returns chunk size or negative. */
long oc_repair_plan(const oc_clay *c, int rotated, int lost, const int *avail, int navail,
                    size_t blob_len, size_t stripe, int *lost_shards, int *helper_slices,
                    int *helper_shards, int *planes /* ns*d*beta */) {
    size_t ns = oc_num_stripes(blob_len, stripe);
    size_t eff = blob_len < stripe ? blob_len : stripe;
    size_t cs = oc_chunk_size_for(c, eff);
    if (cs % c->alpha) return -2;
    int n = c->n;
    for (size_t s = 0; s < ns; s++) {
        int ls = oc_slice_to_shard(rotated, n, (int)s, lost);
        int av[OC_MAXQT];
        for (int i = 0; i < navail; i++) av[i] = oc_slice_to_shard(rotated, n, (int)s, avail[i]);
        int hs[OC_MAXQT];
        int h = oc_minimum_to_repair(c, ls, av, navail, hs);
        if (h < 0) return -1;
        lost_shards[s] = ls;
        int pl[OC_MAXALPHA];
        int nb = oc_repair_subchunks(c, ls, pl);
        for (int j = 0; j < h; j++) {
            helper_shards[s * c->d + j] = hs[j];
            helper_slices[s * c->d + j] = oc_shard_to_slice(rotated, n, (int)s, hs[j]);
            for (int b = 0; b < nb; b++) planes[(s * c->d + j) * c->beta + b] = pl[b];
        }
    }
    return (long)cs;
}

/* ---------------- CPU baseline helper: encode many objects on T threads ---------------- */
typedef struct {
    const oc_clay *c; const uint8_t *data; size_t len; uint8_t *out; size_t out_stride;
    int nobj, tid, nthr;
} enc_job;

static void *enc_worker(void *arg) {
    enc_job *j = (enc_job *)arg;
    for (int o = j->tid; o < j->nobj; o += j->nthr)
        oc_slicer_encode(j->c, 1, 2, 0x100714, 0, j->data + (size_t)o * j->len, j->len, j->out + (size_t)o * j->out_stride);
    return NULL;
}

/* encode nobj objects (each len bytes, contiguous) with nthr threads; rotated, clay profile. */
int oc_slicer_encode_many(const oc_clay *c, const uint8_t *data, size_t len, int nobj,
                          uint8_t *out, size_t out_stride, int nthr) {
    if (nthr < 1) nthr = 1;
    pthread_t th[256];
    enc_job jobs[256];
    if (nthr > 256) nthr = 256;
    for (int i = 0; i < nthr; i++) {
        jobs[i].c = c; jobs[i].data = data; jobs[i].len = len; jobs[i].out = out; jobs[i].out_stride = out_stride;
        jobs[i].nobj = nobj; jobs[i].tid = i; jobs[i].nthr = nthr;
        pthread_create(&th[i], NULL, enc_worker, &jobs[i]);
    }
    for (int i = 0; i < nthr; i++) pthread_join(th[i], NULL);
    return 0;
}

/* ---------------- CPU baseline helpers for the decode / repair / recover bench lines ----------------
 * One object per task, tasks spread over nthr threads (the same shape as oc_slicer_encode_many).
 * Object o's 20 slices are at slices + o * obj_stride (slice i at + i * slice_len). */
typedef struct {
    const oc_clay *c; const uint8_t *slices; size_t obj_stride, slice_len; const uint32_t *masks;
    const int *lost; const int *down; uint8_t *out; size_t out_stride; int nobj, tid, nthr, kind; int *status;
} many_job;

/* Slicer::decode from the slices marked in masks[o] (slicer.rs:298-364) */
static int decode_one(const many_job *j, int o) {
    int av[OC_MAXQT];
    for (int i = 0; i < j->c->n; i++) av[i] = (j->masks[o] >> i) & 1;
    long r = oc_slicer_decode(j->c, 1, j->slices + (size_t)o * j->obj_stride, av, j->slice_len,
                              j->out + (size_t)o * j->out_stride);
    return r < 0 ? (int)r : 0;
}

/* Slicer::repair of slice lost[o] (repair.rs:324-367): plan from the available slices (all but
 * lost[o] and down[o]), the helpers' sub-chunks gathered per stripe as extract_repair_data sends
 * them (repair.rs:97-130), ClayCode::repair per stripe, then the metadata suffix. */
static int repair_one(const many_job *j, int o) {
    const oc_clay *c = j->c;
    int n = c->n, d = c->d, beta = c->beta, lost = j->lost[o], down = j->down ? j->down[o] : -1;
    const uint8_t *base = j->slices + (size_t)o * j->obj_stride;
    const uint8_t *meta = base + j->slice_len - OC_META;
    uint64_t blob_len = get_u64(meta + 8), S = get_u64(meta + 16);
    int avail[OC_MAXQT], na = 0;
    for (int i = 0; i < n; i++) if (i != lost && i != down) avail[na++] = i;
    size_t ns = oc_num_stripes(blob_len, S);
    int *ls = (int *)malloc(sizeof(int) * ns), *hsl = (int *)malloc(sizeof(int) * ns * d);
    int *hsh = (int *)malloc(sizeof(int) * ns * d), *pl = (int *)malloc(sizeof(int) * ns * d * beta);
    long cs = oc_repair_plan(c, 1, lost, avail, na, blob_len, S, ls, hsl, hsh, pl);
    int rc = 0;
    if (cs <= 0) { rc = -1; goto done; }
    size_t sc = (size_t)cs / c->alpha, rb = (size_t)beta * sc;
    uint8_t *hb = (uint8_t *)malloc((size_t)d * rb);
    uint8_t *dst = j->out + (size_t)o * j->out_stride;
    for (size_t s = 0; s < ns && !rc; s++) {
        int ids[OC_MAXQT], ord[OC_MAXQT];
        for (int h = 0; h < d; h++) ord[h] = h;
        for (int a = 0; a < d; a++)       /* oc_clay_repair takes helpers by ascending shard id */
            for (int b = a + 1; b < d; b++)
                if (hsh[s * d + ord[b]] < hsh[s * d + ord[a]]) { int t = ord[a]; ord[a] = ord[b]; ord[b] = t; }
        for (int h = 0; h < d; h++) {
            int jh = ord[h];
            ids[h] = hsh[s * d + jh];
            const uint8_t *chunk = base + (size_t)hsl[s * d + jh] * j->slice_len + s * (size_t)cs;
            for (int b = 0; b < beta; b++)
                memcpy(hb + (size_t)h * rb + b * sc, chunk + (size_t)pl[(s * d + jh) * beta + b] * sc, sc);
        }
        if (oc_clay_repair(c, ls[s], ids, d, hb, (size_t)cs, dst + s * (size_t)cs)) rc = -2;
    }
    memcpy(dst + ns * (size_t)cs, meta, OC_META);
    free(hb);
done:
    free(ls); free(hsl); free(hsh); free(pl);
    return rc;
}

/* node recover (network/node/src/features/spool/recover.rs:411-442): Slicer::decode from the
 * slices in masks[o], Slicer::encode of the blob, keep slice lost[o] */
static int recover_one(const many_job *j, int o) {
    const oc_clay *c = j->c;
    int av[OC_MAXQT], first = -1;
    for (int i = 0; i < c->n; i++) { av[i] = (j->masks[o] >> i) & 1; if (av[i] && first < 0) first = i; }
    if (first < 0) return -1;
    const uint8_t *base = j->slices + (size_t)o * j->obj_stride;
    const uint8_t *meta = base + (size_t)first * j->slice_len + j->slice_len - OC_META;
    uint64_t blob_len = get_u64(meta + 8), ci = get_u64(meta + 40);
    uint8_t *blob = (uint8_t *)malloc(blob_len ? blob_len : 1);
    long r = oc_slicer_decode(c, 1, base, av, j->slice_len, blob);
    if (r < 0) { free(blob); return (int)r; }
    size_t S, ns, cs, sl = oc_slicer_geometry(c, blob_len, &S, &ns, &cs);
    uint8_t *all = (uint8_t *)malloc((size_t)c->n * sl);
    oc_slicer_encode(c, 1, get_u64(meta + 24), get_u64(meta + 32), ci, blob, blob_len, all);
    memcpy(j->out + (size_t)o * j->out_stride, all + (size_t)j->lost[o] * sl, sl);
    free(all); free(blob);
    return 0;
}

static void *many_worker(void *arg) {
    many_job *j = (many_job *)arg;
    for (int o = j->tid; o < j->nobj; o += j->nthr) {
        int r = j->kind == 0 ? decode_one(j, o) : j->kind == 1 ? repair_one(j, o) : recover_one(j, o);
        if (r) j->status[o] = r;
    }
    return NULL;
}

/* kind 0 = decode, 1 = repair, 2 = recover; status[o] gets a negative code on failure (else 0).
 * Returns the number of failed objects. */
int oc_slicer_many(const oc_clay *c, int kind, const uint8_t *slices, size_t obj_stride, size_t slice_len,
                   const uint32_t *masks, const int *lost, const int *down, int nobj,
                   uint8_t *out, size_t out_stride, int nthr, int *status) {
    if (nthr < 1) nthr = 1;
    if (nthr > 256) nthr = 256;
    pthread_t th[256];
    many_job jobs[256];
    for (int o = 0; o < nobj; o++) status[o] = 0;
    for (int i = 0; i < nthr; i++) {
        many_job t = {c, slices, obj_stride, slice_len, masks, lost, down, out, out_stride, nobj, i, nthr, kind, status};
        jobs[i] = t;
        pthread_create(&th[i], NULL, many_worker, &jobs[i]);
    }
    for (int i = 0; i < nthr; i++) pthread_join(th[i], NULL);
    int bad = 0;
    for (int o = 0; o < nobj; o++) bad += status[o] != 0;
    return bad;
}
