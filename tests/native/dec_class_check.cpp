// Host check of the decode / recover class kernels' relabelling (tape_amd/csrc/dec_class.hpp):
// the class representative's plane program, with every node and plane mapped through the
// survivor set's relabelling exactly as the generated kernels map them (canonical known node j ->
// the pattern's known[j], canonical erased node e -> erased[e], canonical plane digit -> the
// physical node's x), interpreted byte by byte with the pattern's own 2-bit-field tables (D4), must
// reproduce the data chunks (decode) or the lost node's chunk (recover) of a stripe encoded by the
// oracle (oracle/clay_oracle.c).  Decode: all 77,520 survivor sets of Clay(20,7,16); recover:
// every lost node of a sample of them.  Built and run by tests/test_dec_class_host.py.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>
#include "dec_class.hpp"

extern "C" {
int oc_clay_sizeof(void);
int oc_clay_init(void *c, int n, int k, int d);
size_t oc_chunk_size_for(const void *c, size_t input_len);
int oc_clay_encode(const void *c, const uint8_t *data, size_t len, uint8_t *out);
}

using namespace tec;

static uint8_t mul4(const uint32_t t[4], uint8_t x) {  // PermTab4 product, one byte
    uint8_t r = 0;
    for (int f = 0; f < 4; f++) r ^= (uint8_t)(t[f] >> (8 * ((x >> (2 * f)) & 3)));
    return r;
}
static uint8_t pft3(uint8_t a, uint8_t b) { return (uint8_t)(a ^ gf_mul(2, (uint8_t)(a ^ b))); }

struct Prog {
    GpePattern P0;
    DecProgHdr H;
    std::vector<DecStep> steps;
};

// Interpret class `id`'s program on pattern P (physical).  Returns false on a wrong byte.
// id < 0: a pattern's own program (ClayHost::dec_prog, physical nodes and planes, data output),
// as the hipRTC pattern kernels run it
static bool run(const Prog &pg, int id, const GpePattern &P, const uint8_t *chunks, size_t cs, size_t sc, int lost) {
    const DecClassSpec s = dec_class_spec(id < 0 ? 0 : id);
    const int NK = (int)P.nknown, NE = (int)P.nerased;
    auto phys = [&](int c) {
        if (id < 0) return c;
        const auto sl = dec_class_slot(s, c);
        return sl.first ? (int)P.known[sl.second] : (int)P.erased[sl.second];
    };
    auto kidx = [&](int c) {
        if (id >= 0) return dec_class_slot(s, c).second;
        for (int j = 0; j < NK; j++)
            if ((int)P.known[j] == c) return j;
        return 0;
    };
    // a wrong program (the negative check) can map a digit to the other column: -1, never indexed
    auto plane = [&](uint32_t z) {
        if (id < 0) return (int)z;
        const int d0 = phys((int)z / 10), d1 = phys(10 + (int)z % 10) - 10;
        return d0 >= 0 && d0 < 10 && d1 >= 0 && d1 < 10 ? d0 * 10 + d1 : -1;
    };
    bool wrong = false;
    const size_t outn = lost < 0 ? (size_t)kDecClassK * cs : cs;
    std::vector<uint8_t> out(outn, 0xEE);
    uint8_t slot[512], scr[512];
    bool slot_ok[512], scr_ok[512];
    auto in = [&](int node, int z, size_t b) {
        if (node < 0 || node >= 20 || z < 0) {
            wrong = true;
            return (uint8_t)0x5A;
        }
        return chunks[(size_t)node * cs + (size_t)z * sc + b];
    };
    for (size_t b = 0; b < sc; b++) {
        memset(slot_ok, 0, sizeof slot_ok);
        memset(scr_ok, 0, sizeof scr_ok);
        for (const DecStep &S : pg.steps) {
            const int zp = plane(S.z);
            auto put = [&](uint32_t loc, uint8_t v) {
                if (loc == kLocNone) return;
                const uint32_t ty = loc >> 24, ix = loc & 0xffffffu;
                if (ty == kLocStage) {
                    const uint32_t it = S.out[ix];
                    const int node = phys((int)(it & 0xffu)), zz = plane((it >> 8) & 0xffu);
                    if (zz < 0) {
                        wrong = true;
                        return;
                    }
                    if (lost < 0 && node < kDecClassK) out[(size_t)node * cs + (size_t)zz * sc + b] = v;
                    if (lost >= 0 && node == lost) out[(size_t)zz * sc + b] = v;
                } else if (ix < 512) {
                    (ty == kLocSlot ? slot : scr)[ix] = v;
                    (ty == kLocSlot ? slot_ok : scr_ok)[ix] = true;
                }
            };
            auto get = [&](uint32_t loc) {
                const uint32_t ty = loc >> 24, ix = loc & 0xffffffu;
                if (ix >= 512) return (uint8_t)0x5A;
                return (ty == kLocSlot ? slot_ok : scr_ok)[ix] ? (ty == kLocSlot ? slot : scr)[ix] : (uint8_t)0x5A;
            };
            uint8_t u[kDecMaxK], v[kDecMaxE] = {};
            struct Pend { int j; uint8_t p, o; };
            std::vector<Pend> pend;
            for (int j = 0; j < NK; j++) {
                const uint8_t o = in((int)P.known[j], zp, b);
                if (S.kk[j] == kKnPark) {  // U parked by the type-1 step; the row is not read here
                    u[j] = get(S.kp[j]);
                    continue;
                }
                if (S.kk[j] == kKnRed) u[j] = o;
                else if (S.kk[j] == kKnInput || S.kk[j] == kKnInputU) {
                    const uint8_t pv = in((int)P.known[kidx((int)(S.kp[j] & 0xffu))], plane(S.kp[j] >> 8), b);
                    u[j] = pft3(o, pv);
                    if (S.kk[j] == kKnInputU) pend.push_back({j, pv, o});
                }
                else u[j] = pft3(o, get(S.kp[j]));
                put(S.kout[j], o);
            }
            for (int e = 0; e < NE; e++)
                if (S.ek[e] == kErFinish) v[e] = get(S.ep[e]);
            for (const auto &q : pend) {  // in-row pairs, after the step's reads
                put(S.kpark[q.j], pft3(q.p, q.o));
                put(S.kpout[q.j], q.p);
            }
            for (int e = 0; e < NE; e++) {
                if (S.ek[e] == kErSkip) continue;
                uint8_t a = 0;
                for (int j = 0; j < NK; j++) a ^= mul4(P.D4[e][j], u[j]);
                switch (S.ek[e]) {
                    case kErRed: put(S.ed0[e], a); break;
                    case kErType1:
                    case kErType1U: {
                        const uint8_t k = in((int)P.known[kidx((int)(S.ep[e] & 0xffu))], plane(S.ep[e] >> 8), b);
                        const uint8_t w = (uint8_t)(gf_mul(kPft.t_u[0], (uint8_t)(a ^ k)) ^ k);
                        if (S.ek[e] == kErType1U) {
                            put(S.ed0[e], pft3(k, w));
                            put(S.epd[e], k);
                        } else {
                            put(S.ed0[e], w);
                        }
                        put(S.ed1[e], w);
                        break;
                    }
                    case kErPark: put(S.ep[e], a); break;
                    case kErFinish:
                        put(S.ed0[e], pft3(a, v[e]));
                        put(S.epd[e], pft3(v[e], a));
                        break;
                    default: break;
                }
            }
        }
    }
    if (wrong) return false;
    if (lost < 0) return memcmp(out.data(), chunks, outn) == 0;
    return memcmp(out.data(), chunks + (size_t)lost * cs, cs) == 0;
}

int main(int argc, char **argv) {
    const int recover_every = argc > 1 ? atoi(argv[1]) : 20;  // recover: every lost node of 1 in N sets
    ClayHost h;
    if (h.init(20, 7, 16) != 0) return 2;
    std::vector<uint8_t> oc((size_t)oc_clay_sizeof());
    oc_clay_init(oc.data(), 20, 7, 16);
    const size_t len = 2800;  // sc = 2 bytes: chunk 200 B
    const size_t cs = oc_chunk_size_for(oc.data(), len), sc = cs / 100;
    std::vector<uint8_t> data(len), chunks(20 * cs);
    std::mt19937 rng(7);
    for (auto &x : data) x = (uint8_t)rng();
    if (oc_clay_encode(oc.data(), data.data(), len, chunks.data()) != 0) return 2;
    std::vector<Prog> progs(kDecClasses);
    for (int id = 0; id < kDecClasses; id++)
        if (!dec_class_prog(h, id, progs[id].P0, progs[id].H, progs[id].steps)) {
            printf("FAIL no program for class %d\n", id);
            return 1;
        }
    long count[kDecClasses] = {}, bad = 0, rec_runs = 0, sets = 0;
    std::vector<uint16_t> pool;
    for (uint32_t m = 0; m < (1u << 20); m++) {
        if (__builtin_popcount(m) != 7) continue;
        const uint64_t emask = (~(uint64_t)m) & 0xfffffull;
        GpePattern P;
        pool.clear();
        if (!h.gpe_pattern(emask, P, pool)) return 2;
        const int id = dec_class_of(h, P);
        if (id < 0 || id >= kDecClassesDecode) {
            printf("FAIL no decode class for mask %05x\n", m);
            return 1;
        }
        count[id]++;
        if (!run(progs[id], id, P, chunks.data(), cs, sc, -1)) {
            printf("FAIL decode mask %05x class %d\n", m, id);
            bad++;
        }
        if (sets++ % recover_every == 0)
            for (int lost = 0; lost < 20; lost++) {
                if (!((emask >> lost) & 1ull)) continue;
                GpePattern R = P;
                dec_class_lost_first(R, lost);
                const int rid = dec_class_of(h, R, lost);
                if (rid < kDecClassesDecode) {
                    printf("FAIL no recover class for mask %05x lost %d\n", m, lost);
                    return 1;
                }
                count[rid]++;
                rec_runs++;
                if (!run(progs[rid], rid, R, chunks.data(), cs, sc, lost)) {
                    printf("FAIL recover mask %05x lost %d class %d\n", m, lost, rid);
                    bad++;
                }
            }
    }
    // the patterns' own programs with the in-row pair and type-1 fusions (the hipRTC kernels' form): every 61st
    // erasure set of every size 1..13, both row orientations
    long plain = 0, plain_fused = 0;
    for (uint32_t m = 1, seen_p = 0; m < (1u << 20); m++) {
        const int ne = __builtin_popcount(m);
        if (ne > 13 || seen_p++ % 61) continue;
        GpePattern P;
        pool.clear();
        if (!h.gpe_pattern(h.pad_erasures(m), P, pool)) return 2;
        for (int orient = 0; orient < 2; orient++) {
            Prog pg;
            if (!h.dec_prog(P, orient, pg.H, pg.steps, -1, 0, true)) continue;
            plain_fused += dec_prog_fuse_type1(P, pg.steps);
            plain++;
            if (!run(pg, -1, P, chunks.data(), cs, sc, -1)) {
                printf("FAIL pattern program mask %05x orient %d\n", m, orient);
                bad++;
            }
        }
    }
    // the check can fail: the neighbouring class's program on a pattern must not reproduce it
    long caught = 0, tried = 0;
    long seen = 0;
    for (uint32_t m = 0; m < (1u << 20) && tried < 200; m++) {
        if (__builtin_popcount(m) != 7 || seen++ % 300) continue;
        GpePattern P;
        pool.clear();
        if (!h.gpe_pattern((~(uint64_t)m) & 0xfffffull, P, pool)) return 2;
        const int id = dec_class_of(h, P), wrong = (id + 1) % kDecClassesDecode;
        tried++;
        caught += !run(progs[wrong], wrong, P, chunks.data(), cs, sc, -1);
    }
    if (caught != tried) {
        printf("FAIL a wrong class program passed (%ld of %ld caught)\n", caught, tried);
        return 1;
    }
    printf("sets %ld recover %ld patterns %ld (fused pairs %ld) bad %ld wrong-class caught %ld/%ld counts", sets, rec_runs,
           plain, plain_fused, bad, caught, tried);
    for (int id = 0; id < kDecClasses; id++) printf(" %ld", count[id]);
    printf("\n");
    return bad ? 1 : 0;
}
