// dec_class.hpp -- host side of the ahead-of-time decode class kernels (decode_class.hip, the
// kernels generated from this file at build time by gen_dec_class.cpp).
//
// Slicer::decode (lib/slicer/src/slicer.rs:298-364 -> ClayCoder::decode, clay.rs:106-122) of
// Clay(20,7,16) sees any 7 of the 20 slices: 77,520 survivor sets, each with its own layered-decode
// plane program.  The coupling structure of q = 10, t = 2 is invariant under relabelling the x
// digit of each column (a permutation pi_y of column y's nodes applied to plane digit z_y as well,
// A4: the PFT is symmetric), so two survivor sets related by such a relabelling have isomorphic
// programs.  Slicer::decode outputs the data nodes (0..6, all in column 0), so the relabellings
// that keep data nodes data nodes are S7 x S3 on column 0 and S10 on column 1.  Their orbits on
// 7-of-20 survivor sets are indexed by (a, b, c): a known data nodes, b known column-0 parity
// nodes (7..9), c known column-1 nodes, a + b + c = 7 -- 26 classes.
//
// The representative of class (a, b, c) keeps nodes {0..a-1, 7..7+b-1, 10..10+c-1}.  Its program
// (ClayHost::dec_prog) is written out as straight-line code once, at build time, with every node
// and plane symbolic: canonical known node j is the pattern's known[j], canonical erased node e
// its erased[e] (both lists ascending, and the relabelling is monotone on the known and on the
// erased nodes of each group, so the pattern's own decoding matrix D[e][j] is already in canonical
// order), canonical plane (z0, z1) is physical plane (pi_0(z0), pi_1(z1)).  At run time a kernel
// reads the pattern's node lists and decoding matrix (the device pattern store, as the table
// kernel does) and turns them into slice offsets and plane offsets once per workgroup; the
// program's control -- which loads, which products, where each value goes -- is compile-time.
// Products stay run-time v_perm table products (the matrix belongs to the survivor set).
#pragma once
#include <string>
#include <vector>
#include <cstdio>
#include "clay_host.hpp"

namespace tec {

constexpr int kDecClassN = 20, kDecClassK = 7, kDecClasses = 26;
constexpr uint32_t kDecClassNone = 0xffffffffu;

struct DecClassSpec {
    int a, b, c;  // known data nodes, known column-0 parity nodes, known column-1 nodes
};

inline DecClassSpec dec_class_spec(int id) {
    int i = 0;
    for (int b = 0; b <= 3; b++)
        for (int a = 0; a + b <= 7; a++, i++)
            if (i == id) return DecClassSpec{a, b, 7 - a - b};
    return DecClassSpec{-1, -1, -1};
}

inline int dec_class_index(int a, int b) {
    int i = 0;
    for (int bb = 0; bb <= 3; bb++)
        for (int aa = 0; aa + bb <= 7; aa++, i++)
            if (aa == a && bb == b) return i;
    return -1;
}

// The class of a padded pattern of Clay(20,7,16) (internal ids = node ids, nu = 0), or -1.
inline int dec_class_of(const ClayHost &h, const GpePattern &P) {
    if (h.n != kDecClassN || h.k != kDecClassK || h.q != kRepQ || h.t != 2 || h.nu != 0) return -1;
    if (P.nknown != (uint32_t)kDecClassK || P.nerased != (uint32_t)(kDecClassN - kDecClassK)) return -1;
    int a = 0, b = 0;
    for (uint32_t j = 0; j < P.nknown; j++) {
        a += P.known[j] < 7;
        b += P.known[j] >= 7 && P.known[j] < 10;
    }
    return dec_class_index(a, b);
}

// Canonical node c of class s: (known?, index into the pattern's known / erased list).
inline std::pair<bool, int> dec_class_slot(const DecClassSpec &s, int c) {
    if (c < 10) {
        if (c < s.a) return {true, c};
        if (c < 7) return {false, c - s.a};
        if (c < 7 + s.b) return {true, s.a + (c - 7)};
        return {false, (7 - s.a) + (c - 7 - s.b)};
    }
    const int r = c - 10;
    if (r < s.c) return {true, s.a + s.b + r};
    return {false, (7 - s.a) + (3 - s.b) + (r - s.c)};
}

inline uint64_t dec_class_emask(const DecClassSpec &s) {
    uint64_t m = 0;
    for (int c = 0; c < kDecClassN; c++)
        if (!dec_class_slot(s, c).first) m |= 1ull << c;
    return m;
}

// Program of class `id`'s representative, in the orientation decode_enqueue's table path prefers
// (two workgroups per CU first, then fewer scratch rows).
inline bool dec_class_prog(const ClayHost &h, int id, GpePattern &P, DecProgHdr &H, std::vector<DecStep> &steps) {
    const DecClassSpec s = dec_class_spec(id);
    std::vector<uint16_t> pool;
    if (s.a < 0 || !h.gpe_pattern(dec_class_emask(s), P, pool)) return false;
    bool found = false;
    for (int orient = 0; orient < 2; orient++) {
        DecProgHdr H1;
        std::vector<DecStep> st;
        if (!h.dec_prog(P, orient, H1, st)) continue;
        const auto cost = [](const DecProgHdr &x) { return (x.nslots + 2 > 53 ? 1u << 20 : 0u) + x.nscratch; };
        if (!found || cost(H1) < cost(H)) { H = H1; steps.swap(st); found = true; }
    }
    return found;
}

// LDS bytes of a class kernel with G waves per workgroup (lane-private slot rows, 4 B per lane).
inline size_t dec_class_lds(uint32_t nslots, int G) { return (size_t)(nslots ? nslots : 1) * G * 64u * 4u; }

// Kernel source of class `id` (one translation unit; decode_class_dev.hpp has the helpers).
// t_u: the type-1 coefficient (C = t_u (U ^ Cp) ^ Cp).
inline std::string dec_class_source(const ClayHost &h, int id, uint8_t t_u, DecProgHdr &Hout) {
    GpePattern P;
    DecProgHdr H;
    std::vector<DecStep> steps;
    if (!dec_class_prog(h, id, P, H, steps)) return std::string();
    Hout = H;
    const DecClassSpec cs = dec_class_spec(id);
    const int NK = (int)P.nknown, NE = (int)P.nerased, NS = (int)steps.size();
    std::string s;
    char b[320];
    auto emit = [&](const char *fmt, auto... v) {
        snprintf(b, sizeof b, fmt, v...);
        s += b;
    };
    auto lty = [](uint32_t loc) { return loc >> 24; };
    auto lix = [](uint32_t loc) { return loc & 0xffffffu; };
    auto id2 = [](int a, int c) { return std::to_string(a) + "_" + std::to_string(c); };
    // a canonical node as the expression of its physical id
    auto phys = [&](int c) {
        const auto sl = dec_class_slot(cs, c);
        return std::string(sl.first ? "T.K(" : "T.E(") + std::to_string(sl.second) + ")";
    };
    auto kidx = [&](int node) {  // index of a known canonical node in the known list
        const auto sl = dec_class_slot(cs, node);
        return sl.first ? sl.second : -1;
    };
    emit("// generated by gen_dec_class (dec_class.hpp): class %d = (a %d, b %d, c %d), %d steps, %u slots, "
         "%u scratch rows\n", id, cs.a, cs.b, cs.c, NS, H.nslots, H.nscratch);
    s += "#include \"decode_class_dev.hpp\"\nnamespace tec {\nnamespace dcls {\n";
    emit("template <int G>\n__global__ void __attribute__((amdgpu_flat_work_group_size(1, G * 64), amdgpu_waves_per_eu(4)))\n"
         "dec_class_%d(DecClassArgs a) {\n", id);
    s += "  extern __shared__ __attribute__((aligned(16))) u32 lds[];\n  CTile<G> T(a, reinterpret_cast<u8 *>(lds));\n";
    // per-workgroup offsets: known slices, plane digits, data chunks (only what the program uses;
    // the rest is dead code)
    for (int j = 0; j < NK; j++) emit("  const u32 kb%d = T.kbase(T.K(%d));\n", j, j);
    for (int x = 0; x < 10; x++) emit("  const u32 pz0_%d = %s * 10u * T.sc;\n", x, phys(x).c_str());
    for (int x = 0; x < 10; x++) emit("  const u32 pz1_%d = (%s - 10u) * T.sc;\n", x, phys(10 + x).c_str());
    for (int x = 0; x < kDecClassK; x++) emit("  const u32 ob%d = %s * T.out_stride;\n", x, phys(x).c_str());
    auto poff = [&](uint32_t z) {
        return "pz0_" + std::to_string(z / 10) + " + pz1_" + std::to_string(z % 10);
    };
    auto loads = [&](int st) {
        if (st >= NS) return;
        const DecStep &S = steps[st];
        for (int j = 0; j < NK; j++) {
            emit("  const u32 o%s = T.ld_own(kb%d, %s);\n", id2(st, j).c_str(), j, poff(S.z).c_str());
            if (S.kk[j] == kKnInput)
                emit("  const u32 p%s = T.ld(kb%d, %s);\n", id2(st, j).c_str(), kidx((int)(S.kp[j] & 0xffu)),
                     poff(S.kp[j] >> 8).c_str());
        }
        for (int e = 0; e < NE; e++)
            if (S.ek[e] == kErType1)
                emit("  const u32 t%s = T.ld(kb%d, %s);\n", id2(st, e).c_str(), kidx((int)(S.ep[e] & 0xffu)),
                     poff(S.ep[e] >> 8).c_str());
    };
    auto scr_loads = [&](int st) {
        if (st >= NS) return;
        const DecStep &S = steps[st];
        for (int j = 0; j < NK; j++)
            if (S.kk[j] == kKnLoc && lty(S.kp[j]) == kLocScratch) emit("  const u32 q%s = T.scr_ld(%u);\n", id2(st, j).c_str(), lix(S.kp[j]));
        for (int e = 0; e < NE; e++)
            if (S.ek[e] == kErFinish && lty(S.ep[e]) == kLocScratch) emit("  const u32 r%s = T.scr_ld(%u);\n", id2(st, e).c_str(), lix(S.ep[e]));
    };
    loads(0);
    scr_loads(0);
    for (int st = 0; st < NS; st++) {
        const DecStep &S = steps[st];
        auto put = [&](uint32_t loc, const std::string &v) {
            if (loc == kLocNone) return;
            if (lty(loc) == kLocStage) {
                const uint32_t it = S.out[lix(loc)];
                emit("  T.out_st(ob%u, %s, %s);\n", it & 0xffu, poff((it >> 8) & 0xffu).c_str(), v.c_str());
            } else if (lty(loc) == kLocSlot) {
                emit("  T.lds_st(%u, %s);\n", lix(loc), v.c_str());
            } else {
                emit("  T.scr_st(%u, %s);\n", lix(loc), v.c_str());
            }
        };
        emit("  // step %d: plane (%u, %u)\n", st, S.z / 10, S.z % 10);
        loads(st + 1);
        // uncouple the known nodes (known data rows are copied out as they are)
        for (int j = 0; j < NK; j++) {
            const std::string id = id2(st, j);
            const char *i = id.c_str();
            if (S.kk[j] == kKnRed) emit("  const u32 u%s = o%s;\n", i, i);
            else if (S.kk[j] == kKnInput) emit("  const u32 u%s = pft3(o%s, p%s);\n", i, i, i);
            else if (lty(S.kp[j]) == kLocSlot) emit("  const u32 u%s = pft3(o%s, T.lds_ld(%u));\n", i, i, lix(S.kp[j]));
            else emit("  const u32 u%s = pft3(o%s, q%s);\n", i, i, i);
            put(S.kout[j], "o" + id);
        }
        // pair partners' U, read before this step's writes
        for (int e = 0; e < NE; e++) {
            if (S.ek[e] != kErFinish) continue;
            const std::string id = id2(st, e);
            if (lty(S.ep[e]) == kLocSlot) emit("  const u32 v%s = T.lds_ld(%u);\n", id.c_str(), lix(S.ep[e]));
            else emit("  const u32 v%s = r%s;\n", id.c_str(), id.c_str());
        }
        // MDS: the erased U's this step needs, v_perm products against the pattern's matrix
        bool any = false;
        for (int e = 0; e < NE; e++) any = any || S.ek[e] != kErSkip;
        if (any) {
            for (int j = 0; j < NK; j++) emit("  const Sel s%s(u%s);\n", id2(st, j).c_str(), id2(st, j).c_str());
            for (int e = 0; e < NE; e++) {
                if (S.ek[e] == kErSkip) continue;
                const std::string a = "a" + id2(st, e);
                emit("  u32 %s = 0u;\n  { const auto D = T.mat();\n", a.c_str());
                for (int j = 0; j + 1 < NK; j += 2)
                    emit("  %s = T.mul2(%s, D, %d, %d, s%s, s%s);\n", a.c_str(), a.c_str(), e, j, id2(st, j).c_str(),
                         id2(st, j + 1).c_str());
                if (NK & 1) emit("  %s = T.mul1(%s, D, %d, %d, s%s);\n", a.c_str(), a.c_str(), e, NK - 1, id2(st, NK - 1).c_str());
                s += "  }\n";
                // the result right away (a data row out, a parked / type-1 value to a slot or
                // scratch): its store keeps the next row's table loads from being hoisted here
                const std::string id = id2(st, e);
                const char *i = id.c_str();
                switch (S.ek[e]) {
                    case kErRed: put(S.ed0[e], a); break;
                    case kErType1: {  // C = t_u (U ^ Cp) ^ Cp
                        emit("  const u32 y%s_0 = %s ^ t%s;\n", i, a.c_str(), i);
                        std::string r;
                        for (int bit = 0; bit < 8 && (t_u >> bit); bit++) {
                            if (bit) emit("  const u32 y%s_%d = xt(y%s_%d);\n", i, bit, i, bit - 1);
                            if ((t_u >> bit) & 1) r += (r.empty() ? "" : " ^ ") + ("y" + id + "_" + std::to_string(bit));
                        }
                        emit("  const u32 w%s = %s ^ t%s;\n", i, r.empty() ? "0u" : r.c_str(), i);
                        put(S.ed0[e], "w" + id);
                        put(S.ed1[e], "w" + id);
                        break;
                    }
                    case kErPark: put(S.ep[e], a); break;
                    case kErFinish:
                        put(S.ed0[e], "pft3(" + a + ", v" + id + ")");
                        put(S.epd[e], "pft3(v" + id + ", " + a + ")");
                        break;
                    default: break;
                }
            }
        }
        scr_loads(st + 1);
    }
    s += "}\n";
    emit("template __global__ void dec_class_%d<1>(DecClassArgs);\ntemplate __global__ void dec_class_%d<2>(DecClassArgs);\n", id, id);
    emit("void dec_class_reg_%d(DecClassEntry &e) {\n  e.fn[0] = reinterpret_cast<const void *>(&dec_class_%d<1>);\n"
         "  e.fn[1] = reinterpret_cast<const void *>(&dec_class_%d<2>);\n  e.nslots = %uu;\n  e.nscratch = %uu;\n}\n",
         id, id, id, H.nslots, H.nscratch);
    s += "}  // namespace dcls\n}  // namespace tec\n";
    return s;
}

}  // namespace tec
