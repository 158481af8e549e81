// dec_class.hpp -- host side of the ahead-of-time decode class kernels (decode_class.hip, the
// kernels generated from this file at build time by gen_dec_class.cpp).
//
// Slicer::decode (lib/slicer/src/slicer.rs:298-364 -> ClayCoder::decode, clay.rs:106-122) of
// Clay(20,7,16) sees any 7 of the 20 slices: 77,520 survivor sets, each with its own layered-decode
// plane program.  The coupling structure of q = 10, t = 2 is invariant under relabelling the x
// digit of each column (a permutation pi_y of column y's nodes applied to plane digit z_y as well,
// A4: the PFT is symmetric), so survivor sets related by such a relabelling have isomorphic
// programs.  The class programs output every erased node of column 0 -- the data nodes 0..6 and
// the column-0 parity nodes 7..9 alike (dec_prog's out_mask) -- and the kernel drops the stores
// of the parity ones, so the relabellings are all of S10 x S10 and the classes are indexed by a0,
// the number of known column-0 nodes (0..7; the rest of the 7 are in column 1): 8 classes.
// Treating the three column-0 parity nodes as outputs costs ~5 % more MDS products (weighted over
// all survivor sets; 0 - 16 % by class) and saves the launches that 26 data-only classes needed
// (one launch's floor is a stripe's 100-step chain, whatever its size).
//
// The representative of class a0 keeps nodes {0..a0-1} and {10..10+(7-a0)-1}.  Its program
// (ClayHost::dec_prog) is written out as straight-line code once, at build time, with every node
// and plane symbolic: canonical known node j is the pattern's known[j], canonical erased node e
// its erased[e] (both lists ascending, and the relabelling is monotone on the known and on the
// erased nodes of each column, so the pattern's own decoding matrix D[e][j] is already in
// canonical order), canonical plane (z0, z1) is physical plane (pi_0(z0), pi_1(z1)).  At run time
// a kernel reads the pattern's node lists and decoding matrix (the device pattern store, as the
// table kernel does) and turns them into slice offsets and plane offsets once per workgroup; the
// program's control -- which loads, which products, where each value goes -- is compile-time.
// Products stay run-time v_perm table products (the matrix belongs to the survivor set).
#pragma once
#include <string>
#include <vector>
#include <cstdio>
#include "clay_host.hpp"

namespace tec {

// Classes 0..7: Slicer::decode, a0 known column-0 nodes.  Classes 8..23: node recover
// (recover.rs:411-442, dec_prog's out_node), 8 + 2 a0 + yL: the lost node is in column yL.  For
// recover the one output is the lost node, so data and parity nodes are alike and the same S10 x
// S10 relabellings apply once the lost node is fixed: the pattern's erased list puts the lost node
// first among its column's erased nodes (dec_class_lost_first, with the matrix rows), and the
// representative's lost node is the first erased node of column yL.
constexpr int kDecClassN = 20, kDecClassK = 7, kDecClassesDecode = 8, kDecClasses = 24;
constexpr int kDecClassSplit = 4;  // per-call kernel: waves sharing one 64-column group
constexpr uint64_t kDecClassOutMask = 0x3ffull;  // decode: every column-0 node is an output

struct DecClassSpec {
    int a0;  // known column-0 nodes (the other 7 - a0 known nodes are in column 1)
    int yl;  // recover: the lost node's column; -1 for decode
};

inline DecClassSpec dec_class_spec(int id) {
    if (id < 0 || id >= kDecClasses) return DecClassSpec{-1, -1};
    if (id < kDecClassesDecode) return DecClassSpec{id, -1};
    return DecClassSpec{(id - kDecClassesDecode) / 2, (id - kDecClassesDecode) % 2};
}

// The class of a padded pattern of Clay(20,7,16) (internal ids = node ids, nu = 0), or -1.
// lost >= 0: the recover class of (P, lost node), P's erased list already lost-first.
inline int dec_class_of(const ClayHost &h, const GpePattern &P, int lost = -1) {
    if (h.n != kDecClassN || h.k != kDecClassK || h.q != kRepQ || h.t != 2 || h.nu != 0) return -1;
    if (P.nknown != (uint32_t)kDecClassK || P.nerased != (uint32_t)(kDecClassN - kDecClassK)) return -1;
    int a0 = 0;
    for (uint32_t j = 0; j < P.nknown; j++) a0 += P.known[j] < 10;
    if (lost < 0) return a0;
    if (lost >= kDecClassN || !((P.erased_mask >> lost) & 1ull)) return -1;
    const int yl = lost / 10;
    const uint32_t first = yl == 0 ? 0u : (uint32_t)(10 - a0);  // the lost node's place in the erased list
    if (P.erased[first] != (uint32_t)lost) return -1;
    return kDecClassesDecode + 2 * a0 + yl;
}

// Put the lost node first among its column's erased nodes (P.erased and the matrix rows D, D4),
// the order the recover class kernels' relabelling assumes.  Every program compiled from P after
// this follows the same order.
inline void dec_class_lost_first(GpePattern &P, int lost) {
    int at = -1, first = -1;
    for (uint32_t e = 0; e < P.nerased; e++) {
        if ((int)P.erased[e] == lost) at = (int)e;
        if (first < 0 && (int)P.erased[e] / 10 == lost / 10) first = (int)e;
    }
    if (at < 0 || first < 0 || at == first) return;
    for (int e = at; e > first; e--) {  // rotate [first, at] right by one
        std::swap(P.erased[e], P.erased[e - 1]);
        for (int j = 0; j < kGpeMaxKnown; j++) std::swap(P.D[e][j], P.D[e - 1][j]);
        if (e < kClsMaxE)
            for (int j = 0; j < kClsMaxK; j++)
                for (int f = 0; f < 4; f++) std::swap(P.D4[e][j][f], P.D4[e - 1][j][f]);
    }
}

// Canonical node c of class s: (known?, index into the pattern's known / erased list).
inline std::pair<bool, int> dec_class_slot(const DecClassSpec &s, int c) {
    if (c < 10) return c < s.a0 ? std::make_pair(true, c) : std::make_pair(false, c - s.a0);
    const int r = c - 10, c1 = kDecClassK - s.a0;
    return r < c1 ? std::make_pair(true, s.a0 + r) : std::make_pair(false, (10 - s.a0) + (r - c1));
}

inline uint64_t dec_class_emask(const DecClassSpec &s) {
    uint64_t m = 0;
    for (int c = 0; c < kDecClassN; c++)
        if (!dec_class_slot(s, c).first) m |= 1ull << c;
    return m;
}

// Program of class `id`'s representative: of the two row orientations the one with fewer
// scratch rows (HBM traffic), then fewer MDS rows (VALU), within the LDS of two workgroups per CU.
inline bool dec_class_prog(const ClayHost &h, int id, GpePattern &P, DecProgHdr &H, std::vector<DecStep> &steps,
                           bool fuse = true, bool pairs = true) {
    const DecClassSpec s = dec_class_spec(id);
    std::vector<uint16_t> pool;
    if (s.a0 < 0 || !h.gpe_pattern(dec_class_emask(s), P, pool)) return false;
    bool found = false;
    uint64_t best = 0;
    for (int orient = 0; orient < 2; orient++) {
        DecProgHdr H1;
        std::vector<DecStep> st;
        const uint64_t out_mask = s.yl < 0 ? kDecClassOutMask : 1ull << (s.yl == 0 ? s.a0 : 10 + (kDecClassK - s.a0));
        if (!h.dec_prog(P, orient, H1, st, -1, out_mask, pairs)) continue;
        uint64_t rows = 0;
        for (const DecStep &S : st)
            for (uint32_t e = 0; e < P.nerased; e++) rows += S.ek[e] != kErSkip;
        const uint64_t cost = (H1.nslots + 2 > 53 ? 1ull << 40 : 0ull) + ((uint64_t)H1.nscratch << 20) + rows;
        if (!found || cost < best) { H = H1; steps.swap(st); best = cost; found = true; }
    }
    if (found && fuse) dec_prog_fuse_type1(P, steps);
    return found;
}

// LDS bytes of a class kernel: the batch kernel (G = 2) holds its lane-private slot rows, the
// per-call kernel (G = 1, kDecClassSplit waves on one 64-column group) every slot and scratch row.
inline size_t dec_class_lds(uint32_t nslots, uint32_t nscratch, uint32_t nring, int G) {
    const uint32_t rows = G == 1 ? 2 * nring + nslots + nscratch : nslots;
    return (size_t)(rows ? rows : 1) * G * 64u * 4u;
}

// Kernel source of class `id` (one translation unit; decode_class_dev.hpp has the helpers).
// t_u: the type-1 coefficient (C = t_u (U ^ Cp) ^ Cp).
// Generator options (build-time variants for A/B runs; the defaults are what the library ships):
// wpe = the waves-per-SIMD register budget, late = a step's loads for the next step issued after
// its products instead of at its start.
struct DecClassGenOpt {
    int wpe = 4;
    int deep = 4;  // the per-call kernel's input-load lead, in steps
    bool late = false;
    bool tab4 = true;  // 2-bit-field product tables (PermTab4); false: the 3/3/2-bit PermTab
    int own_aux = 2;   // cache policy of the batch kernel's own-row loads (2: non-temporal)
    int scr_aux = 0;   // ... and of its scratch loads (each scratch row is read once)
    bool fuse = true;   // dec_prog_fuse_type1
    bool pairs = true;  // dec_prog fuse_pairs
    bool tu_perm = true;  // type-1 coefficient as a v_perm table product (false: xtime chain)
    bool drop_branch = true;  // out_st skips a dropped row with a uniform branch (false: range check)
    bool drop_pairs = false;  // decode: skip column-0 pairs whose nodes are both parity (slower: the
                              // 420 uniform branches per kernel cost more scheduling than the rows)
};

inline std::string dec_class_source(const ClayHost &h, int id, uint8_t t_u, DecProgHdr &Hout,
                                    const DecClassGenOpt &opt = DecClassGenOpt()) {
    GpePattern P;
    DecProgHdr H;
    std::vector<DecStep> steps;
    if (!dec_class_prog(h, id, P, H, steps, opt.fuse, opt.pairs)) return std::string();
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
    const PermTab tu_tab = perm_tab(t_u), tu2_tab = perm_tab(gf_mul(2, t_u));
    // a canonical node as the expression of its physical id
    auto phys = [&](int c) {
        const auto sl = dec_class_slot(cs, c);
        return std::string(sl.first ? "T.K(" : "T.E(") + std::to_string(sl.second) + ")";
    };
    auto kidx = [&](int node) {  // index of a known canonical node in the known list
        const auto sl = dec_class_slot(cs, node);
        return sl.first ? sl.second : -1;
    };
    emit("// generated by gen_dec_class (dec_class.hpp): class %d = %d known column-0 nodes, %s, %d steps, %u slots, "
         "%u scratch rows\n", id, cs.a0, cs.yl < 0 ? "decode" : cs.yl == 0 ? "recover, lost node in column 0" :
         "recover, lost node in column 1", NS, H.nslots, H.nscratch);
    s += "#include \"decode_class_dev.hpp\"\nnamespace tec {\nnamespace dcls {\n";
    // One body, two kernels: the batch kernel (G = 2 waves per workgroup, the register budget of
    // opt.wpe waves per SIMD, each step's input loads issued one step ahead) and the per-call
    // kernel (one wave per workgroup, few waves on the chip, so registers are free: the input
    // loads -- read-only slices, never written by the kernel -- issued `deep` steps ahead, which
    // takes the global-memory latency off a lone wave's 100-step chain).  Scratch loads keep
    // their place after the previous step's stores.
    // the per-call kernel's input ring: per step, its own rows, input partners and type-1
    // partners, in that order (ring row i of the step's slot)
    uint32_t nring = 1;
    for (const DecStep &S : steps) {
        uint32_t c = 0;
        for (int j = 0; j < NK; j++) c += (S.kk[j] != kKnPark) + (S.kk[j] == kKnInput || S.kk[j] == kKnInputU);
        for (int e = 0; e < NE; e++) c += S.ek[e] == kErType1 || S.ek[e] == kErType1U;
        nring = std::max(nring, c);
    }
    auto body = [&](bool small) {
    const int depth = small ? opt.deep : 1, W = small ? kDecClassSplit : 1;
    // the per-call kernel: W compute waves share one 64-column group and a loader wave (wv == W)
    // brings each step's input rows into a two-slot LDS ring a step ahead, issuing its global
    // loads `depth` steps ahead (gfx9 counts loads and stores on one vmcnt, so compute waves that
    // loaded would wait on their own output stores every step); every parked value lives in LDS,
    // shared by the waves: ring rows first, then slots, then scratch rows
    const uint32_t ring0 = 0, slot0 = small ? 2 * nring : 0u, scr0 = small ? 2 * nring + H.nslots : 0u;
    if (small)
        emit("__global__ void __attribute__((amdgpu_flat_work_group_size(1, %d), amdgpu_waves_per_eu(1)))\n"
             "dec_class_%d_small(DecClassArgs a) {\n  constexpr int G = 1;\n", 64 * (W + 1), id);
    else
        emit("__global__ void __attribute__((amdgpu_flat_work_group_size(1, 128), amdgpu_waves_per_eu(%d)))\n"
             "dec_class_%d(DecClassArgs a) {\n  constexpr int G = 2;\n", opt.wpe, id);
    emit("  extern __shared__ __attribute__((aligned(16))) u32 lds[];\n  CTile<G, %d> T(a, reinterpret_cast<u8 *>(lds));\n", W);
    // per-workgroup offsets: known slices, plane digits, data chunks (only what the program uses;
    // the rest is dead code)
    for (int j = 0; j < NK; j++) emit("  const u32 kb%d = T.kbase(T.K(%d));\n", j, j);
    for (int x = 0; x < 10; x++) emit("  const u32 pz0_%d = %s * 10u * T.sc;\n", x, phys(x).c_str());
    for (int x = 0; x < 10; x++) emit("  const u32 pz1_%d = (%s - 10u) * T.sc;\n", x, phys(10 + x).c_str());
    // decode: column-0 outputs, a data chunk or dropped (a parity node: an offset past the range);
    // recover: the lost node's chunk is the job's whole output
    if (cs.yl < 0)
        for (int x = 0; x < 10; x++) emit("  const u32 ob%d = T.out_base(%s);\n", x, phys(x).c_str());
    else
        emit("  const u32 ob%d = 0u;\n", cs.yl == 0 ? cs.a0 : 10 + (kDecClassK - cs.a0));
    auto poff = [&](uint32_t z) {
        return "pz0_" + std::to_string(z / 10) + " + pz1_" + std::to_string(z % 10);
    };
    // per-call kernel: the step's input rows in ring order (expression of the global load)
    auto ring_list = [&](int st) {
        std::vector<std::string> L;
        const DecStep &S = steps[st];
        for (int j = 0; j < NK; j++)
            if (S.kk[j] != kKnPark) L.push_back("T.ld_own(kb" + std::to_string(j) + ", " + poff(S.z) + ")");
        for (int j = 0; j < NK; j++)
            if (S.kk[j] == kKnInput || S.kk[j] == kKnInputU) L.push_back("T.ld(kb" + std::to_string(kidx((int)(S.kp[j] & 0xffu))) + ", " + poff(S.kp[j] >> 8) + ")");
        for (int e = 0; e < NE; e++)
            if (S.ek[e] == kErType1 || S.ek[e] == kErType1U) L.push_back("T.ld(kb" + std::to_string(kidx((int)(S.ep[e] & 0xffu))) + ", " + poff(S.ep[e] >> 8) + ")");
        return L;
    };
    auto ring_row = [&](int st, int i) { return ring0 + (uint32_t)(st & 1) * nring + (uint32_t)i; };
    // loader: issue step st's global loads into L<st>_i (declared at function scope)
    auto loader_issue = [&](int st) {
        if (st >= NS) return;
        const auto L = ring_list(st);
        for (size_t i = 0; i < L.size(); i++) emit("  L%d_%zu = %s;\n", st, i, L[i].c_str());
    };
    auto loader_put = [&](int st) {  // loader: step st's rows into its ring slot
        if (st >= NS) return;
        const auto L = ring_list(st);
        for (size_t i = 0; i < L.size(); i++) emit("  T.lds_st(%u, L%d_%zu);\n", ring_row(st, (int)i), st, i);
    };
    auto loads = [&](int st) {
        if (st >= NS || small) return;
        const DecStep &S = steps[st];
        for (int j = 0; j < NK; j++) {
            if (S.kk[j] != kKnPark)
                emit("  const u32 o%s = T.ld_aux<%d>(kb%d, %s);\n", id2(st, j).c_str(), opt.own_aux, j, poff(S.z).c_str());
            if (S.kk[j] == kKnInput || S.kk[j] == kKnInputU)
                emit("  const u32 p%s = T.ld(kb%d, %s);\n", id2(st, j).c_str(), kidx((int)(S.kp[j] & 0xffu)),
                     poff(S.kp[j] >> 8).c_str());
        }
        for (int e = 0; e < NE; e++)
            if (S.ek[e] == kErType1 || S.ek[e] == kErType1U)
                emit("  const u32 t%s = T.ld(kb%d, %s);\n", id2(st, e).c_str(), kidx((int)(S.ep[e] & 0xffu)),
                     poff(S.ep[e] >> 8).c_str());
    };
    auto scr_loads = [&](int st) {
        if (st >= NS) return;
        const DecStep &S = steps[st];
        if (small) return;  // LDS rows: read where they are used
        for (int j = 0; j < NK; j++)
            if ((S.kk[j] == kKnLoc || S.kk[j] == kKnPark) && lty(S.kp[j]) == kLocScratch) emit("  const u32 q%s = T.scr_ld<%d>(%u);\n", id2(st, j).c_str(), opt.scr_aux, lix(S.kp[j]));
        for (int e = 0; e < NE; e++)
            if (S.ek[e] == kErFinish && lty(S.ep[e]) == kLocScratch) emit("  const u32 r%s = T.scr_ld<%d>(%u);\n", id2(st, e).c_str(), opt.scr_aux, lix(S.ep[e]));
    };
    // a location's LDS row (per-call kernel: scratch rows after the slots)
    auto lrow = [&](uint32_t loc) { return lty(loc) == kLocSlot ? slot0 + lix(loc) : scr0 + lix(loc); };
    for (int d = 0; d < depth; d++) loads(d);
    scr_loads(0);
    if (small) {  // the loader's registers, its first `depth` steps of loads, step 0's ring slot
        for (int st = 0; st < NS; st++) {
            const size_t nl = ring_list(st).size();
            for (size_t i = 0; i < nl; i++) emit("  u32 L%d_%zu;\n", st, i);
        }
        emit("  if (T.wv == %du) {\n", W);
        for (int d = 0; d < depth; d++) loader_issue(d);
        loader_put(0);
        s += "  }\n  T.sync();\n";
    }
    for (int st = 0; st < NS; st++) {
        const DecStep &S = steps[st];
        auto put = [&](uint32_t loc, const std::string &v) {
            if (loc == kLocNone) return;
            if (lty(loc) == kLocStage) {
                const uint32_t it = S.out[lix(loc)];
                emit("  T.%s(ob%u, %s, %s);\n", opt.drop_branch ? "out_st" : "out_st_oob", it & 0xffu,
                     poff((it >> 8) & 0xffu).c_str(), v.c_str());
            } else if (lty(loc) == kLocSlot || small) {
                emit("  T.lds_st(%u, %s);\n", lrow(loc), v.c_str());
            } else {
                emit("  T.scr_st(%u, %s);\n", lix(loc), v.c_str());
            }
        };
        // per-call kernel: which of the W waves does a known row's copy / an erased row's work
        std::vector<int> own_e(NE, 0);
        int nw = 0;
        for (int e = 0; e < NE; e++)
            if (S.ek[e] != kErSkip) own_e[e] = nw++ % W;
        emit("  // step %d: plane (%u, %u)\n", st, S.z / 10, S.z % 10);
        if (!opt.late) loads(st + depth);
        if (small) {
            // this step's input rows from the ring (compute waves; the loader's copy is unused)
            const DecStep &S0 = S;
            int i = 0;
            for (int j = 0; j < NK; j++)
                if (S0.kk[j] != kKnPark) emit("  const u32 o%s = T.lds_ld(%u);\n", id2(st, j).c_str(), ring_row(st, i++));
            for (int j = 0; j < NK; j++)
                if (S0.kk[j] == kKnInput || S0.kk[j] == kKnInputU) emit("  const u32 p%s = T.lds_ld(%u);\n", id2(st, j).c_str(), ring_row(st, i++));
            for (int e = 0; e < NE; e++)
                if (S0.ek[e] == kErType1 || S0.ek[e] == kErType1U) emit("  const u32 t%s = T.lds_ld(%u);\n", id2(st, e).c_str(), ring_row(st, i++));
            // loader: step st + depth's global loads, step st + 1's rows into the other slot
            emit("  if (T.wv == %du) {\n", W);
            loader_issue(st + depth);
            loader_put(st + 1);
            s += "  }\n";
        }
        // uncouple the known nodes (known data rows are copied out as they are)
        for (int j = 0; j < NK; j++) {
            const std::string id = id2(st, j);
            const char *i = id.c_str();
            if (S.kk[j] == kKnRed) emit("  const u32 u%s = o%s;\n", i, i);
            else if (S.kk[j] == kKnInput || S.kk[j] == kKnInputU) emit("  const u32 u%s = pft3(o%s, p%s);\n", i, i, i);
            else if (S.kk[j] == kKnPark && (lty(S.kp[j]) == kLocSlot || small)) emit("  const u32 u%s = T.lds_ld(%u);\n", i, lrow(S.kp[j]));
            else if (S.kk[j] == kKnPark) emit("  const u32 u%s = q%s;\n", i, i);
            else if (lty(S.kp[j]) == kLocSlot || small) emit("  const u32 u%s = pft3(o%s, T.lds_ld(%u));\n", i, i, lrow(S.kp[j]));
            else emit("  const u32 u%s = pft3(o%s, q%s);\n", i, i, i);
            if (!small) put(S.kout[j], "o" + id);
        }
        // pair partners' U, read before this step's writes
        for (int e = 0; e < NE; e++) {
            if (S.ek[e] != kErFinish) continue;
            const std::string id = id2(st, e);
            if (lty(S.ep[e]) == kLocSlot || small) emit("  const u32 v%s = T.lds_ld(%u);\n", id.c_str(), lrow(S.ep[e]));
            else emit("  const u32 v%s = r%s;\n", id.c_str(), id.c_str());
        }
        // in-row known pairs: the partner's U parked, its row out -- after every read of the step
        // (a location is reusable from its consumer step on)
        auto pair_puts = [&](int j) {
            if (S.kk[j] != kKnInputU) return;
            const std::string id = id2(st, j);
            put(S.kpark[j], "pft3(p" + id + ", o" + id + ")");
            put(S.kpout[j], "p" + id);
        };
        if (!small)
            for (int j = 0; j < NK; j++) pair_puts(j);
        if (small) {
            // every wave has read what this step reads before any wave writes (a location is
            // reused from its consumer step on); the known rows' copies, spread over the waves
            s += "  T.sync();\n";
            for (int j = 0; j < NK; j++)
                if (S.kout[j] != kLocNone || S.kk[j] == kKnInputU) {
                    emit("  if (T.wv == %du) {\n", j % W);
                    put(S.kout[j], "o" + id2(st, j));
                    pair_puts(j);
                    s += "  }\n";
                }
        }
        // MDS: the erased U's this step needs, v_perm products against the pattern's matrix
        bool any = false;
        for (int e = 0; e < NE; e++) any = any || S.ek[e] != kErSkip;
        for (int w = 0; w < (any ? W : 0); w++) {
            if (small) emit("  if (T.wv == %du) {\n", w);
            for (int j = 0; j < NK; j++)
                emit("  const %s s%s(u%s);\n", opt.tab4 ? "Sel4" : "Sel", id2(st, j).c_str(), id2(st, j).c_str());
            for (int e = 0; e < NE; e++) {
                if (S.ek[e] == kErSkip || own_e[e] != w) continue;
                const std::string a = "a" + id2(st, e);
                // decode: a red row whose only use is a column-0 parity node's output (dropped) is
                // not computed (uniform branch on the relabelled node)
                const bool drop_red = cs.yl < 0 && S.ek[e] == kErRed && S.ed0[e] != kLocNone &&
                                      lty(S.ed0[e]) == kLocStage && (S.out[lix(S.ed0[e])] & 0xffu) < 10u;
                if (drop_red) emit("  if (ob%u != T.kDropBase) {\n", S.out[lix(S.ed0[e])] & 0xffu);
                // decode: a pair of column-0 nodes (park, then finish at the partner's plane) both
                // of which are parity nodes feeds nothing but dropped outputs: skipped alike at
                // both steps (the condition is symmetric in the pair)
                const int ecan = e < 10 - cs.a0 ? cs.a0 + e : -1;  // canonical column-0 erased node
                const bool drop_pair = opt.drop_pairs && cs.yl < 0 && ecan >= 0 &&
                                       (S.ek[e] == kErPark || S.ek[e] == kErFinish);
                if (drop_pair) emit("  if (ob%d != T.kDropBase || ob%u != T.kDropBase) {\n", ecan, S.z / 10);
                emit("  u32 %s = 0u;\n  { const auto D = T.%s();\n", a.c_str(), opt.tab4 ? "mat4" : "mat");
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
                    case kErRed:
                        put(S.ed0[e], a);
                        if (drop_red) s += "  }\n";
                        break;
                    case kErType1:
                    case kErType1U: {  // C = t_u (U ^ Cp) ^ Cp
                        // t_u * y as a v_perm table product of compile-time tables (~10 VALU;
                        // the xtime chain of t_u = 0xf4 was ~37)
                        if (opt.tu_perm) {
                            emit("  const Sel y%s(%s ^ t%s);\n", i, a.c_str(), i);
                            emit("  const u32 w%s = perm_mul_acc(t%s, y%s, 0x%08xu, 0x%08xu, 0x%08xu, 0x%08xu, 0x%08xu);\n",
                                 i, i, i, tu_tab.t[0], tu_tab.t[1], tu_tab.t[2], tu_tab.t[3], tu_tab.t[4]);
                        } else {  // the xtime chain
                            emit("  const u32 y%s_0 = %s ^ t%s;\n", i, a.c_str(), i);
                            std::string r;
                            for (int bit = 0; bit < 8 && (t_u >> bit); bit++) {
                                if (bit) emit("  const u32 y%s_%d = xt(y%s_%d);\n", i, bit, i, bit - 1);
                                if ((t_u >> bit) & 1) r += (r.empty() ? "" : " ^ ") + ("y" + id + "_" + std::to_string(bit));
                            }
                            emit("  const u32 w%s = %s ^ t%s;\n", i, r.empty() ? "0u" : r.c_str(), i);
                        }
                        if (S.ek[e] == kErType1U && opt.tu_perm) {
                            // the partner's U = pft3(Cp, C) = Cp ^ (2 t_u)(U ^ Cp): a second table
                            // product of the same selectors; its row out
                            emit("  const u32 x%s = perm_mul_acc(t%s, y%s, 0x%08xu, 0x%08xu, 0x%08xu, 0x%08xu, 0x%08xu);\n",
                                 i, i, i, tu2_tab.t[0], tu2_tab.t[1], tu2_tab.t[2], tu2_tab.t[3], tu2_tab.t[4]);
                            put(S.ed0[e], "x" + id);
                            put(S.epd[e], "t" + id);
                        } else if (S.ek[e] == kErType1U) {  // the partner's U parked, its row out
                            put(S.ed0[e], "pft3(t" + id + ", w" + id + ")");
                            put(S.epd[e], "t" + id);
                        } else {
                            put(S.ed0[e], "w" + id);
                        }
                        put(S.ed1[e], "w" + id);
                        break;
                    }
                    case kErPark:
                        put(S.ep[e], a);
                        if (drop_pair) s += "  }\n";
                        break;
                    case kErFinish:
                        put(S.ed0[e], "pft3(" + a + ", v" + id + ")");
                        put(S.epd[e], "pft3(v" + id + ", " + a + ")");
                        if (drop_pair) s += "  }\n";
                        break;
                    default: break;
                }
            }
            if (small) s += "  }\n";
        }
        if (small) s += "  T.sync();\n";  // this step's values visible to every wave
        if (opt.late) loads(st + depth);
        scr_loads(st + 1);
    }
    s += "}\n";
    };
    body(true);
    body(false);
    emit("void dec_class_reg_%d(DecClassEntry &e) {\n  e.fn[0] = reinterpret_cast<const void *>(&dec_class_%d_small);\n"
         "  e.fn[1] = reinterpret_cast<const void *>(&dec_class_%d);\n  e.nslots = %uu;\n  e.nscratch = %uu;\n"
         "  e.nring = %uu;\n}\n", id, id, id, H.nslots, H.nscratch, nring);
    s += "}  // namespace dcls\n}  // namespace tec\n";
    return s;
}

}  // namespace tec
