// clay_host.hpp -- host-side Clay layout math: node/plane geometry, repair planning and the
// erasure-pattern tables the GPU engines consume.  Pure integer bookkeeping (the reference's
// clay_codes::ClayCode::{new, minimum_to_repair} and the layered-decode ordering).
#pragma once
#include <algorithm>
#include <map>
#include <tuple>
#include <vector>
#include <stdint.h>
#include <stddef.h>
#include <vector>
#include <algorithm>
#include "kernels.hpp"

namespace tec {

struct ClayHost {
    int n = 0, k = 0, m = 0, d = 0, q = 0, t = 0, nu = 0, qt = 0, alpha = 0, beta = 0;
    Mat G;                       // qt x (k+nu) systematic generator (A2)
    std::vector<uint32_t> qpow;  // q^i, i <= t

    // ClayCoder::new asserts (clay.rs:24-34) + layout limits of the GPU engines.
    // returns 0 ok, -1 invalid params, -2 unsupported layout.
    int init(int n_, int k_, int d_) {
        if (!(n_ > k_ && k_ > 0 && d_ >= k_ + 1 && d_ <= n_ - 1)) return -1;
        n = n_; k = k_; m = n_ - k_; d = d_;
        q = d - k + 1;
        nu = (q - (n % q)) % q;
        t = (n + nu) / q;
        qt = q * t;
        if (qt > kMaxNodes || qt > 64 || t >= 16) return -2;
        long a = 1;
        for (int i = 0; i < t; i++) {
            a *= q;
            if (a > 4096) return -2;
        }
        alpha = (int)a;
        beta = alpha / q;
        if (m > kGpeMaxErased || k + nu > kGpeMaxKnown) return -2;
        // LDS budget of the generic engine: 2 * m * alpha words of 16 B per block
        if ((size_t)2 * m * alpha * kGpeWords * 4 + (size_t)alpha * t > 150 * 1024) return -2;
        G = rs_generator(k + nu, qt);
        qpow.assign(16, 0);
        uint32_t p = 1;
        for (int i = 0; i <= t && i < 16; i++) { qpow[i] = p; p *= (uint32_t)q; }
        return 0;
    }

    int ext_to_int(int e) const { return e < k ? e : e + nu; }
    int int_to_ext(int i) const { return i < k ? i : (i < k + nu ? -1 : i - nu); }
    int digit(int z, int y) const { return (int)((uint32_t)z / qpow[t - 1 - y] % (uint32_t)q); }

    // ClayCoder::chunk_size_for  clay.rs:61-73
    size_t chunk_size_for(size_t len) const {
        const size_t min_size = (size_t)k * alpha * 2;
        size_t padded = len == 0 ? min_size : ((len + min_size - 1) / min_size) * min_size;
        if (padded < min_size) padded = min_size;
        return padded / k;
    }

    // get_repair_subchunks, expanded ascending (A6)
    std::vector<int> repair_planes(int lost_ext) const {
        const int lost = ext_to_int(lost_ext);
        const int y = lost / q, x = lost % q;
        const int seq = (int)qpow[t - 1 - y], nseq = (int)qpow[y];
        std::vector<int> out;
        int index = x * seq;
        for (int s = 0; s < nseq; s++) {
            for (int j = index; j < index + seq; j++) out.push_back(j);
            index += q * seq;
        }
        return out;
    }

    // minimum_to_repair (A6): column-mates of the lost node, then ascending available ids.
    // returns 0 and d helper ext ids (ascending), or -1 (not enough helpers), -2 (column-mate
    // unavailable / bad index).
    int min_to_repair(int lost_ext, const std::vector<int> &avail, std::vector<int> &helpers) const {
        if (lost_ext < 0 || lost_ext >= n) return -2;
        if ((int)avail.size() < d) return -1;
        std::vector<char> isav(n, 0), chosen(n, 0);
        for (int a : avail)
            if (a >= 0 && a < n) isav[a] = 1;
        const int lost = ext_to_int(lost_ext);
        int cnt = 0;
        for (int j = 0; j < q; j++) {
            if (j == lost % q) continue;
            const int e = int_to_ext((lost / q) * q + j);
            if (e < 0) continue;
            if (!isav[e]) return -2;
            if (!chosen[e]) { chosen[e] = 1; cnt++; }
        }
        for (int id = 0; id < n && cnt < d; id++)
            if (isav[id] && !chosen[id] && id != lost_ext) { chosen[id] = 1; cnt++; }
        if (cnt != d) return -1;
        helpers.clear();
        for (int id = 0; id < n; id++)
            if (chosen[id]) helpers.push_back(id);
        return 0;
    }

    // MDS decoding matrix for an internal erased set of size m: D = G_E * inv(G_known).
    bool decoder(uint64_t erased_mask, std::vector<int> &known, std::vector<int> &erased, Mat &D) const {
        const int kk = k + nu;
        known.clear();
        erased.clear();
        for (int i = 0; i < qt; i++) {
            if ((erased_mask >> i) & 1ull) erased.push_back(i);
            else if ((int)known.size() < kk) known.push_back(i);
        }
        if ((int)known.size() != kk) return false;
        Mat sub{};
        sub.rows = sub.cols = kk;
        for (int r = 0; r < kk; r++)
            for (int c = 0; c < kk; c++) sub.v[r][c] = G.v[known[r]][c];
        if (!mat_invert(sub)) return false;
        D = Mat{};
        D.rows = (int)erased.size();
        D.cols = kk;
        for (size_t e = 0; e < erased.size(); e++)
            for (int j = 0; j < kk; j++) {
                uint8_t acc = 0;
                for (int l = 0; l < kk; l++) acc ^= gf_mul(G.v[erased[e]][l], sub.v[l][j]);
                D.v[e][j] = acc;
            }
        return true;
    }

    // A7: pad an internal erased set with the lowest parity nodes until it has m members.
    uint64_t pad_erasures(uint64_t mask) const {
        int cnt = __builtin_popcountll(mask);
        for (int i = k + nu; cnt < m && i < qt; i++)
            if (!((mask >> i) & 1ull)) { mask |= 1ull << i; cnt++; }
        return mask;
    }


    // Staged-decode program (decode_stage.hip) for an erasure pattern: planes row by row along
    // `orient` (0: rows = plane digit of column 0, 1: of column 1), within a row the planes whose
    // inner digit is a known node first; every value a later plane needs gets a storage slot
    // (lane-private LDS if consumed in the same row, per-stripe scratch otherwise).  Follows
    // Ceph decode_layered (oracle/clay_oracle.c decode_layered) value by value; returns false
    // when a dependency would be consumed before it is produced (then the generic engine runs).
    //
    // out_node < 0: the output is the data (Slicer::decode): every data node's C, item x = node.
    // out_node >= 0: the output is that one node's chunk, item x = 0 (node recover's lost slice,
    // recover.rs:411-442: a parity node's C comes out of the same layered decode, so nothing is
    // re-encoded); pairs of erased nodes neither of which is output are skipped either way.
    // out_mask != 0 (decode class kernels): the output nodes are exactly those of the mask (items
    // keep their node ids); the kernel drops the outputs that are not data rows.
    // fuse_pairs (generated kernels only): known pairs coupled within a row of planes as kKnInputU /
    // kKnPark (kernels.hpp).
    bool dec_prog(const GpePattern &P, int orient, DecProgHdr &H, std::vector<DecStep> &out, int out_node = -1,
                  uint64_t out_mask = 0, bool fuse_pairs = false) const {
        if (q != kRepQ || t != 2 || nu != 0 || alpha != kRepQ * kRepQ) return false;
        if (P.nknown > (uint32_t)kDecMaxK || P.nerased > (uint32_t)kDecMaxE) return false;
        const uint64_t em = P.erased_mask;
        auto er = [&](int node) { return ((em >> node) & 1ull) != 0; };
        auto isdata = [&](int node) {  // an output node
            return out_mask ? ((out_mask >> node) & 1ull) != 0 : out_node < 0 ? node < k : node == out_node;
        };
        const uint32_t relabel = out_node < 0 || out_mask ? 0xffu : 0u;
        const int yo = orient ? 1 : 0, yi = 1 - yo;
        std::vector<int> rows, cols;
        for (int pass = 0; pass < 2; pass++)
            for (int r = 0; r < q; r++) {
                if (er(yo * q + r) == (pass == 1)) rows.push_back(r);
                if (er(yi * q + r) == (pass == 1)) cols.push_back(r);
            }
        std::vector<int> order, pos(alpha, -1);
        for (int r : rows)
            for (int c : cols) {
                const int d0 = yo == 0 ? r : c, d1 = yo == 0 ? c : r;
                pos[d0 * q + d1] = (int)order.size();
                order.push_back(d0 * q + d1);
            }
        // values: (kind 0 = C / 1 = U, node, plane) -> producer / consumer step (flat index: this
        // runs once per new pattern on the decode path, where random survivor sets are the norm)
        struct Val { int prod = -1, cons = -1; uint32_t loc = kLocNone; };
        std::vector<int> vid((size_t)3 * qt * alpha, -1);  // kinds: C, U of an erased node, U of a known one
        std::vector<Val> vals;
        vals.reserve(512);
        auto val = [&](int kind, int node, int z) {
            int &id = vid[((size_t)kind * qt + node) * alpha + z];
            if (id < 0) {
                id = (int)vals.size();
                vals.push_back(Val{});
            }
            return id;
        };
        struct Ref { int val = -1; };  // value reference to patch with its location
        out.assign(alpha, DecStep{});
        std::vector<std::vector<std::pair<uint32_t *, int>>> patches(1);
        auto &pl = patches[0];
        uint32_t max_out = 0;
        for (int st = 0; st < alpha; st++) {
            const int z = order[st];
            DecStep &S = out[st];
            S.z = (uint32_t)z;
            for (int i = 0; i < kDecMaxK; i++) S.kk[i] = kKnRed, S.kp[i] = 0, S.kout[i] = S.kpark[i] = S.kpout[i] = kLocNone;
            for (int i = 0; i < kDecMaxE; i++) S.ek[i] = kErSkip, S.ep[i] = 0, S.ed0[i] = S.ed1[i] = S.epd[i] = kLocNone;
            auto add_out = [&](int node, int plane) -> uint32_t {
                if (S.nout >= (uint32_t)kDecMaxOutProg) return kLocNone;
                S.out[S.nout] = (relabel == 0xffu ? (uint32_t)node : relabel) | ((uint32_t)plane << 8);
                return (kLocStage << 24) | S.nout++;
            };
            bool ok = true;
            for (uint32_t j = 0; j < P.nknown; j++) {
                const int N = P.known[j], x = N % q, y = N / q, zy = digit(z, y);
                const int M = y * q + zy, zsw = z + (x - zy) * (int)qpow[t - 1 - y];
                const bool row_pair = fuse_pairs && zy != x && !er(M) && pos[zsw] / q == st / q;
                if (row_pair && pos[zsw] < st) {  // the pair's first step parked this U and stored the row
                    const int v = val(2, N, z);
                    if (vals[v].prod < 0 || vals[v].cons >= 0) return false;
                    vals[v].cons = st;
                    S.kk[j] = kKnPark;
                    pl.push_back({&S.kp[j], v});
                    continue;
                }
                if (isdata(N)) { S.kout[j] = add_out(N, z); ok = ok && S.kout[j] != kLocNone; }
                if (zy == x) { S.kk[j] = kKnRed; continue; }
                if (!er(M)) {
                    S.kk[j] = kKnInput;
                    S.kp[j] = (uint32_t)M | ((uint32_t)zsw << 8);
                    if (row_pair) {  // first of the pair: the partner's U and row too
                        S.kk[j] = kKnInputU;
                        const int v = val(2, M, zsw);
                        vals[v].prod = st;
                        pl.push_back({&S.kpark[j], v});
                        if (isdata(M)) { S.kpout[j] = add_out(M, zsw); ok = ok && S.kpout[j] != kLocNone; }
                    }
                } else {
                    const int v = val(0, M, zsw);  // C of the erased partner, recovered earlier
                    if (vals[v].cons >= 0) return false;
                    vals[v].cons = st;
                    S.kk[j] = kKnLoc;
                    pl.push_back({&S.kp[j], v});
                }
            }
            for (uint32_t e = 0; e < P.nerased; e++) {
                const int N = P.erased[e], x = N % q, y = N / q, zy = digit(z, y);
                if (zy == x) {  // red: C = U
                    if (isdata(N)) { S.ek[e] = kErRed; S.ed0[e] = add_out(N, z); ok = ok && S.ed0[e] != kLocNone; }
                    continue;
                }
                const int M = y * q + zy, zsw = z + (x - zy) * (int)qpow[t - 1 - y];
                if (!er(M)) {  // type-1; the known partner consumes this C later
                    S.ek[e] = kErType1;
                    S.ep[e] = (uint32_t)M | ((uint32_t)zsw << 8);
                    const int v = val(0, N, z);
                    vals[v].prod = st;
                    pl.push_back({&S.ed0[e], v});
                    if (isdata(N)) { S.ed1[e] = add_out(N, z); ok = ok && S.ed1[e] != kLocNone; }
                    continue;
                }
                if (!isdata(N) && !isdata(M)) continue;  // a parity pair nobody reads
                if (pos[z] < pos[zsw]) {  // park this U for the pair's later plane
                    S.ek[e] = kErPark;
                    const int v = val(1, N, z);
                    vals[v].prod = st;
                    pl.push_back({&S.ep[e], v});
                } else {  // finish the pair: both C's
                    S.ek[e] = kErFinish;
                    const int v = val(1, M, zsw);
                    if (vals[v].prod < 0 || vals[v].cons >= 0) return false;
                    vals[v].cons = st;
                    pl.push_back({&S.ep[e], v});
                    if (isdata(N)) { S.ed0[e] = add_out(N, z); ok = ok && S.ed0[e] != kLocNone; }
                    if (isdata(M)) { S.epd[e] = add_out(M, zsw); ok = ok && S.epd[e] != kLocNone; }
                }
            }
            if (!ok) return false;
            max_out = std::max(max_out, S.nout);
        }
        // storage: lane-private LDS slot when producer and consumer share a row, scratch otherwise;
        // interval colouring, a location reusable from its value's consumer step on
        std::vector<int> idx(vals.size());
        for (size_t i = 0; i < vals.size(); i++) {
            if (vals[i].prod < 0 || vals[i].cons < 0 || vals[i].prod >= vals[i].cons) return false;
            idx[i] = (int)i;
        }
        std::sort(idx.begin(), idx.end(), [&](int a, int b) { return vals[a].prod < vals[b].prod; });
        // first fit (the lowest free location), linear: producers come in step order, so a
        // location is released when the producers pass its occupant's consumer step -- per step a
        // list of the locations it frees, and the free ones as a bit set (this runs once per new
        // pattern; random survivor sets make that once per stripe)
        struct Alloc {
            uint64_t avail[8] = {};   // locations < 512 (the kernels index < 256)
            int n = 0, next_rel = 0;
            std::vector<int> head, link;  // per step: first location it frees; per location: next
            explicit Alloc(int steps) : head((size_t)steps + 1, -1) {}
            int take(int prod, int cons) {
                for (; next_rel <= prod; next_rel++)
                    for (int l = head[(size_t)next_rel]; l >= 0; l = link[(size_t)l])
                        if (l < 512) avail[l >> 6] |= 1ull << (l & 63);
                int l = -1;
                for (int w = 0; w < 8 && l < 0; w++)
                    if (avail[w]) l = w * 64 + __builtin_ctzll(avail[w]);
                if (l < 0) {
                    l = n++;
                    link.push_back(-1);
                } else {
                    avail[l >> 6] &= ~(1ull << (l & 63));
                }
                link[(size_t)l] = head[(size_t)cons];
                head[(size_t)cons] = l;
                return l;
            }
        } slot_alloc(alpha), scr_alloc(alpha);
        for (int i : idx) {
            Val &V = vals[i];
            const bool same_row = V.prod / q == V.cons / q;
            const int l = (same_row ? slot_alloc : scr_alloc).take(V.prod, V.cons);
            V.loc = ((same_row ? kLocSlot : kLocScratch) << 24) | (uint32_t)l;
        }
        for (auto &p : pl) *p.first = vals[p.second].loc;
        H = DecProgHdr{};
        H.nsteps = (uint32_t)alpha;
        H.nslots = (uint32_t)slot_alloc.n;
        H.nscratch = (uint32_t)scr_alloc.n;
        H.max_out = max_out;
        for (uint32_t j = 0; j < P.nknown; j++) H.knode[j] = P.known[j];
        return true;
    }

    // Packed step (DecStepP) of a dec_prog step; false when a location index needs > 8 bits.
    static bool dec_pack(const DecStep &S, DecStepP &P) {
        bool ok = true;
        auto loc10 = [&](uint32_t loc) -> uint32_t {
            if (loc == kLocNone) return kLoc10None;
            const uint32_t ty = loc >> 24, ix = loc & 0xffffffu;
            if (ix >= 256 || ty > kLocScratch) { ok = false; return kLoc10None; }
            return ty << 8 | ix;
        };
        P = DecStepP{};
        if (S.z >= 256 || S.nout > (uint32_t)kDecMaxOut) return false;
        P.w[kDpHdr] = S.z | S.nout << 8;
        for (int j = 0; j < kDecMaxK; j++) {
            const uint32_t src = S.kk[j] == kKnLoc ? loc10(S.kp[j]) : (S.kk[j] == kKnInput ? S.kp[j] : 0u);
            P.w[kDpKd + j] = S.kk[j] << 28 | loc10(S.kout[j]) << 16 | src;
        }
        for (int e = 0; e < kDecMaxE; e++) {
            const uint32_t ek = S.ek[e];
            const uint32_t src = ek == kErType1 ? S.ep[e] : ((ek == kErPark || ek == kErFinish) ? loc10(S.ep[e]) : 0u);
            P.w[kDpEd + e] = ek << 28 | src;
            P.w[kDpEo + e] = loc10(S.ed0[e]) | loc10(S.ed1[e]) << 10 | loc10(S.epd[e]) << 20;
        }
        for (uint32_t r = 0; r < S.nout; r++) P.w[kDpOut + r / 2] |= (S.out[r] & 0xffffu) << (16 * (r & 1));
        return ok;
    }

    // Layered-decode pattern for the generic engine.  planes: appended to `pool`.
    bool gpe_pattern(uint64_t erased_mask, GpePattern &P, std::vector<uint16_t> &pool) const {
        std::vector<int> known, erased;
        Mat D;
        if (!decoder(erased_mask, known, erased, D)) return false;
        P = GpePattern{};
        P.erased_mask = erased_mask;
        P.nknown = (uint32_t)known.size();
        P.nerased = (uint32_t)erased.size();
        P.alpha = (uint32_t)alpha;
        for (size_t i = 0; i < known.size(); i++) P.known[i] = (uint8_t)known[i];
        for (size_t i = 0; i < erased.size(); i++) P.erased[i] = (uint8_t)erased[i];
        for (size_t e = 0; e < erased.size(); e++)
            for (size_t j = 0; j < known.size(); j++) P.D[e][j] = perm_tab(D.v[e][j]);
        if (erased.size() <= (size_t)kClsMaxE && known.size() <= (size_t)kClsMaxK)
            for (size_t e = 0; e < erased.size(); e++)
                for (size_t j = 0; j < known.size(); j++) {
                    const PermTab4 t = perm_tab4(D.v[e][j]);
                    for (int f = 0; f < 4; f++) P.D4[e][j][f] = t.t[f];
                }
        std::vector<int> score(alpha, 0);
        int maxs = 0;
        for (int z = 0; z < alpha; z++) {
            int s = 0;
            for (int y = 0; y < t; y++)
                if ((erased_mask >> (y * q + digit(z, y))) & 1ull) s++;
            score[z] = s;
            maxs = std::max(maxs, s);
        }
        if (maxs + 2 > 16) return false;
        P.planes_off = (uint32_t)pool.size();
        P.nlevels = (uint32_t)maxs + 1;
        for (int L = 0; L <= maxs; L++) {
            P.level_start[L] = (uint32_t)(pool.size() - P.planes_off);
            for (int z = 0; z < alpha; z++)
                if (score[z] == L) pool.push_back((uint16_t)z);
        }
        P.level_start[maxs + 1] = (uint32_t)(pool.size() - P.planes_off);
        return true;
    }

    // Repair pattern (Ceph repair_one_lost_chunk): erased = lost column + aloof nodes.
    // Uniform per-plane program of a repair pattern for the staged kernel (q = beta = kRepQ).
    bool rep_prog(const RepPattern &P, const uint16_t *pool, const uint16_t *pind, RepProg &R) const {
        if (q != kRepQ || (int)P.beta != kRepQ || t != 2) return false;
        R = RepProg{};
        const uint64_t amask = P.aloof_mask;
        const int lost = (int)P.lost, xl = lost % q, yl = lost / q;
        auto aidx = [&](int node) { return __builtin_popcountll(amask & ((1ull << node) - 1ull)); };
        for (uint32_t e = 0; e < P.nerased; e++) {
            const int node = P.erased[e], x = node % q;
            R.enode[e] = (uint32_t)node;
            if ((amask >> node) & 1ull) { R.ekind[e] = 0; R.erow[e] = (uint32_t)aidx(node); }
            else if (node == lost) { R.ekind[e] = 1; R.erow[e] = 0; }
            else { R.ekind[e] = x < xl ? 2 : 3; R.erow[e] = (uint32_t)(x < xl ? x + 1 : x); }
        }
        for (uint32_t j = 0; j < P.nknown; j++) R.knode0[j] = P.known[j];
        const uint16_t *planes = pool + P.planes_off;
        const uint32_t np = P.level_start[P.nlevels];
        if (np != (uint32_t)kRepQ) return false;
        for (uint32_t pi = 0; pi < np; pi++) {
            RepProg::Step &S = R.step[pi];
            const int z = planes[pi];
            S.z = (uint32_t)z;
            S.ri = pind[z];
            for (uint32_t j = 0; j < P.nknown; j++) {
                const int node = P.known[j], x = node % q, y = node / q, zy = digit(z, y);
                if (zy == x) { S.kkind[j] = 0; continue; }
                const int sw = y * q + zy;
                const int zsw = z + (x - zy) * (int)qpow[t - 1 - y];
                const int rsw = pind[zsw];
                if ((amask >> sw) & 1ull) {
                    S.kkind[j] = x > zy ? 4 : 3;
                    S.krow[j] = (uint32_t)(aidx(sw) * kRepQ + rsw);
                } else {
                    S.kkind[j] = x > zy ? 2 : 1;
                    S.knode[j] = (uint32_t)sw;
                    S.krow[j] = (uint32_t)rsw;
                }
            }
            for (int r = 0; r < kRepQ; r++) {
                const int x = r == 0 ? xl : (r - 1 < xl ? r - 1 : r);
                S.oplane[r] = (uint32_t)(z + (x - xl) * (int)qpow[t - 1 - yl]);
            }
        }
        return true;
    }

    bool rep_pattern(int lost_ext, const std::vector<int> &helpers_ext, RepPattern &P,
                     std::vector<uint16_t> &pool, std::vector<uint16_t> &pind) const {
        const int lost = ext_to_int(lost_ext);
        std::vector<char> is_helper(qt, 0);
        for (int h : helpers_ext) is_helper[ext_to_int(h)] = 1;
        uint64_t aloof = 0, emask = 0;
        for (int e = 0; e < n; e++) {
            const int i = ext_to_int(e);
            if (!is_helper[i] && e != lost_ext) aloof |= 1ull << i;
        }
        for (int i = 0; i < q; i++) emask |= 1ull << (lost - lost % q + i);
        emask |= aloof;
        if (__builtin_popcountll(emask) != m) return false;
        std::vector<int> known, erased;
        Mat D;
        if (!decoder(emask, known, erased, D)) return false;
        P = RepPattern{};
        P.erased_mask = emask;
        P.aloof_mask = aloof;
        P.nknown = (uint32_t)known.size();
        P.nerased = (uint32_t)erased.size();
        P.beta = (uint32_t)beta;
        P.lost = (uint32_t)lost;
        for (size_t i = 0; i < known.size(); i++) P.known[i] = (uint8_t)known[i];
        for (size_t i = 0; i < erased.size(); i++) P.erased[i] = (uint8_t)erased[i];
        for (size_t e = 0; e < erased.size(); e++)
            for (size_t j = 0; j < known.size(); j++) P.D[e][j] = perm_tab(D.v[e][j]);
        const std::vector<int> rp = repair_planes(lost_ext);
        const size_t base = pind.size();
        pind.resize(base + alpha, 0xffff);
        for (size_t i = 0; i < rp.size(); i++) pind[base + rp[i]] = (uint16_t)i;
        std::vector<int> order(rp.size());
        int maxo = 0;
        for (size_t i = 0; i < rp.size(); i++) {
            int o = 0;
            for (int nd = 0; nd < qt; nd++)
                if ((((aloof >> nd) & 1ull) || nd == lost) && digit(rp[i], nd / q) == nd % q) o++;
            order[i] = o;
            maxo = std::max(maxo, o);
        }
        if (maxo + 2 > 16) return false;
        P.planes_off = (uint32_t)pool.size();
        P.nlevels = (uint32_t)maxo + 1;
        for (int L = 0; L <= maxo; L++) {
            P.level_start[L] = (uint32_t)(pool.size() - P.planes_off);
            for (size_t i = 0; i < rp.size(); i++)
                if (order[i] == L) pool.push_back((uint16_t)rp[i]);
        }
        P.level_start[maxo + 1] = (uint32_t)(pool.size() - P.planes_off);
        return true;
    }
};

// (dec_prog programs of the generated class kernels and the hipRTC pattern kernels)
// A type-1 step (erased N at plane z, known partner M at plane z') has both of the values the
// partner's own step z' combines -- Cp = M's row at z' (its type-1 read) and C = N's new value --
// so it parks M's U = pft3(Cp, C) in C's location and, when M is an output, stores Cp out itself
// (epd: an item of its own step).  The partner's step then reads U (kKnPark) and does not load its
// own row: the row was read once instead of twice.  Returns the number of fused pairs.
inline int dec_prog_fuse_type1(const GpePattern &P, std::vector<DecStep> &steps) {
    std::vector<int> at(256, -1);
    for (size_t st = 0; st < steps.size(); st++) at[steps[st].z & 0xffu] = (int)st;
    int fused = 0;
    for (DecStep &S : steps)
        for (uint32_t e = 0; e < P.nerased; e++) {
            if (S.ek[e] != kErType1 || S.ed0[e] == kLocNone) continue;
            const uint32_t M = S.ep[e] & 0xffu, zp = S.ep[e] >> 8;
            if (zp >= 256 || at[zp] < 0) continue;
            DecStep &T = steps[(size_t)at[zp]];
            int j = -1;
            for (uint32_t i = 0; i < P.nknown; i++)
                if (P.known[i] == M) j = (int)i;
            if (j < 0 || T.kk[j] != kKnLoc || T.kp[j] != S.ed0[e]) continue;
            if (T.kout[j] != kLocNone) {  // M is an output: its row goes out from this step
                if ((T.kout[j] >> 24) != kLocStage || S.nout >= (uint32_t)kDecMaxOutProg) continue;
                S.out[S.nout] = T.out[T.kout[j] & 0xffffffu];
                S.epd[e] = (kLocStage << 24) | S.nout++;
                T.kout[j] = kLocNone;
            }
            S.ek[e] = kErType1U;
            T.kk[j] = kKnPark;
            fused++;
        }
    return fused;
}

}  // namespace tec
