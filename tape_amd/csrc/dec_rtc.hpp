// dec_rtc.hpp -- host side of the per-pattern decode kernels (dec_fixed.hpp): one erasure
// pattern's plane program (ClayHost::dec_prog) written out as the straight-line source of the
// kernel `tec_dec_fixed`, which engine.cpp compiles with hipRTC.
#pragma once
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>
#include "kernels.hpp"

namespace tec {

constexpr const char *kDecFixedKernel = "tec_dec_fixed";

// waves per SIMD the 8-column kernels are compiled for (TEC_DEC_JIT_WPE, measurement knob)
inline int dec_fixed_wpe8() {
    static const int w = [] {
        const char *e = tec_knob("TEC_DEC_JIT_WPE");
        const int v = e ? atoi(e) : 3;  // 3: 4.78 ms; 2: 5.34; 4: spills, 7.88 (1024 x 4 MiB, 13 erasures)
        return v >= 1 && v <= 8 ? v : 3;
    }();
    return w;
}

// LDS bytes of a pattern's kernel: two staging buffers of max_out rows, then the slots (rows of
// G waves x 64 lanes x wb bytes)
inline size_t dec_fixed_lds(const DecProgHdr &H, int G, bool direct, int wb) {
    return (size_t)((direct ? 0 : 2 * H.max_out) + H.nslots) * G * 64u * (uint32_t)wb;
}

// The kernel source for known nodes P.known, decoding matrix D[e][j] (GF(2^8) coefficients of
// erased e over known j), the unpacked steps of dec_prog, G waves per workgroup, and the type-1
// coefficient t_u (C = t_u (U ^ Cp) ^ Cp), wb columns per lane (4, or 8 for direct output).
inline std::string dec_fixed_source(const GpePattern &P, const uint8_t (*D)[kGpeMaxKnown], const DecProgHdr &H,
                                    const std::vector<DecStep> &steps, int G, uint8_t t_u, bool direct, int wb) {
    const int NK = (int)P.nknown, NE = (int)P.nerased, NS = (int)steps.size();
    const uint32_t MO = H.max_out, SLOT0 = direct ? 0 : 2 * MO;
    std::string s;
    char b[256];
    auto emit = [&](const char *fmt, auto... v) {
        snprintf(b, sizeof b, fmt, v...);
        s += b;
    };
    auto lty = [](uint32_t loc) { return loc >> 24; };
    auto lix = [](uint32_t loc) { return loc & 0xffffffu; };
    auto id2 = [](int a, int c) { return std::to_string(a) + "_" + std::to_string(c); };
    static const bool tu_perm = [] {  // TEC_DEC_JIT_TU=xt: the xtime chain (measurement)
        const char *e = tec_knob("TEC_DEC_JIT_TU");
        return !(e && e[0] == 'x');
    }();
    const PermTab tu_tab = perm_tab(t_u);
    if (direct) s += "#define TEC_DFIX_RAW 1\n";  // words kept in load order (dec_fixed.hpp Tile::rot)
    s += "#include \"dec_fixed.hpp\"\nusing namespace tec::dfix;\n";
    emit("typedef Lane<%d>::V VT;\n#define VZ (Lane<%d>::zero())\n", wb, wb);
    // flush items per step (data chunk x | plane << 8), scalar-loaded after each step's barrier
    if (!direct) emit("__constant__ unsigned short kItems[%d][%d] = {\n", std::max(NS, 1), kDecMaxOut);
    for (int st = 0; st < NS && !direct; st++) {
        s += "{";
        for (int r = 0; r < kDecMaxOut; r++)
            emit("%u%s", r < (int)steps[st].nout ? steps[st].out[r] & 0xffffu : 0u, r + 1 < kDecMaxOut ? "," : "");
        s += st + 1 < NS ? "},\n" : "}\n";
    }
    if (!direct) s += "};\n";
    emit("extern \"C\" __global__ void __attribute__((amdgpu_flat_work_group_size(1, %d), amdgpu_waves_per_eu(%d)))\n",
         G * 64, wb == 8 ? dec_fixed_wpe8() : 4);
    emit("%s(Args a) {\n  extern __shared__ __attribute__((aligned(16))) u32 lds[];\n", kDecFixedKernel);
    emit("  const Tile<%d, %d> T(a, reinterpret_cast<u8 *>(lds));\n", G, wb);
    // loads of step st: own rows, input partners, type-1 partners; then its scratch reads
    auto loads = [&](int st) {
        if (st >= NS) return;
        const DecStep &S = steps[st];
        for (int j = 0; j < NK; j++) {
            if (S.kk[j] != kKnPark) emit("  const VT o%s = T.ld(%u, %u);\n", id2(st, j).c_str(), (unsigned)H.knode[j], S.z);
            if (S.kk[j] == kKnInput || S.kk[j] == kKnInputU) emit("  const VT p%s = T.ld(%u, %u);\n", id2(st, j).c_str(), S.kp[j] & 0xffu, S.kp[j] >> 8);
        }
        for (int e = 0; e < NE; e++)
            if (S.ek[e] == kErType1 || S.ek[e] == kErType1U) emit("  const VT t%s = T.ld(%u, %u);\n", id2(st, e).c_str(), S.ep[e] & 0xffu, S.ep[e] >> 8);
    };
    auto scr_loads = [&](int st) {
        if (st >= NS) return;
        const DecStep &S = steps[st];
        for (int j = 0; j < NK; j++)
            if ((S.kk[j] == kKnLoc || S.kk[j] == kKnPark) && lty(S.kp[j]) == kLocScratch) emit("  const VT q%s = T.scr_ld(%u);\n", id2(st, j).c_str(), lix(S.kp[j]));
        for (int e = 0; e < NE; e++)
            if (S.ek[e] == kErFinish && lty(S.ep[e]) == kLocScratch) emit("  const VT r%s = T.scr_ld(%u);\n", id2(st, e).c_str(), lix(S.ep[e]));
    };
    loads(0);
    scr_loads(0);
    for (int st = 0; st < NS; st++) {
        const DecStep &S = steps[st];
        const uint32_t sb = (uint32_t)(st & 1) * MO;
        auto put = [&](uint32_t loc, const std::string &v) {
            if (loc == kLocNone) return;
            if (lty(loc) == kLocStage && direct)
                emit("  T.out_st(%u, %u, %s);\n", S.out[lix(loc)] & 0xffu, (S.out[lix(loc)] >> 8) & 0xffu, v.c_str());
            else if (lty(loc) == kLocStage) emit("  T.lds_st(%u, %s);\n", sb + lix(loc), v.c_str());
            else if (lty(loc) == kLocSlot) emit("  T.lds_st(%u, %s);\n", SLOT0 + lix(loc), v.c_str());
            else emit("  T.scr_st(%u, %s);\n", lix(loc), v.c_str());
        };
        emit("  // step %d: plane %u\n", st, S.z);
        loads(st + 1);
        // uncouple the known nodes; known data rows are staged as they are
        for (int j = 0; j < NK; j++) {
            const std::string id = id2(st, j);
            const char *i = id.c_str();
            if (S.kk[j] == kKnPark) {  // U parked by the type-1 step (which also stored the row out)
                if (lty(S.kp[j]) == kLocSlot) emit("  const VT u%s = T.lds_ld(%u);\n", i, SLOT0 + lix(S.kp[j]));
                else emit("  const VT u%s = q%s;\n", i, i);
                continue;
            }
            emit("  const VT c%s = T.rot(o%s);\n", i, i);
            if (S.kk[j] == kKnRed) emit("  const VT u%s = c%s;\n", i, i);
            else if (S.kk[j] == kKnInput || S.kk[j] == kKnInputU) emit("  const VT u%s = pft3(c%s, T.rot(p%s));\n", i, i, i);
            else if (lty(S.kp[j]) == kLocSlot) emit("  const VT u%s = pft3(c%s, T.lds_ld(%u));\n", i, i, SLOT0 + lix(S.kp[j]));
            else emit("  const VT u%s = pft3(c%s, q%s);\n", i, i, i);
            put(S.kout[j], "c" + id);
        }
        // pair partners' U, read before this step's writes (a location is reusable from its consumer on)
        for (int e = 0; e < NE; e++) {
            if (S.ek[e] != kErFinish) continue;
            const std::string id = id2(st, e);
            if (lty(S.ep[e]) == kLocSlot) emit("  const VT v%s = T.lds_ld(%u);\n", id.c_str(), SLOT0 + lix(S.ep[e]));
            else emit("  const VT v%s = r%s;\n", id.c_str(), id.c_str());
        }
        // in-row known pairs (direct output only): the partner's U parked, its row out, after the
        // step's reads
        for (int j = 0; j < NK; j++) {
            if (S.kk[j] != kKnInputU) continue;
            const std::string id = id2(st, j);
            put(S.kpark[j], "pft3(T.rot(p" + id + "), c" + id + ")");
            put(S.kpout[j], "T.rot(p" + id + ")");
        }
        // MDS: the erased U's this step needs, j-major over xtime multiples, XOR3 pairs
        std::vector<std::string> acc(NE), pend(NE);
        int tmp = 0;
        for (int j = 0; j < NK; j++) {
            int top = -1;
            for (int e = 0; e < NE; e++)
                if (S.ek[e] != kErSkip)
                    for (int i = 0; i < 8; i++)
                        if ((D[e][j] >> i) & 1) top = std::max(top, i);
            if (top < 0) continue;
            std::vector<std::string> m(top + 1);
            m[0] = "u" + id2(st, j);
            for (int i = 1; i <= top; i++) {
                m[i] = "m" + id2(st, j) + "_" + std::to_string(i);
                emit("  const VT %s = xt(%s);\n", m[i].c_str(), m[i - 1].c_str());
            }
            for (int e = 0; e < NE; e++) {
                if (S.ek[e] == kErSkip) continue;
                for (int i = 0; i <= top; i++) {
                    if (!((D[e][j] >> i) & 1)) continue;
                    if (pend[e].empty()) { pend[e] = m[i]; continue; }
                    const std::string nm = "x" + id2(st, tmp++);
                    if (acc[e].empty()) emit("  const VT %s = %s ^ %s;\n", nm.c_str(), pend[e].c_str(), m[i].c_str());
                    else emit("  const VT %s = xor3(%s, %s, %s);\n", nm.c_str(), acc[e].c_str(), pend[e].c_str(), m[i].c_str());
                    acc[e] = nm;
                    pend[e].clear();
                }
            }
        }
        for (int e = 0; e < NE; e++) {
            if (S.ek[e] == kErSkip) continue;
            const std::string nm = "a" + id2(st, e);
            const std::string v = acc[e].empty() ? (pend[e].empty() ? "VZ" : pend[e])
                                                 : (pend[e].empty() ? acc[e] : acc[e] + " ^ " + pend[e]);
            emit("  const VT %s = %s;\n", nm.c_str(), v.c_str());
        }
        // results: staged data rows, parked / type-1 values in slots or scratch
        for (int e = 0; e < NE; e++) {
            const std::string id = id2(st, e), a = "a" + id;
            const char *i = id.c_str();
            switch (S.ek[e]) {
                case kErRed: put(S.ed0[e], a); break;
                case kErType1:
                case kErType1U: {  // C = t_u (U ^ Cp) ^ Cp
                    emit("  const VT k%s = T.rot(t%s);\n", i, i);
                    emit("  const VT y%s_0 = %s ^ k%s;\n", i, a.c_str(), i);
                    if (tu_perm) {  // t_u * y as a v_perm product of compile-time tables
                        emit("  const VT w%s = mulk(y%s_0, 0x%08xu, 0x%08xu, 0x%08xu, 0x%08xu, 0x%08xu) ^ k%s;\n", i, i,
                             tu_tab.t[0], tu_tab.t[1], tu_tab.t[2], tu_tab.t[3], tu_tab.t[4], i);
                    } else {
                        std::string r;
                        for (int bit = 0; bit < 8 && (t_u >> bit); bit++) {
                            if (bit) emit("  const VT y%s_%d = xt(y%s_%d);\n", i, bit, i, bit - 1);
                            if ((t_u >> bit) & 1) r += (r.empty() ? "" : " ^ ") + ("y" + id + "_" + std::to_string(bit));
                        }
                        emit("  const VT w%s = %s ^ k%s;\n", i, r.empty() ? "VZ" : r.c_str(), i);
                    }
                    if (S.ek[e] == kErType1U) {  // the partner's U parked, its row out (direct output only)
                        put(S.ed0[e], "pft3(k" + id + ", w" + id + ")");
                        put(S.epd[e], "k" + id);
                    } else {
                        put(S.ed0[e], "w" + id);
                    }
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
        scr_loads(st + 1);
        if (!direct) {  // staged rows: flushed whole after the step's barrier
            s += "  T.barrier();\n";
            emit("  T.flush(%u, kItems[%d], %u);\n", sb, st, S.nout);
        }
    }
    s += "}\n";
    return s;
}

}  // namespace tec
