// Row loads per stripe column of each class program (dec_class.hpp dec_class_prog, with the load
// fusions): own rows not parked by a type-1 or in-row pair step, known-partner rows and type-1
// partner rows.  Printed one class per line; tests/test_dec_class_host.py pins the counts so a
// change that loses a fusion shows up on the CPU.
#include <cstdio>
#include "dec_class.hpp"
using namespace tec;
int main() {
    ClayHost h;
    if (h.init(20, 7, 16) != 0) return 2;
    for (int id = 0; id < kDecClasses; id++) {
        GpePattern P;
        DecProgHdr H;
        std::vector<DecStep> st;
        if (!dec_class_prog(h, id, P, H, st)) return 1;
        long loads = 0, fused_t1 = 0, fused_pairs = 0;
        for (const DecStep &S : st) {
            for (uint32_t j = 0; j < P.nknown; j++) {
                loads += S.kk[j] != kKnPark;
                loads += S.kk[j] == kKnInput || S.kk[j] == kKnInputU;
                fused_pairs += S.kk[j] == kKnInputU;
            }
            for (uint32_t e = 0; e < P.nerased; e++) {
                loads += S.ek[e] == kErType1 || S.ek[e] == kErType1U;
                fused_t1 += S.ek[e] == kErType1U;
            }
        }
        printf("%d %ld %ld %ld %u %u\n", id, loads, fused_t1, fused_pairs, H.nslots, H.nscratch);
    }
    return 0;
}
