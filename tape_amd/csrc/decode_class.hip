// decode_class.hip -- registry and launcher of the decode class kernels (dec_class.hpp; bodies
// generated at build time into build/gen/dec_class_<id>.hip by gen_dec_class).
#include "decode_class_dev.hpp"
#include "dec_class.hpp"

namespace tec {
namespace dcls {
#include "dec_class_reg.inc"
}  // namespace dcls

static const dcls::DecClassEntry *dec_class_table() {
    static const dcls::DecClassEntry *t = [] {
        static dcls::DecClassEntry e[kDecClasses];
        for (int i = 0; i < kDecClasses; i++) dcls::kDecClassReg[i](e[i]);
        return e;
    }();
    return t;
}

bool dec_class_info(int id, uint32_t *nslots, uint32_t *nscratch) {
    if (id < 0 || id >= kDecClasses) return false;
    const dcls::DecClassEntry &e = dec_class_table()[id];
    if (!e.fn[0] || !e.fn[1]) return false;
    if (nslots) *nslots = e.nslots;
    if (nscratch) *nscratch = e.nscratch;
    return true;
}

// workgroups per stripe: 64-word groups, G of them per workgroup
uint32_t dec_class_wgs(uint32_t sc, uint32_t G) {
    const uint32_t wps = (sc + 3) / 4, groups = (wps + 63) / 64;
    return (groups + G - 1) / G;
}

size_t dec_class_scratch_bytes(int id, uint32_t njobs, uint32_t sc, uint32_t G) {
    uint32_t ns = 0, nscr = 0;
    if (!dec_class_info(id, &ns, &nscr) || G == 1) return 0;  // the per-call kernel parks in LDS
    return (size_t)njobs * dec_class_wgs(sc, G) * (nscr ? nscr : 1) * G * 256u;
}

hipError_t launch_dec_class(int id, const GpeJob *jobs, const GpePattern *patterns, uint32_t njobs, uint32_t sc,
                            uint64_t in_stride, uint64_t out_stride, uint32_t n, uint8_t *scratch, uint32_t G,
                            hipStream_t s) {
    const DecClassSpec spec = dec_class_spec(id);
    if (njobs == 0) return hipSuccess;
    uint32_t nslots = 0, nscr = 0;
    if (!dec_class_info(id, &nslots, &nscr) || (G != 1 && G != 2) || sc < 8 || n != (uint32_t)kDecClassN)
        return hipErrorInvalidValue;
    dcls::DecClassArgs a{};
    a.jobs = jobs;
    a.patterns = patterns;
    a.scratch = scratch;
    a.in_stride = in_stride;
    a.out_stride = out_stride;
    a.njobs = njobs;
    a.sc = sc;
    a.wps = (sc + 3) / 4;
    a.wgs_per_stripe = dec_class_wgs(sc, G);
    a.n = n;
    a.nscratch = nscr;
    // decode writes the k data chunks of a stripe, recover the lost node's one chunk
    const uint64_t full = spec.yl < 0 ? (uint64_t)kDecClassK * out_stride : out_stride;
    a.out_full = full > 0xffffffffull ? 0xffffffffu : (uint32_t)full;
    const uint64_t blocks = (uint64_t)njobs * a.wgs_per_stripe;
    if (blocks > 0x7fffffffull) return hipErrorInvalidValue;
    const size_t lds = dec_class_lds(nslots, nscr, dec_class_table()[id].nring, (int)G);
    const void *fn = dec_class_table()[id].fn[G - 1];
    hipError_t e = ensure_dyn_lds(fn, lds);
    if (e != hipSuccess) return e;
    void *args[] = {&a};
    // G = 1: the per-call kernel, kDecClassSplit compute waves and a loader wave per 64-column group
    const uint32_t threads = G == 1 ? 64u * (kDecClassSplit + 1) : G * 64u;
    e = hipLaunchKernel(fn, dim3((uint32_t)blocks), dim3(threads), args, lds, s);
    return e != hipSuccess ? e : hipGetLastError();
}

}  // namespace tec
