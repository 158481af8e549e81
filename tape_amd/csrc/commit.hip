// commit.hip -- slice commitments on the device: the step right after encode in
// BlobEncoder::encode_with_proofs (sdk/src/codec/encoder.rs:226-234): hash_leaf of each of the
// n slices, the height-H merkle root (root_from_leaf_hashes, lib/crypto/src/merkle/tree.rs:344-350)
// and one proof per slice (create_proof_from_leaf_hashes, tree.rs:353-358, 397-455).
//
// MI355X mapping.  SHA-256 is sequential within a message, so the parallelism is the number of
// slices: one lane per slice stream (20 per object; a 1024-object batch is 320 waves, one per
// SIMD at most).  A lane walks its slice in 64-byte blocks with the next block's 16 dword loads
// issued before the current block is compressed; the block schedule is unrolled with the rotates
// as v_alignbit, Ch/Maj/Sigma as v_bitop3 and the sums as v_add3.  "LEAF" is the first message
// word, so slice word j is message word j + 1: 4-aligned loads, no byte shifting.  The tree
// (≈ 2n pair hashes per object) is one lane per object.
#include "kernels.hpp"
#include "sha256.hpp"

namespace tec {
namespace commit {

constexpr uint64_t kLeafBlocksPerLaunch = 1536;  // ~3.5 ms of one stream's SHA-256

// Blocks [b0, b1) of every stream.  A stream's state between launches lives in its own leaf-hash
// slot (8 words, the size of the digest): launches after the first load it, launches before the
// last store it, and the last stores the digest.  Long slices are hashed in several launches of
// about kLeafBlocksPerLaunch blocks (a 30 ms launch holds up any copy queued behind it
// on a shared hardware queue; ~3 ms launches do not).
#ifndef TEC_LEAF_PRIO
#define TEC_LEAF_PRIO 3
#endif
__global__ void __launch_bounds__(64) leaf_kernel(CommitArgs a, uint64_t b0, uint64_t b1) {
    // Wave priority (r05): a group's hashing runs beside the next groups' encodes and copies, and
    // a leaf wave is one slice's serial SHA-256 chain.  Sharing a SIMD with encode waves at equal
    // priority it issued at a fraction of its rate, the group's hashing fell behind the encodes
    // (one launch per group, one slice per lane: 64 waves for 205 objects), and the slot streams
    // then waited for the hashed group buffers -- the 4 GiB-group runs at 7.5 GiB/s.
    // The leaf waves are few; they take issue priority on their SIMDs.
    if constexpr (TEC_LEAF_PRIO > 0) __builtin_amdgcn_s_setprio(TEC_LEAF_PRIO);
    const uint32_t total = a.nobj * a.n;
    const uint32_t gid = blockIdx.x * 64u + threadIdx.x;
    const bool live = gid < total;
    const uint32_t g = live ? gid : total - 1u;  // idle lanes redo the last stream, no store
    const uint32_t obj = g / a.n, sl = g - obj * a.n;
    const uint32_t *p = reinterpret_cast<const uint32_t *>(a.slices + obj * a.obj_stride + sl * a.slice_len);
    const uint64_t L = a.slice_len, M = L + 4u;       // message bytes ("LEAF" || slice)
    const uint64_t T = (M + 8u) / 64u + 1u;           // blocks incl. padding and length
    const uint64_t nfull = L >= 60u ? (L - 60u) / 64u + 1u : 0u;  // blocks 0 .. nfull-1 hold data only
    if (b1 > T) b1 = T;
    uint32_t *out = reinterpret_cast<uint32_t *>(a.leaf + (uint64_t)g * 32u);
    uint32_t st[8];
    if (b0 == 0) {
        sha::init(st);
    } else {
#pragma unroll
        for (int i = 0; i < 8; i++) st[i] = out[i];
    }
    // raw (little-endian) words of the next two blocks, loaded two blocks ahead and byte-swapped
    // only when their block starts, so a load's latency hides behind two compressions (the hashing
    // runs beside copies and encodes, whose traffic lengthens it)
    uint32_t w[16], n1[16], n2[16];
    const uint64_t dend = nfull < b1 ? nfull : b1;
    auto ldblk = [&](uint64_t b, uint32_t *dst) {
        if (b == 0) {
            dst[0] = sha::bswap(sha::kLeafWord);
#pragma unroll
            for (int k = 1; k < 16; k++) dst[k] = p[k - 1];
        } else {
            const uint32_t *q = p + b * 16u - 1u;
#pragma unroll
            for (int k = 0; k < 16; k++) dst[k] = q[k];
        }
    };
    if (b0 < dend) ldblk(b0, n1);
    if (b0 + 1 < dend) ldblk(b0 + 1, n2);
    for (uint64_t b = b0; b < dend; b++) {
#pragma unroll
        for (int k = 0; k < 16; k++) {
            w[k] = sha::bswap(n1[k]);
            n1[k] = n2[k];
        }
        if (b + 2 < dend) ldblk(b + 2, n2);
        sha::compress(st, w);
    }
    // the last data bytes, the 0x80 terminator, zeros and the bit length (L % 4 == 0)
    for (uint64_t b = (nfull > b0 ? nfull : b0); b < b1; b++) {
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const uint64_t gw = b * 16u + (uint64_t)k, pos = gw * 4u;
            w[k] = gw == 0 ? sha::kLeafWord : (pos < M ? sha::bswap(p[gw - 1u]) : (pos == M ? 0x80000000u : 0u));
        }
        if (b + 1 == T) {
            w[14] = (uint32_t)((M * 8u) >> 32);
            w[15] = (uint32_t)(M * 8u);
        }
        sha::compress(st, w);
    }
    if (!live) return;
    if (b1 < T) {
#pragma unroll
        for (int i = 0; i < 8; i++) out[i] = st[i];
    } else {
#pragma unroll
        for (int i = 0; i < 8; i++) out[i] = sha::bswap(st[i]);
    }
}

// Root and proofs of one object from its n leaf hashes: layer by layer, an odd layer padded
// with EMPTY_ROOTS[level] (tree.rs:430-440); proof[i][level] = sibling of i's node (tree.rs:442-455).
__global__ void __launch_bounds__(64) tree_kernel(CommitArgs a) {
    const uint32_t obj = blockIdx.x * 64u + threadIdx.x;
    if (obj >= a.nobj) return;
    const uint32_t n = a.n, H = a.height;
    uint8_t layer[kCommitMaxLeaves + 1][32];
    uint8_t empty[32];
    sha::hash_leaf(nullptr, 0, empty);
    const uint8_t *lv = a.leaf + (uint64_t)obj * n * 32u;
    for (uint32_t i = 0; i < n; i++)
        for (int j = 0; j < 32; j++) layer[i][j] = lv[i * 32u + j];
    uint32_t c = n;
    for (uint32_t l = 0; l < H; l++) {
        if (c & 1u) {
            for (int j = 0; j < 32; j++) layer[c][j] = empty[j];
            c++;
        }
        if (a.proof)
            for (uint32_t i = 0; i < n; i++) {
                const uint32_t sib = (i >> l) ^ 1u;
                uint8_t *pr = a.proof + (((uint64_t)obj * n + i) * H + l) * 32u;
                for (int j = 0; j < 32; j++) pr[j] = layer[sib][j];
            }
        for (uint32_t k = 0; k < c / 2; k++) {
            uint8_t t[32];
            sha::hash_pair(layer[2 * k], layer[2 * k + 1], t);
            for (int j = 0; j < 32; j++) layer[k][j] = t[j];
        }
        c /= 2;
        uint8_t e2[32];
        sha::hash_pair(empty, empty, e2);
        for (int j = 0; j < 32; j++) empty[j] = e2[j];
    }
    if (a.root)
        for (int j = 0; j < 32; j++) a.root[(uint64_t)obj * 32u + j] = layer[0][j];
}

}  // namespace commit

hipError_t launch_commit(const CommitArgs &a, hipStream_t s) {
    if (a.nobj == 0 || a.n == 0) return hipSuccess;
    if (a.n > (uint32_t)kCommitMaxLeaves || a.slice_len % 4u || !a.leaf) return hipErrorInvalidValue;
    const uint64_t total = (uint64_t)a.nobj * a.n;
    const uint64_t T = ((uint64_t)a.slice_len + 4u + 8u) / 64u + 1u;  // blocks per stream
    const uint64_t nl = (T + commit::kLeafBlocksPerLaunch - 1) / commit::kLeafBlocksPerLaunch, per = (T + nl - 1) / nl;
    hipError_t e = hipSuccess;
    for (uint64_t b0 = 0; b0 < T && e == hipSuccess; b0 += per) {
        hipLaunchKernelGGL(commit::leaf_kernel, dim3((uint32_t)((total + 63) / 64)), dim3(64), 0, s, a, b0, b0 + per);
        e = hipGetLastError();
    }
    if (e != hipSuccess || !a.root) return e;
    hipLaunchKernelGGL(commit::tree_kernel, dim3((a.nobj + 63) / 64), dim3(64), 0, s, a);
    return hipGetLastError();
}

}  // namespace tec
