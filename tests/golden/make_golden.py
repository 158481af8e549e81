#!/usr/bin/env python3
"""Generate tests/golden/clay_golden.json from the CPU oracle (run in the build container).

What these fixtures pin: GPU == CPU restatement, and the restatement against itself over time
(any change to the oracle's algebra shows up as a fixture diff).  They do NOT pin the reference:
`clay-codes` 0.1.1 / `reed-solomon-erasure` 6.0.0 are absent and no Rust toolchain exists, so
reference byte-parity of parity slices is UNPINNED (DESIGN.md "Parity status").  The values the
reference's own tests do pin (sizes, metadata, rotation, helper counts) are asserted separately
in tests/test_oracle_reference.py.

Contents (all inputs deterministic: SplitMix64 per SURVEY 8d, or the (i % 251) pattern of
lib/slicer/src/slicer.rs:397-399):
  slicer:  Slicer::clay_default().encode, per-slice SHA-256 + geometry, several sizes / rotation /
           chunk_index;
  raw:     ClayCoder::encode per profile, per-chunk SHA-256;
  tiny:    full hex bytes of small encodes (readable byte-level vectors);
  plans:   minimum_to_repair for every lost node of (20,7,16) with all others available, and the
           repair plan of a 1 MiB object for lost slice 3.
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import oracle as O  # noqa: E402

MiB = 1 << 20


def sha(b) -> str:
    return hashlib.sha256(bytes(b)).hexdigest()


def payload(kind: str, n: int) -> bytes:
    if kind == "pattern251":
        return O.test_pattern(n)
    seed = int(kind.split(":")[1])
    return O.splitmix64_bytes(seed, n).tobytes()


SLICER_CASES = [  # (payload, length, rotated, chunk_index)
    ("splitmix:1", 0, True, 0),
    ("splitmix:1", 1, True, 0),
    ("splitmix:2", 1000, True, 0),
    ("splitmix:3", 100_000, True, 0),
    ("splitmix:4", 100_001, False, 0),
    ("splitmix:5", 1_000_001, True, 5),
    ("splitmix:1", MiB, True, 0),          # SURVEY 8d plumbing object
    ("pattern251", MiB, True, 0),
    ("splitmix:7", 4 * MiB, True, 0),      # BASELINE object size
]
RAW_CASES = [((20, 7, 16), 10_000), ((20, 10, 19), 10_000), ((12, 8, 11), 5_000), ((6, 3, 5), 777),
             ((20, 5, 14), 3_001), ((20, 7, 19), 2_000)]
TINY_CASES = [((6, 3, 5), 40), ((4, 2, 3), 9)]


def main():
    out = {"generator": "tests/golden/make_golden.py (oracle/clay_oracle.c)", "slicer": [], "raw": [], "tiny": [],
           "plans": {}}
    c716 = O.OracleClay(20, 7, 16)
    for kind, n, rot, ci in SLICER_CASES:
        data = payload(kind, n)
        S, ns, cs, sl = O.geometry(c716, n)
        slices = O.slicer_encode(c716, data, rotated=rot, chunk_index=ci)
        out["slicer"].append({"payload": kind, "len": n, "rotated": rot, "chunk_index": ci,
                              "stripe_size": S, "num_stripes": ns, "chunk_size": cs, "slice_len": sl,
                              "payload_sha256": sha(data), "slice_sha256": [sha(s) for s in slices]})
    for (n, k, d), ln in RAW_CASES:
        c = O.OracleClay(n, k, d)
        data = O.splitmix64_bytes(ln, ln).tobytes()
        chunks = c.encode(data)
        out["raw"].append({"params": [n, k, d], "len": ln, "seed": ln, "chunk_size": len(chunks[0]),
                           "chunk_sha256": [sha(x) for x in chunks]})
    for (n, k, d), ln in TINY_CASES:
        c = O.OracleClay(n, k, d)
        data = bytes((7 * i + 3) & 0xFF for i in range(ln))
        chunks = c.encode(data)
        out["tiny"].append({"params": [n, k, d], "data_hex": data.hex(), "chunks_hex": [x.hex() for x in chunks]})
    rep = {}
    for lost in range(20):
        avail = [j for j in range(20) if j != lost]
        rep[str(lost)] = [[h, p] for h, p in c716.minimum_to_repair(lost, avail)]
    out["plans"]["minimum_to_repair_20_7_16_all_available"] = rep
    cs, stripes = O.repair_plan(c716, 3, [j for j in range(20) if j != 3], MiB, 1_000_000)
    out["plans"]["slicer_repair_plan_1MiB_lost3"] = {"chunk_size": cs, "stripes": stripes}
    path = os.path.join(HERE, "clay_golden.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)
    print(path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
