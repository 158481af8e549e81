"""Debug aid (not a test): encode one object on the GPU and print where its slices differ from
the oracle, as (slice, stripe, node, plane, byte range) runs.   python scripts/dbg_encode.py [len]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import tape_amd as T  # noqa: E402
from oracle import oracle as O  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_001
data = O.splitmix64_bytes(5, n).tobytes()
s = T.Slicer.clay_default()
got = s.encode(data)
exp = O.slicer_encode(O.OracleClay(20, 7, 16), data)
cs, sc = 143_000, 1_430
runs = 0
for i, (g, e) in enumerate(zip(got, exp)):
    if g == e:
        continue
    a, b = np.frombuffer(g, np.uint8), np.frombuffer(e, np.uint8)
    bad = np.nonzero(a != b)[0]
    print(f"slice {i}: {len(bad)} bytes differ (len {len(a)})")
    # runs of consecutive differing offsets
    starts = [bad[0]] + [bad[k] for k in range(1, len(bad)) if bad[k] != bad[k - 1] + 1]
    ends = [bad[k] for k in range(len(bad) - 1) if bad[k + 1] != bad[k] + 1] + [bad[-1]]
    for st, en in list(zip(starts, ends))[:12]:
        stripe, r = divmod(int(st), cs)
        plane, c = divmod(r, sc)
        node = (i - 7 * stripe) % 20
        print(f"  [{st}, {en}] stripe {stripe} node {node} plane {plane} cols {c}..{c + en - st}"
              f" got {a[st:min(en + 1, st + 8)].tolist()} exp {b[st:min(en + 1, st + 8)].tolist()}")
        runs += 1
    if runs > 60:
        break
print("ok" if runs == 0 else "mismatch")
