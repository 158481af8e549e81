#!/usr/bin/env python3
"""Generate tape_amd/csrc/mds_slp.inc: the Clay(20,7,16) per-plane MDS (13 parity U's from the 7
data U's, A2 generator V.inv(V_top) over GF(2^8)/0x11D) as a straight-line XOR program over the
56 xtime multiples 2^i u_x, with common subexpressions shared.

Why: encode_dma's MDS computed each of the 13 rows as its own XOR of the multiples its
coefficients select (346 two-input XORs per plane word).  The generator's coefficients repeat
(each column holds most values twice), so randomized greedy pair elimination (Paar's algorithm)
finds ~130.  Every single-use intermediate is then inlined into its consumer, and each node with
n operands costs ceil((n - 1) / 2) v_bitop3 XOR3 instructions.

Two programs: SCALED (level-1 planes: rows 7..9 pre-multiplied by the PFT's t_u, as
enc_common.hpp's Gt) and plain.  The kernel side checks the program at compile time against
rs_generator (enc_common.hpp: slp_ok), so a stale or wrong file does not build.

  python3 scripts/gen_mds_slp.py            # writes tape_amd/csrc/mds_slp.inc
  python3 scripts/gen_mds_slp.py --check    # exit 1 if the file differs from a fresh run
"""
import os
import random
import sys
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tape_amd", "csrc", "mds_slp.inc")

EXP = [0] * 512
LOG = [0] * 256
_x = 1
for _i in range(255):
    EXP[_i] = _x
    LOG[_x] = _i
    _x <<= 1
    if _x & 0x100:
        _x ^= 0x11D
for _i in range(255, 512):
    EXP[_i] = EXP[_i - 255]


def mul(a, b):
    return 0 if a == 0 or b == 0 else EXP[LOG[a] + LOG[b]]


def inv(a):
    return EXP[255 - LOG[a]]


def gpow(r, c):
    if c == 0:
        return 1
    return 0 if r == 0 else EXP[(LOG[r] * c) % 255]


def generator(k, n):
    V = [[gpow(r, c) for c in range(k)] for r in range(n)]
    A = [V[i][:] + [1 if i == j else 0 for j in range(k)] for i in range(k)]
    for c in range(k):
        p = next(r for r in range(c, k) if A[r][c])
        A[c], A[p] = A[p], A[c]
        iv = inv(A[c][c])
        A[c] = [mul(v, iv) for v in A[c]]
        for r in range(k):
            if r != c and A[r][c]:
                f = A[r][c]
                A[r] = [a ^ mul(f, b) for a, b in zip(A[r], A[c])]
    Vi = [row[k:] for row in A]
    G = [[0] * k for _ in range(n)]
    for r in range(n):
        for c in range(k):
            s = 0
            for j in range(k):
                s ^= mul(V[r][j], Vi[j][c])
            G[r][c] = s
    return G


def pft_t_u():
    """t_u of gf.hpp's Pft for orientation 1 (type-1 recovery, self = hi): solve RS(2,2)."""
    g4 = generator(2, 4)

    def coef(a, b, w):
        m = [[g4[a][0], g4[a][1]], [g4[b][0], g4[b][1]]]
        det = mul(m[0][0], m[1][1]) ^ mul(m[0][1], m[1][0])
        di = inv(det)
        mi = [[mul(m[1][1], di), mul(m[0][1], di)], [mul(m[1][0], di), mul(m[0][0], di)]]
        ca = mul(g4[w][0], mi[0][0]) ^ mul(g4[w][1], mi[1][0])
        cb = mul(g4[w][0], mi[0][1]) ^ mul(g4[w][1], mi[1][1])
        return ca, cb

    # o = 1: self C at 0, partner C at 1, self U at 2, partner U at 3; t: from (su, pc) -> sc
    t_u, _ = coef(2, 1, 0)
    return t_u


K, N, NR = 7, 20, 13
LOCAL = "--global" not in sys.argv


def rows_of(G):
    rows = []
    for r in range(K, N):
        s = set()
        for c in range(K):
            for i in range(8):
                if G[r][c] >> i & 1:
                    s.add(c * 8 + i)
        rows.append(s)
    return rows


def paar(rows, nsig, rng, local):
    """Greedy pair elimination.  local: only pairs of one input's multiples (then every
    intermediate belongs to one input and the schedule keeps few values live)."""
    rows = [set(r) for r in rows]
    defs = []  # (a, b) for signal nsig + idx
    col = {s: s // 8 for s in range(nsig)}
    nxt = nsig
    while True:
        pc = Counter()
        for r in rows:
            l = sorted(r)
            for i in range(len(l)):
                for j in range(i + 1, len(l)):
                    if not local or col[l[i]] == col[l[j]]:
                        pc[(l[i], l[j])] += 1
        if not pc:
            break
        best = max(pc.values())
        if best < 2:
            break
        cands = [p for p, m in pc.items() if m == best]
        a, b = cands[rng.randrange(len(cands))]
        defs.append((a, b))
        col[nxt] = col[a]
        for r in rows:
            if a in r and b in r:
                r.discard(a)
                r.discard(b)
                r.add(nxt)
        nxt += 1
    return defs, rows


def lower(defs, rows, nsig):
    """Inline single-use intermediates; return (ops, cost).  ops: list of (dst, [operands]),
    dst >= nsig intermediates (materialised) then outputs as ('o', r)."""
    uses = Counter()
    for a, b in defs:
        uses[a] += 1
        uses[b] += 1
    for r in rows:
        for s in r:
            uses[s] += 1
    operands = {}

    def expand(s):
        if s < nsig or uses[s] != 1:
            return [s]
        a, b = defs[s - nsig]
        return expand(a) + expand(b)

    ops = []
    for idx, (a, b) in enumerate(defs):
        s = nsig + idx
        if uses[s] >= 2:
            operands[s] = expand(a) + expand(b)
            ops.append((s, operands[s]))
    for r, row in enumerate(rows):
        ops.append((("o", r), sum((expand(s) for s in sorted(row)), [])))
    cost = sum((len(o) - 1 + 1) // 2 for _, o in ops)
    return ops, cost


def best_program(rows, tries, seed, local):
    rng = random.Random(seed)
    best = None
    for _ in range(tries):
        defs, rest = paar(rows, 56, rng, local)
        ops, cost = lower(defs, rest, 56)
        if local:  # scheduled cost with inputs in order (the schedule is what runs)
            _, cost, peak, _ = schedule(ops, list(range(7)))
            cost = (cost, peak)
        if best is None or cost < best[1]:
            best = (ops, cost)
    return best


def schedule(ops, order):
    """Accumulator schedule: inputs' multiples are produced in `order`; every node (shared
    intermediate or output row) XORs in its operands as soon as they exist, two at a time
    (v_bitop3 XOR3 into the accumulator), an odd one waiting for the next.  Returns the flat
    program [(kind, dst, srcs)] and its (instructions, peak live values)."""
    pos = {x: i for i, x in enumerate(order)}
    ready = {s: pos[s // 8] for s in range(56)}
    nodes = []  # (key, operands)
    for dst, o in ops:
        nodes.append((dst, list(o)))
    for key, o in nodes:
        ready[key] = max(ready[s] for s in o)
    slot = {}
    nslot = 56
    for key, _ in nodes:
        slot[key] = nslot
        nslot += 1
    prog = []
    state = {key: None for key, _ in nodes}   # 'acc' once started
    pend = {key: [] for key, _ in nodes}
    cost = 0
    for t in range(7):
        prog.append(("mult", order[t], []))
        for key, o in nodes:
            new = pend[key] + [slot.get(s, s) for s in o if ready[s] == t]
            pend[key] = []
            if not new:
                continue
            last = ready[key] == t
            d = slot[key]
            if state[key] is None:
                if len(new) >= 3:
                    prog.append(("x3", d, new[:3])); new = new[3:]; cost += 1
                elif len(new) == 2:
                    prog.append(("x2", d, new[:2])); new = []; cost += 1
                elif last:
                    prog.append(("mv", d, new[:1])); new = []
                else:
                    pend[key] = new
                    continue
                state[key] = "acc"
            while len(new) >= 2:
                prog.append(("x3", d, [d] + new[:2])); new = new[2:]; cost += 1
            if new:
                if last:
                    prog.append(("x2", d, [d, new[0]])); cost += 1
                else:
                    pend[key] = new
    # peak live: a value is live from its definition to its last use
    last_use = {}
    defined = {}
    for i, (k, d, src) in enumerate(prog):
        for s_ in src:
            last_use[s_] = i
        if k == "mult":
            for j in range(8):
                defined.setdefault(8 * d + j, i)
        else:
            defined.setdefault(d, i)
    outs = [slot[key] for key, _ in nodes if isinstance(key, tuple)]
    for o_ in outs:
        last_use[o_] = len(prog)
    peak = 0
    for i in range(len(prog) + 1):
        live = sum(1 for v, a in defined.items() if a <= i and last_use.get(v, a) >= i)
        peak = max(peak, live)
    return prog, cost, peak, slot


def emit_program(name, ops, order):
    prog, cost, peak, slot = schedule(ops, order)
    out_slot = {key[1]: slot[key] for key in slot if isinstance(key, tuple)}
    lines = ["// %s: %d XOR instructions, peak %d live values, inputs in order %s"
             % (name, cost, peak, order),
             "inline constexpr SlpProg %s = {%d, {" % (name, len(prog))]
    kinds = {"mult": 0, "mv": 1, "x2": 2, "x3": 3}
    for k, d, src in prog:
        src = list(src) + [0] * (3 - len(src))
        lines.append("    {%d, %d, %d, %d, %d}," % (kinds[k], d, src[0], src[1], src[2]))
    lines.append("}, {%s}};" % ", ".join(str(out_slot[r]) for r in range(NR)))
    return lines, len(prog), max(slot.values()) + 1, cost, peak


def verify(ops, rows):
    sig = {s: 1 << s for s in range(56)}
    out = {}
    for dst, o in ops:
        v = 0
        for s in o:
            v ^= sig[s]
        if isinstance(dst, tuple):
            out[dst[1]] = v
        else:
            sig[dst] = v
    for r, row in enumerate(rows):
        want = 0
        for s in row:
            want ^= 1 << s
        assert out[r] == want, r


def best_order(ops):
    import itertools
    best = None
    for order in itertools.permutations(range(7)):
        _, cost, peak, _ = schedule(ops, list(order))
        key = (peak, cost)
        if best is None or key < best[0]:
            best = (key, list(order))
    return best[1]


def main():
    G = generator(K, N)
    t_u = pft_t_u()
    Gt = [row[:] for row in G]
    for r in range(K, 10):
        Gt[r] = [mul(t_u, v) for v in G[r]]
    text = [
        "// mds_slp.inc -- GENERATED by scripts/gen_mds_slp.py (do not edit): the Clay(20,7,16) plane MDS",
        "// as a shared-XOR program over the 56 xtime multiples (signal 8x + i = 2^i u_x), scheduled as",
        "// accumulators.  Op = {kind, dst, a, b, c}: kind 0 = multiples of input dst into 8 dst..8 dst + 7,",
        "// 1: dst = a, 2: dst = a ^ b, 3: dst = a ^ b ^ c (v_bitop3).  out[r] = slot of parity row 7 + r.",
        "// Checked against rs_generator at compile time (enc_common.hpp: slp_ok).",
    ]
    mx_ops = mx_slots = 0
    for name, g in (("kSlpScaled", Gt), ("kSlpPlain", G)):
        rows = rows_of(g)
        ops, _ = best_program(rows, 200, 12345, LOCAL)
        verify(ops, rows)
        order = list(range(7)) if LOCAL else best_order(ops)
        lines, nops, nslots, cost, peak = emit_program(name, ops, order)
        mx_ops = max(mx_ops, nops)
        mx_slots = max(mx_slots, nslots)
        text += lines
        print(name, "cost", cost, "peak", peak, "ops", nops, "slots", nslots, file=sys.stderr)
    text.append("static_assert(kSlpMaxOps >= %d && kSlpSlots >= %d, \"SlpProg capacity\");" % (mx_ops, mx_slots))
    out = "\n".join(text) + "\n"
    if "--check" in sys.argv:
        with open(OUT) as f:
            sys.exit(0 if f.read() == out else 1)
    with open(OUT, "w") as f:
        f.write(out)


if __name__ == "__main__":
    main()
