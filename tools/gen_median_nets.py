#!/usr/bin/env python
"""Generates fedml_amd/csrc/median_nets.h: straight-line selection networks for the coordinate-wise
median kernel (robust.hip).

For every bucket size B in 8, 16, ..., 128: Batcher's odd-even merge sort of P2 = next power of two
>= B keys, where the P2 - B extra inputs are compile-time sentinels -- Lc low (below every key)
and Hc high, Lc chosen so that the lower median of the B keys, rank (B-1)//2, is rank P2/2 - 1 of
all P2.  A comparator with a constant input is a renaming (no instruction); the rest are kept in
SSA form and pruned backwards to what the output at rank P2/2 - 1 depends on (a comparator whose
min or max half is dead emits only the other half).  The kernel pads K real keys to B with
runtime low/high sentinels in the same way (robust.hip), so one network serves K in (B-8, B].

Also SortNet<N> (N = 36, 40, ..., 64: a sort of N keys) for the two-lanes-per-column kernel k_median_2l.

Run: python tools/gen_median_nets.py   (prints the min/max count per B)
"""
from __future__ import annotations

import os
import sys

BUCKETS = list(range(8, 129, 8))


# A 16-key sorting network of 60 comparators (Green's construction: four hypercube layers, then 28
# comparators), against Batcher's 63.  Used as the base case of the merge sort below: the 32-key sort
# becomes 2 x 60 + 65 = 185 comparators (Batcher 191), the 64-key sort 531 (Batcher 543).  Checked
# exhaustively over all 2^16 0-1 inputs by verify_g16() (0-1 principle) on every generation.
G16 = [(0, 13), (1, 12), (2, 15), (3, 14), (4, 8), (5, 6), (7, 11), (9, 10),
       (0, 5), (1, 7), (2, 9), (3, 4), (6, 13), (8, 14), (10, 15), (11, 12),
       (0, 1), (2, 3), (4, 5), (6, 8), (7, 9), (10, 11), (12, 13), (14, 15),
       (0, 2), (1, 3), (4, 10), (5, 11), (6, 7), (8, 9), (12, 14), (13, 15),
       (1, 2), (3, 12), (4, 6), (5, 7), (8, 10), (9, 11), (13, 14),
       (1, 4), (2, 6), (5, 8), (7, 10), (9, 13), (11, 14),
       (2, 4), (3, 6), (9, 12), (11, 13),
       (3, 5), (6, 8), (7, 9), (10, 12),
       (3, 4), (5, 6), (7, 8), (9, 10), (11, 12),
       (6, 7), (8, 9)]


# Base case of the merge sort: G16 (default; r04ae, 3 interleaved pairs: median K = 128 1.156-1.164
# -> 1.090-1.095 ms, K = 32 0.2675-0.269 -> 0.262-0.265, bit-exact) or Batcher's own 16-key sort
# (`--batcher`, the r01-r04 networks).
BASE16 = "--batcher" not in sys.argv


def verify_g16():
    n = 16
    for v in range(1 << n):
        bits = [(v >> i) & 1 for i in range(n)]
        for i, j in G16:
            if bits[i] > bits[j]:
                bits[i], bits[j] = bits[j], bits[i]
        assert all(bits[i] <= bits[i + 1] for i in range(n - 1)), v


def oddeven_merge_sort(n, base16=BASE16):
    comps = []

    def merge(lo, hi, r):
        step = r * 2
        if step < hi - lo:
            merge(lo, hi, step)
            merge(lo + r, hi, step)
            comps.extend((i, i + r) for i in range(lo + r, hi - r, step))
        else:
            comps.append((lo, lo + r))

    def sort(lo, hi):
        if base16 and hi - lo + 1 == 16:
            comps.extend((lo + a, lo + b) for a, b in G16)
        elif hi - lo >= 1:
            mid = lo + (hi - lo) // 2
            sort(lo, mid)
            sort(mid + 1, hi)
            merge(lo, hi, 1)

    sort(0, n - 1)
    return comps  # (i, j), i < j: i receives the min, j the max


def network(B):
    """SSA nodes ('min'|'max', a, b) and the output operand; operands: ('x', i) input i,
    ('n', id) node id."""
    n = 1
    while n < B:
        n *= 2
    lc = n // 2 - 1 - (B - 1) // 2
    hc = n - B - lc
    pos = [("x", i) for i in range(B)] + [("L",)] * lc + [("H",)] * hc
    nodes = []
    const = lambda o: o[0] in ("L", "H")
    for i, j in oddeven_merge_sort(n):
        a, b = pos[i], pos[j]
        if const(a) and const(b):
            pos[i], pos[j] = (a, b) if (a[0] == "L" or b[0] == "H") else (b, a)
        elif const(a) or const(b):
            c, v = (a, b) if const(a) else (b, a)
            pos[i], pos[j] = (c, v) if c[0] == "L" else (v, c)
        else:
            nodes.append(("min", a, b))
            lo = ("n", len(nodes) - 1)
            nodes.append(("max", a, b))
            pos[i], pos[j] = lo, ("n", len(nodes) - 1)
    out = pos[n // 2 - 1]
    assert not const(out)
    need, stack = set(), [out]
    while stack:
        x = stack.pop()
        if x[0] == "n" and x[1] not in need:
            need.add(x[1])
            stack += [nodes[x[1]][1], nodes[x[1]][2]]
    return nodes, need, out


def emit(B):
    nodes, need, out = network(B)
    ref = lambda o: f"x[{o[1]}]" if o[0] == "x" else f"n{o[1]}"
    lines = [f"template <> struct MidNet<{B}> {{",
             f"  template <typename K> __device__ __forceinline__ static K run(const K (&x)[{B}]) {{"]
    for i in sorted(need):
        op, a, b = nodes[i]
        lines.append(f"    const K n{i} = k{op}({ref(a)}, {ref(b)});")
    lines.append(f"    return {ref(out)};")
    lines.append("  }")
    lines.append("};")
    return "\n".join(lines), len(need)


def check_midnet(B, cols=4096, seed=0):
    """Evaluates the pruned network on random columns with many ties: the rank-(B-1)//2 key."""
    import numpy as np
    nodes, need, out = network(B)
    rng = np.random.default_rng(seed + B)
    x = rng.integers(0, 7, size=(B, cols)).astype(np.float64)
    x[:, : cols // 2] = rng.standard_normal((B, cols // 2))
    val = {}
    get = lambda o: x[o[1]] if o[0] == "x" else val[o[1]]
    for i in sorted(need):
        op, a, b = nodes[i]
        val[i] = (np.minimum if op == "min" else np.maximum)(get(a), get(b))
    assert (get(out) == np.sort(x, axis=0)[(B - 1) // 2]).all(), B


def check_sortnet(N, ops, pos, cols=4096, seed=0):
    import numpy as np
    rng = np.random.default_rng(seed + 1000 + N)
    x = rng.integers(0, 5, size=(N, cols)).astype(np.float64)
    x[:, : cols // 2] = rng.standard_normal((N, cols // 2))
    val = {}
    get = lambda o: x[o[1]] if o[0] == "x" else val[o[1]][0 if o[2] == "min" else 1]
    for a, b, t in ops:
        val[t] = (np.minimum(get(a), get(b)), np.maximum(get(a), get(b)))
    assert (np.stack([get(pos[i]) for i in range(N)]) == np.sort(x, axis=0)).all(), N


def main(path):
    verify_g16()
    body, counts = [], {}
    for B in BUCKETS:
        check_midnet(B)
        code, ops = emit(B)
        counts[B] = ops
        body.append(f"// B = {B}: {ops} min/max ops\n" + code)
    body.append("template <int B, typename K> __device__ __forceinline__ K select_mid(const K (&x)[B]) {\n"
                "  return MidNet<B>::run(x);\n}")
    # k_median_2l / k_median_4l (robust.hip): a column's B keys split over two (four) lanes, N = B/2
    # (B/4) keys each; every lane sorts its N keys in place (all N outputs are used by the merge).
    # Network: odd-even merge sort of the next power of two >= N with the extra inputs compile-time
    # high sentinels folded away (a comparator with a constant input is a renaming).
    lines = ["template <int N> struct SortNet;"]
    counts2 = {}
    for N in [32] + list(range(36, 65, 4)):
        P2 = 1 << (N - 1).bit_length()  # network of the next power of two (32 for N = 32)
        pos = [("x", i) for i in range(N)] + [("H",)] * (P2 - N)
        ops = []
        tmp = 0
        for i, j in oddeven_merge_sort(P2):
            a, b = pos[i], pos[j]
            if a[0] == "H" and b[0] == "H":
                continue
            if a[0] == "H" or b[0] == "H":  # the constant high goes to the max side
                pos[i], pos[j] = (b, a) if a[0] == "H" else (a, b)
                continue
            ops.append((a, b, tmp))
            pos[i], pos[j] = ("t", tmp, "min"), ("t", tmp, "max")
            tmp += 1
        assert all(pos[i][0] != "H" for i in range(N))
        check_sortnet(N, ops, pos)
        # emit in SSA over named temporaries; the outputs are copied back to x[0..N-1]
        ref = lambda o: f"x[{o[1]}]" if o[0] == "x" else ("i" if o[2] == "min" else "a") + str(o[1])
        L = [f"template <> struct SortNet<{N}> {{",
             f"  template <typename K> __device__ __forceinline__ static void run(K (&x)[{N}]) {{"]
        for a, b, t in ops:
            L.append(f"    const K i{t} = kmin({ref(a)}, {ref(b)}), a{t} = kmax({ref(a)}, {ref(b)});")
        moved = [i for i in range(N) if pos[i] != ("x", i)]
        for i in moved:  # read every output before any x[] is overwritten
            L.append(f"    const K o{i} = {ref(pos[i])};")
        for i in moved:
            L.append(f"    x[{i}] = o{i};")
        L += ["  }", "};"]
        lines.append("\n".join(L))
        counts2[N] = 2 * len(ops)
    body.append("// SortNet<N>::run(x): x[0..N-1] ascending (k_median_2l, k_median_4l); min/max per N: " + str(counts2) +
                "\n" + "\n\n".join(lines))
    hdr = (
        "// median_nets.h -- GENERATED by tools/gen_median_nets.py; do not edit.\n"
        "// MidNet<B>::run(keys): the key at rank (B-1)/2 of B keys, by a pruned Batcher odd-even merge\n"
        + ("// network of the next power of two (16-key blocks: a 60-comparator network) with compile-time\n"
           "// sentinels folded away.  Keys: uint32 or\n" if BASE16 else
           "// network of the next power of two with compile-time sentinels folded away.  Keys: uint32 or\n") +
        "// float (one coordinate per lane) or two uint16 keys packed in 32 bits (two coordinates per lane,\n"
        "// v_pk_min_u16 / v_pk_max_u16).  Used by the k_median kernels (robust.hip).\n"
        "#pragma once\n\n"
        "typedef unsigned short fa_u16x2 __attribute__((ext_vector_type(2)));\n"
        "__device__ __forceinline__ unsigned kmin(unsigned a, unsigned b) { return min(a, b); }\n"
        "__device__ __forceinline__ unsigned kmax(unsigned a, unsigned b) { return max(a, b); }\n"
        "__device__ __forceinline__ fa_u16x2 kmin(fa_u16x2 a, fa_u16x2 b) { return __builtin_elementwise_min(a, b); }\n"
        "__device__ __forceinline__ fa_u16x2 kmax(fa_u16x2 a, fa_u16x2 b) { return __builtin_elementwise_max(a, b); }\n"
        "// float keys (r03): IEEE 754-2019 minimum / maximum -- one v_minimum3_f32 / v_maximum3_f32 on gfx950,\n"
        "// no input canonicalisation, -0 < +0, and a NaN input turns both outputs NaN, so a column with a NaN\n"
        "// selects NaN (every input reaches the selected output) -- no per-key conversion or NaN test.\n"
        "__device__ __forceinline__ float kmin(float a, float b) { return __builtin_elementwise_minimum(a, b); }\n"
        "__device__ __forceinline__ float kmax(float a, float b) { return __builtin_elementwise_maximum(a, b); }\n\n"
        "template <int B> struct MidNet;\n\n"
    )
    with open(path, "w") as f:
        f.write(hdr + "\n\n".join(body) + "\n")
    print(counts)


if __name__ == "__main__":
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    args = [a for a in sys.argv[1:] if a != "--batcher"]
    main(args[0] if args else os.path.join(root, "fedml_amd", "csrc", "median_nets.h"))
