"""CPU check of the generated selection networks (fedml_amd/csrc/median_nets.h, tools/
gen_median_nets.py): every MidNet<B> returns the lower median of B keys, on random keys with
many ties, and the committed header is what the generator produces."""
from __future__ import annotations

import os
import random
import re
import sys

import pytest

from conftest import ROOT

HDR = os.path.join(ROOT, "fedml_amd", "csrc", "median_nets.h")


def _networks():
    src = open(HDR).read()
    out = {}
    for m in re.finditer(r"struct MidNet<(\d+)> \{\n.*?static K run\(const K \(&x\)\[\d+\]\) \{\n(.*?)\n  \}\n\};",
                         src, re.S):
        out[int(m.group(1))] = [l.strip() for l in m.group(2).split("\n")]
    return out


def _run(stmts, x):
    env = {}
    val = lambda t: x[int(t[2:-1])] if t.startswith("x[") else env[t]
    for s in stmts:
        m = re.match(r"const K (n\d+) = k(min|max)\(([^,]+), ([^)]+)\);", s)
        if m:
            a, b = val(m.group(3)), val(m.group(4))
            env[m.group(1)] = min(a, b) if m.group(2) == "min" else max(a, b)
            continue
        m = re.match(r"return (.+);", s)
        assert m, s
        return val(m.group(1))


def test_all_buckets_present():
    assert sorted(_networks()) == list(range(8, 129, 8))


@pytest.mark.parametrize("B", list(range(8, 129, 8)))
def test_network_selects_lower_median(B):
    stmts = _networks()[B]
    rng = random.Random(B)
    for trial in range(100):
        hi = rng.choice([3, 40, 2 ** 32 - 1])  # heavy ties .. distinct
        x = [rng.randrange(0, hi) for _ in range(B)]
        assert _run(stmts, x) == sorted(x)[(B - 1) // 2], (B, trial)


def test_header_matches_generator(tmp_path):
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import gen_median_nets
    out = tmp_path / "nets.h"
    gen_median_nets.main(str(out))
    assert out.read_text() == open(HDR).read()
