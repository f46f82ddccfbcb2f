"""k_pairdist_rot's task map (fedml_amd/csrc/pairrot.hip rot_slot / rot_pair), restated: for every
K = 2..128 each pair i < j < K comes from exactly one (slot, lane r, accumulator m) -- the kernel
writes every partial-sum entry once, and no accumulator of a real pair is dropped."""
from collections import Counter

import pytest


def rot_slot(s, G):
    nx = G * (G - 1) // 2
    if s < nx:
        i, rem = 0, s
        while rem >= G - 1 - i:
            rem -= G - 1 - i
            i += 1
        return i, i + 1 + rem, True
    if s < nx + (G + 1) // 2:
        a = 2 * (s - nx)
        return a, (a + 1 if a + 1 < G else -1), False
    return -1, -1, False


def rot_pair(a, b, cross, r, m, k):
    if a < 0:
        return None
    if cross:
        i, j = 16 * a + r, 16 * b + ((r + m) & 15)
        return (i, j) if j < k else None
    g, d = (a, m + 1) if m < 8 else (b, m - 7)
    if g < 0 or (d == 8 and r >= 8):
        return None
    x, y = 16 * g + r, 16 * g + ((r + d) & 15)
    i, j = min(x, y), max(x, y)
    return (i, j) if j < k else None


@pytest.mark.parametrize("k", list(range(2, 129)))
def test_every_pair_once(k):
    G = (k + 15) // 16
    nslots = G * (G - 1) // 2 + (G + 1) // 2
    wpt = (nslots + 1) // 2
    assert wpt <= 16  # one task set fits a 1,024-thread workgroup
    c = Counter()
    for js in range(2 * wpt):
        a, b, x = rot_slot(js, G)
        for r in range(16):
            for m in range(16):
                p = rot_pair(a, b, x, r, m, k)
                if p:
                    c[p] += 1
    assert set(c) == {(i, j) for i in range(k) for j in range(i + 1, k)}
    assert set(c.values()) == {1}
