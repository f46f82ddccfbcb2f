"""Restatement of numpy's legacy RandomState(seed).randint(0, p, size) -- TEST INFRASTRUCTURE ONLY.

SecAgg's server re-expands every client's mask with `np.random.seed(s); np.random.randint(0, p,
size=d)` (python/fedml/cross_silo/secagg/sa_fedml_aggregator.py:104-131).  The algorithm lives in
numpy (a third-party dependency of the reference, `numpy` in python/setup.py; legacy RandomState
streams are frozen across numpy versions), restated here from its published source:
  numpy/random/_mt19937.pyx `_legacy_seeding` -> mt19937_seed (init_genrand, Matsumoto-Nishimura),
  numpy/random/src/mt19937/mt19937.c mt19937_gen / mt19937_next (twist + tempering),
  numpy/random/src/distributions/distributions.c random_bounded_uint64_fill with use_masked=True
  (rng = p - 1 <= 0xFFFFFFFF: 32-bit draws, mask = smallest 2^k - 1 >= rng, reject draw & mask >
  rng; larger rng: 64-bit draws next32 << 32 | next32, same masked rejection).
Pinned against numpy.random itself by tests/test_oracle_finite.py (the checker's checker); the
device kernel (fa_mt_randint_sum) is compared with numpy and with this restatement.  Vectorised
with numpy per twist block; fine for the sizes the tests use.
"""
from __future__ import annotations

import numpy as np

N, M = 624, 397
MATRIX_A, UPPER, LOWER = np.uint32(0x9908B0DF), np.uint32(0x80000000), np.uint32(0x7FFFFFFF)


def seed_state(seed: int) -> np.ndarray:
    if not 0 <= int(seed) <= 0xFFFFFFFF:
        raise ValueError("Seed must be between 0 and 2**32 - 1")
    mt = np.empty(N, dtype=np.uint32)
    x = int(seed)
    for i in range(N):
        mt[i] = x
        x = (1812433253 * (x ^ (x >> 30)) + i + 1) & 0xFFFFFFFF
    return mt


def twist(mt: np.ndarray) -> None:
    """mt19937_gen in place, in the three dependency-free ranges."""
    def mix(cur, nxt, far):
        y = (cur & UPPER) | (nxt & LOWER)
        return far ^ (y >> np.uint32(1)) ^ np.where(y & np.uint32(1), MATRIX_A, np.uint32(0))
    a = N - M
    mt[:a] = mix(mt[:a], mt[1:a + 1], mt[M:N])
    mt[a:2 * a] = mix(mt[a:2 * a], mt[a + 1:2 * a + 1], mt[0:a])
    nxt = np.concatenate([mt[2 * a + 1:N], mt[0:1]])
    mt[2 * a:N] = mix(mt[2 * a:N], nxt, mt[a:N - a])


def temper(y: np.ndarray) -> np.ndarray:
    y = y ^ (y >> np.uint32(11))
    y = y ^ ((y << np.uint32(7)) & np.uint32(0x9D2C5680))
    y = y ^ ((y << np.uint32(15)) & np.uint32(0xEFC60000))
    return y ^ (y >> np.uint32(18))


def randint(seed: int, p: int, n: int) -> np.ndarray:
    """np.random.seed(seed); np.random.randint(0, p, size=n) (int64)."""
    rng = int(p) - 1
    out = np.zeros(n, dtype=np.int64)
    if rng == 0 or n == 0:
        seed_state(seed)
        return out
    mask = rng
    for sh in (1, 2, 4, 8, 16, 32):
        mask |= mask >> sh
    mt = seed_state(seed)
    got = 0
    while got < n:
        twist(mt)
        w = temper(mt).astype(np.uint64)
        if rng <= 0xFFFFFFFF:
            v = w & np.uint64(mask)
        else:
            v = ((w[0::2] << np.uint64(32)) | w[1::2]) & np.uint64(mask)
        v = v[v <= np.uint64(rng)]
        take = min(n - got, v.size)
        out[got:got + take] = v[:take].astype(np.int64)
        got += take
    return out


def randint_sum(seeds, signs, p: int, n: int) -> np.ndarray:
    """mod(sum_s sign_s * randint(seed_s, p, n), p) in [0, p) -- fa_mt_randint_sum's contract."""
    acc = np.zeros(n, dtype=object)
    for s, g in zip(seeds, signs):
        acc = acc + int(g) * randint(s, p, n).astype(object)
    return np.array([int(a) % int(p) for a in acc], dtype=np.int64)
