"""Host-side pieces of SecAgg's server (python/fedml/core/mpc/secagg.py) the mask re-expansion needs.

BGW decoding of one secret from T + 1 shares is O(T^2) scalar work on the host (control logic);
what it produces are the PRG seeds whose numpy MT19937 streams form the aggregate mask -- those
streams are expanded on the device (fa_mt_randint_sum, include/fedagg_finite.h).  The modular
helpers are lightsecagg.py's (the reference's secagg.py:8-38 copies them; PI there starts from
np.int64(1), which wraps identically).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np

from .lightsecagg import PI, divmod  # noqa: A004


def gen_BGW_lambda_s(alpha_s, p):  # noqa: N802  (the reference's name)
    """secagg.py:180-189: Lagrange coefficients at 0 of the evaluation points alpha_s."""
    lambda_s = np.zeros((1, len(alpha_s)), dtype="int64")
    for i in range(len(alpha_s)):
        cur = alpha_s[i]
        den = PI([cur - o for o in alpha_s if cur != o], p)
        num = PI([0 - o for o in alpha_s if cur != o], p)
        lambda_s[0][i] = divmod(num, den, p)
    return lambda_s.astype("int64")


def BGW_decoding(f_eval, worker_idx, p):  # noqa: N802
    """secagg.py:192-210: the secret from the shares f_eval [RT x d] of workers worker_idx."""
    alpha_s = np.array(np.int64(np.mod(range(1, np.max(worker_idx) + 2), p)))
    lambda_s = gen_BGW_lambda_s([alpha_s[i] for i in worker_idx], p).astype("int64")
    return np.mod(np.dot(lambda_s, f_eval), p)


def _seed(v) -> int:
    """np.random.seed's legacy check (numpy/random/_mt19937.pyx _legacy_seeding)."""
    v = int(v)
    if v > 2 ** 32 - 1 or v < 0:
        raise ValueError("Seed must be between 0 and 2**32 - 1")
    return v


def mask_streams(num_clients: int, flags, active_clients: Sequence[int], SS_rx, public_key_list, T: int,
                 p: int) -> Tuple[List[int], List[int]]:
    """The (seed, sign) streams of sa_fedml_aggregator.py:92-136's loop, in its order: a client whose
    model arrived (flag set) contributes +randint(seed = its decoded b_u); a dropped client i
    contributes, for every j != i, -randint(s_uv) (j < i) or +randint(s_uv) (j > i) with
    s_uv = np.mod(s_sk_dec * pk_j, p) in numpy int64 (wrapping) arithmetic.  Seeds are checked as
    np.random.seed checks them, at the same point of the loop."""
    seeds, signs = [], []
    idx = list(active_clients[: T + 1])
    for i in range(num_clients):
        shares = np.reshape(SS_rx[i, idx], (T + 1, 1))
        dec = BGW_decoding(shares, idx, p)
        if flags[i]:
            seeds.append(_seed(dec[0][0]))
            signs.append(1)
            continue
        pk = public_key_list[1, :]
        for j in range(num_clients):
            s_uv = np.mod(dec[0][0] * pk[j], p)
            if j == i:
                continue
            seeds.append(_seed(s_uv))
            signs.append(-1 if j < i else 1)
    return seeds, signs
