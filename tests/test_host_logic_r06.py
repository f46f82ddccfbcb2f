"""Host-side logic added in round 6, on the CPU (no HIP call):
  * the Krum kappa memo's decision (AggEngine._gram_memo_form): copy kappa_max on a shape's first call
    and every GRAM_RETRY-th call after it; go straight to the direct kernels while the last copied
    kappa_max said the guard fell back, except on those re-check calls; never read a copy whose
    event has not completed;
  * the bench line's `clock` block (bench.ClockSampler.summary) and its no-op path when amdsmi cannot
    read the table."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class _Ev:
    def __init__(self, done=True):
        self.done = done

    def query(self):
        return self.done


def _engine():
    from fedml_amd.engine import AggEngine
    return AggEngine.__new__(AggEngine)  # no native context: only the memo's bookkeeping is used


def _memo(eng, key, km, limit, done=True):
    eng.__dict__.setdefault("_gram_memo", {})[key] = {"km": torch.tensor([km], dtype=torch.float64), "calls": 0,
                                                      "fell": False, "ev": _Ev(done), "limit": limit,
                                                      "pending": True}


def test_memo_first_call_copies_and_runs_the_gram_form():
    eng = _engine()
    assert eng._gram_memo_form((12, (100,))) == (False, True)


def test_memo_sticky_direct_with_periodic_recheck():
    eng = _engine()
    key = (12, (50_021,))
    _memo(eng, key, float("inf"), 16.0)  # the first call's copy: fell back
    R = eng.GRAM_RETRY
    seen = [eng._gram_memo_form(key) for _ in range(2 * R)]
    # calls 1..R-1 direct without a copy; call R re-checks (Gram form + copy); then direct again
    assert seen[:R - 1] == [(True, False)] * (R - 1)
    assert seen[R - 1] == (False, True)
    assert seen[R:2 * R - 1] == [(True, False)] * (R - 1)


def test_memo_recovers_when_the_recheck_passes():
    eng = _engine()
    key = (40, (7850,))
    _memo(eng, key, float("inf"), 12.0)
    R = eng.GRAM_RETRY
    for _ in range(R - 1):
        assert eng._gram_memo_form(key)[0]
    assert eng._gram_memo_form(key) == (False, True)  # re-check call
    m = eng._gram_memo[key]
    m["km"][0], m["pending"], m["ev"] = 3.0, True, _Ev(True)  # its copy: within the limit
    assert eng._gram_memo_form(key) == (False, False)   # Gram form again, no copy


def test_memo_never_reads_an_unfinished_copy():
    eng = _engine()
    key = (64, (11_699_132,))
    _memo(eng, key, float("inf"), 16.0, done=False)  # the copy is still in flight
    assert eng._gram_memo_form(key) == (False, False)  # treated as not fallen back
    eng._gram_memo[key]["ev"].done = True
    assert eng._gram_memo_form(key) == (True, False)


def test_clock_summary_and_missing_table():
    import bench
    cs = bench.ClockSampler.__new__(bench.ClockSampler)
    cs.period, cs.h, cs.err = 0.01, None, "RuntimeError: no table"
    with cs as c:
        pass
    assert c.summary() == {"error": "RuntimeError: no table"}
    cs.samples = [{"gfx_mhz": 2300.0 + i, "mem_mhz": 2000.0, "power_w": 900.0, "hotspot_c": 47.0, "hbm_c": None,
                   "throttle": i % 2} for i in range(5)]
    s = cs.summary()
    assert s["samples"] == 5 and s["gfx_mhz"] == {"median": 2302.0, "min": 2300.0, "max": 2304.0}
    assert "hbm_c" not in s and s["throttle_frac"] == 0.4
    with bench.ClockSampler.maybe(None) as z:
        assert z is None
    assert cs.sample_now() == {"error": "RuntimeError: no table"}
