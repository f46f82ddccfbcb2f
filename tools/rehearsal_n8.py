#!/usr/bin/env python
"""The bench's own N-rank chain on the CPU (parent -> torch.distributed.run -> N gloo ranks), for the
metric (ordered / ordered_all / reduce_scatter), hier and gossip configs, with the local reductions
of tests/rehearsal_engine.py (the C oracle) injected.  Writes one JSON line per run (the bench's
line plus the wall time) to the given path; exits 1 if any run fails or is not bit-exact.

    python tools/rehearsal_n8.py profiles/r05/rehearsal_n8.jsonl [--gpus 8]
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

RUNS = [
    ["--config", "metric", "--clients", "128", "--params", "40000"],
    ["--config", "metric", "--clients", "128", "--params", "40000", "--collective", "ordered_all"],
    ["--config", "metric", "--clients", "128", "--params", "40000", "--collective", "reduce_scatter"],
    ["--config", "metric", "--clients", "128", "--params", "40000", "--layout", "arena", "--chunks", "3"],
    ["--config", "hier", "--clients", "64", "--params", "8000"],
    ["--config", "hier", "--clients", "64", "--params", "8000", "--collective", "ordered_all"],
    ["--config", "gossip", "--clients", "256", "--params", "3000"],
]


def run(extra, gpus=8, timeout=600):
    env = dict(os.environ, FEDML_AMD_BENCH_REHEARSAL="cpu", FEDML_AMD_BENCH_ENGINE="rehearsal_engine:make",
               PYTHONPATH=os.path.join(ROOT, "tests") + os.pathsep + os.environ.get("PYTHONPATH", ""),
               OMP_NUM_THREADS="1")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--steps", "2", "--warmup", "1",
           "--soak-seconds", "0", "--no-cpu-baseline"] + extra
    t0 = time.perf_counter()
    p = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=timeout)
    wall = time.perf_counter() - t0
    lines = [ln for ln in p.stdout.splitlines() if ln.lstrip().startswith("{")]
    if p.returncode != 0 or not lines:
        err = p.stderr
        i = err.find("Traceback")  # the first rank's failure, not the launcher's summary of it
        raise RuntimeError(f"{' '.join(extra)}: rc {p.returncode}\n{err[i:i + 4000] if i >= 0 else err[-3000:]}")
    d = json.loads(lines[-1])
    d["rehearsal_cmd"] = "bench.py --gpus %d %s" % (gpus, " ".join(extra))
    d["rehearsal_wall_s"] = round(wall, 2)
    return d


def main(path, gpus=8):
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    bad = 0
    with open(path, "w") as f:
        for extra in RUNS:
            d = run(extra, gpus)
            # reduce / all_reduce / reduce_scatter sum in the backend's order: 1e-6 normwise
            backend_order = any(c in extra for c in ("reduce", "all_reduce", "reduce_scatter"))
            ok = d["n_gpus"] == gpus and (d["parity"].startswith("bit-exact") or
                                          (backend_order and d["parity"].startswith("within 1e-6")))
            bad += not ok
            f.write(json.dumps(d) + "\n")
            f.flush()
            print(f"{'ok ' if ok else 'BAD'} {d['rehearsal_wall_s']:6.1f} s  {d['rehearsal_cmd']}: {d['parity']}")
    return 1 if bad else 0


if __name__ == "__main__":
    g = 8
    if "--gpus" in sys.argv:
        g = int(sys.argv[sys.argv.index("--gpus") + 1])
    sys.exit(main(sys.argv[1], g))
