# r03s: full GPU suite + smoke + default bench + cfg5/samask/lr lines after this session's kernel changes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
for c in gossip samask lr; do
  timeout -k 10 400 python bench.py --config $c > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || { tail -20 gpurun_out/bench_$c.err; exit 1; }
  C=$c python -c 'import json,os;d=json.load(open("gpurun_out/bench_%s.json" % os.environ["C"]));print(os.environ["C"], d["value"], d["unit"], (d.get("roofline") or {}).get("frac"), (d.get("cpu_baseline") or {}).get("value"), d.get("parity"))'
done
