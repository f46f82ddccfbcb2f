# r03af: regression after the float-key median networks -- GPU suite, smoke, default bench, the median
# bench lines (K = 32 / 128 with their CPU baselines, K = 64 / 100).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03af
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03af/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r03af/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r03af/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03af/smoke.log 2>&1 || { cat gpurun_out/r03af/smoke.log; exit 1; }
tail -1 gpurun_out/r03af/smoke.log
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 420 python bench.py "$@" > gpurun_out/r03af/$n.json 2> gpurun_out/r03af/$n.err || { echo "FAIL $n"; tail -5 gpurun_out/r03af/$n.err; exit 1; }
  N=$n python -c 'import json,os;n=os.environ["N"];d=[json.loads(l) for l in open("gpurun_out/r03af/%s.json" % n) if l.startswith("{")][-1];r=d.get("roofline") or {};c=d.get("cpu_baseline") or {};print(n, d["value"], d["unit"], d.get("ms_per_step"), r.get("kernel_avg_ms"), r.get("frac"), c.get("value"), c.get("unit"), "|", d.get("parity"))'
}
run metric
run median32 --config median --clients 32
run median128 --config median --clients 128
run median64 --config median --clients 64 --no-cpu-baseline
run median100 --config median --clients 100 --no-cpu-baseline
