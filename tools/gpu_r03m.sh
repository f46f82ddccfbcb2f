# r03m: small host round (one-call C++ path + one-workgroup kernel + completion word): parity tests,
# then cfg1 latency A/B (FA_HOST1=1 / 0) with the reference loop timed in the same run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_host_small.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_host.log 2>&1 || { tail -30 gpurun_out/pytest_host.log; exit 1; }
tail -1 gpurun_out/pytest_host.log
for rep in 1 2 3; do
  for f in 1 0; do
    FA_HOST1=$f timeout -k 10 200 python bench.py --config lr --steps 3000 --warmup 200 $( [ $rep = 1 ] && [ $f = 1 ] || echo --no-cpu-baseline ) > gpurun_out/lr_$f.json 2> gpurun_out/lr_$f.err || { tail -5 gpurun_out/lr_$f.err; exit 1; }
    F=$f python -c 'import json,os;d=json.load(open("gpurun_out/lr_%s.json" % os.environ["F"]));print("host1", os.environ["F"], d["value"], d["unit"], d.get("parity"), (d.get("cpu_baseline") or {}).get("value"))'
  done
done
