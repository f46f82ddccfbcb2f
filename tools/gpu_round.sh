# One GPU session: parity tests, HBM probe, kernel-variant sweep, rocprofv3 evidence.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
fault() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -6 gpurun_out/pytest_gpu.log; fault $rc && exit $rc
timeout -k 10 200 python tools/hbm_probe.py 16 > gpurun_out/hbm_probe.json 2>gpurun_out/hbm_probe.err; rc=$?
cat gpurun_out/hbm_probe.json; fault $rc && exit $rc
for v in ${VARIANTS:-0 1 2 3 4 5 6 7 8}; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --variant $v > gpurun_out/bench_v$v.json 2>>gpurun_out/bench_sweep.err; rc=$?
  echo "variant $v: $(python -c "import json;d=json.load(open('gpurun_out/bench_v$v.json'));print(d['value'], d['roofline']['kernel_avg_ms'], d['parity'])")"
  fault $rc && exit $rc
done
[ -n "$NOPROF" ] || bash tools/profile.sh ${TAG:-r01}
