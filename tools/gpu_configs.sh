# All bench configurations on one GPU (1 JSON line each) + GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
fault() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
if [ -z "$NOTEST" ]; then
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_gpu.log; fault $rc && exit $rc
fi
for c in ${CONFIGS:-metric resnet18 vit_bf16 hier gossip}; do
  timeout -k 10 400 python bench.py --config $c --steps 10 --warmup 3 ${BENCH_EXTRA:-} > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err; rc=$?
  echo "== $c rc=$rc"; cat gpurun_out/bench_$c.json; tail -3 gpurun_out/bench_$c.err
  fault $rc && exit $rc
done
exit 0
