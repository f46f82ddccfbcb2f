set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
fault() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_gpu.log; fault $rc && exit $rc
for c in metric resnet18 vit_bf16 hier gossip; do
  timeout -k 10 400 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/arena_$c.json 2> gpurun_out/arena_$c.err; rc=$?
  echo "== $c rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/arena_$c.json'));print(d['value'], d['ms_per_step'], d['roofline']['achieved'], d['roofline']['frac'], d['parity'])")"
  fault $rc && exit $rc
done
for v in 0 4 6 7 8; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --variant $v > gpurun_out/arena_v$v.json 2>>gpurun_out/arena_sweep.err; rc=$?
  echo "variant $v: $(python -c "import json;d=json.load(open('gpurun_out/arena_v$v.json'));print(d['value'], d['roofline']['kernel_avg_ms'], d['parity'])")"
  fault $rc && exit $rc
done
