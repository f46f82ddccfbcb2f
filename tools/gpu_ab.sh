# Interleaved A/B of kernel variants (3 rounds), host-path bench, and rocprof of the default bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
fault() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
for rep in 1 2 3; do
  for v in ${VARIANTS:-0 4 7}; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --check-samples 0 --variant $v > gpurun_out/ab_v${v}_$rep.json 2>>gpurun_out/ab.err; rc=$?
    fault $rc && exit $rc
    echo "rep $rep variant $v: $(python -c "import json;d=json.load(open('gpurun_out/ab_v${v}_$rep.json'));print(d['value'], d['roofline']['kernel_avg_ms'])")"
  done
done
for extra in "" "--pinned"; do
  timeout -k 10 400 python bench.py --config host --steps 3 --warmup 1 --no-cpu-baseline $extra > gpurun_out/host$extra.json 2>gpurun_out/host.err; rc=$?
  fault $rc && exit $rc
  echo "host $extra: $(cat gpurun_out/host$extra.json)"
done
BENCH_ARGS="--config resnet18 --steps 5 --warmup 2 --no-cpu-baseline --check-samples 0" timeout -k 10 400 bash tools/profile.sh r01_resnet18 > gpurun_out/prof_resnet.log 2>&1; rc=$?; tail -5 gpurun_out/prof_resnet.log
fault $rc && exit $rc
bash tools/profile.sh r01 2>&1 | tail -30
