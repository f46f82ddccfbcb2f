# r04b: the metric on SEPARATELY allocated client tensors (SURVEY §8(d)'s literal input) + its rocprof;
# cfg2 separate tensors: host-phase probe, 3 interleaved bench lines, rocprof of k_wsum_pair; the host
# path (pinned / pageable, 16 M and the metric's 125 M) with parity; the self-launched one-rank chain.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r04b; mkdir -p $O
export TMPDIR=/tmp
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1],d['value'],d['unit'],d['ms_per_step'],r.get('kernel_avg_ms'),r.get('frac'),'|',d.get('parity'))" $1; }
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 420 python bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "FAIL $n"; tail -8 $O/$n.err; exit 1; }
  line $O/$n.json
}
run metric_tensors --layout tensors --steps 20 --warmup 5
BENCH_ARGS="--layout tensors --steps 5 --warmup 2 --no-cpu-baseline --check-samples 0" bash tools/profile.sh r04_metric_tensors || exit 1
timeout -k 10 300 python tools/cfg2_host_probe.py --out $O/cfg2_probe.json > $O/cfg2_probe.log 2>&1 || { echo "probe FAIL"; tail -8 $O/cfg2_probe.log; exit 1; }
cat $O/cfg2_probe.json
for rep in 1 2 3; do
  run cfg2_tensors_r$rep --config resnet18 --layout tensors --steps 50 --warmup 10 --no-cpu-baseline
  run cfg2_tiled_r$rep --config resnet18 --steps 50 --warmup 10 --no-cpu-baseline
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cfg2prof -o run -- python3 bench.py --config resnet18 --layout tensors --steps 50 --warmup 10 --no-cpu-baseline > $O/cfg2prof.json 2> $O/cfg2prof.err || { echo "rocprof cfg2 FAIL"; tail -5 $O/cfg2prof.err; exit 1; }
find $O/cfg2prof -name "*kernel_stats.csv" -exec cp {} $O/cfg2_tensors_kernel_stats.csv \;
head -5 $O/cfg2_tensors_kernel_stats.csv
run host_pinned_16M --config host --pinned --steps 5 --warmup 2
run host_pageable_16M --config host --steps 5 --warmup 2
timeout -k 10 300 python bench.py --gpus 1 --self-launch --steps 10 --warmup 3 --no-cpu-baseline > $O/selflaunch.json 2> $O/selflaunch.err || { echo "self-launch FAIL"; tail -8 $O/selflaunch.err; exit 1; }
line $O/selflaunch.json
run host_pageable_125M --config host --params 125000000 --steps 3 --warmup 1
run host_pinned_125M --config host --pinned --params 125000000 --steps 3 --warmup 1
