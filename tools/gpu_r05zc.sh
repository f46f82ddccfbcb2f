# r05zc: bench.py's loop-mode timing (one event pair around the timed steps instead of one per
# step, for workloads whose step is the timed call): the default line and the short-step lines at
# the sustained clock, with the per-launch mode's numbers from r05_lines / r05z for comparison.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05zc; mkdir -p $O
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1].split('/')[-1],d['value'],d['unit'],d['ms_per_step'],r.get('kernel_avg_ms'),r.get('bound'),r.get('frac'),(d.get('sustained') or {}).get('ms_per_step'),d.get('parity'))" $1; }
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
line $O/bench_default.json
B="--no-cpu-baseline --soak-seconds 2"
cfg() {
  n=$1; shift
  timeout -k 10 400 python bench.py $B "$@" > $O/$n.json 2> $O/$n.err || { tail -10 $O/$n.err; exit 1; }
  line $O/$n.json
}
cfg cfg2_tiled --config resnet18 --layout tiled --steps 100 --warmup 400
cfg cfg2_tensors --config resnet18 --layout tensors --steps 100 --warmup 400
cfg cfg4_hier --config hier --steps 30 --warmup 30
cfg median32 --config median --clients 32 --steps 100 --warmup 400
cfg median128 --config median --clients 128 --layout tiled --steps 50 --warmup 100
cfg krum32 --config krum --clients 32 --steps 100 --warmup 300 --check-samples 1
cfg krum128 --config krum --clients 128 --steps 30 --warmup 50 --check-samples 1
cfg metric_tensors --config metric --layout tensors --steps 10 --warmup 5
exit 0
