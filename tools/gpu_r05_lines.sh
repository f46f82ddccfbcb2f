# r05: the config lines at the chip's sustained clock.  r05t (tools/host_cost_probe.py): the Krum K = 32
# pass ran 337 -> 288 -> 279 us per call over three consecutive 40-call reps after 5 warmup calls
# (the host issues a call in ~40 us): a few ms of warmup leave short-step lines on the clock ramp.
# Here every short-step line warms up for >= ~100 ms of its own work before its timed steps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05_lines; mkdir -p $O
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1].split('/')[-1],d['value'],d['unit'],d['ms_per_step'],r.get('kernel_avg_ms'),r.get('frac'),(d.get('sustained') or {}).get('ms_per_step'),d.get('parity'))" $1; }
B="--no-cpu-baseline --soak-seconds 2"
cfg() {
  n=$1; shift
  timeout -k 10 400 python bench.py $B "$@" > $O/$n.json 2> $O/$n.err || { tail -10 $O/$n.err; exit 1; }
  line $O/$n.json
}
cfg cfg2_tiled --config resnet18 --layout tiled --steps 100 --warmup 400
cfg cfg2_tensors --config resnet18 --layout tensors --steps 100 --warmup 400
cfg cfg3_vit --config vit_bf16 --steps 30 --warmup 30
cfg cfg4_hier --config hier --steps 30 --warmup 30
cfg cfg5_gossip --config gossip --steps 30 --warmup 30
cfg median32 --config median --clients 32 --steps 100 --warmup 400
cfg median128 --config median --clients 128 --layout tiled --steps 50 --warmup 100
cfg krum32 --config krum --clients 32 --steps 100 --warmup 300 --check-samples 1
cfg krum64 --config krum --clients 64 --steps 50 --warmup 100 --check-samples 1
cfg krum128 --config krum --clients 128 --steps 30 --warmup 50 --check-samples 1
cfg secagg --config secagg --steps 30 --warmup 50
exit 0
