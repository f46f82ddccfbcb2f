# r05zf: bench.py's default warmup (3 steps, then ~0.2 s of the workload's own steps on one GPU):
# the default line and short-step config lines with no --warmup flag.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05zf; mkdir -p $O
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1].split('/')[-1],d['value'],d['unit'],d['ms_per_step'],d['warmup'],r.get('kernel_avg_ms'),r.get('frac'),d.get('parity'))" $1; }
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/default.json 2> $O/default.err || { tail -10 $O/default.err; exit 1; }
line $O/default.json
for c in "krum --clients 32" "median --clients 128" "resnet18 --layout tensors" "resnet18"; do
  n=$(echo $c | tr ' ' '_' | tr -d '-')
  timeout -k 10 400 python bench.py --config $c --no-cpu-baseline --soak-seconds 0 > $O/$n.json 2> $O/$n.err || { tail -10 $O/$n.err; exit 1; }
  line $O/$n.json
done
