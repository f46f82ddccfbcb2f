# r06ai: the final bench.py after the clock-sampler change -- the driver's own `python bench.py` twice,
# the loopback rank chain, and cfg2 / cfg4 / Krum K = 128 lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06ai; mkdir -p $O
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};c=d.get('cold') or {};print(sys.argv[1].split('/')[-1],d['value'],d['ms_per_step'],d['warmup'],r.get('frac'),r.get('frac_of_ceiling'),'cold',c.get('ms'),(d.get('sustained') or {}).get('ms_per_step'),d['config'].get('arena_placement'),(d.get('cpu_baseline') or {}).get('value'),str(d.get('parity'))[:40])" $1; }
for i in 1 2; do
  timeout -k 10 400 python bench.py > $O/default_$i.json 2> $O/default_$i.err || { tail -5 $O/default_$i.err; exit 1; }
  line $O/default_$i.json
done
timeout -k 10 400 python bench.py --gpus 1 --self-launch --loopback --cold-reps 0 --no-cpu-baseline > $O/loopback.json 2> $O/loopback.err || { tail -5 $O/loopback.err; exit 1; }
line $O/loopback.json
for c in resnet18 hier "krum --clients 128"; do
  n=$(echo $c | tr -d ' -')
  timeout -k 10 400 python bench.py --config $c --no-cpu-baseline > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
  line $O/$n.json
done
exit 0
