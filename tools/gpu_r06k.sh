# r06k: the line's new `clock` block (amdsmi gpu_metrics sampled through the timed steps and the
# read probe): three default lines as fresh processes, then Krum K = 128 and median K = 128.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06k; mkdir -p $O
export TMPDIR=/tmp
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};c=r.get('measured_read_ceiling') or (r.get('hbm') or {});print(sys.argv[1].split('/')[-1],d['value'],d['ms_per_step'],r.get('frac'),r.get('frac_of_ceiling'),json.dumps(d.get('clock'))[:400]);print('  probe clock',json.dumps((r.get('measured_read_ceiling') or {}).get('clock'))[:300])" $1; }
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > $O/metric_$i.json 2> $O/metric_$i.err || { tail -5 $O/metric_$i.err; exit 1; }
  line $O/metric_$i.json
done
timeout -k 10 300 python bench.py --config krum --clients 128 --no-cpu-baseline --cold-reps 0 --check-samples 0 > $O/krum128.json 2> $O/krum128.err || { tail -5 $O/krum128.err; exit 1; }
line $O/krum128.json
timeout -k 10 300 python bench.py --config median --clients 128 --no-cpu-baseline --cold-reps 0 > $O/median128.json 2> $O/median128.err || { tail -5 $O/median128.err; exit 1; }
line $O/median128.json
exit 0
