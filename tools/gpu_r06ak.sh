# r06ak: the final tree -- the whole -m gpu suite, smoke(), the driver's own `python bench.py` twice,
# and cfg2 tiled / Krum K = 32 lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06ak; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};c=d.get('cold') or {};print(sys.argv[1].split('/')[-1],d['value'],d['ms_per_step'],r.get('kernel_avg_ms'),r.get('frac'),r.get('frac_of_ceiling'),'cold',c.get('ms'),(d.get('sustained') or {}).get('ms_per_step'),d['config'].get('arena_placement'),str(d.get('parity'))[:30])" $1; }
for i in 1 2; do
  timeout -k 10 400 python bench.py > $O/default_$i.json 2> $O/default_$i.err || { tail -5 $O/default_$i.err; exit 1; }
  line $O/default_$i.json
done
for c in resnet18 "krum --clients 32"; do
  n=$(echo $c | tr -d ' -')
  timeout -k 10 400 python bench.py --config $c --no-cpu-baseline > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
  line $O/$n.json
done
exit 0
