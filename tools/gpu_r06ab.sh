# r06ab: the arena placement check in the product (ClientArena._place: re-allocate a 16+ GiB tiled
# group whose quick kernel / read-probe ratio exceeds 1.07, best of at most 3 blocks): its GPU tests,
# then the driver's own `python bench.py` in 5 fresh processes (each line names its ratios).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06ab; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_arena_contig.py > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc = 0 ] || exit $rc
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};c=d.get('cold') or {};print(sys.argv[1].split('/')[-1],d['value'],d['ms_per_step'],r.get('frac'),r.get('frac_of_ceiling'),'cold',c.get('ms'),d['config'].get('arena_placement'),str(d.get('parity'))[:30])" $1; }
for i in 1 2 3 4 5; do
  timeout -k 10 400 python bench.py --no-cpu-baseline > $O/default_$i.json 2> $O/default_$i.err || { tail -5 $O/default_$i.err; exit 1; }
  line $O/default_$i.json
done
exit 0
