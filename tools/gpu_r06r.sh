# r06r: contiguous arenas in the product (ClientArena -> fa_device_alloc_contiguous): the new tests,
# then the default line in 8 fresh processes alternating FEDML_AMD_ARENA_ALLOC=contiguous / torch.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06r; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_arena_contig.py tests/test_gpu_tiled.py > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc = 0 ] || exit $rc
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1].split('/')[-1],d['value'],d['ms_per_step'],r.get('frac'),r.get('frac_of_ceiling'),d['config'].get('arena_alloc'),(d.get('clock') or {}).get('gfx_mhz'),str(d.get('parity'))[:40])" $1; }
for i in 1 2 3 4; do
  for a in contiguous torch; do
    FEDML_AMD_ARENA_ALLOC=$a timeout -k 10 300 python bench.py --no-cpu-baseline --cold-reps 0 --soak-seconds 0 > $O/metric_${a}_$i.json 2> $O/metric_${a}_$i.err || { tail -5 $O/metric_${a}_$i.err; exit 1; }
    line $O/metric_${a}_$i.json
  done
done
exit 0
