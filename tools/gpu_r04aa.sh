# r04aa: ragged last tile first (workgroup 0) + unrolled scalar tail loops in the wsum / grouped
# kernels -- weighted-sum GPU tests, then hier at P = 11.70 / 12.58 / 10.49 M with and without the
# tail split, the metric (default) and cfg2, 2 reps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r04aa; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_tiled.py tests/test_gpu_configs.py > $O/pytest.txt 2>&1 \
  || { echo "pytest FAIL"; tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1],d['value'],d['unit'],d['ms_per_step'],r.get('kernel_avg_ms'),r.get('frac'),'|',(d.get('parity') or '')[:30])" $1; }
b() { n=$1; shift; timeout -k 10 300 python bench.py "$@" --steps 20 --warmup 3 --no-cpu-baseline --soak-seconds 0 > $O/$n.json 2> $O/$n.err || { echo "FAIL $n"; tail -8 $O/$n.err; exit 1; }; line $O/$n.json; }
for rep in 1 2; do
  for P in 11699132 12582912 10485760; do
    b hier_P${P}_r$rep --config hier --params $P --check-samples 0
    FA_GROUPED_SPLIT=0 b hier_P${P}_nosplit_r$rep --config hier --params $P --check-samples 0
  done
  b metric_r$rep
  b resnet18_r$rep --config resnet18
done
b hier_parity --config hier
