# r04z: grouped-kernel tail split (per-group short tasks for the last partial round) -- grouped GPU
# tests (incl. the new split-size cases), then hier at P = 10.49 / 11.70 / 12.58 M with the split
# (default) and without (FA_GROUPED_SPLIT=0), 2 interleaved reps, and a parity run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r04z; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -k "group or hier or seq or tail_split" > $O/pytest_split.txt 2>&1 \
  || { echo "pytest split FAIL"; tail -40 $O/pytest_split.txt; exit 1; }
tail -1 $O/pytest_split.txt
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1],d['value'],d['unit'],d['ms_per_step'],r.get('kernel_avg_ms'),r.get('frac'),'|',(d.get('parity') or '')[:30])" $1; }
b() { n=$1; shift; timeout -k 10 200 python bench.py "$@" --steps 20 --warmup 3 --no-cpu-baseline --soak-seconds 0 > $O/$n.json 2> $O/$n.err || { echo "FAIL $n"; tail -8 $O/$n.err; exit 1; }; line $O/$n.json; }
for rep in 1 2; do
  for P in 11699132 12582912 10485760; do
    b hier_P${P}_split_r$rep --config hier --params $P --check-samples 0
    FA_GROUPED_SPLIT=0 b hier_P${P}_fused_r$rep --config hier --params $P --check-samples 0
  done
done
b hier_split_parity --config hier
