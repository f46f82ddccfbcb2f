# r04n: k_pairdist_circ with KC = 32 at 3 waves / 168 VGPRs (no spill) -- tests, then circ vs lane at
# K = 8 / 12 / 16 / 24 / 28 / 32 (2 interleaved reps) to set the K ranges each kernel takes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r04n; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_robust.py -k "pair or krum" > $O/pytest_circ.txt 2>&1 \
  || { echo "pytest circ FAIL"; tail -40 $O/pytest_circ.txt; exit 1; }
tail -1 $O/pytest_circ.txt
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1],d['value'],d['unit'],d['ms_per_step'],r.get('kernel_avg_ms'),r.get('frac'),'|',d.get('parity','')[:40])" $1; }
b() { timeout -k 10 300 python bench.py --config krum --clients ${K:-32} --steps 20 --warmup 3 --no-cpu-baseline --soak-seconds 0 > $O/$1.json 2> $O/$1.err || { echo "FAIL $1"; tail -8 $O/$1.err; exit 1; }; line $O/$1.json; }
for rep in 1 2; do
  for K in 32 28 24 16 12 8; do
    K=$K b K${K}_circ_r$rep
    K=$K FA_PAIR_CIRC=0 b K${K}_lane_r$rep
  done
done
