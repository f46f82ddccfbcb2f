# r04m: k_pairdist_circ (K <= 32, circulant pairs, wave-private staging) -- pair / Krum GPU tests on
# the default (circ) and FA_PAIR_CIRC=0, then Krum K = 32 / 16 / 24 circ vs lane kernel (2 interleaved
# reps), rocprof kernel stats of K = 32 circ.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r04m; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_robust.py -k "pair or krum" > $O/pytest_circ.txt 2>&1 \
  || { echo "pytest circ FAIL"; tail -40 $O/pytest_circ.txt; exit 1; }
tail -1 $O/pytest_circ.txt
FA_PAIR_CIRC=0 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_robust.py -k "pair or krum" > $O/pytest_lane.txt 2>&1 \
  || { echo "pytest lane FAIL"; tail -40 $O/pytest_lane.txt; exit 1; }
tail -1 $O/pytest_lane.txt
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1],d['value'],d['unit'],d['ms_per_step'],r.get('kernel_avg_ms'),r.get('frac'),'|',d.get('parity','')[:60])" $1; }
b() { timeout -k 10 300 python bench.py --config krum --clients ${K:-32} --steps 20 --warmup 3 --no-cpu-baseline --soak-seconds 0 > $O/$1.json 2> $O/$1.err || { echo "FAIL $1"; tail -8 $O/$1.err; exit 1; }; line $O/$1.json; }
for rep in 1 2; do
  for K in 32 16 24; do
    K=$K b K${K}_circ_r$rep
    K=$K FA_PAIR_CIRC=0 b K${K}_lane_r$rep
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/rp32 -o run -- python3 bench.py --config krum --clients 32 --steps 10 --warmup 2 --no-cpu-baseline --soak-seconds 0 > $O/rp_K32.json 2> $O/rp_K32.err \
  || { echo "rocprof FAIL"; tail -5 $O/rp_K32.err; exit 1; }
find /tmp/rp32 -name "*kernel_stats.csv" -exec cp {} $O/krum_K32_circ_kernel_stats.csv \;
head -4 $O/krum_K32_circ_kernel_stats.csv
