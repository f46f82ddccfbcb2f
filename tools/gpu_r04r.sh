# r04r: k_median_2lp (loads one column block ahead of the network) -- median GPU tests on the default
# (2lp) and FA_MEDIAN_2LP=0, then K = 128 / 100 / 72 tiled + K = 128 client-major, 2lp (reps 8 / 32)
# vs 2l, 2 interleaved reps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r04r; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_robust.py -k "median" > $O/pytest_2lp.txt 2>&1 \
  || { echo "pytest 2lp FAIL"; tail -40 $O/pytest_2lp.txt; exit 1; }
tail -1 $O/pytest_2lp.txt
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1],d['value'],d['unit'],d['ms_per_step'],r.get('kernel_avg_ms'),r.get('frac'),'|',d.get('parity','')[:30])" $1; }
b() { timeout -k 10 300 python bench.py --config median --clients ${K:-128} --layout ${L:-tiled} --steps 20 --warmup 3 --no-cpu-baseline --soak-seconds 0 > $O/$1.json 2> $O/$1.err || { echo "FAIL $1"; tail -8 $O/$1.err; exit 1; }; line $O/$1.json; }
for rep in 1 2; do
  for K in 128 100 72; do
    K=$K b K${K}_2lp8_r$rep
    K=$K FA_MEDIAN_2LP_REPS=32 b K${K}_2lp32_r$rep
    K=$K FA_MEDIAN_2LP=0 b K${K}_2l_r$rep
  done
  K=128 L=arena b K128_arena_2lp8_r$rep
  K=128 L=arena FA_MEDIAN_2LP=0 b K128_arena_2l_r$rep
done
