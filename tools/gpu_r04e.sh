# r04e: median column tiles per workgroup (FA_MEDIAN_REPS) -- parity with reps 8, interleaved timing of
# reps 1 / 4 / 8 on tiled and client-major rows, K = 128 and 32; pairwise tests (the 4x4 kernels again).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r04e; mkdir -p $O
FA_MEDIAN_REPS=8 timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_robust.py -k "median" > $O/pytest_reps8.txt 2>&1 \
  || { echo "pytest FAIL"; tail -30 $O/pytest_reps8.txt; exit 1; }
tail -1 $O/pytest_reps8.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_robust.py -k "pairwise or krum" > $O/pytest_pair.txt 2>&1 \
  || { echo "pytest pair FAIL"; tail -30 $O/pytest_pair.txt; exit 1; }
tail -1 $O/pytest_pair.txt
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1],d['value'],d['unit'],d['ms_per_step'],r.get('kernel_avg_ms'),r.get('frac'),'|',d.get('parity'))" $1; }
for rep in 1 2; do
  for K in 128 32; do
    for lay in tiled arena; do
      for r in 1 4 8; do
        n=median_${lay}_K${K}_reps${r}_r$rep
        FA_MEDIAN_REPS=$r timeout -k 10 300 python bench.py --config median --clients $K --layout $lay --steps 20 --warmup 3 --no-cpu-baseline > $O/$n.json 2> $O/$n.err \
          || { echo "FAIL $n"; tail -8 $O/$n.err; exit 1; }
        line $O/$n.json
      done
    done
  done
done
