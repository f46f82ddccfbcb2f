# median: branch-free 32-bit-offset kernel (default) vs the generic form (FA_MEDIAN_FULL=0), + robust tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r02k
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_robust.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r02k/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r02k/pytest.log; [ $rc -eq 0 ] || exit $rc
for K in 32 64 100 128 96 8 13; do for F in 1 0; do
  FA_MEDIAN_FULL=$F $T 200 python bench.py --config median --clients $K --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r02k/med_K${K}_F$F.json 2> gpurun_out/r02k/err || { tail gpurun_out/r02k/err; exit 1; }
  echo "K=$K off=$F $(python -c "import json;d=json.load(open('gpurun_out/r02k/med_K${K}_F$F.json'));print(d['roofline']['kernel_avg_ms'],d['roofline']['frac'],d['parity'])")"
done; done
