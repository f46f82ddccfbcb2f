# median: branch-free K == B kernel vs the generic form (FA_MEDIAN_FULL=0), K = 32 / 64 / 128, + robust tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r02j
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_robust.py tests/test_promotion.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r02j/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r02j/pytest.log; [ $rc -eq 0 ] || exit $rc
for K in 32 64 128 96; do for F in 1 0 1 0; do
  FA_MEDIAN_FULL=$F $T 200 python bench.py --config median --clients $K --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r02j/med_K${K}_F$F.json 2> gpurun_out/r02j/err || { tail gpurun_out/r02j/err; exit 1; }
  echo "K=$K full=$F $(python -c "import json;d=json.load(open('gpurun_out/r02j/med_K${K}_F$F.json'));print(d['roofline']['kernel_avg_ms'],d['roofline']['frac'],d['parity'])")"
done; done
for D in bf16; do for K in 32 64; do for F in 1 0; do
  FA_MEDIAN_FULL=$F $T 200 python bench.py --config median --dtype $D --clients $K --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r02j/med_${D}_K${K}_F$F.json 2> gpurun_out/r02j/err || { tail gpurun_out/r02j/err; exit 1; }
  echo "$D K=$K full=$F $(python -c "import json;d=json.load(open('gpurun_out/r02j/med_${D}_K${K}_F$F.json'));print(d['roofline']['kernel_avg_ms'],d['roofline']['frac'],d['parity'])")"
done; done; done
