# r03ad: float keys as the only form -- median GPU tests, then the lanes-per-column choice re-measured
# with float keys (FA_MEDIAN_LANES=1 k_median_off vs 2 k_median_2l), interleaved, 2 reps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_robust.py -m gpu -k median -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_med.log 2>&1 || { tail -30 gpurun_out/pytest_med.log; exit 1; }
echo "median tests: $(tail -1 gpurun_out/pytest_med.log)"
for rep in 1 2; do
  for K in 72 80 96 128; do
    for L in 2 1; do
      FA_MEDIAN_LANES=$L timeout -k 10 120 python bench.py --config median --clients $K --no-cpu-baseline --check-samples 20000 --steps 20 --warmup 3 > gpurun_out/m.json 2>gpurun_out/m.err || { echo FAIL $K $L; tail -5 gpurun_out/m.err; exit 1; }
      L=$L K=$K python -c 'import json,os;d=json.load(open("gpurun_out/m.json"));print("rep lanes", os.environ["L"], "K="+os.environ["K"], d["roofline"]["kernel_avg_ms"], d["value"], d.get("parity"))'
    done
  done
done
