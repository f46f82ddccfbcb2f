# r03t: median 2l XCD-contiguous map A/B (FA_MEDIAN_XCD 0/1, interleaved x3) at K = 128 / 100, parity on.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_robust.py -m gpu -k median -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_med.log 2>&1 || { tail -30 gpurun_out/pytest_med.log; exit 1; }
FA_MEDIAN_XCD=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_robust.py -m gpu -k median -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_med_x.log 2>&1 || { tail -30 gpurun_out/pytest_med_x.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/pytest_med.log) / xcd $(tail -1 gpurun_out/pytest_med_x.log)"
for rep in 1 2 3; do
  for K in 128 100; do
    for x in 0 1; do
      FA_MEDIAN_XCD=$x timeout -k 10 120 python bench.py --config median --clients $K --no-cpu-baseline --check-samples 20000 --steps 20 --warmup 3 > gpurun_out/m.json 2>gpurun_out/m.err || { echo FAIL $K $x; tail -5 gpurun_out/m.err; exit 1; }
      X=$x K=$K python -c 'import json,os;d=json.load(open("gpurun_out/m.json"));print("xcd", os.environ["X"], "K="+os.environ["K"], d["roofline"]["kernel_avg_ms"], d["value"], d.get("parity"))'
    done
  done
done
