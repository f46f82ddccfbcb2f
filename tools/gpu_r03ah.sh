# r03ah: float16 two-per-lane median on packed float keys (v_pk_minimum3_f16) -- median GPU tests, then
# the fp16 / bf16 median bench lines at K = 32 / 64 (bf16 keeps the uint16 keys: the reference row).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_robust.py -m gpu -k median -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_med.log 2>&1 || { tail -30 gpurun_out/pytest_med.log; exit 1; }
echo "median tests: $(tail -1 gpurun_out/pytest_med.log)"
for rep in 1 2; do
  for K in 32 64; do
    for D in fp16 bf16; do
      timeout -k 10 120 python bench.py --config median --clients $K --dtype $D --no-cpu-baseline --check-samples 20000 --steps 20 --warmup 3 > gpurun_out/m.json 2>gpurun_out/m.err || { echo FAIL $K $D; tail -5 gpurun_out/m.err; exit 1; }
      D=$D K=$K python -c 'import json,os;d=json.load(open("gpurun_out/m.json"));print("rep", os.environ["D"], "K="+os.environ["K"], d["roofline"]["kernel_avg_ms"], d["value"], d.get("parity"))'
    done
  done
done
