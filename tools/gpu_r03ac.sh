# r03ac: float-key median networks (IEEE minimum / maximum, FA_MEDIAN_FKEY) -- parity of every median
# test in both key forms, then an interleaved 3-rep A/B at K = 32 / 64 / 100 / 128 (fp32).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for F in 1 0; do
  FA_MEDIAN_FKEY=$F timeout -k 10 300 python -u -m pytest tests/test_gpu_robust.py -m gpu -k median -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_med_fk$F.log 2>&1 || { tail -30 gpurun_out/pytest_med_fk$F.log; exit 1; }
  echo "fkey $F: $(tail -1 gpurun_out/pytest_med_fk$F.log)"
done
for rep in 1 2 3; do
  for K in 32 64 100 128; do
    for F in 0 1; do
      FA_MEDIAN_FKEY=$F timeout -k 10 120 python bench.py --config median --clients $K --no-cpu-baseline --check-samples 20000 --steps 20 --warmup 3 > gpurun_out/m.json 2>gpurun_out/m.err || { echo FAIL $K $F; tail -5 gpurun_out/m.err; exit 1; }
      F=$F K=$K python -c 'import json,os;d=json.load(open("gpurun_out/m.json"));print("rep fkey", os.environ["F"], "K="+os.environ["K"], d["roofline"]["kernel_avg_ms"], d["value"], d.get("parity"))'
    done
  done
done
