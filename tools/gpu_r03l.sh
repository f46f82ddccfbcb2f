# r03l: k_median_4l parity (FA_MEDIAN_LANES=4 / 41) + interleaved A/B vs k_median_2l at K = 128 / 100,
# then the round-end style session (GPU suite, smoke, default bench).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o gpurun_out/doorbell_probe tools/doorbell_probe.hip 2>/dev/null || exit 1
timeout -k 10 60 gpurun_out/doorbell_probe 3000 > gpurun_out/doorbell.json || { echo doorbell probe failed; exit 1; }
cat gpurun_out/doorbell.json
for L in 4 41; do
  FA_MEDIAN_LANES=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_robust.py -m gpu -k median -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_med_$L.log 2>&1 || { tail -30 gpurun_out/pytest_med_$L.log; exit 1; }
  echo "lanes $L: $(tail -1 gpurun_out/pytest_med_$L.log)"
done
for rep in 1 2 3; do
  for K in 128 100; do
    for L in 2 4 41; do
      FA_MEDIAN_LANES=$L timeout -k 10 120 python bench.py --config median --clients $K --no-cpu-baseline --check-samples 20000 --steps 20 --warmup 3 > gpurun_out/m.json 2>gpurun_out/m.err || { echo FAIL $K $L; tail -5 gpurun_out/m.err; exit 1; }
      L=$L K=$K python -c 'import json,os;d=json.load(open("gpurun_out/m.json"));print("rep", os.environ["L"], "K="+os.environ["K"], d["roofline"]["kernel_avg_ms"], d["value"], d.get("parity"))'
    done
  done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
