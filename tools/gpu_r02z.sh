# after k_median_2l (K in (64,128]) + half-precision Krum: full GPU suite, smoke, rocprof of median K=128 / K=100
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r02z
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02z/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r02z/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r02z/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r02z/smoke.log 2>&1 || { tail -20 gpurun_out/r02z/smoke.log; exit 1; }
tail -1 gpurun_out/r02z/smoke.log
for K in 128 100; do
 BENCH_ARGS="--config median --clients $K --steps 10 --warmup 2 --no-cpu-baseline" timeout -k 10 900 bash tools/profile.sh r02z_median_K$K || exit 1
done
ls gpurun_out/summary
