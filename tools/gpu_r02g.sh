# full -m gpu suite, smoke, fedopt rocprof (trace + FETCH/WRITE PMC)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r02g.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu_r02g.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/pytest_gpu_r02g.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r02g.log 2>&1 || { cat gpurun_out/smoke_r02g.log; exit 1; }
tail -2 gpurun_out/smoke_r02g.log
BENCH_ARGS="--config fedopt --steps 5 --warmup 2 --no-cpu-baseline --check-samples 0" KERNEL=k_fedavg timeout -k 10 900 bash tools/profile.sh r02g_fedopt > gpurun_out/prof_fedopt.log 2>&1; rc=$?
tail -12 gpurun_out/prof_fedopt.log; exit $rc
