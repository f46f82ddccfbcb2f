set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
echo "== rocminfo-lite"; (rocm-smi --showproductname 2>&1 | head -20) || true
nproc; echo OMP=$OMP_NUM_THREADS
timeout -k 10 240 python -c "import torch; print(torch.__version__, torch.cuda.is_available(), torch.cuda.get_device_name(0))"
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu_r1a.log 2>&1; rc=$?; tail -30 gpurun_out/pytest_gpu_r1a.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -5
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_r1a.json 2> gpurun_out/bench_r1a.err; rc=$?; cat gpurun_out/bench_r1a.json; tail -5 gpurun_out/bench_r1a.err; exit $rc
