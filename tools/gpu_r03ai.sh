# r03ai: after reverting the float16 packed float-key experiment (r03ah: parity failure) -- median GPU
# tests, then the fragmented variant sweep (tools/gpu_r03ag.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_robust.py -m gpu -k median -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_med.log 2>&1 || { tail -30 gpurun_out/pytest_med.log; exit 1; }
echo "median tests: $(tail -1 gpurun_out/pytest_med.log)"
bash tools/gpu_r03ag.sh
