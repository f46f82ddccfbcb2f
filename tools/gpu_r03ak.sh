# r03ak: median GPU tests with the packed (two-per-lane, uint16-key) special-value cases added.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_robust.py -m gpu -k median -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_med.log 2>&1 || { tail -30 gpurun_out/pytest_med.log; exit 1; }
echo "median tests: $(tail -1 gpurun_out/pytest_med.log)"
