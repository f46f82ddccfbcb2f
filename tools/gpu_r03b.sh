# r03b: full GPU suite after the ownership / sampling / match_rows changes
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r03b; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -60 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
