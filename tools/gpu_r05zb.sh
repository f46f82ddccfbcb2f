# r05zb: staged tables across streams (tests/test_gpu_slots.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05zb; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_slots.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
