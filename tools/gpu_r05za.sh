# r05za: the ring kernel's segment-order cases (tests/test_gpu_robust.py::test_pairwise_ring_segment_orders)
# plus the robust pairwise / Krum tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05za; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_robust.py -x -q --timeout 120 --timeout-method thread -k "pairwise or krum" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
