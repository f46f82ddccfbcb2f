# r03h: finite-field (incl. SecAgg mask) + robust GPU tests, then the Krum A/B of r03g
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r03h; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_finite.py -x -q --timeout 120 --timeout-method thread > $O/finite.log 2>&1 || { tail -40 $O/finite.log; exit 1; }
tail -1 $O/finite.log
bash tools/gpu_r03g.sh
