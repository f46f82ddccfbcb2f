# GPU check: parity tests, smoke, bench.  Stops at the first GPU fault / abort / timeout.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
fault() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 120 python tools/debug_f16.py 2>&1 | tail -40; rc=$?; fault $rc && exit $rc
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_gpu.log; fault $rc && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -5; rc=$?; fault $rc && exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err; exit $rc
