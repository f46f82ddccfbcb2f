# checkpoint: full GPU suite, smoke, default bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r02ar
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02ar/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r02ar/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r02ar/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r02ar/smoke.log 2>&1 || { tail -20 gpurun_out/r02ar/smoke.log; exit 1; }
tail -1 gpurun_out/r02ar/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r02ar/bench.json 2>gpurun_out/r02ar/bench.err || { tail -5 gpurun_out/r02ar/bench.err; exit 1; }
cat gpurun_out/r02ar/bench.json
