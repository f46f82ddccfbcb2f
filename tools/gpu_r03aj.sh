# r03aj: final check of the committed tree (library rebuilt after the f16 revert): GPU suite, smoke,
# default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03aj
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03aj/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r03aj/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r03aj/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03aj/smoke.log 2>&1 || { cat gpurun_out/r03aj/smoke.log; exit 1; }
tail -1 gpurun_out/r03aj/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r03aj/bench_default.json 2> gpurun_out/r03aj/bench_default.err || { tail -20 gpurun_out/r03aj/bench_default.err; exit 1; }
python -c 'import json;d=json.load(open("gpurun_out/r03aj/bench_default.json"));print("metric", d["value"], d["roofline"]["frac"], d["cpu_baseline"]["value"], d["parity"])'
