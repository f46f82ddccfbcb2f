# r03ab: two-stream SecAgg expansion test + full GPU suite + smoke + samask bench line after the
# work-space guard (ctx->mt_ev) and the per-stream engine scratch.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_finite.py -m gpu -x -q --timeout 120 --timeout-method thread -k "two_streams or jump_ahead" > gpurun_out/pytest_mt.log 2>&1 || { tail -30 gpurun_out/pytest_mt.log; exit 1; }
tail -1 gpurun_out/pytest_mt.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py --config samask --no-cpu-baseline > gpurun_out/bench_samask.json 2> gpurun_out/bench_samask.err || { tail -20 gpurun_out/bench_samask.err; exit 1; }
python -c 'import json;d=json.load(open("gpurun_out/bench_samask.json"));print("samask", d["value"], d["ms_per_step"], d.get("parity"))'
