# r03x: round-end style check after this session's changes: GPU suite, smoke, default bench, the N-rank
# path rehearsed on one GPU over gloo (N = 2 metric, N = 4 hier, N = 2 gossip), distributed GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 1; }
python -c 'import json;d=json.load(open("gpurun_out/bench_default.json"));print("metric", d["value"], d["roofline"]["frac"], d["parity"])'
FEDML_AMD_BENCH_REHEARSAL=1 timeout -k 10 400 python bench.py --gpus 2 --params 12500000 --no-cpu-baseline > gpurun_out/reh2.json 2> gpurun_out/reh2.err || { tail -20 gpurun_out/reh2.err; exit 1; }
python -c 'import json;d=json.load(open("gpurun_out/reh2.json"));print("reh N=2", d["n_gpus"], d["value"], d.get("parity"))'
FEDML_AMD_BENCH_REHEARSAL=1 timeout -k 10 400 python bench.py --gpus 4 --config hier --no-cpu-baseline > gpurun_out/reh4h.json 2> gpurun_out/reh4h.err || { tail -20 gpurun_out/reh4h.err; exit 1; }
python -c 'import json;d=json.load(open("gpurun_out/reh4h.json"));print("reh N=4 hier", d["n_gpus"], d["value"], d.get("parity"))'
FEDML_AMD_BENCH_REHEARSAL=1 timeout -k 10 400 python bench.py --gpus 2 --config gossip --no-cpu-baseline > gpurun_out/reh2g.json 2> gpurun_out/reh2g.err || { tail -20 gpurun_out/reh2g.err; exit 1; }
python -c 'import json;d=json.load(open("gpurun_out/reh2g.json"));print("reh N=2 gossip", d["n_gpus"], d["value"], d.get("parity"))'
