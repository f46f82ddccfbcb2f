# arrival path: pipelined pack/H2D + one D2H per dtype group -- ingest GPU tests, phase probe, arrival bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r02ad
timeout -k 10 600 python -u -m pytest tests/test_gpu_ingest.py tests/test_gpu_drivers.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02ad/tests.log 2>&1 || { tail -40 gpurun_out/r02ad/tests.log; exit 1; }
tail -1 gpurun_out/r02ad/tests.log
timeout -k 10 300 python tools/arrival_probe.py > gpurun_out/r02ad/arrival_probe.json 2>gpurun_out/r02ad/probe.err || { tail -5 gpurun_out/r02ad/probe.err; exit 1; }
cat gpurun_out/r02ad/arrival_probe.json
timeout -k 10 400 python bench.py --config arrival --steps 20 --warmup 3 > gpurun_out/r02ad/arrival.json 2>gpurun_out/r02ad/arrival.err || { tail -5 gpurun_out/r02ad/arrival.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r02ad/arrival.json'));print(d['value'], d['latency_ms'], d['parity'], d['cpu_baseline']['value'] if d.get('cpu_baseline') else None)"
