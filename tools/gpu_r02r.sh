# host planning in C++ (plan_outputs): full GPU suite, b2b host probe, cfg2 tensors bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r02r
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02r/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r02r/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r02r/gpu_tests.log
timeout -k 10 200 python tools/host_probe_b2b.py > gpurun_out/r02r/b2b.json 2>/dev/null || { echo probe failed; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r02r/b2b.json'));print(d['b2b_keep'], d['b2b_drop'])"
timeout -k 10 200 python bench.py --config resnet18 --layout tensors --no-cpu-baseline --steps 30 --warmup 5 > gpurun_out/r02r/tensors.json 2>gpurun_out/r02r/tensors.err || { tail -3 gpurun_out/r02r/tensors.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r02r/tensors.json'));print(d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'], d['parity'])"
