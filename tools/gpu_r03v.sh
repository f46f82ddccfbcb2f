# r03v: cfg2 separate tensors: kernel time (rocprof) vs agg() call time; the jump kernel with scalar-load positions.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rt -o rt -- python bench.py --config resnet18 --layout tensors --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/rt.json 2> gpurun_out/rt.err || { tail -5 gpurun_out/rt.err; exit 1; }
python -c 'import json;d=json.load(open("gpurun_out/rt.json"));print("resnet18 tensors (under rocprof)", d["value"], d["ms_per_step"], d["roofline"].get("kernel_avg_ms"))'
timeout -k 10 300 python tools/host_probe_tensors.py > gpurun_out/hpt.json 2> gpurun_out/hpt.err || { tail -5 gpurun_out/hpt.err; exit 1; }
cat gpurun_out/hpt.json | head -40
timeout -k 10 300 python -u -m pytest tests/test_gpu_finite.py -m gpu -x -q -k "mt_ or secagg" --timeout 200 --timeout-method thread > gpurun_out/pytest_v.log 2>&1 || { tail -30 gpurun_out/pytest_v.log; exit 1; }
tail -1 gpurun_out/pytest_v.log
timeout -k 10 300 python bench.py --config samask --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/sa.json 2> gpurun_out/sa.err || { tail -5 gpurun_out/sa.err; exit 1; }
python -c 'import json;d=json.load(open("gpurun_out/sa.json"));print("samask", d["value"], d["unit"], d.get("parity"))'
