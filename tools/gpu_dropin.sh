# GPU tests (drop-in path) + state_dict-path benches (cfg2/cfg3 tensors, fragmented metric).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
run() { timeout -k 10 300 python bench.py "$@" --no-cpu-baseline > gpurun_out/ab.json 2>>gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
        python -c "import json,sys;d=json.load(open('gpurun_out/ab.json'));print(sys.argv[1:], d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['parity'])" "$@"; }
run --config resnet18 --layout tensors
run --config resnet18 --layout tiled
run --config vit_bf16 --layout tensors
run --config fragmented
