# Tiled-arena parity tests, then interleaved A/B of the metric (client-major vs tiled arena) + hier/cfg2/cfg3.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_tiled.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_tiled.log 2>&1 || { tail -40 gpurun_out/pytest_tiled.log; exit 1; }
tail -2 gpurun_out/pytest_tiled.log
run() { timeout -k 10 300 python bench.py "$@" --no-cpu-baseline > gpurun_out/ab.json 2>>gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
        python -c "import json,sys;d=json.load(open('gpurun_out/ab.json'));print(sys.argv[1:], d['value'], d['roofline']['kernel_avg_ms'], d['parity'])" "$@"; }
for r in 1 2 3; do run --layout arena; run --layout tiled; done
run --config hier --layout arena; run --config hier --layout tiled
run --config resnet18 --layout arena; run --config resnet18 --layout tiled
run --config vit_bf16 --layout arena; run --config vit_bf16 --layout tiled
