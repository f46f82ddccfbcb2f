# Run-to-run variation of the default bench on one box (order effects, step count, CPU baseline).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
run() { timeout -k 10 300 python bench.py "$@" --check-samples 0 > gpurun_out/var.json 2>>gpurun_out/var.err || exit 1
        python -c "import json,sys;d=json.load(open('gpurun_out/var.json'));print(sys.argv[1:], d['value'], d['roofline']['kernel_avg_ms'])" "$@"; }
run --no-cpu-baseline
run --no-cpu-baseline --steps 5 --warmup 2
run --no-cpu-baseline --steps 30
run --no-cpu-baseline
run --no-cpu-baseline --layout tensors
run --no-cpu-baseline
