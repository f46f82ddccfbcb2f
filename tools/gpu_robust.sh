# Robust-aggregation GPU tests + median/krum benches.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_robust.py tests/test_defender.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_robust.log 2>&1 || { tail -40 gpurun_out/pytest_robust.log; exit 1; }
tail -2 gpurun_out/pytest_robust.log
run() { timeout -k 10 300 python bench.py "$@" --no-cpu-baseline > gpurun_out/ab.json 2>>gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
        python -c "import json,sys;d=json.load(open('gpurun_out/ab.json'));print(sys.argv[1:], d['value'], d['ms_per_step'], d['roofline'].get('kernel_avg_ms'), d['roofline'].get('achieved'), d['parity'])" "$@"; }
for K in 8 16 32 64 100 128; do run --config median --clients $K; done
run --config krum; run --config krum --clients 128
