# r05v: after removing the ring kernel's measurement knobs and its 16-wave variant: robust pairwise /
# Krum tests, then K = 32 / 128 lines at the sustained clock.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05v; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_robust.py -x -q --timeout 120 --timeout-method thread -k "pairwise or krum" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1],d['value'],d['ms_per_step'],r.get('kernel_avg_ms'),d.get('pair_form'),d.get('parity'))" $1; }
for K in 32 128; do
  timeout -k 10 300 python bench.py --config krum --clients $K --steps 50 --warmup 150 --no-cpu-baseline --soak-seconds 0 --check-samples 1 > $O/K$K.json 2> $O/K$K.err || { tail -5 $O/K$K.err; exit 1; }
  line $O/K$K.json
done
