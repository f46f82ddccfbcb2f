# r03d: Krum pair kernels with strict-upper tiles + within-block phase: parity + timings
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r03d; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_robust.py -x -q --timeout 120 --timeout-method thread > $O/robust_tests.log 2>&1 || { tail -40 $O/robust_tests.log; exit 1; }
tail -1 $O/robust_tests.log
for K in 4 16 32 64 100 128; do
  timeout -k 10 120 python bench.py --config krum --clients $K --no-cpu-baseline --steps 10 --warmup 2 > $O/bench_K$K.json 2> $O/bench_K$K.err || { tail -5 $O/bench_K$K.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_K$K.json'));print($K, d['roofline']['kernel_avg_ms'], d['parity'])"
done
