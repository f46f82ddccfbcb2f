# r05u(b): the 16x16 Gram form for K in (32, 64] (16 waves: 4 tile sets x 4 splits, one workgroup per CU) vs the
# 12-wave 32x32 form (FA_GRAM16=0): robust pairwise / Krum tests, then K = 40 / 64 A/B at the
# sustained clock (100 warmup steps), 3 interleaved reps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05ub; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_robust.py -x -q --timeout 120 --timeout-method thread -k "pairwise or krum" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1],d['value'],d['ms_per_step'],r.get('kernel_avg_ms'),d.get('pair_form'),d.get('parity'))" $1; }
for rep in 1 2 3; do
  for v in K64_1 K64_0 K40_1 K40_0 K128_1; do
    K=${v%_*}; K=${K#K}; S=${v#*_}
    FA_GRAM16=$S timeout -k 10 300 python bench.py --config krum --clients $K --steps 50 --warmup 100 --no-cpu-baseline --soak-seconds 0 --check-samples $([ $rep = 1 ] && echo 1 || echo 0) > $O/${v}_$rep.json 2> $O/${v}_$rep.err || { tail -5 $O/${v}_$rep.err; exit 1; }
    line $O/${v}_$rep.json
  done
done
