# r05y: the 16x16 Gram forms with y = x - c formed once per chunk in place (shared centre row, two more barriers)
# vs the 32x32 forms (FA_GRAM16=0, unchanged: the box calibration; r05_final2 on the previous binary: K = 64
# 0.822, K = 128 2.086 ms): robust tests, then K = 64 / 128, 3 interleaved reps at the sustained clock.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05y; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_robust.py -x -q --timeout 120 --timeout-method thread -k "pairwise or krum" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1],d['value'],d['ms_per_step'],r.get('kernel_avg_ms'),d.get('pair_form'),d.get('parity'))" $1; }
for rep in 1 2 3; do
  for v in K64_1 K64_0 K128_1 K128_0; do
    K=${v%_*}; K=${K#K}; S=${v#*_}
    FA_GRAM16=$S timeout -k 10 300 python bench.py --config krum --clients $K --steps 50 --warmup 100 --no-cpu-baseline --soak-seconds 0 --check-samples $([ $rep = 1 ] && echo 1 || echo 0) > $O/${v}_$rep.json 2> $O/${v}_$rep.err || { tail -5 $O/${v}_$rep.err; exit 1; }
    line $O/${v}_$rep.json
  done
done
