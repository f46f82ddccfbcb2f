# r06ad: Krum K <= 32 on the bf16x3 form (Gram3Cfg<1>: the one diagonal-pair set in 4 coordinate
# splits, four 4-wave workgroups per CU; FA_GRAM3_K32=1) vs the f32 LDS-DMA ring kernel: band / robust
# tests with it, then K = 32 / 20 / 8, 3 interleaved pairs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06ad; mkdir -p $O
export TMPDIR=/tmp
FA_GRAM3_K32=1 timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_krum_band.py tests/test_gpu_robust.py -k "band or pairwise or krum or gram" > $O/tests_k32.log 2>&1; rc=$?
tail -2 $O/tests_k32.log; [ $rc = 0 ] || exit $rc
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1].split('/')[-1],d['value'],d['ms_per_step'],r.get('kernel_avg_ms'),d.get('pair_form'),str(d.get('parity'))[:60])" $1; }
for K in 32 20 8; do
  for i in 1 2 3; do
    for l in 1 0; do
      FA_GRAM3_K32=$l timeout -k 10 300 python bench.py --config krum --clients $K --no-cpu-baseline --soak-seconds 0 --cold-reps 0 $([ $i = 1 ] || echo --check-samples 0) > $O/krum${K}_g${l}_$i.json 2> $O/krum${K}_g${l}_$i.err || { tail -5 $O/krum${K}_g${l}_$i.err; exit 1; }
      line $O/krum${K}_g${l}_$i.json
    done
  done
done
exit 0
