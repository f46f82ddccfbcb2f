# r06s: Krum K in (32, 64] on the two-workgroup bf16x3 layout (Gram3Cfg<2, 1>: 8 waves, 2 splits, two
# workgroups per CU -- two chunks of loads in flight per CU instead of one; FA_GRAM3_L2=1): the band
# and robust tests with it, then K = 64 / 40 A/B, 3 interleaved pairs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06s; mkdir -p $O
export TMPDIR=/tmp
FA_GRAM3_L2=1 timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_krum_band.py tests/test_gpu_robust.py -k "band or pairwise or krum or gram" > $O/tests_l2.log 2>&1; rc=$?
tail -2 $O/tests_l2.log; [ $rc = 0 ] || exit $rc
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1].split('/')[-1],d['value'],d['ms_per_step'],r.get('kernel_avg_ms'),d.get('pair_form'),str(d.get('parity'))[:60])" $1; }
for K in 64 40; do
  for i in 1 2 3; do
    for l in 1 0; do
      FA_GRAM3_L2=$l timeout -k 10 300 python bench.py --config krum --clients $K --no-cpu-baseline --soak-seconds 0 --cold-reps 0 $([ $i = 1 ] || echo --check-samples 0) > $O/krum${K}_l${l}_$i.json 2> $O/krum${K}_l${l}_$i.err || { tail -5 $O/krum${K}_l${l}_$i.err; exit 1; }
      line $O/krum${K}_l${l}_$i.json
    done
  done
done
exit 0
