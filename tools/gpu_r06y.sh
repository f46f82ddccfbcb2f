# r06y: K in (64, 96] on two workgroups per CU (Gram3Cfg<3, 1>: client pointers in LDS, two planes
# live at a time in the MFMA phase: 124 VGPRs, 81.7 KB LDS; FA_GRAM3_L3=1): band / robust tests with
# it, then K = 96 / 80 A/B against the one-workgroup layout, 3 interleaved pairs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06y; mkdir -p $O
export TMPDIR=/tmp
FA_GRAM3_L3=1 timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_krum_band.py tests/test_gpu_robust.py -k "band or pairwise or krum or gram" > $O/tests_l3.log 2>&1; rc=$?
tail -2 $O/tests_l3.log; [ $rc = 0 ] || exit $rc
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1].split('/')[-1],d['value'],d['ms_per_step'],r.get('kernel_avg_ms'),d.get('pair_form'),str(d.get('parity'))[:60])" $1; }
for K in 96 80; do
  for i in 1 2 3; do
    for l in 1 0; do
      FA_GRAM3_L3=$l timeout -k 10 300 python bench.py --config krum --clients $K --no-cpu-baseline --soak-seconds 0 --cold-reps 0 $([ $i = 1 ] || echo --check-samples 0) > $O/krum${K}_l${l}_$i.json 2> $O/krum${K}_l${l}_$i.err || { tail -5 $O/krum${K}_l${l}_$i.err; exit 1; }
      line $O/krum${K}_l${l}_$i.json
    done
  done
done
exit 0
