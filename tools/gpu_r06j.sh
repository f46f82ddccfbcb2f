# r06j: the bf16x3 Gram form extended to K in (64, 96] (k_pair_gram3<3>: 7 waves, one per tile set,
# no coordinate split) -- the band and Krum tests, then Krum K = 80 / 96 with it and with the f32
# form (FA_GRAM3=0), 2 interleaved pairs each; the memo now copying kappa_max every GRAM_RETRY-th call
# only: Krum K = 32 with it vs no memo (FEDML_AMD_KRUM_STICKY=0), 2 interleaved pairs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06j; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_krum_band.py tests/test_gpu_robust.py > $O/tests_krum.log 2>&1; rc=$?
tail -2 $O/tests_krum.log; [ $rc = 0 ] || exit $rc
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1].split('/')[-1],d['value'],d['ms_per_step'],r.get('kernel_avg_ms'),d.get('pair_form'),str(d.get('parity'))[:70])" $1; }
for K in 96 80; do
  for i in 1 2; do
    for g in 1 0; do
      FA_GRAM3=$g timeout -k 10 400 python bench.py --config krum --clients $K --no-cpu-baseline --soak-seconds 0 --cold-reps 0 > $O/krum${K}_g${g}_$i.json 2> $O/krum${K}_g${g}_$i.err || { tail -5 $O/krum${K}_g${g}_$i.err; exit 1; }
      line $O/krum${K}_g${g}_$i.json
    done
  done
done
for i in 1 2; do
  for st in 0 1; do
    FEDML_AMD_KRUM_STICKY=$st timeout -k 10 300 python bench.py --config krum --clients 32 --no-cpu-baseline --soak-seconds 0 --cold-reps 0 --check-samples 0 > $O/krum32_s${st}_$i.json 2> $O/krum32_s${st}_$i.err || { tail -5 $O/krum32_s${st}_$i.err; exit 1; }
    line $O/krum32_s${st}_$i.json
  done
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r06j_k96 -o run -- python3 bench.py --config krum --clients 96 --no-cpu-baseline --soak-seconds 3 --cold-reps 0 --check-samples 0 > $O/prof_krum96.json 2> $O/prof_krum96.err || { tail -5 $O/prof_krum96.err; exit 1; }
cp $(find /tmp/r06j_k96 -name '*kernel_stats.csv' | head -1) $O/prof_krum96_kernel_stats.csv
head -6 $O/prof_krum96_kernel_stats.csv | cut -c1-150
exit 0
