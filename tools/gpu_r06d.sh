# r06d: the bf16x3 split form (FA_GRAM3=1) after r06b: per-chunk float32 runs for K > 96 and the
# bias term in the guard's model.  (1) the error sweep at K = 40 / 64 / 100 / 128; (2) the band,
# forms and Krum GPU tests with it; (3) interleaved A/B of the Krum K = 128 and K = 64 lines, 3 pairs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06d; mkdir -p $O
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
export FA_GRAM3=1
timeout -k 10 600 env KS=40,64,100,128 python tools/krum_kappa_sweep.py > $O/sweep_gram3.jsonl 2> $O/sweep_gram3.err || { tail -5 $O/sweep_gram3.err; exit 1; }
echo sweep_gram3 $(wc -l < $O/sweep_gram3.jsonl)
timeout -k 10 900 $T tests/test_gpu_krum_band.py tests/test_gpu_robust.py -k "band or pairwise or krum or sticky" > $O/tests_gram3.log 2>&1; rc=$?
tail -3 $O/tests_gram3.log; [ $rc = 0 ] || exit $rc
unset FA_GRAM3
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1].split('/')[-1],d['value'],d['ms_per_step'],r.get('kernel_avg_ms'),r.get('frac'),d.get('pair_form'),d.get('kappa_max'),d.get('parity'),'cold',(d.get('cold') or {}).get('ms'))" $1; }
for i in 1 2 3; do
  for k in 128 64; do
    for g in 0 1; do
      FA_GRAM3=$g timeout -k 10 300 python bench.py --config krum --clients $k --no-cpu-baseline --soak-seconds 0 --cold-reps 0 > $O/krum${k}_g${g}_$i.json 2> $O/krum${k}_g${g}_$i.err || { tail -5 $O/krum${k}_g${g}_$i.err; exit 1; }
      line $O/krum${k}_g${g}_$i.json
    done
  done
done
exit 0
