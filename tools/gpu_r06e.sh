# r06e: the pipelined bf16x3 form for K > 96 (FA_GRAM3=2, k_pair_gram3p) against the two-phase form
# (FA_GRAM3=1, the default): the band / forms / Krum tests and the error sweep with it, then 3
# interleaved pairs of the Krum K = 128 and K = 100 lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06e; mkdir -p $O
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
export FA_GRAM3=2
timeout -k 10 600 env KS=100,128 python tools/krum_kappa_sweep.py > $O/sweep_gram3p.jsonl 2> $O/sweep_gram3p.err || { tail -5 $O/sweep_gram3p.err; exit 1; }
echo sweep_gram3p $(wc -l < $O/sweep_gram3p.jsonl)
timeout -k 10 900 $T tests/test_gpu_krum_band.py tests/test_gpu_robust.py -k "band or pairwise or krum or sticky" > $O/tests_gram3p.log 2>&1; rc=$?
tail -2 $O/tests_gram3p.log; [ $rc = 0 ] || exit $rc
unset FA_GRAM3
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1].split('/')[-1],d['value'],d['ms_per_step'],r.get('kernel_avg_ms'),r.get('frac'),d.get('pair_form'),str(d.get('parity'))[:40])" $1; }
for i in 1 2 3; do
  for k in 128 100; do
    for g in 1 2; do
      FA_GRAM3=$g timeout -k 10 300 python bench.py --config krum --clients $k --no-cpu-baseline --soak-seconds 0 --cold-reps 0 > $O/krum${k}_g${g}_$i.json 2> $O/krum${k}_g${g}_$i.err || { tail -5 $O/krum${k}_g${g}_$i.err; exit 1; }
      line $O/krum${k}_g${g}_$i.json
    done
  done
done
exit 0
