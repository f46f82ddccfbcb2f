# r06b: (1) the Krum kappa band on the box: the new band tests + the robust/Krum GPU tests, default
# forms; the error sweep (tools/krum_kappa_sweep.py) of the forced Gram form; (2) the bf16x3 split
# form for K in (96, 128] (FA_GRAM3=1): the same tests and sweep at K = 100 / 128, and an interleaved
# A/B of the Krum K = 128 line (3 pairs); (3) the metric kernel's translation / clock counters.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06b; mkdir -p $O
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_krum_band.py tests/test_gpu_robust.py -k "band or pairwise or krum or sticky" > $O/tests_default.log 2>&1; rc=$?
tail -3 $O/tests_default.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python tools/krum_kappa_sweep.py > $O/sweep_default.jsonl 2> $O/sweep_default.err || { tail -5 $O/sweep_default.err; exit 1; }
echo sweep_default $(wc -l < $O/sweep_default.jsonl)
export FA_GRAM3=1
timeout -k 10 600 env KS=40,64,100,128 python tools/krum_kappa_sweep.py > $O/sweep_gram3.jsonl 2> $O/sweep_gram3.err || { tail -5 $O/sweep_gram3.err; exit 1; }
echo sweep_gram3 $(wc -l < $O/sweep_gram3.jsonl)
timeout -k 10 900 $T tests/test_gpu_krum_band.py tests/test_gpu_robust.py -k "band or pairwise or krum or sticky" > $O/tests_gram3.log 2>&1; rc=$?
tail -3 $O/tests_gram3.log; [ $rc = 0 ] || exit $rc
unset FA_GRAM3
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1].split('/')[-1],d['value'],d['ms_per_step'],r.get('kernel_avg_ms'),r.get('frac'),d.get('pair_form'),d.get('kappa_max'),d.get('parity'),'cold',(d.get('cold') or {}).get('ms'))" $1; }
for i in 1 2 3; do
  for g in 0 1; do
    FA_GRAM3=$g timeout -k 10 300 python bench.py --config krum --clients 128 --no-cpu-baseline --soak-seconds 0 > $O/krum128_g${g}_$i.json 2> $O/krum128_g${g}_$i.err || { tail -5 $O/krum128_g${g}_$i.err; exit 1; }
    line $O/krum128_g${g}_$i.json
  done
done
C1="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE"
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $C1 --kernel-include-regex 'k_wsum|k_read_probe' -d $O/pmc1 -o pmc --output-format csv -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --check-samples 0 --soak-seconds 0 --cold-reps 0 > $O/pmc1.log 2>&1 \
  || { echo "FAIL pmc1"; tail -5 $O/pmc1.log; exit 1; }
tail -1 $O/pmc1.log | cut -c1-200
exit 0
