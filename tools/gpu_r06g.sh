# r06g: whole client groups unguarded in wsum_tile / k_wsum_grouped (r06: the guarded consume let hipcc
# sink each group's second load behind the first client's arithmetic with a vmcnt(0)).  The -m gpu
# parity tests of the weighted-sum family on the new build, then interleaved A/B against the previous
# build (fedml_amd/ab/libfedagg_prev.so via FEDML_AMD_LIB): the metric line x3 pairs, cfg4 hier x3, FedOpt and
# LightSecAgg (the same fix in k_fedavg_sgd and k_finite_sum) x2.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06g; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu -k "not krum_band" > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc = 0 ] || exit $rc
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1].split('/')[-1],d['value'],d['ms_per_step'],r.get('kernel_avg_ms'),r.get('frac'),r.get('frac_of_ceiling'),str(d.get('parity'))[:40])" $1; }
for i in 1 2 3; do
  for v in prev new; do
    if [ $v = prev ]; then export FEDML_AMD_LIB=$PWD/fedml_amd/ab/libfedagg_prev.so; else unset FEDML_AMD_LIB; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline --soak-seconds 0 --cold-reps 0 > $O/metric_${v}_$i.json 2> $O/metric_${v}_$i.err || { tail -5 $O/metric_${v}_$i.err; exit 1; }
    line $O/metric_${v}_$i.json
    timeout -k 10 300 python bench.py --config hier --no-cpu-baseline --soak-seconds 0 --cold-reps 0 > $O/hier_${v}_$i.json 2> $O/hier_${v}_$i.err || { tail -5 $O/hier_${v}_$i.err; exit 1; }
    line $O/hier_${v}_$i.json
    if [ $i -le 2 ]; then
      for c in fedopt secagg; do
        timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --soak-seconds 0 --cold-reps 0 > $O/${c}_${v}_$i.json 2> $O/${c}_${v}_$i.err || { tail -5 $O/${c}_${v}_$i.err; exit 1; }
        line $O/${c}_${v}_$i.json
      done
    fi
  done
done
unset FEDML_AMD_LIB
exit 0
