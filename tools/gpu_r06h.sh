# r06h: whole row groups unguarded in k_mix_band (cfg5 gossip), interleaved A/B against the build
# without it (fedml_amd/ab/libfedagg_prev.so via FEDML_AMD_LIB), 3 pairs; the mixing GPU tests first.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06h; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu -k "mix or gossip or pushsum or cfg5 or finite or secagg or lsa" > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc = 0 ] || exit $rc
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1].split('/')[-1],d['value'],d['ms_per_step'],r.get('kernel_avg_ms'),r.get('frac'),r.get('frac_of_ceiling'),str(d.get('parity'))[:40])" $1; }
for i in 1 2 3; do
  for v in prev new; do
    if [ $v = prev ]; then export FEDML_AMD_LIB=$PWD/fedml_amd/ab/libfedagg_prev.so; else unset FEDML_AMD_LIB; fi
    timeout -k 10 300 python bench.py --config gossip --no-cpu-baseline --soak-seconds 0 --cold-reps 0 > $O/gossip_${v}_$i.json 2> $O/gossip_${v}_$i.err || { tail -5 $O/gossip_${v}_$i.err; exit 1; }
    line $O/gossip_${v}_$i.json
  done
done
unset FEDML_AMD_LIB
exit 0
