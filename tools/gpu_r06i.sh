# r06i: the final binary -- the whole -m gpu suite and smoke(); the default line twice; the Krum
# kappa memo's copy on a side stream vs no memo at all (FEDML_AMD_KRUM_STICKY=0), K = 32, 3
# interleaved pairs; the sustained-clock trace of Krum K = 32 with it.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06i; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};c=d.get('cold') or {};print(sys.argv[1].split('/')[-1],d['value'],d['ms_per_step'],r.get('kernel_avg_ms'),r.get('frac'),r.get('frac_of_ceiling'),'cold',c.get('ms'),str(d.get('parity'))[:50])" $1; }
for i in 1 2; do
  timeout -k 10 400 python bench.py --no-cpu-baseline > $O/metric_$i.json 2> $O/metric_$i.err || { tail -5 $O/metric_$i.err; exit 1; }
  line $O/metric_$i.json
done
for i in 1 2 3; do
  for st in 0 1; do
    FEDML_AMD_KRUM_STICKY=$st timeout -k 10 300 python bench.py --config krum --clients 32 --no-cpu-baseline --soak-seconds 0 --cold-reps 0 --check-samples 0 > $O/krum32_s${st}_$i.json 2> $O/krum32_s${st}_$i.err || { tail -5 $O/krum32_s${st}_$i.err; exit 1; }
    line $O/krum32_s${st}_$i.json
  done
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r06i_k32 -o run -- python3 bench.py --config krum --clients 32 --no-cpu-baseline --soak-seconds 3 --cold-reps 0 --check-samples 0 > $O/prof_krum32.json 2> $O/prof_krum32.err || { tail -5 $O/prof_krum32.err; exit 1; }
cp $(find /tmp/r06i_k32 -name '*kernel_stats.csv' | head -1) $O/prof_krum32_kernel_stats.csv
head -8 $O/prof_krum32_kernel_stats.csv | cut -c1-150
exit 0
