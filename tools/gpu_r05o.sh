# r05o: where the K = 32 Gram kernel's time goes -- measurement-only knobs of k_pair_gram_glds<3>
# (FA_GRAM_DBG, results wrong by construction): 1 no centre, 2 no float64 flush, 4 no MFMA, 8 the
# read alone, and combinations; kernel time from one rocprofv3 kernel trace per knob.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05o; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_robust.py -x -q --timeout 120 --timeout-method thread -k "pairwise or krum" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for K in 32 128; do
  timeout -k 10 300 python bench.py --config krum --no-cpu-baseline --soak-seconds 0 --steps 20 --warmup 3 --clients $K --check-samples 1 > $O/K$K.json 2> $O/K$K.err || { tail -5 $O/K$K.err; exit 1; }
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1],d['value'],d['ms_per_step'],r.get('kernel_avg_ms'),d.get('pair_form'),d.get('parity'))" $O/K$K.json
done
B="--config krum --no-cpu-baseline --soak-seconds 0 --steps 10 --warmup 2 --check-samples 0 --clients 32"
for d in 0 1 2 4 3 7 8 0; do
  FA_GRAM_DBG=$d timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/d$d -o tr --output-format csv -- python3 bench.py $B > $O/d$d.log 2>&1 || { tail -5 $O/d$d.log; exit 1; }
  python3 -c "
import csv,glob,sys
f=glob.glob('$O/d$d/**/*kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'gram_glds' in r['Name'] or 'gram_reduce' in r['Name'] or 'gram_dist' in r['Name']: print('dbg $d', r['Name'][26:50], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us avg', round(float(r['MinNs'])/1e3,1), 'min')
"
done
