# r05q: K <= 32 Gram ring kernel (symmetric 16x16x4 tiles, float64 flush every 4th chunk): two 8-wave
# workgroups per CU (default) vs one of 16 waves vs the register-staged kernel (FA_GRAM_GLDS=0); tests, 3 reps,
# then the measurement knobs of the default.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05q; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_robust.py -x -q --timeout 120 --timeout-method thread -k "pairwise or krum" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1],d['value'],d['ms_per_step'],r.get('kernel_avg_ms'),d.get('pair_form'),d.get('parity'))" $1; }
B="--config krum --no-cpu-baseline --soak-seconds 0 --steps 20 --warmup 3"
for rep in 1 2 3; do
  for v in 8 16 0; do
    n=K32_g${v}_$rep
    FA_GRAM_GLDS=$v timeout -k 10 300 python bench.py $B --clients 32 --check-samples $([ $rep = 1 ] && echo 1 || echo 0) > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
    line $O/$n.json
  done
done
for K in 20 128; do
  timeout -k 10 300 python bench.py $B --clients $K --check-samples 1 > $O/K$K.json 2> $O/K$K.err || { tail -5 $O/K$K.err; exit 1; }
  line $O/K$K.json
done
B2="--config krum --no-cpu-baseline --soak-seconds 0 --steps 10 --warmup 2 --check-samples 0 --clients 32"
for d in 0 1 2 4 8; do
  FA_GRAM_DBG=$d timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/d$d -o tr --output-format csv -- python3 bench.py $B2 > $O/d$d.log 2>&1 || { tail -5 $O/d$d.log; exit 1; }
  python3 -c "
import csv,glob
f=glob.glob('$O/d$d/**/*kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'gram' in r['Name'] or 'pairdist' in r['Name']: print('dbg $d', r['Name'][26:52], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us avg', round(float(r['MinNs'])/1e3,1), 'min')
"
done
