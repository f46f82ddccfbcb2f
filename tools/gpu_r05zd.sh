# r05zd: k_gram_reduce with 16 entries x 64 row splits per workgroup (was 64 entries x 16): robust
# pairwise / Krum tests, then K = 32 / 64 / 128 lines at the sustained clock and one kernel trace of
# K = 32 (the reduce's duration; r05q: 10.5 us over 512 partials).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05zd; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_robust.py -x -q --timeout 120 --timeout-method thread -k "pairwise or krum" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1].split('/')[-1],d['value'],d['ms_per_step'],r.get('kernel_avg_ms'),r.get('bound'),r.get('frac'),d.get('parity'))" $1; }
for K in 32 64 128; do
  timeout -k 10 300 python bench.py --config krum --clients $K --steps 50 --warmup 150 --no-cpu-baseline --soak-seconds 0 --check-samples 1 > $O/K$K.json 2> $O/K$K.err || { tail -5 $O/K$K.err; exit 1; }
  line $O/K$K.json
done
timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d $O/trace -o tr --output-format csv -- python3 bench.py --config krum --clients 32 --steps 20 --warmup 50 --no-cpu-baseline --check-samples 0 --soak-seconds 0 > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
python3 -c "
import csv,glob
f=glob.glob('$O/trace/**/*kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'gram' in r['Name'] or 'pairdist' in r['Name']: print(r['Name'][26:60], r['Calls'], round(float(r['AverageNs'])/1e3,2), 'us')
"
