# r04x: is the small-model rate set by the last partial round of workgroups?  Tiles of 1,024 floats:
# P = 11,699,132 -> 11,425 tiles (5.58 rounds of 2,048 resident workgroups); 10,485,760 -> 10,240 (5.0);
# 12,582,912 -> 12,288 (6.0).  Metric kernel at K = 32 and the grouped hier kernel (8 x 64), 2 reps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r04x; mkdir -p $O
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1],d['value'],d['unit'],d['ms_per_step'],r.get('kernel_avg_ms'),r.get('frac'))" $1; }
b() { n=$1; shift; timeout -k 10 200 python bench.py "$@" --steps 20 --warmup 3 --no-cpu-baseline --check-samples 0 --soak-seconds 0 > $O/$n.json 2> $O/$n.err || { echo "FAIL $n"; tail -8 $O/$n.err; exit 1; }; line $O/$n.json; }
for rep in 1 2; do
  for P in 10485760 11699132 12582912; do
    b m32_P${P}_r$rep --config metric --clients 32 --params $P
    b hier_P${P}_r$rep --config hier --params $P
  done
done
