# r04q: the median read pattern's own floor on the tiled arena layout (tools/median_access_probe.hip
# run_tiled) beside the client-major rows, then the median bench at K = 128 tiled / arena (2 reps).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r04q; mkdir -p $O
hipcc --offload-arch=gfx950 -O3 -o /tmp/map tools/median_access_probe.hip 2>/dev/null || { echo "probe build FAIL"; exit 1; }
timeout -k 10 120 /tmp/map > $O/median_access_probe.txt 2>&1 || { echo "probe FAIL"; cat $O/median_access_probe.txt; exit 1; }
cat $O/median_access_probe.txt
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1],d['value'],d['unit'],d['ms_per_step'],r.get('kernel_avg_ms'),r.get('frac'))" $1; }
for rep in 1 2; do
  for lay in tiled arena; do
    n=median_K128_${lay}_r$rep
    timeout -k 10 300 python bench.py --config median --clients 128 --layout $lay --steps 20 --warmup 3 --no-cpu-baseline --soak-seconds 0 > $O/$n.json 2> $O/$n.err || { echo "FAIL $n"; tail -5 $O/$n.err; exit 1; }
    line $O/$n.json
  done
done
