# r06aj: do the amdsmi calls themselves slow the host-bound short lines?  cfg2 tiled and Krum K = 32 with
# and without the clock block (--no-clock), 2 interleaved pairs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06aj; mkdir -p $O
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1].split('/')[-1],d['value'],d['ms_per_step'],r.get('kernel_avg_ms'),(d.get('sustained') or {}).get('ms_per_step'))" $1; }
for i in 1 2; do
  for c in resnet18 "krum --clients 32"; do
    n=$(echo $c | tr -d ' -')
    timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --cold-reps 0 --soak-seconds 2 > $O/${n}_clk_$i.json 2> $O/${n}_clk_$i.err || { tail -5 $O/${n}_clk_$i.err; exit 1; }
    line $O/${n}_clk_$i.json
    timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --cold-reps 0 --soak-seconds 2 --no-clock > $O/${n}_noclk_$i.json 2> $O/${n}_noclk_$i.err || { tail -5 $O/${n}_noclk_$i.err; exit 1; }
    line $O/${n}_noclk_$i.json
  done
done
exit 0
