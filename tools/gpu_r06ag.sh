# r06ag: r06af again after moving the amdsmi init (ClockSampler) before the warmup: the short lines'
# timed steps with and without the read probe, 2 rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06ag; mkdir -p $O
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1].split('/')[-1],d['value'],d['ms_per_step'],r.get('kernel_avg_ms'),(d.get('sustained') or {}).get('ms_per_step'))" $1; }
for i in 1 2; do
  for c in "krum --clients 64" "krum --clients 128" "median --clients 128" "krum --clients 32"; do
    n=$(echo $c | tr -d ' -')
    timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --cold-reps 0 --check-samples 0 --soak-seconds 2 > $O/${n}_probe_$i.json 2> $O/${n}_probe_$i.err || { tail -5 $O/${n}_probe_$i.err; exit 1; }
    line $O/${n}_probe_$i.json
    timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --cold-reps 0 --check-samples 0 --soak-seconds 2 --no-read-probe > $O/${n}_noprobe_$i.json 2> $O/${n}_noprobe_$i.err || { tail -5 $O/${n}_noprobe_$i.err; exit 1; }
    line $O/${n}_noprobe_$i.json
  done
done
exit 0
