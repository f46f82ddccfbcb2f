# r06ae: sustained-clock kernel traces of the final binary (auto warmup + a 3 s soak under rocprofv3
# --kernel-trace --stats): Krum K = 32 / 64 / 96 / 128 and median K = 128 -- the numbers the
# "Current numbers" table quotes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06ae; mkdir -p $O
export TMPDIR=/tmp
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1].split('/')[-1],d['value'],d['ms_per_step'],r.get('kernel_avg_ms'),d.get('pair_form'),(d.get('sustained') or {}).get('ms_per_step'))" $1; }
prof() {  # name, bench args
  n=$1; shift
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r06ae_$n -o run -- python3 bench.py "$@" --no-cpu-baseline --soak-seconds 3 --cold-reps 0 --check-samples 0 > $O/prof_$n.json 2> $O/prof_$n.err || { tail -5 $O/prof_$n.err; exit 1; }
  cp $(find /tmp/r06ae_$n -name '*kernel_stats.csv' | head -1) $O/prof_${n}_kernel_stats.csv
  line $O/prof_$n.json
  head -3 $O/prof_${n}_kernel_stats.csv | cut -c1-150
}
prof krum32 --config krum --clients 32
prof krum64 --config krum --clients 64
prof krum96 --config krum --clients 96
prof krum128 --config krum --clients 128
prof median128 --config median --clients 128
exit 0
