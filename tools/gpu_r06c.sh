# r06c: every short-step line with its cold per-round latency (the first call
# after 1 s idle, median of 5) beside the sustained-clock rate, and rocprofv3 kernel traces taken at
# the sustained clock (auto warmup + a 3 s soak: the soak's calls dominate the trace's average) for
# median K = 128 and Krum K = 32 / 64 / 128, so that profiles/ holds the numbers README and DESIGN quote.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06c; mkdir -p $O
export TMPDIR=/tmp
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};c=d.get('cold') or {};print(sys.argv[1].split('/')[-1],d['value'],d['unit'],d['ms_per_step'],r.get('kernel_avg_ms'),r.get('frac'),r.get('frac_of_ceiling'),'cold',c.get('ms'),c.get('event_ms'),d.get('pair_form'),str(d.get('parity'))[:60])" $1; }
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_krum_band.py tests/test_gpu_robust.py -k "band or pairwise or krum or sticky" > $O/tests_krum.log 2>&1; rc=$?
tail -2 $O/tests_krum.log; [ $rc = 0 ] || exit $rc
run() {  # name, bench args
  n=$1; shift
  timeout -k 10 400 python bench.py "$@" --no-cpu-baseline --soak-seconds 0 > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
  line $O/$n.json
}
run median128 --config median --clients 128
run median32 --config median --clients 32
run krum32 --config krum --clients 32
run krum64 --config krum --clients 64
run krum128 --config krum --clients 128
run cfg2_tiled --config resnet18
run cfg2_tensors --config resnet18 --layout tensors
run cfg1_lr --config lr
run cfg3_vit --config vit_bf16
run cfg4_hier --config hier
run cfg5_gossip --config gossip
prof() {  # name, bench args: kernel trace at the sustained clock
  n=$1; shift
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r06c_$n -o run -- python3 bench.py "$@" --no-cpu-baseline --soak-seconds 3 --cold-reps 0 --check-samples 0 > $O/prof_$n.json 2> $O/prof_$n.err || { tail -5 $O/prof_$n.err; exit 1; }
  cp $(find /tmp/r06c_$n -name '*kernel_stats.csv' | head -1) $O/prof_${n}_kernel_stats.csv
  line $O/prof_$n.json
  head -3 $O/prof_${n}_kernel_stats.csv | cut -c1-160
}
prof median128 --config median --clients 128
prof krum32 --config krum --clients 32
prof krum64 --config krum --clients 64
prof krum128 --config krum --clients 128
exit 0
