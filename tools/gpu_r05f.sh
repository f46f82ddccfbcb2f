# r05f: GPU parity suite + smoke on the current code (staging-shadow fix, XCD-contiguous flat launches,
# pair S = 4 knob), then interleaved A/B: literal input with / without the XCD map (FA_XCD_MAP=0 is
# the old round-robin), cfg2 on separate tensors with 1 vs 4 slots per client (FA_PAIR_S=4), and the
# default metric line (tiled arena: unchanged path).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05f; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1],d['value'],d['ms_per_step'],r.get('kernel_avg_ms'),r.get('frac'),d.get('parity'))" $1; }
B="--no-cpu-baseline --soak-seconds 0"
run() { n=$1; shift; env "$@" timeout -k 10 300 python bench.py $B $ARGS > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }; line $O/$n.json; }
for rep in 1 2 3; do
  CS=$([ $rep = 1 ] && echo 65536 || echo 0)
  ARGS="--layout tensors --check-samples $CS"
  run tensors_xcd_$rep FA_XCD_MAP=1
  run tensors_rr_$rep FA_XCD_MAP=0
  ARGS="--config resnet18 --layout tensors --steps 50 --warmup 5 --check-samples $CS"
  run cfg2t_s1_$rep FA_PAIR_S=1
  run cfg2t_s4_$rep FA_PAIR_S=4
  ARGS="--check-samples $CS"
  run metric_$rep FA_XCD_MAP=1
done
