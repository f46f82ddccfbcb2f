# r05c: §8(d)'s literal input (128 separate fp32[125 M] buffers) and the client-major arena are
# ADDRESS-TRANSLATION bound (r05b: UTCL2 busy 96 % of the kernel vs 4 % tiled, UTCL1 misses 330x).
# Prediction: more consecutive 4-KiB slots per client per workgroup (S = 2 / 4, the
# kernel variants 4-6, 8) cut the translation lookups that miss per byte and recover part of the
# 9-13 % gap.  Two interleaved reps of every variant on one box, then the translation counters of
# the best S.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05c; mkdir -p $O
export TMPDIR=/tmp
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1],d['value'],d['ms_per_step'],r.get('kernel_avg_ms'),r.get('frac'),d.get('parity'))" $1; }
B="--no-cpu-baseline --soak-seconds 0 --steps 10 --warmup 2"
for rep in 1 2; do
  for lay in tensors arena; do
    for v in 0 4 5 6 8; do
      n=${lay}_v${v}_$rep
      timeout -k 10 300 python bench.py --layout $lay --variant $v $B --check-samples $([ $rep = 1 ] && echo 8192 || echo 0) > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
      line $O/$n.json
    done
  done
  n=tiled_v0_$rep
  timeout -k 10 300 python bench.py $B --check-samples 0 > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
  line $O/$n.json
done
# cfg1 with the host-resident sum (host_sum.h) and the host/device break-even sweep
timeout -k 10 300 python bench.py --config lr > $O/lr.json 2> $O/lr.err || { tail -5 $O/lr.err; exit 1; }
python -c "import json;d=json.loads(open('$O/lr.json').read().strip().splitlines()[-1]);print('lr',d['value'],d['unit'],d.get('latency_ms'),d['cpu_baseline']['value'],d['parity'],d.get('host_path'));[print(r) for r in d['host_breakeven']['rows']]"
C1="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE"
for v in 5 6; do
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $C1 --kernel-include-regex 'k_wsum' -d $O/pmc_tensors_v$v -o pmc --output-format csv -- python3 bench.py --layout tensors --variant $v --steps 3 --warmup 1 --no-cpu-baseline --check-samples 0 --soak-seconds 0 > $O/pmc_tensors_v$v.log 2>&1 \
    || { echo "FAIL pmc $v"; tail -5 $O/pmc_tensors_v$v.log; exit 1; }
done
exit 0
