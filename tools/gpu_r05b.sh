# r05b: (A) is the first bench process on a fresh box slower? three default metric lines back to back
# as the box's first GPU work (r05a: first 10.02 ms/step, later rocprof runs 9.38); (B) why §8(d)'s
# literal input (128 separate buffers) runs 9-13 % below the tiled arena: address-translation and
# memory-side stall counters for tiled / client-major arena / separate tensors, one pass per counter
# block set, the metric kernel only.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05b; mkdir -p $O
export TMPDIR=/tmp
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1],d['value'],d['ms_per_step'],r.get('kernel_avg_ms'),r.get('frac'),(d.get('sustained') or {}).get('value'))" $1; }
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --check-samples 0 --soak-seconds 3 > $O/first_$i.json 2> $O/first_$i.err || { tail -5 $O/first_$i.err; exit 1; }
  line $O/first_$i.json
done
B="--steps 3 --warmup 1 --no-cpu-baseline --check-samples 0 --soak-seconds 0"
C1="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_MULTI_MISS_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE"
C2="TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum"
for lay in tiled arena tensors; do
  for p in 1 2; do
    [ $p = 1 ] && C=$C1 || C=$C2
    timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $C --kernel-include-regex 'k_wsum' -d $O/pmc_${lay}_$p -o pmc --output-format csv -- python3 bench.py --layout $lay $B > $O/pmc_${lay}_$p.log 2>&1 \
      || { echo "FAIL $lay $p"; tail -5 $O/pmc_${lay}_$p.log; exit 1; }
    echo "== $lay pass $p"; tail -1 $O/pmc_${lay}_$p.log | cut -c1-200
  done
done
exit 0
