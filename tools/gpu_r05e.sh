# r05e: literal input -- XCD-contiguous workgroup -> tile order for the single-segment launch
# (FA_XCD_MAP=2, staged tables FA_INLINE_DESC=0) so a CU's concurrent workgroups read consecutive
# tiles (the same translation pages of every client).  Prediction: UTCL1 misses drop
# several-fold at S = 1; time -2..-5 %.  Interleaved reps + one counter pass each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05e; mkdir -p $O
export TMPDIR=/tmp
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1],d['value'],d['ms_per_step'],r.get('kernel_avg_ms'),r.get('frac'),d.get('parity'))" $1; }
B="--no-cpu-baseline --soak-seconds 0 --steps 10 --warmup 2"
run() { n=$1; shift; env "$@" timeout -k 10 300 python bench.py $B $ARGS > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }; line $O/$n.json; }
for rep in 1 2; do
  for lay in tensors arena; do
    CS=$([ $rep = 1 ] && echo 8192 || echo 0)
    ARGS="--layout $lay --check-samples $CS"
    run ${lay}_inl_$rep FA_XCD_MAP=1
    run ${lay}_staged_rr_$rep FA_INLINE_DESC=0 FA_XCD_MAP=1
    run ${lay}_staged_xcd_$rep FA_INLINE_DESC=0 FA_XCD_MAP=2
    ARGS="--layout $lay --variant 6 --check-samples $CS"
    run ${lay}_v6_xcd_$rep FA_XCD_MAP=2
  done
done
C1="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE"
FA_INLINE_DESC=0 FA_XCD_MAP=2 timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $C1 --kernel-include-regex 'k_wsum' -d $O/pmc_tensors_xcd -o pmc --output-format csv -- python3 bench.py --layout tensors --steps 3 --warmup 1 --no-cpu-baseline --check-samples 0 --soak-seconds 0 > $O/pmc_tensors_xcd.log 2>&1 || { echo "FAIL pmc"; tail -5 $O/pmc_tensors_xcd.log; exit 1; }
exit 0
