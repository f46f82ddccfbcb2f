# r04t: VALU utilisation of the Krum tile kernels (K = 128 k_pairdist, K = 32 k_pairdist_lane): SQ
# instruction / active-cycle counters + GRBM_GUI_ACTIVE in one pass each, kernel trace for durations.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r04t; mkdir -p $O
export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
for K in 128 32; do
  [ $K = 128 ] && R='k_pairdist<' || R='k_pairdist_lane'
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C --kernel-include-regex "$R" -d $O/pmc_$K -o pmc --output-format csv -- python3 bench.py --config krum --clients $K --no-cpu-baseline --check-samples 0 --steps 3 --warmup 1 --soak-seconds 0 > $O/pmc_$K.log 2>&1 \
    || { echo "FAIL $K"; tail -5 $O/pmc_$K.log; exit 1; }
  ls $O/pmc_$K
done
