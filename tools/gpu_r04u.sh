# r04u: where k_median_2l (K = 128, tiled) spends its cycles: SQ instruction / active / wait counters,
# resident waves, GRBM_GUI_ACTIVE (clock), one pass + kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r04u; mkdir -p $O
export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C --kernel-include-regex "k_median" -d $O/pmc -o pmc --output-format csv -- python3 bench.py --config median --clients 128 --layout tiled --no-cpu-baseline --check-samples 0 --steps 3 --warmup 1 --soak-seconds 0 > $O/pmc.log 2>&1 \
  || { echo "FAIL"; tail -5 $O/pmc.log; exit 1; }
ls $O/pmc
