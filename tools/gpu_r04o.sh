# r04o: SQ counters of k_pairdist_circ at K = 32 and 16 (LDS bank conflicts, issue / wait split).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r04o; mkdir -p $O
export TMPDIR=/tmp
CC="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
CD="SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVES SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD"
for K in 32 16; do
  for p in C D; do
    [ $p = C ] && CN="$CC" || CN="$CD"
    timeout -s KILL 120 rocprofv3 --pmc $CN --kernel-include-regex k_pairdist_circ -d $O/pmc_${K}_$p -o pmc --output-format csv -- python3 bench.py --config krum --clients $K --no-cpu-baseline --check-samples 0 --steps 3 --warmup 1 --soak-seconds 0 > $O/pmc_${K}_$p.log 2>&1 \
      || { echo "FAIL $K $p"; tail -5 $O/pmc_${K}_$p.log; exit 1; }
    f=$(find $O/pmc_${K}_$p -name "*counter_collection.csv" | head -1)
    python3 tools/pmc_sq.py $f | tee $O/pmc_${K}_$p.txt
  done
done
