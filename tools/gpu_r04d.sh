# r04d: k_pairdist_oq with float32 level-2 sums (L2F, 3 waves/SIMD) vs float64 run sums (2 waves/SIMD) vs
# the 4x4-tile kernels: parity, interleaved timing, SQ counters at K = 128 / 32.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r04d; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_robust.py -k "pairwise or krum" > $O/pytest.txt 2>&1 \
  || { echo "pytest FAIL"; tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1],d['value'],d['unit'],d['ms_per_step'],r.get('kernel_avg_ms'),'|',d.get('parity'))" $1; }
var() { case $1 in l2f) echo "FA_PAIR_OQ=1 FA_PAIR_OQ_L2F=1";; d64) echo "FA_PAIR_OQ=1 FA_PAIR_OQ_L2F=0";; old) echo "FA_PAIR_OQ=0";; esac; }
for rep in 1 2; do
  for K in 128 32 64; do
    for v in l2f d64 old; do
      n=krum_K${K}_${v}_r$rep
      env $(var $v) timeout -k 10 300 python bench.py --config krum --clients $K --steps 10 --warmup 3 --no-cpu-baseline > $O/$n.json 2> $O/$n.err \
        || { echo "FAIL $n"; tail -8 $O/$n.err; exit 1; }
      line $O/$n.json
    done
  done
done
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
D="SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD"
for K in 128 32; do
  for v in l2f d64 old; do
    for pass in C D; do
      eval cnt=\$$pass
      env $(var $v) timeout -s KILL 120 rocprofv3 --pmc $cnt --kernel-include-regex k_pairdist -d $O/pmc_${K}_${v}_$pass -o pmc --output-format csv -- python3 bench.py --config krum --clients $K --no-cpu-baseline --check-samples 0 --steps 3 --warmup 1 > $O/pmc_${K}_${v}_$pass.log 2>&1 \
        || { echo "PMC FAIL $K $v $pass"; tail -5 $O/pmc_${K}_${v}_$pass.log; exit 1; }
      f=$(find $O/pmc_${K}_${v}_$pass -name "*counter_collection.csv" | head -1)
      python3 tools/pmc_sq.py $f > $O/pmc_${K}_${v}_$pass.txt 2>&1; cat $O/pmc_${K}_${v}_$pass.txt
    done
  done
done
