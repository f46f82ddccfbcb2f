# r03c: Krum k_pairdist instruction-mix PMC, K = 32 and 128, separate passes
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r03c; mkdir -p $O
export TMPDIR=/tmp
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU"
B="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD"
for K in 32 128; do
  timeout -k 10 120 python bench.py --config krum --clients $K --no-cpu-baseline --steps 5 --warmup 2 > $O/bench_K$K.json 2> $O/bench_K$K.err || { tail -5 $O/bench_K$K.err; exit 1; }
  cat $O/bench_K$K.json
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt_K$K -o kt --output-format csv -- python3 bench.py --config krum --clients $K --no-cpu-baseline --check-samples 0 --steps 5 --warmup 1 > $O/kt_K$K.log 2>&1 || { tail -5 $O/kt_K$K.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc $A --kernel-include-regex k_pairdist -d $O/pa_K$K -o pmc --output-format csv -- python3 bench.py --config krum --clients $K --no-cpu-baseline --check-samples 0 --steps 2 --warmup 1 > $O/pa_K$K.log 2>&1 || { echo FAIL A $K; tail -5 $O/pa_K$K.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc $B --kernel-include-regex k_pairdist -d $O/pb_K$K -o pmc --output-format csv -- python3 bench.py --config krum --clients $K --no-cpu-baseline --check-samples 0 --steps 2 --warmup 1 > $O/pb_K$K.log 2>&1 || { echo FAIL B $K; tail -5 $O/pb_K$K.log; exit 1; }
done
find $O -name "*.csv" | head -20
