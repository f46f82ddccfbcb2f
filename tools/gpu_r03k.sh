# r03k: round-3 profiles of the headline metric (kernel trace + FETCH/WRITE PMC) and the median K=128 instruction mix
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r03k; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -5 $O/bench_default.err; exit 1; }
cat $O/bench_default.json
bash tools/profile.sh r03_metric || exit 1
M="--config median --clients 128 --no-cpu-baseline --check-samples 0 --steps 3 --warmup 1"
timeout -k 10 120 python bench.py --config median --clients 128 --no-cpu-baseline --steps 10 --warmup 2 > $O/median_K128.json 2> $O/median.err || { tail -5 $O/median.err; exit 1; }
cat $O/median_K128.json
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU"
B="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE"
timeout -s KILL 90 rocprofv3 --pmc $A --kernel-include-regex k_median -d $O/ma -o pmc --output-format csv -- python3 bench.py $M > $O/ma.log 2>&1 || { echo FAIL A; tail -5 $O/ma.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc $B --kernel-include-regex k_median -d $O/mb -o pmc --output-format csv -- python3 bench.py $M > $O/mb.log 2>&1 || { echo FAIL B; tail -5 $O/mb.log; exit 1; }
ls gpurun_out/summary
echo done
