# SQ counters of k_pairdist (wave cycles split into waiting / issuing, LDS conflicts) for a few K.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/kpmc
export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
p() { timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex k_pairdist -d gpurun_out/kpmc/K$1 -o pmc --output-format csv -- python3 bench.py --config krum --clients $1 --no-cpu-baseline --check-samples 0 --steps 3 --warmup 1 > gpurun_out/kpmc/K$1.log 2>&1 || { echo FAIL $1; tail -5 gpurun_out/kpmc/K$1.log; exit 1; }; }
for K in ${KS:-32 64 128}; do p $K; done
