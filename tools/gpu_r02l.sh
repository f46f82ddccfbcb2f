# k_pairdist variants: parity under each (staging width NP, GMID float64-in-partial-row), timings
# over K, then SQ counters of the built-in choice.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r02l
export TMPDIR=/tmp
T="tests/test_gpu_robust.py -k pairwise"
timeout -k 10 240 env FA_PAIR_NP=16 FA_PAIR_GMID=1 python -u -m pytest $T -x -q --timeout 120 --timeout-method thread > gpurun_out/r02l/t_np16_g.log 2>&1 || { tail -30 gpurun_out/r02l/t_np16_g.log; exit 1; }
tail -1 gpurun_out/r02l/t_np16_g.log
timeout -k 10 240 env FA_PAIR_NP=32 python -u -m pytest $T -x -q --timeout 120 --timeout-method thread > gpurun_out/r02l/t_np32.log 2>&1 || { tail -30 gpurun_out/r02l/t_np32.log; exit 1; }
tail -1 gpurun_out/r02l/t_np32.log
r() { timeout -k 10 120 env FA_PAIR_NP=$2 FA_PAIR_GMID=$3 python bench.py --config krum --clients $1 --no-cpu-baseline --check-samples 0 --steps 8 --warmup 2 > gpurun_out/r02l/ks.json 2>gpurun_out/r02l/ks.err || { echo FAIL $1 $2 $3; tail -3 gpurun_out/r02l/ks.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/r02l/ks.json'));print('K=$1 np=$2 gmid=$3', d['roofline']['kernel_avg_ms'])" | tee -a gpurun_out/r02l/sweep.txt; }
for K in 8 32 64 100 128; do for np in 8 16 32; do for g in 0 1; do r $K $np $g; done; done; done
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
for K in 32 128; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex k_pairdist -d gpurun_out/r02l/pmcK$K -o pmc --output-format csv -- python3 bench.py --config krum --clients $K --no-cpu-baseline --check-samples 0 --steps 3 --warmup 1 > gpurun_out/r02l/pmcK$K.log 2>&1 || { echo PMCFAIL $K; tail -5 gpurun_out/r02l/pmcK$K.log; exit 1; }
done
echo done
