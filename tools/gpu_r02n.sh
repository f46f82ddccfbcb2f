# k_pairdist r02n: parity, then timings over K and SQ counters at K = 32 / 128.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r02n
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_robust.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r02n/t.log 2>&1 || { tail -30 gpurun_out/r02n/t.log; exit 1; }
tail -1 gpurun_out/r02n/t.log
r() { timeout -k 10 120 python bench.py --config krum --clients $1 --no-cpu-baseline --check-samples ${CS:-0} --steps 8 --warmup 2 > gpurun_out/r02n/K$1.json 2>gpurun_out/r02n/ks.err || { echo FAIL $1; tail -3 gpurun_out/r02n/ks.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/r02n/K$1.json'));print('K=$1', d['roofline']['kernel_avg_ms'], d['roofline'].get('frac'), d.get('parity'))" | tee -a gpurun_out/r02n/sweep.txt; }
for K in 8 16 32 64 100 128; do r $K; done
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
for K in 32 128; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex k_pairdist -d gpurun_out/r02n/pmcK$K -o pmc --output-format csv -- python3 bench.py --config krum --clients $K --no-cpu-baseline --check-samples 0 --steps 3 --warmup 1 > gpurun_out/r02n/pmcK$K.log 2>&1 || { echo PMCFAIL $K; tail -5 gpurun_out/r02n/pmcK$K.log; exit 1; }
done
echo done
