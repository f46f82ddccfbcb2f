# r03q: SecAgg jump kernel with pair-index positions: parity, bench, kernel trace, one SQ PMC pass on k_mt_jump.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_finite.py -m gpu -x -q -k "mt_ or secagg" --timeout 200 --timeout-method thread > gpurun_out/pytest_q.log 2>&1 || { tail -30 gpurun_out/pytest_q.log; exit 1; }
tail -1 gpurun_out/pytest_q.log
for rep in 1 2; do
  timeout -k 10 300 python bench.py --config samask --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/sa.json 2> gpurun_out/sa.err || { tail -5 gpurun_out/sa.err; exit 1; }
  python -c 'import json;d=json.load(open("gpurun_out/sa.json"));print("samask", d["value"], d["unit"], d.get("parity"))'
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sa -o sa -- python bench.py --config samask --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/sa_prof.json 2> gpurun_out/sa_prof.err || { tail -5 gpurun_out/sa_prof.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY --kernel-include-regex k_mt_jump --output-format csv -d gpurun_out/pmc_jump -o j -- python bench.py --config samask --no-cpu-baseline --steps 1 --warmup 0 --check-samples 0 > gpurun_out/pmc_jump.json 2> gpurun_out/pmc_jump.err || { tail -5 gpurun_out/pmc_jump.err; exit 1; }
find gpurun_out/pmc_jump -name "*counter_collection.csv" | head -1
