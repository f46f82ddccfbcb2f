# k_pairdist bound analysis: FA_PAIR_MODE 0 = normal, 1 = pair loop only (no staging / barriers,
# results wrong), 2 = staging only (no pair loop).  Timings only.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r02m
r() { timeout -k 10 120 env FA_PAIR_MODE=$2 python bench.py --config krum --clients $1 --no-cpu-baseline --check-samples 0 --steps 8 --warmup 2 > gpurun_out/r02m/ks.json 2>gpurun_out/r02m/ks.err || { echo FAIL $1 $2; tail -3 gpurun_out/r02m/ks.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/r02m/ks.json'));print('K=$1 mode=$2', d['roofline']['kernel_avg_ms'])" | tee -a gpurun_out/r02m/sweep.txt; }
for K in 8 32 64 128; do for m in 0 1 2; do r $K $m; done; done
echo done
