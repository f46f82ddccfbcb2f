# k_pairdist r02o: staging width NP = 8 / 16 (FA_PAIR_NP), parity under NP=16, timings over K.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r02o
timeout -k 10 300 env FA_PAIR_NP=16 python -u -m pytest tests/test_gpu_robust.py -k pairwise -x -q --timeout 120 --timeout-method thread > gpurun_out/r02o/t.log 2>&1 || { tail -30 gpurun_out/r02o/t.log; exit 1; }
tail -1 gpurun_out/r02o/t.log
r() { timeout -k 10 120 env FA_PAIR_NP=$2 python bench.py --config krum --clients $1 --no-cpu-baseline --check-samples 0 --steps 8 --warmup 2 > gpurun_out/r02o/ks.json 2>gpurun_out/r02o/ks.err || { echo FAIL $1; tail -3 gpurun_out/r02o/ks.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/r02o/ks.json'));print('K=$1 np=$2', d['roofline']['kernel_avg_ms'])" | tee -a gpurun_out/r02o/sweep.txt; }
for K in 8 16 32 64 100 128; do for np in 8 16; do r $K $np; done; done
echo done
