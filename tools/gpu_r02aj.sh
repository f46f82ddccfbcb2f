# Krum K <= 32: register double-buffered LDS reads (PF) vs the r01 loop, interleaved; robust tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r02aj
timeout -k 10 600 python -u -m pytest tests/test_gpu_robust.py -m gpu -x -q --timeout 120 --timeout-method thread -k "pairwise or krum" > gpurun_out/r02aj/robust.log 2>&1 || { tail -40 gpurun_out/r02aj/robust.log; exit 1; }
tail -1 gpurun_out/r02aj/robust.log
for K in 32 16 8 24; do
 for M in 0 1 0 1; do
  FA_PAIR_PF=$M timeout -k 10 120 python bench.py --config krum --clients $K --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/r02aj/k.json 2>gpurun_out/r02aj/k.err || { tail -3 gpurun_out/r02aj/k.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r02aj/k.json'));print($K, 'PF=$M', d['roofline']['kernel_avg_ms'], str(d['parity'])[:40])" | tee -a gpurun_out/r02aj/ab.txt
 done
done
