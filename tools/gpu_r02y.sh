# k_median_2l generalised to N = B/2 (B = 72..128): robust GPU tests (default dispatch), A/B vs k_median_off per bucket
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r02y
timeout -k 10 600 python -u -m pytest tests/test_gpu_robust.py -m gpu -x -q --timeout 120 --timeout-method thread -k median > gpurun_out/r02y/robust.log 2>&1 || { tail -40 gpurun_out/r02y/robust.log; exit 1; }
tail -1 gpurun_out/r02y/robust.log
for K in 128 121 120 112 104 100 97 96 88 80 72 65; do
 for M in 0 1 0 1; do
  FA_MEDIAN_2L=$M timeout -k 10 120 python bench.py --config median --clients $K --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/r02y/m.json 2>gpurun_out/r02y/m.err || { tail -3 gpurun_out/r02y/m.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r02y/m.json'));print($K, '2L=$M', d['roofline']['kernel_avg_ms'], d['roofline']['frac'], str(d['parity'])[:40])" | tee -a gpurun_out/r02y/ab.txt
 done
done
