# two-lanes-per-column median (k_median_2l): robust GPU tests, then A/B against k_median_off
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r02x
timeout -k 10 600 python -u -m pytest tests/test_gpu_robust.py -m gpu -x -q --timeout 120 --timeout-method thread -k median > gpurun_out/r02x/robust.log 2>&1 || { tail -40 gpurun_out/r02x/robust.log; exit 1; }
tail -1 gpurun_out/r02x/robust.log
for K in 128 100 120 97 96 80 72; do
 for M in 0 1 0 1; do
  FA_MEDIAN_2L=$M timeout -k 10 120 python bench.py --config median --clients $K --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/r02x/m.json 2>gpurun_out/r02x/m.err || { tail -3 gpurun_out/r02x/m.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r02x/m.json'));print($K, '2L=$M', d['roofline']['kernel_avg_ms'], d['roofline']['frac'], str(d['parity'])[:40])" | tee -a gpurun_out/r02x/ab.txt
 done
done
