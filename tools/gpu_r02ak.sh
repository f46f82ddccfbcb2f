# k_median_2l: sentinel masking only on the last 8 slots -- median GPU tests + timings (compare r02y)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r02ak
timeout -k 10 600 python -u -m pytest tests/test_gpu_robust.py -m gpu -x -q --timeout 120 --timeout-method thread -k median > gpurun_out/r02ak/robust.log 2>&1 || { tail -40 gpurun_out/r02ak/robust.log; exit 1; }
tail -1 gpurun_out/r02ak/robust.log
for K in 100 120 121 97 80 128; do
 for r in 1 2; do
  timeout -k 10 120 python bench.py --config median --clients $K --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/r02ak/m.json 2>gpurun_out/r02ak/m.err || { tail -3 gpurun_out/r02ak/m.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r02ak/m.json'));print($K, d['roofline']['kernel_avg_ms'], d['roofline']['frac'], str(d['parity'])[:40])" | tee -a gpurun_out/r02ak/t.txt
 done
done
