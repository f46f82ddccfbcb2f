# k_median_2l below K = 64 (B = 40..64, N = 20..32) vs k_median_off: interleaved A/B (parity checked per run)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r02ab
for K in 64 56 48 40 33; do
 for M in 0 1 0 1; do
  FA_MEDIAN_2L=$M timeout -k 10 120 python bench.py --config median --clients $K --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/r02ab/m.json 2>gpurun_out/r02ab/m.err || { tail -3 gpurun_out/r02ab/m.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r02ab/m.json'));print($K, '2L=$M', d['roofline']['kernel_avg_ms'], d['roofline']['frac'], str(d['parity'])[:40])" | tee -a gpurun_out/r02ab/ab.txt
 done
done
