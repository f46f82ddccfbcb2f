# median B = 128: W = 2 (spills) vs W = 1 (no spills) A/B, interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r02w
for K in 128 100 120; do
 for W in 0 1 0 1; do
  FA_MEDIAN_W1=$W timeout -k 10 120 python bench.py --config median --clients $K --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/r02w/m.json 2>gpurun_out/r02w/m.err || { tail -3 gpurun_out/r02w/m.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r02w/m.json'));print($K, 'W1=$W', d['roofline']['kernel_avg_ms'], d['roofline']['frac'], str(d['parity'])[:40])" | tee -a gpurun_out/r02w/ab.txt
 done
done
