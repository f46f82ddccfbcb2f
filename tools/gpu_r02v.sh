# Krum distances: workgroup count sweep (bytes in flight per CU), FA_PAIR_BLOCKS override
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r02v
for K in 32 128 8 64; do
 for B in 1024 1280 2048 4096 512; do
  FA_PAIR_BLOCKS=$B timeout -k 10 120 python bench.py --config krum --clients $K --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/r02v/k.json 2>gpurun_out/r02v/k.err || { tail -3 gpurun_out/r02v/k.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r02v/k.json'));print($K, $B, d['roofline']['kernel_avg_ms'], d['parity'][:40])" | tee -a gpurun_out/r02v/sweep.txt
 done
done
