set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
r() { timeout -k 10 200 python bench.py --config krum --clients $K --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/k.json 2>>gpurun_out/k.err || { echo FAIL $K $FA_KRUM_ESPLIT $FA_KRUM_PER $FA_KRUM_BLOCKS; tail -3 gpurun_out/k.err; return 0; }
      python -c "import json,os;d=json.load(open('gpurun_out/k.json'));print(os.environ.get('K'), 'esplit', os.environ.get('FA_KRUM_ESPLIT'), 'per', os.environ.get('FA_KRUM_PER'), 'blocks', os.environ.get('FA_KRUM_BLOCKS'), d['roofline']['kernel_avg_ms'], d['parity'][:30])"; }
for K in 8 32; do export K
 for B in 512 1024 2048; do export FA_KRUM_BLOCKS=$B
  for ES in 0 4 2; do export FA_KRUM_ESPLIT=$ES
   for PER in 8 16 32 64; do export FA_KRUM_PER=$PER; r; done; done; done; done
