# Interleaved A/B of the weighted-sum kernel variants on the default (tiled) metric.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for rep in 1 2; do for v in 0 1 2 4 5 7 8; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --check-samples 4096 --variant $v > gpurun_out/v.json 2>>gpurun_out/v.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/v.json'));print('variant', $v, d['value'], d['roofline']['kernel_avg_ms'], d['parity'][:9])"
done; done
