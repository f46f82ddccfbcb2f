# cfg2 / cfg3 (state_dict layouts) on one GPU in every arena layout + the arena GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread tests/test_gpu_pair.py -k "pair or arena or state_dict or layout" > gpurun_out/pytest_arena.log 2>&1 || { tail -20 gpurun_out/pytest_arena.log; exit 1; }
tail -2 gpurun_out/pytest_arena.log
for c in resnet18 vit_bf16; do
  for l in arena tiled; do
    timeout -k 10 300 python bench.py --config $c --layout $l --steps ${STEPS:-50} --warmup 5 --no-cpu-baseline > gpurun_out/bench_${c}_$l.json 2> gpurun_out/bench_${c}_$l.err || { tail -5 gpurun_out/bench_${c}_$l.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/bench_${c}_$l.json'));print('$c $l',d['value'],d['ms_per_step'],d['roofline'].get('kernel_avg_ms'),d.get('parity'))"
  done
done
