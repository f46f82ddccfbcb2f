# r03u: separate-tensor drop-in paths: cfg3 ViT bf16 (k_wsum, ctx variants 0/4/5/6) and cfg2 ResNet-18
# (k_wsum_pair, FA_PAIR_S=2 vs default), interleaved x2, parity on.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
r() { timeout -k 10 300 python bench.py --config $1 --layout tensors --no-cpu-baseline --steps 20 --warmup 5 $2 > gpurun_out/u.json 2> gpurun_out/u.err || { echo FAIL $1 $2; tail -5 gpurun_out/u.err; exit 1; }
      A="$1 $2 $3" python -c 'import json,os;d=json.load(open("gpurun_out/u.json"));print(os.environ["A"], d["value"], d["ms_per_step"], d["roofline"].get("kernel_avg_ms"), d["roofline"].get("frac"), d.get("parity"))'; }
for rep in 1 2; do
  for v in 0 4 5 6; do r vit_bf16 "--variant $v"; done
  r resnet18 "" default
  FA_PAIR_S=2 r resnet18 "" S2
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_finite.py -m gpu -x -q -k "mt_ or secagg" --timeout 200 --timeout-method thread > gpurun_out/pytest_u.log 2>&1 || { tail -30 gpurun_out/pytest_u.log; exit 1; }
FA_MT_JUMP_SPOS=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_finite.py -m gpu -x -q -k "mt_ or secagg" --timeout 200 --timeout-method thread > gpurun_out/pytest_u1.log 2>&1 || { tail -30 gpurun_out/pytest_u1.log; exit 1; }
echo "mt tests: $(tail -1 gpurun_out/pytest_u.log) / spos $(tail -1 gpurun_out/pytest_u1.log)"
for rep in 1 2 3; do
  for sp in 0 1; do
    FA_MT_JUMP_SPOS=$sp timeout -k 10 300 python bench.py --config samask --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/sa.json 2> gpurun_out/sa.err || { tail -5 gpurun_out/sa.err; exit 1; }
    SP=$sp python -c 'import json,os;d=json.load(open("gpurun_out/sa.json"));print("spos", os.environ["SP"], d["value"], d["unit"], d.get("parity"))'
  done
done
