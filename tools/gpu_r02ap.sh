# XCD-contiguous mapping on by default for multi-segment launches: full GPU suite + fragmented/cfg2-tensors bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r02ap
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02ap/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r02ap/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r02ap/gpu_tests.log
timeout -k 10 300 python bench.py --config fragmented --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/r02ap/fragmented.json 2>gpurun_out/r02ap/f.err || { tail -3 gpurun_out/r02ap/f.err; exit 1; }
timeout -k 10 300 python bench.py --config resnet18 --layout tensors --no-cpu-baseline --steps 30 --warmup 5 > gpurun_out/r02ap/resnet18_tensors.json 2>gpurun_out/r02ap/r.err || { tail -3 gpurun_out/r02ap/r.err; exit 1; }
for f in fragmented resnet18_tensors; do python -c "import json;d=json.load(open('gpurun_out/r02ap/$f.json'));print('$f', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'], str(d['parity'])[:30])"; done
