# XCD-contiguous mapping also for the staged pair kernel (cfg2 separate tensors): pair/parity tests, A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r02aq
timeout -k 10 600 python -u -m pytest tests/test_gpu_pair.py tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02aq/tests.log 2>&1 || { tail -30 gpurun_out/r02aq/tests.log; exit 1; }
tail -1 gpurun_out/r02aq/tests.log
for M in 0 1 0 1 0 1; do
  FA_XCD_MAP=$M timeout -k 10 300 python bench.py --config resnet18 --layout tensors --no-cpu-baseline --steps 30 --warmup 5 > gpurun_out/r02aq/b.json 2>gpurun_out/r02aq/b.err || { tail -3 gpurun_out/r02aq/b.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r02aq/b.json'));print('resnet18_tensors', 'xcd=$M', d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'], str(d['parity'])[:30])" | tee -a gpurun_out/r02aq/ab.txt
done
