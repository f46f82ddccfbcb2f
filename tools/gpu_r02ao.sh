# XCD-contiguous workgroup->tile mapping (FA_XCD_MAP=1) for the staged multi-segment kernel: the
# fragmented metric (204 tensors/client) and cfg2 on separate tensors, interleaved A/B; parity each run
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r02ao
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02ao/parity.log 2>&1 || { tail -30 gpurun_out/r02ao/parity.log; exit 1; }
FA_XCD_MAP=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02ao/parity_x.log 2>&1 || { tail -30 gpurun_out/r02ao/parity_x.log; exit 1; }
tail -1 gpurun_out/r02ao/parity.log; tail -1 gpurun_out/r02ao/parity_x.log
for C in fragmented resnet18; do
 for M in 0 1 0 1; do
  A="--config $C --no-cpu-baseline --steps 10 --warmup 3"; [ $C = resnet18 ] && A="$A --layout tensors --steps 30 --warmup 5"
  FA_XCD_MAP=$M timeout -k 10 300 python bench.py $A > gpurun_out/r02ao/b.json 2>gpurun_out/r02ao/b.err || { tail -3 gpurun_out/r02ao/b.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r02ao/b.json'));print('$C', 'xcd=$M', d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'], str(d['parity'])[:30])" | tee -a gpurun_out/r02ao/ab.txt
 done
done
