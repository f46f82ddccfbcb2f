# descriptor tables staged on a side stream: full GPU suite, then A/B (FA_STAGE_SIDE=0/1) of the
# separate-tensors drop-in (cfg2) -- back-to-back GPU time per call and the bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r02al
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02al/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r02al/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r02al/gpu_tests.log
for M in 0 1 0 1; do
 FA_STAGE_SIDE=$M timeout -k 10 200 python tools/host_probe_b2b.py > gpurun_out/r02al/b2b_$M.json 2>/dev/null || { echo probe failed; exit 1; }
 FA_STAGE_SIDE=$M timeout -k 10 200 python bench.py --config resnet18 --layout tensors --no-cpu-baseline --steps 30 --warmup 5 > gpurun_out/r02al/t_$M.json 2>gpurun_out/r02al/t.err || { tail -3 gpurun_out/r02al/t.err; exit 1; }
 python -c "import json;b=json.load(open('gpurun_out/r02al/b2b_$M.json'));d=json.load(open('gpurun_out/r02al/t_$M.json'));print('side=$M', b.get('b2b_keep'), b.get('b2b_drop'), d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'], d['parity'][:30])" | tee -a gpurun_out/r02al/ab.txt
done
