# half-precision Krum (fa_pairwise_sqdist_rt): robust GPU tests + fp32 Krum timing unchanged
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r02u
timeout -k 10 600 python -u -m pytest tests/test_gpu_robust.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02u/robust.log 2>&1 || { tail -40 gpurun_out/r02u/robust.log; exit 1; }
tail -1 gpurun_out/r02u/robust.log
for K in 32 128; do
timeout -k 10 200 python bench.py --config krum --clients $K --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/r02u/krum_K$K.json 2>gpurun_out/r02u/krum_K$K.err || { tail -3 gpurun_out/r02u/krum_K$K.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r02u/krum_K$K.json'));print($K, d['roofline']['kernel_avg_ms'], d['parity'])"
done
