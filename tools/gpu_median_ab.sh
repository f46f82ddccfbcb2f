# Robust GPU tests, then the fp32 median two-per-lane kernel A/B (FA_MEDIAN_X2=1/0) at K = 8 / 16 / 32.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_robust.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_robust.log 2>&1 || { tail -30 gpurun_out/pytest_robust.log; exit 1; }
tail -2 gpurun_out/pytest_robust.log
for rep in 1 2; do
  for k in 8 16 32; do
    for f in 1 0; do
      FA_MEDIAN_X2=$f timeout -k 10 300 python bench.py --config median --clients $k --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/med_${k}_$f.json 2> gpurun_out/med_${k}_$f.err || { tail -5 gpurun_out/med_${k}_$f.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/med_${k}_$f.json'));print('rep $rep K=$k x2=$f',d['value'],d['ms_per_step'],d['roofline'].get('kernel_avg_ms'),d.get('parity'))"
    done
  done
done
