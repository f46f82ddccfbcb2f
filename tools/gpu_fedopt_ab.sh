# GPU tests + inline-vs-staged tables A/B on the fedopt config (interleaved).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for rep in 1 2; do
  for f in 1 0; do
    for c in ${CONFIGS:-fedopt}; do
      FA_INLINE_DESC=$f timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab_${c}_$f.json 2> gpurun_out/ab_${c}_$f.err || { tail -5 gpurun_out/ab_${c}_$f.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/ab_${c}_$f.json'));print('rep $rep inline=$f $c',d['value'],d['ms_per_step'],d['roofline'].get('kernel_avg_ms'),d.get('parity'))"
    done
  done
done
