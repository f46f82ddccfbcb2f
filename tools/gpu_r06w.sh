# r06w: the bf16x3 Gram kernels issuing the next chunk's loads vector by vector during the split
# (unconditional loads, the row mask applied at use) -- band / robust tests, then interleaved A/B
# against HEAD bc9fcea (fedml_amd/ab/libfedagg_prev.so) at K = 128 / 96 / 64, 3 pairs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06w; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_krum_band.py tests/test_gpu_robust.py > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc = 0 ] || exit $rc
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1].split('/')[-1],d['value'],d['ms_per_step'],r.get('kernel_avg_ms'),d.get('pair_form'),str(d.get('parity'))[:60])" $1; }
for K in 128 96 64; do
  for i in 1 2 3; do
    for v in prev new; do
      if [ $v = prev ]; then export FEDML_AMD_LIB=$PWD/fedml_amd/ab/libfedagg_prev.so; else unset FEDML_AMD_LIB; fi
      timeout -k 10 300 python bench.py --config krum --clients $K --no-cpu-baseline --soak-seconds 0 --cold-reps 0 $([ $i = 1 ] || echo --check-samples 0) > $O/krum${K}_${v}_$i.json 2> $O/krum${K}_${v}_$i.err || { tail -5 $O/krum${K}_${v}_$i.err; exit 1; }
      line $O/krum${K}_${v}_$i.json
    done
  done
done
unset FEDML_AMD_LIB
exit 0
