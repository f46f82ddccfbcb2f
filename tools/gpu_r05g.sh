# r05g: the Gram-form Krum distances (fa_pairwise_sqdist_gram, f32 MFMA) -- robust GPU tests, then
# interleaved A/B against the direct kernel (FEDML_AMD_KRUM_FORM=direct) at K = 32 / 128 / 64 / 100,
# and a kernel trace of the Gram form.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05g; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_robust.py -x -q --timeout 120 --timeout-method thread -k "pairwise or krum" > $O/pytest_krum.log 2>&1 || { tail -40 $O/pytest_krum.log; exit 1; }
tail -2 $O/pytest_krum.log
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1],d['value'],d['ms_per_step'],r.get('kernel_avg_ms'),d.get('pair_form'),d.get('kappa_max'),d.get('parity'))" $1; }
B="--config krum --no-cpu-baseline --soak-seconds 0 --steps 20 --warmup 3"
for rep in 1 2; do
  for K in 32 128 64 100; do
    for f in gram direct; do
      n=K${K}_${f}_$rep
      FEDML_AMD_KRUM_FORM=$f timeout -k 10 300 python bench.py $B --clients $K --check-samples $([ $rep = 1 ] && echo 1 || echo 0) > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
      line $O/$n.json
    done
  done
done
for K in 32 128; do
  FEDML_AMD_KRUM_FORM=gram timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_K$K -o run -- python3 bench.py $B --clients $K --check-samples 0 > $O/trace_K$K.log 2>&1 || { tail -5 $O/trace_K$K.log; exit 1; }
done
find $O -name "*kernel_stats.csv" | head
