# r05i: Gram-form Krum -- the product default (FEDML_AMD_KRUM_FORM unset: Gram + device-guarded direct
# fallback), and the workgroup count for K = 32 / 128 (FA_GRAM_BLOCKS), 2 interleaved reps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05i; mkdir -p $O
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1],d['value'],d['ms_per_step'],r.get('kernel_avg_ms'),d.get('pair_form'),d.get('kappa_max'),d.get('parity'))" $1; }
B="--config krum --no-cpu-baseline --soak-seconds 0 --steps 20 --warmup 3"
for rep in 1 2; do
  for K in 32 128; do
    for nb in default 512 2048; do
      n=K${K}_nb${nb}_$rep
      if [ $nb = default ]; then E=""; else E="FA_GRAM_BLOCKS=$nb"; fi
      env $E timeout -k 10 300 python bench.py $B --clients $K --check-samples $([ $rep = 1 ] && echo 1 || echo 0) > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
      line $O/$n.json
    done
  done
done
