# r04c: the octet x quad Krum kernel (k_pairdist_oq): robust GPU tests (pairwise / Krum parity incl.
# g18 fixtures, bf16/f16/f64), then an interleaved A/B against the 4x4-tile kernels (FA_PAIR_OQ=0).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r04c; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_robust.py tests/test_gpu_pair.py -k "pairwise or krum or pair or staged" > $O/pytest.txt 2>&1 \
  || { echo "pytest FAIL"; tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
FA_PAIR_OQ_PF=0 timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_robust.py -k "pairwise" > $O/pytest_pf0.txt 2>&1 \
  || { echo "pytest PF0 FAIL"; tail -30 $O/pytest_pf0.txt; exit 1; }
tail -1 $O/pytest_pf0.txt
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1],d['value'],d['unit'],d['ms_per_step'],r.get('kernel_avg_ms'),'|',d.get('parity'))" $1; }
for rep in 1 2; do
  for K in 32 128 64 100 16; do
    for oq in 1p 1 0; do
      pf=1; [ "$oq" = "1" ] && pf=0
      n=krum_K${K}_oq${oq}_r$rep
      FA_PAIR_OQ=${oq%p} FA_PAIR_OQ_PF=$pf timeout -k 10 300 python bench.py --config krum --clients $K --steps 10 --warmup 3 --no-cpu-baseline > $O/$n.json 2> $O/$n.err \
        || { echo "FAIL $n"; tail -8 $O/$n.err; exit 1; }
      line $O/$n.json
    done
  done
done
for rep in 1 2 3; do
  for ru in 1 0; do
    n=cfg2_tensors_reuse${ru}_r$rep
    FA_STAGE_REUSE=$ru timeout -k 10 300 python bench.py --config resnet18 --layout tensors --steps 50 --warmup 10 --no-cpu-baseline > $O/$n.json 2> $O/$n.err \
      || { echo "FAIL $n"; tail -8 $O/$n.err; exit 1; }
    line $O/$n.json
  done
done
