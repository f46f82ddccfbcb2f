# r04f: k_pairdist_rot (DPP row-rotation pair kernel, pairrot.hip) -- parity of the robust / pairwise
# GPU tests on the rot path (default) and the tile path (FA_PAIR_ROT=0), then interleaved A/B of the
# Krum bench at K = 32 / 64 / 128 (3 pairs at 32 and 128), rocprof kernel stats of both at K = 32 / 128.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r04f; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_robust.py tests/test_gpu_pair.py -k "pair or krum" > $O/pytest_rot.txt 2>&1 \
  || { echo "pytest rot FAIL"; tail -40 $O/pytest_rot.txt; exit 1; }
tail -1 $O/pytest_rot.txt
FA_PAIR_ROT=0 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_robust.py tests/test_gpu_pair.py -k "pair or krum" > $O/pytest_tile.txt 2>&1 \
  || { echo "pytest tile FAIL"; tail -30 $O/pytest_tile.txt; exit 1; }
tail -1 $O/pytest_tile.txt
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1],d['value'],d['unit'],d['ms_per_step'],r.get('kernel_avg_ms'),r.get('frac'),'|',d.get('parity'))" $1; }
for rep in 1 2 3; do
  for K in 32 128 64; do
    [ $K = 64 ] && [ $rep != 1 ] && continue
    for v in 1 0; do
      n=krum_K${K}_rot${v}_r$rep
      FA_PAIR_ROT=$v timeout -k 10 300 python bench.py --config krum --clients $K --steps 20 --warmup 3 --no-cpu-baseline > $O/$n.json 2> $O/$n.err \
        || { echo "FAIL $n"; tail -8 $O/$n.err; exit 1; }
      line $O/$n.json
    done
  done
done
for K in 32 128; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/rp_$K -o run -- python3 bench.py --config krum --clients $K --steps 10 --warmup 2 --no-cpu-baseline > $O/rp_K$K.json 2> $O/rp_K$K.err \
    || { echo "rocprof FAIL $K"; tail -5 $O/rp_K$K.err; exit 1; }
  find /tmp/rp_$K -name "*kernel_stats.csv" -exec cp {} $O/krum_K${K}_rot_kernel_stats.csv \;
  head -4 $O/krum_K${K}_rot_kernel_stats.csv
done
