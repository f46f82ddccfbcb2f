# r04w: Krum tile loops unrolled 4 with the shuffle-broadcast pair_tile (libfedagg_u4.so) vs the
# round-end kernels (libfedagg_base.so): pair tests on u4, then 3 interleaved pairs at K = 128 / 32.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r04w; mkdir -p $O
use() { cp fedml_amd/libfedagg_$1.so fedml_amd/libfedagg.so; }
use u4
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_robust.py -k "pair or krum" > $O/pytest_u4.txt 2>&1 \
  || { echo "pytest u4 FAIL"; tail -40 $O/pytest_u4.txt; exit 1; }
tail -1 $O/pytest_u4.txt
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1],d['value'],d['unit'],d['ms_per_step'],r.get('kernel_avg_ms'),r.get('frac'),'|',(d.get('parity') or '')[:40])" $1; }
b() { timeout -k 10 200 python bench.py --config krum --clients $K --steps 20 --warmup 3 --no-cpu-baseline --soak-seconds 0 > $O/$1.json 2> $O/$1.err || { echo "FAIL $1"; tail -8 $O/$1.err; exit 1; }; line $O/$1.json; }
for rep in 1 2 3; do
  for K in 128 32; do
    use base; K=$K b K${K}_base_r$rep
    use u4; K=$K b K${K}_u4_r$rep
  done
done
use base
