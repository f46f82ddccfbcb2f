# r04s: k_pairdist_ring (loader waves + 4-slot LDS ring, counters instead of a barrier per chunk;
# FA_PAIR_RING=1, kp > 32) -- pair / Krum GPU tests with the ring, then K = 128 / 64 / 100 ring vs
# k_pairdist, 2 interleaved reps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r04s; mkdir -p $O
FA_PAIR_RING=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_robust.py -k "pair or krum" > $O/pytest_ring.txt 2>&1 \
  || { echo "pytest ring FAIL"; tail -40 $O/pytest_ring.txt; exit 1; }
tail -1 $O/pytest_ring.txt
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1],d['value'],d['unit'],d['ms_per_step'],r.get('kernel_avg_ms'),r.get('frac'),'|',d.get('parity','')[:40])" $1; }
b() { timeout -k 10 200 python bench.py --config krum --clients ${K:-128} --steps 10 --warmup 3 --no-cpu-baseline --soak-seconds 0 > $O/$1.json 2> $O/$1.err || { echo "FAIL $1"; tail -8 $O/$1.err; exit 1; }; line $O/$1.json; }
for rep in 1 2; do
  for K in 128 64 100; do
    K=$K FA_PAIR_RING=1 b K${K}_ring_r$rep
    K=$K b K${K}_tile_r$rep
  done
done
