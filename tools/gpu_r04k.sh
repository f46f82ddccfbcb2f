# r04k: k_pairdist_rot with software-pipelined differences (no s_nop, no shared DPP movs) -- probe
# (dpipe row), pair tests (default policy and FA_PAIR_ROT=1), Krum K = 32 / 16 rot vs tile (2 reps),
# and the cache-resident decomposition (FA_PAIR_ROT_DBG=1) of the rot kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r04k; mkdir -p $O
export TMPDIR=/tmp
hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize -o /tmp/dpp_rate_probe tools/dpp_rate_probe.hip 2>/dev/null || { echo "probe build FAIL"; exit 1; }
timeout -k 10 120 /tmp/dpp_rate_probe > $O/dpp_rate_probe.txt 2>&1 || { echo "probe FAIL"; cat $O/dpp_rate_probe.txt; exit 1; }
cat $O/dpp_rate_probe.txt
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_robust.py -k "pair or krum" > $O/pytest_def.txt 2>&1 \
  || { echo "pytest default FAIL"; tail -40 $O/pytest_def.txt; exit 1; }
tail -1 $O/pytest_def.txt
FA_PAIR_ROT=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_robust.py -k "pair or krum" > $O/pytest_rot1.txt 2>&1 \
  || { echo "pytest rot1 FAIL"; tail -40 $O/pytest_rot1.txt; exit 1; }
tail -1 $O/pytest_rot1.txt
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1],d['value'],d['unit'],d['ms_per_step'],r.get('kernel_avg_ms'),r.get('frac'))" $1; }
b() { timeout -k 10 300 python bench.py --config krum --clients ${K:-32} --steps 20 --warmup 3 --no-cpu-baseline --check-samples ${CS:-65536} > $O/$1.json 2> $O/$1.err || { echo "FAIL $1"; tail -8 $O/$1.err; exit 1; }; line $O/$1.json; }
for rep in 1 2; do
  for K in 32 16; do
    K=$K b K${K}_rot_r$rep
    K=$K FA_PAIR_ROT=0 b K${K}_tile_r$rep
  done
done
K=32 CS=0 FA_PAIR_ROT_DBG=1 b K32_cached
K=32 CS=0 FA_PAIR_ROT_P=3 b K32_P3
