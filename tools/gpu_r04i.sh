# r04i: k_pairdist_rot SMALL (K <= 32: both groups per wave, P units in flight) -- pair tests on the
# default policy (rot at K <= 32) and with FA_PAIR_ROT=1 (rot at every K), then Krum K = 32 over
# P = 2 / 3 / 4 and replicas R = 4 / 5 / 8 against the tile kernel (interleaved), SQ counters of the best.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r04i; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_robust.py -k "pair or krum" > $O/pytest_def.txt 2>&1 \
  || { echo "pytest default FAIL"; tail -40 $O/pytest_def.txt; exit 1; }
tail -1 $O/pytest_def.txt
FA_PAIR_ROT=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_robust.py -k "pair or krum" > $O/pytest_rot1.txt 2>&1 \
  || { echo "pytest rot1 FAIL"; tail -40 $O/pytest_rot1.txt; exit 1; }
tail -1 $O/pytest_rot1.txt
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1],d['value'],d['unit'],d['ms_per_step'],r.get('kernel_avg_ms'),r.get('frac'))" $1; }
b() { timeout -k 10 300 python bench.py --config krum --clients ${K:-32} --steps 20 --warmup 3 --no-cpu-baseline --check-samples 0 > $O/$1.json 2> $O/$1.err || { echo "FAIL $1"; tail -8 $O/$1.err; exit 1; }; line $O/$1.json; }
for rep in 1 2; do
  FA_PAIR_ROT=0 b tile_r$rep
  for P in 2 3 4; do
    for R in 4 5 8; do
      FA_PAIR_ROT_P=$P FA_PAIR_ROT_R=$R b rot_P${P}_R${R}_r$rep
    done
  done
done
K=16 b k16_rot; K=16 FA_PAIR_ROT=0 b k16_tile
CC="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC"
CD="SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_WAVES SQ_INSTS_SMEM SQ_WAIT_INST_LDS"
for p in C D; do
  [ $p = C ] && CN="$CC" || CN="$CD"
  timeout -s KILL 120 rocprofv3 --pmc $CN --kernel-include-regex k_pairdist_rot -d $O/pmc_32_$p -o pmc --output-format csv -- python3 bench.py --config krum --clients 32 --no-cpu-baseline --check-samples 0 --steps 3 --warmup 1 > $O/pmc_32_$p.log 2>&1 \
    || { echo "FAIL pmc $p"; tail -5 $O/pmc_32_$p.log; exit 1; }
  f=$(find $O/pmc_32_$p -name "*counter_collection.csv" | head -1)
  python3 tools/pmc_sq.py $f | tee $O/pmc_32_$p.txt
done
