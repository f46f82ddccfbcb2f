# r04l: Krum K = 32 launch shapes of k_pairdist_lane with small workgroups (one / two waves, more
# workgroups) -- FA_PAIR_SPLIT (coordinate slices) x FA_PAIR_BLOCKS, 2 reps, default interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r04l; mkdir -p $O
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1],d['value'],d['unit'],d['ms_per_step'],r.get('kernel_avg_ms'),r.get('frac'),d.get('parity','')[:40])" $1; }
b() { timeout -k 10 300 python bench.py --config krum --clients ${K:-32} --steps 20 --warmup 3 --no-cpu-baseline --soak-seconds 0 > $O/$1.json 2> $O/$1.err || { echo "FAIL $1"; tail -8 $O/$1.err; exit 1; }; line $O/$1.json; }
for rep in 1 2; do
  b def_r$rep
  for cfg in "2 2048" "2 4096" "2 8192" "4 2048" "4 4096" "9 2048"; do
    set -- $cfg
    FA_PAIR_SPLIT=$1 FA_PAIR_BLOCKS=$2 b s$1_b$2_r$rep
  done
done
