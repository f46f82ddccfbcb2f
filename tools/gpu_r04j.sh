# r04j: is k_pairdist_rot (K = 32 / 16) memory- or VALU-bound?  FA_PAIR_ROT_DBG=1: every load re-reads
# the replica's first unit (cache-resident, full pair math); =2: all loads, no pair math.  Then the
# effective clock of the normal kernel (GRBM_GUI_ACTIVE / 8 / kernel time, MI355X_MICROARCH.md DVFS).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r04j; mkdir -p $O
export TMPDIR=/tmp
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1],d['value'],d['unit'],d['ms_per_step'],r.get('kernel_avg_ms'),r.get('frac'))" $1; }
b() { timeout -k 10 300 python bench.py --config krum --clients ${K:-32} --steps 20 --warmup 3 --no-cpu-baseline --check-samples 0 > $O/$1.json 2> $O/$1.err || { echo "FAIL $1"; tail -8 $O/$1.err; exit 1; }; line $O/$1.json; }
for K in 32 16; do
  K=$K b K${K}_normal
  K=$K FA_PAIR_ROT_DBG=1 b K${K}_cached
  K=$K FA_PAIR_ROT_DBG=2 b K${K}_nomath
  K=$K FA_PAIR_ROT=0 b K${K}_tile
done
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex k_pairdist -d $O/clk -o clk --output-format csv -- python3 bench.py --config krum --clients 32 --no-cpu-baseline --check-samples 0 --steps 10 --warmup 2 > $O/clk.log 2>&1 || { echo "FAIL clk"; tail -5 $O/clk.log; exit 1; }
find $O/clk -name "*.csv" | head
