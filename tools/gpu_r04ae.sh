# r04ae: median networks with a 60-comparator 16-key block (tools/gen_median_nets.py; libfedagg_new.so)
# vs the Batcher-only networks (libfedagg_base.so = ba897a2): median GPU tests on new, 3 interleaved
# pairs of median K = 32 / 64 / 128 on the tiled arena, then the round-end evidence (tools/gpu_r04ad.sh)
# on the base library.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r04ae; mkdir -p $O
use() { cp fedml_amd/libfedagg_$1.so fedml_amd/libfedagg.so; }
use new
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -k "median" > $O/pytest_new.txt 2>&1 \
  || { echo "pytest new FAIL"; tail -40 $O/pytest_new.txt; exit 1; }
tail -1 $O/pytest_new.txt
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1],d['value'],d['unit'],d['ms_per_step'],r.get('kernel_avg_ms'),r.get('frac'),'|',(d.get('parity') or '')[:30])" $1; }
b() { n=$1; shift; timeout -k 10 300 python bench.py "$@" --steps 20 --warmup 3 --no-cpu-baseline --soak-seconds 0 > $O/$n.json 2> $O/$n.err || { echo "FAIL $n"; tail -8 $O/$n.err; exit 1; }; line $O/$n.json; }
for rep in 1 2 3; do
  for v in base new; do use $v
    for k in 32 64 128; do b med${k}_${v}_r$rep --config median --clients $k --layout tiled; done
  done
done
use base
[ -z "$EVIDENCE" ] || CONFIGS="metric hier gossip" bash tools/gpu_r04ad.sh
