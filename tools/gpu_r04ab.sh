# r04ab: ragged last tile first + unrolled scalar tails (libfedagg_new.so) vs the previous kernels
# (libfedagg_base.so): metric 3 interleaved pairs, hier (11.70 M) and cfg2 2 pairs each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r04ab; mkdir -p $O
use() { cp fedml_amd/libfedagg_$1.so fedml_amd/libfedagg.so; }
use new
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_tiled.py tests/test_gpu_configs.py tests/test_gpu_distributed.py > $O/pytest_new.txt 2>&1 \
  || { echo "pytest new FAIL"; tail -40 $O/pytest_new.txt; exit 1; }
tail -1 $O/pytest_new.txt
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1],d['value'],d['unit'],d['ms_per_step'],r.get('kernel_avg_ms'),r.get('frac'),'|',(d.get('parity') or '')[:30])" $1; }
b() { n=$1; shift; timeout -k 10 300 python bench.py "$@" --steps 20 --warmup 3 --no-cpu-baseline --soak-seconds 0 > $O/$n.json 2> $O/$n.err || { echo "FAIL $n"; tail -8 $O/$n.err; exit 1; }; line $O/$n.json; }
for rep in 1 2 3; do
  for v in base new; do use $v; b metric_${v}_r$rep; done
done
for rep in 1 2; do
  for v in base new; do use $v; b hier_${v}_r$rep --config hier; b resnet18_${v}_r$rep --config resnet18; done
done
use new
