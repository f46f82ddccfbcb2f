# r03aa: Krum launch-shape re-sweep after r03 (workgroups, LDS budget), interleaved x2, parity on.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
r() {  # label, K, env...
  local lab=$1 K=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --config krum --clients $K --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/k.json 2> gpurun_out/k.err || { echo FAIL $lab; tail -5 gpurun_out/k.err; exit 1; }
  L="$lab K=$K" python -c 'import json,os;d=json.load(open("gpurun_out/k.json"));print(os.environ["L"], d["value"], d["ms_per_step"], d["roofline"].get("kernel_avg_ms"), d.get("parity")[:40])'
}
for rep in 1 2; do
  r default 128 X=1
  r blocks256 128 FA_PAIR_BLOCKS=256
  r blocks512 128 FA_PAIR_BLOCKS=512
  r blocks2048 128 FA_PAIR_BLOCKS=2048
  r lds120 128 FA_PAIR_LDS_KB=120
  r default 32 X=1
  r blocks512 32 FA_PAIR_BLOCKS=512
  r blocks2048 32 FA_PAIR_BLOCKS=2048
  r npl8 32 FA_PAIR_NPL=8
done
