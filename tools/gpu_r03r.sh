# r03r: banded gossip variants (FA_BAND_VAR 0-4, interleaved x2) with parity, SecAgg dropped-4 after the group-size fix.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for rep in 1 2; do
  for v in 0 1 2 3 4; do
    FA_BAND_VAR=$v timeout -k 10 300 python bench.py --config gossip --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/g_$v.json 2> gpurun_out/g_$v.err || { tail -5 gpurun_out/g_$v.err; exit 1; }
    V=$v python -c 'import json,os;d=json.load(open("gpurun_out/g_%s.json" % os.environ["V"]));print("band", os.environ["V"], d["value"], d["ms_per_step"], d["roofline"].get("kernel_avg_ms"), d.get("parity"))'
  done
done
timeout -k 10 300 python bench.py --config samask --variant 4 --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/sa_d4.json 2> gpurun_out/sa_d4.err || { tail -5 gpurun_out/sa_d4.err; exit 1; }
python -c 'import json;d=json.load(open("gpurun_out/sa_d4.json"));print("dropped4", d["value"], d["unit"], d.get("parity"))'
