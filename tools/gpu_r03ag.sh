# r03ag: fragmented metric (204 tensors / client, 26,112 allocations) -- kernel variant sweep (tile
# depth S = 1 / 2 / 4, U clients per step), interleaved, 2 reps; a TLB-reach hypothesis (bigger tiles
# per client per workgroup = fewer translations per byte).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for rep in 1 2; do
  for V in 0 5 4 6 1; do
    timeout -k 10 300 python bench.py --config fragmented --variant $V --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/f.json 2>gpurun_out/f.err || { echo FAIL $V; tail -5 gpurun_out/f.err; exit 1; }
    V=$V python -c 'import json,os;d=json.load(open("gpurun_out/f.json"));print("rep variant", os.environ["V"], d["ms_per_step"], d["value"], d["roofline"]["frac"], d.get("parity"))'
  done
done
