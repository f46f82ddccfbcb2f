# r03z: SecAgg two-part pipeline (FA_MT_PIPE 1/0, interleaved x3) with parity tests, 152-stream line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_finite.py -m gpu -x -q -k "mt_ or secagg" --timeout 200 --timeout-method thread > gpurun_out/pytest_z.log 2>&1 || { tail -30 gpurun_out/pytest_z.log; exit 1; }
tail -1 gpurun_out/pytest_z.log
for rep in 1 2 3; do
  for pp in 1 0; do
    FA_MT_PIPE=$pp timeout -k 10 300 python bench.py --config samask --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/sa.json 2> gpurun_out/sa.err || { tail -5 gpurun_out/sa.err; exit 1; }
    PP=$pp python -c 'import json,os;d=json.load(open("gpurun_out/sa.json"));print("pipe", os.environ["PP"], d["value"], d["unit"], d.get("parity"))'
  done
done
timeout -k 10 300 python bench.py --config samask --variant 4 --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/sa_d4.json 2> gpurun_out/sa_d4.err || { tail -5 gpurun_out/sa_d4.err; exit 1; }
python -c 'import json;d=json.load(open("gpurun_out/sa_d4.json"));print("dropped4", d["value"], d["unit"], d.get("parity"))'
