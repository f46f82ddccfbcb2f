# r03w: SecAgg jump split into half-range workgroups: parity, bench x3, kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_finite.py -m gpu -x -q -k "mt_ or secagg" --timeout 200 --timeout-method thread > gpurun_out/pytest_w.log 2>&1 || { tail -30 gpurun_out/pytest_w.log; exit 1; }
tail -1 gpurun_out/pytest_w.log
for rep in 1 2 3; do
  timeout -k 10 300 python bench.py --config samask --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/sa.json 2> gpurun_out/sa.err || { tail -5 gpurun_out/sa.err; exit 1; }
  python -c 'import json;d=json.load(open("gpurun_out/sa.json"));print("samask", d["value"], d["unit"], d.get("parity"))'
done
timeout -k 10 300 python bench.py --config samask --variant 4 --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/sa_d4.json 2> gpurun_out/sa_d4.err || { tail -5 gpurun_out/sa_d4.err; exit 1; }
python -c 'import json;d=json.load(open("gpurun_out/sa_d4.json"));print("dropped4", d["value"], d["unit"], d.get("parity"))'
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sa -o sa -- python bench.py --config samask --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/sa_prof.json 2> gpurun_out/sa_prof.err || { tail -5 gpurun_out/sa_prof.err; exit 1; }
