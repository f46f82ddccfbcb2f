# r03p: SecAgg jump-ahead (even/odd b64 jump kernel, vector plane fold): parity, chunk-size A/B, kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_finite.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_p.log 2>&1 || { tail -30 gpurun_out/pytest_p.log; exit 1; }
tail -1 gpurun_out/pytest_p.log
for rep in 1 2; do
  for L in def 7 9; do
    if [ $L = def ]; then unset FA_MT_JUMP_LOG2; else export FA_MT_JUMP_LOG2=$L; fi
    timeout -k 10 300 python bench.py --config samask --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/sa_$L.json 2> gpurun_out/sa_$L.err || { tail -5 gpurun_out/sa_$L.err; exit 1; }
    L=$L python -c 'import json,os;d=json.load(open("gpurun_out/sa_%s.json" % os.environ["L"]));print("log2", os.environ["L"], d["value"], d["unit"], d.get("parity"))'
  done
done
unset FA_MT_JUMP_LOG2
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sa -o sa -- python bench.py --config samask --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/sa_prof.json 2> gpurun_out/sa_prof.err || { tail -5 gpurun_out/sa_prof.err; exit 1; }
timeout -k 10 300 python bench.py --config samask --variant 4 --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/sa_d4.json 2> gpurun_out/sa_d4.err || { tail -5 gpurun_out/sa_d4.err; exit 1; }
python -c 'import json;d=json.load(open("gpurun_out/sa_d4.json"));print("dropped4", d["value"], d["unit"], d.get("parity"))'
