# r03o: SecAgg jump-ahead parity + A/B (FA_MT_JUMP=1/0) + kernel trace; host1 multi-workgroup parity + cfg1 latency.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_finite.py tests/test_gpu_host_small.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_o.log 2>&1 || { tail -30 gpurun_out/pytest_o.log; exit 1; }
tail -1 gpurun_out/pytest_o.log
for rep in 1 2; do
  for f in 1 0; do
    FA_MT_JUMP=$f timeout -k 10 300 python bench.py --config samask --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/sa_$f.json 2> gpurun_out/sa_$f.err || { tail -5 gpurun_out/sa_$f.err; exit 1; }
    F=$f python -c 'import json,os;d=json.load(open("gpurun_out/sa_%s.json" % os.environ["F"]));print("mtjump", os.environ["F"], d["value"], d["unit"], d.get("parity"))'
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sa -o sa -- python bench.py --config samask --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/sa_prof.json 2> gpurun_out/sa_prof.err || { tail -5 gpurun_out/sa_prof.err; exit 1; }
find gpurun_out/prof_sa -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/sa_kernel_stats.csv
head -12 gpurun_out/sa_kernel_stats.csv
for rep in 1 2; do
  timeout -k 10 200 python bench.py --config lr --steps 3000 --warmup 200 $( [ $rep = 1 ] || echo --no-cpu-baseline ) > gpurun_out/lr_$rep.json 2> gpurun_out/lr_$rep.err || { tail -5 gpurun_out/lr_$rep.err; exit 1; }
  R=$rep python -c 'import json,os;d=json.load(open("gpurun_out/lr_%s.json" % os.environ["R"]));print("lr", d["value"], d["unit"], d.get("parity"), (d.get("cpu_baseline") or {}).get("value"))'
done
