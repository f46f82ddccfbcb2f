# r06ac: the final binary (after f2f1cd2, the arena placement check) -- rocprofv3 trace + FETCH_SIZE + WRITE_SIZE passes of the default metric
# line (tools/profile.sh), the whole -m gpu suite, smoke(), the driver's own `python bench.py` twice,
# and the one-GPU RCCL rank chain (--self-launch --loopback).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06ac; mkdir -p $O
export TMPDIR=/tmp
bash tools/profile.sh r06ac_metric > $O/profile.log 2>&1 || { tail -5 $O/profile.log; exit 1; }
tail -12 $O/profile.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};c=d.get('cold') or {};print(sys.argv[1].split('/')[-1],d['value'],d['ms_per_step'],r.get('kernel_avg_ms'),r.get('frac'),r.get('frac_of_ceiling'),'cold',c.get('ms'),d['config'].get('arena_alloc'),(d.get('cpu_baseline') or {}).get('value'),str(d.get('parity'))[:50])" $1; }
for i in 1 2; do
  timeout -k 10 400 python bench.py > $O/default_$i.json 2> $O/default_$i.err || { tail -5 $O/default_$i.err; exit 1; }
  line $O/default_$i.json
done
timeout -k 10 400 python bench.py --gpus 1 --self-launch --loopback --cold-reps 0 --no-cpu-baseline > $O/loopback.json 2> $O/loopback.err || { tail -5 $O/loopback.err; exit 1; }
line $O/loopback.json
exit 0
