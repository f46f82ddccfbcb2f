# r05 final re-check after the last Gram-form changes (K in (32, 64] balanced 16x16 sets, knob
# cleanup): the whole GPU suite, smoke(), the default bench line, Krum K = 32 / 64 / 128 lines at the
# sustained clock, rocprof + PMC of the K = 64 kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05_final2; mkdir -p $O gpurun_out/summary
export TMPDIR=/tmp
fault() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
cat $O/bench_default.json
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1].split('/')[-1],d['value'],d['unit'],d['ms_per_step'],r.get('kernel_avg_ms'),r.get('bound'),r.get('frac'),d.get('parity'))" $1; }
for K in 32 64 128; do
  timeout -k 10 300 python bench.py --config krum --clients $K --steps 50 --warmup 150 --no-cpu-baseline --soak-seconds 0 --check-samples 1 > $O/krum$K.json 2> $O/krum$K.err || { tail -5 $O/krum$K.err; exit 1; }
  line $O/krum$K.json
done
BENCH_ARGS="--config krum --clients 64 --steps 5 --warmup 2 --no-cpu-baseline --check-samples 0 --soak-seconds 0" KERNEL=k_pair_gram timeout -k 10 900 bash tools/profile.sh r05f_krum64 > gpurun_out/summary/r05f_krum64.log 2>&1; rc=$?
echo "== krum64 rc=$rc"; grep -E '"kernel"|avg_ns|traffic_over' gpurun_out/summary/r05f_krum64.log
fault $rc && exit $rc
exit 0
