# r06f: round-end checks on one box with the final binary: the whole -m gpu suite, smoke(), the
# default bench line (as the driver runs it), its rocprofv3 kernel trace and FETCH_SIZE / WRITE_SIZE
# passes (tools/profile.sh), and the metric kernel's translation / clock counters.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06f; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -5 $O/bench_default.err; exit 1; }
python -c "import json;d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1]);r=d['roofline'];print(d['value'],d['ms_per_step'],r['kernel_avg_ms'],r['frac'],r.get('frac_of_ceiling'),r['measured_read_ceiling']['value'],d['cold']['ms'],d['parity'])"
timeout -k 10 900 bash tools/profile.sh r06f > $O/profile.log 2>&1 || { tail -5 $O/profile.log; exit 1; }
tail -3 $O/profile.log
C1="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE"
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $C1 --kernel-include-regex 'k_wsum|k_read_probe' -d $O/pmc1 -o pmc --output-format csv -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --check-samples 0 --soak-seconds 0 --cold-reps 0 > $O/pmc1.log 2>&1 \
  || { echo "FAIL pmc1"; tail -5 $O/pmc1.log; exit 1; }
tail -1 $O/pmc1.log | cut -c1-200
exit 0
