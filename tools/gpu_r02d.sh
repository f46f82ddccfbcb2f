# cfg1 latency (host / tensors / adopted), all drop-in GPU tests, cfg2 adopted under rocprof, HBM probe at cfg2 size
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_drivers.py tests/test_gpu_e2e.py tests/test_gpu_ingest.py tests/test_promotion.py tests/test_gpu_pair.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r02d.log 2>&1; rc=$?; tail -8 gpurun_out/pytest_r02d.log; [ $rc -eq 0 ] || exit $rc
for L in host tensors adopted; do
  $T 200 python bench.py --config lr --layout $( [ $L = host ] && echo tiled || echo $L ) --steps 2000 --warmup 200 > gpurun_out/lr_$L.json 2> gpurun_out/lr_$L.err || { tail -20 gpurun_out/lr_$L.err; exit 1; }
  cat gpurun_out/lr_$L.json
done
PROBE_BIG=0 $T 200 python tools/hbm_probe.py 1.44 > gpurun_out/hbm_1p44b.json 2> gpurun_out/hbm.err || { tail gpurun_out/hbm.err; exit 1; }
cat gpurun_out/hbm_1p44b.json
export TMPDIR=/tmp
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_r18a -o run -- python3 bench.py --config resnet18 --layout adopted --steps 30 --warmup 3 --no-cpu-baseline --check-samples 0 > gpurun_out/prof_r18a.json 2> gpurun_out/prof_r18a.err; rc=$?
echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
find /tmp/prof_r18a -name "*kernel_stats.csv" -exec cp {} gpurun_out/r02d_resnet18_adopted_kernel_stats.csv \;
grep -E "wsum" gpurun_out/r02d_resnet18_adopted_kernel_stats.csv | cut -c1-250
