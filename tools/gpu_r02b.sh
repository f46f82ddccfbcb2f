# Round 2 session b: ingest/driver/e2e tests, the arrival latency bench, cfg2 layouts + variant sweep.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_ingest.py tests/test_gpu_e2e.py tests/test_gpu_drivers.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r02b.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_r02b.log; [ $rc -eq 0 ] || exit $rc
$T 300 python bench.py --config arrival --steps 10 --warmup 3 > gpurun_out/arrival.json 2> gpurun_out/arrival.err || { tail -20 gpurun_out/arrival.err; exit 1; }
cat gpurun_out/arrival.json
$T 300 python bench.py --config arrival --steps 10 --warmup 3 --arrival-gap-ms 5 --no-cpu-baseline > gpurun_out/arrival5.json 2> gpurun_out/arrival5.err || { tail -20 gpurun_out/arrival5.err; exit 1; }
cat gpurun_out/arrival5.json
for L in tiled arena tensors adopted; do
  $T 200 python bench.py --config resnet18 --layout $L --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/r18_$L.json 2> gpurun_out/r18_$L.err || { tail -20 gpurun_out/r18_$L.err; exit 1; }
  echo "layout=$L"; cat gpurun_out/r18_$L.json
done
for V in 1 2 4 5 6 7 8; do
  $T 200 python bench.py --config resnet18 --layout arena --variant $V --steps 50 --warmup 5 --no-cpu-baseline --check-samples 0 > gpurun_out/r18_v$V.json 2> gpurun_out/r18_v$V.err || { tail -20 gpurun_out/r18_v$V.err; exit 1; }
  echo "variant=$V $(python -c "import json;d=json.load(open('gpurun_out/r18_v$V.json'));print(d['value'],d['roofline']['kernel_avg_ms'])")"
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_r18 -o run -- python3 bench.py --config resnet18 --layout tiled --steps 20 --warmup 2 --no-cpu-baseline --check-samples 0 > gpurun_out/prof_r18.json 2> gpurun_out/prof_r18.err; rc=$?
echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
find /tmp/prof_r18 -name "*kernel_stats.csv" -exec cp {} gpurun_out/r02b_resnet18_tiled_kernel_stats.csv \;
head -5 gpurun_out/r02b_resnet18_tiled_kernel_stats.csv | cut -c1-200
