# host-time probe of the adopted drop-in path, the HBM read ceiling at cfg2's size, cfg2 adopted bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_promotion.py tests/test_gpu_ingest.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r02c.log 2>&1; rc=$?; tail -8 gpurun_out/pytest_r02c.log; [ $rc -eq 0 ] || exit $rc
$T 120 python tools/host_probe_adopted.py > gpurun_out/host_probe_adopted.json 2> gpurun_out/host_probe.err || { tail gpurun_out/host_probe.err; exit 1; }
cat gpurun_out/host_probe_adopted.json
PROBE_BIG=0 $T 200 python tools/hbm_probe.py 1.44 > gpurun_out/hbm_1p44.json 2> gpurun_out/hbm.err || { tail gpurun_out/hbm.err; exit 1; }
cat gpurun_out/hbm_1p44.json
for L in adopted arena tiled; do
  $T 200 python bench.py --config resnet18 --layout $L --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/r18c_$L.json 2> gpurun_out/r18c_$L.err || { tail -20 gpurun_out/r18c_$L.err; exit 1; }
  echo "layout=$L $(python -c "import json;d=json.load(open('gpurun_out/r18c_$L.json'));print(d['value'],d['ms_per_step'],d['roofline']['kernel_avg_ms'],d['parity'])")"
done
