# r04a: device visibility probe; the loopback ordered exchange (-m gpu, distributed + ingest + finite);
# the self-launched one-rank chain with the loopback exchange; the default bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04a
bash tools/probe_dev.sh > gpurun_out/r04a/probe_dev.txt 2>&1
python -c "import bench; print('visible_gpu_count', bench.visible_gpu_count())" >> gpurun_out/r04a/probe_dev.txt 2>&1
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_distributed.py tests/test_gpu_ingest.py tests/test_gpu_finite.py tests/test_gpu_robust.py > gpurun_out/r04a/pytest.txt 2>&1 \
  || { echo "pytest FAIL"; tail -30 gpurun_out/r04a/pytest.txt; exit 1; }
tail -3 gpurun_out/r04a/pytest.txt
timeout -k 10 300 python bench.py --gpus 1 --self-launch --loopback --steps 10 --warmup 3 \
  > gpurun_out/r04a/selflaunch_loopback.json 2> gpurun_out/r04a/selflaunch_loopback.err \
  || { echo "self-launch FAIL"; tail -20 gpurun_out/r04a/selflaunch_loopback.err; exit 1; }
cat gpurun_out/r04a/selflaunch_loopback.json
timeout -k 10 300 python bench.py --gpus 1 --self-launch --loopback --collective ordered_all --config hier --steps 5 --warmup 2 \
  > gpurun_out/r04a/selflaunch_loopback_hier.json 2> gpurun_out/r04a/selflaunch_loopback_hier.err \
  || { echo "self-launch hier FAIL"; tail -20 gpurun_out/r04a/selflaunch_loopback_hier.err; exit 1; }
cat gpurun_out/r04a/selflaunch_loopback_hier.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r04a/bench_default.json 2> gpurun_out/r04a/bench_default.err \
  || { echo "bench FAIL"; tail -20 gpurun_out/r04a/bench_default.err; exit 1; }
cat gpurun_out/r04a/bench_default.json
for rep in 1 2; do
  for lay in tiled arena; do
    for K in 32 128; do
      timeout -k 10 300 python bench.py --config median --clients $K --layout $lay --steps 20 --warmup 3 --no-cpu-baseline \
        > gpurun_out/r04a/median_${lay}_K${K}_r${rep}.json 2> gpurun_out/r04a/median_${lay}_K${K}_r${rep}.err \
        || { echo "median FAIL"; tail -20 gpurun_out/r04a/median_${lay}_K${K}_r${rep}.err; exit 1; }
      python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d['roofline'];print(sys.argv[1],d['value'],r['kernel_avg_ms'],r['frac'],d['parity'])" gpurun_out/r04a/median_${lay}_K${K}_r${rep}.json
    done
  done
done
