# Round 2, first GPU session: new config/ingest tests, the existing distributed/tiled suites, the
# default bench, and the N > 1 bench path rehearsed on one GPU (gloo) for every collective.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T="timeout -k 10"
$T 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_ingest.py tests/test_gpu_distributed.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_r02a.log 2>&1
rc=$?; tail -30 gpurun_out/pytest_r02a.log; [ $rc -eq 0 ] || exit $rc
$T 400 python bench.py > gpurun_out/bench_r02a.json 2> gpurun_out/bench_r02a.err || { tail -20 gpurun_out/bench_r02a.err; exit 1; }
cat gpurun_out/bench_r02a.json
export FEDML_AMD_BENCH_REHEARSAL=1
for C in ordered ordered_all reduce_scatter reduce; do
  $T 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 2 --steps 3 --warmup 1 --params 12500000 --collective $C --no-cpu-baseline > gpurun_out/reh2_$C.json 2> gpurun_out/reh2_$C.err
  rc=$?; echo "N=2 collective=$C rc=$rc"; cat gpurun_out/reh2_$C.json; [ $rc -eq 0 ] || { tail -30 gpurun_out/reh2_$C.err; exit $rc; }
done
$T 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29534 \
  bench.py --gpus 4 --steps 3 --warmup 1 --params 12500000 --no-cpu-baseline > gpurun_out/reh4_ordered.json 2> gpurun_out/reh4_ordered.err
rc=$?; echo "N=4 ordered rc=$rc"; cat gpurun_out/reh4_ordered.json; [ $rc -eq 0 ] || { tail -30 gpurun_out/reh4_ordered.err; exit $rc; }
for CFG in hier gossip resnet18; do
  $T 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29535 \
    bench.py --gpus 2 --steps 2 --warmup 1 --config $CFG --no-cpu-baseline > gpurun_out/reh2_$CFG.json 2> gpurun_out/reh2_$CFG.err
  rc=$?; echo "N=2 config=$CFG rc=$rc"; cat gpurun_out/reh2_$CFG.json; [ $rc -eq 0 ] || { tail -30 gpurun_out/reh2_$CFG.err; exit $rc; }
done
