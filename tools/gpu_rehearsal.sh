# Rehearse bench.py's N > 1 path on ONE GPU: NPROC ranks on device 0 over gloo (not a measurement).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export FEDML_AMD_BENCH_REHEARSAL=1
for C in ${COLLS:-reduce_scatter reduce}; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node ${NPROC:-2} --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus ${NPROC:-2} --steps 3 --warmup 1 --params ${P:-12500000} --collective $C > gpurun_out/reh_$C.json 2> gpurun_out/reh_$C.err
  echo "collective=$C rc=$?"; cat gpurun_out/reh_$C.json
done
