# r04ad: round-end evidence on the final code (after the ragged-tile-first change in the weighted
# sums and mixing kernels): GPU parity suite + smoke + default bench, every config line once, and
# rocprof trace + FETCH/WRITE passes for the configs whose kernels changed.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
NOPROF=1 TAG=r04ad bash tools/gpu_session.sh || exit 1
mkdir -p gpurun_out/r04ad && cp gpurun_out/pytest_gpu.log gpurun_out/smoke.log gpurun_out/bench_default.json gpurun_out/r04ad/
sed -e 's#O=gpurun_out/r04v#O=gpurun_out/r04ad#' tools/gpu_r04v.sh > /tmp/r04ad_configs.sh
bash /tmp/r04ad_configs.sh || exit 1
ROUND=r04ad CONFIGS="${CONFIGS:-metric resnet18 hier gossip}" bash tools/gpu_profiles.sh
