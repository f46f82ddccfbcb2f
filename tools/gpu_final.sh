# Round-end evidence: GPU tests, smoke, default bench (CPU baseline), rocprof stats + PMC for the changed configs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
NOPROF=1 TAG=${ROUND:-r01h} bash tools/gpu_session.sh || exit 1
ROUND=${ROUND:-r01h} CONFIGS="${CONFIGS:-metric resnet18 vit_bf16}" bash tools/gpu_profiles.sh
