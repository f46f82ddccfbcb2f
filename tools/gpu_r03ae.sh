# r03ae: read-pattern probe for the median kernels (tools/median_access_probe.hip): K rows streamed
# with 4-byte vs 16-byte loads per lane, K = 32 / 64 / 128, 11.69 M coordinates.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o gpurun_out/median_access_probe tools/median_access_probe.hip 2>/dev/null || exit 1
timeout -k 10 120 gpurun_out/median_access_probe | tee gpurun_out/median_access_probe.json
