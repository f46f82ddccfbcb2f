# r03al: packed float16 IEEE minimum / maximum probe (tools/pk_minimum_probe.hip).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o gpurun_out/pk_minimum_probe tools/pk_minimum_probe.hip 2>/dev/null || exit 1
timeout -k 10 60 gpurun_out/pk_minimum_probe | tee gpurun_out/pk_minimum_probe.txt
