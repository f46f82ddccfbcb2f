# rocprofv3 after the XCD-contiguous mapping: kernel stats of cfg2 on separate tensors (k_wsum_pair,
# trace only) and the final k_median_2l at K = 128 (trace + PMC).  (The fragmented config's FETCH_SIZE
# pass segfaulted under rocprofv3 in the first attempt of this script -- rc 139 -- and is not repeated.)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r02at
TRACE_ONLY=1 KERNEL=k_wsum_pair BENCH_ARGS="--config resnet18 --layout tensors --steps 20 --warmup 5 --no-cpu-baseline" timeout -k 10 600 bash tools/profile.sh r02_resnet18_tensors || exit 1
KERNEL=k_median_2l BENCH_ARGS="--config median --clients 128 --steps 10 --warmup 2 --no-cpu-baseline" timeout -k 10 600 bash tools/profile.sh r02_median_K128_final || exit 1
ls gpurun_out/summary
