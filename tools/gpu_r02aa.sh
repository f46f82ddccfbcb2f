# round-2 record: rocprofv3 kernel stats + PMC HBM traffic of the default bench (metric) and median K = 128
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r02aa
BENCH_ARGS="--steps 10 --warmup 3 --no-cpu-baseline" timeout -k 10 1000 bash tools/profile.sh r02_metric || exit 1
KERNEL=k_median_2l BENCH_ARGS="--config median --clients 128 --steps 10 --warmup 2 --no-cpu-baseline" timeout -k 10 900 bash tools/profile.sh r02_median_K128 || exit 1
ls gpurun_out/summary
