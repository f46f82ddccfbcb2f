# rocprofv3 evidence for the bench's dominant kernel (run on the GPU box from the repo root):
#   1. kernel trace + stats of the bench command (average kernel duration)
#   2. PMC pass FETCH_SIZE, 3. PMC pass WRITE_SIZE (separate passes: TCC slots on gfx950)
# Outputs land in gpurun_out/prof_<tag>/; tools/pmc_traffic.py summarises them into profiles/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r01}
shift || true
BENCH_ARGS=${BENCH_ARGS:-"--steps 5 --warmup 2 --no-cpu-baseline --check-samples 0 --soak-seconds 0"}
OUT=/tmp/prof_$TAG  # raw traces stay off gpurun_out (copied back only if < 64 MiB)
mkdir -p $OUT
fault() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $BENCH_ARGS > $OUT/trace_bench.json 2> $OUT/trace.err; rc=$?
echo "trace rc=$rc"; fault $rc && exit $rc
if [ -n "$TRACE_ONLY" ]; then mkdir -p gpurun_out/summary; python3 tools/pmc_traffic.py $OUT $TAG gpurun_out/summary; exit 0; fi
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py $BENCH_ARGS > $OUT/fetch_bench.json 2> $OUT/fetch.err; rc=$?
echo "fetch rc=$rc"; fault $rc && exit $rc
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py $BENCH_ARGS > $OUT/write_bench.json 2> $OUT/write.err; rc=$?
echo "write rc=$rc"; fault $rc && exit $rc
mkdir -p gpurun_out/summary
python3 tools/pmc_traffic.py $OUT $TAG gpurun_out/summary || true
# keep gpurun_out small (it is copied back only if < 64 MiB): drop the raw traces
rm -rf $OUT/trace $OUT/fetch $OUT/write
