# GPU pytest only: PYTEST_ARGS (default: the whole -m gpu suite).  Stops on a fault / timeout.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ARGS=${PYTEST_ARGS:-tests -m gpu}
timeout -k 10 ${TEST_TIMEOUT:-900} python -m pytest $ARGS -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -25 gpurun_out/pytest_gpu.log
exit $rc
