set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 200 python tools/host_probe_tensors2.py > gpurun_out/host_probe_tensors2.json 2> gpurun_out/hpt.err || { tail gpurun_out/hpt.err; exit 1; }
cat gpurun_out/host_probe_tensors2.json
