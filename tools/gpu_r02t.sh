# launch-shape probe: tail of one-tile-per-workgroup launches at cfg2 / cfg3 / metric sizes
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r02t
PROBE_BIG=1 timeout -k 10 300 python tools/tail_probe.py > gpurun_out/r02t/tail_probe.json 2>gpurun_out/r02t/tail_probe.err || { tail -5 gpurun_out/r02t/tail_probe.err; exit 1; }
cat gpurun_out/r02t/tail_probe.json
