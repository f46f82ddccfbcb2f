# r06aa: does a quick kernel / read-probe ratio right after allocation predict the arena's steady
# metric time (tools/placement_probe.py, 3 contiguous arenas per process, 4 processes)?
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06aa; mkdir -p $O
for i in 1 2 3 4; do
  timeout -k 10 240 python tools/placement_probe.py > $O/place_$i.json 2> $O/place_$i.err || { tail -5 $O/place_$i.err; exit 1; }
  cat $O/place_$i.json
done
exit 0
