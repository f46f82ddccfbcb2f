# r06p: contiguous vs torch arenas (tools/mode_probe6.py) in 5 fresh processes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06p; mkdir -p $O
for i in 1 2 3 4 5; do
  ORDER=$([ $((i % 2)) = 1 ] && echo T0,C0,C1 || echo C0,T0,C1) timeout -k 10 240 python tools/mode_probe6.py > $O/mode6_$i.json 2> $O/mode6_$i.err || { tail -5 $O/mode6_$i.err; exit 1; }
  grep -v amdgpu.ids $O/mode6_$i.err | tail -2; cat $O/mode6_$i.json
done
exit 0
