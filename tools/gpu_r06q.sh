# r06q: arena start offset within one allocation (tools/mode_probe7.py): 3 contiguous, 1 torch.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06q; mkdir -p $O
for i in 1 2 3 4; do
  FLAGS=$([ $i = 4 ] && echo -1 || echo 4) timeout -k 10 240 python tools/mode_probe7.py > $O/mode7_$i.json 2> $O/mode7_$i.err || { tail -5 $O/mode7_$i.err; exit 1; }
  cat $O/mode7_$i.json
done
exit 0
