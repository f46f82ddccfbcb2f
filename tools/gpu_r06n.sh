# r06n: arena x output placement (tools/mode_probe4.py) in 4 fresh processes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06n; mkdir -p $O
for i in 1 2 3 4; do
  timeout -k 10 200 python tools/mode_probe4.py > $O/mode4_$i.json 2> $O/mode4_$i.err || { tail -5 $O/mode4_$i.err; exit 1; }
  cat $O/mode4_$i.json
done
exit 0
