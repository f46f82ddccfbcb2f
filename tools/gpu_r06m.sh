# r06m: output placements (tools/mode_probe3.py) in 4 fresh processes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06m; mkdir -p $O
for i in 1 2 3 4; do
  timeout -k 10 200 python tools/mode_probe3.py > $O/mode3_$i.json 2> $O/mode3_$i.err || { tail -5 $O/mode3_$i.err; exit 1; }
  tail -2 $O/mode3_$i.err
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1][-12:],' '.join(f\"{k}:{v['ms_med']}/{v['fill_GBs']}\" for k,v in d.items()))" $O/mode3_$i.json
done
exit 0
