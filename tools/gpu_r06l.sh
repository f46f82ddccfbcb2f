# r06l: the metric's process-level modes -- tools/mode_probe2.py (one arena, 4 output buffers at
# different placements, interleaved) in 4 fresh processes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06l; mkdir -p $O
for i in 1 2 3 4; do
  timeout -k 10 200 python tools/mode_probe2.py > $O/mode2_$i.json 2> $O/mode2_$i.err || { tail -5 $O/mode2_$i.err; exit 1; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1][-12:],[(v['ms_med'],v['ms_min']) for v in d['outs'].values()],d['probe_GBs_best'])" $O/mode2_$i.json
done
exit 0
