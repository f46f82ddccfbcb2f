# r05d: client passes vs the translation working set (tools/translation_probe.py), separate buffers
# and client-major arena rows, 4 interleaved reps each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05d; mkdir -p $O
for lay in tensors arena; do
  LAYOUT=$lay timeout -k 10 300 python tools/translation_probe.py > $O/probe_$lay.json 2> $O/probe_$lay.err || { tail -5 $O/probe_$lay.err; exit 1; }
  cat $O/probe_$lay.json
done
