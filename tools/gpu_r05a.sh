# r05a: rocprof evidence of the HEAD binary, one box, one session:
# the default bench line, then kernel trace + FETCH_SIZE + WRITE_SIZE passes of the dominant kernel
# for the metric (k_wsum_inl), cfg4 hier (k_wsum_grouped), cfg5 gossip (k_mix_band), cfg2 tiled
# (k_wsum_pair_inl), cfg2 on separate tensors (k_wsum_pair) and median K = 128 tiled (k_median_2l);
# plus the box's counter list (input to the literal-layout and median counter passes).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05a; mkdir -p $O gpurun_out/summary
export TMPDIR=/tmp
fault() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 120 rocprofv3 --list-avail > $O/counters_avail.txt 2>&1; echo "list-avail rc=$?"
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
cat $O/bench_default.json
P="--steps 5 --warmup 2 --no-cpu-baseline --check-samples 0 --soak-seconds 0"
prof() {
  tag=$1; shift
  BENCH_ARGS="$* $P" KERNEL=${KERNEL:-k_} timeout -k 10 900 bash tools/profile.sh $tag > gpurun_out/summary/$tag.log 2>&1; rc=$?
  echo "== $tag rc=$rc"; tail -24 gpurun_out/summary/$tag.log
  fault $rc && exit $rc
  rm -rf /tmp/prof_$tag
  return 0
}
prof r05_metric --config metric
prof r05_hier --config hier
prof r05_gossip --config gossip
prof r05_resnet18 --config resnet18
prof r05_resnet18_tensors --config resnet18 --layout tensors
prof r05_median128 --config median --clients 128 --layout tiled
prof r05_metric_tensors --config metric --layout tensors
exit 0
