# rocprofv3 evidence for the configs (summaries only are kept under gpurun_out/summary).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/summary
fault() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
for cfg in ${CONFIGS:-metric resnet18 vit_bf16 gossip hier secagg fedopt median krum}; do
  tag=${ROUND:-r01}_$cfg
  TO=""; [ "$cfg" = vit_bf16 ] && TO=1   # rocprofv3 --pmc segfaulted on this config (round 1): trace only
  TRACE_ONLY=$TO BENCH_ARGS="--config $cfg --steps 5 --warmup 2 --no-cpu-baseline --check-samples 0 --soak-seconds 0" KERNEL=${KERNEL:-k_} timeout -k 10 900 bash tools/profile.sh $tag > gpurun_out/summary/$tag.log 2>&1; rc=$?
  echo "== $cfg rc=$rc"; tail -22 gpurun_out/summary/$tag.log
  fault $rc && exit $rc
  rm -rf /tmp/prof_$tag
done
exit 0
