# r05 round-end evidence of the HEAD binary, one box, one session: the whole GPU suite, smoke(), the
# default bench line, rocprof kernel trace + FETCH_SIZE + WRITE_SIZE of every dominant kernel
# (-> profiles/r05f_*, pmc_traffic.json), and one bench line per BASELINE config / robust workload.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05_final; mkdir -p $O gpurun_out/summary
export TMPDIR=/tmp
fault() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
cat $O/bench_default.json
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1].split('/')[-1],d['value'],d['unit'],d['ms_per_step'],r.get('kernel_avg_ms'),r.get('frac'),d.get('parity'))" $1; }
B="--no-cpu-baseline --soak-seconds 0"
cfg() {
  n=$1; shift
  timeout -k 10 400 python bench.py $B "$@" > $O/$n.json 2> $O/$n.err || { tail -10 $O/$n.err; exit 1; }
  line $O/$n.json
}
cfg cfg1_lr --config lr
cfg cfg2_tiled --config resnet18 --layout tiled --steps 50 --warmup 5
cfg cfg2_tensors --config resnet18 --layout tensors --steps 50 --warmup 5
cfg cfg3_vit --config vit_bf16 --steps 20 --warmup 3
cfg cfg4_hier --config hier
cfg cfg5_gossip --config gossip
cfg metric_tensors --config metric --layout tensors
cfg median32 --config median --clients 32 --steps 20 --warmup 3
cfg median128 --config median --clients 128 --layout tiled --steps 20 --warmup 3
cfg krum32 --config krum --clients 32 --steps 20 --warmup 3 --check-samples 1
cfg krum64 --config krum --clients 64 --steps 20 --warmup 3 --check-samples 1
cfg krum128 --config krum --clients 128 --steps 20 --warmup 3 --check-samples 1
cfg fedopt --config fedopt
cfg secagg --config secagg
P="--steps 5 --warmup 2 --no-cpu-baseline --check-samples 0 --soak-seconds 0"
prof() {
  tag=$1; kern=$2; shift 2
  BENCH_ARGS="$* $P" KERNEL=$kern timeout -k 10 900 bash tools/profile.sh $tag > gpurun_out/summary/$tag.log 2>&1; rc=$?
  echo "== $tag rc=$rc"; grep -E '"kernel"|avg_ns|traffic_over' gpurun_out/summary/$tag.log
  fault $rc && exit $rc
  rm -rf /tmp/prof_$tag
  return 0
}
prof r05f_metric k_wsum --config metric
prof r05f_hier k_wsum --config hier
prof r05f_gossip k_mix --config gossip
prof r05f_resnet18 k_wsum --config resnet18 --layout tiled
prof r05f_resnet18_tensors k_wsum --config resnet18 --layout tensors
prof r05f_median128 k_median --config median --clients 128 --layout tiled
prof r05f_metric_tensors k_wsum --config metric --layout tensors
prof r05f_krum32 k_pair_gram_ring --config krum --clients 32
prof r05f_krum128 k_pair_gram --config krum --clients 128
exit 0
