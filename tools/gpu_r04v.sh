# r04v: every BASELINE config and the extra workloads once on the round-end code (one box, one
# session): cfg2-cfg5, fedopt, secagg (LightSecAgg reconstruct), fragmented metric, median / Krum
# K = 128, the host path, the literal-input metric.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r04v; mkdir -p $O
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1],d['value'],d['unit'],d['ms_per_step'],r.get('kernel_avg_ms'),r.get('frac'),'|',(d.get('parity') or '')[:50])" $1; }
b() { n=$1; shift; timeout -k 10 400 python bench.py "$@" --no-cpu-baseline --soak-seconds 0 > $O/$n.json 2> $O/$n.err || { echo "FAIL $n"; tail -8 $O/$n.err; exit 1; }; line $O/$n.json; }
b resnet18 --config resnet18
b vit_bf16 --config vit_bf16
b hier --config hier
b gossip --config gossip
b fedopt --config fedopt --layout tiled
b secagg --config secagg
b fragmented --config fragmented
b metric_tensors --layout tensors
b median128 --config median --clients 128 --layout tiled
b krum128 --config krum --clients 128
b host --config host
