# r03y: every bench configuration on ONE box with this session's code (one JSON line each, with the
# CPU baselines), for DESIGN §5's snapshot table.  Each step has its own time limit; a failure stops.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03y
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 420 python bench.py "$@" > gpurun_out/r03y/$n.json 2> gpurun_out/r03y/$n.err || { echo "FAIL $n"; tail -5 gpurun_out/r03y/$n.err; exit 1; }
  N=$n python -c 'import json,os;n=os.environ["N"];d=[json.loads(l) for l in open("gpurun_out/r03y/%s.json" % n) if l.startswith("{")][-1];r=d.get("roofline") or {};c=d.get("cpu_baseline") or {};print(n, d["value"], d["unit"], d.get("ms_per_step"), r.get("kernel_avg_ms"), r.get("frac"), c.get("value"), c.get("unit"), "|", d.get("parity"))'
}
run metric
run fragmented --config fragmented
run resnet18_tiled --config resnet18
run resnet18_adopted --config resnet18 --layout adopted
run resnet18_tensors --config resnet18 --layout tensors
run vit_tiled --config vit_bf16
run vit_tensors --config vit_bf16 --layout tensors
run hier --config hier
run gossip --config gossip
run fedopt --config fedopt
run secagg --config secagg
run samask --config samask
run samask_d4 --config samask --variant 4
run median32 --config median --clients 32
run median128 --config median --clients 128
run krum32 --config krum --clients 32
run krum128 --config krum --clients 128
run lr --config lr
run arrival --config arrival
run dropin_cpu --config dropin_cpu
