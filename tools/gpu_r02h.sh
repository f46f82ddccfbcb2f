# round-2 refresh of every bench config (one JSON line each) + the device-ingest probe
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r02h
T="timeout -k 10"
$T 120 python tools/ingest_probe.py > gpurun_out/r02h/ingest_probe.json 2> gpurun_out/r02h/ingest.err || { tail gpurun_out/r02h/ingest.err; exit 1; }
cat gpurun_out/r02h/ingest_probe.json
run() { name=$1; shift; $T 400 python bench.py "$@" > gpurun_out/r02h/$name.json 2> gpurun_out/r02h/$name.err; rc=$?; echo "$name rc=$rc $(head -c 300 gpurun_out/r02h/$name.json)"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r02h/$name.err; exit $rc; }; }
run metric --cpu-seconds 6
run resnet18 --steps 50 --warmup 5 --no-cpu-baseline
run resnet18_adopted --config resnet18 --layout adopted --steps 50 --warmup 5 --no-cpu-baseline
run vit_bf16 --config vit_bf16 --steps 20 --warmup 3 --no-cpu-baseline
run vit_bf16_adopted --config vit_bf16 --layout adopted --steps 20 --warmup 3 --no-cpu-baseline
run hier --config hier --steps 20 --warmup 3 --no-cpu-baseline
run gossip --config gossip --steps 10 --warmup 2 --no-cpu-baseline
run fedopt --config fedopt --steps 10 --warmup 2 --cpu-seconds 6
run median --config median --steps 20 --warmup 3 --cpu-seconds 4
run median128 --config median --clients 128 --steps 10 --warmup 2 --no-cpu-baseline
run krum --config krum --steps 20 --warmup 3 --cpu-seconds 4
run krum128 --config krum --clients 128 --steps 5 --warmup 1 --no-cpu-baseline
run secagg --config secagg --steps 10 --warmup 2 --cpu-seconds 4
run fragmented --config fragmented --steps 10 --warmup 2 --no-cpu-baseline
run dropin_cpu --config dropin_cpu --steps 10 --warmup 2
run host --config host --steps 5 --warmup 1 --no-cpu-baseline
run arrival --config arrival --steps 10 --warmup 3 --cpu-seconds 4
run lr_tensors --config lr --layout tensors --steps 2000 --warmup 200
