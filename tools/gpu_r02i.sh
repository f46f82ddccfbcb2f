set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r02h
T="timeout -k 10"
run() { name=$1; shift; $T 400 python bench.py "$@" > gpurun_out/r02h/$name.json 2> gpurun_out/r02h/$name.err; rc=$?; echo "$name rc=$rc $(head -c 300 gpurun_out/r02h/$name.json)"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r02h/$name.err; exit $rc; }; }
run resnet18 --config resnet18 --steps 50 --warmup 5 --no-cpu-baseline
run dropin_cpu --config dropin_cpu --steps 10 --warmup 2
run host --config host --steps 5 --warmup 1 --no-cpu-baseline
run arrival --config arrival --steps 10 --warmup 3 --cpu-seconds 4
run lr_tensors --config lr --layout tensors --steps 2000 --warmup 200
