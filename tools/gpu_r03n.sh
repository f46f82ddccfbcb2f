# r03n: doorbell probe with the multi-workgroup sweep, then cfg1 latency A/B (FA_HOST1=1 / 0).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o gpurun_out/doorbell_probe tools/doorbell_probe.hip 2>/dev/null || exit 1
timeout -k 10 60 gpurun_out/doorbell_probe 3000 > gpurun_out/doorbell.json || { echo doorbell probe failed; exit 1; }
cat gpurun_out/doorbell.json
for rep in 1 2 3; do
  for f in 1 0; do
    FA_HOST1=$f timeout -k 10 200 python bench.py --config lr --steps 3000 --warmup 200 $( [ $rep = 1 ] && [ $f = 1 ] || echo --no-cpu-baseline ) > gpurun_out/lr_$f.json 2> gpurun_out/lr_$f.err || { tail -5 gpurun_out/lr_$f.err; exit 1; }
    F=$f python -c 'import json,os;d=json.load(open("gpurun_out/lr_%s.json" % os.environ["F"]));print("host1", os.environ["F"], d["value"], d["unit"], d.get("parity"), (d.get("cpu_baseline") or {}).get("value"))'
    [ $rep = 1 ] && [ $f = 1 ] && cp gpurun_out/lr_1.json gpurun_out/lr_host1_full.json
  done
done
true
