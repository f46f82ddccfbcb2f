# A/B median builds (tools/var/lib_*.so copied over fedml_amd/libfedagg.so in the box's copy; "cur" =
# the tree's build).  Env: VARS (builds), DT (fp32|bf16|fp16), KS, CS (parity samples).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out tools/var
cp fedml_amd/libfedagg.so tools/var/lib_cur.so
r() { timeout -k 10 120 python bench.py --config median --clients $1 --dtype ${DT:-fp32} --no-cpu-baseline --check-samples ${CS:-0} --steps 10 --warmup 3 > gpurun_out/m.json 2>gpurun_out/m.err || { echo FAIL $1; tail -3 gpurun_out/m.err; exit 1; }
      V=$V K=$1 python -c 'import json,os;d=json.load(open("gpurun_out/m.json"));print(os.environ["V"], os.environ.get("DT","fp32"), "K="+os.environ["K"], d["roofline"]["kernel_avg_ms"], d["value"], d.get("parity"))'; }
for V in ${VARS:-cur}; do cp tools/var/lib_$V.so fedml_amd/libfedagg.so; for K in ${KS:-16 32 64 128}; do r $K; done; done
cp tools/var/lib_cur.so fedml_amd/libfedagg.so
