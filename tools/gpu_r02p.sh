# staging copy kernel vs hipMemcpyAsync (FA_STAGE_COPY=0): host/GPU per call of agg() on separate
# tensors, then the full GPU test suite and the cfg2 tensors bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r02p
timeout -k 10 200 python tools/host_probe_b2b.py > gpurun_out/r02p/b2b_copy.json 2>/dev/null || { echo probe1 failed; exit 1; }
timeout -k 10 200 env FA_STAGE_COPY=0 python tools/host_probe_b2b.py > gpurun_out/r02p/b2b_memcpy.json 2>/dev/null || { echo probe2 failed; exit 1; }
python - <<'P'
import json
for n in ("copy","memcpy"):
    d=json.load(open(f"gpurun_out/r02p/b2b_{n}.json")); print(n, d["b2b_keep"], d["b2b_drop"])
P
for v in 1 0; do timeout -k 10 200 env FA_STAGE_COPY=$v python bench.py --config resnet18 --layout tensors --no-cpu-baseline --steps 30 --warmup 5 > gpurun_out/r02p/tensors_$v.json 2>gpurun_out/r02p/tensors_$v.err || { echo bench $v failed; tail -3 gpurun_out/r02p/tensors_$v.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r02p/tensors_$v.json'));print('stage_copy=$v', d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'], d['parity'])"; done
echo done
