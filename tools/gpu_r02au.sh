# XCD-contiguous mapping on cfg3 (ViT-B/16 bf16, K = 128) through agg() on separate tensors: interleaved A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r02au
for M in 0 1 0 1; do
  FA_XCD_MAP=$M timeout -k 10 300 python bench.py --config vit_bf16 --layout tensors --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/r02au/b.json 2>gpurun_out/r02au/b.err || { tail -3 gpurun_out/r02au/b.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r02au/b.json'));print('vit_bf16_tensors', 'xcd=$M', d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'], str(d['parity'])[:30])" | tee -a gpurun_out/r02au/ab.txt
done
