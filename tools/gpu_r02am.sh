# k_median_2l occupancy (no NaN-flag array: N x 512 B LDS; waves/EU 8/6/5 by N) vs the committed kernel:
# median GPU tests on the new library, then interleaved A/B by swapping the library file
# (tools/ab/libfedagg_{base,new}.so were built from the parent commit and this one; not kept in the tree)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r02am
cp tools/ab/libfedagg_new.so fedml_amd/libfedagg.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_robust.py -m gpu -x -q --timeout 120 --timeout-method thread -k median > gpurun_out/r02am/robust.log 2>&1 || { tail -40 gpurun_out/r02am/robust.log; exit 1; }
tail -1 gpurun_out/r02am/robust.log
for K in 128 100 80 72 112; do
 for V in base new base new; do
  cp tools/ab/libfedagg_$V.so fedml_amd/libfedagg.so
  timeout -k 10 120 python bench.py --config median --clients $K --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/r02am/m.json 2>gpurun_out/r02am/m.err || { tail -3 gpurun_out/r02am/m.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r02am/m.json'));print($K, '$V', d['roofline']['kernel_avg_ms'], d['roofline']['frac'], str(d['parity'])[:30])" | tee -a gpurun_out/r02am/ab.txt
 done
done
cp tools/ab/libfedagg_new.so fedml_amd/libfedagg.so
