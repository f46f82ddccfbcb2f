# cfg1 latency breakdown; cfg2 drop-in layouts A/B on one box under rocprof (pure kernel times) + bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T="timeout -k 10"
$T 200 python tools/lr_probe.py > gpurun_out/lr_probe.json 2> gpurun_out/lr_probe.err || { tail gpurun_out/lr_probe.err; exit 1; }
cat gpurun_out/lr_probe.json
export TMPDIR=/tmp
for L in adopted arena tiled tensors; do
  $T 200 python bench.py --config resnet18 --layout $L --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/r18e_$L.json 2> gpurun_out/r18e_$L.err || { tail -20 gpurun_out/r18e_$L.err; exit 1; }
  echo "bench layout=$L $(python -c "import json;d=json.load(open('gpurun_out/r18e_$L.json'));print(d['value'],d['ms_per_step'],d['roofline']['kernel_avg_ms'])")"
  $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_r18e_$L -o run -- python3 bench.py --config resnet18 --layout $L --steps 30 --warmup 3 --no-cpu-baseline --check-samples 0 > /dev/null 2> gpurun_out/prof_r18e_$L.err; rc=$?
  [ $rc -eq 0 ] || { echo "rocprof rc=$rc"; exit $rc; }
  find /tmp/prof_r18e_$L -name "*kernel_stats.csv" -exec cp {} gpurun_out/r02e_resnet18_${L}_kernel_stats.csv \;
  echo "rocprof layout=$L"; grep -E "wsum|copyBuffer" gpurun_out/r02e_resnet18_${L}_kernel_stats.csv | awk -F'",' '{print substr($1,1,60)}' ; grep -E "wsum" gpurun_out/r02e_resnet18_${L}_kernel_stats.csv | awk -F',' '{print "calls",$(NF-6),"avg_ns",$(NF-4),"min",$(NF-2)}'
done
