# r05x: the literal-input metric (128 separate fp32[125 M] buffers) under workgroup -> tile maps:
# XCD-contiguous (default), round-robin (FA_XCD_MAP=0), and the spread map with S = 64 / 256 / 1,024
# regions read at once (FA_XCD_MAP=3/4/5) -- if DRAM channel / bank camping of the 128 streams at equal
# offsets is what holds the literal input below the tiled arena, spreading the concurrent tiles over
# the address space helps; 2 interleaved reps, 20 steps after 5 warmup.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05x; mkdir -p $O
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1].split('/')[-1],d['value'],d['ms_per_step'],r.get('kernel_avg_ms'),r.get('frac'),d.get('parity'))" $1; }
for rep in 1 2; do
  for m in 1 0 3 4 5; do
    FA_XCD_MAP=$m timeout -k 10 300 python bench.py --layout tensors --steps 20 --warmup 5 --no-cpu-baseline --soak-seconds 0 --check-samples $([ $rep = 1 ] && echo 65536 || echo 0) > $O/map${m}_$rep.json 2> $O/map${m}_$rep.err || { tail -5 $O/map${m}_$rep.err; exit 1; }
    line $O/map${m}_$rep.json
  done
done
