# r05r: (0) the Gram kernel without padding masks, float64 flushes every 2nd / 4th chunk, and for
# K in (96, 128] the 12-wave 16x16 form (FA_GRAM16=0: the 10-wave 32x32 form): robust tests, then
# K = 64 and K = 100 / 128 A/B, 3 interleaved reps; (1) rocprof evidence of the K = 32 Krum ring kernel (kernel trace + FETCH_SIZE + WRITE_SIZE
# passes -> profiles/pmc_traffic.json); (2) the timeline of cfg2 on separate tensors (what sits
# between consecutive k_wsum_pair kernels).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05r; mkdir -p $O gpurun_out/summary
export TMPDIR=/tmp
fault() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_robust.py -x -q --timeout 120 --timeout-method thread -k "pairwise or krum" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1],d['value'],d['ms_per_step'],r.get('kernel_avg_ms'),d.get('pair_form'),d.get('parity'))" $1; }
for rep in 1 2 3; do
  for v in K64_1 K100_1 K100_0 K128_1 K128_0; do
    K=${v%_*}; K=${K#K}; S=${v#*_}
    FA_GRAM16=$S timeout -k 10 300 python bench.py --config krum --clients $K --steps 20 --warmup 3 --no-cpu-baseline --soak-seconds 0 --check-samples $([ $rep = 1 ] && echo 1 || echo 0) > $O/${v}_$rep.json 2> $O/${v}_$rep.err || { tail -5 $O/${v}_$rep.err; exit 1; }
    line $O/${v}_$rep.json
  done
done
P="--steps 5 --warmup 2 --no-cpu-baseline --check-samples 0 --soak-seconds 0"
BENCH_ARGS="--config krum --clients 32 $P" KERNEL=k_pair_gram_ring timeout -k 10 900 bash tools/profile.sh r05_krum32 > gpurun_out/summary/r05_krum32.log 2>&1; rc=$?
echo "== krum32 rc=$rc"; tail -20 gpurun_out/summary/r05_krum32.log
fault $rc && exit $rc
timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d $O/cfg2t -o tr -- python3 bench.py --config resnet18 --layout tensors --steps 20 --warmup 3 --no-cpu-baseline --check-samples 0 --soak-seconds 0 > $O/cfg2t.log 2>&1 || { tail -5 $O/cfg2t.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r05r/cfg2t/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if "distribution" not in r["Kernel_Name"] and "normal" not in r["Kernel_Name"]]
rows = rows[-16:]
t0 = int(rows[0]["Start_Timestamp"])
for r in rows:
    print(round((int(r["Start_Timestamp"]) - t0) / 1e3, 2), round((int(r["End_Timestamp"]) - t0) / 1e3, 2), r["Kernel_Name"][:80])
PY
