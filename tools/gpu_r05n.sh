# r05n: K <= 32 Gram kernel on an LDS-DMA ring (k_pair_gram_glds<NB>, NB = 3 / 4 buffers) vs the
# register-staged k_pair_gram<1> (FA_GRAM_GLDS=0): robust pairwise / Krum GPU tests, then K = 32
# interleaved A/B, 3 reps, then one kernel trace of the default.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05n; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_robust.py -x -q --timeout 120 --timeout-method thread -k "pairwise or krum" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1],d['value'],d['ms_per_step'],r.get('kernel_avg_ms'),d.get('pair_form'),d.get('kappa_max'),d.get('parity'))" $1; }
B="--config krum --no-cpu-baseline --soak-seconds 0 --steps 20 --warmup 3"
for rep in 1 2 3; do
  for v in 3 4 0; do
    n=K32_glds${v}_$rep
    E="FA_GRAM_GLDS=$v"
    env $E timeout -k 10 300 python bench.py $B --clients 32 --check-samples $([ $rep = 1 ] && echo 1 || echo 0) > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
    line $O/$n.json
  done
done
timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d $O/trace -o tr --output-format csv -- python3 bench.py $B --clients 32 --check-samples 0 > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r05n/trace/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(r["Name"][:90], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us")
f = glob.glob("gpurun_out/r05n/trace/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-14:]
t0 = int(rows[0]["Start_Timestamp"])
for r in rows:
    print(round((int(r["Start_Timestamp"]) - t0) / 1e3, 2), round((int(r["End_Timestamp"]) - t0) / 1e3, 2), r["Kernel_Name"][:70])
PY
