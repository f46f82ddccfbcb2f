# r05k: K <= 32 Gram kernel with a register ring of PD chunks in flight (k_pair_gram<1, VEC, PD>) --
# parity (robust pairwise/Krum tests), then K = 32 interleaved A/B over PD = 1 / 2 / 3 / 4, then one
# kernel trace of the product default.  First the whole GPU suite (the slot protocol changed: no
# per-call event for a use whose table was already staged); 3ev = FA_SLOT_EVENT=1 (the old protocol).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05k; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1],d['value'],d['ms_per_step'],r.get('kernel_avg_ms'),d.get('pair_form'),d.get('kappa_max'),d.get('parity'))" $1; }
B="--config krum --no-cpu-baseline --soak-seconds 0 --steps 20 --warmup 3"
for rep in 1 2 3; do
  for v in 1 2 3 4 3ev; do
    n=K32_pd${v}_$rep
    case $v in 3ev) E="FA_GRAM_PD=3 FA_SLOT_EVENT=1";; *) E="FA_GRAM_PD=$v";; esac
    env $E timeout -k 10 300 python bench.py $B --clients 32 --check-samples $([ $rep = 1 ] && echo 1 || echo 0) > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
    line $O/$n.json
  done
done
timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d $O/trace -o tr --output-format csv -- python3 bench.py $B --clients 32 --check-samples 0 > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r05k/trace/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(r["Name"][:90], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us")
f = glob.glob("gpurun_out/r05k/trace/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-14:]
t0 = int(rows[0]["Start_Timestamp"])
for r in rows:
    print(round((int(r["Start_Timestamp"]) - t0) / 1e3, 2), round((int(r["End_Timestamp"]) - t0) / 1e3, 2), r["Kernel_Name"][:70])
PY
