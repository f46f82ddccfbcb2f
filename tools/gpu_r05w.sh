# r05w: what bounds cfg3 (ViT-B/16 bf16, K = 128, k_wsum_pair_inl on bf16) and cfg5 (k_mix_band):
# VALU utilisation + clock (SQ_INSTS_VALU, SQ_ACTIVE_INST_VALU, SQ_WAVE_CYCLES, SQ_BUSY_CYCLES,
# GRBM_GUI_ACTIVE) in one pass with the kernel trace, per workload.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05w; mkdir -p $O
export TMPDIR=/tmp
C="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
for w in vit gossip metric; do
  case $w in vit) A="--config vit_bf16"; R=k_wsum;; gossip) A="--config gossip"; R=k_mix;; metric) A="--config metric"; R=k_wsum;; esac
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $C --kernel-include-regex $R -d $O/pmc_$w -o pmc --output-format csv -- python3 bench.py $A --no-cpu-baseline --check-samples 0 --steps 5 --warmup 5 --soak-seconds 0 > $O/pmc_$w.log 2>&1 \
    || { echo "FAIL $w"; tail -5 $O/pmc_$w.log; exit 1; }
done
python3 - <<'PY'
import csv, collections, glob, json
out = {}
for w in ("vit", "gossip", "metric"):
    f = glob.glob(f"gpurun_out/r05w/pmc_{w}/**/*counter_collection.csv", recursive=True)[0]
    per = collections.defaultdict(list); dur = []
    for r in csv.DictReader(open(f)):
        per[r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    med = {c: sorted(v)[len(v) // 2] for c, v in per.items()}
    ms = sorted(dur)[len(dur) // 2]
    gui = med["GRBM_GUI_ACTIVE"]
    res = {"kernel_ms": round(ms, 4), "clock_ghz": round(gui / 8 / (ms * 1e6), 3),
           "valu_busy_frac": round(med["SQ_ACTIVE_INST_VALU"] / (gui / 8 * 256 * 4) if gui else 0, 3),
           "waves_per_simd": round(med["SQ_WAVE_CYCLES"] / (gui / 8 * 1024) if gui else 0, 2),
           "valu_per_wave": round(med["SQ_INSTS_VALU"] / med["SQ_WAVES"], 1) if med.get("SQ_WAVES") else None,
           "counters": {c: round(v) for c, v in med.items()}}
    out[w] = res
    print(w, json.dumps({k: v for k, v in res.items() if k != "counters"}))
json.dump(out, open("gpurun_out/r05w/valu_summary.json", "w"), indent=1)
PY
