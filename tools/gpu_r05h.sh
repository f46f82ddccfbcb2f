# r05h: why the Gram-form Krum kernel runs at ~half its MFMA floor: SQ counters (MFMA busy, wait
# states, LDS conflicts) + GRBM clock for K = 32 and 128, one pass each with the kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05h; mkdir -p $O
export TMPDIR=/tmp
C="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU_MFMA_F32 GRBM_GUI_ACTIVE GRBM_COUNT"
for K in 32 128; do
  FEDML_AMD_KRUM_FORM=gram timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C --kernel-include-regex 'k_pair_gram' -d $O/pmc_$K -o pmc --output-format csv -- python3 bench.py --config krum --clients $K --no-cpu-baseline --check-samples 0 --steps 3 --warmup 1 --soak-seconds 0 > $O/pmc_$K.log 2>&1 \
    || { echo "FAIL $K"; tail -5 $O/pmc_$K.log; exit 1; }
done
python3 - <<'PY'
import csv, collections, glob
for K in (32, 128):
    f = glob.glob(f"gpurun_out/r05h/pmc_{K}/**/*counter_collection.csv", recursive=True)[0]
    per = collections.defaultdict(dict); dur = {}
    for r in csv.DictReader(open(f)):
        per[r["Counter_Name"]][r["Dispatch_Id"]] = float(r["Counter_Value"])
        dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    med = {c: sorted(d.values())[len(d) // 2] for c, d in per.items()}
    ms = sorted(dur.values())[len(dur) // 2]
    print(K, "ms", round(ms, 4), {c: round(v) for c, v in med.items()})
    print("   clock GHz", round(med["GRBM_GUI_ACTIVE"] / 8 / (ms * 1e6), 3), "mfma busy / (gui*4 SIMD... )", med["SQ_VALU_MFMA_BUSY_CYCLES"] / med["GRBM_GUI_ACTIVE"])
PY
