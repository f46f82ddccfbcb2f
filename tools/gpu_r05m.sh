# r05m: Gram-form Krum chunk dealing -- contiguous run per workgroup (default) vs round-robin
# (FA_GRAM_ILV=1: the workgroups read one compact window of every client at a time), K = 32 / 64 /
# 128, 3 interleaved reps; then translation / memory-stall counters of the K = 32 kernel both ways.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05m; mkdir -p $O
export TMPDIR=/tmp
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1],d['value'],d['ms_per_step'],r.get('kernel_avg_ms'),d.get('pair_form'),d.get('parity'))" $1; }
B="--config krum --no-cpu-baseline --soak-seconds 0 --steps 20 --warmup 3"
for rep in 1 2 3; do
  for K in 32 64 128; do
    for ilv in 0 1; do
      n=K${K}_ilv${ilv}_$rep
      FA_GRAM_ILV=$ilv timeout -k 10 300 python bench.py $B --clients $K --check-samples $([ $rep = 1 ] && echo 1 || echo 0) > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
      line $O/$n.json
    done
  done
done
C1="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_MULTI_MISS_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE"
C2="TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum"
for ilv in 0 1; do
  for p in 1 2; do
    [ $p = 1 ] && C=$C1 || C=$C2
    FA_GRAM_ILV=$ilv timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C --kernel-include-regex 'k_pair_gram' -d $O/pmc_${ilv}_$p -o pmc --output-format csv -- python3 bench.py $B --clients 32 --check-samples 0 --steps 3 --warmup 1 > $O/pmc_${ilv}_$p.log 2>&1 \
      || { echo "FAIL $ilv $p"; tail -5 $O/pmc_${ilv}_$p.log; exit 1; }
  done
done
python3 - <<'PY'
import csv, collections, glob
for ilv in (0, 1):
    out = {}
    for p in (1, 2):
        f = glob.glob(f"gpurun_out/r05m/pmc_{ilv}_{p}/**/*counter_collection.csv", recursive=True)[0]
        per = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            per[r["Counter_Name"]].append(float(r["Counter_Value"]))
        out.update({c: sorted(v)[len(v) // 2] for c, v in per.items()})
    print("ilv", ilv, {c: round(v) for c, v in out.items()})
    if "GRBM_UTCL2_BUSY" in out:
        print("   UTCL2 busy frac", round(out["GRBM_UTCL2_BUSY"] / out["GRBM_GUI_ACTIVE"], 3))
PY
