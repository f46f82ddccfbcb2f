# r06a: VERDICT r05 item 2 (the headline's two modes) and item 3 (the in-process read ceiling).
# (1) three default lines as separate fresh processes (each now carries the read probe over its own
#     arena); (2) two arenas in one process (tools/mode_probe.py); (3) two default lines under
#     rocprofv3 --kernel-trace --stats; (4) one translation / clock PMC pass of the metric kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06a; mkdir -p $O
export TMPDIR=/tmp
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};c=r.get('measured_read_ceiling') or {};print(sys.argv[1].split('/')[-1],d['value'],d['ms_per_step'],r.get('kernel_avg_ms'),r.get('frac'),'ceiling',c.get('value'),c.get('median'),'frac_of_ceiling',r.get('frac_of_ceiling'),'sust',(d.get('sustained') or {}).get('value'),'cold',(d.get('cold') or {}).get('ms'))" $1; }
B="--no-cpu-baseline --check-samples 0 --soak-seconds 2 --cold-reps 3"
for i in 1 2 3; do
  timeout -k 10 300 python bench.py $B > $O/default_$i.json 2> $O/default_$i.err || { tail -5 $O/default_$i.err; exit 1; }
  line $O/default_$i.json
done
timeout -k 10 300 python tools/mode_probe.py > $O/mode_probe.json 2> $O/mode_probe.err || { tail -5 $O/mode_probe.err; exit 1; }
cat $O/mode_probe.err | tail -3
for i in 1 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r06a_tr$i -o run -- python3 bench.py $B --cold-reps 0 > $O/rocprof_$i.json 2> $O/rocprof_$i.err || { tail -5 $O/rocprof_$i.err; exit 1; }
  line $O/rocprof_$i.json
  cp $(find /tmp/r06a_tr$i -name '*kernel_stats.csv' | head -1) $O/rocprof_${i}_kernel_stats.csv
  head -4 $O/rocprof_${i}_kernel_stats.csv | cut -c1-200
done
C1="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE"
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $C1 --kernel-include-regex 'k_wsum|k_read_probe' -d $O/pmc1 -o pmc --output-format csv -- python3 bench.py --steps 4 --warmup 2 $B --cold-reps 0 --soak-seconds 0 > $O/pmc1.log 2>&1 \
  || { echo "FAIL pmc1"; tail -5 $O/pmc1.log; exit 1; }
tail -1 $O/pmc1.log | cut -c1-300
exit 0
