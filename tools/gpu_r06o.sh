# r06o: counters of the slow vs the fast arena (tools/mode_probe5.py) -- two PMC passes in separate
# processes (each process has its own slow arena: the split is by the process's own timing).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06o; mkdir -p $O
export TMPDIR=/tmp
C1="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE"
C2="TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum"
C3="TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum"
i=0
for C in "$C1" "$C2" "$C3" "$C1"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $C --kernel-include-regex 'k_wsum' -d $O/pmc$i -o pmc --output-format csv -- python3 tools/mode_probe5.py > $O/pmc$i.json 2> $O/pmc$i.err || { echo "FAIL pmc$i"; tail -5 $O/pmc$i.err; exit 1; }
  cat $O/pmc$i.json | cut -c1-400
done
exit 0
