# r06al: the final bench.py's lines for the rest of the table -- Krum K = 64 / 96 / 128, median K = 32 /
# 128, cfg3 ViT bf16, cfg4 hierarchical, cfg5 gossip (cold latency and sustained rate beside each).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06al; mkdir -p $O
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};c=d.get('cold') or {};print(sys.argv[1].split('/')[-1],d['value'],d['ms_per_step'],r.get('kernel_avg_ms'),r.get('frac'),'cold',c.get('ms'),'sust',(d.get('sustained') or {}).get('ms_per_step'),str(d.get('parity'))[:40])" $1; }
for c in "krum --clients 64" "krum --clients 96" "krum --clients 128" "median --clients 32" "median --clients 128" vit_bf16 hier gossip; do
  n=$(echo $c | tr -d ' -')
  timeout -k 10 400 python bench.py --config $c --no-cpu-baseline --soak-seconds 2 > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
  line $O/$n.json
done
exit 0
