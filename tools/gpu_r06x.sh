# r06x: does contiguous memory remove the literal input's translation cost (r05b: UTCL2 busy 96 %
# when every workgroup touches 128 pieces 500 MB apart)?  The client-major arena (--layout arena: one
# allocation, now contiguous) vs the same with FEDML_AMD_ARENA_ALLOC=torch vs 128 separate tensors,
# 2 interleaved rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06x; mkdir -p $O
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1].split('/')[-1],d['value'],d['ms_per_step'],r.get('kernel_avg_ms'),r.get('frac'),r.get('frac_of_ceiling'),str(d.get('parity'))[:40])" $1; }
for i in 1 2; do
  timeout -k 10 300 python bench.py --layout arena --no-cpu-baseline --cold-reps 0 --soak-seconds 0 > $O/arena_contig_$i.json 2> $O/arena_contig_$i.err || { tail -5 $O/arena_contig_$i.err; exit 1; }
  line $O/arena_contig_$i.json
  FEDML_AMD_ARENA_ALLOC=torch timeout -k 10 300 python bench.py --layout arena --no-cpu-baseline --cold-reps 0 --soak-seconds 0 > $O/arena_torch_$i.json 2> $O/arena_torch_$i.err || { tail -5 $O/arena_torch_$i.err; exit 1; }
  line $O/arena_torch_$i.json
  timeout -k 10 300 python bench.py --layout tensors --no-cpu-baseline --cold-reps 0 --soak-seconds 0 > $O/tensors_$i.json 2> $O/tensors_$i.err || { tail -5 $O/tensors_$i.err; exit 1; }
  line $O/tensors_$i.json
done
exit 0
