# r05l: the slot protocol A/B -- FA_SLOT_EVENT=1 (an event per call at release() and a host wait at
# acquire, the r04 protocol) vs the default (no event for a use whose table was already staged), on
# every staged-table path: cfg2 on separate tensors (k_wsum_pair), cfg2 tiled, cfg3 ViT bf16, median
# K = 128, Krum K = 128; 3 interleaved reps, parity checked on rep 1.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05l; mkdir -p $O
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1],d['value'],d['ms_per_step'],r.get('kernel_avg_ms'),r.get('frac'),d.get('parity'))" $1; }
for rep in 1 2 3; do
  CS=$([ $rep = 1 ] && echo 65536 || echo 0)
  for cfg in cfg2t cfg2 cfg3 med128 krum128; do
    case $cfg in
      cfg2t) A="--config resnet18 --layout tensors --steps 50 --warmup 5";;
      cfg2) A="--config resnet18 --steps 50 --warmup 5";;
      cfg3) A="--config vit_bf16 --steps 20 --warmup 3";;
      med128) A="--config median --clients 128 --steps 20 --warmup 3";;
      krum128) A="--config krum --clients 128 --steps 20 --warmup 3";;
    esac
    for ev in 0 1; do
      n=${cfg}_ev${ev}_$rep
      FA_SLOT_EVENT=$ev timeout -k 10 300 python bench.py $A --no-cpu-baseline --soak-seconds 0 --check-samples $CS > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
      line $O/$n.json
    done
  done
done
