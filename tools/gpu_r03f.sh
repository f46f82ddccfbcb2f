# r03f: Krum defaults after the split heuristic + LDS cap A/B for 1024-thread groups
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r03f; mkdir -p $O
run() { K=$1; L=$2; FA_PAIR_LDS_KB=$L timeout -k 10 120 python bench.py --config krum --clients $K --no-cpu-baseline --check-samples 0 --steps 10 --warmup 2 > $O/K${K}_l$L.json 2> $O/K${K}_l$L.err || { tail -3 $O/K${K}_l$L.err; return 1; }; python -c "import json;d=json.load(open('$O/K${K}_l$L.json'));print($K, '$L', d['roofline']['kernel_avg_ms'])"; }
for K in 16 32 48 64 96 100 128; do run $K 80 || exit 1; done
for L in 110 150; do for K in 100 128; do run $K $L || exit 1; done; done
for K in 100 128; do run $K 80 || exit 1; done
