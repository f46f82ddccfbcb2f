# r03e: Krum esplit sweep (FA_PAIR_SPLIT) after the strict-upper-tile change
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r03e; mkdir -p $O
run() { K=$1; E=$2; FA_PAIR_SPLIT=$E timeout -k 10 120 python bench.py --config krum --clients $K --no-cpu-baseline --check-samples 0 --steps 10 --warmup 2 > $O/K${K}_e$E.json 2> $O/K${K}_e$E.err || { tail -3 $O/K${K}_e$E.err; return 1; }; python -c "import json;d=json.load(open('$O/K${K}_e$E.json'));print($K, '$E', d['roofline']['kernel_avg_ms'])"; }
for E in 0 4 7 9 14 18 27 36; do run 32 $E || exit 1; done
for E in 0 1 2 3 4 6 8; do run 64 $E || exit 1; done
for E in 0 1 2 3; do run 100 $E || exit 1; done
for E in 0 1 2; do run 128 $E || exit 1; done
