# r03g: Krum A/B: register prefetch (FA_PAIR_PF) x lane staging depth (FA_PAIR_NPL), interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r03g; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_robust.py -x -q --timeout 120 --timeout-method thread -k "pair or krum" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() { K=$1; PF=$2; NPL=$3; FA_PAIR_PF=$PF FA_PAIR_NPL=$NPL timeout -k 10 120 python bench.py --config krum --clients $K --no-cpu-baseline --check-samples 0 --steps 10 --warmup 2 > $O/K${K}_pf${PF}_n$NPL.json 2> $O/K${K}.err || { tail -3 $O/K${K}.err; return 1; }; python -c "import json;d=json.load(open('$O/K${K}_pf${PF}_n$NPL.json'));print($K, 'pf$PF npl$NPL', d['roofline']['kernel_avg_ms'])"; }
for rep in 1 2; do
for K in 16 32; do for PF in 0 1; do for NPL in 8 16; do run $K $PF $NPL || exit 1; done; done; done
for K in 64 100 128; do for PF in 0 1; do run $K $PF 8 || exit 1; done; done
done
FA_PAIR_NPL=16 timeout -k 10 300 python -u -m pytest tests/test_gpu_robust.py -x -q --timeout 120 --timeout-method thread -k "pair or krum" > $O/tests_npl16.log 2>&1 || { tail -30 $O/tests_npl16.log; exit 1; }
tail -1 $O/tests_npl16.log
