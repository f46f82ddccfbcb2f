# r03a: bench self-launch rehearsal (N=2, N=4 over gloo on one device), default N=1 bench, smoke
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r03a; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_distributed.py -x -v --timeout 120 --timeout-method thread > $O/dist_tests.log 2>&1 || { tail -40 $O/dist_tests.log; exit 1; }
tail -1 $O/dist_tests.log
FEDML_AMD_BENCH_REHEARSAL=1 timeout -k 10 400 python bench.py --gpus 2 --params 12500000 --steps 3 --warmup 1 > $O/reh2.json 2> $O/reh2.err || { tail -30 $O/reh2.err; exit 1; }
cat $O/reh2.json
FEDML_AMD_BENCH_REHEARSAL=1 timeout -k 10 400 python bench.py --gpus 4 --params 12500000 --steps 3 --warmup 1 --config hier > $O/reh4h.json 2> $O/reh4h.err || { tail -30 $O/reh4h.err; exit 1; }
cat $O/reh4h.json
timeout -k 10 60 python bench.py --gpus 2 > $O/n2_refused.txt 2>&1; echo "N=2 on a 1-GPU box rc=$?"; tail -2 $O/n2_refused.txt
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
