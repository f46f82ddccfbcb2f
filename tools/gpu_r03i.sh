# r03i: finite (SecAgg mask) tests, SecAgg mask bench, then the Krum A/B (r03g)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r03i; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_distributed.py -x -q --timeout 120 --timeout-method thread > $O/dist.log 2>&1 || { tail -40 $O/dist.log; exit 1; }
tail -1 $O/dist.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_finite.py -x -q --timeout 120 --timeout-method thread > $O/finite.log 2>&1 || { tail -40 $O/finite.log; exit 1; }
tail -1 $O/finite.log
for D in 0 4; do
  timeout -k 10 300 python bench.py --config samask --variant $D --steps 5 --warmup 1 > $O/samask_d$D.json 2> $O/samask_d$D.err || { tail -5 $O/samask_d$D.err; exit 1; }
  cat $O/samask_d$D.json
done
bash tools/gpu_r03g.sh
