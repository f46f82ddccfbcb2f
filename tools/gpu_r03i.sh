# r03i: finite (SecAgg mask) tests, SecAgg mask bench, then the Krum A/B (r03g)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r03i; mkdir -p $O




for D in 0 4; do
  timeout -k 10 300 python bench.py --config samask --variant $D --steps 5 --warmup 1 > $O/samask_d$D.json 2> $O/samask_d$D.err || { tail -5 $O/samask_d$D.err; exit 1; }
  cat $O/samask_d$D.json
done
bash tools/gpu_r03g.sh
