# r05ze: the final HEAD binary: the whole GPU suite, smoke(), cfg2 lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05ze; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1].split('/')[-1],d['value'],d['unit'],d['ms_per_step'],r.get('kernel_avg_ms'),r.get('frac'),d.get('parity'))" $1; }
for c in tensors tiled; do
  timeout -k 10 300 python bench.py --config resnet18 --layout $c --steps 100 --warmup 400 --no-cpu-baseline --soak-seconds 0 > $O/cfg2_$c.json 2> $O/cfg2_$c.err || { tail -5 $O/cfg2_$c.err; exit 1; }
  line $O/cfg2_$c.json
done
