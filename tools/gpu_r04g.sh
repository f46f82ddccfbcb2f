# r04g: VALU rate probe of the pair step (plain / DPP / DPP interleaved / packed), then k_pairdist_rot
# with interleaved difference pairs: pair tests + Krum A/B at K = 32 / 128 (rot vs tile).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r04g; mkdir -p $O
hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize -o /tmp/dpp_rate_probe tools/dpp_rate_probe.hip 2>/dev/null || { echo "probe build FAIL"; exit 1; }
timeout -k 10 120 /tmp/dpp_rate_probe > $O/dpp_rate_probe.txt 2>&1 || { echo "probe FAIL"; cat $O/dpp_rate_probe.txt; exit 1; }
cat $O/dpp_rate_probe.txt
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_robust.py -k "pair or krum" > $O/pytest_rot.txt 2>&1 \
  || { echo "pytest rot FAIL"; tail -40 $O/pytest_rot.txt; exit 1; }
tail -1 $O/pytest_rot.txt
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[1],d['value'],d['unit'],d['ms_per_step'],r.get('kernel_avg_ms'),r.get('frac'),'|',d.get('parity'))" $1; }
for K in 32 128; do
  for v in 1 0; do
    n=krum_K${K}_rot${v}
    FA_PAIR_ROT=$v timeout -k 10 300 python bench.py --config krum --clients $K --steps 20 --warmup 3 --no-cpu-baseline > $O/$n.json 2> $O/$n.err \
      || { echo "FAIL $n"; tail -8 $O/$n.err; exit 1; }
    line $O/$n.json
  done
done
