# r03j: SecAgg mask kernel v2 (out-of-place generation) parity + timing; Krum defaults (NPL 16 lane); PMC + kernel stats for both
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r03j; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_finite.py -x -q --timeout 120 --timeout-method thread -k "mt_randint or mask" > $O/finite.log 2>&1 || { tail -40 $O/finite.log; exit 1; }
tail -1 $O/finite.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_robust.py -x -q --timeout 120 --timeout-method thread -k "pair or krum" > $O/robust.log 2>&1 || { tail -40 $O/robust.log; exit 1; }
tail -1 $O/robust.log
for D in 0 4; do
  timeout -k 10 300 python bench.py --config samask --variant $D --steps 5 --warmup 1 > $O/samask_d$D.json 2> $O/samask_d$D.err || { tail -5 $O/samask_d$D.err; exit 1; }
  python -c "import json;d=json.load(open('$O/samask_d$D.json'));print('samask d$D', d['value'], d['cpu_baseline']['value'], d['parity'][:40])"
done
for K in 16 32 64 100 128; do
  timeout -k 10 120 python bench.py --config krum --clients $K --no-cpu-baseline --steps 10 --warmup 2 > $O/krum_K$K.json 2> $O/krum_K$K.err || { tail -3 $O/krum_K$K.err; exit 1; }
  python -c "import json;d=json.load(open('$O/krum_K$K.json'));print('krum', $K, d['roofline']['kernel_avg_ms'], d['parity'][:40])"
done
for K in 32 128; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt_krum_K$K -o kt --output-format csv -- python3 bench.py --config krum --clients $K --no-cpu-baseline --check-samples 0 --steps 5 --warmup 1 > $O/kt_krum_K$K.log 2>&1 || { tail -5 $O/kt_krum_K$K.log; exit 1; }
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt_samask -o kt --output-format csv -- python3 bench.py --config samask --steps 3 --warmup 1 --no-cpu-baseline > $O/kt_samask.log 2>&1 || { tail -5 $O/kt_samask.log; exit 1; }
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU"
B="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD"
for K in 32 128; do
  timeout -s KILL 90 rocprofv3 --pmc $A --kernel-include-regex k_pairdist -d $O/pa_K$K -o pmc --output-format csv -- python3 bench.py --config krum --clients $K --no-cpu-baseline --check-samples 0 --steps 2 --warmup 1 > $O/pa_K$K.log 2>&1 || { echo FAIL A $K; tail -5 $O/pa_K$K.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc $B --kernel-include-regex k_pairdist -d $O/pb_K$K -o pmc --output-format csv -- python3 bench.py --config krum --clients $K --no-cpu-baseline --check-samples 0 --steps 2 --warmup 1 > $O/pb_K$K.log 2>&1 || { echo FAIL B $K; tail -5 $O/pb_K$K.log; exit 1; }
done
echo done
