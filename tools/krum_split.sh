# k_pairdist: robust GPU tests, then timings over K (FA_PAIR_SPLIT="esplit" overrides; "-" = built-in)
# for this build and, if present, tools/var/lib_old.so (the previous build) on the same box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_robust.py -x -q --timeout 120 --timeout-method thread > gpurun_out/krum_tests.log 2>&1 || { tail -30 gpurun_out/krum_tests.log; exit 1; }
tail -1 gpurun_out/krum_tests.log
r() { if [ "$2" = "-" ]; then unset FA_PAIR_SPLIT; else export FA_PAIR_SPLIT=$2; fi
      timeout -k 10 120 python bench.py --config krum --clients $1 --no-cpu-baseline --check-samples 0 --steps 8 --warmup 2 > gpurun_out/ks.json 2>gpurun_out/ks.err || { echo FAIL $1 $2; tail -3 gpurun_out/ks.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/ks.json'));print('$V', 'K=$1', 'split=$2', d['roofline']['kernel_avg_ms'])"; }
V=new
for s in ${S8:-- 128 256 341}; do r 8 $s; done
for s in ${S16:-- 50 100}; do r 16 $s; done
for s in ${S32:-- 14 21 28}; do r 32 $s; done
for s in ${S64:-- 5 6 7}; do r 64 $s; done
for s in ${S100:-- 3}; do r 100 $s; done
for s in ${S128:--}; do r 128 $s; done
if [ -n "$OLD" ] && [ -f tools/var/lib_old.so ]; then V=old; cp tools/var/lib_old.so fedml_amd/libfedagg.so; for K in 8 32 64 128; do r $K -; done; fi
