# arrival path pack: native (C++ threads) vs torch copy_ (OpenMP) vs torch + OMP_WAIT_POLICY=PASSIVE
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r02ah
timeout -k 10 600 python -u -m pytest tests/test_gpu_ingest.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02ah/tests.log 2>&1 || { tail -40 gpurun_out/r02ah/tests.log; exit 1; }
tail -1 gpurun_out/r02ah/tests.log
for M in native torch; do
 FEDML_AMD_PACK=$M PROBE_SPLIT=1 timeout -k 10 300 python tools/arrival_probe.py > gpurun_out/r02ah/p_$M.json 2>gpurun_out/r02ah/s_$M.txt || { tail -5 gpurun_out/r02ah/s_$M.txt; exit 1; }
 echo $M $(cat gpurun_out/r02ah/p_$M.json) $(grep resident gpurun_out/r02ah/s_$M.txt)
done
OMP_WAIT_POLICY=PASSIVE FEDML_AMD_PACK=torch PROBE_SPLIT=1 timeout -k 10 300 python tools/arrival_probe.py > gpurun_out/r02ah/p_passive.json 2>gpurun_out/r02ah/s_passive.txt || exit 1
echo torch_passive $(cat gpurun_out/r02ah/p_passive.json) $(grep resident gpurun_out/r02ah/s_passive.txt)
for T in 4 16; do
 FEDML_AMD_PACK_THREADS=$T timeout -k 10 300 python tools/arrival_probe.py > gpurun_out/r02ah/p_t$T.json 2>/dev/null || exit 1
 echo native_threads$T $(cat gpurun_out/r02ah/p_t$T.json)
done
