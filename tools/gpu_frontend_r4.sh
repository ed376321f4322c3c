# round 4: the served front-end (persistent wave) -- our C++ harness, then the
# reference front-ends over it, then the 32-caller bench (and 8 callers, and
# 32 callers that yield at once)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r4
timeout -k 10 60 ./pmdfc_amd/lib/test_gpu_kv 200000 8 > gpurun_out/r4/test_gpu_kv.log 2>&1; rc=$?; tail -16 gpurun_out/r4/test_gpu_kv.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_dropin.py > gpurun_out/r4/dropin.log 2>&1; rc=$?; tail -3 gpurun_out/r4/dropin.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 ./pmdfc_amd/lib/bench_frontend 32 16384 > gpurun_out/r4/frontend.json 2> gpurun_out/r4/frontend.err; rc=$?; tail -c 1500 gpurun_out/r4/frontend.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 ./pmdfc_amd/lib/bench_frontend 8 32768 > gpurun_out/r4/frontend_t8.json 2>> gpurun_out/r4/frontend.err || exit 1
timeout -k 10 300 ./pmdfc_amd/lib/bench_frontend 16 16384 > gpurun_out/r4/frontend_t16.json 2>> gpurun_out/r4/frontend.err || exit 1
echo frontend variants done
