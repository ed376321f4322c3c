# round-3 starting point: the new parity tests, the config-2 line and an SQ
# counter pass over the insert kernels
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r03base
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "find_anyway or split_loss or mixed" tests/test_gpu_dropin.py > gpurun_out/r03base/tests.log 2>&1 || { tail -30 gpurun_out/r03base/tests.log; exit 1; }
tail -2 gpurun_out/r03base/tests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r03base/bench.json 2> gpurun_out/r03base/bench.err || exit 1
echo bench ok
bash tools/gpu_pmc_sq.sh > gpurun_out/r03base/sq.log 2>&1 || exit 1
cp -r gpurun_out/sq gpurun_out/r03base/
echo sq ok
