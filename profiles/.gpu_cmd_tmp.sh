set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_prof.log 2>&1; rc=$?; echo "prof rc=$rc"; tail -2 gpurun_out/bench_prof.log | cut -c1-600
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/ -v -m gpu -x --timeout 300 --timeout-method thread --durations=12 > gpurun_out/t3.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -30 gpurun_out/t3.log
