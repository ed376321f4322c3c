set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -q -m gpu -x --timeout 300 --timeout-method thread --durations=8 > gpurun_out/t1.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -25 gpurun_out/t1.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 > gpurun_out/b1.json 2> gpurun_out/b1.err; rc=$?; echo "bench rc=$rc"; cat gpurun_out/b1.json; tail -5 gpurun_out/b1.err
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bprof.json 2> gpurun_out/bprof.err; echo "prof rc=$?"
find gpurun_out/prof -name "*stats*" | head
