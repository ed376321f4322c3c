set -o pipefail
mkdir -p gpurun_out
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/ -q -m gpu -x --timeout 300 --timeout-method thread --durations=8 > gpurun_out/t2.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -40 gpurun_out/t2.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b2.json 2> gpurun_out/b2.err; rc=$?; echo "bench rc=$rc"; cat gpurun_out/b2.json; tail -5 gpurun_out/b2.err
