set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/t3.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/t3.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_prof.log 2>&1; rc=$?; echo "prof rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcf -o run -- python3 tools/insert_run.py 24 > gpurun_out/pmcf.log 2>&1; echo "pmc fetch rc=$?"
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcw -o run -- python3 tools/insert_run.py 24 > gpurun_out/pmcw.log 2>&1; echo "pmc write rc=$?"
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-300; tail -1 gpurun_out/bench.log | grep -o '"kernel_ms_per_step[^}]*}'
