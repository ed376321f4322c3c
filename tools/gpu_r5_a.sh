set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5a
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_serve.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r5a/serve.log 2>&1
rc=$?
tail -5 gpurun_out/r5a/serve.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r5a/bench.json 2> gpurun_out/r5a/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d gpurun_out/r5a/tr -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r5a/bench_tr.json 2> gpurun_out/r5a/bench_tr.err || exit 1
f=$(ls gpurun_out/r5a/tr/*/run_kernel_trace.csv gpurun_out/r5a/tr/run_kernel_trace.csv 2>/dev/null | head -n1)
python3 tools/trace_gaps.py "$f" > gpurun_out/r5a/gaps.txt
python3 tools/trace_overlap.py "$f" > gpurun_out/r5a/overlap.txt
cat gpurun_out/r5a/bench.json gpurun_out/r5a/gaps.txt gpurun_out/r5a/overlap.txt
exit $rc
