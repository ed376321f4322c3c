set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5s
timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r5s/bench.json 2> gpurun_out/r5s/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d gpurun_out/r5s/tr -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r5s/bench_tr.json 2> gpurun_out/r5s/bench_tr.err || exit 1
f=$(ls gpurun_out/r5s/tr/*/run_kernel_trace.csv gpurun_out/r5s/tr/run_kernel_trace.csv 2>/dev/null | head -n1)
python3 tools/trace_gaps.py "$f" > gpurun_out/r5s/gaps.txt
python3 tools/trace_overlap.py "$f" > gpurun_out/r5s/overlap.txt
cat gpurun_out/r5s/bench.json gpurun_out/r5s/gaps.txt gpurun_out/r5s/overlap.txt
