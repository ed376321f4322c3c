set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/trp
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d gpurun_out/trp -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/trp/bench.json 2> gpurun_out/trp/bench.err || exit 1
python3 tools/trace_overlap.py gpurun_out/trp/run_kernel_trace.csv
