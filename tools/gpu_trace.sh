# kernel trace of one non-pipelined config-2 step, per-batch breakdown
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/tr
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/tr -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-pipeline > gpurun_out/tr/bench.json 2> gpurun_out/tr/bench.err
python3 tools/trace_batches.py gpurun_out/tr/run_kernel_trace.csv
