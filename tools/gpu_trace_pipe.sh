# kernel trace of one PIPELINED config-2 step (the insert pipeline as the
# headline runs it), per-batch timeline of the bucket passes; env for A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/trpipe${TRP_TAG:-}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
python3 tools/trace_pipe.py $O/run_kernel_trace.csv > $O/timeline.txt
tail -1 $O/timeline.txt
