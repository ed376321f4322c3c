# kernel trace of the routed config-2 path on one rank (bench --route): where
# the step goes beyond the engine's own kernels (pack, RCCL, unpack, host gaps)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/rtr
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/rtr -o run -- python3 bench.py --route --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/rtr/bench.json 2> gpurun_out/rtr/bench.err || exit 1
f=$(find gpurun_out/rtr -name 'run_kernel_trace.csv' | head -1)
python3 tools/trace_busy.py "$f" --from-kernel k_init_segments > gpurun_out/rtr/busy.txt && cat gpurun_out/rtr/busy.txt
