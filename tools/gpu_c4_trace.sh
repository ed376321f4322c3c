# kernel trace + stats of one config-4 step on one GPU (direct engine)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/c4tr
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d $OUT -o run -- python3 bench.py --config 4 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 1
head -40 $OUT/run_kernel_stats.csv | cut -d, -f1-4
