# kernel trace of config 4 (which first-pass kernels run, their durations)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r5am
mkdir -p $O
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -f csv -d $O/t -o run -- python3 bench.py --config 4 --steps 2 --warmup 1 --no-cpu-baseline > $O/b.json 2> $O/t.err || exit 1
find $O/t -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
cut -d, -f1-7 $O/kernel_stats.csv | head -40
