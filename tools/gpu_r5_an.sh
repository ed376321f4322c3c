# kernel trace of the CCEH_hybrid(2) ramp (config 2 from 2 segments), batch by batch
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r5an
mkdir -p $O
timeout -s KILL 300 rocprofv3 --kernel-trace -f csv -d $O/t -o run -- python3 bench.py --config 2 --init-cap 2 --steps 1 --warmup 0 --no-cpu-baseline --no-pipeline > $O/b.json 2> $O/t.err || exit 1
find $O/t -name "*kernel_trace.csv" -exec cp {} $O/kernel_trace.csv \;
rm -rf $O/t
ls -la $O
