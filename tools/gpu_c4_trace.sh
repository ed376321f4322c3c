# kernel traces of config 4 (one shard: 2^28 preloaded, 50/50 mixed batches),
# direct and through the 1-rank routed path, for the per-batch cost breakdown
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/c4
timeout -k 10 400 python3 bench.py --config 4 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/c4/direct.json 2> gpurun_out/c4/direct.err || exit 1
timeout -k 10 400 python3 bench.py --config 4 --route --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/c4/routed.json 2> gpurun_out/c4/routed.err || exit 1
timeout -k 10 500 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/c4/tr -o routed -- python3 bench.py --config 4 --route --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/c4/routed_tr.json 2> gpurun_out/c4/routed_tr.err || exit 1
head -30 gpurun_out/c4/tr/routed_kernel_stats.csv
