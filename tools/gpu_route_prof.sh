# kernel trace + stats of the routed config-2 / config-4 lines on one GPU (1-rank RCCL group)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_route
mkdir -p $OUT
for c in 2 4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d $OUT/c$c -o run -- python3 bench.py --config $c --route --steps 1 --warmup 1 --no-cpu-baseline > $OUT/c$c.json 2> $OUT/c$c.err || exit 1
done
for c in 2 4; do
  f=$(find $OUT/c$c -name "*kernel_stats.csv" | head -1)
  echo "== config $c"; head -16 "$f" | cut -d, -f1-5
done
