#!/bin/bash
# Collects the rocprofv3 evidence committed under profiles/<round>/ (run on the
# GPU box from the repo root: bash profiles/run_profile.sh r02).
#  1. kernel trace + stats of the bench's own config-2 step, batch by batch
#     (--no-pipeline: no kernel overlaps another, so each kernel's average
#     duration is comparable with the bench's HIP-event classes);
#  2. FETCH_SIZE and WRITE_SIZE, each in its own --pmc pass (never combined
#     with a trace domain; MI355X_MICROARCH.md rocprofv3 / HBM sections), over
#     the same full 64-batch config-2 run, summarised per kernel by
#     tools/pmc_summary.py (KiB -> bytes, FETCH_SIZE doubled on gfx950).
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
R=${1:-r03}
OUT=gpurun_out/prof_$R
mkdir -p $OUT
B="python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-pipeline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d $OUT/trace -o run -- $B > $OUT/bench_trace.json 2> $OUT/bench_trace.err
echo "trace done"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -T -f csv -d $OUT/pmc_fetch -o run -- $B > $OUT/pmc_fetch.json 2> $OUT/pmc_fetch.err
echo "fetch done"
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -T -f csv -d $OUT/pmc_write -o run -- $B > $OUT/pmc_write.json 2> $OUT/pmc_write.err
echo "write done"
python3 tools/pmc_summary.py $OUT/pmc_config2.json $OUT/pmc_fetch $OUT/pmc_write > /dev/null
ls -R $OUT | head -40
