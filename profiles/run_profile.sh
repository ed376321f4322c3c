#!/bin/bash
# Collects the rocprofv3 evidence committed under profiles/ (run on the GPU box
# from the repo root).  Counter passes are separate from the trace pass and
# never combined with sys/runtime/hip traces (MI355X_MICROARCH.md HBM section).
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_${1:-r01}
mkdir -p $OUT
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d $OUT/trace -o run -- $B > $OUT/bench_trace.json 2> $OUT/bench_trace.err
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -f csv --kernel-include-regex "k_get|k_process|k_split" -d $OUT/pmc_fetch -o run -- $B > /dev/null 2> $OUT/pmc_fetch.err
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -f csv --kernel-include-regex "k_get|k_process|k_split" -d $OUT/pmc_write -o run -- $B > /dev/null 2> $OUT/pmc_write.err
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_HIT_sum TCC_MISS_sum -T -f csv --kernel-include-regex "k_get" -d $OUT/pmc_ea -o run -- $B > /dev/null 2> $OUT/pmc_ea.err || true
echo done
