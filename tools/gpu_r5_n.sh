# timeline of pipelined config-2 insert batches (in-kernel stamps)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r5n
mkdir -p $O
timeout -k 10 300 python3 -u tools/timeline.py 40 8 > $O/timeline.txt 2>&1; rc=$?; cat $O/timeline.txt; exit $rc
