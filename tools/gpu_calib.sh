# counter calibration: FETCH_SIZE and WRITE_SIZE (separate passes) over
# kernels of known byte counts (tools/calib_fetch.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/calib
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -T -f csv -d $O/fetch -o run -- python3 tools/calib_fetch.py > $O/plan.json 2> $O/fetch.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -T -f csv -d $O/write -o run -- python3 tools/calib_fetch.py > $O/plan_w.json 2> $O/write.err || exit 1
python3 tools/calib_summary.py $O/calibration.json $O/plan.json $O/fetch $O/write
