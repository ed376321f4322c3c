# k_split_park data loss: which path (team / fences / off)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r5ab
mkdir -p $O
T="tests/test_gpu_cbf.py::test_cbf_feeds_fused_probe_then_get tests/test_gpu_parity.py::test_insert_batches_equals_batch_by_batch"
for v in "PMDFC_SPLIT_PARK=0" "PMDFC_SPLIT_PARK=1" "PMDFC_SPLIT_TEAM_MAX=0" "PMDFC_SPLIT_TEAM_MAX=100000" "PMDFC_LIB=pmdfc_amd/lib/ab/fenceall/libpmdfc_cceh.so" "PMDFC_LIB=pmdfc_amd/lib/ab/fenceall/libpmdfc_cceh.so PMDFC_SPLIT_TEAM_MAX=0"; do
  env $v timeout -k 10 300 python3 -u -m pytest $T -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1; rc=$?
  echo "$v -> rc=$rc $(tail -1 $O/t.log)"
done
