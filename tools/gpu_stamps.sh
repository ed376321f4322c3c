# per-phase wave timing of the insert kernels (debug stamps), config-2 shape
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/phase_stamps.py ${STAMP_BATCHES:-46} > gpurun_out/stamps.txt 2>&1; rc=$?; cat gpurun_out/stamps.txt; exit $rc
