# parity of the insert path + headline bench + phase stamps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/gpu_quick.sh || exit 1
bash tools/gpu_stamps.sh > /dev/null 2>&1; grep -A12 "k_apply" gpurun_out/stamps.txt
