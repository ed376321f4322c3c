# kernel traces of config 4 (one mixed step) and of one non-pipelined config-2 step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/gpu_c4_trace.sh || exit 1
bash tools/gpu_trace.sh || exit 1
