# round 5, final tree: the whole GPU suite with smoke, then the evidence
# (kernel trace + PMC passes of the bench's config-2 run, every bench line)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
bash tools/gpu_full_tests.sh || exit 1
bash tools/gpu_evidence.sh r05 || exit 1
echo "final done"
