# round 5 final tree, part 1: the whole GPU suite + smoke, then the kernel
# trace and PMC passes of the bench's own config-2 run (tools/run_profile.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
bash tools/gpu_full_tests.sh || exit 1
bash tools/run_profile.sh r05 > gpurun_out/prof_r05.log 2>&1 || { tail -5 gpurun_out/prof_r05.log; exit 1; }
echo "profile done"
