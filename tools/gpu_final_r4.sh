# round 4, final tree: the front-end harness and benches, the whole GPU suite
# with smoke, then the evidence (trace, PMC passes, every bench line)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
bash tools/gpu_frontend_r4.sh > gpurun_out/final_fe.log 2>&1 || { echo "frontend failed"; tail -20 gpurun_out/final_fe.log; exit 1; }
echo "frontend ok"
bash tools/gpu_full_tests.sh || exit 1
bash tools/gpu_evidence.sh r04 || exit 1
echo "final done"
