# kernel trace of the per-op front-end (bench_frontend, 32 callers, short run):
# what one small batch costs on the GPU
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ftr
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/ftr -o fe -- ./pmdfc_amd/lib/bench_frontend 32 4096 > gpurun_out/ftr/fe.json 2> gpurun_out/ftr/fe.err
head -12 gpurun_out/ftr/fe_kernel_stats.csv
