# occ-merge A/B + parity subset + hosted world-2 native tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5c
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "config2 or small_batches_exact or insert_batches or mixed_matches" > gpurun_out/r5c/parity.log 2>&1 || { tail -30 gpurun_out/r5c/parity.log; exit 1; }
tail -2 gpurun_out/r5c/parity.log
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_dist2.py -x -v --timeout 200 --timeout-method thread -k host_staged > gpurun_out/r5c/dist2.log 2>&1; echo "dist2 rc $?"; tail -8 gpurun_out/r5c/dist2.log
for i in 1 2; do
for m in 0 1; do
PMDFC_OCC_MERGE=$m timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r5c/bench_m$m.$i.json 2>/dev/null || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/r5c/bench_m$m.$i.json'));print('merge',$m,d['value'],d['ms_per_step'],d['kernel_ms_per_step'])"
done; done
