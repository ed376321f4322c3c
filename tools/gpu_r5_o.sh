# config 2 with the Get batches as one launch (GetBatches) vs one Get per batch
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r5o
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "config2_64M or mixed_batches or insert_batches" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_gb.$i.json 2>/dev/null || exit 1
python3 -c "import json;d=json.load(open('$O/bench_gb.$i.json'));print('getbatches',d['value'],d['ms_per_step'],d['kernel_ms_per_step'], d['roofline']['random_access_roofline']['step_frac'])"
PMDFC_LIB=pmdfc_amd/lib/ab/pergets/libpmdfc_cceh.so timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_pg.$i.json 2>/dev/null || exit 1
python3 -c "import json;d=json.load(open('$O/bench_pg.$i.json'));print('per-batch',d['value'],d['ms_per_step'],d['kernel_ms_per_step'], d['roofline']['random_access_roofline']['step_frac'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d $O/t2 -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > /dev/null 2> $O/t2.err || exit 1
head -12 $O/t2/run_kernel_stats.csv | cut -c1-110
