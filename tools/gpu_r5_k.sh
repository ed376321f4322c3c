# mixed batches: the key set emptied on a side stream + thread-per-op verify;
# parity of the mixed paths, then config 4 / 3 A/B against the previous tree
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r5k
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_serve.py tests/test_gpu_dist2.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for c in 4 3; do
  for v in new old new old; do
    L=""; [ $v = old ] && L=pmdfc_amd/lib/ab/pre_iclr/libpmdfc_cceh.so
    PMDFC_LIB=$L timeout -k 10 400 python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $O/c$c.$v.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.loads(open('$O/c$c.$v.json').read().strip().splitlines()[-1]);print('c$c $v',d['value'],d['ms_per_step'])"
  done
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -f csv -d $O/t4 -o run -- python3 bench.py --config 4 --steps 1 --warmup 0 --no-cpu-baseline > /dev/null 2> $O/t4.err || exit 1
head -16 $O/t4/run_kernel_stats.csv | cut -c1-120
