# smaller k_split / k_apply_parked / k_bucket grids (one dispatch round): A/B on config 2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r5p
mkdir -p $O
for i in 1 2; do
for v in base grids grids2; do
  L=""; [ $v != base ] && L=pmdfc_amd/lib/ab/$v/libpmdfc_cceh.so
  PMDFC_LIB=$L timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_$v.$i.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('$O/bench_$v.$i.json'));print('$v',d['value'],d['ms_per_step'],d['kernel_ms_per_step'], d['roofline']['random_access_roofline']['step_frac'])"
done
done
PMDFC_LIB=pmdfc_amd/lib/ab/grids/libpmdfc_cceh.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "config2_64M or insert_batches or split_loss or mixed_matches or wide" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
