# k_split_park, team-only splits (2 waves/SIMD, no spills): parity with it on, A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r5ad
mkdir -p $O
PMDFC_SPLIT_PARK=1 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cbf.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
for f in 1 0; do
  PMDFC_SPLIT_PARK=$f timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/c2_sp$f.$i.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('$O/c2_sp$f.$i.json'));print('split_park=$f',d['value'],d['ms_per_step'],d['kernel_ms_per_step'], d['roofline']['random_access_roofline']['step_frac'])"
done
done
