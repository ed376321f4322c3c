# config 2: the 64-batch Get launch with a capped grid (PMDFC_GET_GRID blocks, looping) vs one block per 128 Gets
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r5z
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "config2_64M" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
PMDFC_GET_GRID=4096 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "config2_64M" >> $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
for g in 0 2048 4096 8192 16384; do
  PMDFC_GET_GRID=$g timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/c2_g$g.$i.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('$O/c2_g$g.$i.json'));print('grid $g',d['value'],d['ms_per_step'],d['kernel_ms_per_step']['get'], d['roofline']['random_access_roofline']['step_frac'])"
done
done
