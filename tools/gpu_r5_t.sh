# the CCEH_hybrid(2) ramp line x2 (ramp grids as round 4), config 2 x1, fused-final parity (PMDFC_FUSE_FINAL=2)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r5t
mkdir -p $O
for i in 1 2; do
  timeout -k 10 400 python3 bench.py --config 2 --init-cap 2 --steps 2 --warmup 1 --no-cpu-baseline > $O/ic2.$i.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('$O/ic2.$i.json').read().strip().splitlines()[-1]);print('ic2',d['value'],d['ms_per_step'],d.get('kernel_ms_per_step'))"
done
timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench.json 2>/dev/null || exit 1
python3 -c "import json;d=json.load(open('$O/bench.json'));print('config2',d['value'],d['ms_per_step'],d['kernel_ms_per_step'], d['roofline']['random_access_roofline']['step_frac'])"
PMDFC_FUSE_FINAL=2 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/tests_fused.log 2>&1 || { tail -30 $O/tests_fused.log; exit 1; }
tail -2 $O/tests_fused.log
