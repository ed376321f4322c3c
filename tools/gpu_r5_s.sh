# the ramp (CCEH_hybrid(2)): grids and the fused final pass; config 2 unaffected
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r5s
mkdir -p $O
for f in 1 0 2; do
  PMDFC_FUSE_FINAL=$f timeout -k 10 400 python3 bench.py --config 2 --init-cap 2 --steps 2 --warmup 1 --no-cpu-baseline > $O/ic2_f$f.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('$O/ic2_f$f.json').read().strip().splitlines()[-1]);print('ic2 fuse=$f',d['value'],d['ms_per_step'],d.get('kernel_ms_per_step'))"
done
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench.$i.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('$O/bench.$i.json'));print('config2',d['value'],d['ms_per_step'],d['kernel_ms_per_step'], d['roofline']['random_access_roofline']['step_frac'])"
done
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_serve.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
