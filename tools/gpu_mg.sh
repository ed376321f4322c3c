# mixed Get A/B: mixed parity tests, then configs 4 and 3 at PMDFC_MG_U = 4, 2, 1
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_trace.py tests/test_gpu_scale.py > gpurun_out/mg_tests.log 2>&1; rc=$?; tail -2 gpurun_out/mg_tests.log; [ $rc -eq 0 ] || exit $rc
for u in 4 2 1; do
  for c in 4 3; do
    PMDFC_MG_U=$u timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > gpurun_out/mg_${u}_${c}.json 2> gpurun_out/mg_${u}_${c}.err || exit 1
    python3 -c "
import json,sys; d=json.loads(open('gpurun_out/mg_${u}_${c}.json').read().strip().splitlines()[-1])
print('U $u config $c', d['value'], d['ms_per_step'], d['correct'], d.get('kernel_ms_per_step') or '')
"
  done
done
