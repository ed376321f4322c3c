# mixed-batch iteration: parity of every mixed path, then configs 4, 3 and 2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_trace.py tests/test_gpu_scale.py tests/test_gpu_route.py tests/test_gpu_extent.py > gpurun_out/m_tests.log 2>&1; rc=$?; tail -2 gpurun_out/m_tests.log; [ $rc -eq 0 ] || exit $rc
for c in 4 3 2; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > gpurun_out/m_bench$c.json 2> gpurun_out/m_bench$c.err || exit 1
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/m_bench$c.json').read().strip().splitlines()[-1])
print('config $c', d['value'], d['ms_per_step'], d['correct'], d.get('kernel_ms_per_step') or d.get('kernel_ms_events_pass'))
"
done
