# one perf step: GPU parity (insert + mixed paths), the headline bench, optional config-4 line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/s_tests.log 2>&1; rc=$?; tail -3 gpurun_out/s_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/s_bench.json 2> gpurun_out/s_bench.err || exit 1
python3 -c "
import json; d=json.loads(open('gpurun_out/s_bench.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['correct'], d['kernel_ms_per_step'])
for k,v in d['roofline']['per_kernel'].items(): print(' ', k, v['avg_launch_us'], v['frac'])
"
if [ "${STEP_C4:-0}" = 1 ]; then
  timeout -k 10 300 python -u bench.py --config 4 --no-cpu-baseline > gpurun_out/s_bench4.json 2> gpurun_out/s_bench4.err || exit 1
  tail -c 400 gpurun_out/s_bench4.json
fi
exit 0
