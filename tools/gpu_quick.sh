# quick GPU iteration: the parity suite of the insert path, the headline bench,
# then (QUICK_TRACE=1) a kernel trace of one non-pipelined step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py ${QUICK_K:+-k "$QUICK_K"} > gpurun_out/q_tests.log 2>&1; rc=$?; tail -3 gpurun_out/q_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/q_bench.json 2> gpurun_out/q_bench.err || exit 1
python3 -c "
import json; d=json.loads(open('gpurun_out/q_bench.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['correct'], d['kernel_ms_per_step'])
for k,v in d['roofline']['per_kernel'].items(): print(' ', k, v['avg_launch_us'], v['frac'])
"
[ "${QUICK_TRACE:-0}" = 1 ] && bash tools/gpu_trace.sh
exit 0
