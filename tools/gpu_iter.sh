# one perf iteration: insert-path parity, the headline bench, phase stamps of batch 45
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/q_tests.log 2>&1; rc=$?; tail -2 gpurun_out/q_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/q_bench.json 2> gpurun_out/q_bench.err || exit 1
python3 -c "
import json; d=json.loads(open('gpurun_out/q_bench.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['correct'], d['kernel_ms_per_step'])
for k,v in d['roofline']['per_kernel'].items(): print(' ', k, v['avg_launch_us'], v['frac'])
"
timeout -k 10 300 python3 tools/phase_stamps.py 45 > gpurun_out/stamps.txt 2>&1 || exit 1
grep -A30 "^k_apply" gpurun_out/stamps.txt | head -28
