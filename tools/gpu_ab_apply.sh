# the insert parity suite, then config 2 with the lean first pass and without (A/B), then a kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/ab
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/ab/tests.log 2>&1; rc=$?; tail -2 gpurun_out/ab/tests.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0; do
  PMDFC_FAST_APPLY=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/ab/bench_fast$v.json 2> gpurun_out/ab/bench_fast$v.err || exit 1
  python3 -c "
import json; d=json.loads(open('gpurun_out/ab/bench_fast$v.json').read().strip().splitlines()[-1])
print('fast=$v', d['value'], d['ms_per_step'], d['correct'], d['kernel_ms_per_step'])"
done
bash tools/gpu_trace.sh
