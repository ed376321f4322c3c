# mixed-path step: parity (insert/mixed fixtures + full-size config 3/4 shard), config 4 and 3 bench lines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_scale.py > gpurun_out/mx_tests.log 2>&1; rc=$?; tail -2 gpurun_out/mx_tests.log; [ $rc -eq 0 ] || exit $rc
for c in 4 3; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > gpurun_out/mx_c$c.json 2> gpurun_out/mx_c$c.err || exit 1
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['correct'], d.get('kernel_ms_per_step'))" gpurun_out/mx_c$c.json
done
