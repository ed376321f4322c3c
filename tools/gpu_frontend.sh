# front-end: the drop-in harnesses (reference test_KV / replay_KV / NuMA_KV over
# the GPU backend, our C++ harness, 32 callers) and the config-8 line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dropin.py > gpurun_out/f_tests.log 2>&1; rc=$?; tail -3 gpurun_out/f_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config 8 --steps 2 > gpurun_out/f_bench8.json 2> gpurun_out/f_bench8.err || exit 1
python3 -c "
import json; d=json.loads(open('gpurun_out/f_bench8.json').read().strip().splitlines()[-1]); f=d['frontend']
print('value', d['value'], {k: f[k] for k in f if 'mops' in k or 'batch' in k}, 'cpu', d.get('cpu_baseline',{}).get('value'))
"
