set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/t3.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/t3.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/phase_stamps.py 46 > gpurun_out/stamps.log 2>&1; rc=$?; echo "stamps rc=$rc"; grep -v amdgpu.ids gpurun_out/stamps.log | tail -22
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-300; tail -1 gpurun_out/bench.log | grep -o '"kernel_ms_per_step[^}]*}'
