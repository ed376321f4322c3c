# routing: packer/dedupe parity, the routed full-size config-4 shard and
# config-3 tests, then the routed one-GPU bench lines (--route: a 1-rank RCCL group)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_route.py tests/test_gpu_scale.py > gpurun_out/route_tests.log 2>&1; rc=$?
tail -4 gpurun_out/route_tests.log; [ $rc -eq 0 ] || exit $rc
grep -E "PASSED|FAILED" gpurun_out/route_tests.log | grep -E "scale" || true
timeout -k 10 300 python -u bench.py --config 4 --route --no-cpu-baseline > gpurun_out/route_c4.json 2> gpurun_out/route_c4.err || exit 1
timeout -k 10 300 python -u bench.py --config 2 --route --no-cpu-baseline > gpurun_out/route_c2.json 2> gpurun_out/route_c2.err || exit 1
python3 - <<'PY'
import json
for f in ("route_c4", "route_c2"):
    d = json.loads(open(f"gpurun_out/{f}.json").read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d["correct"], d.get("route_overflow_ops"))
PY
