# round 4: the parity tests of the new first passes, then the bench lines they move
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r4
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "wide or upsert or alternate or split_loss" > gpurun_out/r4/tests.log 2>&1; rc=$?; tail -2 gpurun_out/r4/tests.log; [ $rc -eq 0 ] || exit $rc
for c in "" "--upsert" "--config 3" "--config 4" "--init-cap 2" "--route"; do
  tag=$(echo "c2 $c" | tr -d ' -')
  timeout -k 10 400 python -u bench.py --no-cpu-baseline $c > gpurun_out/r4/bench_$tag.json 2> gpurun_out/r4/bench_$tag.err || exit 1
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/r4/bench_$tag.json').read().strip().splitlines()[-1])
print('$tag', d['value'], d.get('ms_per_step'), d.get('correct'), d.get('kernel_ms_per_step'), d.get('index',{}).get('fast_declined_buckets'))"
done
