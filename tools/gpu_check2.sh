# checkpoint: the whole GPU suite, then config 2, config 4 and config 3 lines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
bash tools/gpu_full_tests.sh || exit 1
for args in "" "--config 4" "--config 3"; do
  tag=$(echo "x$args" | tr -dc 'a-z0-9')
  timeout -k 10 400 python -u bench.py $args --no-cpu-baseline > gpurun_out/c_$tag.json 2> gpurun_out/c_$tag.err || exit 1
  python3 -c "
import json; d=json.loads(open('gpurun_out/c_$tag.json').read().strip().splitlines()[-1])
print('$args', d['value'], d['ms_per_step'], d['correct'], d.get('kernel_ms_per_step'))
"
done
