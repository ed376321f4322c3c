# config lines of bench.py under the current tree: config 2, 2 from CCEH_hybrid(2), 3, 4
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/abc
for c in "--config 2" "--config 2 --init-cap 2" "--config 3" "--config 4" ${AB_EXTRA:-}; do
  tag=$(echo "$c" | tr -dc 'a-z0-9')
  timeout -k 10 600 python -u bench.py $c --no-cpu-baseline > gpurun_out/abc/$tag.json 2> gpurun_out/abc/$tag.err || { echo "failed: $c"; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/abc/$tag.json').read().strip().splitlines()[-1])
print(sys.argv[1], d['value'], d['ms_per_step'], d.get('correct'), d.get('kernel_ms_per_step') or d.get('kernel_ms_events_pass'))" "$c"
done
