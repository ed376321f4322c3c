# full GPU suite + smoke, then config-2 (headline), upsert, 5 and 4 bench lines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/fin
bash tools/gpu_full_tests.sh || exit 1
for c in "" "--config 2 --upsert --no-cpu-baseline" "--config 5 --no-cpu-baseline" "--config 4 --no-cpu-baseline"; do
  tag=$(echo "c$c" | tr -dc 'a-z0-9')
  timeout -k 10 600 python -u bench.py $c > gpurun_out/fin/bench_$tag.json 2> gpurun_out/fin/bench_$tag.err || { echo "failed: $c"; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['correct'])" gpurun_out/fin/bench_$tag.json
done
