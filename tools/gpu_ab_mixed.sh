# A/B of the mixed-batch lines (configs 3 and 4) under environment settings:
# one bench per (argument, config), interleaved; "-" = the tree's own library
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/abm
i=0
for cfg in "$@"; do
  for c in ${AB_CONFIGS:-3 4}; do
    i=$((i + 1))
    [ "$cfg" = "-" ] && cfg=""
    env $cfg timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline ${AB_ARGS:-} > gpurun_out/abm/m$i.json 2> gpurun_out/abm/m$i.err || exit 1
    python3 -c "
import json,sys; d=json.loads(open('gpurun_out/abm/m$i.json').read().strip().splitlines()[-1])
print(sys.argv[1] or '(default)', 'config $c', d['value'], d.get('correct'), d.get('kernel_ms_events_pass'))" "$cfg"
  done
done
