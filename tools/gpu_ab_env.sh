# A/B of config-2 bench lines under environment settings: one bench per
# argument ("VAR=value ..." or "-"), printed as value / ms per step / process class
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/ab
i=0
for cfg in "$@"; do
  i=$((i + 1))
  [ "$cfg" = "-" ] && cfg=""
  env $cfg timeout -k 10 300 python -u bench.py --no-cpu-baseline ${AB_ARGS:-} > gpurun_out/ab/b$i.json 2> gpurun_out/ab/b$i.err || exit 1
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/ab/b$i.json').read().strip().splitlines()[-1])
print(sys.argv[1] or '(default)', d['value'], d['ms_per_step'], d.get('kernel_ms_per_step', d.get('kernel_ms_events_pass')))" "$cfg"
done
