# k_mixed_get: Gets per quad issued together (PMDFC_MG_U 1 / 2 / 4) on the final tree
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r5aq
mkdir -p $O
for c in 4 3; do
for v in "X=1" "PMDFC_MG_U=1" "PMDFC_MG_U=4" "X=1" "PMDFC_MG_U=1" "PMDFC_MG_U=4"; do
  tag=$(echo "$v" | tr -dc 'A-Za-z0-9')
  env $v timeout -k 10 400 python3 bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline > $O/c$c.$tag.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('$O/c$c.$tag.json').read().strip().splitlines()[-1]);print('c$c $v',d['value'],d['ms_per_step'],d.get('kernel_ms_events_pass',{}).get('mixed_get'))"
done
done
