# k_get_pipe with 4 Gets per quad and round vs k_get_u (config 2)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r5aj
mkdir -p $O
for v in "X=1" "PMDFC_GET_PIPE=2048 PMDFC_GET_UNROLL=4" "PMDFC_GET_UNROLL=4" "X=1" "PMDFC_GET_PIPE=2048 PMDFC_GET_UNROLL=4" "PMDFC_GET_UNROLL=4"; do
  tag=$(echo "$v" | tr -dc 'A-Za-z0-9')
  env $v timeout -k 10 400 python3 bench.py --config 2 --steps 5 --warmup 1 --no-cpu-baseline > $O/c2.$tag.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('$O/c2.$tag.json').read().strip().splitlines()[-1]);e=d.get('kernel_ms_per_step',{});print('c2 $v',d['value'],d['ms_per_step'],e.get('get'),d.get('get_mops'))"
done
