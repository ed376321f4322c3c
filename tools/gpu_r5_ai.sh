# pipelined Get launch (k_get_pipe): full GPU suite with a small resident grid (many rounds, tails), then config 2 A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r5ai
mkdir -p $O
PMDFC_GET_PIPE=16 timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests16.log 2>&1 || { tail -30 $O/tests16.log; exit 1; }
tail -1 $O/tests16.log
for v in "X=1" "PMDFC_GET_PIPE=2048" "PMDFC_GET_PIPE=1024" "X=1" "PMDFC_GET_PIPE=2048" "PMDFC_GET_PIPE=1024"; do
  tag=$(echo "$v" | tr -dc 'A-Za-z0-9')
  env $v timeout -k 10 400 python3 bench.py --config 2 --steps 5 --warmup 1 --no-cpu-baseline > $O/c2.$tag.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('$O/c2.$tag.json').read().strip().splitlines()[-1]);e=d.get('kernel_ms_per_step',{});print('c2 $v',d['value'],d['ms_per_step'],e.get('get'),d.get('get_mops'))"
done
