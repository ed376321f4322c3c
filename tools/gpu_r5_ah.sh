# mixed batches: inserted-key set sized from the last batch's insert count vs the whole allocation
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r5ah
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "mixed or split_loss" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for c in 3 4; do
for v in "X=1" "PMDFC_ISET_FULL=1" "X=1" "PMDFC_ISET_FULL=1"; do
  tag=$(echo "$v" | tr -dc 'A-Za-z0-9')
  env $v timeout -k 10 400 python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $O/c$c.$tag.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('$O/c$c.$tag.json').read().strip().splitlines()[-1]);e=d.get('kernel_ms_events_pass',{});print('c$c $v',d['value'],d['ms_per_step'],e.get('mixed_get'),e.get('prep'))"
done
done
