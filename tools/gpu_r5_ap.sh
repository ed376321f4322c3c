# mixed batches: the gated mixed passes on small looping grids when the host expects them off
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r5ap
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for c in 4 3; do
for v in "X=1" "PMDFC_MIXED_SMALL=0" "X=1" "PMDFC_MIXED_SMALL=0"; do
  tag=$(echo "$v" | tr -dc 'A-Za-z0-9')
  env $v timeout -k 10 400 python3 bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline > $O/c$c.$tag.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('$O/c$c.$tag.json').read().strip().splitlines()[-1]);print('c$c $v',d['value'],d['ms_per_step'],d.get('kernel_ms_events_pass'))"
done
done
for v in "X=1" "PMDFC_RAMP_OPS=512" "PMDFC_RAMP_OPS=2048" "PMDFC_RAMP_MIN=1024" "PMDFC_RAMP_MIN=16384" "PMDFC_RAMP_OPS=512 PMDFC_RAMP_MIN=1024" "X=1"; do
  tag=$(echo "$v" | tr -dc 'A-Za-z0-9')
  env $v timeout -k 10 400 python3 bench.py --config 2 --init-cap 2 --steps 3 --warmup 1 --no-cpu-baseline > $O/ic2.$tag.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('$O/ic2.$tag.json').read().strip().splitlines()[-1]);print('ic2 $v',d['value'],d['ms_per_step'],d.get('kernel_ms_per_step',{}).get('final'))"
done
