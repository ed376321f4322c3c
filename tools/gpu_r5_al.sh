# mixed: bulk clear of the inserted-key set by the verify pass when a batch inserts many keys
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r5al
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_route.py tests/test_gpu_serve.py -x -q --timeout 200 --timeout-method thread -k "mixed or split_loss or route or serve" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for c in 4 3; do
for v in "X=1" "PMDFC_LIB=pmdfc_amd/lib/ab/head/libpmdfc_cceh.so" "PMDFC_LIB=pmdfc_amd/lib/ab/nobulk/libpmdfc_cceh.so" "X=1" "PMDFC_LIB=pmdfc_amd/lib/ab/head/libpmdfc_cceh.so" "PMDFC_LIB=pmdfc_amd/lib/ab/nobulk/libpmdfc_cceh.so"; do
  tag=$(echo "$v" | sed 's/.*ab.//;s/.libpmdfc_cceh.so//' | tr -dc 'A-Za-z0-9')
  env $v timeout -k 10 400 python3 bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline > $O/c$c.$tag.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('$O/c$c.$tag.json').read().strip().splitlines()[-1]);print('c$c $tag',d['value'],d['ms_per_step'],d.get('kernel_ms_events_pass'))"
done
done
