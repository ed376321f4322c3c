# mixed batches pipelined (prep of batch i+1 beside batch i): parity, then
# configs 4 / 3 MixedBatches vs one Mixed per batch; k_split reload A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r5m
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_route.py tests/test_gpu_dist2.py tests/test_gpu_dropin.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for c in 4 3; do
  for v in pipe nopipe pipe nopipe; do
    F=""; [ $v = nopipe ] && F=--no-pipeline
    timeout -k 10 400 python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline $F > $O/c$c.$v.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.loads(open('$O/c$c.$v.json').read().strip().splitlines()[-1]);print('c$c $v',d['value'],d['ms_per_step'])"
  done
done
timeout -k 10 400 python3 bench.py --config 4 --route --steps 3 --warmup 1 --no-cpu-baseline > $O/c4route.json 2>/dev/null || exit 1
python3 -c "import json;d=json.loads(open('$O/c4route.json').read().strip().splitlines()[-1]);print('c4 route',d['value'],d['ms_per_step'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -f csv -d $O/t4 -o run -- python3 bench.py --config 4 --steps 1 --warmup 0 --no-cpu-baseline > /dev/null 2> $O/t4.err || exit 1
AB=pmdfc_amd/lib/ab/reload1/libpmdfc_cceh.so
for i in 1 2; do
timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_r0.$i.json 2>/dev/null || exit 1
PMDFC_LIB=$AB timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_r1.$i.json 2>/dev/null || exit 1
for m in 0 1; do python3 -c "import json;d=json.load(open('$O/bench_r$m.$i.json'));print('reload',$m,d['value'],d['ms_per_step'],d['kernel_ms_per_step'])"; done
done
