# coarse partition: parity, A/B (PMDFC_CP=0/1), phase stamps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r5g
mkdir -p $O
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_route.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { tail -40 $O/parity.log; exit 1; }
tail -2 $O/parity.log
for i in 1 2; do
for m in 1 0; do
PMDFC_CP=$m timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_cp$m.$i.json 2>/dev/null || exit 1
python3 -c "import json;d=json.loads(open('$O/bench_cp$m.$i.json').read().strip().splitlines()[-1]);print('cp',$m,d['value'],d['ms_per_step'],d['kernel_ms_per_step'],d['correct'])"
done; done
timeout -k 10 300 python -u tools/phase_stamps.py 46 > $O/stamps.txt 2>&1 || exit 1
head -30 $O/stamps.txt
