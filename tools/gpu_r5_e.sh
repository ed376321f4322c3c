# is k_part on the step's critical path? (delay knob) + N=1 routing shortcut
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r5e
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_route.py -x -q --timeout 200 --timeout-method thread > $O/route.log 2>&1 || { tail -30 $O/route.log; exit 1; }
tail -2 $O/route.log
for d in 0 20 0 20; do
PMDFC_PART_DELAY_US=$d timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_d$d.json 2>/dev/null || exit 1
python3 -c "import json;d=json.load(open('$O/bench_d$d.json'));print('delay',$d,d['value'],d['ms_per_step'],d['kernel_ms_per_step'])"
done
timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --route > $O/bench_route.json 2>/dev/null || exit 1
python3 -c "import json;d=json.load(open('$O/bench_route.json'));print('route',d['value'],d['ms_per_step'])"
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --config 4 --route > $O/bench_c4route.json 2>/dev/null || exit 1
python3 -c "import json;d=json.load(open('$O/bench_c4route.json'));print('c4 route',d['value'],d['ms_per_step'])"
