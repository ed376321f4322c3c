# kernel breakdown of the mixed configs (3, 4) and the CCEH_hybrid(2) ramp
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r5i
mkdir -p $O
timeout -k 10 400 python3 bench.py --config 4 --steps 2 --warmup 1 --no-cpu-baseline > $O/c4.json 2>/dev/null || exit 1
python3 -c "import json;d=json.loads(open('$O/c4.json').read().strip().splitlines()[-1]);print('c4',d['value'],d['ms_per_step'],d.get('kernel_ms_per_step'))"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -f csv -d $O/t4 -o run -- python3 bench.py --config 4 --steps 1 --warmup 0 --no-cpu-baseline > /dev/null 2> $O/t4.err || exit 1
head -25 $O/t4/run_kernel_stats.csv | cut -c1-150
timeout -k 10 400 python3 bench.py --config 3 --steps 2 --warmup 1 --no-cpu-baseline > $O/c3.json 2>/dev/null || exit 1
python3 -c "import json;d=json.loads(open('$O/c3.json').read().strip().splitlines()[-1]);print('c3',d['value'],d['ms_per_step'],d.get('kernel_ms_per_step'))"
timeout -k 10 400 python3 bench.py --init-cap 2 --steps 3 --warmup 1 --no-cpu-baseline > $O/ic2.json 2>/dev/null || exit 1
python3 -c "import json;d=json.loads(open('$O/ic2.json').read().strip().splitlines()[-1]);print('ic2',d['value'],d['ms_per_step'],d.get('kernel_ms_per_step'))"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -f csv -d $O/t2 -o run -- python3 bench.py --init-cap 2 --steps 1 --warmup 0 --no-cpu-baseline > /dev/null 2> $O/t2.err || exit 1
head -25 $O/t2/run_kernel_stats.csv | cut -c1-150
