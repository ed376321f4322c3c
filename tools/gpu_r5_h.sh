# full GPU suite + smoke; launch-cost ubench; split NT A/B; k_part PMC with the coarse partition
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r5h
mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/full_tests.log 2>&1; rc=$?
tail -4 $O/full_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
timeout -k 10 120 tools/ubench_launch > $O/launch.txt 2>&1 || exit 1
cat $O/launch.txt
AB=pmdfc_amd/lib/ab/splitnt1/libpmdfc_cceh.so
for i in 1 2; do
timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_nt0.$i.json 2>/dev/null || exit 1
PMDFC_LIB=$AB timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_nt1.$i.json 2>/dev/null || exit 1
for m in 0 1; do python3 -c "import json;d=json.loads(open('$O/bench_nt$m.$i.json').read().strip().splitlines()[-1]);print('nt',$m,d['value'],d['ms_per_step'],d['kernel_ms_per_step'])"; done
done
B="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-pipeline"
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -T -f csv --kernel-include-regex "k_part|k_apply|k_split" -d $O/w -o run -- $B > /dev/null 2> $O/w.err || exit 1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -T -f csv --kernel-include-regex "k_part|k_apply|k_split" -d $O/f -o run -- $B > /dev/null 2> $O/f.err || exit 1
python3 tools/pmc_summary.py $O/pmc.json $O/f $O/w
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d $O/trace -o run -- $B > $O/bench_trace.json 2> $O/bench_trace.err || exit 1
head -12 $O/trace/run_kernel_stats.csv
