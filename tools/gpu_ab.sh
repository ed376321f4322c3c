# A/B: default library vs $AB_LIBS (PMDFC_AB_LIB), config-2 bench lines; optional WRITE_SIZE pass
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
summ() { python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], d['value'], d['ms_per_step'], d['correct'], d['kernel_ms_per_step'])
for k,v in d['roofline']['per_kernel'].items(): print(' ', k, v['avg_launch_us'], v['frac'])
" $1; }
if [ "${AB_TESTS:-1}" = 1 ]; then
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/ab_tests.log 2>&1; rc=$?; tail -2 gpurun_out/ab_tests.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/ab_A.json 2> gpurun_out/ab_A.err || exit 1
summ gpurun_out/ab_A.json
for L in $AB_LIBS; do
  PMDFC_AB_LIB=$PWD/pmdfc_amd/lib/ab/$L timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/ab_$L.json 2> gpurun_out/ab_$L.err || exit 1
  summ gpurun_out/ab_$L.json
done
if [ "${AB_PMC:-0}" = 1 ]; then
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -T -f csv -d gpurun_out/ab_pmcw -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-pipeline > gpurun_out/ab_pmcw.json 2> gpurun_out/ab_pmcw.err || exit 1
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -T -f csv -d gpurun_out/ab_pmcf -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-pipeline > gpurun_out/ab_pmcf.json 2> gpurun_out/ab_pmcf.err || exit 1
  python3 tools/pmc_summary.py gpurun_out/ab_pmc.json gpurun_out/ab_pmcf gpurun_out/ab_pmcw | python3 -c "import json,sys; d=json.load(sys.stdin); [print(k, v) for k,v in d.items() if k in ('k_part','k_apply','k_split','k_get_u')]"
fi
exit 0
