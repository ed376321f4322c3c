# split linear-store A/B (+ WRITE_SIZE), parity, phase stamps, SQ counters
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r5d
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_serve.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -2 $O/parity.log
AB=pmdfc_amd/lib/ab/splitlin0/libpmdfc_cceh.so
for i in 1 2; do
timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_lin1.$i.json 2>/dev/null || exit 1
PMDFC_LIB=$AB timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_lin0.$i.json 2>/dev/null || exit 1
for m in 1 0; do python3 -c "import json;d=json.load(open('$O/bench_lin$m.$i.json'));print('lin',$m,d['value'],d['ms_per_step'],d['kernel_ms_per_step'])"; done
done
B="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-pipeline"
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -T -f csv --kernel-include-regex "k_split|k_apply|k_part" -d $O/w1 -o run -- $B > /dev/null 2> $O/w1.err || exit 1
PMDFC_LIB=$AB timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -T -f csv --kernel-include-regex "k_split|k_apply|k_part" -d $O/w0 -o run -- $B > /dev/null 2> $O/w0.err || exit 1
python3 tools/pmc_summary.py $O/w1.json $O/w1 > $O/w1.txt; python3 tools/pmc_summary.py $O/w0.json $O/w0 > $O/w0.txt
echo "WRITE lin1"; cat $O/w1.txt; echo "WRITE lin0"; cat $O/w0.txt
timeout -k 10 300 python -u tools/phase_stamps.py 46 > $O/stamps.txt 2>&1 || exit 1
cat $O/stamps.txt
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES -T -f csv --kernel-include-regex "k_apply|k_split|k_part|k_get" -d $O/p1 -o run -- $B > /dev/null 2> $O/p1.err || exit 1
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE -T -f csv --kernel-include-regex "k_apply|k_split|k_part|k_get" -d $O/p2 -o run -- $B > /dev/null 2> $O/p2.err || exit 1
python3 tools/pmc_summary.py $O/sq.json $O/p1 $O/p2 > $O/sq.txt 2>&1
cat $O/sq.txt
timeout -k 10 120 rocprofv3 -L > $O/avail.txt 2>&1 || true
