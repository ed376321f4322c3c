# phase stamps of the config-2 insert kernels + SQ counters + counter list
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5b
timeout -k 10 120 rocprofv3 -L > gpurun_out/r5b/avail.txt 2>&1 || true
timeout -k 10 300 python -u tools/phase_stamps.py 46 > gpurun_out/r5b/stamps.txt 2>&1 || exit 1
B="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-pipeline"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES -T -f csv --kernel-include-regex "k_apply|k_split|k_part|k_get" -d gpurun_out/r5b/p1 -o run -- $B > /dev/null 2> gpurun_out/r5b/p1.err || exit 1
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE -T -f csv --kernel-include-regex "k_apply|k_split|k_part|k_get" -d gpurun_out/r5b/p2 -o run -- $B > /dev/null 2> gpurun_out/r5b/p2.err || exit 1
python3 tools/pmc_summary.py gpurun_out/r5b/sq.json gpurun_out/r5b/p1 gpurun_out/r5b/p2 > gpurun_out/r5b/sq.txt 2>&1
cat gpurun_out/r5b/stamps.txt gpurun_out/r5b/sq.txt | head -120
