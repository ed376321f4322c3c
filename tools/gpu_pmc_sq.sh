# SQ counters of the insert kernels over one non-pipelined config-2 step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/sq
B="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-pipeline"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES -T -f csv --kernel-include-regex "k_apply|k_split|k_part|k_get" -d gpurun_out/sq/p1 -o run -- $B > /dev/null 2> gpurun_out/sq/p1.err
echo p1 $?
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE -T -f csv --kernel-include-regex "k_apply|k_split|k_part|k_get" -d gpurun_out/sq/p2 -o run -- $B > /dev/null 2> gpurun_out/sq/p2.err
echo p2 $?
python3 tools/pmc_summary.py gpurun_out/sq/sq.json gpurun_out/sq/p1 gpurun_out/sq/p2
