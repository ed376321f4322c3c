# SQ counters of the first apply pass (k_apply / k_apply_fast) over one non-pipelined config-2 step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/sqa
B="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-pipeline"
R="k_apply|k_part|k_split"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -T -f csv --kernel-include-regex "$R" -d gpurun_out/sqa/p1 -o run -- $B > /dev/null 2> gpurun_out/sqa/p1.err
echo p1 $?
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -T -f csv --kernel-include-regex "$R" -d gpurun_out/sqa/p2 -o run -- $B > /dev/null 2> gpurun_out/sqa/p2.err
echo p2 $?
timeout -s KILL 240 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum GRBM_GUI_ACTIVE -T -f csv --kernel-include-regex "$R" -d gpurun_out/sqa/p3 -o run -- $B > /dev/null 2> gpurun_out/sqa/p3.err
echo p3 $?
python3 tools/pmc_summary.py gpurun_out/sqa/sq.json gpurun_out/sqa/p1 gpurun_out/sqa/p2 gpurun_out/sqa/p3 > /dev/null
python3 -c "
import json; d=json.load(open('gpurun_out/sqa/sq.json'))
for k,v in d.items():
  w=v.get('SQ_WAVES',1) or 1
  print(k, {c: round(v[c]/w,1) if c.startswith('SQ_') else v[c] for c in v})
"
