# SQ counters of the config-2 kernels on the final tree (k_apply_fast_cp, k_part, k_split, k_get_u)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r5ak
mkdir -p $O
B="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-pipeline"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES -T -f csv --kernel-include-regex "k_apply|k_split|k_part|k_get" -d $O/p1 -o run -- $B > /dev/null 2> $O/p1.err || exit 1
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE -T -f csv --kernel-include-regex "k_apply|k_split|k_part|k_get" -d $O/p2 -o run -- $B > /dev/null 2> $O/p2.err || exit 1
python3 tools/pmc_summary.py $O/sq.json $O/p1 $O/p2 > $O/sq.txt 2>&1
cat $O/sq.txt | python3 -c "
import json,sys
d=json.load(sys.stdin)
for k,v in d.items():
    w=v.get('SQ_WAVE_CYCLES') or 1
    print(k, 'wait_any %.2f'%(v.get('SQ_WAIT_ANY',0)/w), 'wait_inst %.2f'%(v.get('SQ_WAIT_INST_ANY',0)/w), 'active_inst %.2f'%(v.get('SQ_ACTIVE_INST_ANY',0)/w))
"
# mixed configs with the round-4 grids (all passes, or only the final pass) vs the load-based ones
for c in 4 3; do
for v in "X=1" "PMDFC_LIB=pmdfc_amd/lib/ab/oldgrids/libpmdfc_cceh.so" "PMDFC_LIB=pmdfc_amd/lib/ab/fin1024/libpmdfc_cceh.so" "X=1" "PMDFC_LIB=pmdfc_amd/lib/ab/oldgrids/libpmdfc_cceh.so" "PMDFC_LIB=pmdfc_amd/lib/ab/fin1024/libpmdfc_cceh.so"; do
  tag=$(echo "$v" | sed 's/.*ab.//;s/.libpmdfc_cceh.so//' | tr -dc 'A-Za-z0-9')
  env $v timeout -k 10 400 python3 bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline > $O/c$c.$tag.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('$O/c$c.$tag.json').read().strip().splitlines()[-1]);print('c$c $tag',d['value'],d['ms_per_step'],d.get('kernel_ms_events_pass'))"
done
done
