# mixed-batch iteration: the whole GPU suite, then configs 4, 3 and 2, then a config-4 trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/m_tests.log 2>&1; rc=$?; tail -3 gpurun_out/m_tests.log; [ $rc -eq 0 ] || exit $rc
for c in 4 3 2; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > gpurun_out/m_bench$c.json 2> gpurun_out/m_bench$c.err || exit 1
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/m_bench$c.json').read().strip().splitlines()[-1])
print('config $c', d['value'], d['ms_per_step'], d['correct'], d.get('kernel_ms_per_step') or d.get('kernel_ms_events_pass'))
"
done
bash tools/gpu_c4_trace.sh > /dev/null || exit 1
python3 - <<'PY'
import csv
t=list(csv.DictReader(open('gpurun_out/c4tr/run_kernel_trace.csv')))
t.sort(key=lambda x:int(x['Start_Timestamp']))
seq=[(x['Kernel_Name'].split('(')[0].replace('pmdfc::','').replace('void ',''),(int(x['End_Timestamp'])-int(x['Start_Timestamp']))/1e3,int(x['Start_Timestamp']),int(x['End_Timestamp'])) for x in t]
rows=[];i=0
while i<len(seq):
    if seq[i][0]=='k_mixed_prep':
        j=i
        while seq[j][0]!='k_mixed_verify': j+=1
        rows.append(seq[i-3:j+1]); i=j+1
    else: i+=1
for blk in rows[-2:]:
    print(' | '.join(f"{b[0][:14]} {b[1]:.1f}" for b in blk), f" wall {(blk[-1][3]-blk[0][2])/1e3:.1f}")
PY
