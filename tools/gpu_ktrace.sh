# kernel trace of one non-pipelined config-2 step (per-kernel, per-batch durations)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/kt_${KT_TAG:-A}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d $OUT -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-pipeline > $OUT.json 2> $OUT.err || exit 1
python3 - $OUT <<'PY'
import csv, collections, sys, glob
f = glob.glob(sys.argv[1] + "/**/run_kernel_trace.csv", recursive=True)[0]
d = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    n = r['Kernel_Name'].split('(')[0].replace('void ', '').replace('pmdfc::', '')
    d[n].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000)
for k in ['k_scan', 'k_split', 'k_apply_parked', 'k_apply', 'k_part', 'k_get_u', 'k_bucket']:
    v = d[k][-64:]
    if v: print(k, round(sum(v) / len(v), 2), [round(x) for x in v])
PY
