"""Busy time of a rocprofv3 kernel trace: per kernel name (total, calls), the
span of the last `--last` seconds of dispatches, and the share of that span in
which at least one kernel ran (gaps = launch/host stalls).
Usage: trace_busy.py run_kernel_trace.csv [--from-kernel NAME]"""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
start_name = sys.argv[sys.argv.index("--from-kernel") + 1] if "--from-kernel" in sys.argv else None
rows = []
with open(path) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]))
rows.sort()
if start_name:  # from the last quarter's first dispatch of that kernel on
    idx = [i for i, r in enumerate(rows) if r[2].startswith(start_name)]
    if idx:
        rows = rows[idx[len(idx) // 2]:]
t0, t1 = rows[0][0], max(r[1] for r in rows)
busy, cur_s, cur_e = 0, None, None
for s, e, _ in rows:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
tot = defaultdict(lambda: [0, 0])
for s, e, n in rows:
    tot[n][0] += e - s
    tot[n][1] += 1
print(f"span {(t1 - t0) / 1e6:.2f} ms, busy {busy / 1e6:.2f} ms ({busy / (t1 - t0):.2%}), dispatches {len(rows)}")
for n, (t, c) in sorted(tot.items(), key=lambda x: -x[1][0])[:30]:
    print(f"  {t / 1e6:9.3f} ms  {c:6d}  {t / c / 1e3:8.2f} us  {n}")
