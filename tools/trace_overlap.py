"""Overlap of the partition stream with the bucket passes in a PIPELINED
config-2 step (rocprofv3 kernel trace of bench.py without --no-pipeline):
per insert batch, k_part's span and how much of it ran while a bucket-pass
kernel of the engine stream was running.  usage:
trace_overlap.py gpurun_out/trp/run_kernel_trace.csv"""
import csv
import sys

import numpy as np

t = list(csv.DictReader(open(sys.argv[1])))
t.sort(key=lambda x: int(x["Start_Timestamp"]))
seq = [(x["Kernel_Name"].split("(")[0].replace("pmdfc::", "").replace("void ", ""),
        int(x["Start_Timestamp"]), int(x["End_Timestamp"])) for x in t]
bucket = ("k_apply", "k_split", "k_bucket")
parts = [s for s in seq if s[0] == "k_part"][-64:]
t0 = parts[0][1]
other = [s for s in seq if s[0].startswith(bucket) and s[2] > t0]
rows = []
for n, a, b in parts:
    ov = 0
    for _, c, d in other:
        lo, hi = max(a, c), min(b, d)
        if hi > lo:
            ov += hi - lo
    rows.append(((b - a) / 1e3, min(ov, b - a) / 1e3))
r = np.array(rows)
last = max(s[2] for s in seq if s[0].startswith(bucket))
print(f"64 k_part: mean span {r[:, 0].mean():.1f} us, overlapped with bucket passes {r[:, 1].mean():.1f} us "
      f"({r[:, 1].sum() / r[:, 0].sum():.0%}); insert phase wall {(last - t0) / 1e3:.0f} us")
names = sorted({s[0] for s in other})
for nm in names:
    d = [(s[2] - s[1]) / 1e3 for s in other if s[0] == nm]
    print(f"  {nm:28s} n={len(d):4d} mean {np.mean(d):7.1f} us  sum {np.sum(d) / 1e3:6.2f} ms")
