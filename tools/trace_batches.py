"""Per-batch kernel durations from a rocprofv3 kernel trace of bench.py
(insert batches: k_part .. k_bucket), last step only.  usage:
trace_batches.py gpurun_out/prof/run_kernel_trace.csv"""
import csv
import os
import sys

import numpy as np

t = list(csv.DictReader(open(sys.argv[1])))
t.sort(key=lambda x: int(x["Start_Timestamp"]))
seq = [(x["Kernel_Name"].split("(")[0].replace("pmdfc::", "").replace("void ", ""),
        (int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e3, int(x["Start_Timestamp"]),
        int(x["End_Timestamp"])) for x in t]
rows, names = [], None
i = 0
while i < len(seq):
    if seq[i][0] == "k_part":
        j = i + 1
        while j < len(seq) and not seq[j][0].startswith("k_bucket"):
            j += 1
        blk = seq[i:j + 1]
        names = [b[0] for b in blk]
        rows.append([b[1] for b in blk] + [(blk[-1][3] - blk[0][2]) / 1e3])
        i = j + 1
    else:
        i += 1
rows = np.array(rows[-64:])
print(" ".join(f"{n[:9]:>9s}" for n in names + ["wall"]))
for r in rows[::int(os.environ.get("EVERY", 4))]:
    print(" ".join(f"{v:9.1f}" for v in r))
print("sum ms:", " ".join(f"{v:9.2f}" for v in rows.sum(0) / 1e3))
gets = [s[1] for s in seq if s[0].startswith("k_get")]
print(f"k_get: {len(gets)} launches, mean {np.mean(gets[-64:]):.1f} us")
