"""Main-stream gaps of one timed config-2 step (rocprofv3 --kernel-trace csv of
bench.py --steps 2 --warmup 1): the step = from the 4th k_init_segments to
the 5th (warm-up, 2 timed steps, then the bench's own passes).  Prints the
main stream's busy time, its gaps by (kernel before, kernel after), and the
gaps at the group boundaries.  usage: step_gaps.py run_kernel_trace.csv [k]"""
import csv
import sys
from collections import defaultdict

t = list(csv.DictReader(open(sys.argv[1])))
k = int(sys.argv[2]) if len(sys.argv) > 2 else 3
rows = [(x["Kernel_Name"].split("(")[0].replace("void ", "").replace("pmdfc::", ""), int(x["Start_Timestamp"]),
         int(x["End_Timestamp"]), x["Stream_Id"]) for x in t]
rows.sort(key=lambda r: r[1])
inits = [i for i, r in enumerate(rows) if r[0].startswith("k_init_segments")]
i = inits[k]
t0, t1 = rows[i][1], rows[inits[k + 1]][1]
step = [r for r in rows[i:] if r[1] < t1]
te = max(r[2] for r in step if r[0].startswith("k_get_u"))
step = [r for r in step if r[1] <= te]
main = [r for r in step if r[3] == step[0][3]]
busy = sum(r[2] - r[1] for r in main)
print(f"step {(te - t0) / 1e3:.1f} us, main busy {busy / 1e3:.1f}, main idle {(te - t0 - busy) / 1e3:.1f}")
g = defaultdict(list)
for a, b in zip(main, main[1:]):
    g[(a[0][:18], b[0][:18])].append((b[1] - a[2]) / 1e3)
for key, v in sorted(g.items(), key=lambda kv: -sum(kv[1]))[:6]:
    print(f"  {key[0]:20s} -> {key[1]:20s} n={len(v):3d} sum {sum(v):7.1f} mean {sum(v) / len(v):6.2f}")
fc = [r for r in main if r[0].startswith("k_apply_fast_cp")]
print("first pass starts at", round((fc[0][1] - t0) / 1e3, 1), "us")
print("gaps before first passes:", [round((b[1] - a[2]) / 1e3, 1) for a, b in zip(main, main[1:])
                                     if b[0].startswith("k_apply_fast_cp") and (b[1] - a[2]) > 5000])
