"""Where the wall time of a PIPELINED config-2 insert phase goes (rocprofv3
kernel trace of bench.py without --no-pipeline): per kernel name the busy time
of the engine-stream kernels, the idle gaps between consecutive engine-stream
kernels (launch overhead, dependencies), and how much of the phase had a
k_part running beside them.  usage: trace_gaps.py run_kernel_trace.csv"""
import csv
import sys

import numpy as np

t = list(csv.DictReader(open(sys.argv[1])))
t.sort(key=lambda x: int(x["Start_Timestamp"]))
seq = [(x["Kernel_Name"].split("(")[0].replace("pmdfc::", "").replace("void ", "").split("<")[0],
        int(x["Start_Timestamp"]), int(x["End_Timestamp"])) for x in t]
eng = ("k_apply", "k_split", "k_bucket")
parts = [s for s in seq if s[0] == "k_part"][-64:]
t0 = parts[0][1]
ev = [s for s in seq if s[0].startswith(eng) and s[1] >= t0]
t1 = max(s[2] for s in ev)
wall = (t1 - t0) / 1e3
busy = {}
for n, a, b in ev:
    busy.setdefault(n, []).append((b - a) / 1e3)
gaps = []
for (n0, a0, b0), (n1, a1, b1) in zip(ev, ev[1:]):
    gaps.append(((a1 - b0) / 1e3, n0, n1))
g = np.array([x[0] for x in gaps])
print(f"insert phase wall {wall:.0f} us over {len(ev)} engine kernels ({wall / 64:.1f} us per batch)")
for n, d in sorted(busy.items(), key=lambda kv: -sum(kv[1])):
    print(f"  {n:22s} n={len(d):4d} mean {np.mean(d):7.1f} us  sum {np.sum(d) / 1e3:6.3f} ms")
print(f"  gaps between engine kernels: sum {g[g > 0].sum() / 1e3:.3f} ms, mean {g.mean():.2f} us, "
      f"overlapping (<0) {int((g < 0).sum())}")
pairs = {}
for d, a, b in gaps:
    pairs.setdefault((a, b), []).append(d)
for (a, b), d in sorted(pairs.items(), key=lambda kv: -sum(kv[1]))[:8]:
    print(f"    {a:>16s} -> {b:<16s} n={len(d):4d} mean gap {np.mean(d):6.2f} us")
gets = [s for s in seq if s[0].startswith("k_get") and s[1] >= t1][:64]
if gets:
    gw = (gets[-1][2] - gets[0][1]) / 1e3
    gb = sum((s[2] - s[1]) for s in gets) / 1e3
    print(f"get phase: {len(gets)} launches, wall {gw:.0f} us, busy {gb:.0f} us")
