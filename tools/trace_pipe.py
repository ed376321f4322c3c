"""Timeline of the insert phase of the last config-2 step from a rocprofv3
kernel trace of a PIPELINED bench run: per batch, each bucket-pass kernel's
[start, end] in us from the batch's first pass start, and the time from one
first pass to the next.  usage: trace_pipe.py run_kernel_trace.csv [batches]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda x: int(x["Start_Timestamp"]))
want = ("k_apply_fast", "k_apply_fb", "k_split", "k_apply_parked", "k_bucket", "k_part")
seq = []
for x in rows:
    nm = x["Kernel_Name"].split("(")[0].replace("pmdfc::", "").replace("void ", "").split("<")[0]
    if nm.startswith(want):
        seq.append((nm, int(x["Start_Timestamp"]) / 1e3, int(x["End_Timestamp"]) / 1e3, x["Stream_Id"]))
# first passes: k_apply_fast* on the caller's stream (a second look at
# declined buckets, on the engine's second stream, is not one)
s0 = next(r[3] for r in seq if r[0].startswith("k_apply_fast"))
firsts = [i for i, r in enumerate(seq) if r[0].startswith("k_apply_fast") and r[3] == s0]
firsts = firsts[-64:] if "--last" in sys.argv else firsts[:64]
nb = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2].isdigit() else 64
tot = 0.0
for bi, i in enumerate(firsts[:nb]):
    t0 = seq[i][1]
    nxt = seq[firsts[bi + 1]][1] if bi + 1 < len(firsts) else None
    parts = []
    for r in seq[i:]:
        if r[0] == "k_part":
            continue
        if r is not seq[i] and r[0].startswith("k_apply_fast") and r[3] == s0:
            break
        nm = r[0][:10] + ("'" if r[3] != s0 else "")
        parts.append(f"{nm} {r[1] - t0:6.1f}-{r[2] - t0:6.1f}")
    gap = f"next first +{nxt - t0:6.1f}" if nxt else ""
    if nxt:
        tot += nxt - t0
    print(f"{bi:2d} {gap}  " + "  ".join(parts))
last = firsts[min(nb, len(firsts)) - 1]
end = max(r[2] for r in seq[last:] if not (r[0].startswith("k_apply_fast") and r[3] == s0))
print(f"first-to-first total {tot / 1e3:.3f} ms; insert passes span {(end - seq[firsts[0]][1]) / 1e3:.3f} ms")
