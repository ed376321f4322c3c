"""Per-phase timing of k_bucket / k_part from the engine's debug stamps.

Runs config-2 shaped insert batches on one GPU with PMDFC_STAMPS=1 and prints,
for one late batch, the distribution over workgroups of each phase's length
and the spread of workgroup start/end times (GPU box only)."""
import os
import sys

os.environ["PMDFC_STAMPS"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import pmdfc_amd as P  # noqa: E402

B = 1 << 20
NB = int(sys.argv[1]) if len(sys.argv) > 1 else 48
t = P.CCEH(65536, max_batch=B, max_segments=int((1 << 26) / 512 * 1.25) + 65536 + 1024, device=0)
for i in range(NB):
    k = P.gen_keys(1000, i * B, B)
    t.Insert(k, k)
torch.cuda.synchronize()
bk, pt = t.debug_stamps(B)
# calibrate the stamp clock against host time over a busy kernel window
import time
tk = torch.cuda.Event(enable_timing=True); tk2 = torch.cuda.Event(enable_timing=True)
k = P.gen_keys(1000, NB * B, B)
tk.record(); t.Insert(k, k); tk2.record(); torch.cuda.synchronize()
bk2, _ = t.debug_stamps(B)
ev_us = tk.elapsed_time(tk2) * 1e3
span_ticks = bk2[:, 7].max() - bk2[:, 0].min()
print(f"calibration: insert batch {ev_us:.1f} us by events; k_bucket span {span_ticks} ticks -> "
      f"{span_ticks / ev_us:.1f} ticks/us upper bound")
TPU = float(os.environ.get("TICKS_PER_US", "100"))
names = ["collect", "sort", "apply+store", "n/a", "n/a", "n/a", "tail(3->7)"]
t0 = bk[:, 0].min()
fin = bk[:, 8] > 0
if fin.any():
    f0 = bk[fin, 8]
    print(f"k_bucket(final): {int(fin.sum())} active waves, span {(bk[fin, 13].max() - f0.min()) / TPU:.1f} us, "
          f"wave length median {np.median(bk[fin, 13] - f0) / TPU:.1f} us")
    for a_, b_, nm in ((8, 9, "collect"), (9, 10, "sort"), (10, 11, "apply"), (11, 12, "split"), (12, 13, "rest")):
        ok = fin & (bk[:, a_] > 0) & (bk[:, b_] > 0)
        d = (bk[ok, b_].astype(np.int64) - bk[ok, a_].astype(np.int64)) / TPU
        if d.size:
            print(f"  final {nm:8s} n={d.size:5d} mean {d.mean():7.2f}  p50 {np.median(d):7.2f}  p90 {np.percentile(d, 90):7.2f}")
print(f"k_apply: {bk.shape[0]} WGs, span {(bk[:, 7].max() - t0) / TPU:.1f} us "
      f"(first start..last end); WG length median {np.median((bk[:, 7] - bk[:, 0])) / TPU:.1f} us")
starts = (bk[:, 0] - t0) / TPU
print(f"  WG start offsets us: p10 {np.percentile(starts, 10):.1f} p50 {np.percentile(starts, 50):.1f} "
      f"p90 {np.percentile(starts, 90):.1f} max {starts.max():.1f}")
for ph in (0, 1, 2, 6):
    a, b = bk[:, ph], bk[:, ph + 1]
    if ph == 6:
        a = bk[:, 3]
    ok = (a > 0) & (b > 0)
    d = (b[ok].astype(np.int64) - a[ok].astype(np.int64)) / TPU
    if d.size:
        print(f"  {names[ph]:7s} n={d.size:5d} mean {d.mean():7.2f} us  p50 {np.median(d):7.2f}  p90 {np.percentile(d, 90):7.2f}  max {d.max():7.2f}")
for ph, nm in ((8, "bm load"), (9, "ops"), (10, "bm store"), (11, "drain")):
    a_, b_ = (bk[:, 3] if ph == 8 else bk[:, ph - 1]), bk[:, ph]
    ok = (a_ > 0) & (b_ > 0)
    d = (b_[ok].astype(np.int64) - a_[ok].astype(np.int64)) / TPU
    if d.size:
        print(f"  run0 {nm:8s} n={d.size:5d} mean {d.mean():7.2f} us  p50 {np.median(d):7.2f}  p90 {np.percentile(d, 90):7.2f}")
for ph, nm in ((11, "sp load+hash"), (12, "sp clusters"), (13, "sp place"), (14, "sp reload"), (15, "sp store")):
    a_, b_ = bk[:, ph - 1], bk[:, ph]
    ok = (a_ > 0) & (b_ > 0) & (b_ >= a_)
    d = (b_[ok].astype(np.int64) - a_[ok].astype(np.int64)) / TPU
    if d.size:
        print(f"  {nm:14s} n={d.size:5d} mean {d.mean():7.2f} us  p50 {np.median(d):7.2f}  p90 {np.percentile(d, 90):7.2f}")
p0 = pt[:, 0].min()
print(f"k_part: {pt.shape[0]} blocks, span {(pt[:, 3].max() - p0) / TPU:.1f} us")
for ph, nm in enumerate(["rank", "reserve", "write"]):
    d = (pt[:, ph + 1].astype(np.int64) - pt[:, ph].astype(np.int64)) / TPU
    print(f"  {nm:7s} mean {d.mean():7.2f} us  p50 {np.median(d):7.2f}  max {d.max():7.2f}")
s = (pt[:, 0] - p0) / TPU
print(f"  block start offsets us: p50 {np.median(s):.1f} max {s.max():.1f}")
print(t.stats())
