"""Per-phase timing of k_apply / k_split / k_part from the engine's debug stamps.

Runs config-2 shaped insert batches on one GPU with PMDFC_STAMPS=1 and prints,
for the last batch, the distribution over workgroups (waves, splits) of each
phase's length (GPU box only).  usage: phase_stamps.py [batches] [mixed]
("mixed": the stamped batch is a config-4 shaped 50/50 mixed batch -- Gets of
inserted keys, fresh Inserts -- after the insert batches)"""
import os
import sys

os.environ["PMDFC_STAMPS"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import pmdfc_amd as P  # noqa: E402

B = 1 << 20
NB = int(sys.argv[1]) if len(sys.argv) > 1 else 46
TPU = float(os.environ.get("TICKS_PER_US", "100"))  # wall_clock64: 100 MHz
MIXED = len(sys.argv) > 2 and sys.argv[2] == "mixed"
t = P.CCEH(65536, max_batch=B, max_segments=int(os.environ.get("MAXSEG", 1 << 18)), device=0)
for i in range(NB):
    k = P.gen_keys(2, i * B, B)
    t.Insert(k, k)
if MIXED:
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    ins = torch.rand(B, device="cuda", generator=g) < 0.5
    old = P.gen_keys(2, 0, NB * B)[torch.randint(0, NB * B, (B,), device="cuda", generator=g)]
    k = torch.where(ins, P.gen_keys(2, NB * B, B), old)
    t.Mixed(ins.to(torch.uint8), k, k)
torch.cuda.synchronize()
bk, pt, sp = t.debug_stamps(B)


def dist(nm, d):
    d = np.asarray(d, np.float64)
    if d.size:
        print(f"  {nm:14s} n={d.size:6d} mean {d.mean():8.2f} us  p50 {np.median(d):8.2f}  "
              f"p90 {np.percentile(d, 90):8.2f}  max {d.max():8.2f}")


def ph(a, b, ok):
    return (b[ok].astype(np.int64) - a[ok].astype(np.int64)) / TPU


print(f"mixed 50/50 batch after {NB} x 1M inserts" if MIXED else f"batch {NB - 1} of config 2 ({NB} x 1M inserts so far)")
p0 = pt[:, 0].min()
print(f"k_part: {pt.shape[0]} blocks, span {(pt[:, 3].max() - p0) / TPU:.1f} us")
for j, nm in enumerate(["rank", "reserve", "write"]):
    dist(nm, ph(pt[:, j], pt[:, j + 1], pt[:, j + 1] > 0))
ok = bk[:, 7] > 0
t0 = bk[ok, 0].min()
print(f"k_apply (first pass): {int(ok.sum())} waves, span {(bk[ok, 7].max() - t0) / TPU:.1f} us")
dist("start offset", (bk[ok, 0] - t0) / TPU)
dist("wave length", ph(bk[:, 0], bk[:, 7], ok))
for a_, b_, nm in ((0, 1, "collect"), (1, 4, "route"), (4, 5, "sort"), (5, 2, "run starts"),
                   (2, 6, "runs"), (2, 14, " run0 loop"), (14, 15, " run0 wb"), (15, 6, " run0..all"),
                   (6, 3, "store pass"), (3, 7, "tail")):
    dist(nm, ph(bk[:, a_], bk[:, b_], ok & (bk[:, a_] > 0) & (bk[:, b_] > 0) & (bk[:, 2] > 0)))
fc = ok & (bk[:, 2] == 0) & (bk[:, 5] > 0)  # fast_claim waves (no sort stamp)
if fc.any():
    print(f"  fast_claim waves: {int(fc.sum())}")
    for a_, b_, nm in ((0, 1, "collect"), (1, 4, "route+marks"), (4, 5, "claims"), (5, 6, "dep walk"),
                       (5, 10, " list+masks"), (10, 12, " rounds"), (12, 6, " full check"),
                       (6, 3, "commit"), (3, 7, "tail")):
        dist(nm, ph(bk[:, a_], bk[:, b_], fc))
    print("  rounds per wave:", np.bincount((bk[fc, 11] & 0xFFFF).astype(np.int64)).tolist())
    dist("dependent ops", (bk[fc, 11] >> 16).astype(np.float64) * TPU)
fin = bk[:, 13] > 0
if fin.any():
    print(f"k_bucket (final): {int(fin.sum())} active waves, span {(bk[fin, 13].max() - bk[fin, 8].min()) / TPU:.1f} us")
    dist("wave length", ph(bk[:, 8], bk[:, 13], fin))
ok = sp[:, 4] > 0
if ok.any():
    s0 = sp[ok, 5].min()
    fast = sp[:, 6] == 1
    print(f"k_split: {int(ok.sum())} splits stamped ({int((ok & fast).sum())} cluster path, "
          f"{int((ok & ~fast).sum())} generic replay), span {(sp[ok, 4].max() - s0) / TPU:.1f} us")
    dist("start offset", (sp[ok, 5] - s0) / TPU)
    dist("split length", ph(sp[:, 5], sp[:, 4], ok))
    for a_, b_, nm in ((5, 0, "load+hash"), (0, 1, "scan units"), (1, 2, "replay"), (1, 7, " wrap unit"),
                       (7, 2, " sweep"), (2, 3, "reload"), (3, 4, "store")):
        dist(nm, ph(sp[:, a_], sp[:, b_], ok & (sp[:, 7] > 0) if 7 in (a_, b_) else ok))
    for nm, m in (("cluster path", ok & fast), ("generic", ok & ~fast)):
        dist(nm + " replay", ph(sp[:, 1], sp[:, 2], m))
print(t.stats())
