"""Timeline of consecutive PIPELINED config-2 insert batches from the
engine's debug stamps (PMDFC_STAMPS=1, PMDFC_STAMP_ROT=R: batch i stamps set
i % R).  Per batch: k_part blocks [first start, last end], the first apply
pass's waves, the split waves and the final-pass waves, in us from the first
partition of the window; shows whether batch i+1's partition runs under
batch i's passes (GPU box only).  usage: timeline.py [warm_batches] [R]"""
import os
import sys

R = int(sys.argv[2]) if len(sys.argv) > 2 else 8
os.environ["PMDFC_STAMPS"] = "1"
os.environ["PMDFC_STAMP_ROT"] = str(R)
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ctypes as C  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

import pmdfc_amd as P  # noqa: E402
from pmdfc_amd.engine import load_library  # noqa: E402

B = 1 << 20
W = int(sys.argv[1]) if len(sys.argv) > 1 else 40
TPU = 100.0  # wall_clock64 ticks per us
t = P.CCEH(65536, max_batch=B, max_segments=1 << 18, device=0)
keys = P.gen_keys(2, 0, (W + R) * B)
t.InsertBatches(keys[:W * B], keys[:W * B], list(range(0, W * B + 1, B)))
torch.cuda.synchronize()
k2 = keys[W * B:]
t.InsertBatches(k2, k2, list(range(0, R * B + 1, B)))
torch.cuda.synchronize()
nb = 1 << 13
nblk = (B + 8191) // 8192
tot = 16 * nb + 8 * nblk + 8 * 8192
buf = np.zeros(tot * R, np.uint64)
n = C.c_uint32()
rc = load_library().pmdfc_cceh_debug_stamps(t._h, buf.ctypes.data, buf.size, C.byref(n))
assert rc == 0, rc
nb = n.value
tot = 16 * nb + 8 * nblk + 8 * 8192
rows = []
for j in range(R):
    s = buf[j * tot:(j + 1) * tot]
    bk = s[:16 * nb].reshape(nb, 16).astype(np.int64)
    pt = s[16 * nb:16 * nb + 8 * nblk].reshape(nblk, 8).astype(np.int64)
    sp = s[16 * nb + 8 * nblk:].reshape(8192, 8).astype(np.int64)
    p0 = pt[:, 0].min()  # (entries older than the batch's partition: an earlier batch's, stale)
    ok = bk[:, 0] >= p0
    fin = bk[:, 8] >= p0
    spo = (sp[:, 5] >= p0) & (sp[:, 4] >= sp[:, 5])
    rows.append({"part": (pt[:, 0].min(), pt[:, 3].max()),
                 "apply": (bk[ok, 0].min(), bk[ok, 7].max()) if ok.any() else None,
                 "split": (sp[spo, 5].min(), sp[spo, 4].max()) if spo.any() else None,
                 "final": (bk[fin, 8].min(), bk[fin, 8:14].max()) if fin.any() else None})
# the R sets hold batches W..W+R-1 in rotation: order them by partition start
rows.sort(key=lambda r: r["part"][0])
t0 = rows[0]["part"][0]


def sp_(x):
    return "       -        " if x is None else f"{(x[0] - t0) / TPU:7.1f}-{(x[1] - t0) / TPU:7.1f}"


print(f"{R} pipelined batches after {W} (us from the first partition): part | apply | split | final")
for i, r in enumerate(rows):
    print(f"  {i}: part {sp_(r['part'])}  apply {sp_(r['apply'])}  split {sp_(r['split'])}  final {sp_(r['final'])}")
for i in range(1, len(rows)):
    a, p = rows[i - 1], rows[i]
    if a["apply"] is None:
        continue
    prev_end = max(x[1] for x in (a["apply"], a["split"], a["final"]) if x is not None)
    print(f"  batch {i}: partition ends {(p['part'][1] - prev_end) / TPU:+7.1f} us after batch {i - 1}'s last stamped pass; "
          f"its apply starts {(p['apply'][0] - prev_end) / TPU:+7.1f} us after it" if p["apply"] else "")
