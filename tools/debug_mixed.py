"""One mixed scenario on the GPU vs the oracle, listing the first differing Get
results (GPU box).  usage: debug_mixed.py NAME [batch]  (env PMDFC_P1MAX /
PMDFC_CHUNK select the bucket geometry as the tests' "tight" path does)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

import pmdfc_amd as P  # noqa: E402
import scenarios as S  # noqa: E402
from oracle import oracle as O  # noqa: E402

name = sys.argv[1]
init_cap, conv, ops, keys, vals = S.scenarios(O.hash64)[name]
n = keys.size
b = int(sys.argv[2]) if len(sys.argv) > 2 and int(sys.argv[2]) else n
t = P.CCEH(init_cap, convention=conv, max_batch=b, max_segments=8192)
out = np.zeros(n, np.uint64)
st = np.zeros(n, np.uint8)
for off in range(0, n, b):
    o, s = t.Mixed(ops[off:off + b], keys[off:off + b], vals[off:off + b])
    out[off:off + b] = o
    st[off:off + b] = s
orc = O.OracleCCEH(t.initial_depth)
oout, ost = orc.mixed(ops, keys, vals)
get = ops == S.OP_GET
bad = np.where(get & ((out != oout) | (st != ost)))[0]
print("stats", t.stats())
print("gets", int(get.sum()), "differing", bad.size)
for i in bad[:20]:
    prev = np.where((keys[:i] == keys[i]) & (ops[:i] != S.OP_GET))[0]
    print(f" op {i} tile {i // 4096} key {int(keys[i]):#x} gpu ({int(out[i])}, {st[i]}) oracle ({int(oout[i])}, {ost[i]})"
          f" inserts of key before: {prev[-3:].tolist()}")
