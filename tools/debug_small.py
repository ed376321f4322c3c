"""Small insert / mixed cross-check against the oracle with detailed output (GPU box)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np  # noqa: E402

import pmdfc_amd as P  # noqa: E402
from oracle import oracle as O  # noqa: E402
from pmdfc_amd.workload import uniform_keys  # noqa: E402

depth = int(os.environ.get("DBG_DEPTH", "4"))
n = int(os.environ.get("DBG_N", "20000"))
t = P.CCEH(depth=depth, max_batch=1 << 15, max_segments=1024, device=0)
o = O.OracleCCEH(depth)
keys = uniform_keys(7, 0, n)
st = t.Insert(keys, keys)
ost = o.insert(keys, keys)
print("insert status equal:", np.array_equal(st, ost), "stats", t.stats())
d, od = t.dump(), o.dump()
print("depth", d["depth"], od["depth"], "nseg", len(d["local_depth"]), len(od["local_depth"]))
if len(d["local_depth"]) == len(od["local_depth"]):
    print("ld equal", np.array_equal(d["local_depth"], od["local_depth"]))
    K, OK = d["keys"].reshape(-1, 1024), od["keys"].reshape(-1, 1024)
    badseg = np.where((K != OK).any(axis=1))[0]
    print("segments differing:", len(badseg), badseg[:10])
    for sidx in badseg[:2]:
        diff = np.where(K[sidx] != OK[sidx])[0]
        print(" seg", sidx, "ld", d["local_depth"][sidx], "ndiff", len(diff), "first", diff[:12])
        print("  gpu   ", [hex(int(x)) for x in K[sidx][diff[:6]]])
        print("  oracle", [hex(int(x)) for x in OK[sidx][diff[:6]]])
        print("  gpu occupied", int((K[sidx] != 2**64 - 1).sum()), "oracle occupied", int((OK[sidx] != 2**64 - 1).sum()))
v, s = t.Get(keys)
print("get all hit:", bool((s == P.ST_HIT).all()), "misses", int((s != P.ST_HIT).sum()), "wrong", int((v != keys).sum()))
