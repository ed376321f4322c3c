"""Config-2 shaped insert batches (for rocprofv3 counter passes): 64M-key
geometry, N batches of 1M fresh keys, then one timed Get batch."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pmdfc_amd as P  # noqa: E402

B = 1 << 20
NB = int(sys.argv[1]) if len(sys.argv) > 1 else 24
t = P.CCEH(65536, max_batch=B, max_segments=int((1 << 26) / 512 * 1.25) + 65536 + 1024, device=0)
keys = [P.gen_keys(1000, i * B, B) for i in range(NB)]
torch.cuda.synchronize()
for k in keys:
    t.Insert(k, k)
v, s = t.Get(keys[0])
torch.cuda.synchronize()
print("ok", t.stats()["segments"], bool((s == P.ST_HIT).all()))
