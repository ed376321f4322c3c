"""Get-path diagnostic (GPU box only): on the config-2 table, per Get batch i
(the keys of insert batch i), the lines read per Get and the k_get_u launch
time, to see whether later-inserted keys sit deeper in their windows."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pmdfc_amd as P  # noqa: E402

B, NB = 1 << 20, 64
dev = torch.device("cuda", 0)
t = P.CCEH(65536, max_batch=B, max_segments=1 << 18, device=0)
keys = P.gen_keys(1000, 0, NB * B)
t.InsertBatches(keys, keys, list(range(0, NB * B + 1, B)))
torch.cuda.synchronize()
s = torch.cuda.current_stream(dev)
for i in range(0, NB, 3):
    k = keys[i * B:(i + 1) * B]
    t.timing(events=False, count_lines=True)
    t.Get(k)
    torch.cuda.synchronize()
    L = t.last_get_lines() / B
    t.timing(events=False, count_lines=False)
    t.Get(k)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(10):
        t.Get(k)
    e1.record(s)
    torch.cuda.synchronize()
    print(f"batch {i:2d}: lines/get {L:.4f}  k_get_u {e0.elapsed_time(e1) * 100:.1f} us", flush=True)
