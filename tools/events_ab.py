"""A/B on one GPU (no timing events): config-2 step with the pipelined
multi-batch insert vs batch-by-batch inserts, and the cost of per-class
timing events (GPU box only)."""
import sys
import time

sys.path.insert(0, "/root/repo")
import torch  # noqa: E402

import pmdfc_amd as P  # noqa: E402

B = 1 << 20
NK = 1 << 26
nb = NK // B
idx = P.CCEH(65536, max_batch=B, max_segments=int(NK / 512 * 1.25) + 65536 + 1024, device=0)
keys = [P.gen_keys(1000, i * B, B) for i in range(nb)]
allk = torch.cat(keys)
bounds = [i * B for i in range(nb + 1)]


def step(pipe):
    idx.reset()
    if pipe:
        idx.InsertBatches(allk, allk, bounds)
    else:
        for i in range(nb):
            idx.Insert(keys[i], keys[i])
    for i in range(nb):
        idx.Get(keys[i])


for pipe, ev in ((True, False), (False, False), (True, True), (True, False), (False, False)):
    idx.timing(events=ev)
    step(pipe)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        step(pipe)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 3
    print(f"pipelined={pipe} events={ev}: {dt * 1e3:.3f} ms/step  {2 * NK / dt / 1e6:.0f} Mops/s", flush=True)
