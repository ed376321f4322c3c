import sys, time
sys.argv = ["bench.py", "--no-cpu-baseline"]
sys.path.insert(0, "/root/repo")
import torch
import pmdfc_amd as P
B = 1 << 20; NK = 1 << 26; nb = NK // B
idx = P.CCEH(65536, max_batch=B, max_segments=int(NK / 512 * 1.25) + 65536 + 1024, device=0)
keys = [P.gen_keys(1000, i * B, B) for i in range(nb)]
allk = torch.cat(keys); bounds = [i * B for i in range(nb + 1)]
def step():
    idx.reset()
    idx.InsertBatches(allk, allk, bounds)
    for i in range(nb): idx.Get(keys[i])
for ev in (False, True, False):
    idx.timing(events=ev)
    step(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3): step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 3
    print(f"events={ev}: {dt*1e3:.3f} ms/step  {2*NK/dt/1e6:.0f} Mops/s", flush=True)
