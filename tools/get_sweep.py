"""Get-path experiment (GPU box only): k_get_u per 1M-Get launch on the
config-2 table at U = 1, 2, 4 Gets per quad, beside the random-line gather
ceiling at the same launch size (1M lines) and at 64M lines."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pmdfc_amd as P  # noqa: E402
import pmdfc_amd.engine as E  # noqa: E402

B, NB = 1 << 20, 64
dev = torch.device("cuda", 0)
t = P.CCEH(65536, max_batch=B, max_segments=1 << 18, device=0)
keys = P.gen_keys(2, 0, NB * B)
t.InsertBatches(keys, keys, list(range(0, NB * B + 1, B)))
torch.cuda.synchronize()
s = torch.cuda.current_stream(dev)


def timeit(fn, reps=20):
    fn(0)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for r in range(reps):
        fn(r + 1)
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


vo = torch.empty(B, dtype=torch.int64, device=dev)
so = torch.empty(B, dtype=torch.uint8, device=dev)
lib = E.load_library()


def get(r):
    k = keys[(r % NB) * B:(r % NB + 1) * B]
    E._check(lib.pmdfc_cceh_get(t._h, k.data_ptr(), vo.data_ptr(), so.data_ptr(), B, s.cuda_stream), "get")


us = timeit(get)
get(5)
ok = bool((so == P.ST_HIT).all()) and torch.equal(vo, keys[5 * B:6 * B])
print(f"Get (pipe {os.environ.get('PMDFC_GET_PIPE', '1')}, U {os.environ.get('PMDFC_GET_UNROLL', '2')}): "
      f"{us:7.1f} us per 1M Gets  ok={ok}  lines/get {t.stats().get('get_lines', 'n/a')}", flush=True)
if os.environ.get("GATHER", "0") != "1":
    sys.exit(0)
del t
buf = torch.empty(4 << 30, dtype=torch.uint8, device=dev)
buf.random_(0, 255)
table = torch.randint(0, (4 << 30) // 128 // 64, (1 << 18,), dtype=torch.int32, device=dev)
out = torch.empty(1 << 20, dtype=torch.int64, device=dev)
for n in (1 << 20, 1 << 26):
    for depth in (1, 2, 4):
        for name, tb in (("plain", None), ("dep", table)):
            us = timeit(lambda r: E.ubench_gather(buf, n, 64, depth, tb, r + 2, out), reps=5 if n > B else 20)
            print(f"gather {name:5s} 64B x{depth} n={n >> 20}M: {us * B / n:7.1f} us per 1M lines", flush=True)
