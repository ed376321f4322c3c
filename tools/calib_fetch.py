"""Counter calibration for the HBM traffic figures (run under rocprofv3 --pmc).

Launches kernels whose HBM bytes are known exactly, in a fixed order, so that
one `--pmc FETCH_SIZE` pass and one `--pmc WRITE_SIZE` pass attribute counts
to each dispatch (tools/calib_summary.py):
  * k_gather, random whole lines of a 4 GiB buffer (past the 256 MiB
    Infinity Cache), 64-B and 128-B lines, 1/2/4 lines in flight per lane
    group: n_ops * line bytes read (the access shapes of k_get_u / k_apply's
    segment lines);
  * a streaming elementwise pass over 1 GiB (1 GiB read + 1 GiB written), the
    shape of k_part's input stream and k_split's 16-KiB parent reads.
Prints the dispatch order and algorithmic bytes as JSON (first line)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import pmdfc_amd.engine as E  # noqa: E402

dev = torch.device("cuda", 0)
n_ops = 1 << 24
buf = torch.empty(4 << 30, dtype=torch.uint8, device=dev)
buf.random_(0, 255)
out = torch.empty(1 << 20, dtype=torch.int64, device=dev)
plan = []
for line in (64, 128):
    for depth in (1, 2, 4):
        E.ubench_gather(buf, n_ops, line, depth, None, 7, out)
        plan.append({"kernel": "k_gather", "line": line, "depth": depth, "read_bytes": n_ops * line, "write_bytes": 0})
src = buf[: 1 << 30]
dst = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
torch.add(src, 1, out=dst)  # an elementwise kernel (a D2D copy may take a DMA engine)
plan.append({"kernel": "copy", "read_bytes": 1 << 30, "write_bytes": 1 << 30})
torch.cuda.synchronize()
print(json.dumps(plan), flush=True)
