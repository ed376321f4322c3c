"""CPU restatement of the fixed-capacity routing protocol (test infrastructure).

Same pack/split/respond/unpack interface as pmdfc_amd.BlockPacker (the HIP
kernels of pmdfc_amd/csrc/route.hip), in numpy over CPU torch tensors.  It is
the checker for the HIP packer (tests/test_gpu_route.py, bit-exact send
buffers and positions) and drives pmdfc_amd.dist.BlockRouter under gloo
(tests/test_dist_gloo.py).  Owner = top shard_bits of h(key), the bits
CCEH_hybrid indexes its directory with (server/CCEH_hybrid.cpp:119).
"""
import numpy as np
import torch

from oracle import oracle as O
from pmdfc_amd.engine import route_capacity

INVALID = np.uint64(0xFFFFFFFFFFFFFFFF)
ST_ROUTE_OVERFLOW = 9
ST_FILTERED = 7


def owners(keys_u64: np.ndarray, sbits: int) -> np.ndarray:
    if sbits == 0:
        return np.zeros(keys_u64.size, dtype=np.int64)
    return (O.hash64(keys_u64) >> np.uint64(64 - sbits)).astype(np.int64)


def _u(t):
    return t.numpy().view(np.uint64) if t.dtype == torch.int64 else t.numpy()


class TorchBlockPacker:
    def __init__(self, max_batch: int, shard_bits: int, cap: int | None = None):
        self.sbits = shard_bits
        self.G = 1 << shard_bits
        self.max_batch = max_batch
        self.cap = cap or route_capacity(max_batch, shard_bits)
        self.rows = self.G * self.cap

    def pack(self, keys, vals, ops, width, keep=None):
        k = _u(keys)
        n = k.size
        own = owners(k, self.sbits)
        if keep is not None:  # kept home: no slot, pos -2 (kRouteFiltered)
            own = np.where(np.asarray(keep).astype(bool), own, -1)
        send = np.full((self.G, self.cap, width), INVALID, dtype=np.uint64)  # memset 0xFF
        pos = np.full(n, -1, dtype=np.int32)
        for g in range(self.G):
            idx = np.nonzero(own == g)[0][:self.cap]  # batch order; the rest overflow
            m = idx.size
            send[g, :m, 0] = k[idx]
            if width > 1:
                send[g, :m, 1] = _u(vals)[idx]
            if width > 2:
                send[g, :m, 2] = ops.numpy()[idx].astype(np.uint64)
            pos[idx] = g * self.cap + np.arange(m, dtype=np.int32)
        if keep is not None:
            pos[own == -1] = -2
        return torch.from_numpy(send.reshape(-1).view(np.int64)), torch.from_numpy(pos)

    def split(self, recv, width):
        r = recv.numpy().reshape(self.rows, width)
        keys = torch.from_numpy(np.ascontiguousarray(r[:, 0]))
        vals = torch.from_numpy(np.ascontiguousarray(r[:, 1])) if width > 1 else None
        ops = torch.from_numpy(r[:, 2].astype(np.uint8)) if width > 2 else None
        return keys, vals, ops

    def respond(self, vals, st):
        v = vals.numpy()
        return torch.from_numpy(np.stack([v, st.numpy().astype(np.int64)], axis=1).reshape(-1))

    def unpack(self, back, resp_width, pos, n):
        p = pos.numpy().astype(np.int64)
        ok = p >= 0
        st = np.where(p == -2, ST_FILTERED, ST_ROUTE_OVERFLOW).astype(np.uint8)
        if resp_width == 0:
            st[ok] = back.numpy()[p[ok]]
            return None, torch.from_numpy(st)
        b = back.numpy().reshape(-1, 2)
        vals = np.zeros(n, dtype=np.int64)
        vals[ok] = b[p[ok], 0]
        st[ok] = b[p[ok], 1].astype(np.uint8)
        return torch.from_numpy(vals), torch.from_numpy(st)
