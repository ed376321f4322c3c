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
DEDUP_TILE = 1024  # Get dedupe works within tiles of this many Gets (route.hip k_dedupe_tile)


def owners(keys_u64: np.ndarray, sbits: int) -> np.ndarray:
    if sbits == 0:
        return np.zeros(keys_u64.size, dtype=np.int64)
    return (O.hash64(keys_u64) >> np.uint64(64 - sbits)).astype(np.int64)


def _u(t):
    return t.numpy().view(np.uint64) if t.dtype == torch.int64 else t.numpy()


class TorchBlockPacker:
    """The HIP packer's contract in numpy: per-owner FIFO carry (carried ops
    lead the owner's block, the rest of the batch follows in batch order),
    rows past an owner's total padded with INVALID words and rowpos -1, ops
    past the carry capacity dropped as ST_ROUTE_OVERFLOW, Get dedupe by first
    occurrence within each tile of DEDUP_TILE Gets."""

    def __init__(self, max_batch: int, shard_bits: int, cap: int | None = None, carry_cap: int | None = None):
        self.sbits = shard_bits
        self.G = 1 << shard_bits
        self.max_batch = max_batch
        self.cap = cap or route_capacity(max_batch, shard_bits)
        self.carry_cap = carry_cap or max_batch
        self.rows = self.G * self.cap
        self.reset()

    def reset(self):
        e = np.zeros(0, np.uint64)
        self.carry = [(e, e, e, np.zeros(0, np.int64)) for _ in range(self.G)]
        self.ovf = 0

    def pack(self, keys, vals, ops, width, keep=None, base=0, vals_out=None, st_out=None):
        n = 0 if keys is None else keys.numel()
        if n > self.max_batch:
            raise ValueError("batch > max_batch")
        k = _u(keys) if n else np.zeros(0, np.uint64)
        v = _u(vals) if (n and width > 1) else np.zeros(n, np.uint64)
        o = ops.numpy().astype(np.uint64) if (n and width > 2) else np.zeros(n, np.uint64)
        live = np.ones(n, bool) if keep is None else np.asarray(keep).astype(bool)
        own = owners(k, self.sbits)
        so = st_out.numpy() if n else None
        vo = vals_out.numpy() if (n and vals_out is not None) else None

        def not_sent(idx, st):
            so[base + idx] = st
            if vo is not None:
                vo[base + idx] = 0

        if n:
            not_sent(np.nonzero(~live)[0], ST_FILTERED)
        send = np.full((self.G, self.cap, width), INVALID, dtype=np.uint64)
        rowpos = np.full((self.G, self.cap), -1, dtype=np.int64)
        for g in range(self.G):
            idx = np.nonzero(live & (own == g))[0]
            ck, cv, co, cp = self.carry[g]
            qk = np.concatenate([ck, k[idx]])
            qv = np.concatenate([cv, v[idx]])
            qo = np.concatenate([co, o[idx]])
            qp = np.concatenate([cp, base + idx])
            m = min(qk.size, self.cap)
            send[g, :m, 0] = qk[:m]
            if width > 1:
                send[g, :m, 1] = qv[:m]
            if width > 2:
                send[g, :m, 2] = qo[:m]
            rowpos[g, :m] = qp[:m]
            c = min(qk.size - m, self.carry_cap)
            self.carry[g] = (qk[m:m + c], qv[m:m + c], qo[m:m + c], qp[m:m + c])
            drop = qp[m + c:]
            if drop.size:
                so[drop] = ST_ROUTE_OVERFLOW
                if vo is not None:
                    vo[drop] = 0
                self.ovf += drop.size
        return (torch.from_numpy(send.reshape(-1).view(np.int64)),
                torch.from_numpy(rowpos.reshape(-1).astype(np.int32)))

    def unpack(self, back, resp_width, rowpos, vals_out, st_out):
        p = rowpos.numpy().astype(np.int64)
        ok = p >= 0
        so = st_out.numpy()
        if resp_width == 0:
            so[p[ok]] = back.numpy()[ok]
            return
        b = back.numpy().reshape(-1, 2)
        if vals_out is not None:
            vals_out.numpy()[p[ok]] = b[ok, 0]
        so[p[ok]] = b[ok, 1].astype(np.uint8)

    def carried(self):
        return torch.tensor([sum(c[0].size for c in self.carry)], dtype=torch.int64)

    def end_call(self):
        pass

    def overflow_count(self):
        return self.ovf

    def dedupe(self, keys, keep=None, base=0, lead_out=None):
        k = _u(keys)
        n = k.size
        live = np.ones(n, bool) if keep is None else np.asarray(keep).astype(bool)
        lead = np.arange(n, dtype=np.int64)
        for t0 in range(0, n, DEDUP_TILE):  # leader: the key's first Get in its tile
            cand = t0 + np.nonzero((live & (k != INVALID))[t0:t0 + DEDUP_TILE])[0]
            _, first, inv = np.unique(k[cand], return_index=True, return_inverse=True)
            lead[cand] = cand[first[inv]]
        lead_out.numpy()[base:base + n] = (base + lead).astype(np.int32)
        return torch.from_numpy(((lead == np.arange(n)) & live).astype(np.uint8))

    def fill(self, lead, vals_out, st_out):
        ld = lead.numpy().astype(np.int64)
        if vals_out is not None:
            vals_out.numpy()[:] = vals_out.numpy()[ld]
        st_out.numpy()[:] = st_out.numpy()[ld]

    def split(self, recv, width):
        r = recv.numpy().reshape(self.rows, width)
        keys = torch.from_numpy(np.ascontiguousarray(r[:, 0]))
        vals = torch.from_numpy(np.ascontiguousarray(r[:, 1])) if width > 1 else None
        ops = torch.from_numpy(r[:, 2].astype(np.uint8)) if width > 2 else None
        return keys, vals, ops

    def respond(self, vals, st):
        v = vals.numpy()
        return torch.from_numpy(np.stack([v, st.numpy().astype(np.int64)], axis=1).reshape(-1))


def serial_order(batches_per_rank, sbits, cap, carry_cap):
    """The order a BlockRouter call applies ops in, restated independently of
    the packer: per (source rank, owner) FIFO queues; exchange e takes the
    first `cap` ops of every queue after appending batch e's ops (drain
    exchanges append nothing); owners are disjoint, so the global order is
    exchange-major, then source-rank-major, then FIFO.  Ops that find
    `carry_cap` ops still queued after an exchange are dropped.
    batches_per_rank[r][e] = numpy u64 keys of rank r's e-th batch (already
    deduped if the call dedupes).  Returns (order, dropped): lists of
    (rank, batch, index)."""
    world = len(batches_per_rank)
    G = 1 << sbits
    q = [[[] for _ in range(G)] for _ in range(world)]
    order, dropped = [], []
    nb = len(batches_per_rank[0])
    e = 0
    while True:
        for r in range(world):
            if e < nb:
                k = batches_per_rank[r][e]
                own = owners(k, sbits)
                for i in range(k.size):
                    q[r][own[i]].append((r, e, i))
        for r in range(world):
            for g in range(G):
                order.extend(q[r][g][:cap])
                rest = q[r][g][cap:]
                dropped.extend(rest[carry_cap:])
                q[r][g] = rest[:carry_cap]
        e += 1
        if e >= nb and not any(q[r][g] for r in range(world) for g in range(G)):
            return order, dropped
