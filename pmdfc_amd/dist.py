"""Multi-GPU routing for the sharded CCEH.

The key space shards by the top `shard_bits` of h(key) -- the same MSBs CCEH
indexes its directory with (CCEH_hybrid.cpp:119) -- so every segment lives on
exactly one GPU and a per-shard CCEH reproduces the global serial table.
One process per GPU; a batch is exchanged with two all-to-alls (requests out,
responses back) over RCCL (torch.distributed backend "nccl") on xGMI.

Batch order across ranks: the global batch is the rank-major concatenation of
the ranks' batches; all_to_all_single delivers chunks in source-rank order
and route_by_shard keeps batch order inside a destination, so each owner sees
its ops in global batch order and serial semantics hold.

The bucketing function and the local index are pluggable so the exchange
protocol is tested on CPU with gloo (tests/test_dist_gloo.py).
"""
from __future__ import annotations

from typing import Callable

import torch
import torch.distributed as dist


class ShardRouter:
    def __init__(self, index, shard_bits: int, bucket_fn: Callable, group=None):
        """index: object with Insert/Get/Mixed on tensors of this rank's device.
        bucket_fn(keys) -> (perm LongTensor/IntTensor, counts list[int]) grouping
        the batch by owner shard, stable."""
        self.index = index
        self.shard_bits = shard_bits
        self.bucket = bucket_fn
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1

    def _exchange_counts(self, counts, device):
        send = torch.tensor(counts, dtype=torch.int64, device=device)
        recv = torch.empty_like(send)
        dist.all_to_all_single(recv, send, group=self.group)
        return recv.tolist()

    def _a2a(self, x: torch.Tensor, out_rows: int, out_splits, in_splits) -> torch.Tensor:
        out = torch.empty((out_rows,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        dist.all_to_all_single(out, x.contiguous(), output_split_sizes=out_splits,
                               input_split_sizes=in_splits, group=self.group)
        return out

    def _route(self, keys):
        perm, counts = self.bucket(keys)
        perm = perm.long()
        recv_counts = self._exchange_counts(counts, keys.device)
        return perm, counts, recv_counts

    def insert(self, keys: torch.Tensor, values: torch.Tensor) -> torch.Tensor:
        if self.world == 1:
            return self.index.Insert(keys, values)
        perm, counts, rc = self._route(keys)
        payload = torch.stack([keys[perm], values[perm]], dim=1)
        got = self._a2a(payload, sum(rc), rc, counts)
        st = self.index.Insert(got[:, 0].contiguous(), got[:, 1].contiguous())
        back = self._a2a(st, keys.numel(), counts, rc)
        out = torch.empty_like(back)
        out[perm] = back
        return out

    def get(self, keys: torch.Tensor):
        if self.world == 1:
            return self.index.Get(keys)
        perm, counts, rc = self._route(keys)
        got = self._a2a(keys[perm], sum(rc), rc, counts)
        v, st = self.index.Get(got)
        resp = torch.stack([v, st.to(v.dtype)], dim=1)
        back = self._a2a(resp, keys.numel(), counts, rc)
        vals = torch.empty_like(back[:, 0])
        sts = torch.empty(keys.numel(), dtype=torch.uint8, device=keys.device)
        vals[perm] = back[:, 0]
        sts[perm] = back[:, 1].to(torch.uint8)
        return vals, sts

    def mixed(self, ops: torch.Tensor, keys: torch.Tensor, values: torch.Tensor):
        if self.world == 1:
            return self.index.Mixed(ops, keys, values)
        perm, counts, rc = self._route(keys)
        payload = torch.stack([keys[perm], values[perm], ops[perm].to(keys.dtype)], dim=1)
        got = self._a2a(payload, sum(rc), rc, counts)
        v, st = self.index.Mixed(got[:, 2].to(torch.uint8), got[:, 0].contiguous(),
                                 got[:, 1].contiguous())
        resp = torch.stack([v, st.to(v.dtype)], dim=1)
        back = self._a2a(resp, keys.numel(), counts, rc)
        vals = torch.empty_like(back[:, 0])
        sts = torch.empty(keys.numel(), dtype=torch.uint8, device=keys.device)
        vals[perm] = back[:, 0]
        sts[perm] = back[:, 1].to(torch.uint8)
        return vals, sts


class BlockRouter:
    """Routing with fixed-capacity owner blocks: no host sync per batch.

    Each rank packs its batch into 2^shard_bits blocks of `cap` records (one
    per owner, batch order kept inside a block, unused slots keyed INVALID),
    exchanges them with ONE equal-split all_to_all_single, runs the index on
    the 2^shard_bits * cap received rows (padding rows come back
    RESERVED_KEY and are never stored), and returns the responses with a
    second equal-split all-to-all.  Received rows are in source-rank order,
    so the owner sees the ops in global (rank-major) batch order, as with
    ShardRouter.  An op whose owner block is full gets ST_ROUTE_OVERFLOW and
    is not applied (route_capacity keeps that tens of standard deviations
    away for uniform hashes).  Equal splits keep the counts off the host:
    the whole routed batch is enqueued without a synchronisation.

    packer: pmdfc_amd.BlockPacker (the HIP kernels of route.hip) or any
    object with the same pack/split/respond/unpack methods (the CPU restatement
    in tests/route_ref.py drives this class under gloo).  index.max_batch
    must be >= packer.rows."""

    def __init__(self, index, packer, group=None):
        self.index = index
        self.p = packer
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        if self.world != packer.G:
            raise ValueError(f"world size {self.world} != 2^shard_bits {packer.G}")

    def _a2a(self, x: torch.Tensor) -> torch.Tensor:
        # one rank without a process group: the exchange is the identity (with
        # one, bench --route keeps RCCL in the loop to exercise the N > 1 path)
        if self.world == 1 and not dist.is_initialized():
            return x
        out = torch.empty_like(x)
        dist.all_to_all_single(out, x, group=self.group)
        return out

    # the owner's side: received rows -> response rows.  An engine with the
    # record entry points (pmdfc_cceh_insert_records / get_records) runs
    # straight on the received rows; any other index through split/respond.
    def _run_insert(self, recv):
        if hasattr(self.index, "InsertRecords"):
            return self.index.InsertRecords(recv)
        k, v, _ = self.p.split(recv, 2)
        return self.index.Insert(k, v)

    def _run_get(self, recv):
        if hasattr(self.index, "GetRecords"):
            return self.index.GetRecords(recv)
        v, st = self.index.Get(recv)
        return self.p.respond(v, st)

    def _run_mixed(self, recv):
        k, v, o = self.p.split(recv, 3)
        gv, st = self.index.Mixed(o, k, v)
        return self.p.respond(gv, st)

    def insert(self, keys: torch.Tensor, values: torch.Tensor) -> torch.Tensor:
        send, pos = self.p.pack(keys, values, None, 2)
        st = self._run_insert(self._a2a(send))
        return self.p.unpack(self._a2a(st), 0, pos, keys.numel())[1]

    def get(self, keys: torch.Tensor):
        send, pos = self.p.pack(keys, None, None, 1)
        back = self._a2a(self._run_get(self._a2a(send)))
        return self.p.unpack(back, 1, pos, keys.numel())

    def bloom_get(self, bloom, keys: torch.Tensor):
        """The client path across shards (client/rdpma.c:1050-1061):
        probe the replicated bloom filter locally, route only the positives,
        and return bloom-negatives as ST_FILTERED without an exchange or an
        index probe.  bloom: anything with probe(keys) -> u8 per key."""
        keep = bloom.probe(keys)
        send, pos = self.p.pack(keys, None, None, 1, keep=keep)
        back = self._a2a(self._run_get(self._a2a(send)))
        return self.p.unpack(back, 1, pos, keys.numel())

    def mixed(self, ops: torch.Tensor, keys: torch.Tensor, values: torch.Tensor):
        send, pos = self.p.pack(keys, values, ops, 3)
        back = self._a2a(self._run_mixed(self._a2a(send)))
        return self.p.unpack(back, 1, pos, keys.numel())

    # -- consecutive batches, the exchange of batch i+1 overlapping the engine
    # work of batch i: all-to-alls run async on the process group's stream; the
    # current stream waits for batch i's requests only when it needs them
    def _pipelined(self, batches, width, run, resp_width):
        if self.world == 1 and not dist.is_initialized():
            return [self._one(b, width) for b in batches]
        out = [None] * len(batches)
        fw = [None] * len(batches)

        def launch(i):
            b = batches[i]
            send, pos = self.p.pack(b[0], b[1] if width > 1 else None, b[2] if width > 2 else None, width)
            recv = torch.empty_like(send)
            fw[i] = (dist.all_to_all_single(recv, send, group=self.group, async_op=True), recv, pos)

        def finish(p):
            i, w, back, pos = p
            w.wait()
            out[i] = self.p.unpack(back, resp_width, pos, batches[i][0].numel())

        pending = None
        if batches:
            launch(0)
        for i in range(len(batches)):
            if i + 1 < len(batches):
                launch(i + 1)
            w, recv, pos = fw[i]
            fw[i] = None
            w.wait()
            resp = run(recv)
            back = torch.empty_like(resp)
            wb = dist.all_to_all_single(back, resp, group=self.group, async_op=True)
            if pending:  # batch i-1's responses travelled while batch i was applied
                finish(pending)
            pending = (i, wb, back, pos)
        if pending:
            finish(pending)
        return out

    def _one(self, b, width):
        if width == 1:
            return self.get(b[0])
        if width == 2:
            return (None, self.insert(b[0], b[1]))
        return self.mixed(b[2], b[0], b[1])

    def insert_batches(self, batches):
        """[(keys, values)] -> [status]: routed insert batches in order."""
        return [r[1] for r in self._pipelined(batches, 2, self._run_insert, 0)]

    def get_batches(self, batches):
        """[keys] -> [(values, status)]: routed Get batches in order."""
        return self._pipelined([(k,) for k in batches], 1, self._run_get, 1)

    def mixed_batches(self, batches):
        """[(keys, values, ops)] -> [(values, status)]: routed mixed batches in order."""
        return self._pipelined(batches, 3, self._run_mixed, 1)
