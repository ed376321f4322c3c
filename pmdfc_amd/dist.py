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
