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


class RouteOverflowError(RuntimeError):
    """strict BlockRouter: ops were dropped on a full carry (ST_ROUTE_OVERFLOW)."""


class BlockRouter:
    """Routing with fixed-capacity owner blocks: no host sync per batch.

    Each rank packs its batch into 2^shard_bits blocks of `cap` records (one
    per owner, batch order kept inside a block, unused slots keyed INVALID),
    exchanges them with ONE equal-split all_to_all_single, runs the index on
    the 2^shard_bits * cap received rows (padding rows come back
    RESERVED_KEY and are never stored), and returns the responses with a
    second equal-split all-to-all.  Equal splits keep the counts off the
    host: the whole routed batch is enqueued without a synchronisation.

    Skew never drops an op.  Ops past `cap` for one owner wait in the
    packer's per-owner FIFO carry and lead that owner's block in the next
    exchange; a call (insert / get / mixed / *_batches) ends with drain
    exchanges until every rank's carry is empty -- one small all-reduce and
    one host read per call, not per batch.  The order ops are applied in is
    exchange-major, then source-rank-major (all_to_all_single concatenates
    blocks by source), then each rank's FIFO order per owner, so a rank's ops
    on one key (one owner) apply in its batch order.  With no skew every op
    travels in its own batch's exchange, and the order is the rank-major
    concatenation of the ranks' batches.

    Get-only batches also send one row per distinct key of each 1024-Get
    tile (dedupe_gets): the first Get of a key in its tile is routed and the
    others copy its result.  A Get-only global batch changes nothing, so this
    is exact; it keeps a Zipf-hot key (one row per tile instead of one per
    Get) from filling its owner's block.

    Only an op that finds its owner's carry full (carry_cap ops already
    waiting: sustained skew) comes back ST_ROUTE_OVERFLOW unapplied; with
    strict=True the call then raises RouteOverflowError on every rank.

    packer: pmdfc_amd.BlockPacker (the HIP kernels of route.hip) or any
    object with the same methods (the CPU restatement in tests/route_ref.py
    drives this class under gloo).

    Under a gloo process group (tests: several ranks sharing one GPU) device
    payloads are staged through host memory for the exchange; RCCL moves
    them device to device.  A call that raises (an exchange, the index, a
    strict overflow) resets the packer, so no op of the aborted call stays
    in a carry to be re-sent by the next one."""

    def __init__(self, index, packer, group=None, dedupe_gets: bool = True, strict: bool = False, comm=None):
        self.index = index
        self.p = packer
        self.group = group
        self.dedupe_gets = dedupe_gets
        self.strict = strict
        self.comm = comm
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self._host = dist.is_initialized() and dist.get_backend(group) == "gloo"
        if self.world != packer.G:
            raise ValueError(f"world size {self.world} != 2^shard_bits {packer.G}")
        if comm is not None and comm.world != packer.G:
            raise ValueError(f"communicator of {comm.world} ranks != 2^shard_bits {packer.G}")
        mb = getattr(index, "max_batch", None)
        if mb is not None and mb < packer.rows:
            raise ValueError(f"index max_batch {mb} < the {packer.rows} rows an exchange delivers")
        self._ovf_seen = 0

    def _wire(self) -> bool:
        # one rank without a process group: the exchange is the identity (with
        # one, bench --route keeps RCCL in the loop to exercise the N > 1 path)
        return not (self.world == 1 and not dist.is_initialized())

    def _a2a_async(self, x):
        if not self._wire():
            return None, x
        if self._host and x.device.type != "cpu":  # gloo: through host memory, synchronously
            h = x.cpu()
            out = torch.empty_like(h)
            dist.all_to_all_single(out, h, group=self.group)
            return None, out.to(x.device)
        out = torch.empty_like(x)
        return dist.all_to_all_single(out, x, group=self.group, async_op=True), out

    def _all_reduce(self, t, op):
        if self._host and t.device.type != "cpu":
            h = t.cpu()
            dist.all_reduce(h, op=op, group=self.group)
            return h
        dist.all_reduce(t, op=op, group=self.group)
        return t

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

    def _call(self, batches, width, run, resp_width, keeps=None):
        """Route consecutive batches (tuples keys[, values[, ops]]): the
        request exchange of batch i+1 and the response exchange of batch i-1
        travel on the process group's stream while batch i is applied; then
        drain exchanges until no rank carries ops.  Returns per-batch
        (values | None, status) views of the call's outputs."""
        if not batches:
            return []
        try:
            return self._call_body(batches, width, run, resp_width, keeps)
        except BaseException:
            self.p.reset()  # no op of this call may lead the next call's exchange
            self._ovf_seen = 0  # (the reset clears the packer's overflow count too)
            raise

    def _call_body(self, batches, width, run, resp_width, keeps):
        sizes = [b[0].numel() for b in batches]
        bases = [0]
        for n in sizes:
            bases.append(bases[-1] + n)
        total = bases[-1]
        dev = batches[0][0].device
        vals_out = torch.empty(total, dtype=torch.int64, device=dev) if resp_width else None
        st_out = torch.empty(total, dtype=torch.uint8, device=dev)
        dedupe = width == 1 and self.dedupe_gets
        lead = torch.empty(total, dtype=torch.int32, device=dev) if dedupe else None
        nb = len(batches)

        def pack(i):
            if i >= nb:  # drain: only the carried ops
                return self.p.pack(None, None, None, width, None, 0, vals_out, st_out)
            b = batches[i]
            keep = keeps[i] if keeps is not None else None
            if dedupe:
                keep = self.p.dedupe(b[0], keep, bases[i], lead)
            return self.p.pack(b[0], b[1] if width > 1 else None, b[2] if width > 2 else None, width, keep,
                               bases[i], vals_out, st_out)

        def finish(p):
            w, back, rowpos = p
            if w is not None:
                w.wait()
            self.p.unpack(back, resp_width, rowpos, vals_out, st_out)

        def launch(i):
            send, rowpos = pack(i)
            w, recv = self._a2a_async(send)
            return w, recv, rowpos

        fw = launch(0)
        pending = None
        i = 0
        while True:
            if i + 1 < nb:
                nxt = launch(i + 1)
            w, recv, rowpos = fw
            if w is not None:
                w.wait()
            wb, back = self._a2a_async(run(recv))
            if pending:  # the previous exchange's responses travelled while this one was applied
                finish(pending)
            pending = (wb, back, rowpos)
            i += 1
            if i < nb:
                fw = nxt
                continue
            # drain: every rank takes part until no rank carries ops
            c = self.p.carried()
            if self._wire() and self.world > 1:
                c = self._all_reduce(c, dist.ReduceOp.MAX)
            if int(c.item()) == 0:
                break
            fw = launch(nb)
        finish(pending)
        self.p.end_call()
        if dedupe:
            self.p.fill(lead, vals_out, st_out)
        if self.strict:
            self._check_overflow(dev)
        return [(vals_out[bases[j]:bases[j + 1]] if resp_width else None, st_out[bases[j]:bases[j + 1]])
                for j in range(nb)]

    def _check_overflow(self, dev):
        n = self.p.overflow_count()
        t = torch.tensor([n - self._ovf_seen], dtype=torch.int64, device=dev)
        if self._wire() and self.world > 1:
            t = self._all_reduce(t, dist.ReduceOp.SUM)
        self._ovf_seen = n
        if int(t.item()):
            raise RouteOverflowError(f"{int(t.item())} ops dropped on a full routing carry (ST_ROUTE_OVERFLOW)")

    def insert(self, keys: torch.Tensor, values: torch.Tensor) -> torch.Tensor:
        return self._call([(keys, values)], 2, self._run_insert, 0)[0][1]

    def get(self, keys: torch.Tensor):
        return self._call([(keys,)], 1, self._run_get, 1)[0]

    def bloom_get(self, bloom, keys: torch.Tensor):
        """The client path across shards (client/rdpma.c:1050-1061):
        probe the replicated bloom filter locally, route only the positives,
        and return bloom-negatives as ST_FILTERED without an exchange or an
        index probe.  bloom: anything with probe(keys) -> u8 per key."""
        return self._call([(keys,)], 1, self._run_get, 1, keeps=[bloom.probe(keys)])[0]

    def mixed(self, ops: torch.Tensor, keys: torch.Tensor, values: torch.Tensor):
        return self._call([(keys, values, ops)], 3, self._run_mixed, 1)[0]

    def insert_batches(self, batches):
        """[(keys, values)] -> [status]: routed insert batches in order."""
        if self._native():
            bounds = self._bounds([b[0] for b in batches])
            st = self.insert_concat(torch.cat([b[0] for b in batches]), torch.cat([b[1] for b in batches]), bounds)
            return [st[bounds[j]:bounds[j + 1]] for j in range(len(batches))]
        return [r[1] for r in self._call(batches, 2, self._run_insert, 0)]

    def get_batches(self, batches):
        """[keys] -> [(values, status)]: routed Get batches in order."""
        if self._native():
            bounds = self._bounds(batches)
            v, st = self.get_concat(torch.cat(list(batches)), bounds)
            return [(v[bounds[j]:bounds[j + 1]], st[bounds[j]:bounds[j + 1]]) for j in range(len(batches))]
        return self._call([(k,) for k in batches], 1, self._run_get, 1)

    # ---- the native loop (pmdfc_route_batches: RCCL from C++, one call for
    # all batches): the same packs, exchanges and drains as _call_body
    def _native(self) -> bool:
        return self.comm is not None and hasattr(self.p, "route_batches")

    @staticmethod
    def _bounds(keys_list):
        b = [0]
        for k in keys_list:
            b.append(b[-1] + k.numel())
        return b

    def insert_concat(self, keys, values, bounds):
        """Routed insert batches given as one array and batch bounds (ops
        bounds[i] .. bounds[i+1]-1 form batch i) -> call-global statuses."""
        if not self._native():
            st = self.insert_batches([(keys[bounds[j]:bounds[j + 1]], values[bounds[j]:bounds[j + 1]])
                                      for j in range(len(bounds) - 1)])
            return torch.cat(st)
        st = torch.empty(bounds[-1] - bounds[0], dtype=torch.uint8, device=keys.device)
        try:
            self.p.route_batches(self.index, self.comm, 2, keys, values, bounds, False, None, st)
        except BaseException:
            self.p.reset()
            raise
        if self.strict:
            self._check_overflow(keys.device)
        return st

    def get_concat(self, keys, bounds):
        """Routed Get batches as one array and bounds -> (values, statuses)."""
        if not self._native():
            r = self.get_batches([keys[bounds[j]:bounds[j + 1]] for j in range(len(bounds) - 1)])
            return torch.cat([x[0] for x in r]), torch.cat([x[1] for x in r])
        n = bounds[-1] - bounds[0]
        v = torch.empty(n, dtype=torch.int64, device=keys.device)
        st = torch.empty(n, dtype=torch.uint8, device=keys.device)
        try:
            self.p.route_batches(self.index, self.comm, 1, keys, None, bounds, self.dedupe_gets, v, st)
        except BaseException:
            self.p.reset()
            raise
        if self.strict:
            self._check_overflow(keys.device)
        return v, st

    def mixed_batches(self, batches):
        """[(keys, values, ops)] -> [(values, status)]: routed mixed batches in order."""
        if self._native():
            bounds = self._bounds([b[0] for b in batches])
            v, st = self.mixed_concat(torch.cat([b[2] for b in batches]), torch.cat([b[0] for b in batches]),
                                      torch.cat([b[1] for b in batches]), bounds)
            return [(v[bounds[j]:bounds[j + 1]], st[bounds[j]:bounds[j + 1]]) for j in range(len(batches))]
        return self._call(batches, 3, self._run_mixed, 1)

    def mixed_concat(self, ops, keys, values, bounds):
        """Routed mixed batches as one array each and bounds -> (values, statuses)."""
        if not self._native():
            r = self.mixed_batches([(keys[bounds[j]:bounds[j + 1]], values[bounds[j]:bounds[j + 1]],
                                     ops[bounds[j]:bounds[j + 1]]) for j in range(len(bounds) - 1)])
            return torch.cat([x[0] for x in r]), torch.cat([x[1] for x in r])
        n = bounds[-1] - bounds[0]
        ops = ops.to(torch.uint8).contiguous()
        v = torch.empty(n, dtype=torch.int64, device=keys.device)
        st = torch.empty(n, dtype=torch.uint8, device=keys.device)
        try:
            self.p.route_mixed_batches(self.index, self.comm, ops, keys, values, bounds, v, st)
        except BaseException:
            self.p.reset()
            raise
        if self.strict:
            self._check_overflow(keys.device)
        return v, st
