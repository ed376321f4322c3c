"""The HIP routing path (route.hip through pmdfc_amd.BlockPacker) against a
real peer: two ranks on ONE MI355X, each with its own engine (shard 0 / 1 of
the hash prefix) and its own HIP packer, exchanging over a gloo process group
(BlockRouter stages the device payloads through host memory under gloo; RCCL
moves them device to device on a multi-GPU node).  Every result and both
shards' tables equal ONE serial oracle run in the order the protocol promises
(tests/route_ref.py serial_order, restated from the queues alone), including
owner skew that forces carried exchanges and Zipf Gets deduplicated per tile.
Not a scaling measurement: it proves the HIP pack / carry / unpack / dedupe
with a peer."""
import os

import numpy as np
import pytest

import scenarios as S
from oracle import oracle as O
from pmdfc_amd.workload import uniform_keys, zipf_ranks

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

from test_dist_gloo import _free_port, _owner_skewed  # noqa: E402

WORLD, SBITS, MAXB, DEPTH = 2, 1, 4096, 6


def _worker(rank, port, streams, gets, cap, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        import pmdfc_amd as P
        from pmdfc_amd.dist import BlockRouter
        dev = torch.device("cuda", 0)
        pk = P.BlockPacker(0, MAXB, SBITS, cap=cap)
        idx = P.CCEH(depth=DEPTH, shard_bits=SBITS, shard_id=rank, max_batch=pk.rows, max_segments=4096)
        r = BlockRouter(idx, pk, strict=True)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)
        outs = []
        for v, st in r.mixed_batches([(t(k), t(v), torch.from_numpy(o).to(dev)) for o, k, v in streams[rank]]):
            outs.append((v.cpu().numpy().view(np.uint64).copy(), st.cpu().numpy().copy()))
        carried = int(pk.carried().item())
        gouts = []
        for v, st in r.get_batches([t(k) for k in gets[rank]]):
            gouts.append((v.cpu().numpy().view(np.uint64).copy(), st.cpu().numpy().copy()))
        d = idx.dump()
        q.put((rank, outs, gouts, d["keys"], d["values"], d["local_depth"], d["prefix"], carried,
               pk.overflow_count()))
        idx.close()
        pk.close()
    finally:
        dist.barrier()
        dist.destroy_process_group()


@pytest.mark.parametrize("cap", [None, 600])
def test_hip_router_world2_one_gpu(cap):
    """Mixed batches whose keys pile onto owner 0 (60 % of each rank's
    distinct keys) -- cap 600 forces several carried exchanges per batch --
    then Zipf(0.99) Get batches over everything inserted (deduplicated per
    1024-Get tile on the device)."""
    from route_ref import ST_ROUTE_OVERFLOW, route_capacity, serial_order
    nb, n = 3, 3000
    capv = cap or route_capacity(MAXB, SBITS)
    streams = []
    for r in range(WORLD):
        bs = []
        for e in range(nb):
            keys = _owner_skewed(1700 + 10 * r + e, n, SBITS, 0, 0.6)
            rng = np.random.default_rng(1900 + 10 * r + e)
            ops = (rng.random(n) < 0.5).astype(np.uint8)
            pool = np.concatenate([keys, _owner_skewed(1700 + 10 * ((r + 1) % WORLD) + e, n, SBITS, 0, 0.6)])
            gk = pool[rng.integers(0, pool.size, n)]
            keys = np.where(ops == 1, keys, gk)
            vals = np.where(ops == 1, S._vals(keys), np.uint64(0))
            bs.append((ops, keys, vals))
        streams.append(bs)
    rng = np.random.default_rng(77)
    allk = np.concatenate([b[1] for r in range(WORLD) for b in streams[r]] + [uniform_keys(1999, 0, 500)])
    gets = [[allk[zipf_ranks(rng, allk.size, 0.99, MAXB)] for _ in range(2)] for _ in range(WORLD)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, streams, gets, cap, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(WORLD):
        out = q.get(timeout=240)
        res[out[0]] = out[1:]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    order, dropped = serial_order([[b[1] for b in streams[r]] for r in range(WORLD)], SBITS, capv, MAXB)
    assert not dropped
    g = O.OracleCCEH(DEPTH)
    o = np.array([streams[r][e][0][i] for r, e, i in order], np.uint8)
    k = np.array([streams[r][e][1][i] for r, e, i in order], np.uint64)
    v = np.array([streams[r][e][2][i] for r, e, i in order], np.uint64)
    gv, gs = g.mixed(o, k, v)
    exp = {(r, e): (np.zeros(n, np.uint64), np.zeros(n, np.uint8)) for r in range(WORLD) for e in range(nb)}
    for j, (r, e, i) in enumerate(order):
        exp[(r, e)][0][i] = gv[j]
        exp[(r, e)][1][i] = gs[j]
    for r in range(WORLD):
        outs, gouts, _, _, _, _, carried, ovf = res[r]
        assert carried == 0 and ovf == 0
        for e in range(nb):
            got_v, got_s = outs[e]
            assert not (got_s == ST_ROUTE_OVERFLOW).any()
            assert np.array_equal(got_s, exp[(r, e)][1]), (r, e)
            assert np.array_equal(got_v, exp[(r, e)][0]), (r, e)
        for e, keys in enumerate(gets[r]):  # a Get-only batch changes nothing
            ev, es = g.get(keys)
            assert np.array_equal(gouts[e][1], es) and np.array_equal(gouts[e][0], ev), (r, e)
    gd = g.dump()
    ks, vs = [], []
    for r in range(WORLD):
        _, _, kk, vv, ld, pf, _, _ = res[r]
        own = (pf.astype(np.uint64) >> (ld.astype(np.uint64) - np.uint64(SBITS))) == np.uint64(r)
        ks.append(kk.reshape(-1, 1024)[own].ravel())
        vs.append(vv.reshape(-1, 1024)[own].ravel())
    assert np.array_equal(np.concatenate(ks), gd["keys"])
    assert np.array_equal(np.concatenate(vs), gd["values"])


def _native_worker(rank, port, streams, gets, cap, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        import pmdfc_amd as P
        from pmdfc_amd.dist import BlockRouter
        d = rank % torch.cuda.device_count()  # (one GPU: both ranks on it, which RCCL refuses)
        dev = torch.device("cuda", d)
        torch.cuda.set_device(d)
        try:
            comm = P.Comm(d)
        except P.PmdfcError as e:
            q.put((rank, "skip", str(e)))
            return
        pk = P.BlockPacker(d, MAXB, SBITS, cap=cap)
        idx = P.CCEH(depth=DEPTH, shard_bits=SBITS, shard_id=rank, max_batch=pk.rows, max_segments=4096,
                     device=d)
        r = BlockRouter(idx, pk, strict=True, comm=comm)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)
        st = [s.cpu().numpy().copy() for s in r.insert_batches([(t(k), t(v)) for k, v in streams[rank]])]
        gouts = [(v.cpu().numpy().view(np.uint64).copy(), s.cpu().numpy().copy())
                 for v, s in r.get_batches([t(k) for k in gets[rank]])]
        q.put((rank, st, gouts, int(pk.carried().item()), pk.overflow_count()))
        idx.close()
        pk.close()
        comm.close()
    finally:
        dist.barrier()
        dist.destroy_process_group()


@pytest.mark.parametrize("cap", [None, 600])
def test_native_router_world2_one_gpu(cap):
    """pmdfc_route_batches with a real peer: two ranks, each with its own
    engine shard, HIP packer and a two-rank RCCL communicator of the engine's
    own (grouped send/recv of the peer blocks, the local block never copied).
    Insert batches skewed onto owner 0 (cap 600: carried exchanges and drains),
    then Zipf Gets: every result equals ONE serial oracle run in the
    protocol's order.  Rank r on GPU r % count: on a one-GPU box RCCL refuses
    two ranks on one device and the test skips."""
    from route_ref import route_capacity, serial_order
    nb, n = 3, 3000
    capv = cap or route_capacity(MAXB, SBITS)
    streams = []
    for r in range(WORLD):
        bs = []
        for e in range(nb):
            keys = _owner_skewed(2700 + 10 * r + e, n, SBITS, 0, 0.6)
            bs.append((keys, S._vals(keys)))
        streams.append(bs)
    rng = np.random.default_rng(78)
    allk = np.concatenate([b[0] for r in range(WORLD) for b in streams[r]] + [uniform_keys(2999, 0, 500)])
    gets = [[allk[zipf_ranks(rng, allk.size, 0.99, MAXB)] for _ in range(2)] for _ in range(WORLD)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_native_worker, args=(r, port, streams, gets, cap, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(WORLD):
        out = q.get(timeout=240)
        res[out[0]] = out[1:]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    if any(v[0] == "skip" for v in res.values()):
        pytest.skip("RCCL: " + next(v[1] for v in res.values() if v[0] == "skip"))
    order, dropped = serial_order([[b[0] for b in streams[r]] for r in range(WORLD)], SBITS, capv, MAXB)
    assert not dropped
    g = O.OracleCCEH(DEPTH)
    k = np.array([streams[r][e][0][i] for r, e, i in order], np.uint64)
    v = np.array([streams[r][e][1][i] for r, e, i in order], np.uint64)
    gs = g.insert(k, v)
    exp = {(r, e): np.zeros(n, np.uint8) for r in range(WORLD) for e in range(nb)}
    for j, (r, e, i) in enumerate(order):
        exp[(r, e)][i] = gs[j]
    for r in range(WORLD):
        st, gouts, carried, ovf = res[r]
        assert carried == 0 and ovf == 0
        for e in range(nb):
            assert np.array_equal(st[e], exp[(r, e)]), (r, e)
        for e, keys in enumerate(gets[r]):
            ev, es = g.get(keys)
            assert np.array_equal(gouts[e][1], es) and np.array_equal(gouts[e][0], ev), (r, e)


def _hosted_worker(rank, port, kind, streams, gets, cap, q, maxb=MAXB):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        import pmdfc_amd as P
        from pmdfc_amd.dist import BlockRouter
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(0)
        comm = P.Comm(0, host_staged=True)
        pk = P.BlockPacker(0, maxb, SBITS, cap=cap)
        idx = P.CCEH(depth=DEPTH, shard_bits=SBITS, shard_id=rank, max_batch=pk.rows, max_segments=4096)
        r = BlockRouter(idx, pk, strict=True, comm=comm)
        assert r._native()
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)
        if kind == "mixed":
            outs = [(v.cpu().numpy().view(np.uint64).copy(), s.cpu().numpy().copy())
                    for v, s in r.mixed_batches([(t(k), t(v), torch.from_numpy(o).to(dev)) for o, k, v in streams[rank]])]
        else:
            outs = [s.cpu().numpy().copy() for s in r.insert_batches([(t(k), t(v)) for k, v in streams[rank]])]
        gouts = [(v.cpu().numpy().view(np.uint64).copy(), s.cpu().numpy().copy())
                 for v, s in r.get_batches([t(k) for k in gets[rank]])]
        d = idx.dump()
        q.put((rank, outs, gouts, int(pk.carried().item()), pk.overflow_count(), comm.exchanges,
               d["keys"], d["values"], d["local_depth"], d["prefix"], pk.rows))
        idx.close()
        pk.close()
        comm.close()
    finally:
        dist.barrier()
        dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["insert", "mixed"])
@pytest.mark.parametrize("cap,maxb,n,nb", [(None, MAXB, 3000, 3), (600, MAXB, 3000, 3), (None, 65536, 60000, 2),
                                          (12000, 65536, 60000, 2)])
def test_native_router_world2_host_staged(kind, cap, maxb, n, nb):
    """The native C++ routed loop (pmdfc_route_batches / pmdfc_route_mixed_batches)
    with a REAL peer on one GPU: two ranks, each with its own engine shard and
    HIP packer, the loop's exchanges and its drain all-reduce carried over gloo
    on host copies (pmdfc_comm_create_host) -- the same packs, local-block
    placement (rank * cap offsets), carries, drains and unpacks as over RCCL,
    only the transport differs.  Owner skew (60 % onto owner 0; cap 600:
    carried exchanges and drains), then Zipf Gets deduplicated per tile.
    Two geometries: 4,096-op batches of 3,000 ops, and 65,536-op batches of
    60,000 ops (the production block capacity B/G (1 + 1/16) + 1024 rows, or a
    12,000-row cap with carries, over tables that split and grow their
    sub-directories between exchanges).  Every op equals ONE serial oracle in
    route_ref.serial_order, and both shards' tables reassemble the oracle's."""
    from route_ref import ST_ROUTE_OVERFLOW, route_capacity, serial_order
    capv = cap or route_capacity(maxb, SBITS)
    streams = []
    for r in range(WORLD):
        bs = []
        for e in range(nb):
            keys = _owner_skewed(3700 + 10 * r + e, n, SBITS, 0, 0.6)
            if kind == "mixed":
                rng = np.random.default_rng(3900 + 10 * r + e)
                ops = (rng.random(n) < 0.5).astype(np.uint8)
                pool = np.concatenate([keys, _owner_skewed(3700 + 10 * ((r + 1) % WORLD) + e, n, SBITS, 0, 0.6)])
                keys = np.where(ops == 1, keys, pool[rng.integers(0, pool.size, n)])
                bs.append((ops, keys, np.where(ops == 1, S._vals(keys), np.uint64(0))))
            else:
                bs.append((keys, S._vals(keys)))
        streams.append(bs)
    kidx = 1 if kind == "mixed" else 0
    rng = np.random.default_rng(79)
    allk = np.concatenate([b[kidx] for r in range(WORLD) for b in streams[r]] + [uniform_keys(3999, 0, 500)])
    gets = [[allk[zipf_ranks(rng, allk.size, 0.99, min(maxb, 3 * n // 2))] for _ in range(2)] for _ in range(WORLD)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_hosted_worker, args=(r, port, kind, streams, gets, cap, q, maxb)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(WORLD):
        out = q.get(timeout=240)
        res[out[0]] = out[1:]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    order, dropped = serial_order([[b[kidx] for b in streams[r]] for r in range(WORLD)], SBITS, capv, maxb)
    assert not dropped
    g = O.OracleCCEH(DEPTH)
    k = np.array([streams[r][e][kidx][i] for r, e, i in order], np.uint64)
    if kind == "mixed":
        o = np.array([streams[r][e][0][i] for r, e, i in order], np.uint8)
        v = np.array([streams[r][e][2][i] for r, e, i in order], np.uint64)
        gv, gs = g.mixed(o, k, v)
    else:
        v = np.array([streams[r][e][1][i] for r, e, i in order], np.uint64)
        gs = g.insert(k, v)
        gv = np.zeros(gs.size, np.uint64)
    exp = {(r, e): (np.zeros(n, np.uint64), np.zeros(n, np.uint8)) for r in range(WORLD) for e in range(nb)}
    for j, (r, e, i) in enumerate(order):
        exp[(r, e)][0][i] = gv[j]
        exp[(r, e)][1][i] = gs[j]
    ks, vs = [], []
    for r in range(WORLD):
        outs, gouts, carried, ovf, nx, kk, vv, ld, pf, rows = res[r]
        assert carried == 0 and ovf == 0
        assert rows == WORLD * capv  # the block geometry the test means
        assert nx >= 2 * nb  # the peer blocks did travel (a request and a response exchange per batch)
        for e in range(nb):
            if kind == "mixed":
                got_v, got_s = outs[e]
                assert np.array_equal(got_v, exp[(r, e)][0]), (r, e)
            else:
                got_s = outs[e]
            assert not (got_s == ST_ROUTE_OVERFLOW).any()
            assert np.array_equal(got_s, exp[(r, e)][1]), (r, e)
        for e, keys in enumerate(gets[r]):  # a Get-only batch changes nothing
            ev, es = g.get(keys)
            assert np.array_equal(gouts[e][1], es) and np.array_equal(gouts[e][0], ev), (r, e)
        own = (pf.astype(np.uint64) >> (ld.astype(np.uint64) - np.uint64(SBITS))) == np.uint64(r)
        ks.append(kk.reshape(-1, 1024)[own].ravel())
        vs.append(vv.reshape(-1, 1024)[own].ravel())
    gd = g.dump()
    assert np.array_equal(np.concatenate(ks), gd["keys"])
    assert np.array_equal(np.concatenate(vs), gd["values"])
