"""bench.py -- batched CCEH lookup+insert throughput on MI355X (BASELINE.json).

Workload (BASELINE.json configs[1]), per GPU:
  64M unique uniform u64 keys (splitmix64 stream, value = key as in
  server/test_KV.cpp:206), CCEH_hybrid(65536) (initial depth 16),
  64 Insert batches of 1M keys, then 64 Get batches of 1M keys (100% hit).
One step = that whole job on a freshly reset index.  Keys are generated into
HBM before the timed region.  With --gpus N (torchrun, one process per GPU)
each rank owns the hash-prefix shard `rank` (top log2 N bits of h(key)) and
feeds its own 64M-key stream; every batch is routed to the owners with RCCL
all-to-alls over xGMI and the results come back the same way (weak scaling).

Prints ONE JSON line on rank 0 (stdout); diagnostics go to stderr.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

import pmdfc_amd as P  # noqa: E402
from pmdfc_amd.dist import BlockRouter  # noqa: E402

METRIC = "batched CCEH lookup+insert Mops/s (1/2/4/8 GPU) + % HBM random-access roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--keys", type=int, default=1 << 26, help="keys per GPU")
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("--init-cap", type=int, default=65536)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=1 << 24)
    ap.add_argument("--config", type=int, default=2, choices=[2, 3, 4, 5, 6, 7],
                    help="2: insert-then-get (headline); 3: YCSB 95/5 Zipf over 256M replay-shape "
                         "keys; 4: 50/50 mixed over 2^28 preloaded keys per GPU (routed for N > 1); 5: bloom probe fused ahead of Get (1e9 bits, k=4); 6: server counting-BF maintenance; 7: replay_KV trace ingestion + replay")
    ap.add_argument("--mixed-batches", type=int, default=16)
    ap.add_argument("--route", action="store_true",
                    help="one GPU: run the N>1 routed path anyway (pack, RCCL all-to-all over a "
                         "1-rank group, unpack) to measure its cost")
    return ap.parse_args()


def main():
    a = parse()
    if a.config == 3:
        return config3(a)
    if a.config == 5:
        return config5(a)
    if a.config == 6:
        return config6(a)
    if a.config == 7:
        return config7(a)
    if a.config == 4:
        return config4(a)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        log(f"note: --gpus {a.gpus} but WORLD_SIZE {world}; using WORLD_SIZE")
    if world & (world - 1):
        raise SystemExit("world size must be a power of two (hash-prefix shards)")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    routed = world > 1 or a.route
    if routed:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        dist.init_process_group("nccl", device_id=dev, rank=rank, world_size=world)
    sbits = int(math.log2(world))
    B, NK = a.batch, a.keys
    nb = NK // B
    depth = P.depth_for_hybrid(a.init_cap)
    max_segs = int(NK / 512 * 1.25) + (1 << (depth - sbits)) + 1024
    # routed: the engine takes the 2^sbits owner blocks of every rank's pack
    # (fixed capacity, INVALID-padded; pmdfc_amd.dist.BlockRouter)
    packer = P.BlockPacker(local, B, sbits) if routed else None
    max_batch = packer.rows if routed else B
    idx = P.CCEH(depth=depth, shard_bits=sbits, shard_id=rank, max_batch=max_batch,
                 max_segments=max_segs, device=local)
    router = BlockRouter(idx, packer) if routed else None

    # inputs resident in HBM before timing
    keys = [P.gen_keys(1000 + rank, i * B, B, device=local) for i in range(nb)]
    st_ins = [torch.empty(B, dtype=torch.uint8, device=dev) for _ in range(nb)]
    out_get = [None] * nb
    torch.cuda.synchronize()

    # one GPU: the 64 batches go through the multi-batch entry point
    # (pmdfc_cceh_insert_batches: same batches, same order, same results; the
    # next batch is partitioned while the current one is applied)
    allk = None if routed else torch.cat(keys)
    bounds = [i * B for i in range(nb + 1)]

    def step(pipelined=True):
        idx.reset()
        if routed:  # consecutive batches, exchange of batch i+1 overlapping batch i
            st_ins[:] = router.insert_batches([(k, k) for k in keys])
            out_get[:] = router.get_batches(keys)
            return
        if pipelined:
            st_all = idx.InsertBatches(allk, allk, bounds)
            for i in range(nb):
                st_ins[i] = st_all[i * B:(i + 1) * B]
        else:
            for i in range(nb):
                st_ins[i] = idx.Insert(keys[i], keys[i])
        for i in range(nb):
            out_get[i] = idx.Get(keys[i])

    for _ in range(a.warmup):
        step()
    # the timed steps run without HIP events: an event at every kernel-class
    # boundary (6 per insert batch) costs ~6 % of the step; the per-class
    # kernel times come from one more, identical step with events (below)
    idx.timing(events=False)
    if routed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    if routed:
        dist.barrier()
    t1 = time.perf_counter()
    idx.timing(events=True)
    idx.timing_read(reset=True)
    # the measured kernel durations (HIP events on the engine stream), batch by
    # batch so no class overlaps another (the timed steps overlap each batch's
    # k_part with the previous batch's apply chain)
    step(pipelined=False)
    torch.cuda.synchronize()
    idx.timing(events=False)
    kt = idx.timing_read(reset=True)
    el = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    if routed:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())

    # correctness of the last timed step (outside the timed region)
    bad = 0
    for i in range(nb):
        bad += int((st_ins[i] != P.ST_INSERTED).sum())
        v, s = out_get[i]
        bad += int(((s != P.ST_HIT) | (v != keys[i])).sum())
    stats = idx.stats()

    # lines per Get on the final table (instrumented k_get, not timed)
    idx.timing(events=False, count_lines=True)
    probe_keys = keys[nb // 2] if world == 1 else None
    lines_per_get = None
    if world == 1:
        idx.Get(probe_keys)
        torch.cuda.synchronize()
        lines_per_get = idx.last_get_lines() / B
    idx.timing(events=False, count_lines=False)

    ops_total = 2 * NK * world * a.steps
    value = ops_total / elapsed / 1e6

    # per-class kernel time on this rank's stream (HIP events over the timed region)
    cls = {k: {"ms": v[0], "launches": v[1]} for k, v in kt.items() if v[1]}  # one step
    dominant = max(cls, key=lambda k: cls[k]["ms"]) if cls else None

    res = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "Mops/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(elapsed / a.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic",
        "config": {
            "workload": "config2: per GPU 64M unique uniform u64 keys (value=key), CCEH_hybrid(65536); "
                        "64 Insert batches of 1M then 64 Get batches of 1M (100% hit); index reset each step",
            "keys_per_gpu": NK, "batch": B, "init_cap": a.init_cap,
            "parallelism": f"hash-prefix shards x{world}" + (", RCCL all-to-all routing (fixed-capacity owner blocks)" if routed else ""),
        },
        "correct": bad == 0,
        "index": {"depth": stats["depth"], "segments": stats["segments"], "splits_per_step": stats["splits"],
                  "insert_passes_per_step": stats["insert_passes"] / max(1, stats["batches"]) if stats["batches"] else None},
        "kernel_ms_per_step": {k: round(v["ms"], 3) for k, v in cls.items()},
    }
    if rank == 0 and world == 1:
        ceil = gather_ceiling(dev, B)
        res["roofline"] = roofline(cls, lines_per_get, B, nb, NK, stats, a.steps, ceil)
        res["get_mops"] = round(NK / (cls["get"]["ms"] / 1e3) / 1e6, 1) if "get" in cls else None
        if not a.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(a, depth)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if routed:
        dist.destroy_process_group()


def gather_ceiling(dev, B, reps=20):
    """Measured random 64-B line gather rate (k_get's access shape) from a
    2 GiB buffer (past the 256 MiB MALL), plain and through a dependent 1 MiB
    u32 table (like the directory).  GB/s of 64-B lines."""
    import pmdfc_amd.engine as E
    buf = torch.empty(2 << 30, dtype=torch.uint8, device=dev)
    buf.random_(0, 255)
    table = torch.randint(0, (2 << 30) // 64 // 64, (1 << 18,), dtype=torch.int32, device=dev)
    out = torch.empty(B, dtype=torch.int64, device=dev)
    res = {}
    for name, tb in (("plain", None), ("dep_table", table)):
        E.ubench_gather64(buf, B, tb, 1, out)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for r in range(reps):
            E.ubench_gather64(buf, B, tb, r + 2, out)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / reps
        res[name] = {"us_per_1M": round(us, 2), "line_GBs": round(B * 64 / (us * 1e-6) / 1e9, 1)}
    del buf
    return res


def roofline(cls, lines_per_get, B, nb, NK, stats, steps, ceil):
    """Roofline of the dominant kernel over the timed region (HIP events on
    the engine stream, one launch per batch per class).  Algorithmic bytes
    (DESIGN.md §5):
      k_get          per Get: 8 key + 64*L + 8 value + 1 status, L = 64-B lines
                     probed, measured on the final table by the instrumented k_get;
      k_apply        (first apply pass) per insert: 16 (key, value) + 1 status +
                     64 (the line of the claimed slot), + 256 per segment run
                     (occupancy bitmap read + write);
      k_scan+k_split per split: 16 KiB parent read + 2 x 16 KiB children written;
      k_part         per op: 16 (key, value) in + 20 (record) out."""
    per = {}
    g = cls.get("get")
    if g and lines_per_get is not None:
        b = B * (17 + 64 * lines_per_get)
        avg = g["ms"] / g["launches"] / 1e3
        per["get"] = {"kernel": "k_get_u", "bytes_per_launch": int(b), "avg_launch_us": round(avg * 1e6, 2),
                      "achieved": round(b / avg / 1e9, 1), "lines_per_get": round(lines_per_get, 4)}
    runs = stats["segment_runs"] / max(1, stats["batches"])  # per batch (the index is reset each step)
    splits_per_batch = stats["splits"] / max(1, nb)
    pr = cls.get("process")
    if pr:
        b = B * (16 + 1 + 64) + runs * 256
        avg = pr["ms"] / pr["launches"] / 1e3
        per["process"] = {"kernel": "k_apply", "bytes_per_launch": int(b),
                          "avg_launch_us": round(avg * 1e6, 2), "achieved": round(b / avg / 1e9, 1),
                          "runs_per_batch": int(runs)}
    rt = cls.get("route")
    if rt:
        b = B * (16 + 20)  # key + value in, a 20-B record out per op
        avg = rt["ms"] / rt["launches"] / 1e3
        per["route"] = {"kernel": "k_part", "bytes_per_launch": int(b),
                        "avg_launch_us": round(avg * 1e6, 2), "achieved": round(b / avg / 1e9, 1)}
    sp = cls.get("split")
    if sp:
        b = splits_per_batch * 49152
        avg = sp["ms"] / sp["launches"] / 1e3
        per["split"] = {"kernel": "k_scan+k_split", "bytes_per_launch": int(b),
                        "avg_launch_us": round(avg * 1e6, 2), "achieved": round(b / avg / 1e9, 1),
                        "splits_per_batch": round(splits_per_batch, 1)}
    dom = max(cls, key=lambda k: cls[k]["ms"])
    pick = per.get(dom) or per.get("get") or {}
    out = {"bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK_GBS, "traffic": None,
           "dominant_class": dom}
    out.update(pick)
    # HBM bytes per launch from the committed rocprofv3 PMC passes (FETCH_SIZE
    # and WRITE_SIZE in separate runs, tools/pmc_summary.py: KiB, gfx950
    # FETCH_SIZE doubled); PMC cannot run inside this process
    pmc_file = os.path.join(REPO, "profiles", "r01", "pmc_traffic.json")
    sym = {"k_apply": "k_apply<false>", "k_get_u": "k_get_u<2, false>", "k_part": "k_part"}.get(out.get("kernel"))
    if sym and os.path.exists(pmc_file):
        pmc = json.load(open(pmc_file)).get(sym)
        if pmc and "hbm_bytes_upper" in pmc:
            out["traffic"] = pmc["hbm_bytes_upper"]
            out["traffic_source"] = (f"profiles/r01/pmc_traffic.json [{sym}], mean of "
                                     f"{pmc['dispatches']} dispatches (tools/insert_run.py, config-2 geometry)")
    if "achieved" in out:
        out["frac"] = round(out["achieved"] / HBM_PEAK_GBS, 4)
    out["per_kernel"] = per
    out["random_gather_ceiling"] = ceil
    if "get" in per and ceil:
        # the metric's "% HBM random-access roofline": Gets against the measured
        # random 64-B line gather rate
        out["get_vs_gather_ceiling"] = round(ceil["plain"]["us_per_1M"] * (B / 1e6) * lines_per_get /
                                             (per["get"]["avg_launch_us"]), 4)
    return out


def cpu_baseline(a, depth):
    """CPU baseline on this host's cores, same workload shape, bounded sample.
    Preferred: the reference's own CCEH_hybrid.cpp (oracle/_ref/ref_driver,
    built from /root/reference in the build container; kind "reference") with
    test_KV's thread pattern (server/test_KV.cpp:204-303, minus the sleep(1)),
    including its clflush emulation (server/util/persist.h:31-41).  Fallback:
    the oracle port, 1 thread."""
    import subprocess
    n = a.cpu_sample
    ref = os.path.join(REPO, "oracle", "_ref", "ref_driver")
    threads = max(1, min(16, os.cpu_count() or 1))
    if os.path.exists(ref):
        try:
            runs = {}
            for T in sorted({1, threads}):
                out = subprocess.run([ref, "bench", str(n), str(T), str(a.init_cap), "1000"],
                                     capture_output=True, text=True, timeout=300, check=True).stdout
                ti, tg, failed = out.split()
                runs[T] = (float(ti), float(tg), int(failed))
            ti, tg, failed = runs[threads]
            return {"value": round(2 * n / (ti + tg) / 1e6, 3), "unit": "Mops/s", "cores": threads,
                    "kind": "reference",
                    "sample": f"reference CCEH_hybrid({a.init_cap}) (-O2), first {n} keys of the rank-0 "
                              f"stream, {threads} threads insert (clflush emulation on) then Get; "
                              f"failedSearch={failed}",
                    "insert_mops": round(n / ti / 1e6, 3), "get_mops": round(n / tg / 1e6, 3),
                    "one_thread": {"insert_mops": round(n / runs[1][0] / 1e6, 3),
                                   "get_mops": round(n / runs[1][1] / 1e6, 3)}}
        except Exception as e:  # fall through to the port
            log(f"reference cpu baseline failed: {e}")
    try:
        from oracle import oracle as O
        from pmdfc_amd.workload import uniform_keys
        k = uniform_keys(1000, 0, n)
        o = O.OracleCCEH(depth, reserve_segments=int(n / 400) + (1 << depth))
        t_ins = o.time_insert(k, flush_ns=10)
        t_get, miss = o.time_get(k, threads=1)
        return {"value": round(2 * n / (t_ins + t_get) / 1e6, 3), "unit": "Mops/s", "cores": 1,
                "kind": "port",
                "sample": f"oracle port, first {n} keys of the rank-0 stream: insert (clflush emulation "
                          f"10 ns/line) then Get, 1 thread; misses={miss}",
                "insert_mops": round(n / t_ins / 1e6, 3), "get_mops": round(n / t_get / 1e6, 3)}
    except Exception as e:  # never let the CPU leg break the GPU line
        return {"value": None, "unit": "Mops/s", "cores": 1, "kind": "port", "sample": f"failed: {e}"}


def replay_key(rank: torch.Tensor) -> torch.Tensor:
    """server/replay_KV.cpp:218-242 shape: key = (inode << 32) + 4096*page with
    inode = 1 + rank // 256, page = rank % 256."""
    return ((1 + (rank >> 8)) << 32) + ((rank & 255) << 12)


def _time_steps(fn, steps, warmup):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return time.perf_counter() - t0


def config3(a):
    """SURVEY §8d config 3 on one GPU: 268,435,456 preloaded replay-shape keys
    (inode in [1, 2^20], page in [0, 256)), then mixed batches of 1M: 95% Get
    drawn Zipf(0.99) over the preloaded ranks (fixed seeded scramble), 5%
    Insert of fresh keys (inode > 2^20).  One step = --mixed-batches batches."""
    from pmdfc_amd.workload import scramble, zipf_ranks
    dev = torch.device("cuda", 0)
    B = a.batch
    n_pre = 1 << 28
    idx = P.CCEH(a.init_cap, max_batch=B, max_segments=int(n_pre / 500) + 65536 + 262144, device=0)
    t0 = time.perf_counter()
    for off in range(0, n_pre, B):
        k = replay_key(torch.arange(off, off + B, dtype=torch.int64, device=dev))
        st = idx.Insert(k, k)
    torch.cuda.synchronize()
    preload_s = time.perf_counter() - t0
    rng = np.random.default_rng(3)
    nbt = a.mixed_batches
    ops_l, keys_l = [], []
    fresh = 0
    for _ in range(nbt):
        is_ins = rng.random(B) < 0.05
        r = scramble(zipf_ranks(rng, n_pre, 0.99, B), n_pre, 33)
        nf = int(is_ins.sum())
        r[is_ins] = n_pre + fresh + np.arange(nf)
        fresh += nf
        rk = replay_key(torch.from_numpy(r).to(dev))
        ops_l.append(torch.from_numpy(is_ins.astype(np.uint8)).to(dev))
        keys_l.append(rk)
    outs = [None] * nbt

    def step():
        for i in range(nbt):
            outs[i] = idx.Mixed(ops_l[i], keys_l[i], keys_l[i])

    # fresh keys are inserted in the first (warmup) pass; later passes re-insert
    # them -> duplicates, so the timed steps use a fresh index state per run:
    # time exactly one pass over the precomputed batches (steps = 1 pass each)
    idx.timing(events=True)
    idx.timing_read(reset=True)
    el = _time_steps(step, 1, 0)
    kt = idx.timing_read(reset=True)
    idx.timing(events=False)
    bad = 0
    for i in range(nbt):
        v, s = outs[i]
        g = ops_l[i] == 0
        bad += int(((s[g] != P.ST_HIT) | (v[g] != keys_l[i][g])).sum())
        bad += int((s[~g] != P.ST_INSERTED).sum())
    stats = idx.stats()
    res = {"metric": METRIC, "value": round(nbt * B / el / 1e6, 3), "unit": "Mops/s", "n_gpus": 1,
           "steps": 1, "warmup": 0, "ms_per_step": round(el * 1e3, 3), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "u64", "data": "synthetic",
           "config": {"workload": f"config3: 2^28 replay-shape keys preloaded, {nbt} mixed batches of {B}: "
                                  "95% Zipf(0.99) Get / 5% fresh Insert", "init_cap": a.init_cap},
           "correct": bad == 0, "preload_s": round(preload_s, 3),
           "preload_insert_mops": round(n_pre / preload_s / 1e6, 1),
           "index": {"depth": stats["depth"], "segments": stats["segments"]},
           "kernel_ms": {k: round(v[0], 3) for k, v in kt.items() if v[1]}}
    print(json.dumps(res), flush=True)


def config4(a):
    """SURVEY §8d config 4, per GPU: 2^28 uniform keys preloaded (2^31 over
    8 GPUs), then mixed batches of 1M, 50% Get of preloaded keys (uniform) /
    50% Insert of fresh keys.  N > 1: every batch is routed to the owners by
    hash prefix (BlockRouter, RCCL all-to-all), weak scaling; N = 1: the
    engine directly.  One step = --mixed-batches batches."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    routed = world > 1 or a.route
    if routed:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        dist.init_process_group("nccl", device_id=dev, rank=rank, world_size=world)
    sbits = int(math.log2(world))
    B, n_pre, nbt = a.batch, 1 << 28, a.mixed_batches
    depth = P.depth_for_hybrid(a.init_cap)
    packer = P.BlockPacker(local, B, sbits) if routed else None
    idx = P.CCEH(depth=depth, shard_bits=sbits, shard_id=rank, max_batch=packer.rows if routed else B,
                 max_segments=int((n_pre + (a.warmup + a.steps) * nbt * B // 2) / 480) + 65536, device=local)
    router = BlockRouter(idx, packer) if routed else None
    t0 = time.perf_counter()
    pre = [P.gen_keys(4000 + rank, i * B, B, device=local) for i in range(n_pre // B)]
    if routed:
        for i in range(0, len(pre), 16):
            router.insert_batches([(k, k) for k in pre[i:i + 16]])
    else:
        for k in pre:
            idx.Insert(k, k)
    torch.cuda.synchronize()
    preload_s = time.perf_counter() - t0
    rng = np.random.default_rng(4 + rank)
    total = a.warmup + a.steps
    batches = []
    for j in range(total * nbt):
        is_ins = torch.from_numpy((rng.random(B) < 0.5).astype(np.uint8)).to(dev)
        r = torch.from_numpy(rng.integers(0, n_pre, B)).to(dev)  # Gets: uniform over the preload
        fresh = P.gen_keys(4000 + rank, n_pre + j * B, B, device=local)
        batches.append((is_ins, fresh, r))
    allpre = torch.cat(pre)
    del pre
    for j, (is_ins, fresh, r) in enumerate(batches):
        k = torch.where(is_ins.bool(), fresh, allpre[r])
        batches[j] = (k, k, is_ins)
    del allpre
    outs = []

    def run(bs):
        if routed:
            return router.mixed_batches(bs)
        return [idx.Mixed(o, k, v) for k, v, o in bs]

    for w in range(a.warmup):
        run(batches[w * nbt:(w + 1) * nbt])
    torch.cuda.synchronize()
    if routed:
        dist.barrier()
    t1 = time.perf_counter()
    for s_ in range(a.steps):
        o = a.warmup + s_
        outs = run(batches[o * nbt:(o + 1) * nbt])
    torch.cuda.synchronize()
    if routed:
        dist.barrier()
    el = time.perf_counter() - t1
    if routed:
        tt = torch.tensor([el], device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt)
    last = batches[(a.warmup + a.steps - 1) * nbt:]
    bad = 0
    for (k, _, o), (v, st) in zip(last, outs):
        g = o == 0
        bad += int(((st[g] != P.ST_HIT) | (v[g] != k[g])).sum()) + int((st[~g] != P.ST_INSERTED).sum())
    if routed:
        bt = torch.tensor([bad], device=dev)
        dist.all_reduce(bt)
        bad = int(bt)
    n = world * a.steps * nbt * B
    if rank == 0:
        stats = idx.stats()
        res = {"metric": METRIC, "value": round(n / el / 1e6, 3), "unit": "Mops/s", "n_gpus": world,
               "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(el / a.steps * 1e3, 3),
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64",
               "data": "synthetic",
               "config": {"workload": f"config4: per GPU 2^28 preloaded uniform keys, {nbt} mixed batches of {B} "
                                      "per step, 50% Get (preloaded, uniform) / 50% fresh Insert",
                          "keys_per_gpu": n_pre, "batch": B, "init_cap": a.init_cap,
                          "parallelism": f"hash-prefix shards x{world}" + (", RCCL all-to-all routing" if routed else "")},
               "correct": bad == 0, "preload_s": round(preload_s, 2),
               "index": {"depth": stats["depth"], "segments": stats["segments"]}}
        print(json.dumps(res), flush=True)
    if routed:
        dist.destroy_process_group()


def config5(a):
    """the client bloom filter (1e9 bits, k=4, MSB-first)
    built from the 64M inserted keys of config 2, probed ahead of Get on 1M
    keys (50% present / 50% absent): negatives never reach the index."""
    dev = torch.device("cuda", 0)
    B, NK = a.batch, a.keys
    idx = P.CCEH(a.init_cap, max_batch=B, max_segments=int(NK / 512 * 1.25) + 65536 + 1024, device=0)
    bf = P.BloomFilter(1000000000, 4, device=0)
    for i in range(NK // B):
        k = P.gen_keys(1000, i * B, B)
        idx.Insert(k, k)
        bf.add(k)
    probes = []
    for i in range(16):
        present = P.gen_keys(1000, (i * B // 2) % NK, B // 2)
        absent = P.gen_keys(1000, NK + i * B // 2, B // 2)
        probes.append(torch.cat([present, absent]))
    outs = [None] * len(probes)

    def step():
        for i, k in enumerate(probes):
            outs[i] = bf.probe_then_get(idx, k)

    idx.timing(events=True)
    idx.timing_read(reset=True)
    el = _time_steps(step, a.steps, a.warmup)
    kt = idx.timing_read(reset=True)
    filtered = sum(int((o[1] == P.ST_FILTERED).sum()) for o in outs)
    bad = 0
    for i, k in enumerate(probes):
        v, s = outs[i]
        bad += int(((s[: B // 2] != P.ST_HIT) | (v[: B // 2] != k[: B // 2])).sum())
        bad += int((s[B // 2:] == P.ST_HIT).sum())
    n = len(probes) * B * a.steps
    res = {"metric": METRIC, "value": round(n / el / 1e6, 3), "unit": "Mops/s", "n_gpus": 1,
           "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(el / a.steps * 1e3, 3),
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64",
           "data": "synthetic",
           "config": {"workload": "config5: bloom 1e9 bits k=4 over 64M keys, 16 x 1M fused probe+Get, "
                                  "50% present / 50% absent", "init_cap": a.init_cap},
           "correct": bad == 0, "filtered_fraction_of_absent": round(filtered / (len(probes) * B / 2), 4),
           "kernel_ms": {k: round(v[0], 3) for k, v in kt.items() if v[1]}}
    print(json.dumps(res), flush=True)


def config6(a):
    """the server's counting bloom filter maintenance
    (server/KV.cpp:113-121, counting_bloom_filter.h): 1e9 u8 counters, k=4.
    One step = Clear, 64 Insert batches of 1M keys (the config-2 stream), one
    ToOrdinaryBloomFilter pack (what rdma_svr.cpp:256-264 does every 10 s),
    one Delete batch of 1M present keys.  value = Insert Mops/s."""
    dev = torch.device("cuda", 0)
    B, NK, m, k = a.batch, a.keys, 1000000000, 4
    f = P.CountingBloomFilter(k, m, device=0)
    keys = [P.gen_keys(1000, i * B, B) for i in range(NK // B)]
    dels = P.gen_keys(1000, 7 * B, B)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
    acc = {"insert": 0.0, "pack": 0.0, "delete": 0.0}
    state = {"deleted": None}

    def step(record=False):
        f.Clear()
        ev[0].record()
        for kk in keys:
            f.Insert(kk)
        ev[1].record()
        f.ToOrdinaryBloomFilter()
        ev[2].record()
        state["deleted"] = f.Delete(dels)
        ev[3].record()
        if record:
            torch.cuda.synchronize()
            acc["insert"] += ev[0].elapsed_time(ev[1])
            acc["pack"] += ev[1].elapsed_time(ev[2])
            acc["delete"] += ev[2].elapsed_time(ev[3])

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step(record=True)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    ins_ms = acc["insert"] / a.steps
    pack_ms = acc["pack"] / a.steps
    del_ms = acc["delete"] / a.steps
    # correctness: every deleted key was present (Delete = 1); inserted keys of
    # other batches still pass QueryBitBloom on the packed bitmap; the packed
    # bitmap's popcount equals the nonzero counters of the reference's pack
    ok = bool((state["deleted"] == 1).all())
    f.ToOrdinaryBloomFilter()
    ok &= bool((f.QueryBitBloom(keys[0]) == 1).all())
    absent = P.gen_keys(1000, NK + 12345, B)
    fpr = float(f.QueryBitBloom(absent).float().mean())
    n_ins = len(keys) * B
    bytes_ins = n_ins / len(keys) * (8 + k * 128)  # per launch: key + k random 64 B lines read+written
    ins_us = ins_ms * 1e3 / len(keys)
    pack_bytes = m + m / 8
    # HBM bytes per launch from the committed PMC passes (FETCH_SIZE / WRITE_SIZE,
    # tools/pmc_summary.py): random line RMWs count FETCH_SIZE as is ("lower"),
    # the streaming pack doubles it per the MI355X guide's gfx950 note ("upper")
    tr_ins = tr_pack = None
    pmc = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "r01", "pmc_traffic_cbf.json")
    if os.path.exists(pmc):
        with open(pmc) as fh:
            pj = json.load(fh)
        tr_ins = pj.get("k_cbf_insert", {}).get("hbm_bytes_lower")
        tr_pack = pj.get("k_cbf_pack", {}).get("hbm_bytes_upper")
    res = {"metric": METRIC, "value": round(n_ins / (ins_ms / 1e3) / 1e6, 3), "unit": "Mops/s", "n_gpus": 1,
           "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(el / a.steps * 1e3, 3),
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
           "data": "synthetic",
           "config": {"workload": f"config6 (SURVEY 8f rank 2): server counting BF 1e9 u8 counters k=4; "
                                  f"{len(keys)} Insert batches of {B} (config-2 keys), pack, 1 Delete batch of {B}"},
           "correct": ok, "fpr_absent": round(fpr, 5),
           "insert_ms": round(ins_ms, 3), "pack_ms": round(pack_ms, 3), "delete_ms": round(del_ms, 3),
           "delete_mops": round(B / (del_ms / 1e3) / 1e6, 1),
           "roofline": {"bound": "hbm", "unit": "GB/s", "peak": 8000.0, "kernel": "k_cbf_insert",
                        "bytes_per_launch": int(bytes_ins), "avg_launch_us": round(ins_us, 2),
                        "achieved": round(bytes_ins / ins_us / 1e3, 1),
                        "frac": round(bytes_ins / ins_us / 1e3 / 8000.0, 4), "traffic": tr_ins,
                        "traffic_source": "profiles/r01/pmc_traffic_cbf.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes)",
                        "per_kernel": {"pack": {"kernel": "k_cbf_pack", "bytes_per_launch": int(pack_bytes),
                                                "avg_launch_us": round(pack_ms * 1e3, 1),
                                                "achieved": round(pack_bytes / (pack_ms * 1e3) / 1e3, 1),
                                                "frac": round(pack_bytes / (pack_ms * 1e3) / 1e3 / 8000.0, 4),
                                                "traffic": tr_pack}}}}
    if not a.no_cpu_baseline:
        from oracle import oracle as O  # the CPU baseline leg only (test infrastructure)
        n_cpu = 1 << 22
        o = O.OracleCBF(m, k)
        ck = keys[0][:n_cpu].cpu().numpy().view(np.uint64)
        t1 = time.perf_counter()
        o.insert(ck)
        cs = time.perf_counter() - t1
        res["cpu_baseline"] = {"value": round(n_cpu / cs / 1e6, 3), "unit": "Mops/s", "cores": 1,
                               "kind": "port", "sample": f"oracle CountingBloomFilter Insert, {n_cpu} keys, 1e9 counters, k=4"}
    print(json.dumps(res), flush=True)


def config7(a):
    """replay_KV (server/replay_KV.cpp:209-275) on the GPU.
    A synthetic 4M-line trace (32M page ops, 210 MB of text) resident in HBM;
    one step = parse it into the op/key stream (pmdfc_trace_parse) and replay
    all ops through mixed batches of 1M (W pages Insert, R pages Get; failed
    searches counted).  value = replayed ops/s including the parse."""
    from pmdfc_amd.workload import synth_trace
    dev = torch.device("cuda", 0)
    t0 = time.perf_counter()
    text = synth_trace(11, 4 << 20)
    gen_s = time.perf_counter() - t0
    d_text = torch.from_numpy(np.frombuffer(text, np.uint8).copy()).to(dev)
    rd = P.TraceReader(0)
    _, _, info = rd.parse(d_text, 0)
    n = info["trace_ops"]
    st = {}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    acc = [0.0, 0.0]

    def step(record=False):
        idx = st.get("idx")
        if idx is None:
            # replay_KV's default table size: 10 GiB * 10 / 4096 (replay_KV.cpp:182-185)
            idx = st["idx"] = P.CCEH(26214400, convention="src", max_batch=a.batch,
                                     max_segments=int(n / 400) + 65536, device=0)
        else:
            idx.reset()
        ev[0].record()
        ops, keys, _ = rd.parse(d_text, n)
        ev[1].record()
        st["r"] = P.replay(idx, ops, keys, a.batch)
        ev[2].record()
        if record:
            torch.cuda.synchronize()
            acc[0] += ev[0].elapsed_time(ev[1])
            acc[1] += ev[1].elapsed_time(ev[2])

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(a.steps):
        step(record=True)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t1) / a.steps
    parse_ms, replay_ms = acc[0] / a.steps, acc[1] / a.steps
    r = st["r"]
    res = {"metric": METRIC, "value": round(n / el / 1e6, 3), "unit": "Mops/s", "n_gpus": 1,
           "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(el * 1e3, 3), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "u8/u64", "data": "synthetic",
           "config": {"workload": f"config7 (SURVEY 8f rank 3): replay_KV trace of {info['lines']} lines "
                                  f"({len(text) / 1e6:.0f} MB text, {n} page ops) parsed on device and replayed "
                                  f"in mixed batches of {a.batch}, KV over src/cceh CCEH(26214400) (replay_KV's default)",
                      "init_cap": 26214400},
           "correct": r["put"] + r["get"] == n, "replay": r, "trace_gen_s": round(gen_s, 2),
           "parse_ms": round(parse_ms, 3), "parse_GBs_text": round(len(text) / (parse_ms * 1e6), 2),
           "replay_ms": round(replay_ms, 3), "replay_mops": round(n / (replay_ms * 1e3), 1)}
    if not a.no_cpu_baseline:
        from oracle import oracle as O  # CPU baseline leg only (test infrastructure)
        sample = text[: 1 << 22]
        sample = sample[: sample.rfind(b"\n") + 1]
        _, _, si = rd.parse(torch.from_numpy(np.frombuffer(sample, np.uint8).copy()).to(dev), 0)
        t2 = time.perf_counter()
        O.parse_replay_trace(sample, si["trace_ops"])
        cs = time.perf_counter() - t2
        res["cpu_baseline"] = {"value": round(len(sample) / cs / 1e6, 3), "unit": "MB/s text parsed",
                               "cores": 1, "kind": "port",
                               "sample": "oracle parse_replay_trace (pure Python) over a 4 MB prefix of the trace"}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
