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
from pmdfc_amd.dist import ShardRouter  # noqa: E402

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
    ap.add_argument("--cpu-sample", type=int, default=1 << 23)
    return ap.parse_args()


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        log(f"note: --gpus {a.gpus} but WORLD_SIZE {world}; using WORLD_SIZE")
    if world & (world - 1):
        raise SystemExit("world size must be a power of two (hash-prefix shards)")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    sbits = int(math.log2(world))
    B, NK = a.batch, a.keys
    nb = NK // B
    depth = P.depth_for_hybrid(a.init_cap)
    max_segs = int(NK / 512 * 1.25) + (1 << (depth - sbits)) + 1024
    max_batch = B if world == 1 else B + B // 4 + 65536
    idx = P.CCEH(depth=depth, shard_bits=sbits, shard_id=rank, max_batch=max_batch,
                 max_segments=max_segs, device=local)
    router = ShardRouter(idx, sbits, lambda k: P.route_by_shard(k, sbits))

    # inputs resident in HBM before timing
    keys = [P.gen_keys(1000 + rank, i * B, B, device=local) for i in range(nb)]
    st_ins = [torch.empty(B, dtype=torch.uint8, device=dev) for _ in range(nb)]
    out_get = [None] * nb
    torch.cuda.synchronize()

    def step():
        idx.reset()
        for i in range(nb):
            st_ins[i] = router.insert(keys[i], keys[i])
        for i in range(nb):
            out_get[i] = router.get(keys[i])

    for _ in range(a.warmup):
        step()
    idx.timing(events=True)
    idx.timing_read(reset=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    idx.timing(events=False)
    kt = idx.timing_read(reset=True)
    el = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    if world > 1:
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
    cls = {k: {"ms": v[0] / a.steps, "launches": v[1] / a.steps} for k, v in kt.items() if v[1]}
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
            "parallelism": f"hash-prefix shards x{world}" + (", RCCL all-to-all routing" if world > 1 else ""),
        },
        "correct": bad == 0,
        "index": {"depth": stats["depth"], "segments": stats["segments"], "splits_per_step": stats["splits"],
                  "insert_passes_per_step": stats["insert_passes"] / max(1, stats["batches"]) if stats["batches"] else None},
        "kernel_ms_per_step": {k: round(v["ms"], 3) for k, v in cls.items()},
    }
    if rank == 0 and world == 1:
        res["roofline"] = roofline(cls, lines_per_get, B, nb, NK, stats)
        res["get_mops"] = round(NK / (cls["get"]["ms"] / 1e3) / 1e6, 1) if "get" in cls else None
        if not a.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(a, depth)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


def roofline(cls, lines_per_get, B, nb, NK, stats):
    """Roofline of the dominant kernel class over the timed region.
    k_get: algorithmic bytes per Get = 8 (key) + 64*L (window lines up to the
    match / first empty slot) + 8 (value) + 1 (status), L measured by the
    instrumented k_get on the final table."""
    dom = max(cls, key=lambda k: cls[k]["ms"])
    out = {"bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK_GBS, "kernel": dom, "traffic": None}
    if dom == "get" or True:
        g = cls.get("get")
        if g and lines_per_get is not None:
            per_launch_bytes = B * (17 + 64 * lines_per_get)
            avg_s = g["ms"] / g["launches"] / 1e3
            ach = per_launch_bytes / avg_s / 1e9
            out.update({"kernel": "k_get", "achieved": round(ach, 1), "frac": round(ach / HBM_PEAK_GBS, 4),
                        "bytes_per_launch": int(per_launch_bytes), "avg_launch_us": round(avg_s * 1e6, 2),
                        "lines_per_get": round(lines_per_get, 4), "dominant_class": dom})
    return out


def cpu_baseline(a, depth):
    """Oracle (clean-room port of serial CCEH_hybrid) on this host: a bounded
    sample of the same workload, 1 thread, reference clflush emulation on."""
    try:
        from oracle import oracle as O
        from pmdfc_amd.workload import uniform_keys
        n = a.cpu_sample
        k = uniform_keys(1000, 0, n)
        o = O.OracleCCEH(depth, reserve_segments=int(n / 400) + (1 << depth))
        t_ins = o.time_insert(k, flush_ns=10)
        t_get, miss = o.time_get(k, threads=1)
        o2 = O.OracleCCEH(depth, reserve_segments=int(n / 400) + (1 << depth))
        t_ins_nf = o2.time_insert(k, flush_ns=0)
        return {"value": round(2 * n / (t_ins + t_get) / 1e6, 3), "unit": "Mops/s", "cores": 1,
                "kind": "port",
                "sample": f"first {n} keys of the rank-0 stream: insert (clflush emulation 10 ns/line, "
                          f"server/util/persist.h:31-41) then Get, 1 thread; misses={miss}",
                "insert_mops": round(n / t_ins / 1e6, 3), "get_mops": round(n / t_get / 1e6, 3),
                "insert_mops_flush_off": round(n / t_ins_nf / 1e6, 3)}
    except Exception as e:  # never let the CPU leg break the GPU line
        return {"value": None, "unit": "Mops/s", "cores": 1, "kind": "port", "sample": f"failed: {e}"}


if __name__ == "__main__":
    main()
