"""bench.py -- batched CCEH lookup+insert throughput on MI355X (BASELINE.json).

Workload (BASELINE.json configs[1]), per GPU:
  64M unique uniform u64 keys (splitmix64 stream, value = key as in
  server/test_KV.cpp:206), CCEH_hybrid(65536) (initial depth 16),
  64 Insert batches of 1M keys, then 64 Get batches of 1M keys (100% hit).
One step = that whole job on a freshly reset index.  Keys are generated into
HBM before the timed region.

With --gpus N > 1 (under torchrun, or spawned by this script itself: one
process per GPU) the workload is the same config 2, weak-scaled: per GPU 64M
keys of its own stream; each rank owns the hash-prefix shard `rank` (top
log2 N bits of h(key)), and every batch is routed to the owners with RCCL
all-to-alls over xGMI (pmdfc_amd.dist.BlockRouter) and the results come back
the same way.  So the driver's 1 -> 8 curve compares one workload.  BASELINE
configs[3] (2^28 preloaded keys per GPU, mixed 50/50,
routed) is its own line: --config 4.

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
    ap.add_argument("--cpu-sample", type=int, default=1 << 23,
                    help="keys of the CPU baseline thread sweep (1/8 of config 2, same load trajectory)")
    ap.add_argument("--cpu-full", type=int, default=1 << 26,
                    help="keys of the CPU baseline's headline run at the best thread count (config 2: 2^26; 0 = skip)")
    ap.add_argument("--config", type=int, default=None, choices=[2, 3, 4, 5, 6, 7, 8],
                    help="default: 2 (the headline; at N > 1 weak-scaled and routed).  2: insert-then-get; 3: YCSB "
                         "95/5 Zipf over 256M replay-shape keys; 4: 50/50 mixed over 2^28 preloaded keys per "
                         "GPU (routed for N > 1); 5: bloom probe fused ahead of Get (1e9 bits, k=4); 6: server "
                         "counting-BF maintenance; 7: replay_KV trace ingestion + replay; 8: the per-op "
                         "batching front-end at 32 caller threads")
    ap.add_argument("--mixed-batches", type=int, default=16)
    ap.add_argument("--upsert", action="store_true",
                    help="config 2 in last-writer-wins mode (PMDFC_CFG_UPSERT)")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="config 2: time batch-by-batch inserts (the profiled form; kernels never overlap)")
    ap.add_argument("--serve-waves", type=int, default=8,
                    help="config 8: serving waves of the per-op front-end (rings by hash prefix)")
    ap.add_argument("--route", action="store_true",
                    help="one GPU: run the N>1 routed path anyway (pack, RCCL all-to-all over a "
                         "1-rank group, unpack) to measure its cost")
    return ap.parse_args()


def spawn_ranks(a) -> int:
    """`--gpus N` without a launcher: start N rank processes of this script,
    one per GPU (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 /
    MASTER_PORT set, as torchrun would), before this process touches the GPU.
    Returns the first nonzero exit status (the other ranks are then stopped)."""
    import socket
    import subprocess
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    procs = []
    for r in range(a.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.gpus),
                   LOCAL_WORLD_SIZE=str(a.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code and not rc:
                rc = code
                for q in live:  # a rank failed: the others would wait in a collective forever
                    q.terminate()
        time.sleep(0.05)
    return rc


_JSON_FD = None


def emit(res):
    """The ONE result line, on the real stdout (library banners -- RCCL's
    version lines at communicator creation -- went to stderr)."""
    line = (json.dumps(res) + "\n").encode()
    if _JSON_FD is None:
        sys.stdout.write(line.decode())
        sys.stdout.flush()
    else:
        os.write(_JSON_FD, line)


def main():
    global _JSON_FD
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(a))
    # everything but the result line goes to stderr (RCCL prints its version
    # banner to fd 1 when a communicator is created)
    sys.stdout.flush()
    _JSON_FD = os.dup(1)
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        log(f"note: --gpus {a.gpus} but WORLD_SIZE {world}; using WORLD_SIZE")
    if world & (world - 1):
        raise SystemExit("world size must be a power of two (hash-prefix shards)")
    cfg = a.config or 2
    if world > 1 and cfg not in (2, 4):
        raise SystemExit(f"--config {cfg} is a one-GPU line")
    return {2: config2, 3: config3, 4: config4, 5: config5, 6: config6, 7: config7, 8: config8}[cfg](a)


def _dist_setup(a):
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
    return world, rank, local, dev, routed


def config2(a):
    """BASELINE configs[1], the N = 1 headline."""
    world, rank, local, dev, routed = _dist_setup(a)
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
                 max_segments=max_segs, device=local, upsert=a.upsert)
    # routed: the whole call in C++ over an RCCL communicator of the engine's
    # own (pmdfc_route_batches; the exchange of batch i+1 overlaps batch i).
    # The config-2 stream holds no repeated key (splitmix64 of distinct
    # indices), so its Get batches skip the hot-key dedupe pass.
    comm = P.Comm(local) if routed else None
    router = BlockRouter(idx, packer, comm=comm, dedupe_gets=False) if routed else None

    # inputs resident in HBM before timing
    keys = [P.gen_keys(1000 + rank, i * B, B, device=local) for i in range(nb)]
    st_ins = [torch.empty(B, dtype=torch.uint8, device=dev) for _ in range(nb)]
    out_get = [None] * nb
    torch.cuda.synchronize()

    # one GPU: the 64 batches go through the multi-batch entry point
    # (pmdfc_cceh_insert_batches: same batches, same order, same results; the
    # next batch is partitioned while the current one is applied)
    allk = torch.cat(keys)
    bounds = [i * B for i in range(nb + 1)]
    pipelined = not a.no_pipeline

    def step(pipe=True):
        idx.reset()
        if routed:
            st_all = router.insert_concat(allk, allk, bounds)
            v_all, s_all = router.get_concat(allk, bounds)
            for i in range(nb):
                st_ins[i] = st_all[i * B:(i + 1) * B]
                out_get[i] = (v_all[i * B:(i + 1) * B], s_all[i * B:(i + 1) * B])
            return
        if pipe:
            st_all = idx.InsertBatches(allk, allk, bounds)
            for i in range(nb):
                st_ins[i] = st_all[i * B:(i + 1) * B]
            # the 64 Get batches through the multi-batch entry point
            # (pmdfc_cceh_get_batches: same batches, same results, one launch)
            v_all, s_all = idx.GetBatches(allk, bounds)
            for i in range(nb):
                out_get[i] = (v_all[i * B:(i + 1) * B], s_all[i * B:(i + 1) * B])
        else:
            for i in range(nb):
                st_ins[i] = idx.Insert(keys[i], keys[i])
            for i in range(nb):
                out_get[i] = idx.Get(keys[i])

    for _ in range(a.warmup):
        step(pipelined)
    # the timed steps run without HIP events: an event at every kernel-class
    # boundary (6 per insert batch) costs ~6 % of the step; the per-class
    # kernel times come from one more, identical step with events (below)
    idx.timing(events=False)
    if routed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step(pipelined)
    torch.cuda.synchronize()
    if routed:
        dist.barrier()
    t1 = time.perf_counter()
    idx.timing(events=True)
    idx.timing_read(reset=True)
    # the measured kernel durations (HIP events on the engine stream), batch by
    # batch so no class overlaps another (the pipelined steps overlap each
    # batch's k_part with the previous batch's apply chain)
    step(False)
    torch.cuda.synchronize()
    idx.timing(events=False)
    kt = idx.timing_read(reset=True)
    el = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    if routed:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())

    # correctness of the last step (outside the timed region)
    bad = 0
    for i in range(nb):
        bad += int((st_ins[i] != P.ST_INSERTED).sum())
        v, s = out_get[i]
        bad += int(((s != P.ST_HIT) | (v != keys[i])).sum())
    stats = idx.stats()

    # lines per Get on the final table (instrumented k_get, not timed)
    idx.timing(events=False, count_lines=True)
    lines_per_get = None
    if world == 1:
        idx.Get(keys[nb // 2])
        torch.cuda.synchronize()
        lines_per_get = idx.last_get_lines() / B
    idx.timing(events=False, count_lines=False)

    ops_total = 2 * NK * world * a.steps
    value = ops_total / elapsed / 1e6
    cls = {k: {"ms": v[0], "launches": v[1]} for k, v in kt.items() if v[1]}  # one step
    wl = ("config2: per GPU 64M unique uniform u64 keys (value=key), CCEH_hybrid(65536); "
          "64 Insert batches of 1M then 64 Get batches of 1M (100% hit); index reset each step")
    if a.upsert:
        wl += "; upsert (last-writer-wins) mode"
    if not pipelined and not routed:
        wl += "; batch-by-batch inserts (no partition overlap) and Gets"
    elif not routed:
        wl += ("; the insert batches through InsertBatches (batch i+1 partitioned while batch i is applied), "
               "the Get batches through GetBatches (one launch over the 64 batches; per-op results as batch by batch)")
    if routed:
        wl += (f"; {world} hash-prefix shards, every batch routed to its owners and back "
               f"(RCCL all-to-all from C++, pmdfc_route_batches), weak scaling")
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
            "workload": wl,
            "keys_per_gpu": NK, "batch": B, "init_cap": a.init_cap,
            "parallelism": f"hash-prefix shards x{world}" + (", RCCL all-to-all routing (fixed-capacity owner blocks)" if routed else ""),
        },
        "correct": bad == 0,
        "index": {"depth": stats["depth"], "segments": stats["segments"], "splits_per_step": stats["splits"],
                  "insert_passes_per_step": stats["insert_passes"] / max(1, stats["batches"]) if stats["batches"] else None,
                  "fast_declined_buckets": stats.get("fast_declined")},
        "kernel_ms_per_step": {k: round(v["ms"], 3) for k, v in cls.items()},
    }
    if rank == 0 and world == 1:
        ceil = gather_ceiling(dev)
        res["roofline"] = roofline(cls, lines_per_get, B, nb, NK, stats, a.steps, ceil,
                                   ms_per_step=round(elapsed / a.steps * 1e3, 3))
        res["get_mops"] = round(NK / (cls["get"]["ms"] / 1e3) / 1e6, 1) if "get" in cls else None
        if not a.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(a)
    if rank == 0:
        emit(res)
    if routed:
        dist.destroy_process_group()


def gather_ceiling(dev, n_ops=1 << 26, reps=3, batch=1 << 20, breps=16):
    """Measured random-access ceilings of this GPU, the denominators of the
    metric's "% HBM random-access roofline":
      * gathers in k_get's shape (a 4-lane group reads one random line, 16 B
        per lane) from a 4 GiB buffer (past the 256 MiB Infinity Cache),
        `depth` independent lines in flight per lane group (1, 2, 4), 64-B and
        128-B lines; plain and through a dependent 1 MiB u32 table (the
        directory);
      * scattered 16-B stores in an insert's pair-store shape (one lane, one
        random 16-B slot of the same buffer), 1 or 4 in flight per lane.
    Two regimes: n_ops (64M) per launch, and `batch` (1M, the engine's batch)
    per launch, `breps` launches back to back -- the regime the engine's
    kernels run in (a launch's stores land in the Infinity Cache and are
    written back under the next launches).  The model (_line_model) takes the
    batch-regime rates: gather_G_lines_s, scatter_G_stores_s."""
    import pmdfc_amd.engine as E
    buf = torch.empty(4 << 30, dtype=torch.uint8, device=dev)
    buf.random_(0, 255)
    table = torch.randint(0, (4 << 30) // 128 // 64, (1 << 18,), dtype=torch.int32, device=dev)
    out = torch.empty(1 << 20, dtype=torch.int64, device=dev)
    res = {}
    s = torch.cuda.current_stream(dev)

    def timed(fn, r_):
        fn(1)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for r in range(r_):
            fn(r + 2)
        e1.record(s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / r_

    for line in (64, 128):
        for depth in (1, 2, 4):
            for name, tb in (("plain", None), ("dep_table", table)):
                us = timed(lambda seed: E.ubench_gather(buf, n_ops, line, depth, tb, seed, out), reps)
                res[f"{name}_{line}B_x{depth}"] = {"us_per_launch": round(us, 1),
                                                    "line_GBs": round(n_ops * line / (us * 1e-6) / 1e9, 1),
                                                    "G_lines_s": round(n_ops / (us * 1e-6) / 1e9, 2)}
    for depth in (1, 2, 4):
        us = timed(lambda seed: E.ubench_gather(buf, batch, 64, depth, None, seed * 7919, out), breps)
        res[f"batch_plain_64B_x{depth}"] = {"us_per_launch": round(us, 2), "G_lines_s": round(batch / (us * 1e-6) / 1e9, 2)}
    for depth in (1, 4):
        us = timed(lambda seed: E.ubench_scatter16(buf, n_ops, depth, seed), reps)
        res[f"scatter_16B_x{depth}"] = {"us_per_launch": round(us, 1), "G_stores_s": round(n_ops / (us * 1e-6) / 1e9, 2)}
        us = timed(lambda seed: E.ubench_scatter16(buf, batch, depth, seed * 7919), breps)
        res[f"batch_scatter_16B_x{depth}"] = {"us_per_launch": round(us, 2),
                                              "G_stores_s": round(batch / (us * 1e-6) / 1e9, 2)}
    del buf
    best64 = max(v["line_GBs"] for k, v in res.items() if k.startswith("plain_64B"))
    res["best_plain_64B_GBs"] = best64
    res["gather_G_lines_s"] = max(v["G_lines_s"] for k, v in res.items() if k.startswith("batch_plain_64B"))
    res["scatter_G_stores_s"] = max(v["G_stores_s"] for k, v in res.items() if k.startswith("batch_scatter_16B"))
    res["sustained_gather_G_lines_s"] = max(v["G_lines_s"] for k, v in res.items() if k.startswith("plain_64B"))
    res["sustained_scatter_G_stores_s"] = max(v["G_stores_s"] for k, v in res.items() if k.startswith("scatter_16B"))
    res["n_ops"] = n_ops
    res["batch"] = batch
    return res


# the newest round's counter summary of this bench's own config-2 run
# (tools/run_profile.sh; the evidence script writes it before the bench lines)
PMC_FILE = next((f for f in (os.path.join(REPO, "profiles", r, "pmc_config2.json") for r in ("r06", "r05", "r04", "r03"))
                 if os.path.exists(f)), os.path.join(REPO, "profiles", "r03", "pmc_config2.json"))
CALIB_FILE = os.path.join(REPO, "profiles", "r03", "calibration", "calibration.json")
# FETCH_SIZE -> read bytes per kernel, by its dominant read shape, from the
# calibration run (tools/calib_fetch.py: kernels of known byte counts under
# the same two --pmc passes).  FETCH_SIZE counts 64 B per read REQUEST
# (MI355X_MICROARCH.md: TCC_EA0_RDREQ x 64 B): a random 64-B line gather is one
# request (x1.00), a random 128-B line or a stream of them two (x2.00).  So for
# k_get_u the figure is requests x 64 B, not DRAM bytes: the box moves random
# 64-B and 128-B lines at one line rate (random_gather_ceiling), so its
# roofline is the line rate (per_kernel line_rate_frac), not these bytes.
# WRITE_SIZE is exact for streaming stores.  k_apply reads its records as a
# stream and 128-B occupancy rows; k_part streams its input; k_split reads
# 16-KiB parents.
FETCH_SHAPE = {"k_get_u": ("random 64-B lines", 64), "k_apply": ("stream + random 128-B lines", 128),
               "k_apply_fast": ("stream + random 128-B lines", 128),
               "k_apply_fast_cp": ("stream + random 128-B lines", 128),
               "k_part": ("stream", 0), "k_split": ("stream (16-KiB parents)", 0)}


def _calib():
    """{64: factor of random 64-B lines, 128: ..., 0: streaming} from the
    committed calibration (None: the guide's blanket x2)."""
    try:
        with open(CALIB_FILE) as f:
            shapes = json.load(f)["shapes"]
    except (OSError, ValueError, KeyError):
        return None
    out = {}
    for p in shapes:
        fac = p.get("algorithmic_over_counted", {}).get("FETCH_SIZE")
        if fac is None:
            continue
        key = p.get("line", 0) if p["kernel"] == "k_gather" else 0
        out.setdefault(key, []).append(fac)
    return {k: sum(v) / len(v) for k, v in out.items()}


def _pmc_traffic():
    """HBM bytes per launch of each kernel from the committed rocprofv3 PMC
    passes over this bench's own config-2 workload (tools/pmc_summary.py:
    FETCH_SIZE and WRITE_SIZE in separate passes, KiB -> bytes), FETCH_SIZE
    scaled by the calibrated factor of the kernel's read shape (FETCH_SHAPE)."""
    if not os.path.exists(PMC_FILE):
        return {}
    with open(PMC_FILE) as f:
        pmc = json.load(f)
    cal = _calib()
    for k, r in pmc.items():
        if "FETCH_SIZE" not in r or "WRITE_SIZE" not in r:
            continue
        shape = FETCH_SHAPE.get(k)
        if cal and shape and shape[1] in cal:
            fac = cal[shape[1]]
            r["fetch_factor"] = round(fac, 4)
            r["fetch_factor_source"] = f"{os.path.relpath(CALIB_FILE, REPO)}: {shape[0]}"
            r["hbm_bytes_calibrated"] = int(r["FETCH_SIZE"] * 1024 * fac + r["WRITE_SIZE"] * 1024)
    return pmc


# Random-access model of each kernel class, per launch: the
# random lines it must load, the random 16-B pairs it must store, and its
# streamed bytes.  Its floor is loads / gather rate + stores / scatter rate +
# stream / 8 TB/s with the rates measured on this GPU (gather_ceiling), and
# line_rate_frac = floor / measured launch time: the metric's "% HBM
# random-access roofline implied by cachelines touched per op".
def _line_model(cname, B, lines_per_get, nb, stats):
    ins = B  # config 2: every insert batch is B fresh keys
    if cname == "get":
        return {"random_loads": lines_per_get * B, "random_stores": 0, "stream_bytes": 17 * B,
                "model": "per Get: the window's 64-B lines probed (instrumented k_get_u), key 8 B + value 8 B + status 1 B streamed"}
    if cname == "process":
        return {"random_loads": ins, "random_stores": ins, "stream_bytes": 20 * ins,
                "model": "per insert: its window's occupancy line (loaded; the claim's atomic OR hits the same line) and its 16-B pair "
                         "(stored at a random slot); its 20-B record streamed"}
    if cname == "route":
        return {"random_loads": 0, "random_stores": 0, "stream_bytes": 37 * B,
                "model": "per op: key + value in (16 B), record out (20 B), status (1 B)"}
    if cname == "split":
        sp = stats["splits"] / max(1, nb)
        return {"random_loads": 0, "random_stores": 0, "stream_bytes": 49152 * sp,
                "model": "per split: the 16-KiB parent read, two 16-KiB children written"}
    if cname == "parked":
        w = stats["deferred_ops"] / max(1, nb)
        return {"random_loads": w, "random_stores": w, "stream_bytes": 20 * w,
                "model": "per parked insert: as the first pass"}
    return None


def roofline(cls, lines_per_get, B, nb, NK, stats, steps, ceil, ms_per_step=None):
    """Roofline of the dominant kernel over the events step (HIP events on
    the engine stream, one launch per batch per class).  Algorithmic bytes
    (DESIGN.md §4):
      k_get          per Get: 8 key + 64*L + 8 value + 1 status, L = 64-B lines
                     probed, measured on the final table by the instrumented k_get;
      k_apply        (first apply pass) per insert: 16 (key, value) + 1 status +
                     64 (the line of the claimed slot), + 256 per segment run
                     (occupancy bitmap read + write);
      k_split        per split: 16 KiB parent read + 2 x 16 KiB children written;
      k_part         per op: 16 (key, value) in + 20 (record) out.
    The top-level achieved / peak / frac are bytes over the 8 TB/s spec (the
    bench contract); per_kernel.*.line_rate_frac and random_access_roofline
    carry the metric's random-access roofline (_line_model)."""
    pmc = _pmc_traffic()
    per = {}
    G = ceil["gather_G_lines_s"] * 1e9 if ceil else None
    Sc = ceil["scatter_G_stores_s"] * 1e9 if ceil else None

    def entry(cname, kernel, sym, b, extra=None):
        c = cls.get(cname)
        if not c:
            return
        avg = c["ms"] / c["launches"] / 1e3
        e = {"kernel": kernel, "bytes_per_launch": int(b), "avg_launch_us": round(avg * 1e6, 2),
             "achieved": round(b / avg / 1e9, 1), "frac": round(b / avg / 1e9 / HBM_PEAK_GBS, 4)}
        pm = None
        for sy in (sym if isinstance(sym, tuple) else (sym,)):
            pm = pm or pmc.get(sy) or pmc.get(sy.split("<")[0])  # summaries key by base name
        if pm and "hbm_bytes_upper" in pm:
            tr = pm.get("hbm_bytes_calibrated", pm["hbm_bytes_upper"])
            e["traffic"] = tr
            e["traffic_upper"] = pm["hbm_bytes_upper"]
            e["traffic_lower"] = pm["hbm_bytes_lower"]
            e["traffic_over_algorithmic"] = round(tr / max(1, b), 3)
            if "fetch_factor" in pm:
                e["fetch_factor"] = pm["fetch_factor"]
                e["fetch_factor_source"] = pm["fetch_factor_source"]
            e["pmc_dispatches"] = pm["dispatches"]
        m = _line_model(cname, B, lines_per_get or 0.0, nb, stats) if G else None
        if m:
            tmin = m["random_loads"] / G + m["random_stores"] / Sc + m["stream_bytes"] / (HBM_PEAK_GBS * 1e9)
            e.update({"random_loads_per_launch": int(m["random_loads"]), "random_stores_per_launch": int(m["random_stores"]),
                      "stream_bytes_per_launch": int(m["stream_bytes"]), "floor_us": round(tmin * 1e6, 2),
                      "line_rate_frac": round(tmin / avg, 4), "line_model": m["model"]})
        if extra:
            e.update(extra)
        per[cname] = e

    if lines_per_get is not None:
        entry("get", "k_get_u", "k_get_u<2, false>", B * (17 + 64 * lines_per_get),
              {"lines_per_get": round(lines_per_get, 4)})
    runs = stats["segment_runs"] / max(1, stats["batches"])  # per batch (the index is reset each step)
    # (the lean first pass: k_apply_fast_cp on the coarse partition at config
    # 2; the committed counters name the one that ran)
    fast = next((k for k in ("k_apply_fast_cp", "k_apply_fast") if k in pmc), "k_apply_fast")
    entry("process", fast, (fast, "k_apply<false>"), B * (16 + 1 + 64) + runs * 256,
          {"runs_per_batch": int(runs)})
    entry("route", "k_part", "k_part", B * (16 + 20))
    splits_per_batch = stats["splits"] / max(1, nb)
    entry("split", "k_split", "k_split", splits_per_batch * 49152,
          {"splits_per_batch": round(splits_per_batch, 1)})
    entry("parked", "k_apply_parked", "k_apply_parked<false>", (stats["deferred_ops"] / max(1, nb)) * 81)
    dom = max(cls, key=lambda k: cls[k]["ms"])
    pick = dict(per.get(dom) or per.get("get") or {})
    out = {"bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK_GBS, "traffic": pick.pop("traffic", None),
           "dominant_class": dom}
    out.update(pick)
    if out["traffic"] is not None:
        out["traffic_source"] = f"{os.path.relpath(PMC_FILE, REPO)} (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over this bench's config-2 run)"
    out["per_kernel"] = per
    out["random_gather_ceiling"] = ceil
    if "get" in per and ceil:
        out["get_vs_gather_ceiling"] = per["get"].get("line_rate_frac")
    if G:
        # the whole step: every class's floor over one step, against the
        # timed (pipelined) step and against the events step's kernel time
        floor_ms = sum(per[c]["floor_us"] * cls[c]["launches"] / 1e3 for c in per if "floor_us" in per[c])
        kern_ms = sum(v["ms"] for v in cls.values())
        out["random_access_roofline"] = {
            "floor_ms_per_step": round(floor_ms, 3),
            "step_ms": ms_per_step,
            "step_frac": round(floor_ms / ms_per_step, 4) if ms_per_step else None,
            "kernel_ms_per_step": round(kern_ms, 3),
            "kernel_frac": round(floor_ms / kern_ms, 4),
            "rates": {"gather_G_lines_s": ceil["gather_G_lines_s"], "scatter_G_stores_s": ceil["scatter_G_stores_s"],
                      "stream_GBs": HBM_PEAK_GBS},
            "note": "floor = random loads / measured gather rate + random 16-B stores / measured scatter rate + "
                    "streamed bytes / 8 TB/s, summed over the step's kernel classes (per_kernel.*.line_model)"}
    return out


def cpu_share():
    """CPUs this process may really use: its affinity set, capped by a cgroup
    CPU quota when there is one (a GPU box shows the whole machine's CPUs in
    the affinity set but grants one GPU's share of them)."""
    cpus = sorted(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except Exception:
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / per
        except Exception:
            pass
    n = len(cpus) if quota is None else max(1, min(len(cpus), int(math.ceil(quota))))
    return cpus[:n], len(cpus), quota


def cpu_baseline(a):
    """CPU baseline on this host's cores: the
    clean-room concurrent restatement of CCEH_hybrid (oracle/cceh_mt.c: the
    reference's segment/directory semaphores, CAS claim, split and doubling)
    under test_KV's harness (server/test_KV.cpp:225-258): T threads pinned one
    per core, contiguous chunks, Insert (value = key) then Get, no sleep(1).
    Bounded sample: the first --cpu-sample keys (8M, 1/8 of config 2) of the
    rank-0 stream into CCEH_hybrid(sample / 1024), the same load trajectory
    (segments split as often per key) as config 2's 64M keys into 65536.
    Sweep T = 1, 2, 4, ... up to the cores of this process, clflush emulation
    on (persist.h:31-41, as the reference times); flush-off at 1 thread and at
    the best T.  value = the best T's (inserts + gets) / time, flush on.
    Calibrated against the reference binary in the build container
    (profiles/r02/cpu_calibration.json)."""
    try:
        from oracle import oracle as O  # the CPU baseline leg only (test infrastructure)
        from pmdfc_amd.workload import uniform_keys
        n = a.cpu_sample
        keys = uniform_keys(1000, 0, n)
        depth = max(1, int(math.log2(max(2, n // 1024))))
        cpus, n_aff, quota = cpu_share()
        ts = sorted({t for t in (1, 2, 4, 8, 16, 32, 64, 128) if t <= len(cpus)} | {len(cpus)})
        sweep = {}
        for T in ts:
            r = O.mt_bench(depth, keys, T, cpus=cpus[:T], flush_ns=10)
            sweep[T] = {"insert_mops": round(n / r["insert_s"] / 1e6, 3), "get_mops": round(n / r["get_s"] / 1e6, 3),
                        "mops": round(2 * n / (r["insert_s"] + r["get_s"]) / 1e6, 3), "failedSearch": r["failed"]}
        best = max(sweep, key=lambda t: sweep[t]["mops"])
        off = {}
        for T in sorted({1, best}):
            r = O.mt_bench(depth, keys, T, cpus=cpus[:T], flush_ns=0)
            off[T] = {"insert_mops": round(n / r["insert_s"] / 1e6, 3), "get_mops": round(n / r["get_s"] / 1e6, 3),
                      "mops": round(2 * n / (r["insert_s"] + r["get_s"]) / 1e6, 3)}
        del keys
        # the headline workload itself at the best thread count: config 2's
        # 64M keys into CCEH_hybrid(65536), Insert then Get (value)
        nf = a.cpu_full
        full = None
        if nf:
            fk = uniform_keys(1000, 0, nf)
            r = O.mt_bench(16, fk, best, cpus=cpus[:best], flush_ns=10)
            full = {"keys": nf, "init_cap": 65536, "threads": best, "insert_mops": round(nf / r["insert_s"] / 1e6, 3),
                    "get_mops": round(nf / r["get_s"] / 1e6, 3),
                    "mops": round(2 * nf / (r["insert_s"] + r["get_s"]) / 1e6, 3), "failedSearch": r["failed"],
                    "seconds": round(r["insert_s"] + r["get_s"], 3)}
            del fk
        return {"value": full["mops"] if full else sweep[best]["mops"], "unit": "Mops/s", "cores": best,
                "kind": "port",
                "sample": (f"concurrent CCEH_hybrid restatement (oracle/cceh_mt.c, -O3) under test_KV's harness, "
                           f"threads pinned one per core, Insert (clflush emulation on) then Get: " +
                           (f"value = config 2's own workload, {nf} keys of the rank-0 stream into "
                            f"CCEH_hybrid(65536), at the best thread count ({best}) of a sweep over the first {n} "
                            f"keys into CCEH_hybrid({1 << depth}) (config 2's load trajectory at 1/8 scale) on the "
                            f"{len(cpus)} cores of this process's CPU share" if full else
                            f"first {n} keys into CCEH_hybrid({1 << depth}) (1/8 of config 2), best of a thread sweep "
                            f"over the {len(cpus)} cores of this process's CPU share")),
                "full_workload": full,
                "flush": "on", "sweep_flush_on": sweep, "flush_off": off,
                "cores_available": len(cpus), "affinity_cpus": n_aff, "cgroup_cpu_quota": quota,
                "calibration": "profiles/r02/cpu_calibration.json (port vs the reference binary, build container)"}
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
    passes = a.warmup + a.steps + 1  # + one pass with HIP events (kernel classes)
    ops_l, keys_l = [], []
    fresh = 0
    for _ in range(passes * nbt):  # every pass inserts keys no earlier pass did
        is_ins = rng.random(B) < 0.05
        r = scramble(zipf_ranks(rng, n_pre, 0.99, B), n_pre, 33)
        nf = int(is_ins.sum())
        r[is_ins] = n_pre + fresh + np.arange(nf)
        fresh += nf
        rk = replay_key(torch.from_numpy(r).to(dev))
        ops_l.append(torch.from_numpy(is_ins.astype(np.uint8)).to(dev))
        keys_l.append(rk)
    outs = [None] * nbt
    cur = [0]

    def step():
        p0 = cur[0] * nbt
        for i in range(nbt):
            outs[i] = idx.Mixed(ops_l[p0 + i], keys_l[p0 + i], keys_l[p0 + i])
        cur[0] += 1

    idx.timing(events=False)
    el = _time_steps(step, a.steps, a.warmup) / a.steps
    bad = 0
    p_last = (cur[0] - 1) * nbt
    for i in range(nbt):
        v, s = outs[i]
        o, k = ops_l[p_last + i], keys_l[p_last + i]
        g = o == 0
        bad += int(((s[g] != P.ST_HIT) | (v[g] != k[g])).sum())
        bad += int((s[~g] != P.ST_INSERTED).sum())
    idx.timing(events=True)
    idx.timing_read(reset=True)
    step()
    torch.cuda.synchronize()
    kt = idx.timing_read(reset=True)
    idx.timing(events=False)
    stats = idx.stats()
    res = {"metric": METRIC, "value": round(nbt * B / el / 1e6, 3), "unit": "Mops/s", "n_gpus": 1,
           "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(el * 1e3, 3), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "u64", "data": "synthetic",
           "config": {"workload": f"config3: 2^28 replay-shape keys preloaded, {nbt} mixed batches of {B} per step: "
                                  "95% Zipf(0.99) Get / 5% fresh Insert (every step inserts new keys)",
                      "init_cap": a.init_cap},
           "correct": bad == 0, "preload_s": round(preload_s, 3),
           "preload_insert_mops": round(n_pre / preload_s / 1e6, 1),
           "index": {"depth": stats["depth"], "segments": stats["segments"]},
           "kernel_ms_events_pass": {k: round(v[0], 3) for k, v in kt.items() if v[1]}}
    emit(res)


def config4(a):
    """SURVEY §8d config 4 (BASELINE configs[3]), per GPU: 2^28 uniform keys
    preloaded (2^31 over 8 GPUs), then mixed batches of 1M, 50% Get of
    preloaded keys (uniform) / 50% Insert of fresh keys.  N > 1 (the default
    workload there): each rank owns the hash-prefix shard `rank` and feeds its
    own stream; every batch is routed to the owners (BlockRouter, RCCL
    all-to-all over xGMI) and answered the same way -- weak scaling.  N = 1:
    the engine directly (--route: through the routed path on a 1-rank group).
    One step = --mixed-batches batches."""
    world, rank, local, dev, routed = _dist_setup(a)
    sbits = int(math.log2(world))
    B, n_pre, nbt = a.batch, 1 << 28, a.mixed_batches
    depth = P.depth_for_hybrid(a.init_cap)
    packer = P.BlockPacker(local, B, sbits) if routed else None
    idx = P.CCEH(depth=depth, shard_bits=sbits, shard_id=rank, max_batch=packer.rows if routed else B,
                 max_segments=int((n_pre + (a.warmup + a.steps) * nbt * B // 2) / 480) + 65536, device=local)
    # routed: the whole call in C++ over the engine's own RCCL communicator
    # (pmdfc_route_mixed_batches: split, pmdfc_cceh_mixed and respond on the
    # owner, the exchanges of neighbouring batches overlapped)
    comm = P.Comm(local) if routed else None
    router = BlockRouter(idx, packer, comm=comm) if routed else None
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
    total = a.warmup + a.steps + 1  # (+1: the HIP-events pass after the timed steps)
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
    # routed: each step's batches as one array per input and batch bounds
    # (resident before the timed region, like the direct batches)
    bounds = [j * B for j in range(nbt + 1)]
    cat = []
    if routed:
        for s_ in range(total):
            bs = batches[s_ * nbt:(s_ + 1) * nbt]
            cat.append((torch.cat([b[2] for b in bs]), torch.cat([b[0] for b in bs])))

    def run(si):
        if routed:
            o, k = cat[si]
            v, st = router.mixed_concat(o, k, k, bounds)
            return [(v[bounds[j]:bounds[j + 1]], st[bounds[j]:bounds[j + 1]]) for j in range(nbt)]
        return [idx.Mixed(o, k, v) for k, v, o in batches[si * nbt:(si + 1) * nbt]]

    for w in range(a.warmup):
        run(w)
    torch.cuda.synchronize()
    if routed:
        dist.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for s_ in range(a.steps):
        outs = run(a.warmup + s_)
    torch.cuda.synchronize()
    if routed:
        dist.barrier()
    el = time.perf_counter() - t1
    if routed:
        tt = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt)
    last = batches[(a.warmup + a.steps - 1) * nbt:(a.warmup + a.steps) * nbt]
    bad = 0
    overflow = 0
    for (k, _, o), (v, st) in zip(last, outs):
        g = o == 0
        bad += int(((st[g] != P.ST_HIT) | (v[g] != k[g])).sum()) + int((st[~g] != P.ST_INSERTED).sum())
        overflow += int((st == P.ST_ROUTE_OVERFLOW).sum())
    if routed:
        bt = torch.tensor([bad, overflow], device=dev)
        dist.all_reduce(bt)
        bad, overflow = int(bt[0]), int(bt[1])
    n = world * a.steps * nbt * B
    # one more step with HIP events on the engine's passes (untimed): where a
    # mixed batch's time goes; routed: the rest of the step is routing
    idx.timing(events=True)
    idx.timing_read(reset=True)
    torch.cuda.synchronize()
    te = time.perf_counter()
    run(a.warmup + a.steps)
    torch.cuda.synchronize()
    ev_step_ms = (time.perf_counter() - te) * 1e3
    kt = idx.timing_read(reset=True)
    idx.timing(events=False)
    stats = idx.stats()
    segs = torch.tensor([stats["segments"]], dtype=torch.int64, device=dev)
    if routed:
        dist.all_reduce(segs)
    if rank == 0:
        res = {"metric": METRIC, "value": round(n / el / 1e6, 3), "unit": "Mops/s", "n_gpus": world,
               "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(el / a.steps * 1e3, 3),
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64",
               "data": "synthetic",
               "config": {"workload": f"config4: per GPU 2^28 preloaded uniform keys ({world << 28} over {world}), "
                                      f"{nbt} mixed batches of {B} per GPU per step, 50% Get (preloaded, uniform) "
                                      "/ 50% fresh Insert",
                          "keys_per_gpu": n_pre, "batch": B, "init_cap": a.init_cap,
                          "parallelism": f"hash-prefix shards x{world}" + (
                              ", RCCL all-to-all routing from C++ (pmdfc_route_mixed_batches)" if routed else "")},
               "correct": bad == 0, "route_overflow_ops": overflow, "preload_s": round(preload_s, 2),
               "index": {"depth": stats["depth"], "segments_all_shards": int(segs.item())},
               "kernel_ms_events_pass": {k: round(v[0], 3) for k, v in kt.items() if v[1]},
               "events_pass_wall_ms": round(ev_step_ms, 3)}
        emit(res)
    if routed:
        dist.destroy_process_group()


def config8(a):
    """the per-op batching front-end (pmdfc_amd/host,
    GpuCCEH : IHash) at the server's concurrency, 32 caller threads
    (NUM_CLIENT x NUM_QUEUES, server/rdma_svr.h:17-18), each pinned to a core:
    per-op Insert, per-op Get, then 50/50 per-op mixed (tools/bench_frontend.cpp).
    value = the mixed phase's per-op calls/s.  The CPU baseline is the
    concurrent CCEH_hybrid restatement called per op by as many threads (the
    reference's own concurrency, which needs no batching)."""
    import subprocess
    threads, per = 32, 1 << 16
    exe = os.path.join(REPO, "pmdfc_amd", "lib", "bench_frontend")
    wv = str(a.serve_waves)
    runs = []
    for _ in range(max(1, a.steps)):
        r = subprocess.run([exe, str(threads), str(per), "256", "65536", "10", wv], capture_output=True, text=True,
                           timeout=600, check=True)
        runs.append(json.loads(r.stdout.strip().splitlines()[-1]))
    best = max(runs, key=lambda x: x["mixed_mops"])
    # the same at 16 callers: the GPU box gives this process a 16-CPU share,
    # so 32 busy callers (and the index's control thread) contend for it
    r16 = subprocess.run([exe, "16", str(per), "256", "65536", "10", wv], capture_output=True, text=True, timeout=600,
                         check=True)
    res16 = json.loads(r16.stdout.strip().splitlines()[-1])
    # one serving wave (one ring), for comparison
    r1 = subprocess.run([exe, str(threads), str(per), "256", "65536", "10", "1"], capture_output=True, text=True,
                        timeout=600, check=True)
    res1 = json.loads(r1.stdout.strip().splitlines()[-1])
    res = {"metric": METRIC, "value": best["mixed_mops"], "unit": "Mops/s", "n_gpus": 1, "steps": len(runs),
           "warmup": 0, "ms_per_step": round(threads * per / best["mixed_mops"] / 1e3, 3),
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64", "data": "synthetic",
           "config": {"workload": f"config8 (SURVEY 8f rank 1): {threads} caller threads x {per} per-op calls "
                                  "through GpuCCEH (IHash) into test_KV's CCEH(26214400): Insert phase, Get phase, "
                                  f"50/50 mixed phase, {a.serve_waves} serving waves (rings by hash prefix); "
                                  "value = mixed calls/s"},
           "correct": best["failedSearch"] == 0 and best["failed_ops"] == 0 and res16["failed_ops"] == 0,
           "serve_waves": best.get("serve_waves"), "frontend": best, "runs": runs, "frontend_16_callers": res16,
           "frontend_one_wave": res1}
    if not a.no_cpu_baseline:
        from oracle import oracle as O  # CPU baseline leg only (test infrastructure)
        from pmdfc_amd.workload import uniform_keys
        cpus, _, _ = cpu_share()
        T = min(threads, len(cpus))
        n = threads * per
        r = O.mt_bench(14, uniform_keys(55, 0, n), T, cpus=cpus[:T], flush_ns=10)
        res["cpu_baseline"] = {"value": round(2 * n / (r["insert_s"] + r["get_s"]) / 1e6, 3), "unit": "Mops/s",
                               "cores": T, "kind": "port",
                               "sample": f"concurrent CCEH_hybrid restatement (oracle/cceh_mt.c), {T} pinned threads, "
                                         f"{n} per-op Inserts (clflush emulation on) then Gets into CCEH(depth 14)",
                               "insert_mops": round(n / r["insert_s"] / 1e6, 3),
                               "get_mops": round(n / r["get_s"] / 1e6, 3)}
    emit(res)


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
    emit(res)


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
    emit(res)


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
    emit(res)


if __name__ == "__main__":
    main()
