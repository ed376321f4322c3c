"""pmdfc_amd -- MI355X-native batched CCEH index engine for the JULEE/PMDFC
server path.  The compute lives in lib/libpmdfc_cceh.so
(hand-written gfx950 HIP kernels behind the C-ABI in include/pmdfc_cceh.h)."""
from .engine import (CCEH, Comm, BloomFilter, CountingBloomFilter, TraceReader, replay, BlockPacker, route_capacity, PmdfcError, depth_for_hybrid, depth_for_src, gen_keys,  # noqa: F401
                     hash64, load_library, route_by_shard, OP_GET, OP_INSERT, ST_MISS, ST_HIT,
                     ST_INSERTED, ST_RESERVED_KEY, ST_UNSPLITTABLE, ST_DEPTH_LIMIT, ST_CAPACITY,
                     ST_FILTERED, ST_WRONG_SHARD, ST_ROUTE_OVERFLOW, ST_SPLIT_LOST, ST_UPDATED, CFG_UPSERT)
from .kv import KV  # noqa: F401,E402
