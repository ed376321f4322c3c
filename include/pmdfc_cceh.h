/*
 * pmdfc_cceh.h -- C-ABI of the MI355X batched CCEH index engine.
 *
 * Drop-in boundary for the JULEE/PMDFC server's hash index.  The engine
 * replaces, batch-wise, the reference interfaces
 *   IHash   server/IHash.h:9-22     (Insert/Get/Utilization/Capacity/Recovery)
 *   ICCEH   server/ICCEH.h:9-27     (CCEH_hybrid's flavour)
 * as implemented by CCEH_hybrid (server/CCEH_hybrid.cpp:79-435) and its twin
 * src/cceh.cpp, and the client bloom probe
 *   bloom_filter_check / bloom_filter_add  client/bloom_filter.c:61-117.
 * Plain pointers and sizes only; no C++ or torch types cross this boundary.
 * The per-op C++ adapters (pmdfc_amd/host/gpu_cceh.h) batch over it.
 *
 * Semantics: a batch is applied as if its ops ran serially, in batch order,
 * on the reference CCEH_hybrid: identical Get results, identical final
 * segment images (canonical directory order) and directory depth.
 * Divergences by contract (DESIGN.md "Contract"): reserved keys rejected,
 * UNSPLITTABLE instead of the reference's endless split, depth capped at 30,
 * capacity bounded by the arena.
 *
 * Device-pointer entry points enqueue on `stream` (a hipStream_t; NULL =
 * the legacy default stream) and return as soon as the work is enqueued:
 * insert, get and mixed never synchronise (splits and directory growth run on
 * the device).  Outputs are valid once the stream reaches that point.
 */
#ifndef PMDFC_CCEH_H_
#define PMDFC_CCEH_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 7: round 4's interface.  8: the round-5 entry points (additive:
 * pmdfc_cceh_get_batches, pmdfc_cceh_mixed_batches, pmdfc_comm_create_host,
 * pmdfc_cceh_serve_start_n), PMDFC_ERR_SIZE, and pmdfc_kv_dump's sized form
 * (pmdfc_kv.h; its signature changed) */
#define PMDFC_ABI_VERSION 8

/* return codes of every entry point */
#define PMDFC_OK 0
#define PMDFC_ERR_ARG (-1)
#define PMDFC_ERR_NOMEM (-2)
#define PMDFC_ERR_HIP (-3)
#define PMDFC_ERR_STATE (-4)
#define PMDFC_ERR_SIZE (-5) /* an output buffer is smaller than the result */

/* per-op opcodes (d_ops) */
#define PMDFC_OP_GET 0
#define PMDFC_OP_INSERT 1

/* per-op status bytes (d_status) */
#define PMDFC_ST_MISS 0          /* Get: not found (reference returns NONE) */
#define PMDFC_ST_HIT 1           /* Get: found, value written */
#define PMDFC_ST_INSERTED 2      /* Insert: stored */
#define PMDFC_ST_RESERVED_KEY 3  /* key == INVALID (2^64-1) or SENTINEL (2^64-2) */
#define PMDFC_ST_UNSPLITTABLE 4  /* window holds 32 entries of this key's hash */
#define PMDFC_ST_DEPTH_LIMIT 5   /* a split would exceed global depth 30 */
#define PMDFC_ST_CAPACITY 6      /* segment arena exhausted */
#define PMDFC_ST_FILTERED 7      /* bloom-negative: miss without an index probe */
#define PMDFC_ST_WRONG_SHARD 8   /* key's hash prefix is owned by another shard */
#define PMDFC_ST_ROUTE_OVERFLOW 9 /* routed batch: the owner's carry was full (carry_cap ops waiting), op not applied */
#define PMDFC_ST_SPLIT_LOST 10    /* mixed batch: a Get whose key a split of the same batch dropped
                                     (CCEH_hybrid.cpp:24-27) and whose drop could not be placed in
                                     the batch order: only when more than 2^18 entries are dropped
                                     in one batch (the device drop log overflowed).  Otherwise the
                                     engine returns the reference's answer (value if the Get
                                     precedes the insert whose split dropped the key, else MISS).
                                     error_flags bit 16 is set when it occurs. */
#define PMDFC_ST_UPDATED 11       /* Insert in upsert mode (PMDFC_CFG_UPSERT): the key was already
                                     in its window; its value was overwritten in place */

/* pmdfc_cceh_config_t.flags */
#define PMDFC_CFG_UPSERT 1u       /* last-writer-wins Insert: the reference's Insert
                                     (CCEH_hybrid.cpp:149-156) with its commented-out overwrite
                                     clause (:153) enabled -- the first slot in probe order that
                                     is empty or holds the key takes the pair.  Default (0): the
                                     reference as shipped, duplicates take new slots. */

typedef struct pmdfc_cceh pmdfc_cceh_t;
typedef struct pmdfc_bloom pmdfc_bloom_t;
typedef struct pmdfc_cbf pmdfc_cbf_t;
typedef struct pmdfc_trace pmdfc_trace_t;

typedef struct pmdfc_cceh_config {
  uint32_t initial_depth;  /* global directory depth at creation (>= 1, >= shard_bits) */
  uint32_t shard_bits;     /* log2(number of shards); 0 = unsharded */
  uint32_t shard_id;       /* this shard's hash prefix (top shard_bits bits) */
  uint32_t max_batch;      /* largest n accepted by one batched call */
  uint64_t max_segments;   /* segment arena capacity (16 KiB each); 0 = auto */
  int32_t device;          /* HIP device ordinal */
  uint32_t flags;          /* PMDFC_CFG_* */
} pmdfc_cceh_config_t;

typedef struct pmdfc_cceh_stats {
  uint32_t depth;          /* reference-visible global depth = max(initial, max local depth) */
  uint32_t phys_depth;     /* directory depth actually allocated (>= depth) */
  uint64_t segments;       /* live segments in this shard */
  uint64_t capacity;       /* segments * 1024 (CCEH::Capacity, CCEH_hybrid.cpp:429) */
  uint64_t max_segments;
  uint64_t splits;
  uint64_t doublings;      /* sub-directory growths (the bucketed form of doubling) */
  uint64_t split_loss;     /* entries dropped by the split replay (Insert4split, :18-28) */
  uint64_t insert_passes;  /* sort/apply/split rounds, summed over bucket chunks */
  uint64_t batches;
  uint64_t segment_runs;   /* (segment, round) runs applied by insert/mixed */
  uint64_t deferred_ops;   /* ops that waited for a split of their segment */
  uint32_t bucket_bits;    /* p1: the directory is cut into 2^p1 buckets */
  uint32_t max_rounds;     /* most rounds one bucket chunk needed */
  uint64_t insert_lines;   /* sum over inserts of 64-B lines from y to the claimed slot */
  uint32_t error_flags;    /* sticky device errors: 1 pool exhausted, 2 round guard */
  uint32_t fast_declined;  /* buckets the lean first insert pass handed to the general one (saturates) */
} pmdfc_cceh_stats_t;

/* depth of CCEH_hybrid(initCap) (CCEH_hybrid.cpp:80) and of src/cceh.cpp's
 * CCEH(initCap) (src/cceh.cpp:82) */
uint32_t pmdfc_depth_for_hybrid(uint64_t init_cap);
uint32_t pmdfc_depth_for_src(uint64_t init_cap);

int pmdfc_abi_version(void);
const char* pmdfc_last_error(void);

/* ---- lifecycle ------------------------------------------------------ */
int pmdfc_cceh_create(const pmdfc_cceh_config_t* cfg, pmdfc_cceh_t** out);
int pmdfc_cceh_destroy(pmdfc_cceh_t* t);
/* back to the freshly created state (all keys dropped) */
int pmdfc_cceh_reset(pmdfc_cceh_t* t, void* stream);

/* ---- batched ops on device pointers --------------------------------- */
/* IHash::Insert x n (src/cceh.cpp:94, CCEH_hybrid.cpp:107).  A batch of at
 * most 256 ops is one launch (k_mixed_tiny / k_mixed_small), of at most 8192
 * two once the table is at its bucket resolution (k_part + k_medium), larger
 * ones the general pipeline.  The input and output pointers may be device
 * memory or pinned host memory mapped into the device (hipHostMalloc; the
 * small paths read and write it in place). */
int pmdfc_cceh_insert(pmdfc_cceh_t* t, const uint64_t* d_keys, const uint64_t* d_values,
                      uint8_t* d_status, uint64_t n, void* stream);
/* Consecutive Insert batches [bounds[i], bounds[i+1]) of the arrays, i <
 * nbatches (host array of nbatches + 1 offsets, each batch <= max_batch):
 * exactly pmdfc_cceh_insert on each batch in order, but batch i+1 is
 * partitioned on an internal stream while batch i is applied.  Never
 * synchronises; results are ordered on `stream` like pmdfc_cceh_insert. */
int pmdfc_cceh_insert_batches(pmdfc_cceh_t* t, const uint64_t* d_keys, const uint64_t* d_values,
                              uint8_t* d_status, const uint64_t* bounds, uint32_t nbatches,
                              void* stream);
/* IHash::Get x n (CCEH_hybrid.cpp:343).  Never synchronises. */
int pmdfc_cceh_get(pmdfc_cceh_t* t, const uint64_t* d_keys, uint64_t* d_values_out,
                   uint8_t* d_status, uint64_t n, void* stream);
/* Get batches [bounds[i], bounds[i+1]) (i < nbatches; keys, values and
 * statuses indexed from the array starts): the same results as one
 * pmdfc_cceh_get per batch, as ONE launch over their union (Get batches
 * change nothing, so no boundary is needed between them).  Never
 * synchronises. */
int pmdfc_cceh_get_batches(pmdfc_cceh_t* t, const uint64_t* d_keys, uint64_t* d_values_out,
                           uint8_t* d_status, const uint64_t* bounds, uint32_t nbatches, void* stream);
/* IHash/ICCEH::FindAnyway x n (CCEH_hybrid.cpp:482-496, twin src/cceh.cpp:
 * 457-471): the first pair holding the key in directory order, then SLOT order
 * 0..1023 -- not Get's probe order, so a key with several copies in a window
 * that wraps past slot 1023 can return another copy than Get.
 * Misses are PMDFC_ST_MISS with value 0 (reference: NONE).  Diagnostic: one
 * wave reads the whole 16 KiB segment per key.  Never synchronises. */
int pmdfc_cceh_find_anyway(pmdfc_cceh_t* t, const uint64_t* d_keys, uint64_t* d_values_out,
                           uint8_t* d_status, uint64_t n, void* stream);
/* Interleaved Insert/Get in batch order; a Get observes exactly the inserts
 * before it in the batch.  d_values_in is read for inserts, d_values_out is
 * written for gets (0 for inserts and misses).  Small and medium batches take
 * the one- and two-launch paths of pmdfc_cceh_insert and answer every Get in
 * batch order; larger ones answer some Gets early and place a split's drops
 * through a drop log (PMDFC_ST_SPLIT_LOST only if it overflows); pointers as
 * there. */
int pmdfc_cceh_mixed(pmdfc_cceh_t* t, const uint8_t* d_ops, const uint64_t* d_keys,
                     const uint64_t* d_values_in, uint64_t* d_values_out,
                     uint8_t* d_status, uint64_t n, void* stream);
/* Mixed batches [bounds[i], bounds[i+1]) in order (i < nbatches, each at
 * most max_batch ops): one pmdfc_cceh_mixed per batch (the routed loop's
 * one-rank call, MixedBatches).  Never synchronises. */
int pmdfc_cceh_mixed_batches(pmdfc_cceh_t* t, const uint8_t* d_ops, const uint64_t* d_keys,
                             const uint64_t* d_values_in, uint64_t* d_values_out, uint8_t* d_status,
                             const uint64_t* bounds, uint32_t nbatches, void* stream);

/* ---- serving (the per-op front-end, pmdfc_amd/host/batch_core.*) ------ */
/* Rings in coherent pinned host memory (hipHostMalloc with
 * hipHostMallocCoherent | hipHostMallocMapped), ring_size places each (a
 * power of two).  A caller publishes the op of place p (p = 0, 1, ...) in
 * req[p % ring_size] as two 16-B halves, lo = {key, seq} and hi = {value,
 * seq} with seq = PMDFC_SERVE_SEQ(p, op), each written with ONE aligned
 * 16-byte store (atomic on x86-64 CPUs with AVX).  The device reads both
 * halves of 64 places in one round trip and takes a place only when both
 * carry the expected word (so no ordering between the halves is needed).
 * The device answers in resp[p % ring_size] with one 16-B store: value,
 * status, seq = (uint32_t)(p + 1).  Place p may be rewritten (p +
 * ring_size) only after its response was read. */
#define PMDFC_SERVE_INSERT 1u     /* op bit 0: Insert (else Get) */
#define PMDFC_SERVE_CBF 2u        /* op bit 1: the Insert also counts in the attached counting BF */
#define PMDFC_SERVE_SEQ(p, op) ((uint32_t)((((uint64_t)(p) + 1u) << 2) | ((op) & 3u)))
typedef struct pmdfc_serve_req {
  uint64_t key;
  uint32_t seq, pad0;
  uint64_t value;
  uint32_t seq2, pad1;
} pmdfc_serve_req;
typedef struct pmdfc_serve_resp {
  uint64_t value;
  uint32_t status, seq;
} pmdfc_serve_resp;
typedef struct pmdfc_serve_ctl {
  uint32_t stop;             /* host: 1 = the wave exits at its next poll */
  uint32_t pad0[15];
  uint64_t heartbeat;        /* host: moved at least every ~100 ms while serving (else the wave exits after ~1 s) */
  uint64_t prof[6];          /* device: wall-clock ticks (100 MHz) this wave spent reading requests, counting
                                the BF, applying, answering; polls that found nothing; ticks since the wave
                                started (written every 256 chunks and at exit) */
  uint64_t reloads;          /* device: chunks after which the wave reloaded its LDS copy of the directory
                                bucket headers (the chunk's ordered path may have changed one) */
  uint64_t head;             /* device: places answered (the wave's next place) */
  uint64_t chunks;           /* device: chunks served by this wave */
  uint32_t alive;            /* host sets 1 before the launch, the wave clears it when it exits */
  uint32_t idle;             /* device: 1 after ~1 ms without ops (the host may stop it) */
  uint32_t pad2[10];
} pmdfc_serve_ctl;
/* Launch the serving wave on `stream` (it runs until ctl->stop): places from
 * head0 on, in ring order, at most 64 per chunk, each chunk applied as one
 * batch of pmdfc_cceh_mixed would be (the one-launch small-batch path:
 * exactly the serial reference).  cbf (nullable, same device): Inserts with
 * PMDFC_SERVE_CBF also increment it (CountingBloomFilter::Insert).  While the
 * wave runs, nothing else may use the index, and a device-wide
 * synchronisation waits for the wave: stop it first (ctl->stop, then wait for
 * ctl->alive == 0).  Host pointers; the engine maps them. */
int pmdfc_cceh_serve_start(pmdfc_cceh_t* t, pmdfc_serve_req* req, pmdfc_serve_resp* resp,
                           pmdfc_serve_ctl* ctl, uint64_t ring_size, uint64_t head0,
                           pmdfc_cbf_t* cbf, void* stream);

/* Several serving waves at once (one launch of nwaves workgroups): wave w
 * serves ring w -- places req[w * ring_size ...], resp[w * ring_size ...],
 * ctl[w] -- from ctl[w].head on.  Ring w must carry only ops whose directory
 * bucket has w in its top log2(nwaves) bits, i.e. whose hash h has
 * ((h << shard_bits) >> (64 - log2(nwaves))) == w: the waves then touch
 * disjoint segments, sub-directories and headers, and each ring's order is
 * the serial order of its keys (ops of different rings commute).  nwaves: a
 * power of two <= pmdfc_cceh_serve_waves_max(t) (the directory buckets at
 * the start, capped at 64).  Otherwise as pmdfc_cceh_serve_start; each wave
 * exits on its own ctl->stop. */
#define PMDFC_SERVE_WAVES_MAX 64
uint32_t pmdfc_cceh_serve_waves_max(pmdfc_cceh_t* t);
int pmdfc_cceh_serve_start_n(pmdfc_cceh_t* t, uint32_t nwaves, pmdfc_serve_req* req, pmdfc_serve_resp* resp,
                             pmdfc_serve_ctl* ctl, uint64_t ring_size, pmdfc_cbf_t* cbf, void* stream);

/* ---- host-pointer convenience (synchronous) -------------------------- */
int pmdfc_cceh_mixed_host(pmdfc_cceh_t* t, const uint8_t* ops, const uint64_t* keys,
                          const uint64_t* values_in, uint64_t* values_out,
                          uint8_t* status, uint64_t n);

/* ---- introspection (synchronous) ------------------------------------- */
int pmdfc_cceh_stats(pmdfc_cceh_t* t, pmdfc_cceh_stats_t* out);
/* CCEH::Utilization (CCEH_hybrid.cpp:412-427), percent */
int pmdfc_cceh_utilization(pmdfc_cceh_t* t, double* out);
/* Canonical dump to HOST buffers: segments in directory order, each once.
 * dir_canon: 2^(depth - shard_bits) entries of the logical directory;
 * local_depth/prefix: nseg entries (prefix = top local_depth bits of the hash);
 * keys/values: nseg*1024 (values 0 where key == INVALID).  Any pointer may be
 * NULL.  *nseg_out receives the segment count; call with keys == NULL first to
 * size the buffers. */
int pmdfc_cceh_dump(pmdfc_cceh_t* t, uint32_t* dir_canon, uint32_t* local_depth,
                    uint64_t* prefix, uint64_t* keys, uint64_t* values, uint64_t* nseg_out);

/* ---- kernel timing (HIP events on the launching stream) -------------- */
/* kernel classes */
#define PMDFC_K_GET 0
#define PMDFC_K_PREP 1
#define PMDFC_K_ROUTE 2
#define PMDFC_K_FINAL 3
#define PMDFC_K_PROCESS 4
#define PMDFC_K_SPLIT 5
#define PMDFC_K_PARKED 6
#define PMDFC_K_MIXED_GET 7
#define PMDFC_K_BLOOM 8
#define PMDFC_K_COUNT 9
/* flags: 1 = record HIP events around every launch, 2 = count the 64-B lines
 * read by pmdfc_cceh_get (k_get<true>, one partial sum per block) */
int pmdfc_cceh_timing_enable(pmdfc_cceh_t* t, int flags);
/* total milliseconds and launch counts per class since the last reset */
int pmdfc_cceh_timing_read(pmdfc_cceh_t* t, double* ms_out, uint64_t* launches_out, int reset);
/* lines of 64 B read by the Get probes of the last pmdfc_cceh_get call (only
 * counted while flag 2 is set) */
int pmdfc_cceh_last_get_lines(pmdfc_cceh_t* t, uint64_t* lines);

/* Measurement tool: wall-clock (100 MHz) phase stamps of the last insert/mixed
 * batch, 16 per k_bucket workgroup then 8 per k_part block; only when the engine
 * was created with PMDFC_STAMPS=1 in the environment.  *nbuckets = 2^p1. */
int pmdfc_cceh_debug_stamps(pmdfc_cceh_t* t, uint64_t* host_out, uint64_t n, uint32_t* nbuckets);

/* ---- utilities -------------------------------------------------------- */
/* h() = std::_Hash_bytes(&key, 8, 0xc70697) (server/util/hash.h:252) */
int pmdfc_hash64(const uint64_t* d_keys, uint64_t* d_out, uint64_t n, void* stream);
/* splitmix64 key stream, identical to pmdfc_amd.workload.uniform_keys */
int pmdfc_gen_keys(uint64_t seed, uint64_t start, uint64_t* d_out, uint64_t n, void* stream);
/* Stable partition of n keys by owner shard (top shard_bits of h()): writes the
 * permutation (batch indices grouped by owner, batch order kept inside a
 * group) and per-owner counts (2^shard_bits u64).  Synchronous. */
int pmdfc_route_by_shard(const uint64_t* d_keys, uint64_t n, uint32_t shard_bits,
                         uint32_t* d_perm, uint64_t* h_counts, int device, void* stream);

/* ---- multi-GPU routing without host sync ------------------
 * Replaces the per-op owner choice of NuMA_KV::Get(key, uid, node)
 * (server/NuMA_KV.cpp:136-151) for a batch sharded by hash prefix.  Each rank
 * packs its batch into 2^shard_bits owner blocks of `cap` records (owner =
 * top shard_bits of h(key); unused slots hold key INVALID, which an engine
 * answers RESERVED_KEY and never stores), exchanges the blocks with one
 * equal-split all-to-all, runs the engine on the 2^shard_bits * cap received
 * rows, returns responses with a second equal-split all-to-all and unpacks
 * them into call-global outputs.
 *
 * No op is dropped under skew: the ops past `cap` for one owner wait in that
 * owner's FIFO carry (device memory) and lead that owner's block in the next
 * pack, so every (rank, owner) stream of ops is applied in order, cap ops per
 * exchange.  A call ends with drain exchanges (packs of n = 0) until the
 * carried count of every rank is 0.  The applied order is exchange-major,
 * then source-rank-major (the all-to-all concatenates blocks by source), then
 * each rank's FIFO order.  Only an op that finds its owner's carry full
 * (carry_cap ops waiting) gets PMDFC_ST_ROUTE_OVERFLOW (sticky count:
 * pmdfc_router_overflow_count).
 * `width`: u64 words per record, 1 = key (Get), 2 = key, value (Insert),
 * 3 = key, value, op (mixed). */
/* The engine side of a routed exchange, straight on the received rows (no
 * unpacking pass): IHash::Insert (CCEH_hybrid.cpp:107-298) of n interleaved
 * {key, value} records, and IHash::Get (CCEH_hybrid.cpp:343-389) writing n
 * 16-B {value, status} response records. */
int pmdfc_cceh_insert_records(pmdfc_cceh_t* t, const uint64_t* d_records, uint8_t* d_status, uint64_t n,
                              void* stream);
int pmdfc_cceh_get_records(pmdfc_cceh_t* t, const uint64_t* d_keys, uint64_t* d_resp, uint64_t n,
                           void* stream);

typedef struct pmdfc_router pmdfc_router_t;
typedef struct {
  uint32_t shard_bits; /* 2^shard_bits owners, shard_bits <= 4 */
  uint32_t max_batch;  /* ops per pack */
  uint64_t cap;        /* rows per owner block */
  uint64_t carry_cap;  /* ops per owner the carry holds (0: max_batch) */
  int32_t device;
  uint32_t flags;      /* 0 */
} pmdfc_router_config;
int pmdfc_router_create(const pmdfc_router_config* cfg, pmdfc_router_t** out);
int pmdfc_router_destroy(pmdfc_router_t* r);
uint64_t pmdfc_router_rows(const pmdfc_router_t* r); /* 2^shard_bits * cap */
/* Pack n ops (output indices base .. base + n - 1 of the call) behind the
 * carried ones into d_send (rows * width u64) and d_rowpos (rows u32: the
 * call-global output index of each row, ~0 for padding).  Ops kept home
 * (d_keep[i] == 0; d_keep may be NULL) get status PMDFC_ST_FILTERED and
 * value 0 in the outputs right away, so do ops dropped on a full carry
 * (PMDFC_ST_ROUTE_OVERFLOW).  d_values_out may be NULL (Insert calls). */
int pmdfc_router_pack(pmdfc_router_t* r, const uint64_t* d_keys, const uint64_t* d_values, const uint8_t* d_ops,
                      const uint8_t* d_keep, uint64_t n, uint32_t width, uint32_t base, uint64_t* d_send,
                      uint32_t* d_rowpos, uint64_t* d_values_out, uint8_t* d_status_out, void* stream);
/* returned response rows (resp_width 0: u8 status rows; 1: 16-B {value,
 * status} rows) -> call-global outputs through the pack's d_rowpos */
int pmdfc_router_unpack(pmdfc_router_t* r, const void* d_back, uint32_t resp_width, const uint32_t* d_rowpos,
                        uint64_t* d_values_out, uint8_t* d_status_out, void* stream);
/* ops waiting in the carry after the last pack -> *d_out (device u64) */
int pmdfc_router_carried(pmdfc_router_t* r, uint64_t* d_out, void* stream);
/* the call's carry is drained: the next pack may use another width */
int pmdfc_router_end_call(pmdfc_router_t* r);
/* ops dropped on a full carry since create / reset (synchronises the stream) */
int pmdfc_router_overflow_count(pmdfc_router_t* r, uint64_t* h_out, void* stream);
/* drop the carry and the overflow count (an abandoned call) */
int pmdfc_router_reset(pmdfc_router_t* r, void* stream);
/* Get batches: one routed row per distinct key of each tile of 1024 Gets
 * (i / 1024).  For each Get i, the leader is the first Get of the same key in
 * its tile; d_keep_out[i] = 1 for leaders (and d_keep_in[i], if given),
 * d_lead_out[base + i] = base + leader.  Keys INVALID and kept-home Gets are
 * their own leaders.  (A hot key keeps one row per tile: n / 1024 rows.) */
int pmdfc_router_dedupe(pmdfc_router_t* r, const uint64_t* d_keys, const uint8_t* d_keep_in, uint64_t n,
                        uint32_t base, uint8_t* d_keep_out, uint32_t* d_lead_out, void* stream);
/* followers take their leader's value and status: out[i] = out[lead[i]] */
int pmdfc_router_fill(const uint32_t* d_lead, uint64_t n, uint64_t* d_values_out, uint8_t* d_status_out,
                      int device, void* stream);
/* received rows of `width` words -> engine arrays (d_values / d_ops by width) */
int pmdfc_route_split(const uint64_t* d_recv, uint64_t rows, uint32_t width, uint64_t* d_keys,
                      uint64_t* d_values, uint8_t* d_ops, int device, void* stream);
/* engine results -> 16-B response rows {value, status} */
int pmdfc_route_respond(const uint64_t* d_values, const uint8_t* d_status, uint64_t rows,
                        uint64_t* d_resp, int device, void* stream);

/* ---- native routed batches (RCCL from C++, no Python in the loop) -------
 * A communicator of its own over RCCL (xGMI between the GPUs of a node):
 * rank 0 makes the id, every rank passes the same bytes (the caller
 * broadcasts them, e.g. with torch.distributed). */
#define PMDFC_COMM_ID_BYTES 128
typedef struct pmdfc_comm pmdfc_comm_t;
int pmdfc_comm_id(uint8_t* id_out);  /* PMDFC_COMM_ID_BYTES bytes */
int pmdfc_comm_create(const uint8_t* id, int nranks, int rank, int device, pmdfc_comm_t** out);
/* A communicator whose exchanges go through the caller's own transport
 * instead of RCCL (tests on one GPU, where RCCL refuses two ranks on one
 * device; or any host-side fabric): the routed loop synchronises the
 * exchanges' stream, copies the nranks send blocks to pinned host memory and
 * calls xchg(ctx, send, recv, block_bytes) -- an all-to-all of equal blocks
 * (block p of send goes to rank p, block p of recv came from rank p; the
 * local block is ignored: it never moves) -- then copies the peer blocks back
 * to the device; amax(ctx, &v) replaces v by its maximum over the ranks (the
 * drain's carried count).  Both return 0 on success.  The protocol around
 * them (packs, carries, drains, unpacks) is the RCCL communicator's. */
typedef int (*pmdfc_host_exchange_fn)(void* ctx, const void* send, void* recv, uint64_t block_bytes);
typedef int (*pmdfc_host_allreduce_fn)(void* ctx, uint64_t* value);
int pmdfc_comm_create_host(int nranks, int rank, int device, pmdfc_host_exchange_fn xchg,
                           pmdfc_host_allreduce_fn amax, void* ctx, pmdfc_comm_t** out);
int pmdfc_comm_destroy(pmdfc_comm_t* c);
/* Route nb consecutive batches (ops bounds[i] .. bounds[i+1]-1 of d_keys /
 * d_values) to their owners and back, exactly as pmdfc_amd.dist.BlockRouter
 * does with the entry points above (same packs, same exchange order, same
 * carries and drains, so the same results): per batch pack -> all-to-all ->
 * the owner's engine straight on the received rows -> all-to-all back ->
 * unpack, with the exchange of batch i+1 and the return of batch i-1 on the
 * communicator's stream while batch i is applied.  width 2: Insert
 * (d_values_out unused); width 1: Get (dedupe != 0: one row per distinct key
 * of each 1,024-Get tile, pmdfc_router_dedupe / _fill).  Every rank calls
 * with the same nb; one host synchronisation per call (the drain's carried
 * counts).  Outputs are call-global (bounds[nb] ops). */
int pmdfc_route_batches(pmdfc_router_t* r, pmdfc_cceh_t* t, pmdfc_comm_t* c, uint32_t width,
                        const uint64_t* d_keys, const uint64_t* d_values, const uint64_t* bounds, uint64_t nb,
                        uint32_t dedupe, uint64_t* d_values_out, uint8_t* d_status_out, void* stream);
/* The same loop for mixed batches (d_ops: PMDFC_OP_* per op, rows of
 * {key, value, op}): the owner splits the received rows, applies them with
 * pmdfc_cceh_mixed and answers {value, status} rows, as BlockRouter.mixed
 * does (server/NuMA_KV.cpp:136-151 applies each request on its owner). */
int pmdfc_route_mixed_batches(pmdfc_router_t* r, pmdfc_cceh_t* t, pmdfc_comm_t* c, const uint8_t* d_ops,
                              const uint64_t* d_keys, const uint64_t* d_values, const uint64_t* bounds, uint64_t nb,
                              uint64_t* d_values_out, uint8_t* d_status_out, void* stream);

/* Measurement tool: n_ops random 64-B line gathers (k_get's access shape) from
 * d_buf (nlines lines); with d_table (tmask+1 u32 entries) each line index
 * first goes through one dependent table load, like the directory. */
int pmdfc_ubench_gather64(const void* d_buf, uint64_t nlines, const uint32_t* d_table,
                          uint32_t tmask, uint64_t n_ops, uint64_t seed, uint64_t* d_out,
                          void* stream);
/* Measurement tool, the bench's gather ceiling: n_ops random lines of
 * line_bytes (64 or 128) from d_buf (nbytes), line_bytes/16 lanes per line,
 * `depth` (1, 2 or 4) independent lines in flight per lane group, optionally
 * through the dependent table; one u64 per lane group into d_out[g & omask]
 * (omask + 1 entries, a power of two). */
int pmdfc_ubench_gather(const void* d_buf, uint64_t nbytes, uint32_t line_bytes, uint32_t depth,
                        const uint32_t* d_table, uint32_t tmask, uint64_t n_ops, uint64_t seed,
                        uint64_t* d_out, uint64_t omask, void* stream);
/* Measurement tool, the bench's scatter ceiling: n_ops random 16-B stores
 * (an insert's pair store) into d_buf (nbytes), one lane per store, `depth`
 * (1 or 4) stores issued back to back per lane. */
int pmdfc_ubench_scatter16(void* d_buf, uint64_t nbytes, uint32_t depth, uint64_t n_ops, uint64_t seed,
                           void* stream);

/* ---- bloom filter (client/bloom_filter.c, MSB-first u64 words) -------- */
int pmdfc_bloom_create(uint64_t nbits, uint32_t k, int device, pmdfc_bloom_t** out);
int pmdfc_bloom_destroy(pmdfc_bloom_t* b);
int pmdfc_bloom_clear(pmdfc_bloom_t* b, void* stream);
/* bloom_filter_add x n (client/bloom_filter.c:61-80) */
int pmdfc_bloom_add(pmdfc_bloom_t* b, const uint64_t* d_keys, uint64_t n, void* stream);
/* bloom_filter_check x n (client/bloom_filter.c:82-117): d_out[i] = 0/1 */
int pmdfc_bloom_probe(pmdfc_bloom_t* b, const uint64_t* d_keys, uint8_t* d_out, uint64_t n,
                      void* stream);
/* bitmap as the server ships it (rdma_svr.cpp:157-251): ceil(nbits/64) u64 */
int pmdfc_bloom_bitmap(pmdfc_bloom_t* b, uint64_t** d_bitmap, uint64_t* nwords);
/* bloom_filter_set (client/bloom_filter.c:119-124): load a bitmap shipped by
 * the server (host memory, ceil(nbits/64) u64); and the reverse copy */
int pmdfc_bloom_set_bitmap_host(pmdfc_bloom_t* b, const uint64_t* host_words, uint64_t nwords);
int pmdfc_bloom_get_bitmap_host(pmdfc_bloom_t* b, uint64_t* host_words, uint64_t nwords);
/* fused client path: bloom-negative keys get PMDFC_ST_FILTERED without an
 * index probe (client/rdpma.c:1050-1061), the rest an index Get */
int pmdfc_bloom_probe_then_get(pmdfc_bloom_t* b, pmdfc_cceh_t* t, const uint64_t* d_keys,
                               uint64_t* d_values_out, uint8_t* d_status, uint64_t n,
                               void* stream);

/* ---- server counting bloom filter (server/util/counting_bloom_filter.h) --
 * CountingBloomFilter<Key_t>(numHashes=k, numBits=nbits) (:60-65) as u8
 * device counters plus the packed MSB-first bitmap.  Batches equal the
 * reference applied key by key in batch order; KV::Insert (server/KV.cpp:
 * 113-121) calls pmdfc_cbf_insert after pmdfc_cceh_insert on the same stream.
 * 0 < nbits < 2^31 (ComputeHash's int index, :249-254), 0 < k <= 64. */
int pmdfc_cbf_create(uint64_t nbits, uint32_t k, int device, pmdfc_cbf_t** out);
int pmdfc_cbf_destroy(pmdfc_cbf_t* f);
int pmdfc_cbf_clear(pmdfc_cbf_t* f, void* stream);
/* Insert x n (:109-118): saturating += 1 at each of the k indices */
int pmdfc_cbf_insert(pmdfc_cbf_t* f, const uint64_t* d_keys, uint64_t n, void* stream);
/* the same for the Insert ops of a mixed batch (d_ops[i] == PMDFC_OP_INSERT):
 * KV::Insert's bf->Insert(key) after hash->Insert (server/KV.cpp:113-114) */
int pmdfc_cbf_insert_ops(pmdfc_cbf_t* f, const uint8_t* d_ops, const uint64_t* d_keys, uint64_t n,
                         void* stream);
/* Delete x n in batch order (:120-131): d_deleted[i] = Query(key_i) at its
 * turn; if so its k counters -= 1 (uint8 wrap, as the reference) */
int pmdfc_cbf_delete(pmdfc_cbf_t* f, const uint64_t* d_keys, uint8_t* d_deleted, uint64_t n,
                     void* stream);
/* Query x n (:133-143) on the counters */
int pmdfc_cbf_query(pmdfc_cbf_t* f, const uint64_t* d_keys, uint8_t* d_out, uint64_t n,
                    void* stream);
/* ToOrdinaryBloomFilter (:202-215): counters -> MSB-first bitmap */
int pmdfc_cbf_pack(pmdfc_cbf_t* f, void* stream);
/* QueryBitBloom x n (:145-158) on the last packed bitmap */
int pmdfc_cbf_query_bits(pmdfc_cbf_t* f, const uint64_t* d_keys, uint8_t* d_out, uint64_t n,
                         void* stream);
/* send_bf (rdma_svr.cpp:157-251) on one GPU: copy the packed bitmap into a
 * client filter of the same nbits (bloom_filter_set, client/bloom_filter.c:119-124) */
int pmdfc_cbf_export(pmdfc_cbf_t* f, pmdfc_bloom_t* b, void* stream);
/* device views and host copies (GetBaseAddr :74-76, GetBoolBitArray :93-95) */
int pmdfc_cbf_counters(pmdfc_cbf_t* f, uint8_t** d_counters, uint64_t** d_bitmap, uint64_t* nwords);
int pmdfc_cbf_get_counters_host(pmdfc_cbf_t* f, uint8_t* host, uint64_t nbits);
int pmdfc_cbf_get_bitmap_host(pmdfc_cbf_t* f, uint64_t* host, uint64_t nwords);

/* ---- extents ------------------------------------------
 * convention 0 = CCEH_hybrid: Insert_extent(key, value, len)
 *   (CCEH_hybrid.cpp:90-105), Get_extent(key) (:330-341, first nonzero Get of
 *   key - key % 2^h, h < 30);  convention 1 = src/cceh.cpp:
 *   Insert_extent(key, cluster, len, value) (:308-330), Get_extent(key,
 *   cluster) (:381-391).  d_clusters may be NULL (all 0; unused by hybrid).
 * insert_extent expands the batch on the device into its sub-extent heads and
 * inserts them in batch order (the reference's calls in order); it
 * synchronises once to size the expansion and returns it in *n_entries.
 * lens must be < 2^31 (the reference's int shifts overflow beyond). */
int pmdfc_cceh_insert_extent(pmdfc_cceh_t* t, int convention, const uint64_t* d_keys,
                             const uint64_t* d_clusters, const uint64_t* d_lens,
                             const uint64_t* d_values, uint64_t n, uint64_t* n_entries,
                             void* stream);
int pmdfc_cceh_get_extent(pmdfc_cceh_t* t, int convention, const uint64_t* d_keys,
                          const uint64_t* d_clusters, uint64_t* d_values_out, uint8_t* d_status,
                          uint64_t n, void* stream);

/* ---- replay_KV trace ingestion (server/replay_KV.cpp:209-247) -----------
 * A text trace (device bytes, lines "seq ts OP inode inode_size offset size")
 * becomes the first num_data ops of the reference's expansion, on the device:
 * d_ops[i] = PMDFC_OP_INSERT for 'W' pages, PMDFC_OP_GET for 'R' pages;
 * d_keys[i] = (inode << 32) + offset + 4096*b.  Synchronises (one host read
 * of the line count; info is host memory).  info[0] ops produced, [1] lines,
 * [2] ops in the whole trace, [3] the line at which the reference stops
 * reading, [4] first malformed line (~0 if none).  Returns PMDFC_ERR_ARG when
 * a malformed line precedes the stop line (the reference throws or reads out
 * of range) or the trace holds fewer than num_data ops (the reference replays
 * past its vectors). */
int pmdfc_trace_create(int device, pmdfc_trace_t** out);
int pmdfc_trace_destroy(pmdfc_trace_t* t);
int pmdfc_trace_parse(pmdfc_trace_t* t, const char* d_text, uint64_t nbytes, uint64_t num_data,
                      uint8_t* d_ops, uint64_t* d_keys, uint64_t* info, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* PMDFC_CCEH_H_ */
