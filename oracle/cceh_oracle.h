/*
 * cceh_oracle.h -- CPU restatement of the reference's serial CCEH_hybrid index,
 * its hash functions and the client bloom filter.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker for the HIP
 * engine in pmdfc_amd/.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.  The product path never links or calls it.
 *
 * Parity pin: the restatement is checked against golden vectors produced by the
 * reference's own CCEH_hybrid.cpp compiled from /root/reference (oracle/Makefile,
 * target `ref`, outputs in oracle/_ref/) and against the reference's own
 * known-answer test server/bftest.cpp (tests/test_oracle_golden.py).
 *
 * Every function cites the reference file:line it restates
 * (paths relative to the reference repository root).
 */
#ifndef PMDFC_CCEH_ORACLE_H_
#define PMDFC_CCEH_ORACLE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* server/util/pair.h:9-11 */
#define OC_INVALID   (~(uint64_t)0)
#define OC_SENTINEL  (~(uint64_t)0 - 1)

/* server/CCEH_hybrid.h:14-19, :28 */
#define OC_SLOTS_PER_SEGMENT 1024u
#define OC_PROBE_WINDOW      32u   /* kNumPairPerCacheLine * kNumCacheLine */
#define OC_MAX_DEPTH         30u   /* build contract: directory never exceeds 2^30 */

/* per-op codes and statuses; identical to include/pmdfc_cceh.h */
enum {
  OC_OP_GET = 0,
  OC_OP_INSERT = 1,
};
enum {
  OC_ST_MISS = 0,
  OC_ST_HIT = 1,
  OC_ST_INSERTED = 2,
  OC_ST_RESERVED_KEY = 3,
  OC_ST_UNSPLITTABLE = 4,
  OC_ST_DEPTH_LIMIT = 5,
  OC_ST_CAPACITY = 6,
  OC_ST_FILTERED = 7,
  OC_ST_UPDATED = 11,   /* upsert mode: the key's slot was overwritten */
};

/* ---- hashes ---------------------------------------------------------- */
/* h(key,8,0xc70697) = std::_Hash_bytes  (server/util/hash.h:7-10,252-254) */
uint64_t oc_hash64(uint64_t key);
/* murmur2(&key, 8, seed), 32-bit result (server/util/hash.h:42-91,
 * client/hash.h:48-97) */
uint32_t oc_murmur2(uint64_t key, uint32_t seed);
void oc_hash64_batch(const uint64_t* keys, uint64_t* out, size_t n);
void oc_murmur2_batch(const uint64_t* keys, uint32_t seed, uint32_t* out, size_t n);

/* ---- CCEH ------------------------------------------------------------ */
typedef struct oc_cceh oc_cceh;

typedef struct oc_stats {
  uint64_t splits;
  uint64_t doublings;
  uint64_t split_loss;      /* entries dropped by Insert4split */
  uint64_t gets;
  uint64_t get_hits;
  uint64_t get_lines;       /* 64-B lines read by gets (early exit) */
  uint64_t get_lines_full;  /* lines the reference's full 32-slot scan reads */
  uint64_t inserts;
  uint64_t insert_lines;    /* 64-B lines scanned to find the claimed slot */
  uint64_t early_exit_mismatch; /* gets where early exit != full scan (must be 0) */
} oc_stats;

/* CCEH_hybrid::CCEH(initCap): depth = floor(log2(initCap)) (CCEH_hybrid.cpp:79-85).
 * src/cceh.cpp:80-88 uses floor(log2(initCap/1024)); see oc_depth_for_*. */
oc_cceh* oc_create(uint32_t initial_depth, size_t reserve_segments);
/* CCEH::FindAnyway (CCEH_hybrid.cpp:482-496): directory order, then slot order */
int oc_find_anyway(const oc_cceh* t, uint64_t key, uint64_t* value);
void oc_find_anyway_batch(const oc_cceh* t, const uint64_t* keys, size_t n, uint64_t* out_values,
                          uint8_t* out_status);
void oc_destroy(oc_cceh* t);
/* last-writer-wins Insert: CCEH_hybrid.cpp:143-156 with the overwrite clause
 * of :153 enabled (see cceh_oracle.c) */
void oc_set_upsert(oc_cceh* t, int on);
uint32_t oc_depth_for_hybrid(uint64_t init_cap);
uint32_t oc_depth_for_src(uint64_t init_cap);

int oc_insert(oc_cceh* t, uint64_t key, uint64_t value);       /* returns OC_ST_* */
int oc_get(oc_cceh* t, uint64_t key, uint64_t* value);         /* returns OC_ST_* */
void oc_mixed(oc_cceh* t, const uint8_t* ops, const uint64_t* keys,
              const uint64_t* values, size_t n, uint64_t* out_values,
              uint8_t* out_status);
void oc_insert_batch(oc_cceh* t, const uint64_t* keys, const uint64_t* values,
                     size_t n, uint8_t* out_status);
void oc_get_batch(oc_cceh* t, const uint64_t* keys, size_t n,
                  uint64_t* out_values, uint8_t* out_status);

/* introspection */
uint32_t oc_depth(const oc_cceh* t);
uint32_t oc_num_segments(const oc_cceh* t);
void oc_get_stats(const oc_cceh* t, oc_stats* out);
double oc_utilization(const oc_cceh* t);   /* CCEH_hybrid.cpp:412-427 */
uint64_t oc_capacity(const oc_cceh* t);    /* CCEH_hybrid.cpp:429-435 */
/* Canonical dump: segments in directory order (each once, at the first
 * directory index that points to it).  keys/values are n_seg*1024 each;
 * values of empty slots are reported as 0.  dir_canon[x] = canonical index. */
void oc_dump(const oc_cceh* t, uint32_t* dir_canon, uint32_t* local_depth,
             uint64_t* prefix, uint64_t* keys, uint64_t* values);

/* ---- bloom filter (client/bloom_filter.c:61-117; MSB-first u64 words) --- */
void oc_bloom_add(uint64_t* bitmap, uint64_t nbits, uint32_t k, uint64_t key);
int oc_bloom_check(const uint64_t* bitmap, uint64_t nbits, uint32_t k, uint64_t key,
                   uint32_t* probes_out);
void oc_bloom_add_batch(uint64_t* bitmap, uint64_t nbits, uint32_t k,
                        const uint64_t* keys, size_t n);
void oc_bloom_check_batch(const uint64_t* bitmap, uint64_t nbits, uint32_t k,
                          const uint64_t* keys, size_t n, uint8_t* out,
                          uint64_t* total_probes);

/* ---- counting bloom filter (server/util/counting_bloom_filter.h) ------ */
void oc_cbf_insert(uint8_t* counters, uint64_t nbits, uint32_t k, uint64_t key);
int oc_cbf_query(const uint8_t* counters, uint64_t nbits, uint32_t k, uint64_t key);
int oc_cbf_delete(uint8_t* counters, uint64_t nbits, uint32_t k, uint64_t key);
void oc_cbf_to_bitmap(const uint8_t* counters, uint64_t nbits, uint64_t* bitmap);
void oc_cbf_insert_batch(uint8_t* counters, uint64_t nbits, uint32_t k, const uint64_t* keys,
                         uint64_t n);
void oc_cbf_delete_batch(uint8_t* counters, uint64_t nbits, uint32_t k, const uint64_t* keys,
                         uint64_t n, uint8_t* deleted);

/* ---- CPU baseline timing helpers (bench.py cpu_baseline leg) ---------- */
/* Inserts with the reference's clflush emulation when flush_ns > 0
 * (server/util/persist.h:31-41).  Returns elapsed seconds. */
double oc_time_insert(oc_cceh* t, const uint64_t* keys, size_t n, int flush_ns);
/* Gets from `threads` pthreads over contiguous chunks
 * (server/test_KV.cpp:225-258, without the sleep(1)).  Returns seconds;
 * *misses receives the number of keys whose value != key. */
double oc_time_get(oc_cceh* t, const uint64_t* keys, size_t n, int threads,
                   uint64_t* misses);

/* ---- concurrent restatement (cceh_mt.c): the CPU baseline ------------ */
/* CCEH_hybrid's segment/directory semaphores, CAS slot claim, non-INPLACE
 * split and directory doubling, called concurrently (CCEH_hybrid.h:40-140,
 * CCEH_hybrid.cpp:107-389).  flush_ns > 0 emulates clflush (persist.h:31-41). */
typedef struct oc_mt oc_mt;
oc_mt* oc_mt_create(uint32_t initial_depth, int flush_ns);
void oc_mt_destroy(oc_mt* t);
void oc_mt_insert(oc_mt* t, uint64_t key, uint64_t value);
uint64_t oc_mt_get(oc_mt* t, uint64_t key); /* NONE (0) on a miss */
uint32_t oc_mt_depth(const oc_mt* t);
uint64_t oc_mt_segments(const oc_mt* t);

typedef struct oc_mt_result {
  double insert_s, get_s;   /* wall time of each phase */
  uint64_t failed;          /* Gets whose value != key (test_KV's failedSearch) */
  uint32_t depth;
  uint64_t segments;
} oc_mt_result;
/* test_KV's harness (server/test_KV.cpp:204-308, no sleep(1)): a fresh
 * CCEH_hybrid at initial_depth, `threads` threads pinned to cpus[i] (NULL:
 * unpinned) over contiguous chunks, insert (value = key) then Get. */
int oc_mt_bench(uint32_t initial_depth, const uint64_t* keys, size_t n, int threads, const int* cpus,
                int flush_ns, oc_mt_result* out);

#ifdef __cplusplus
}
#endif
#endif
