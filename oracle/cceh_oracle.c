/*
 * cceh_oracle.c -- CPU restatement of the reference's serial CCEH_hybrid.
 *
 * TEST INFRASTRUCTURE ONLY (see cceh_oracle.h).  Never linked by the product.
 *
 * Semantics restated (paths relative to the reference root):
 *   hash     server/util/hash.h:7-10,252-254 -> libstdc++ std::_Hash_bytes,
 *            MurmurHash64A-style, len 8, seed 0xc70697 (third-party: libstdc++
 *            hash_bytes.cc, GCC 11; pinned by KATs in tests/golden).
 *   murmur2  server/util/hash.h:42-91 == client/hash.h:48-97.
 *   Insert   server/CCEH_hybrid.cpp:107-298 (serial path; the stale-pattern
 *            clause of :149-156 never fires in the non-INPLACE build, so the
 *            claim is the first INVALID slot of the 32-slot window).
 *   Split    server/CCEH_hybrid.cpp:18-28,47-66 (non-INPLACE; slot-order
 *            replay, silent drop when the child window is full).
 *   Dir      server/CCEH_hybrid.cpp:197-295 (doubling / stride update).
 *   Get      server/CCEH_hybrid.cpp:343-389 (first key match in probe order).
 *   Upsert   (opt-in, oc_set_upsert) the Insert of :143-156 with the
 *            commented-out overwrite clause of :153 enabled.  As written
 *            there the clause compares the slot's key with itself (`_key` is
 *            the slot's key, :141) and would claim every first slot; the
 *            evident intent, restated here, is `target->_[loc].key == key`:
 *            the first slot in probe order that is INVALID or holds the key
 *            takes the pair (last-writer-wins, north_star).
 *
 * Build-contract divergences (documented in DESIGN.md):
 *   - keys INVALID/SENTINEL are rejected (reference: undefined);
 *   - an insert whose window holds 32 entries of identical hash returns
 *     UNSPLITTABLE (reference: loops forever);
 *   - the directory depth is capped at OC_MAX_DEPTH (reference: OOM);
 *   - child 0 of a split reuses the parent's storage (reference leaks it);
 *     segment identity is therefore compared in canonical directory order.
 */
#include "cceh_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#if defined(__x86_64__)
#include <x86intrin.h>
#endif

/* ------------------------------------------------------------------ hashes */

static inline uint64_t shift_mix(uint64_t v) { return v ^ (v >> 47); }

uint64_t oc_hash64(uint64_t key) {
  /* libstdc++ _Hash_bytes for len == 8 (one aligned 8-byte block, no tail) */
  const uint64_t mul = 0xc6a4a7935bd1e995ULL;
  const uint64_t seed = 0xc70697ULL;
  uint64_t hash = seed ^ (8ULL * mul);
  uint64_t data = shift_mix(key * mul) * mul;
  hash ^= data;
  hash *= mul;
  hash = shift_mix(hash) * mul;
  hash = shift_mix(hash);
  return hash;
}

uint32_t oc_murmur2(uint64_t key, uint32_t seed) {
  /* 32-bit MurmurHash2 over the 8 little-endian key bytes */
  const uint32_t m = 0x5bd1e995u;
  uint32_t h = seed ^ 8u;
  uint32_t blocks[2] = {(uint32_t)key, (uint32_t)(key >> 32)};
  for (int i = 0; i < 2; ++i) {
    uint32_t k = blocks[i];
    k *= m;
    k ^= k >> 24;
    k *= m;
    h *= m;
    h ^= k;
  }
  h ^= h >> 13;
  h *= m;
  h ^= h >> 15;
  return h;
}

void oc_hash64_batch(const uint64_t* keys, uint64_t* out, size_t n) {
  for (size_t i = 0; i < n; ++i) out[i] = oc_hash64(keys[i]);
}

void oc_murmur2_batch(const uint64_t* keys, uint32_t seed, uint32_t* out, size_t n) {
  for (size_t i = 0; i < n; ++i) out[i] = oc_murmur2(keys[i], seed);
}

/* ------------------------------------------------------- flush emulation */
/* server/util/persist.h:7,13,31-41: clflush + busy-wait
 * kWriteLatencyInNS*CPU_FREQ_MHZ/1000 TSC ticks per 64-B line. */
static int g_flush_ns = 0;

static inline void emu_flush(const void* p, size_t len) {
  if (g_flush_ns <= 0) return;
#if defined(__x86_64__)
  const unsigned long ticks = (unsigned long)g_flush_ns * 1994UL / 1000UL;
  uintptr_t a = (uintptr_t)p & ~(uintptr_t)63;
  _mm_mfence();
  for (; a < (uintptr_t)p + len; a += 64) {
    unsigned long until = __rdtsc() + ticks;
    _mm_clflush((const void*)a);
    while (__rdtsc() < until) _mm_pause();
  }
  _mm_mfence();
#else
  (void)p;
  (void)len;
#endif
}

/* -------------------------------------------------------------------- CCEH */

typedef struct {
  uint64_t key;
  uint64_t value;
} oc_pair;

struct oc_cceh {
  oc_pair* slots;      /* cap_segs * 1024 */
  uint32_t* ldepth;    /* cap_segs */
  uint32_t nsegs, cap_segs;
  uint32_t* dir;       /* 2^depth */
  uint32_t depth;
  int upsert;          /* last-writer-wins Insert (oc_set_upsert) */
  oc_stats st;
};

static void reserve_segments(oc_cceh* t, uint32_t need) {
  if (need <= t->cap_segs) return;
  uint32_t cap = t->cap_segs ? t->cap_segs : 16;
  while (cap < need) cap *= 2;
  t->slots = (oc_pair*)realloc(t->slots, (size_t)cap * OC_SLOTS_PER_SEGMENT * sizeof(oc_pair));
  t->ldepth = (uint32_t*)realloc(t->ldepth, (size_t)cap * sizeof(uint32_t));
  t->cap_segs = cap;
}

static void init_segment(oc_cceh* t, uint32_t s, uint32_t depth) {
  oc_pair* p = t->slots + (size_t)s * OC_SLOTS_PER_SEGMENT;
  for (uint32_t i = 0; i < OC_SLOTS_PER_SEGMENT; ++i) {
    p[i].key = OC_INVALID; /* Pair::Pair() pair.h:17-18 */
    p[i].value = 0;        /* reference: uninitialized; reported as 0 */
  }
  t->ldepth[s] = depth;
}

uint32_t oc_depth_for_hybrid(uint64_t init_cap) {
  /* static_cast<size_t>(log2(initCap))  CCEH_hybrid.cpp:80 */
  return (uint32_t)(size_t)log2((double)init_cap);
}

uint32_t oc_depth_for_src(uint64_t init_cap) {
  /* static_cast<size_t>(log2(initCap/Segment::kNumSlot))  src/cceh.cpp:82 */
  return (uint32_t)(size_t)log2((double)(init_cap / OC_SLOTS_PER_SEGMENT));
}

oc_cceh* oc_create(uint32_t initial_depth, size_t reserve) {
  if (initial_depth < 1 || initial_depth > OC_MAX_DEPTH) return NULL;
  oc_cceh* t = (oc_cceh*)calloc(1, sizeof(oc_cceh));
  uint32_t n = 1u << initial_depth;
  reserve_segments(t, (uint32_t)(reserve > n ? reserve : n));
  t->depth = initial_depth;
  t->dir = (uint32_t*)malloc((size_t)n * sizeof(uint32_t));
  for (uint32_t i = 0; i < n; ++i) {
    init_segment(t, i, initial_depth);
    t->dir[i] = i;
  }
  t->nsegs = n;
  return t;
}

void oc_set_upsert(oc_cceh* t, int on) { t->upsert = on != 0; }

void oc_destroy(oc_cceh* t) {
  if (!t) return;
  free(t->slots);
  free(t->ldepth);
  free(t->dir);
  free(t);
}

static inline oc_pair* seg_ptr(const oc_cceh* t, uint32_t s) {
  return t->slots + (size_t)s * OC_SLOTS_PER_SEGMENT;
}

/* Segment::Insert4split  CCEH_hybrid.cpp:18-28 */
static int insert4split(oc_pair* seg, uint64_t key, uint64_t value, uint32_t loc) {
  for (uint32_t i = 0; i < OC_PROBE_WINDOW; ++i) {
    uint32_t slot = (loc + i) % OC_SLOTS_PER_SEGMENT;
    if (seg[slot].key == OC_INVALID) {
      seg[slot].key = key;
      seg[slot].value = value;
      return 1;
    }
  }
  return 0; /* reference prints to cerr and drops the entry (:27) */
}

/* Segment::Split (non-INPLACE)  CCEH_hybrid.cpp:47-66.  Child 0 is written in
 * place of the parent, child 1 into a new segment; returns child 1's id. */
static uint32_t split_segment(oc_cceh* t, uint32_t s) {
  static oc_pair parent[OC_SLOTS_PER_SEGMENT];
  uint32_t ld = t->ldepth[s];
  reserve_segments(t, t->nsegs + 1);
  uint32_t s1 = t->nsegs++;
  memcpy(parent, seg_ptr(t, s), sizeof(parent));
  init_segment(t, s, ld + 1);
  init_segment(t, s1, ld + 1);
  oc_pair* c[2] = {seg_ptr(t, s), seg_ptr(t, s1)};
  const uint64_t pattern = 1ULL << (63 - ld); /* :52 */
  for (uint32_t i = 0; i < OC_SLOTS_PER_SEGMENT; ++i) {
    uint64_t k = parent[i].key;
    /* An INVALID entry is also replayed by the reference, but writing an
     * INVALID key into the first INVALID slot leaves the keys unchanged. */
    if (k == OC_INVALID) continue;
    uint64_t kh = oc_hash64(k);
    uint32_t loc = (uint32_t)(kh & 0xFF) * 4;
    if (!insert4split(c[(kh & pattern) ? 1 : 0], k, parent[i].value, loc))
      t->st.split_loss++;
  }
  emu_flush(c[0], 16400);
  emu_flush(c[1], 16400);
  t->st.splits++;
  return s1;
}

static void double_directory(oc_cceh* t) {
  /* CCEH_hybrid.cpp:208-223: new[2i] = new[2i+1] = old[i] */
  uint32_t n = 1u << t->depth;
  uint32_t* nd = (uint32_t*)malloc((size_t)n * 2 * sizeof(uint32_t));
  for (uint32_t i = 0; i < n; ++i) nd[2 * i] = nd[2 * i + 1] = t->dir[i];
  free(t->dir);
  t->dir = nd;
  t->depth++;
  emu_flush(nd, (size_t)n * 2 * sizeof(uint32_t) * 2 /* 8-B pointers */);
  t->st.doublings++;
}

static inline uint64_t dir_index(uint64_t h, uint32_t depth) {
  return h >> (64 - depth);
}

int oc_insert(oc_cceh* t, uint64_t key, uint64_t value) {
  if (key == OC_INVALID || key == OC_SENTINEL) return OC_ST_RESERVED_KEY;
  const uint64_t h = oc_hash64(key);
  const uint32_t y = (uint32_t)(h & 0xFF) * 4; /* :109 */
  t->st.inserts++;
  for (;;) {
    uint32_t s = t->dir[dir_index(h, t->depth)]; /* :117-120 */
    oc_pair* seg = seg_ptr(t, s);
    for (uint32_t i = 0; i < OC_PROBE_WINDOW; ++i) { /* :143-168 */
      uint32_t loc = (y + i) % OC_SLOTS_PER_SEGMENT;
      if (t->upsert && seg[loc].key == key) { /* :153, enabled (upsert mode) */
        seg[loc].value = value;
        emu_flush(&seg[loc], sizeof(oc_pair));
        t->st.insert_lines += i / 4 + 1;
        return OC_ST_UPDATED;
      }
      if (seg[loc].key == OC_INVALID) {
        seg[loc].value = value;
        seg[loc].key = key;
        emu_flush(&seg[loc], sizeof(oc_pair));
        t->st.insert_lines += i / 4 + 1;
        return OC_ST_INSERTED;
      }
    }
    /* window full: the reference would split forever if all 32 entries share
     * this key's full hash */
    int same = 1;
    for (uint32_t i = 0; i < OC_PROBE_WINDOW && same; ++i)
      same = oc_hash64(seg[(y + i) % OC_SLOTS_PER_SEGMENT].key) == h;
    if (same) return OC_ST_UNSPLITTABLE;
    uint32_t ld = t->ldepth[s];
    if (ld + 1 > OC_MAX_DEPTH) return OC_ST_DEPTH_LIMIT;
    uint32_t s1 = split_segment(t, s);
    if (ld == t->depth) double_directory(t); /* :198-233 */
    /* :243-286: the 2^(depth-ld) entries that pointed at the parent; first
     * half -> child 0, second half -> child 1 */
    uint64_t stride = 1ULL << (t->depth - ld);
    uint64_t base = (h >> (64 - ld)) << (t->depth - ld);
    for (uint64_t i = 0; i < stride; ++i) t->dir[base + i] = (i < stride / 2) ? s : s1;
    emu_flush(&t->dir[base], stride * 8);
  }
}

int oc_get(oc_cceh* t, uint64_t key, uint64_t* value) {
  *value = 0;
  if (key == OC_INVALID || key == OC_SENTINEL) return OC_ST_RESERVED_KEY;
  const uint64_t h = oc_hash64(key);
  const uint32_t y = (uint32_t)(h & 0xFF) * 4;
  const oc_pair* seg = seg_ptr(t, t->dir[dir_index(h, t->depth)]);
  /* reference: full 32-slot scan, first match wins (:372-382) */
  int found_full = -1;
  for (uint32_t i = 0; i < OC_PROBE_WINDOW; ++i) {
    if (seg[(y + i) % OC_SLOTS_PER_SEGMENT].key == key) {
      found_full = (int)i;
      break;
    }
  }
  /* early exit at the first empty slot -- what the GPU does */
  int found_early = -1;
  uint32_t lines = OC_PROBE_WINDOW / 4;
  for (uint32_t i = 0; i < OC_PROBE_WINDOW; ++i) {
    uint64_t k = seg[(y + i) % OC_SLOTS_PER_SEGMENT].key;
    if (k == key) {
      found_early = (int)i;
      lines = i / 4 + 1;
      break;
    }
    if (k == OC_INVALID) {
      lines = i / 4 + 1;
      break;
    }
  }
  t->st.gets++;
  t->st.get_lines += lines;
  t->st.get_lines_full += found_full >= 0 ? (uint32_t)found_full / 4 + 1 : OC_PROBE_WINDOW / 4;
  if (found_early != found_full) t->st.early_exit_mismatch++;
  if (found_full < 0) return OC_ST_MISS;
  t->st.get_hits++;
  *value = seg[(y + (uint32_t)found_full) % OC_SLOTS_PER_SEGMENT].value;
  return OC_ST_HIT;
}

/* CCEH::FindAnyway  CCEH_hybrid.cpp:482-496 (twin src/cceh.cpp:457-471),
 * literally: directory entries 0..2^depth-1, each segment's slots 0..1023, the
 * first pair whose key matches (no window, no early exit; the cout
 * diagnostics are not restated).  Reserved keys are rejected as everywhere. */
int oc_find_anyway(const oc_cceh* t, uint64_t key, uint64_t* value) {
  *value = 0;
  if (key == OC_INVALID || key == OC_SENTINEL) return OC_ST_RESERVED_KEY;
  const uint64_t n = 1ULL << t->depth;
  for (uint64_t i = 0; i < n; ++i) {
    const oc_pair* seg = seg_ptr(t, t->dir[i]);
    for (uint32_t j = 0; j < OC_SLOTS_PER_SEGMENT; ++j)
      if (seg[j].key == key) {
        *value = seg[j].value;
        return OC_ST_HIT;
      }
  }
  return OC_ST_MISS;
}

void oc_find_anyway_batch(const oc_cceh* t, const uint64_t* keys, size_t n, uint64_t* out_values,
                          uint8_t* out_status) {
  for (size_t i = 0; i < n; ++i) out_status[i] = (uint8_t)oc_find_anyway(t, keys[i], &out_values[i]);
}

void oc_mixed(oc_cceh* t, const uint8_t* ops, const uint64_t* keys,
              const uint64_t* values, size_t n, uint64_t* out_values,
              uint8_t* out_status) {
  for (size_t i = 0; i < n; ++i) {
    if (ops[i] == OC_OP_INSERT) {
      out_status[i] = (uint8_t)oc_insert(t, keys[i], values[i]);
      out_values[i] = 0;
    } else {
      uint64_t v;
      out_status[i] = (uint8_t)oc_get(t, keys[i], &v);
      out_values[i] = v;
    }
  }
}

void oc_insert_batch(oc_cceh* t, const uint64_t* keys, const uint64_t* values,
                     size_t n, uint8_t* out_status) {
  for (size_t i = 0; i < n; ++i) {
    int st = oc_insert(t, keys[i], values[i]);
    if (out_status) out_status[i] = (uint8_t)st;
  }
}

void oc_get_batch(oc_cceh* t, const uint64_t* keys, size_t n,
                  uint64_t* out_values, uint8_t* out_status) {
  for (size_t i = 0; i < n; ++i) out_status[i] = (uint8_t)oc_get(t, keys[i], &out_values[i]);
}

uint32_t oc_depth(const oc_cceh* t) { return t->depth; }
uint32_t oc_num_segments(const oc_cceh* t) { return t->nsegs; }
void oc_get_stats(const oc_cceh* t, oc_stats* out) { *out = t->st; }

double oc_utilization(const oc_cceh* t) {
  /* CCEH::Utilization  CCEH_hybrid.cpp:412-427 */
  uint64_t sum = 0, cnt = 0;
  uint64_t n = 1ULL << t->depth;
  for (uint64_t i = 0; i < n; cnt++) {
    uint32_t s = t->dir[i];
    uint32_t ld = t->ldepth[s];
    uint64_t pattern = i >> (t->depth - ld);
    const oc_pair* seg = seg_ptr(t, s);
    for (uint32_t j = 0; j < OC_SLOTS_PER_SEGMENT; ++j) {
      uint64_t kh = oc_hash64(seg[j].key);
      if ((kh >> (64 - ld)) == pattern && seg[j].key != OC_INVALID) sum++;
    }
    i += 1ULL << (t->depth - ld);
  }
  return (double)sum / ((double)cnt * OC_SLOTS_PER_SEGMENT) * 100.0;
}

uint64_t oc_capacity(const oc_cceh* t) {
  /* distinct segments reachable from the directory  CCEH_hybrid.cpp:429-435 */
  return (uint64_t)t->nsegs * OC_SLOTS_PER_SEGMENT;
}

void oc_dump(const oc_cceh* t, uint32_t* dir_canon, uint32_t* local_depth,
             uint64_t* prefix, uint64_t* keys, uint64_t* values) {
  uint64_t n = 1ULL << t->depth;
  uint32_t c = 0;
  uint32_t cur = 0;
  for (uint64_t x = 0; x < n; ++x) {
    uint32_t s = t->dir[x];
    uint32_t ld = t->ldepth[s];
    if ((x & ((1ULL << (t->depth - ld)) - 1)) == 0) {
      cur = c++;
      if (local_depth) local_depth[cur] = ld;
      if (prefix) prefix[cur] = x >> (t->depth - ld);
      const oc_pair* seg = seg_ptr(t, s);
      for (uint32_t j = 0; j < OC_SLOTS_PER_SEGMENT; ++j) {
        size_t o = (size_t)cur * OC_SLOTS_PER_SEGMENT + j;
        if (keys) keys[o] = seg[j].key;
        if (values) values[o] = seg[j].key == OC_INVALID ? 0 : seg[j].value;
      }
    }
    if (dir_canon) dir_canon[x] = cur;
  }
}

/* ------------------------------------------------------------ bloom filter */

static inline uint64_t bloom_index(uint64_t key, uint32_t i, uint64_t nbits) {
  /* client/bloom_filter.c:69,93: hash_funcs[1](data, 8, i) % bitmap_size */
  return (uint64_t)oc_murmur2(key, i) % nbits;
}

void oc_bloom_add(uint64_t* bitmap, uint64_t nbits, uint32_t k, uint64_t key) {
  for (uint32_t i = 0; i < k; ++i) {
    uint64_t idx = bloom_index(key, i, nbits);
    bitmap[idx / 64] |= 1ULL << (63 - idx % 64); /* bloom_filter.c:71-74 */
  }
}

int oc_bloom_check(const uint64_t* bitmap, uint64_t nbits, uint32_t k, uint64_t key,
                   uint32_t* probes_out) {
  uint32_t probes = 0;
  int res = 1;
  for (uint32_t i = 0; i < k; ++i) { /* bloom_filter.c:92-114 */
    uint64_t idx = bloom_index(key, i, nbits);
    probes++;
    if ((bitmap[idx / 64] & (1ULL << (63 - idx % 64))) == 0) {
      res = 0;
      break;
    }
  }
  if (probes_out) *probes_out = probes;
  return res;
}

void oc_bloom_add_batch(uint64_t* bitmap, uint64_t nbits, uint32_t k,
                        const uint64_t* keys, size_t n) {
  for (size_t i = 0; i < n; ++i) oc_bloom_add(bitmap, nbits, k, keys[i]);
}

void oc_bloom_check_batch(const uint64_t* bitmap, uint64_t nbits, uint32_t k,
                          const uint64_t* keys, size_t n, uint8_t* out,
                          uint64_t* total_probes) {
  uint64_t tp = 0;
  for (size_t i = 0; i < n; ++i) {
    uint32_t p;
    out[i] = (uint8_t)oc_bloom_check(bitmap, nbits, k, keys[i], &p);
    tp += p;
  }
  if (total_probes) *total_probes = tp;
}

/* counting_bloom_filter.h:249-254: int idx = murmur2(&key,8,salt) % m */
static inline uint64_t cbf_index(uint64_t key, uint32_t salt, uint64_t nbits) {
  return (uint64_t)(int)((uint64_t)oc_murmur2(key, salt) % nbits);
}

void oc_cbf_insert(uint8_t* counters, uint64_t nbits, uint32_t k, uint64_t key) {
  for (uint32_t i = 0; i < k; ++i) { /* :109-118 (saturating at 255) */
    uint64_t idx = cbf_index(key, i, nbits);
    if (counters[idx] < 255) counters[idx] += 1;
  }
}

int oc_cbf_query(const uint8_t* counters, uint64_t nbits, uint32_t k, uint64_t key) {
  for (uint32_t i = 0; i < k; ++i) /* :133-143 */
    if (counters[cbf_index(key, i, nbits)] == 0) return 0;
  return 1;
}

int oc_cbf_delete(uint8_t* counters, uint64_t nbits, uint32_t k, uint64_t key) {
  if (!oc_cbf_query(counters, nbits, k, key)) return 0; /* :120-131 */
  for (uint32_t i = 0; i < k; ++i) counters[cbf_index(key, i, nbits)] -= 1;
  return 1;
}

void oc_cbf_to_bitmap(const uint8_t* counters, uint64_t nbits, uint64_t* bitmap) {
  /* ToOrdinaryBloomFilter  :202-215 */
  uint64_t nlongs = (nbits + 63) / 64;
  memset(bitmap, 0, nlongs * sizeof(uint64_t));
  for (uint64_t i = 0; i < nbits; ++i)
    if (counters[i] > 0) bitmap[i / 64] |= 1ULL << (63 - i % 64);
}

/* batch forms: Insert / Delete applied one key at a time in batch order */
void oc_cbf_insert_batch(uint8_t* counters, uint64_t nbits, uint32_t k, const uint64_t* keys,
                         uint64_t n) {
  for (uint64_t i = 0; i < n; ++i) oc_cbf_insert(counters, nbits, k, keys[i]);
}

void oc_cbf_delete_batch(uint8_t* counters, uint64_t nbits, uint32_t k, const uint64_t* keys,
                         uint64_t n, uint8_t* deleted) {
  for (uint64_t i = 0; i < n; ++i) deleted[i] = (uint8_t)oc_cbf_delete(counters, nbits, k, keys[i]);
}

/* --------------------------------------------------------- CPU baseline */

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec + ts.tv_nsec * 1e-9;
}

double oc_time_insert(oc_cceh* t, const uint64_t* keys, size_t n, int flush_ns) {
  g_flush_ns = flush_ns;
  double t0 = now_s();
  for (size_t i = 0; i < n; ++i) oc_insert(t, keys[i], keys[i]); /* value = key */
  double t1 = now_s();
  g_flush_ns = 0;
  return t1 - t0;
}

typedef struct {
  const oc_cceh* t;
  const uint64_t* keys;
  size_t from, to;
  uint64_t misses;
} get_job;

static uint64_t get_quiet(const oc_cceh* t, uint64_t key, int* found) {
  /* read-only Get without statistics (thread-safe) */
  const uint64_t h = oc_hash64(key);
  const uint32_t y = (uint32_t)(h & 0xFF) * 4;
  const oc_pair* seg = seg_ptr(t, t->dir[dir_index(h, t->depth)]);
  for (uint32_t i = 0; i < OC_PROBE_WINDOW; ++i) {
    const oc_pair* p = &seg[(y + i) % OC_SLOTS_PER_SEGMENT];
    if (p->key == key) {
      *found = 1;
      return p->value;
    }
  }
  *found = 0;
  return 0;
}

static void* get_worker(void* arg) {
  get_job* j = (get_job*)arg;
  uint64_t miss = 0;
  for (size_t i = j->from; i < j->to; ++i) {
    int f;
    uint64_t v = get_quiet(j->t, j->keys[i], &f);
    if (!f || v != j->keys[i]) miss++;
  }
  j->misses = miss;
  return NULL;
}

double oc_time_get(oc_cceh* t, const uint64_t* keys, size_t n, int threads,
                   uint64_t* misses) {
  if (threads < 1) threads = 1;
  pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
  get_job* jobs = (get_job*)calloc((size_t)threads, sizeof(get_job));
  size_t chunk = n / (size_t)threads;
  double t0 = now_s();
  for (int i = 0; i < threads; ++i) {
    jobs[i].t = t;
    jobs[i].keys = keys;
    jobs[i].from = chunk * (size_t)i;
    jobs[i].to = (i == threads - 1) ? n : chunk * (size_t)(i + 1);
    pthread_create(&th[i], NULL, get_worker, &jobs[i]);
  }
  uint64_t m = 0;
  for (int i = 0; i < threads; ++i) {
    pthread_join(th[i], NULL);
    m += jobs[i].misses;
  }
  double t1 = now_s();
  if (misses) *misses = m;
  free(th);
  free(jobs);
  return t1 - t0;
}
