/*
 * cceh_mt.c -- concurrent CPU restatement of CCEH_hybrid (non-INPLACE build)
 * for the CPU baseline of bench.py.
 *
 * TEST INFRASTRUCTURE ONLY (see cceh_oracle.h): timed by bench.py's
 * cpu_baseline leg and calibrated against the reference binary
 * (oracle/bench_cpu.py); never linked by the product.  The serial parity
 * checker is cceh_oracle.c; this file restates the reference's CONCURRENCY
 * so the baseline pays what the reference pays per op:
 *
 *   Segment::lock / unlock / suspend      server/CCEH_hybrid.h:40-77
 *     sema >= 0 counts holders; suspend CASes it to -1 and waits for the
 *     holders to drain.
 *   Directory::lock / unlock / suspend    server/CCEH_hybrid.h:100-140
 *   CCEH::Insert                          server/CCEH_hybrid.cpp:107-298
 *     lock the target segment, re-check the directory entry and depth, probe
 *     the 32-slot window (a slot is free if INVALID or its key's hash prefix
 *     is stale, :149-156; never SENTINEL), claim it by CAS key -> SENTINEL,
 *     write the value, mfence, write the key, clflush (:157-165).  On a full
 *     window: unlock, suspend, split into two new segments by slot-order
 *     Insert4split (:18-66), then double the directory (:198-233) or update
 *     the stride under the directory lock (:234-295), retry.  Old segments
 *     and directories are leaked by the reference; here they are kept on a
 *     list and freed at destroy.
 *   CCEH::Get                             server/CCEH_hybrid.cpp:343-389
 *     spin while the directory is suspended, read the entry, re-check it,
 *     full 32-slot scan (no early exit).  The reference's non-INPLACE Get
 *     calls target->unlock() on a re-check mismatch without having locked;
 *     that stray decrement is not restated.
 *   clflush emulation                     server/util/persist.h:27-41
 *     clflush + busy-wait kWriteLatencyInNS * CPU_FREQ_MHZ / 1000 TSC ticks
 *     per 64-B line (10 ns at the reference's 1994 MHz constant), optional.
 *   Harness                               server/test_KV.cpp:204-308
 *     T threads pinned one per CPU, contiguous key chunks, value = key,
 *     insert phase then search phase, failedSearch counted; without the
 *     search threads' sleep(1) (:211), which the reference times.
 */
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#if defined(__x86_64__)
#include <x86intrin.h>
#endif

#include "cceh_oracle.h"

#define MT_SLOTS 1024u
#define MT_WINDOW 32u
#define MT_CPU_FREQ_MHZ 1994u /* persist.h:7 */

typedef struct {
  uint64_t key;
  uint64_t value;
} mt_pair;

typedef struct mt_seg {
  mt_pair p[MT_SLOTS];
  int64_t sema;
  uint64_t local_depth;
} __attribute__((aligned(64))) mt_seg;

typedef struct {
  mt_seg** e;
  int64_t sema;
  uint64_t capacity;
  uint64_t depth;
} mt_dir;

struct oc_mt {
  mt_dir* volatile dir;
  int flush_ns;
  pthread_mutex_t gc_mu;  /* leaked segments / directories, freed at destroy */
  void** gc;
  size_t ngc, capgc;
  int64_t segments;       /* live segments (atomic) */
};

/* h() (server/util/hash.h:7-10,252-254), inlined as the reference's is */
static inline uint64_t mt_hash(uint64_t key) {
  const uint64_t mul = 0xc6a4a7935bd1e995ULL;
  uint64_t hash = 0xc70697ULL ^ (8ULL * mul);
  uint64_t d = key * mul;
  d = (d ^ (d >> 47)) * mul;
  hash = (hash ^ d) * mul;
  hash = (hash ^ (hash >> 47)) * mul;
  return hash ^ (hash >> 47);
}

#define CAS64(p, expp, v) __atomic_compare_exchange_n((p), (expp), (v), 0, __ATOMIC_ACQUIRE, __ATOMIC_ACQUIRE)
#define LOAD(p) __atomic_load_n((p), __ATOMIC_ACQUIRE)
#define STORE(p, v) __atomic_store_n((p), (v), __ATOMIC_RELEASE)

static inline void mt_mfence(void) { __atomic_thread_fence(__ATOMIC_SEQ_CST); }

static inline void mt_clflush(const oc_mt* t, const void* data, size_t len) {
  if (t->flush_ns <= 0) return;
#if defined(__x86_64__)
  const unsigned long ticks = (unsigned long)t->flush_ns * MT_CPU_FREQ_MHZ / 1000UL;
  uintptr_t a = (uintptr_t)data & ~(uintptr_t)63;
  _mm_mfence();
  for (; a < (uintptr_t)data + len; a += 64) {
    const unsigned long until = __rdtsc() + ticks;
    _mm_clflush((const void*)a);
    while (__rdtsc() < until) _mm_pause();
  }
  _mm_mfence();
#else
  (void)data;
  (void)len;
#endif
}

static void gc_push(oc_mt* t, void* p) {
  pthread_mutex_lock(&t->gc_mu);
  if (t->ngc == t->capgc) {
    t->capgc = t->capgc ? 2 * t->capgc : 1024;
    t->gc = (void**)realloc(t->gc, t->capgc * sizeof(void*));
  }
  t->gc[t->ngc++] = p;
  pthread_mutex_unlock(&t->gc_mu);
}

/* ---- Segment / Directory semaphores (CCEH_hybrid.h:40-77, :100-140) ---- */
static int sema_lock(int64_t* sema) {
  int64_t val = LOAD(sema);
  while (val > -1) {
    if (CAS64(sema, &val, val + 1)) return 1;
    val = LOAD(sema);
  }
  return 0;
}

static void sema_unlock(int64_t* sema) {
  int64_t val = LOAD(sema);
  while (!CAS64(sema, &val, val - 1)) val = LOAD(sema);
}

static int sema_suspend(int64_t* sema) {
  int64_t val;
  do {
    val = LOAD(sema);
    if (val < 0) return 0;
  } while (!CAS64(sema, &val, -1));
  /* the reference waits for sema == -val-1: with the holders' unlocks
   * decrementing from -1, that is when all val holders have left */
  const int64_t wait = 0 - val - 1;
  while (val && LOAD(sema) != wait) {
#if defined(__x86_64__)
    _mm_pause();
#endif
  }
  return 1;
}

static mt_seg* seg_new(oc_mt* t, uint64_t depth) {
  mt_seg* s = NULL;
  if (posix_memalign((void**)&s, 64, sizeof(mt_seg))) return NULL;
  for (uint32_t i = 0; i < MT_SLOTS; ++i) s->p[i].key = OC_INVALID; /* Pair() pair.h:17-18 */
  s->sema = 0;
  s->local_depth = depth;
  gc_push(t, s);
  __atomic_add_fetch(&t->segments, 1, __ATOMIC_RELAXED);
  return s;
}

static mt_dir* dir_new(oc_mt* t, uint64_t depth) {
  mt_dir* d = (mt_dir*)calloc(1, sizeof(mt_dir));
  d->depth = depth;
  d->capacity = 1ULL << depth;
  if (posix_memalign((void**)&d->e, 64, d->capacity * sizeof(mt_seg*))) return NULL;
  gc_push(t, d->e);
  gc_push(t, d);
  return d;
}

/* Segment::Insert4split (CCEH_hybrid.cpp:18-28) */
static void insert4split(mt_seg* s, uint64_t key, uint64_t value, uint32_t loc) {
  for (uint32_t i = 0; i < MT_WINDOW; ++i) {
    const uint32_t slot = (loc + i) % MT_SLOTS;
    if (s->p[slot].key == OC_INVALID) {
      s->p[slot].key = key;
      s->p[slot].value = value;
      return;
    }
  }
  /* the reference prints to cerr and drops the entry (:27) */
}

/* Segment::Split, non-INPLACE (CCEH_hybrid.cpp:47-66) */
static void seg_split(oc_mt* t, mt_seg* src, mt_seg** s0, mt_seg** s1) {
  *s0 = seg_new(t, src->local_depth + 1);
  *s1 = seg_new(t, src->local_depth + 1);
  const uint64_t pattern = 1ULL << (64 - src->local_depth - 1);
  for (uint32_t i = 0; i < MT_SLOTS; ++i) {
    const uint64_t kh = mt_hash(src->p[i].key);
    insert4split((kh & pattern) ? *s1 : *s0, src->p[i].key, src->p[i].value, (uint32_t)(kh & 0xFF) * 4);
  }
  mt_clflush(t, *s0, sizeof(mt_seg));
  mt_clflush(t, *s1, sizeof(mt_seg));
}

oc_mt* oc_mt_create(uint32_t depth, int flush_ns) {
  if (depth < 1 || depth > OC_MAX_DEPTH) return NULL;
  oc_mt* t = (oc_mt*)calloc(1, sizeof(oc_mt));
  pthread_mutex_init(&t->gc_mu, NULL);
  t->flush_ns = flush_ns;
  mt_dir* d = dir_new(t, depth);
  for (uint64_t i = 0; i < d->capacity; ++i) d->e[i] = seg_new(t, depth);
  t->dir = d;
  return t;
}

void oc_mt_destroy(oc_mt* t) {
  if (!t) return;
  for (size_t i = 0; i < t->ngc; ++i) free(t->gc[i]);
  free(t->gc);
  pthread_mutex_destroy(&t->gc_mu);
  free(t);
}

/* CCEH::Insert (CCEH_hybrid.cpp:107-298) */
void oc_mt_insert(oc_mt* t, uint64_t key, uint64_t value) {
  const uint64_t h = mt_hash(key);
  const uint32_t y = (uint32_t)(h & 0xFF) * 4;
  for (;;) { /* RETRY */
    mt_dir* d = LOAD(&t->dir);
    const uint64_t depth = d->depth;
    uint64_t x = h >> (64 - depth);
    mt_seg* target = LOAD(&d->e[x]);
    if (!sema_lock(&target->sema)) {
      sched_yield();
      continue;
    }
    mt_dir* d2 = LOAD(&t->dir);
    if (target != LOAD(&d2->e[h >> (64 - depth)])) {
      sema_unlock(&target->sema);
      sched_yield();
      continue;
    }
    const uint64_t pattern = x >> (depth - target->local_depth);
    if (depth != LOAD(&t->dir)->depth) {
      sema_unlock(&target->sema);
      sched_yield();
      continue;
    }
    for (uint32_t i = 0; i < MT_WINDOW; ++i) {
      const uint32_t loc = (y + i) % MT_SLOTS;
      uint64_t k0 = LOAD(&target->p[loc].key);
      if (((mt_hash(k0) >> (64 - target->local_depth)) != pattern || k0 == OC_INVALID) && k0 != OC_SENTINEL) {
        if (CAS64(&target->p[loc].key, &k0, OC_SENTINEL)) {
          target->p[loc].value = value;
          mt_mfence();
          STORE(&target->p[loc].key, key);
          mt_clflush(t, &target->p[loc], sizeof(mt_pair));
          sema_unlock(&target->sema);
          return;
        }
      }
    }
    /* COLLISION: split */
    const uint64_t tld = target->local_depth;
    sema_unlock(&target->sema);
    if (!sema_suspend(&target->sema)) {
      sched_yield();
      continue;
    }
    if (tld != LOAD(&LOAD(&t->dir)->e[x])->local_depth) {
      STORE(&target->sema, 0);
      sched_yield();
      continue;
    }
    mt_seg *s0, *s1;
    seg_split(t, target, &s0, &s1);
    d = LOAD(&t->dir);
    if (target->local_depth == d->depth) {
      /* directory doubling (:198-233) */
      if (!sema_suspend(&d->sema)) {
        STORE(&target->sema, 0);
        __atomic_sub_fetch(&t->segments, 2, __ATOMIC_RELAXED);
        sched_yield();
        continue;
      }
      mt_dir* nd = dir_new(t, d->depth + 1);
      for (uint64_t i = 0; i < d->capacity; ++i) {
        if (i == x) {
          nd->e[2 * i] = s0;
          nd->e[2 * i + 1] = s1;
        } else {
          nd->e[2 * i] = nd->e[2 * i + 1] = d->e[i];
        }
      }
      mt_clflush(t, nd->e, sizeof(mt_seg*) * nd->capacity);
      mt_clflush(t, nd, sizeof(mt_dir));
      STORE(&t->dir, nd);
      mt_clflush(t, (const void*)&t->dir, sizeof(void*));
    } else {
      /* stride update (:234-295) */
      if (!sema_lock(&d->sema)) {
        STORE(&target->sema, 0);
        __atomic_sub_fetch(&t->segments, 2, __ATOMIC_RELAXED);
        sched_yield();
        continue;
      }
      x = h >> (64 - d->depth);
      if (d->depth == target->local_depth + 1) {
        if (x % 2 == 0) {
          STORE(&d->e[x + 1], s1);
          mt_mfence();
          STORE(&d->e[x], s0);
          mt_clflush(t, &d->e[x], 16);
        } else {
          STORE(&d->e[x], s1);
          mt_mfence();
          STORE(&d->e[x - 1], s0);
          mt_clflush(t, &d->e[x - 1], 16);
        }
      } else {
        const uint64_t stride = 1ULL << (d->depth - target->local_depth);
        const uint64_t loc = x - (x % stride);
        for (uint64_t i = 0; i < stride / 2; ++i) STORE(&d->e[loc + stride / 2 + i], s1);
        for (uint64_t i = 0; i < stride / 2; ++i) STORE(&d->e[loc + i], s0);
        mt_clflush(t, &d->e[loc], sizeof(void*) * stride);
      }
      sema_unlock(&d->sema);
    }
    __atomic_sub_fetch(&t->segments, 1, __ATOMIC_RELAXED); /* the parent is dead */
    sched_yield();
  }
}

/* CCEH::Get (CCEH_hybrid.cpp:343-389) */
uint64_t oc_mt_get(oc_mt* t, uint64_t key) {
  const uint64_t h = mt_hash(key);
  const uint32_t y = (uint32_t)(h & 0xFF) * 4;
  for (;;) {
    while (LOAD(&LOAD(&t->dir)->sema) < 0) {
#if defined(__x86_64__)
      _mm_pause();
#endif
    }
    mt_dir* d = LOAD(&t->dir);
    const uint64_t depth = d->depth;
    mt_seg* target = LOAD(&d->e[h >> (64 - depth)]);
    if (target != LOAD(&LOAD(&t->dir)->e[h >> (64 - depth)])) {
      sched_yield();
      continue;
    }
    for (uint32_t i = 0; i < MT_WINDOW; ++i) {
      const uint32_t loc = (y + i) % MT_SLOTS;
      if (LOAD(&target->p[loc].key) == key) return target->p[loc].value;
    }
    return 0; /* NONE */
  }
}

uint32_t oc_mt_depth(const oc_mt* t) { return (uint32_t)t->dir->depth; }
uint64_t oc_mt_segments(const oc_mt* t) { return (uint64_t)t->segments; }

/* ---- the test_KV harness (server/test_KV.cpp:204-308) ------------------ */
typedef struct {
  oc_mt* t;
  const uint64_t* keys;
  size_t from, to;
  uint64_t failed;
  pthread_barrier_t* bar;
} mt_job;

static void* insert_worker(void* arg) {
  mt_job* j = (mt_job*)arg;
  pthread_barrier_wait(j->bar);
  for (size_t i = j->from; i < j->to; ++i) oc_mt_insert(j->t, j->keys[i], j->keys[i]);
  return NULL;
}

static void* get_worker(void* arg) {
  mt_job* j = (mt_job*)arg;
  uint64_t f = 0;
  pthread_barrier_wait(j->bar);
  for (size_t i = j->from; i < j->to; ++i) f += oc_mt_get(j->t, j->keys[i]) != j->keys[i];
  j->failed = f;
  return NULL;
}

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec + ts.tv_nsec * 1e-9;
}

/* one phase: T threads pinned to cpus[i] (or unpinned if cpus is NULL); the
 * clock starts when every thread is created and released by the barrier */
static double run_phase(oc_mt* t, const uint64_t* keys, size_t n, int T, const int* cpus,
                        void* (*fn)(void*), uint64_t* failed) {
  pthread_t* th = (pthread_t*)calloc((size_t)T, sizeof(pthread_t));
  mt_job* jobs = (mt_job*)calloc((size_t)T, sizeof(mt_job));
  pthread_barrier_t bar;
  pthread_barrier_init(&bar, NULL, (unsigned)T + 1);
  const size_t chunk = n / (size_t)T;
  for (int i = 0; i < T; ++i) {
    jobs[i].t = t;
    jobs[i].keys = keys;
    jobs[i].from = chunk * (size_t)i;
    jobs[i].to = i == T - 1 ? n : chunk * (size_t)(i + 1);
    jobs[i].bar = &bar;
    pthread_attr_t at;
    pthread_attr_init(&at);
    if (cpus) {
      cpu_set_t set;
      CPU_ZERO(&set);
      CPU_SET(cpus[i], &set);
      pthread_attr_setaffinity_np(&at, sizeof(set), &set);
    }
    pthread_create(&th[i], &at, fn, &jobs[i]);
    pthread_attr_destroy(&at);
  }
  pthread_barrier_wait(&bar);
  const double t0 = now_s();
  uint64_t f = 0;
  for (int i = 0; i < T; ++i) {
    pthread_join(th[i], NULL);
    f += jobs[i].failed;
  }
  const double el = now_s() - t0;
  pthread_barrier_destroy(&bar);
  free(th);
  free(jobs);
  if (failed) *failed = f;
  return el;
}

int oc_mt_bench(uint32_t depth, const uint64_t* keys, size_t n, int threads, const int* cpus, int flush_ns,
                oc_mt_result* out) {
  if (threads < 1 || !out) return -1;
  oc_mt* t = oc_mt_create(depth, flush_ns);
  if (!t) return -1;
  out->insert_s = run_phase(t, keys, n, threads, cpus, insert_worker, NULL);
  out->get_s = run_phase(t, keys, n, threads, cpus, get_worker, &out->failed);
  out->depth = oc_mt_depth(t);
  out->segments = oc_mt_segments(t);
  oc_mt_destroy(t);
  return 0;
}
