// cceh_engine.hip -- host side of the MI355X batched CCEH engine and the
// C-ABI declared in include/pmdfc_cceh.h.
//
// The engine owns its HBM (segment arena, occupancy bitmaps, local depths,
// directory, batch workspaces) and drives the kernels of cceh_kernels.hip.
// Insert/mixed batches run a short pass loop:
//     route (segment id per pending op) -> stable radix sort by segment
//     -> k_process (one lane per segment run, batch order)
//     -> [host reads 1 control block] -> directory doubling if needed
//     -> k_split (one wave per full segment) -> compact deferred ops -> repeat
// Pure Get batches are one sync-free kernel (k_get).
#include <hip/hip_runtime.h>
#include <cstdlib>
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_select.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/pmdfc_cceh.h"
#include "cceh_device.h"
#include "cceh_kernels.h"

using namespace pmdfc;

namespace {

thread_local std::string g_err;

int fail(int code, const char* what, hipError_t e = hipSuccess) {
  char buf[512];
  if (e != hipSuccess)
    snprintf(buf, sizeof buf, "%s: %s", what, hipGetErrorString(e));
  else
    snprintf(buf, sizeof buf, "%s", what);
  g_err = buf;
  return code;
}

#define HIPCHK(x)                                   \
  do {                                              \
    hipError_t e_ = (x);                            \
    if (e_ != hipSuccess) return fail(PMDFC_ERR_HIP, #x, e_); \
  } while (0)

uint32_t ceil_log2(uint64_t v) {
  uint32_t b = 0;
  while ((1ULL << b) < v) ++b;
  return b;
}

struct DevGuard {
  int prev = -1;
  explicit DevGuard(int d) {
    (void)hipGetDevice(&prev);
    if (prev != d) (void)hipSetDevice(d);
  }
  ~DevGuard() {
    int cur;
    (void)hipGetDevice(&cur);
    if (prev >= 0 && cur != prev) (void)hipSetDevice(prev);
  }
};

struct Timing {
  bool on = false;
  struct Rec {
    int cls;
    hipEvent_t a, b;
  };
  std::vector<Rec> recs;
  std::vector<hipEvent_t> pool;
  double ms[PMDFC_K_COUNT] = {0};
  uint64_t launches[PMDFC_K_COUNT] = {0};

  hipEvent_t ev() {
    if (!pool.empty()) {
      hipEvent_t e = pool.back();
      pool.pop_back();
      return e;
    }
    hipEvent_t e;
    (void)hipEventCreate(&e);
    return e;
  }
  void flush() {
    for (auto& r : recs) {
      (void)hipEventSynchronize(r.b);
      float t = 0;
      (void)hipEventElapsedTime(&t, r.a, r.b);
      ms[r.cls] += t;
      launches[r.cls] += 1;
      pool.push_back(r.a);
      pool.push_back(r.b);
    }
    recs.clear();
  }
  ~Timing() {
    flush();
    for (auto e : pool) (void)hipEventDestroy(e);
  }
};

struct Scope {
  Timing* t;
  int cls;
  hipStream_t s;
  hipEvent_t a = nullptr;
  Scope(Timing* t_, int c, hipStream_t s_) : t(t_), cls(c), s(s_) {
    if (t->on) {
      a = t->ev();
      (void)hipEventRecord(a, s);
    }
  }
  ~Scope() {
    if (t->on) {
      hipEvent_t b = t->ev();
      (void)hipEventRecord(b, s);
      t->recs.push_back({cls, a, b});
      if (t->recs.size() > 4096) t->flush();
    }
  }
};

}  // namespace

struct pmdfc_cceh {
  pmdfc_cceh_config_t cfg{};
  int dev = 0;
  uint32_t D0 = 1, Dp = 1, sbits = 0, shard = 0;
  uint64_t max_segs = 0;
  uint32_t max_batch = 0;

  ulonglong2* pairs = nullptr;
  uint32_t* occ = nullptr;
  uint8_t* ldep = nullptr;
  uint32_t* dir = nullptr;
  uint32_t* dir_alt = nullptr;
  uint64_t dir_cap = 0, dir_alt_cap = 0;  // entries

  DevCtl* ctl = nullptr;
  DevCtl* hctl = nullptr;  // pinned mirror

  uint64_t* hbuf = nullptr;
  uint32_t *skey_in = nullptr, *skey_out = nullptr, *sval_in = nullptr, *sval_out = nullptr;
  uint32_t* pend = nullptr;
  uint8_t* flags = nullptr;
  uint8_t* touched = nullptr;
  uint32_t* split_list = nullptr;
  uint32_t* partials = nullptr;
  uint32_t* sel_count = nullptr;
  unsigned long long* popc = nullptr;
  void* tmp = nullptr;
  size_t tmp_bytes = 0;
  // bucket fast path
  uint64_t* rec = nullptr;
  uint8_t* pstate = nullptr;
  uint8_t* bwork = nullptr;
  uint32_t* hist = nullptr;
  uint32_t* inc = nullptr;
  uint64_t hist_cap = 0;
  bool use_bucket = true;

  // host mirrors (exact after every sync)
  uint32_t nsegs = 0, max_ld = 0;
  uint64_t splits = 0, doublings = 0, passes = 0, batches = 0, split_loss = 0, deferred_ops = 0;
  uint64_t last_get_n = 0, last_get_blocks = 0;
  bool last_get_counted = false;
  bool count_lines = false;
  Timing timing;
  std::mutex mu;

  Geo geo() const { return Geo{dir, Dp, sbits, shard}; }
  uint64_t dir_entries() const { return 1ULL << (Dp - sbits); }
};

struct pmdfc_bloom {
  int dev = 0;
  uint64_t nbits = 0, nwords = 0;
  uint32_t k = 0;
  uint64_t* bm = nullptr;
};

// ------------------------------------------------------------------ helpers

static int ensure_alt(pmdfc_cceh* t, uint64_t entries) {
  if (t->dir_alt_cap >= entries) return PMDFC_OK;
  if (t->dir_alt) HIPCHK(hipFree(t->dir_alt));
  t->dir_alt = nullptr;
  HIPCHK(hipMalloc(&t->dir_alt, entries * sizeof(uint32_t)));
  t->dir_alt_cap = entries;
  return PMDFC_OK;
}

static int double_dir(pmdfc_cceh* t, hipStream_t s) {
  if (t->Dp + 1 > kMaxDepth) return fail(PMDFC_ERR_STATE, "directory depth limit");
  const uint64_t n_new = t->dir_entries() * 2;
  int rc = ensure_alt(t, n_new);
  if (rc) return rc;
  launch_double(t->dir, t->dir_alt, n_new, s);
  std::swap(t->dir, t->dir_alt);
  std::swap(t->dir_cap, t->dir_alt_cap);
  t->Dp += 1;
  t->doublings += 1;
  return PMDFC_OK;
}

static int sync_ctl(pmdfc_cceh* t, hipStream_t s) {
  HIPCHK(hipMemcpyAsync(t->hctl, t->ctl, sizeof(DevCtl), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  t->nsegs = std::min<uint64_t>(t->hctl->nsegs, t->max_segs);
  t->max_ld = t->hctl->max_ld;
  t->split_loss = t->hctl->split_loss;
  t->splits = t->hctl->splits;
  return PMDFC_OK;
}

static int init_state(pmdfc_cceh* t, hipStream_t s) {
  const uint32_t n0 = 1u << (t->D0 - t->sbits);
  t->Dp = t->D0;
  launch_init_segments(t->pairs, t->occ, t->ldep, t->dir, n0, t->D0, s);
  DevCtl c{};
  c.nsegs = n0;
  c.max_ld = t->D0;
  *t->hctl = c;
  HIPCHK(hipMemcpyAsync(t->ctl, t->hctl, sizeof(DevCtl), hipMemcpyHostToDevice, s));
  HIPCHK(hipStreamSynchronize(s));
  t->nsegs = n0;
  t->max_ld = t->D0;
  t->splits = t->doublings = t->passes = t->batches = t->split_loss = t->deferred_ops = 0;
  return PMDFC_OK;
}

// Insert/mixed pass loop over the pending ops.  pend == nullptr means the
// identity list 0..npend-1.
static int run_passes(pmdfc_cceh* t, const uint8_t* ops, const uint64_t* keys, const uint64_t* vin,
                      uint64_t* vout, uint8_t* st, uint64_t n, const uint32_t* pend0,
                      uint64_t npend, hipStream_t s) {
  const uint32_t* pend = pend0;
  uint32_t guard = 0;
  while (npend > 0) {
    if (++guard > 4096) return fail(PMDFC_ERR_STATE, "insert pass loop did not converge");
    const uint32_t bits = std::max<uint32_t>(1, ceil_log2((uint64_t)t->nsegs + 1));
    const uint32_t sent = (uint32_t)((1ULL << bits) - 1);
    {
      Scope sc(&t->timing, PMDFC_K_ROUTE, s);
      launch_route(pend, npend, t->hbuf, st, t->geo(), sent, t->skey_in, t->sval_in, s);
    }
    {
      Scope sc(&t->timing, PMDFC_K_SORT, s);
      size_t bytes = t->tmp_bytes;
      HIPCHK(rocprim::radix_sort_pairs(t->tmp, bytes, t->skey_in, t->skey_out, t->sval_in,
                                       t->sval_out, (size_t)npend, 0u, bits, s));
    }
    HIPCHK(hipMemsetAsync(&t->ctl->n_split, 0, 3 * sizeof(uint32_t), s));  // n_split, n_deferred, need_double
    HIPCHK(hipMemsetAsync(t->flags, 0, n, s));
    {
      Scope sc(&t->timing, PMDFC_K_PROCESS, s);
      launch_process(t->skey_out, t->sval_out, npend, sent, ops, keys, vin, vout, st, t->hbuf,
                     t->pairs, t->occ, t->ldep, t->flags, t->split_list, t->ctl, t->Dp,
                     (uint32_t)t->max_segs, s);
    }
    int rc = sync_ctl(t, s);
    if (rc) return rc;
    t->passes += 1;
    const uint32_t nsplit = t->hctl->n_split;
    if (nsplit == 0) break;
    if (t->hctl->need_double) {
      rc = double_dir(t, s);
      if (rc) return rc;
    }
    {
      Scope sc(&t->timing, PMDFC_K_SPLIT, s);
      launch_split(nsplit, t->split_list, t->pairs, t->occ, t->ldep, t->dir, t->Dp, t->sbits,
                   t->ctl, s);
    }
    npend = t->hctl->n_deferred;
    if (npend == 0) break;
    {
      Scope sc(&t->timing, PMDFC_K_SELECT, s);
      size_t bytes = t->tmp_bytes;
      HIPCHK(rocprim::select(t->tmp, bytes, rocprim::counting_iterator<uint32_t>(0), t->flags,
                             t->pend, t->sel_count, (size_t)n, s));
    }
    pend = t->pend;
  }
  // a pass that only split (no ops left) still needs the final depths
  if (t->hctl->n_split) {
    int rc = sync_ctl(t, s);
    if (rc) return rc;
  }
  t->batches += 1;
  return PMDFC_OK;
}

// Bucket fast path (bucket.hip).  Returns 1 if it is not applicable for the
// current geometry (caller falls back to run_passes).
// Bucket fast path (bucket.hip).  Returns 1 if it is not applicable for the
// current geometry (caller falls back to run_passes).
static int choose_p1(const pmdfc_cceh* t, uint64_t n, uint32_t* p1_out, uint32_t* bbits_out) {
  const uint32_t Dl = t->Dp - t->sbits;
  const uint32_t lmin = t->D0 - t->sbits;  // local depths never shrink below D0
  const uint32_t cap = std::min<uint32_t>(12u, lmin);
  if (cap < 1) return 1;
  uint32_t p1 = 1;
  while (p1 < cap && (n >> (p1 + 1)) >= 192) ++p1;
  if (Dl > p1 + 9) p1 = Dl - 9;  // directory slice <= 512 bins
  if (p1 > cap || p1 < 1) return 1;
  *p1_out = p1;
  *bbits_out = Dl - p1;
  return 0;
}

static int run_bucket(pmdfc_cceh* t, const uint8_t* ops, const uint64_t* keys, const uint64_t* vin,
                      uint64_t* vout, uint8_t* st, uint64_t n, const uint32_t* pend,
                      const uint32_t* npend_dev, uint32_t p1, uint32_t bbits, hipStream_t s) {
  const uint32_t nblk = part_blocks(n);
  const uint64_t hn = (uint64_t)nblk << p1;
  {
    Scope sc(&t->timing, PMDFC_K_ROUTE, s);
    launch_part_hist(pend, npend_dev, n, n, st, t->hbuf, t->sbits, p1, t->hist, s);
    size_t bytes = t->tmp_bytes;
    HIPCHK(rocprim::inclusive_scan(t->tmp, bytes, t->hist, t->inc, (size_t)hn, rocprim::plus<uint32_t>(), s));
    launch_part_scatter(pend, npend_dev, n, n, st, t->hbuf, t->sbits, p1, bbits, t->hist, t->inc,
                        t->rec, s);
  }
  HIPCHK(hipMemsetAsync(t->pstate, 0, n, s));
  HIPCHK(hipMemsetAsync(t->bwork, 0, (size_t)1 << p1, s));
  HIPCHK(hipMemsetAsync(t->flags, 0, n, s));
  HIPCHK(hipMemsetAsync(&t->ctl->n_split, 0, 3 * sizeof(uint32_t), s));
  HIPCHK(hipMemsetAsync(t->ctl->pass_split, 0, sizeof(t->ctl->pass_split), s));
  for (uint32_t pass = 0; pass < kBucketPasses; ++pass) {
    const bool last = pass + 1 == kBucketPasses;
    uint32_t* q = t->split_list + (size_t)pass * 2 * t->max_batch;
    {
      Scope sc(&t->timing, PMDFC_K_PROCESS, s);
      BucketLaunch L{};
      L.rec = t->rec;
      L.inc = t->inc;
      L.nmax = n;
      L.p1 = p1;
      L.bbits = bbits;
      L.gdepth = t->Dp;
      L.sbits = t->sbits;
      L.pass = pass;
      L.last = last ? 1u : 0u;
      L.ops = ops;
      L.keys = keys;
      L.vin = vin;
      L.vout = vout;
      L.st = st;
      L.pairs = t->pairs;
      L.occ = t->occ;
      L.dir = t->dir;
      L.pstate = t->pstate;
      L.bwork = t->bwork;
      L.hostdef = t->flags;
      L.split_list = q;
      L.ctl = t->ctl;
      L.max_segments = (uint32_t)t->max_segs;
      launch_bucket(L, s);
    }
    if (!last) {
      Scope sc(&t->timing, PMDFC_K_SPLIT, s);
      launch_split_q(q, &t->ctl->pass_split[pass], t->pairs, t->occ, t->ldep, t->dir, t->Dp,
                     t->sbits, t->ctl, 2048, s);
    }
  }
  int rc = sync_ctl(t, s);
  if (rc) return rc;
  t->passes += 1;
  const uint32_t ndef = t->hctl->n_deferred;
  t->deferred_ops += ndef;
  if (ndef == 0) {
    t->batches += 1;
    return PMDFC_OK;
  }
  // left over after the device passes, or waiting for a directory doubling
  if (t->hctl->need_double) {
    rc = double_dir(t, s);
    if (rc) return rc;
  }
  {
    Scope sc(&t->timing, PMDFC_K_SELECT, s);
    size_t bytes = t->tmp_bytes;
    HIPCHK(rocprim::select(t->tmp, bytes, rocprim::counting_iterator<uint32_t>(0), t->flags,
                           t->pend, t->sel_count, (size_t)n, s));
  }
  return run_passes(t, ops, keys, vin, vout, st, n, t->pend, ndef, s);
}

static int pre_batch(pmdfc_cceh* t, uint64_t n, hipStream_t s) {
  if (n > t->max_batch) return fail(PMDFC_ERR_ARG, "n exceeds max_batch");
  // keep one bit of directory headroom so splits rarely need a doubling pass
  if (t->max_ld >= t->Dp && t->Dp < kMaxDepth) return double_dir(t, s);
  return PMDFC_OK;
}

// ------------------------------------------------------------------- C-ABI

extern "C" {

int pmdfc_abi_version(void) { return PMDFC_ABI_VERSION; }
const char* pmdfc_last_error(void) { return g_err.c_str(); }

uint32_t pmdfc_depth_for_hybrid(uint64_t init_cap) {
  return (uint32_t)(size_t)std::log2((double)init_cap);  // CCEH_hybrid.cpp:80
}

uint32_t pmdfc_depth_for_src(uint64_t init_cap) {
  return (uint32_t)(size_t)std::log2((double)(init_cap / kSlots));  // src/cceh.cpp:82
}

int pmdfc_cceh_create(const pmdfc_cceh_config_t* cfg, pmdfc_cceh_t** out) {
  if (!cfg || !out) return fail(PMDFC_ERR_ARG, "null argument");
  *out = nullptr;
  if (cfg->initial_depth < 1 || cfg->initial_depth > kMaxDepth)
    return fail(PMDFC_ERR_ARG, "initial_depth must be in [1, 30] (CCEH(initCap) needs initCap >= 2)");
  if (cfg->shard_bits > cfg->initial_depth || cfg->shard_bits > 16)
    return fail(PMDFC_ERR_ARG, "shard_bits must be <= initial_depth (and <= 16)");
  if (cfg->shard_bits && cfg->shard_id >= (1u << cfg->shard_bits))
    return fail(PMDFC_ERR_ARG, "shard_id out of range");
  if (cfg->max_batch == 0) return fail(PMDFC_ERR_ARG, "max_batch must be > 0");
  DevGuard g(cfg->device);
  auto* t = new pmdfc_cceh();
  t->cfg = *cfg;
  t->dev = cfg->device;
  t->D0 = cfg->initial_depth;
  t->sbits = cfg->shard_bits;
  t->shard = cfg->shard_id;
  t->max_batch = cfg->max_batch;
  const uint64_t n0 = 1ULL << (t->D0 - t->sbits);
  uint64_t ms = cfg->max_segments;
  if (ms == 0) {
    size_t fr = 0, tot = 0;
    (void)hipMemGetInfo(&fr, &tot);
    ms = std::min<uint64_t>((uint64_t)(fr * 0.5) / (kSlots * 16 + 160), 1ULL << 22);
  }
  ms = std::max<uint64_t>(ms, n0 + 1);
  if (ms > kMaxSegments) ms = kMaxSegments;  // 26-bit segment ids in directory entries
  t->max_segs = ms;
  hipError_t e;
#define ALLOC(p, bytes)                                                   \
  do {                                                                    \
    e = hipMalloc(&(p), (bytes));                                         \
    if (e != hipSuccess) {                                                \
      pmdfc_cceh_destroy(t);                                              \
      return fail(PMDFC_ERR_NOMEM, "hipMalloc " #p, e);                   \
    }                                                                     \
  } while (0)
  ALLOC(t->pairs, ms * kSlots * sizeof(ulonglong2));
  ALLOC(t->occ, ms * 32 * sizeof(uint32_t));
  ALLOC(t->ldep, ms);
  ALLOC(t->touched, ms);
  t->dir_cap = std::max<uint64_t>(n0 * 4, 1024);
  ALLOC(t->dir, t->dir_cap * sizeof(uint32_t));
  ALLOC(t->ctl, sizeof(DevCtl));
  const uint64_t B = t->max_batch;
  ALLOC(t->hbuf, B * sizeof(uint64_t));
  ALLOC(t->skey_in, B * sizeof(uint32_t));
  ALLOC(t->skey_out, B * sizeof(uint32_t));
  ALLOC(t->sval_in, B * sizeof(uint32_t));
  ALLOC(t->sval_out, B * sizeof(uint32_t));
  ALLOC(t->pend, B * sizeof(uint32_t));
  ALLOC(t->flags, B);
  ALLOC(t->split_list, 2 * B * kBucketPasses * sizeof(uint32_t));
  ALLOC(t->partials, (B / 64 + 2) * sizeof(uint32_t));
  ALLOC(t->sel_count, sizeof(uint32_t) * 2);
  ALLOC(t->popc, sizeof(unsigned long long));
  ALLOC(t->rec, B * sizeof(uint64_t));
  ALLOC(t->pstate, B);
  ALLOC(t->bwork, 4096);
  t->hist_cap = (uint64_t)part_blocks(B) << 12;
  ALLOC(t->hist, t->hist_cap * sizeof(uint32_t));
  ALLOC(t->inc, t->hist_cap * sizeof(uint32_t));
  e = hipHostMalloc(&t->hctl, sizeof(DevCtl), hipHostMallocDefault);
  if (e != hipSuccess) {
    pmdfc_cceh_destroy(t);
    return fail(PMDFC_ERR_NOMEM, "hipHostMalloc", e);
  }
  // temp storage: max of radix sort and select at max_batch
  size_t b1 = 0, b2 = 0;
  (void)rocprim::radix_sort_pairs(nullptr, b1, t->skey_in, t->skey_out, t->sval_in, t->sval_out,
                            (size_t)B, 0u, 32u, (hipStream_t)0);
  (void)rocprim::select(nullptr, b2, rocprim::counting_iterator<uint32_t>(0), t->flags, t->pend,
                  t->sel_count, (size_t)B, (hipStream_t)0);
  size_t b3 = 0;
  (void)rocprim::inclusive_scan(nullptr, b3, t->hist, t->inc, (size_t)t->hist_cap,
                                rocprim::plus<uint32_t>(), (hipStream_t)0);
  t->tmp_bytes = std::max(std::max(b1, b2), b3) + 256;
  ALLOC(t->tmp, t->tmp_bytes);
#undef ALLOC
  if (const char* e = getenv("PMDFC_GENERIC_PATH")) t->use_bucket = e[0] == '0';
  int rc = init_state(t, (hipStream_t)0);
  if (rc) {
    pmdfc_cceh_destroy(t);
    return rc;
  }
  *out = t;
  return PMDFC_OK;
}

int pmdfc_cceh_destroy(pmdfc_cceh_t* t) {
  if (!t) return PMDFC_OK;
  DevGuard g(t->dev);
  (void)hipDeviceSynchronize();
  t->timing.flush();
  void* ptrs[] = {t->pairs, t->occ, t->ldep, t->touched, t->dir, t->dir_alt, t->ctl, t->hbuf,
                  t->skey_in, t->skey_out, t->sval_in, t->sval_out, t->pend, t->flags,
                  t->split_list, t->partials, t->sel_count, t->popc, t->tmp, t->rec, t->pstate,
                  t->bwork, t->hist, t->inc};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  if (t->hctl) (void)hipHostFree(t->hctl);
  delete t;
  return PMDFC_OK;
}

int pmdfc_cceh_reset(pmdfc_cceh_t* t, void* stream) {
  if (!t) return fail(PMDFC_ERR_ARG, "null engine");
  std::lock_guard<std::mutex> lk(t->mu);
  DevGuard g(t->dev);
  return init_state(t, (hipStream_t)stream);
}

int pmdfc_cceh_get(pmdfc_cceh_t* t, const uint64_t* keys, uint64_t* vout, uint8_t* st, uint64_t n,
                   void* stream) {
  if (!t || (n && (!keys || !vout || !st))) return fail(PMDFC_ERR_ARG, "null argument");
  if (n == 0) return PMDFC_OK;
  std::lock_guard<std::mutex> lk(t->mu);
  DevGuard g(t->dev);
  hipStream_t s = (hipStream_t)stream;
  const bool count = t->count_lines && n <= t->max_batch;
  {
    Scope sc(&t->timing, PMDFC_K_GET, s);
    launch_get(count, keys, vout, st, n, t->geo(), t->pairs, t->partials, s);
  }
  t->last_get_n = n;
  t->last_get_counted = count;
  {
    const char* e = getenv("PMDFC_GET_UNROLL");
    int U = e ? atoi(e) : 2;
    if (U != 1 && U != 2 && U != 4) U = 2;
    t->last_get_blocks = ((n + U - 1) / U + 63) / 64;
  }
  HIPCHK(hipGetLastError());
  return PMDFC_OK;
}

int pmdfc_cceh_insert(pmdfc_cceh_t* t, const uint64_t* keys, const uint64_t* vin, uint8_t* st,
                      uint64_t n, void* stream) {
  if (!t || (n && (!keys || !vin || !st))) return fail(PMDFC_ERR_ARG, "null argument");
  if (n == 0) return PMDFC_OK;
  std::lock_guard<std::mutex> lk(t->mu);
  DevGuard g(t->dev);
  hipStream_t s = (hipStream_t)stream;
  int rc = pre_batch(t, n, s);
  if (rc) return rc;
  {
    Scope sc(&t->timing, PMDFC_K_PREP, s);
    launch_prep(keys, t->hbuf, st, nullptr, n, t->sbits, t->shard, s);
  }
  uint32_t p1, bbits;
  if (t->use_bucket && choose_p1(t, n, &p1, &bbits) == 0)
    rc = run_bucket(t, nullptr, keys, vin, nullptr, st, n, nullptr, nullptr, p1, bbits, s);
  else
    rc = run_passes(t, nullptr, keys, vin, nullptr, st, n, nullptr, n, s);
  if (rc) return rc;
  HIPCHK(hipGetLastError());
  return PMDFC_OK;
}

int pmdfc_cceh_mixed(pmdfc_cceh_t* t, const uint8_t* ops, const uint64_t* keys, const uint64_t* vin,
                     uint64_t* vout, uint8_t* st, uint64_t n, void* stream) {
  if (!t || (n && (!ops || !keys || !vin || !vout || !st))) return fail(PMDFC_ERR_ARG, "null argument");
  if (n == 0) return PMDFC_OK;
  std::lock_guard<std::mutex> lk(t->mu);
  DevGuard g(t->dev);
  hipStream_t s = (hipStream_t)stream;
  int rc = pre_batch(t, n, s);
  if (rc) return rc;
  {
    Scope sc(&t->timing, PMDFC_K_PREP, s);
    launch_prep(keys, t->hbuf, st, vout, n, t->sbits, t->shard, s);
    HIPCHK(hipMemsetAsync(t->touched, 0, t->nsegs, s));
    launch_mark(ops, t->hbuf, st, n, t->geo(), t->touched, s);
  }
  {
    Scope sc(&t->timing, PMDFC_K_MIXED_GET, s);
    launch_mixed_get(ops, keys, t->hbuf, st, vout, n, t->geo(), t->pairs, t->touched, t->flags, s);
  }
  {
    Scope sc(&t->timing, PMDFC_K_SELECT, s);
    size_t bytes = t->tmp_bytes;
    HIPCHK(rocprim::select(t->tmp, bytes, rocprim::counting_iterator<uint32_t>(0), t->flags,
                           t->pend, t->sel_count, (size_t)n, s));
  }
  uint32_t p1, bbits;
  if (t->use_bucket && choose_p1(t, n, &p1, &bbits) == 0) {
    rc = run_bucket(t, ops, keys, vin, vout, st, n, t->pend, t->sel_count, p1, bbits, s);
  } else {
    HIPCHK(hipMemcpyAsync(&t->hctl->npend, t->sel_count, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    rc = run_passes(t, ops, keys, vin, vout, st, n, t->pend, t->hctl->npend, s);
  }
  if (rc) return rc;
  HIPCHK(hipGetLastError());
  return PMDFC_OK;
}

int pmdfc_cceh_mixed_host(pmdfc_cceh_t* t, const uint8_t* ops, const uint64_t* keys,
                          const uint64_t* vin, uint64_t* vout, uint8_t* st, uint64_t n) {
  if (!t) return fail(PMDFC_ERR_ARG, "null engine");
  DevGuard g(t->dev);
  for (uint64_t off = 0; off < n; off += t->max_batch) {
    const uint64_t m = std::min<uint64_t>(t->max_batch, n - off);
    uint8_t *d_ops = nullptr, *d_st = nullptr;
    uint64_t *d_keys = nullptr, *d_vin = nullptr, *d_vout = nullptr;
    HIPCHK(hipMalloc(&d_ops, m));
    HIPCHK(hipMalloc(&d_st, m));
    HIPCHK(hipMalloc(&d_keys, m * 8));
    HIPCHK(hipMalloc(&d_vin, m * 8));
    HIPCHK(hipMalloc(&d_vout, m * 8));
    HIPCHK(hipMemcpy(d_ops, ops + off, m, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(d_keys, keys + off, m * 8, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(d_vin, vin + off, m * 8, hipMemcpyHostToDevice));
    int rc = pmdfc_cceh_mixed(t, d_ops, d_keys, d_vin, d_vout, d_st, m, nullptr);
    if (rc == PMDFC_OK) {
      HIPCHK(hipMemcpy(vout + off, d_vout, m * 8, hipMemcpyDeviceToHost));
      HIPCHK(hipMemcpy(st + off, d_st, m, hipMemcpyDeviceToHost));
    }
    (void)hipFree(d_ops);
    (void)hipFree(d_st);
    (void)hipFree(d_keys);
    (void)hipFree(d_vin);
    (void)hipFree(d_vout);
    if (rc) return rc;
  }
  return PMDFC_OK;
}

int pmdfc_cceh_stats(pmdfc_cceh_t* t, pmdfc_cceh_stats_t* out) {
  if (!t || !out) return fail(PMDFC_ERR_ARG, "null argument");
  std::lock_guard<std::mutex> lk(t->mu);
  DevGuard g(t->dev);
  HIPCHK(hipDeviceSynchronize());
  int rc = sync_ctl(t, (hipStream_t)0);
  if (rc) return rc;
  out->depth = std::max(t->D0, t->max_ld);
  out->phys_depth = t->Dp;
  out->segments = t->nsegs;
  out->capacity = (uint64_t)t->nsegs * kSlots;
  out->max_segments = t->max_segs;
  out->splits = t->splits;
  out->doublings = t->doublings;
  out->split_loss = t->split_loss;
  out->insert_passes = t->passes;
  out->batches = t->batches;
  out->segment_runs = t->hctl->runs;
  out->deferred_ops = t->deferred_ops;
  return PMDFC_OK;
}

int pmdfc_cceh_utilization(pmdfc_cceh_t* t, double* out) {
  if (!t || !out) return fail(PMDFC_ERR_ARG, "null argument");
  std::lock_guard<std::mutex> lk(t->mu);
  DevGuard g(t->dev);
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemset(t->popc, 0, sizeof(unsigned long long)));
  launch_popcount(t->occ, (uint64_t)t->nsegs * 32, t->popc, (hipStream_t)0);
  unsigned long long c = 0;
  HIPCHK(hipMemcpy(&c, t->popc, sizeof c, hipMemcpyDeviceToHost));
  *out = (double)c / ((double)t->nsegs * kSlots) * 100.0;
  return PMDFC_OK;
}

int pmdfc_cceh_dump(pmdfc_cceh_t* t, uint32_t* dir_canon, uint32_t* local_depth, uint64_t* prefix,
                    uint64_t* keys, uint64_t* values, uint64_t* nseg_out) {
  if (!t) return fail(PMDFC_ERR_ARG, "null engine");
  std::lock_guard<std::mutex> lk(t->mu);
  DevGuard g(t->dev);
  HIPCHK(hipDeviceSynchronize());
  int rc = sync_ctl(t, (hipStream_t)0);
  if (rc) return rc;
  const uint32_t D = std::max(t->D0, t->max_ld);  // logical global depth
  const uint64_t nlog = 1ULL << (D - t->sbits);
  const uint32_t shift = t->Dp - D;
  std::vector<uint32_t> pdir(t->dir_entries());
  HIPCHK(hipMemcpy(pdir.data(), t->dir, pdir.size() * 4, hipMemcpyDeviceToHost));
  std::vector<uint8_t> ld(t->nsegs);
  HIPCHK(hipMemcpy(ld.data(), t->ldep, t->nsegs, hipMemcpyDeviceToHost));
  std::vector<uint32_t> order;
  uint32_t cur = 0;
  for (uint64_t x = 0; x < nlog; ++x) {
    const uint32_t sid = de_seg(pdir[x << shift]);
    const uint32_t L = ld[sid];
    const uint32_t Ll = L - t->sbits;
    const uint32_t Dl = D - t->sbits;
    if ((x & ((1ULL << (Dl - Ll)) - 1)) == 0) {
      cur = (uint32_t)order.size();
      order.push_back(sid);
      if (local_depth) local_depth[cur] = L;
      if (prefix) prefix[cur] = ((uint64_t)t->shard << Ll) | (x >> (Dl - Ll));
    }
    if (dir_canon) dir_canon[x] = cur;
  }
  if (nseg_out) *nseg_out = order.size();
  if (keys || values) {
    std::vector<ulonglong2> buf(kSlots);
    for (size_t i = 0; i < order.size(); ++i) {
      HIPCHK(hipMemcpy(buf.data(), t->pairs + (size_t)order[i] * kSlots, kSlots * 16,
                       hipMemcpyDeviceToHost));
      for (uint32_t j = 0; j < kSlots; ++j) {
        if (keys) keys[i * kSlots + j] = buf[j].x;
        if (values) values[i * kSlots + j] = buf[j].x == kInvalid ? 0 : buf[j].y;
      }
    }
  }
  return PMDFC_OK;
}

int pmdfc_cceh_timing_enable(pmdfc_cceh_t* t, int on) {
  if (!t) return fail(PMDFC_ERR_ARG, "null engine");
  std::lock_guard<std::mutex> lk(t->mu);
  t->timing.on = (on & 1) != 0;
  t->count_lines = (on & 2) != 0;
  return PMDFC_OK;
}

int pmdfc_cceh_timing_read(pmdfc_cceh_t* t, double* ms_out, uint64_t* launches_out, int reset) {
  if (!t) return fail(PMDFC_ERR_ARG, "null engine");
  std::lock_guard<std::mutex> lk(t->mu);
  DevGuard g(t->dev);
  t->timing.flush();
  for (int i = 0; i < PMDFC_K_COUNT; ++i) {
    if (ms_out) ms_out[i] = t->timing.ms[i];
    if (launches_out) launches_out[i] = t->timing.launches[i];
    if (reset) {
      t->timing.ms[i] = 0;
      t->timing.launches[i] = 0;
    }
  }
  return PMDFC_OK;
}

int pmdfc_cceh_last_get_lines(pmdfc_cceh_t* t, uint64_t* lines) {
  if (!t || !lines) return fail(PMDFC_ERR_ARG, "null argument");
  std::lock_guard<std::mutex> lk(t->mu);
  if (!t->last_get_counted) return fail(PMDFC_ERR_STATE, "last get was not counted (enable timing)");
  DevGuard g(t->dev);
  HIPCHK(hipDeviceSynchronize());
  const uint64_t nb = t->last_get_blocks;
  std::vector<uint32_t> p(nb);
  HIPCHK(hipMemcpy(p.data(), t->partials, nb * 4, hipMemcpyDeviceToHost));
  uint64_t sum = 0;
  for (auto v : p) sum += v;
  *lines = sum;
  return PMDFC_OK;
}

int pmdfc_hash64(const uint64_t* keys, uint64_t* out, uint64_t n, void* stream) {
  if (n && (!keys || !out)) return fail(PMDFC_ERR_ARG, "null argument");
  launch_hash(keys, out, n, (hipStream_t)stream);
  HIPCHK(hipGetLastError());
  return PMDFC_OK;
}

int pmdfc_gen_keys(uint64_t seed, uint64_t start, uint64_t* out, uint64_t n, void* stream) {
  if (n && !out) return fail(PMDFC_ERR_ARG, "null argument");
  launch_gen_keys(seed, start, out, n, (hipStream_t)stream);
  HIPCHK(hipGetLastError());
  return PMDFC_OK;
}

int pmdfc_route_by_shard(const uint64_t* keys, uint64_t n, uint32_t shard_bits, uint32_t* perm,
                         uint64_t* h_counts, int device, void* stream) {
  if (shard_bits > 16 || (n && (!keys || !perm || !h_counts))) return fail(PMDFC_ERR_ARG, "bad argument");
  DevGuard g(device);
  hipStream_t s = (hipStream_t)stream;
  const uint32_t G = 1u << shard_bits;
  if (n == 0) {
    for (uint32_t i = 0; i < G; ++i) h_counts[i] = 0;
    return PMDFC_OK;
  }
  uint32_t *own = nullptr, *own2 = nullptr, *idx = nullptr;
  uint64_t* starts = nullptr;
  void* tmp = nullptr;
  size_t bytes = 0;
  HIPCHK(hipMallocAsync((void**)&own, n * 4, s));
  HIPCHK(hipMallocAsync((void**)&own2, n * 4, s));
  HIPCHK(hipMallocAsync((void**)&idx, n * 4, s));
  HIPCHK(hipMallocAsync((void**)&starts, (G + 1) * 8, s));
  if (shard_bits == 0) {
    launch_owner(keys, n, 0, own, perm, s);  // own unused
    h_counts[0] = n;
  } else {
    launch_owner(keys, n, shard_bits, own, idx, s);
    HIPCHK(rocprim::radix_sort_pairs(nullptr, bytes, own, own2, idx, perm, (size_t)n, 0u, shard_bits, s));
    HIPCHK(hipMallocAsync(&tmp, bytes + 16, s));
    HIPCHK(rocprim::radix_sort_pairs(tmp, bytes, own, own2, idx, perm, (size_t)n, 0u, shard_bits, s));
    launch_bounds(own2, n, G, starts, s);
    std::vector<uint64_t> st(G + 1);
    HIPCHK(hipMemcpyAsync(st.data(), starts, (G + 1) * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    for (uint32_t i = 0; i < G; ++i) h_counts[i] = st[i + 1] - st[i];
    HIPCHK(hipFreeAsync(tmp, s));
  }
  HIPCHK(hipFreeAsync(own, s));
  HIPCHK(hipFreeAsync(own2, s));
  HIPCHK(hipFreeAsync(idx, s));
  HIPCHK(hipFreeAsync(starts, s));
  HIPCHK(hipStreamSynchronize(s));
  return PMDFC_OK;
}

int pmdfc_ubench_gather64(const void* buf, uint64_t nlines, const uint32_t* table, uint32_t tmask,
                          uint64_t n_ops, uint64_t seed, uint64_t* out, void* stream) {
  if (!buf || !out || nlines == 0) return fail(PMDFC_ERR_ARG, "bad argument");
  launch_gather64(buf, nlines, table, tmask, n_ops, seed, out, (hipStream_t)stream);
  HIPCHK(hipGetLastError());
  return PMDFC_OK;
}

// ------------------------------------------------------------------- bloom

int pmdfc_bloom_create(uint64_t nbits, uint32_t k, int device, pmdfc_bloom_t** out) {
  if (!out || nbits == 0 || k == 0 || k > 64 || nbits >= (1ULL << 32))
    return fail(PMDFC_ERR_ARG, "bloom: need 0 < nbits < 2^32 (unsigned int index, bloom_filter.c:87) and 0 < k <= 64");
  DevGuard g(device);
  auto* b = new pmdfc_bloom();
  b->dev = device;
  b->nbits = nbits;
  b->nwords = (nbits + 63) / 64;
  b->k = k;
  hipError_t e = hipMalloc(&b->bm, b->nwords * 8);
  if (e != hipSuccess) {
    delete b;
    return fail(PMDFC_ERR_NOMEM, "bloom hipMalloc", e);
  }
  e = hipMemset(b->bm, 0, b->nwords * 8);
  if (e != hipSuccess) {
    (void)hipFree(b->bm);
    delete b;
    return fail(PMDFC_ERR_HIP, "bloom memset", e);
  }
  *out = b;
  return PMDFC_OK;
}

int pmdfc_bloom_destroy(pmdfc_bloom_t* b) {
  if (!b) return PMDFC_OK;
  DevGuard g(b->dev);
  (void)hipDeviceSynchronize();
  (void)hipFree(b->bm);
  delete b;
  return PMDFC_OK;
}

int pmdfc_bloom_clear(pmdfc_bloom_t* b, void* stream) {
  if (!b) return fail(PMDFC_ERR_ARG, "null bloom");
  DevGuard g(b->dev);
  HIPCHK(hipMemsetAsync(b->bm, 0, b->nwords * 8, (hipStream_t)stream));
  return PMDFC_OK;
}

int pmdfc_bloom_add(pmdfc_bloom_t* b, const uint64_t* keys, uint64_t n, void* stream) {
  if (!b || (n && !keys)) return fail(PMDFC_ERR_ARG, "null argument");
  DevGuard g(b->dev);
  launch_bloom_add(b->bm, b->nbits, b->k, keys, n, (hipStream_t)stream);
  HIPCHK(hipGetLastError());
  return PMDFC_OK;
}

int pmdfc_bloom_probe(pmdfc_bloom_t* b, const uint64_t* keys, uint8_t* out, uint64_t n, void* stream) {
  if (!b || (n && (!keys || !out))) return fail(PMDFC_ERR_ARG, "null argument");
  DevGuard g(b->dev);
  launch_bloom_probe(b->bm, b->nbits, b->k, keys, out, n, (hipStream_t)stream);
  HIPCHK(hipGetLastError());
  return PMDFC_OK;
}

int pmdfc_bloom_bitmap(pmdfc_bloom_t* b, uint64_t** d_bitmap, uint64_t* nwords) {
  if (!b || !d_bitmap || !nwords) return fail(PMDFC_ERR_ARG, "null argument");
  *d_bitmap = b->bm;
  *nwords = b->nwords;
  return PMDFC_OK;
}

int pmdfc_bloom_set_bitmap_host(pmdfc_bloom_t* b, const uint64_t* host, uint64_t nwords) {
  if (!b || !host || nwords != b->nwords) return fail(PMDFC_ERR_ARG, "bitmap size mismatch");
  DevGuard g(b->dev);
  HIPCHK(hipMemcpy(b->bm, host, nwords * 8, hipMemcpyHostToDevice));
  return PMDFC_OK;
}

int pmdfc_bloom_get_bitmap_host(pmdfc_bloom_t* b, uint64_t* host, uint64_t nwords) {
  if (!b || !host || nwords != b->nwords) return fail(PMDFC_ERR_ARG, "bitmap size mismatch");
  DevGuard g(b->dev);
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(host, b->bm, nwords * 8, hipMemcpyDeviceToHost));
  return PMDFC_OK;
}

int pmdfc_bloom_probe_then_get(pmdfc_bloom_t* b, pmdfc_cceh_t* t, const uint64_t* keys,
                               uint64_t* vout, uint8_t* st, uint64_t n, void* stream) {
  if (!b || !t || (n && (!keys || !vout || !st))) return fail(PMDFC_ERR_ARG, "null argument");
  if (b->dev != t->dev) return fail(PMDFC_ERR_ARG, "bloom and index on different devices");
  std::lock_guard<std::mutex> lk(t->mu);
  DevGuard g(t->dev);
  hipStream_t s = (hipStream_t)stream;
  {
    Scope sc(&t->timing, PMDFC_K_BLOOM, s);
    launch_bloom_get(b->bm, b->nbits, b->k, keys, vout, st, n, t->geo(), t->pairs, s);
  }
  HIPCHK(hipGetLastError());
  return PMDFC_OK;
}

}  // extern "C"
