// batch_core.cpp -- the served per-op front-end over the C-ABI (batch_core.h).
#include "batch_core.h"

#include <hip/hip_runtime_api.h>
#include <immintrin.h>
#include <linux/futex.h>
#include <sched.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <thread>

namespace pmdfc_host {

#define CHK(x)                                                                                \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) throw std::runtime_error(std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

static void abi(int rc, const char* what) {
  if (rc != PMDFC_OK) throw std::runtime_error(std::string(what) + ": " + pmdfc_last_error());
}

static inline void cpu_relax() { __builtin_ia32_pause(); }

static void futex_wait(std::atomic<uint32_t>* w, uint32_t expect, long ns) {
  timespec ts{0, ns};
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), FUTEX_WAIT_PRIVATE, expect, &ts, nullptr, 0);
}
static void futex_wake(std::atomic<uint32_t>* w, int n) {
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), FUTEX_WAKE_PRIVATE, n, nullptr, nullptr, 0);
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static const char* status_name(uint8_t s) {
  switch (s) {
    case PMDFC_ST_RESERVED_KEY: return "RESERVED_KEY";
    case PMDFC_ST_UNSPLITTABLE: return "UNSPLITTABLE";
    case PMDFC_ST_DEPTH_LIMIT: return "DEPTH_LIMIT";
    case PMDFC_ST_CAPACITY: return "CAPACITY";
    case PMDFC_ST_WRONG_SHARD: return "WRONG_SHARD";
    case PMDFC_ST_SPLIT_LOST: return "SPLIT_LOST";
    case kBatchFailed: return "BATCH_FAILED";
    default: return "unexpected";
  }
}

bool BatchCore::is_failure(uint8_t op, uint8_t s) {
  if (op == PMDFC_OP_INSERT) return s != PMDFC_ST_INSERTED && s != PMDFC_ST_UPDATED;
  return s != PMDFC_ST_HIT && s != PMDFC_ST_MISS;
}

// the ring words shared with the device: coherent pinned memory, accessed
// with atomics (the device reads and writes them at system scope)
template <class T>
static inline T ld_acq(const T* p) {
  return __atomic_load_n(p, __ATOMIC_ACQUIRE);
}
template <class T>
static inline void st_rel(T* p, T v) {
  __atomic_store_n(p, v, __ATOMIC_RELEASE);
}

// h() = std::_Hash_bytes(&key, 8, 0xc70697) (server/util/hash.h:252), the
// hash the engine indexes with: a ring owns the ops of its hash prefix
static inline uint64_t key_hash(uint64_t key) {
  const uint64_t mul = 0xc6a4a7935bd1e995ULL;
  uint64_t h = 0xc70697ULL ^ (8ULL * mul);
  uint64_t d = key * mul;
  d = (d ^ (d >> 47)) * mul;
  h ^= d;
  h *= mul;
  h = (h ^ (h >> 47)) * mul;
  return h ^ (h >> 47);
}

BatchCore::BatchCore(uint32_t initial_depth, BatchingConfig cfg, uint64_t max_segments) : cfg_(cfg) {
  for (auto& c : fail_by_st_) c.store(0);
  try {
    init(initial_depth, max_segments);
  } catch (...) {
    release();  // the destructor never runs for a constructor that throws
    throw;
  }
}

void BatchCore::init(uint32_t initial_depth, uint64_t max_segments) {
  const BatchingConfig cfg = cfg_;
  pmdfc_cceh_config_t c{};
  c.initial_depth = initial_depth;
  c.max_batch = std::max<uint32_t>(cfg.max_batch, 64);
  c.max_segments = max_segments;
  c.device = cfg.device;
  c.flags = cfg.upsert ? PMDFC_CFG_UPSERT : 0u;
  CHK(hipSetDevice(cfg.device));
  abi(pmdfc_cceh_create(&c, &t_), "pmdfc_cceh_create");
  R_ = 256;
  while (R_ < cfg.ring_size) R_ <<= 1;
  mask_ = R_ - 1;
  // rings: a power of two, at most the directory buckets the table starts
  // with (a ring owns whole buckets; buckets only get finer)
  const uint32_t wmax = std::max<uint32_t>(pmdfc_cceh_serve_waves_max(t_), 1u);
  W_ = 1;
  while (W_ * 2 <= std::min<uint32_t>(std::max<uint32_t>(cfg.serve_waves, 1u), wmax)) W_ *= 2;
  lw_ = 0;
  while ((1u << lw_) < W_) ++lw_;
  hipStream_t st;
  CHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  stream_ = st;
  CHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  sync_ = st;
  const unsigned fl = hipHostMallocCoherent | hipHostMallocMapped;
  CHK(hipHostMalloc((void**)&req_, W_ * R_ * sizeof(pmdfc_serve_req), fl));
  CHK(hipHostMalloc((void**)&resp_, W_ * R_ * sizeof(pmdfc_serve_resp), fl));
  CHK(hipHostMalloc((void**)&ctl_, W_ * sizeof(pmdfc_serve_ctl), fl));
  memset(req_, 0, W_ * R_ * sizeof(pmdfc_serve_req));
  memset(resp_, 0, W_ * R_ * sizeof(pmdfc_serve_resp));
  memset(ctl_, 0, W_ * sizeof(pmdfc_serve_ctl));
  for (uint32_t g = 0; g < W_; ++g) {
    std::unique_ptr<Ring> q(new Ring);
    q->req = req_ + (size_t)g * R_;
    q->resp = resp_ + (size_t)g * R_;
    q->ctl = ctl_ + g;
    q->read.reset(new std::atomic<uint64_t>[R_]);
    q->asleep.reset(new std::atomic<uint8_t>[R_]);
    for (uint64_t i = 0; i < R_; ++i) {
      q->read[i].store(0, std::memory_order_relaxed);
      q->asleep[i].store(0, std::memory_order_relaxed);
    }
    q->async.assign(R_, Async{nullptr, nullptr, 0, 0, 0.0});
    rings_.push_back(std::move(q));
  }
  CHK(hipMalloc((void**)&fa_dev_, 32));
  if (const char* e = getenv("PMDFC_FLOOD_OPS")) cfg_.flood_ops = (uint32_t)atoi(e);  // (tests, A/B)
  fl_cap_ = std::min<uint64_t>(c.max_batch, R_ / 2);
  if (cfg_.flood_ops && fl_cap_ >= 256) {
    CHK(hipHostMalloc((void**)&fl_h_in_, fl_cap_ * 18, hipHostMallocDefault));
    CHK(hipHostMalloc((void**)&fl_h_out_, fl_cap_ * 9, hipHostMallocDefault));
    CHK(hipMalloc((void**)&fl_d_in_, fl_cap_ * 18));
    CHK(hipMalloc((void**)&fl_d_out_, fl_cap_ * 9));
  } else {
    cfg_.flood_ops = 0;
  }
  if (const char* e = getenv("PMDFC_DELIVERY_THREADS")) cfg_.delivery_threads = (uint32_t)atoi(e);  // (tests, A/B)
  D_ = std::max<uint32_t>(1u, std::min<uint32_t>(cfg_.delivery_threads, W_));
  ctl_th_ = std::thread(&BatchCore::control, this);
  for (uint32_t d = 1; d < D_; ++d) dl_th_.emplace_back(&BatchCore::deliver, this, d);
}

uint32_t BatchCore::ring_of(uint64_t key) const {
  return W_ == 1 ? 0u : (uint32_t)(key_hash(key) >> (64 - lw_));
}

uint64_t BatchCore::ops_completed() const {
  uint64_t n = 0;
  for (const auto& q : rings_) n += q->reclaim.load();
  return n;
}

BatchCore::~BatchCore() {
  // every queued op completes first (the callers are gone; callbacks run)
  if (!on_control()) {
    const double t0 = now_us();
    for (auto& q : rings_) {
      const uint64_t target = q->tail.load();
      while (q->reclaim.load() < target && now_us() - t0 < 30e6) std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
  }
  stop_.store(true);
  if (ctl_th_.joinable()) ctl_th_.join();
  for (auto& th : dl_th_)
    if (th.joinable()) th.join();
  {
    std::lock_guard<std::mutex> lk(srv_mu_);
    stop_server();
  }
  release();
}

// frees what the constructor allocated (also after a constructor that threw
// part-way: every member is null until its allocation succeeded)
void BatchCore::release() {
  if (stream_) (void)hipStreamSynchronize((hipStream_t)stream_);
  if (sync_) (void)hipStreamSynchronize((hipStream_t)sync_);
  if (fa_dev_) (void)hipFree(fa_dev_);
  if (fl_h_in_) (void)hipHostFree(fl_h_in_);
  if (fl_h_out_) (void)hipHostFree(fl_h_out_);
  if (fl_d_in_) (void)hipFree(fl_d_in_);
  if (fl_d_out_) (void)hipFree(fl_d_out_);
  if (req_) (void)hipHostFree(req_);
  if (resp_) (void)hipHostFree(resp_);
  if (ctl_) (void)hipHostFree(ctl_);
  if (stream_) (void)hipStreamDestroy((hipStream_t)stream_);
  if (sync_) (void)hipStreamDestroy((hipStream_t)sync_);
  if (t_) pmdfc_cceh_destroy(t_);
  fa_dev_ = nullptr, fl_h_in_ = fl_h_out_ = fl_d_in_ = fl_d_out_ = nullptr;
  req_ = nullptr, resp_ = nullptr, ctl_ = nullptr, stream_ = sync_ = nullptr, t_ = nullptr;
}

void BatchCore::set_error(const std::string& e) {
  std::lock_guard<std::mutex> lk(err_mu_);
  err_ = e;
}

std::string BatchCore::last_error() const {
  std::lock_guard<std::mutex> lk(err_mu_);
  return err_;
}

uint64_t BatchCore::batches_launched() const {
  uint64_t n = chunks_base_.load() + fl_batches_.load();
  for (uint32_t g = 0; g < W_; ++g) n += ld_acq(&ctl_[g].chunks);
  return n;
}

BatchCore::PhaseTimes BatchCore::phase_times() const {
  PhaseTimes p;
  p.batches = batches_launched();
  uint64_t ops = ph_ops_.load(), qns = ph_queue_ns_.load(), gns = ph_gpu_ns_.load(), dns = ph_deliver_ns_.load();
  for (const auto& q : rings_) {
    ops += q->ph_ops.load();
    qns += q->queue_ns.load();
    gns += q->ph_gpu_ns.load();
    dns += q->ph_deliver_ns.load();
  }
  p.ops = ops;
  p.queue_us = qns * 1e-3;
  p.gpu_us = gns * 1e-3;
  p.deliver_us = dns * 1e-3;
  uint64_t d[6];
  for (int i = 0; i < 6; ++i) {
    d[i] = prof_base_[i].load();
    for (uint32_t g = 0; g < W_; ++g) d[i] += ld_acq(&ctl_[g].prof[i]);
  }
  p.dev_read_us = d[0] * 1e-2;  // (100 MHz ticks, summed over the waves)
  p.dev_cbf_us = d[1] * 1e-2;
  p.dev_apply_us = d[2] * 1e-2;
  p.dev_answer_us = d[3] * 1e-2;
  p.dev_empty_polls = d[4];
  p.dev_life_us = d[5] * 1e-2;
  p.wave_starts = starts_.load();
  p.flood_batches = fl_batches_.load();
  p.flood_ops = fl_ops_.load();
  p.flood_us = fl_ns_.load() * 1e-3;
  p.stop_us = stop_ns_.load() * 1e-3;
  return p;
}

// ------------------------------------------------------------ the device waves

// (srv_mu_ held)  Each wave serves from the place after the last one any wave
// of its ring answered (ctl->head, exact while stopped); they exit only when
// stopped (or when the heartbeat stops).
bool BatchCore::start_server() {
  if (running_) return true;
  for (uint32_t g = 0; g < W_; ++g) {
    st_rel(&ctl_[g].stop, 0u);
    st_rel(&ctl_[g].idle, 0u);
    st_rel(&ctl_[g].alive, 1u);
  }
  const int rc = W_ == 1 ? pmdfc_cceh_serve_start(t_, req_, resp_, ctl_, R_, ld_acq(&ctl_->head), bf_, stream_)
                         : pmdfc_cceh_serve_start_n(t_, W_, req_, resp_, ctl_, R_, bf_, stream_);
  if (rc != PMDFC_OK) {
    for (uint32_t g = 0; g < W_; ++g) st_rel(&ctl_[g].alive, 0u);
    set_error(std::string("pmdfc_cceh_serve_start: ") + pmdfc_last_error());
    return false;
  }
  running_ = true;
  starts_.fetch_add(1);
  return true;
}

// (srv_mu_ held)
bool BatchCore::stop_server() {
  if (!running_) return true;
  const double t_stop = now_us();
  for (uint32_t g = 0; g < W_; ++g) st_rel(&ctl_[g].stop, 1u);
  const double t0 = now_us();
  for (uint32_t g = 0; g < W_; ++g) {
    for (uint32_t spin = 0; ld_acq(&ctl_[g].alive) != 0; ++spin) {
      if (now_us() - t0 > 10e6) {
        set_error("BatchCore: the serving waves did not stop within 10 s");
        return false;
      }
      // (they stop within a chunk: spin first -- a sleeping thread of a
      // CPU-quota'd process may wake a scheduling period later)
      if (spin < 4096) cpu_relax();
      else std::this_thread::sleep_for(std::chrono::microseconds(5));
    }
  }
  (void)hipStreamSynchronize((hipStream_t)stream_);
  for (uint32_t g = 0; g < W_; ++g) {
    pmdfc_serve_ctl* c = ctl_ + g;
    chunks_base_.fetch_add(ld_acq(&c->chunks));
    st_rel(&c->chunks, (uint64_t)0);
    reloads_base_.fetch_add(ld_acq(&c->reloads));
    st_rel(&c->reloads, (uint64_t)0);
    for (int i = 0; i < 6; ++i) {
      prof_base_[i].fetch_add(ld_acq(&c->prof[i]));
      st_rel(&c->prof[i], (uint64_t)0);
    }
  }
  running_ = false;
  stop_ns_.fetch_add((uint64_t)((now_us() - t_stop) * 1e3));
  return true;
}

// A flood: the published prefix of ring g's unanswered places (up to
// fl_cap_) as ONE engine batch -- the same serial order its wave would
// apply -- on the synchronous stream; the answers go into the response ring
// as the wave would write them, and head moves past them.  The requests'
// halves are read with 16-B loads (atomic, as the callers' stores).
bool BatchCore::serve_flood(uint32_t g) {
  Ring& q = *rings_[g];
  pmdfc_serve_ctl* ctl = q.ctl;
  const double t_fl = now_us();
  const uint64_t head = ld_acq(&ctl->head);
  const uint64_t lim = std::min<uint64_t>(q.tail.load(std::memory_order_acquire) - head, fl_cap_);
  const uint64_t lo = std::max<uint64_t>(cfg_.flood_ops / W_, 256) / 4;
  if (lim < lo) return false;
  uint64_t* keys = reinterpret_cast<uint64_t*>(fl_h_in_);
  uint64_t* vals = keys + lim;
  uint64_t n = 0;
  bool any_ins = false, any_get = false, any_cbf = false;
  for (; n < lim; ++n) {
    const uint64_t p = head + n;
    const __m128i* e = reinterpret_cast<const __m128i*>(q.req + (p & mask_));
    const __m128i lo = _mm_load_si128(e), hi = _mm_load_si128(e + 1);
    const uint32_t slo = (uint32_t)_mm_cvtsi128_si32(_mm_srli_si128(lo, 8));
    const uint32_t shi = (uint32_t)_mm_cvtsi128_si32(_mm_srli_si128(hi, 8));
    if (slo != shi || (slo >> 2) != (uint32_t)((p + 1) & 0x3FFFFFFFu)) break;  // not published yet
    keys[n] = (uint64_t)_mm_cvtsi128_si64(lo);
    vals[n] = (uint64_t)_mm_cvtsi128_si64(hi);
    const bool ins = (slo & PMDFC_SERVE_INSERT) != 0;
    any_ins |= ins;
    any_get |= !ins;
    any_cbf |= ins && (slo & PMDFC_SERVE_CBF);
    // (ops and cbf ops are filled below, once n is known)
    fl_h_out_[n] = (uint8_t)(slo & 3u);  // (scratch: the op bits)
  }
  if (n < lo) return false;
  // compact: keys, values, ops, cbf ops contiguous for n
  if (n < lim) memmove(keys + n, vals, n * 8);
  vals = keys + n;
  uint8_t* ops = reinterpret_cast<uint8_t*>(vals + n);
  uint8_t* cbf = ops + n;
  for (uint64_t i = 0; i < n; ++i) {
    const uint8_t b = fl_h_out_[i];
    ops[i] = (b & PMDFC_SERVE_INSERT) ? PMDFC_OP_INSERT : PMDFC_OP_GET;
    cbf[i] = ((b & PMDFC_SERVE_INSERT) && (b & PMDFC_SERVE_CBF)) ? PMDFC_OP_INSERT : PMDFC_OP_GET;
  }
  hipStream_t st = (hipStream_t)sync_;
  uint64_t* dk = reinterpret_cast<uint64_t*>(fl_d_in_);
  uint64_t* dv = dk + n;
  uint8_t* dops = reinterpret_cast<uint8_t*>(dv + n);
  uint8_t* dcbf = dops + n;
  uint64_t* dvo = reinterpret_cast<uint64_t*>(fl_d_out_);
  uint8_t* dst = reinterpret_cast<uint8_t*>(dvo + n);
  uint64_t* hvo = reinterpret_cast<uint64_t*>(fl_h_out_);
  uint8_t* hst = reinterpret_cast<uint8_t*>(hvo + n);
  bool ok = hipMemcpyAsync(dk, keys, n * 18, hipMemcpyHostToDevice, st) == hipSuccess;
  int rc = PMDFC_OK;
  if (ok) {
    if (!any_get) rc = pmdfc_cceh_insert(t_, dk, dv, dst, n, st);
    else if (!any_ins) rc = pmdfc_cceh_get(t_, dk, dvo, dst, n, st);
    else rc = pmdfc_cceh_mixed(t_, dops, dk, dv, dvo, dst, n, st);
    if (rc == PMDFC_OK && bf_ && any_cbf) rc = pmdfc_cbf_insert_ops(bf_, dcbf, dk, n, st);
    ok = rc == PMDFC_OK;
  }
  if (ok && any_get) ok = hipMemcpyAsync(hvo, dvo, n * 9, hipMemcpyDeviceToHost, st) == hipSuccess;
  else if (ok) ok = hipMemcpyAsync(hst, dst, n, hipMemcpyDeviceToHost, st) == hipSuccess;
  ok = ok && hipStreamSynchronize(st) == hipSuccess;
  if (!ok) set_error(std::string("flood batch: ") + (rc != PMDFC_OK ? pmdfc_last_error() : "HIP call failed"));
  std::atomic_thread_fence(std::memory_order_release);
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t p = head + i;
    const uint8_t sv = ok ? hst[i] : kBatchFailed;
    const uint64_t v = ok && any_get && sv == PMDFC_ST_HIT ? hvo[i] : 0;
    const __m128i w = _mm_set_epi64x((long long)((uint64_t)sv | ((uint64_t)(uint32_t)(p + 1) << 32)), (long long)v);
    _mm_store_si128(reinterpret_cast<__m128i*>(q.resp + (p & mask_)), w);
  }
  st_rel(&ctl->head, head + n);
  fl_batches_.fetch_add(1);
  fl_ops_.fetch_add(n);
  fl_ns_.fetch_add((uint64_t)((now_us() - t_fl) * 1e3));
  return true;
}

// Every queued op done, then the engine to itself (the wave stopped); the
// control thread starts the wave again when ops wait.
template <class F>
bool BatchCore::with_engine(F f) {
  if (!flush()) return false;
  std::lock_guard<std::mutex> lk(srv_mu_);
  if (!stop_server()) return false;
  f((hipStream_t)sync_);
  return true;
}

// ---------------------------------------------------------------- publish

// the BatchCore whose delivery thread (the control thread included) this is
static thread_local const BatchCore* tls_delivery = nullptr;

bool BatchCore::on_control() const { return tls_delivery == this; }

void BatchCore::write_place(Ring& q, uint64_t p, const Op& r, double t_pub) {
  const uint64_t i = p & mask_;
  q.async[i] = Async{r.cb, r.ctx, r.op, r.key, t_pub};
  // two self-validating 16-B halves, each ONE aligned 16-byte store
  const uint32_t op = (r.op == PMDFC_OP_INSERT ? PMDFC_SERVE_INSERT : 0u) | (r.cbf ? PMDFC_SERVE_CBF : 0u);
  const uint32_t sq = PMDFC_SERVE_SEQ(p, op);
  const __m128i lo = _mm_set_epi32(0, (int)sq, (int)(uint32_t)(r.key >> 32), (int)(uint32_t)r.key);
  const __m128i hi = _mm_set_epi32(0, (int)sq, (int)(uint32_t)(r.value >> 32), (int)(uint32_t)r.value);
  __m128i* e = reinterpret_cast<__m128i*>(q.req + i);
  std::atomic_thread_fence(std::memory_order_release);
  _mm_store_si128(e, lo);
  _mm_store_si128(e + 1, hi);
}

// Reserve n consecutive places of ring g (one atomic add: a run stays
// contiguous in the ring's serial order), wait for each to be free (the ring
// is full only when the results of ring_size earlier ops are not all read
// yet), write, publish.
uint64_t BatchCore::publish(uint32_t g, const Op* r, uint64_t n, double* t_pub) {
  Ring& q = *rings_[g];
  const double t0 = now_us();
  const uint64_t p0 = q.tail.fetch_add(n);
  for (uint64_t k = 0; k < n; ++k) {
    const uint64_t p = p0 + k;
    for (uint32_t spin = 0; p >= q.reclaim.load(std::memory_order_acquire) + R_; ++spin) {
      if (spin < 256) {
        cpu_relax();
        continue;
      }
      // the ring is full: sleep until the control thread frees places
      const uint32_t gen = rgen_.load(std::memory_order_seq_cst);
      rwaiters_.fetch_add(1, std::memory_order_seq_cst);
      if (p >= q.reclaim.load(std::memory_order_seq_cst) + R_) futex_wait(&rgen_, gen, 200000);
      rwaiters_.fetch_sub(1, std::memory_order_relaxed);
    }
    write_place(q, p, r[k], t0);
  }
  const double t1 = now_us();
  if (t_pub) *t_pub = t1;
  q.queue_ns.fetch_add((uint64_t)((t1 - t0) * 1e3) * n, std::memory_order_relaxed);
  return p0;
}

// (control thread) n places only if they are free now: it must never wait
// for a place, since only it frees them
bool BatchCore::try_publish(uint32_t g, const Op* r, uint64_t n) {
  Ring& q = *rings_[g];
  uint64_t t = q.tail.load(std::memory_order_relaxed);
  do {
    if (t + n > q.reclaim.load(std::memory_order_relaxed) + R_) return false;
  } while (!q.tail.compare_exchange_weak(t, t + n, std::memory_order_relaxed));
  const double now = now_us();
  for (uint64_t k = 0; k < n; ++k) write_place(q, t + k, r[k], now);
  return true;
}

void BatchCore::drain_held(uint32_t g) {
  Ring& q = *rings_[g];
  std::lock_guard<std::mutex> lk(q.held_mu);
  struct Count {  // (held_n follows every exit)
    Ring& q;
    ~Count() { q.held_n.store(q.held.size() - q.held_head, std::memory_order_release); }
  } count{q};
  while (q.held_head < q.held.size()) {
    const uint64_t n = std::min<uint64_t>(q.held.size() - q.held_head, 256);
    if (!try_publish(g, q.held.data() + q.held_head, n)) {
      if (n == 1 || !try_publish(g, q.held.data() + q.held_head, 1)) return;  // full: the next reclaim frees places
      q.held_head += 1;
      continue;
    }
    q.held_head += n;
  }
  q.held.clear();
  q.held_head = 0;
}

void BatchCore::count_failure(uint8_t op, uint8_t st, uint64_t key) {
  failed_.fetch_add(1);
  fail_by_st_[st].fetch_add(1);
  const uint32_t bit = 1u << (st < 31 ? st : 31);
  if (!(logged_.fetch_or(bit) & bit))
    fprintf(stderr, "[pmdfc] %s op of key %llu failed with status %u (%s)%s%s\n",
            op == PMDFC_OP_INSERT ? "Insert" : "Get", (unsigned long long)key, st, status_name(st),
            st == kBatchFailed ? ": " : "", st == kBatchFailed ? last_error().c_str() : "");
  if (cfg_.fatal_on_error) {
    fprintf(stderr, "[pmdfc] fatal_on_error: aborting\n");
    abort();
  }
}

// The caller reads its own results: spin on each result word (a short spin,
// then sleeping between polls), read {value, status}, mark the place read so
// the control thread can free it.
uint64_t BatchCore::await(uint32_t g, uint64_t p0, uint64_t n, const Op* r, const uint64_t* idx, uint8_t* status,
                          uint64_t* values, double t_pub) {
  Ring& q = *rings_[g];
  uint64_t bad = 0;
  double t_seen = t_pub;
  for (uint64_t k = 0; k < n; ++k) {
    const uint64_t p = p0 + k, i = p & mask_, o = idx ? idx[k] : k;
    const pmdfc_serve_resp& e = q.resp[i];
    const double t0 = now_us();
    for (uint32_t spin = 0; ld_acq(&e.seq) != (uint32_t)(p + 1); ++spin) {
      if ((spin & 63u) == 0 && now_us() - t0 > cfg_.caller_spin_us) {
        // sleep until the control thread sees answers arrive (it bumps gen_
        // after reading sleepers_, so a wake cannot slip between the
        // re-check and the wait; the timeout is only a safety net)
        const uint32_t gen = gen_.load(std::memory_order_seq_cst);
        q.asleep[i].store(1, std::memory_order_seq_cst);
        sleepers_.fetch_add(1, std::memory_order_seq_cst);
        if (ld_acq(&e.seq) != (uint32_t)(p + 1)) futex_wait(&gen_, gen, 200000);
        sleepers_.fetch_sub(1, std::memory_order_relaxed);
        q.asleep[i].store(0, std::memory_order_relaxed);
      } else {
        cpu_relax();
      }
    }
    if (k + 1 == n) t_seen = now_us();
    const uint8_t st = (uint8_t)e.status;
    const uint64_t v = e.value;
    if (status) status[o] = st;
    if (values) values[o] = st == PMDFC_ST_HIT ? v : 0;
    q.read[i].store(p + 1, std::memory_order_release);
    if (is_failure(r[k].op, st)) {
      ++bad;
      count_failure(r[k].op, st, r[k].key);
    }
  }
  const double t_end = now_us();
  q.ph_ops.fetch_add(n, std::memory_order_relaxed);
  q.ph_gpu_ns.fetch_add((uint64_t)((t_seen - t_pub) * 1e3) * n, std::memory_order_relaxed);
  q.ph_deliver_ns.fetch_add((uint64_t)((t_end - t_seen) * 1e3) * n, std::memory_order_relaxed);
  return bad;
}

uint8_t BatchCore::Insert(uint64_t key, uint64_t value, bool count_bf) {
  uint8_t st = kBatchFailed;
  InsertRun(&key, &value, &st, 1, count_bf);
  return st;
}

uint8_t BatchCore::Get(uint64_t key, uint64_t* value) {
  uint8_t st = kBatchFailed;
  uint64_t v = 0;
  GetRun(&key, &v, &st, 1);
  if (value) *value = v;
  return st;
}


// a blocking call from a completion callback would wait for its own thread
static bool refuse_on(bool ctl, uint8_t* status, uint64_t* values, uint64_t n) {
  if (!ctl) return false;
  for (uint64_t i = 0; i < n; ++i) {
    if (status) status[i] = kBatchFailed;
    if (values) values[i] = 0;
  }
  return true;
}

uint64_t BatchCore::InsertRun(const uint64_t* keys, const uint64_t* values, uint8_t* status, uint64_t n,
                              bool count_bf) {
  if (n == 0) return 0;
  if (refuse_on(on_control(), status, nullptr, n)) {
    set_error("BatchCore: a blocking call from a completion callback (it would deadlock)");
    failed_.fetch_add(n);
    fail_by_st_[kBatchFailed].fetch_add(n);
    return n;
  }
  std::vector<Op> many(n > 1 ? n : 0);
  Op one;
  Op* rs = n > 1 ? many.data() : &one;
  for (uint64_t i = 0; i < n; ++i)
    rs[i] = Op{PMDFC_OP_INSERT, (uint8_t)(count_bf ? 1 : 0), keys[i], values[i], nullptr, nullptr};
  return run(rs, n, status, nullptr);
}

// A run is published in pieces of at most half a ring, each read before the
// next is published (a piece waits for ring places that only the reading of
// earlier results frees).  Several rings: the run's ops are split by ring
// (each ring's ops in run order); a round publishes one piece per ring, then
// awaits them all.
uint64_t BatchCore::run(const Op* rs, uint64_t n, uint8_t* status, uint64_t* values, uint64_t* places) {
  uint64_t bad = 0;
  if (n == 1) {  // a per-op call: its ring, no per-ring containers
    const uint32_t g = ring_of(rs[0].key);
    double t_pub = 0;
    const uint64_t p0 = publish(g, rs, 1, &t_pub);
    if (places) places[0] = p0 | ((uint64_t)g << 48);
    return await(g, p0, 1, rs, nullptr, status, values, t_pub);
  }
  if (W_ == 1) {
    for (uint64_t o = 0; o < n;) {
      const uint64_t m = std::min<uint64_t>(n - o, R_ / 2);
      double t_pub = 0;
      const uint64_t p0 = publish(0, rs + o, m, &t_pub);
      if (places)
        for (uint64_t k = 0; k < m; ++k) places[o + k] = p0 + k;
      bad += await(0, p0, m, rs + o, nullptr, status ? status + o : nullptr, values ? values + o : nullptr, t_pub);
      o += m;
    }
    return bad;
  }
  std::vector<std::vector<uint64_t>> idx(W_);
  for (uint64_t i = 0; i < n; ++i) idx[ring_of(rs[i].key)].push_back(i);
  std::vector<std::vector<Op>> ops(W_);
  for (uint32_t g = 0; g < W_; ++g) {
    ops[g].reserve(idx[g].size());
    for (uint64_t i : idx[g]) ops[g].push_back(rs[i]);
  }
  std::vector<uint64_t> off(W_, 0), p0(W_), m(W_);
  std::vector<double> tp(W_);
  for (bool more = true; more;) {
    more = false;
    for (uint32_t g = 0; g < W_; ++g) {
      m[g] = std::min<uint64_t>(idx[g].size() - off[g], R_ / 2);
      if (!m[g]) continue;
      p0[g] = publish(g, ops[g].data() + off[g], m[g], &tp[g]);
      if (places)
        for (uint64_t k = 0; k < m[g]; ++k) places[idx[g][off[g] + k]] = (p0[g] + k) | ((uint64_t)g << 48);
    }
    for (uint32_t g = 0; g < W_; ++g) {
      if (!m[g]) continue;
      bad += await(g, p0[g], m[g], ops[g].data() + off[g], idx[g].data() + off[g], status, values, tp[g]);
      off[g] += m[g];
      more |= off[g] < idx[g].size();
    }
  }
  return bad;
}

uint64_t BatchCore::GetRun(const uint64_t* keys, uint64_t* values, uint8_t* status, uint64_t n) {
  if (n == 0) return 0;
  if (refuse_on(on_control(), status, values, n)) {
    set_error("BatchCore: a blocking call from a completion callback (it would deadlock)");
    failed_.fetch_add(n);
    fail_by_st_[kBatchFailed].fetch_add(n);
    return n;
  }
  std::vector<Op> many(n > 1 ? n : 0);
  Op one;
  Op* rs = n > 1 ? many.data() : &one;
  for (uint64_t i = 0; i < n; ++i) rs[i] = Op{PMDFC_OP_GET, 0, keys[i], 0, nullptr, nullptr};
  return run(rs, n, status, values);
}

uint64_t BatchCore::MixedRun(const uint8_t* ops, const uint64_t* keys, const uint64_t* values_in,
                             uint64_t* values_out, uint8_t* status, uint64_t n, uint64_t* places, bool count_bf) {
  if (n == 0) return 0;
  if (refuse_on(on_control(), status, values_out, n)) {
    set_error("BatchCore: a blocking call from a completion callback (it would deadlock)");
    failed_.fetch_add(n);
    fail_by_st_[kBatchFailed].fetch_add(n);
    return n;
  }
  std::vector<Op> many(n > 1 ? n : 0);
  Op one;
  Op* rs = n > 1 ? many.data() : &one;
  for (uint64_t i = 0; i < n; ++i) {
    const bool ins = ops[i] == PMDFC_OP_INSERT;
    rs[i] = Op{ins ? (uint8_t)PMDFC_OP_INSERT : (uint8_t)PMDFC_OP_GET, (uint8_t)(ins && count_bf ? 1 : 0), keys[i],
               ins ? values_in[i] : 0, nullptr, nullptr};
  }
  return run(rs, n, status, values_out, places);
}

uint64_t BatchCore::SubmitAsync(uint8_t op, uint64_t key, uint64_t value, OpCallback cb, void* ctx, bool count_bf) {
  const bool ins = op == PMDFC_OP_INSERT;
  const Op r{ins ? (uint8_t)PMDFC_OP_INSERT : (uint8_t)PMDFC_OP_GET, (uint8_t)(ins && count_bf ? 1 : 0), key,
             ins ? value : 0, cb, ctx};
  const uint32_t g = ring_of(key);
  if (on_control()) {  // (published after this round's callbacks, by the ring's delivery thread)
    Ring& h = *rings_[g];
    std::lock_guard<std::mutex> lk(h.held_mu);
    h.held.push_back(r);
    h.held_n.fetch_add(1, std::memory_order_release);
    return ~0ULL;
  }
  return publish(g, &r, 1, nullptr) | ((uint64_t)g << 48);
}

void BatchCore::InsertAsync(uint64_t key, uint64_t value, OpCallback cb, void* ctx, bool count_bf) {
  SubmitAsync(PMDFC_OP_INSERT, key, value, cb, ctx, count_bf);
}

void BatchCore::GetAsync(uint64_t key, OpCallback cb, void* ctx) { SubmitAsync(PMDFC_OP_GET, key, 0, cb, ctx); }

bool BatchCore::flush() {
  if (on_control()) {  // (the ops queued before the callback cannot complete before it returns)
    set_error("BatchCore: a blocking call from a completion callback (it would deadlock); refused");
    return false;
  }
  const double t0 = now_us();
  for (auto& q : rings_) {
    const uint64_t target = q->tail.load();
    while (q->reclaim.load() < target) {
      if (now_us() - t0 > 200.0) std::this_thread::sleep_for(std::chrono::microseconds(20));
      else cpu_relax();
    }
  }
  return true;
}

// ---------------------------------------------------------------- control

// The control thread: heartbeat; frees places in ring order once answered
// and read (running the async ops' callbacks on the way); publishes the async
// ops the callbacks queued; starts the waves when ops wait and none runs,
// stops them once all report idle (so no device-wide synchronisation in the
// process waits on them).
// One ring's answered places, in ring order: async callbacks run, places
// freed once answered and (blocking ones) read; sleeping callers with
// answers counted; callbacks' held ops published; flags for the control loop.
void BatchCore::scan_ring(uint32_t g, double t_scan, Scan& o) {
  Ring& q = *rings_[g];
  bool prog = false;
  for (const uint64_t tail = q.tail.load(std::memory_order_acquire); q.c < tail;) {
    const uint64_t i = q.c & mask_;
    const pmdfc_serve_resp& e = q.resp[i];
    if (ld_acq(&e.seq) != (uint32_t)(q.c + 1)) break;
    // the places ahead: their answers and records, and the callback
    // context of an answered one, fetched while this one's callback runs
    // (each is a line another agent wrote: ~90 ns per op taken one miss
    // after another)
    __builtin_prefetch(&q.resp[(q.c + 16) & mask_]);
    __builtin_prefetch(&q.async[(q.c + 16) & mask_]);
    if (q.c + 8 < tail && ld_acq(&q.resp[(q.c + 8) & mask_].seq) == (uint32_t)(q.c + 9)) {
      const Async& a8 = q.async[(q.c + 8) & mask_];
      if (a8.cb) __builtin_prefetch(a8.ctx, 1);
    }
    const Async& as = q.async[i];
    if (as.cb) {
      const uint8_t st = (uint8_t)e.status;
      const uint64_t v = st == PMDFC_ST_HIT ? e.value : 0;
      if (is_failure(as.op, st)) count_failure(as.op, st, as.key);
      as.cb(as.ctx, st, v);
      ++o.n_cb;
      o.gpu_ns += (uint64_t)(std::max(0.0, t_scan - as.t_pub) * 1e3);
    } else if (q.read[i].load(std::memory_order_acquire) != q.c + 1) {
      break;  // its caller has not read it yet
    }
    ++q.c;
    prog = true;
    if ((q.c & 255u) == 0) q.reclaim.store(q.c, std::memory_order_release);
  }
  if (prog) {
    q.reclaim.store(q.c, std::memory_order_seq_cst);
    o.progress = true;
  }
  // answers arrived for sleeping callers: count them
  const uint64_t tl = q.tail.load(std::memory_order_acquire);
  if (q.seen < q.c) q.seen = q.c;
  while (q.seen < tl && ld_acq(&q.resp[q.seen & mask_].seq) == (uint32_t)(q.seen + 1)) {
    o.nwake += q.asleep[q.seen & mask_].load(std::memory_order_seq_cst);
    ++q.seen;
  }
  if (q.held_n.load(std::memory_order_acquire)) drain_held(g);
  o.held_left |= q.held_n.load(std::memory_order_acquire) != 0;
  const uint64_t tail = q.tail.load(std::memory_order_acquire);
  o.pending |= q.c < tail;
  o.wait_ops |= tail > ld_acq(&q.ctl->head);
  // (the threshold is per ring: the backlog splits over the rings)
  o.flood |= cfg_.flood_ops && tail - std::max(q.seen, q.c) >= std::max<uint64_t>(cfg_.flood_ops / W_, 256);
}

// after a scan: the phase times, publishers waiting for places, sleepers
void BatchCore::finish_scan(const Scan& o, double t_scan) {
  if (o.n_cb) {
    ph_ops_.fetch_add(o.n_cb);
    ph_gpu_ns_.fetch_add(o.gpu_ns);
    ph_deliver_ns_.fetch_add((uint64_t)((now_us() - t_scan) * 1e3));
  }
  if (o.progress && rwaiters_.load(std::memory_order_seq_cst) > 0) {  // publishers wait for places
    rgen_.fetch_add(1, std::memory_order_seq_cst);
    futex_wake(&rgen_, 0x7fffffff);
  }
  const int32_t sl = sleepers_.load(std::memory_order_seq_cst);
  if (o.nwake && sl > 0) {
    gen_.fetch_add(1, std::memory_order_seq_cst);
    // a futex wakes its oldest waiters, which need not be the callers
    // answered now (a preempted caller may have gone to sleep late): with
    // more sleepers than answers, wake them all (the others sleep again)
    futex_wake(&gen_, sl > o.nwake ? 0x7fffffff : o.nwake);
  }
}

// delivery thread d >= 1 (BatchingConfig::delivery_threads): the scans of
// its rings, nothing else (the control thread starts and stops the waves,
// beats the heartbeat and serves floods for every ring)
void BatchCore::deliver(uint32_t d) {
  tls_delivery = this;
  double t_idle = now_us();
  for (;;) {
    Scan o;
    const double t_scan = now_us();
    for (uint32_t g = d; g < W_; g += D_) scan_ring(g, t_scan, o);
    finish_scan(o, t_scan);
    if (stop_.load() && !o.pending && !o.held_left) {
      // (a callback on another thread may still queue ops for my rings)
      bool idle = true;
      for (uint32_t g = 0; g < W_; ++g) {
        const Ring& q = *rings_[g];
        idle &= q.reclaim.load(std::memory_order_acquire) >= q.tail.load(std::memory_order_acquire) &&
                q.held_n.load(std::memory_order_acquire) == 0;
      }
      if (idle) return;
    }
    if (o.progress || o.pending) {
      t_idle = now_us();
      cpu_relax();
      continue;
    }
    if (now_us() - t_idle < 50.0) cpu_relax();
    else std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
}

void BatchCore::control() {
  tls_delivery = this;
  uint64_t beat = 0;
  double t_idle = now_us();
  for (;;) {
    ++beat;
    for (uint32_t g = 0; g < W_; ++g) st_rel(&ctl_[g].heartbeat, beat);
    Scan o;
    // (the async ops' phase times: one clock read per scan, the shared
    // counters updated once per scan)
    const double t_scan = now_us();
    for (uint32_t g = 0; g < W_; g += D_) scan_ring(g, t_scan, o);
    // the other delivery threads' rings: their state from the shared words
    for (uint32_t g = 0; g < W_; ++g) {
      if (g % D_ == 0) continue;
      Ring& q = *rings_[g];
      const uint64_t tail = q.tail.load(std::memory_order_acquire), rc = q.reclaim.load(std::memory_order_acquire);
      o.pending |= rc < tail;
      o.held_left |= q.held_n.load(std::memory_order_acquire) != 0;
      o.wait_ops |= tail > ld_acq(&q.ctl->head);
      o.flood |= cfg_.flood_ops && tail - rc >= std::max<uint64_t>(cfg_.flood_ops / W_, 256);
    }
    finish_scan(o, t_scan);
    const bool progress = o.progress, pending = o.pending, held_left = o.held_left, flood = o.flood,
               wait_ops = o.wait_ops;
    if (stop_.load() && !pending && !held_left) return;
    // a flood (async callers with many ops in flight): large batches here,
    // ring by ring (rings own disjoint buckets: any order of rings is serial)
    if (flood) {
      std::unique_lock<std::mutex> lk(srv_mu_, std::try_to_lock);
      if (lk.owns_lock()) {
        if (running_) stop_server();
        if (!running_) {
          for (uint32_t g = 0; g < W_; ++g)
            while (serve_flood(g)) {
            }
        }
      }
    }
    // the waves: started when ops wait, stopped once every wave reported idle
    // (or one exited by itself -- the watchdog); a running wave publishes
    // head only now and then, a stopped one's is exact
    bool all_idle = true, any_dead = false;
    if (running_)
      for (uint32_t g = 0; g < W_; ++g) {
        all_idle &= ld_acq(&ctl_[g].idle) != 0;
        any_dead |= ld_acq(&ctl_[g].alive) == 0;
      }
    if (running_ ? (all_idle || any_dead) : wait_ops) {
      std::unique_lock<std::mutex> lk(srv_mu_, std::try_to_lock);
      if (lk.owns_lock()) {
        if (running_) stop_server();
        bool waiting = false;
        for (uint32_t g = 0; g < W_; ++g) waiting |= rings_[g]->tail.load(std::memory_order_acquire) > ld_acq(&ctl_[g].head);
        if (!running_ && waiting && !start_server()) {
          // the ops cannot be served: fail them (their callers see kBatchFailed)
          for (uint32_t g = 0; g < W_; ++g) {
            Ring& q = *rings_[g];
            const uint64_t tail = q.tail.load(std::memory_order_acquire);
            for (uint64_t p = ld_acq(&q.ctl->head); p < tail; ++p) {
              pmdfc_serve_resp& r = q.resp[p & mask_];
              r.status = kBatchFailed;
              r.value = 0;
              st_rel(&r.seq, (uint32_t)(p + 1));
            }
            st_rel(&q.ctl->head, tail);
          }
        }
      }
    }
    if (progress || pending) {
      t_idle = now_us();
      cpu_relax();
      continue;
    }
    // nothing to free: spin a little, then nap (callers never wait on this
    // thread for their results; only ring places and callbacks do)
    if (now_us() - t_idle < 50.0) cpu_relax();
    else std::this_thread::sleep_for(std::chrono::microseconds(running_ ? 20 : 100));
  }
}

// ---------------------------------------------------------------- filter, stats

void BatchCore::attach_counting_bf(pmdfc_cbf_t* f) {
  with_engine([&](hipStream_t) { bf_ = f; });
}

int BatchCore::pack_counting_bf() {
  int rc = PMDFC_ERR_STATE;
  if (!with_engine([&](hipStream_t s) {
        if (!bf_) return;
        rc = pmdfc_cbf_pack(bf_, s);
        if (rc == PMDFC_OK) rc = hipStreamSynchronize(s) == hipSuccess ? PMDFC_OK : PMDFC_ERR_HIP;
      }))
    return PMDFC_ERR_STATE;
  return rc;
}

double BatchCore::Utilization() {
  double u = -1.0;
  if (!with_engine([&](hipStream_t) {
        if (pmdfc_cceh_utilization(t_, &u) != PMDFC_OK) {
          set_error(std::string("Utilization: ") + pmdfc_last_error());
          u = -1.0;
        }
      }))
    return -1.0;
  return u;
}

// CCEH::FindAnyway (CCEH_hybrid.cpp:482-496): after every op enqueued so far,
// one key through pmdfc_cceh_find_anyway (diagnostic, so synchronous and
// unbatched; a small device block allocated once)
uint8_t BatchCore::FindAnyway(uint64_t key, uint64_t* value) {
  uint8_t status = kBatchFailed;
  uint64_t v = 0;
  if (!with_engine([&](hipStream_t st) {
        uint64_t* d = fa_dev_;  // key, value, status
        uint8_t* ds = reinterpret_cast<uint8_t*>(fa_dev_ + 2);
        if (hipMemcpyAsync(d, &key, 8, hipMemcpyHostToDevice, st) == hipSuccess &&
            pmdfc_cceh_find_anyway(t_, d, d + 1, ds, 1, st) == PMDFC_OK &&
            hipMemcpyAsync(&v, d + 1, 8, hipMemcpyDeviceToHost, st) == hipSuccess &&
            hipMemcpyAsync(&status, ds, 1, hipMemcpyDeviceToHost, st) == hipSuccess &&
            hipStreamSynchronize(st) == hipSuccess) {
          if (value) *value = v;
        } else {
          status = kBatchFailed;
          set_error(std::string("FindAnyway: ") + pmdfc_last_error());
        }
      }))
    return kBatchFailed;
  return status;
}

int BatchCore::Stats(pmdfc_cceh_stats_t* out) {
  int rc = PMDFC_ERR_STATE;
  if (!with_engine([&](hipStream_t) { rc = pmdfc_cceh_stats(t_, out); })) return PMDFC_ERR_STATE;
  return rc;
}

int BatchCore::Dump(uint64_t dir_cap, uint64_t seg_cap, uint32_t* dir_canon, uint32_t* local_depth, uint64_t* prefix,
                    uint64_t* keys, uint64_t* values, uint64_t* nseg_out, uint64_t* ndir_out) {
  int rc = PMDFC_ERR_STATE;
  // sized and filled in ONE stop of the waves: no op of another thread can
  // split a segment or deepen the directory between the two
  if (!with_engine([&](hipStream_t) {
        pmdfc_cceh_stats_t s{};
        uint64_t nseg = 0;
        rc = pmdfc_cceh_stats(t_, &s);
        if (rc == PMDFC_OK) rc = pmdfc_cceh_dump(t_, nullptr, nullptr, nullptr, nullptr, nullptr, &nseg);
        if (rc != PMDFC_OK) return;
        const uint64_t ndir = 1ULL << s.depth;  // (the front-end's engine is unsharded)
        if (nseg_out) *nseg_out = nseg;
        if (ndir_out) *ndir_out = ndir;
        if ((dir_canon && ndir > dir_cap) || ((local_depth || prefix) && nseg > seg_cap) ||
            ((keys || values) && nseg * 1024 > seg_cap * 1024)) {
          rc = PMDFC_ERR_SIZE;
          return;
        }
        if (dir_canon || local_depth || prefix || keys || values)
          rc = pmdfc_cceh_dump(t_, dir_canon, local_depth, prefix, keys, values, &nseg);
      }))
    return PMDFC_ERR_STATE;
  return rc;
}

uint64_t BatchCore::header_reloads() const {
  uint64_t n = reloads_base_.load();
  for (uint32_t g = 0; g < W_; ++g) n += ld_acq(&ctl_[g].reloads);
  return n;
}

uint64_t BatchCore::Capacity() {
  uint64_t cap = 0;
  if (!with_engine([&](hipStream_t) {
        pmdfc_cceh_stats_t s{};
        if (pmdfc_cceh_stats(t_, &s) == PMDFC_OK) cap = s.capacity;
        else set_error(std::string("Capacity: ") + pmdfc_last_error());
      }))
    return 0;
  return cap;
}

}  // namespace pmdfc_host
