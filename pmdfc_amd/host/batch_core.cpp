// batch_core.cpp -- MPSC batching front-end over the C-ABI (batch_core.h).
#include "batch_core.h"

#include <hip/hip_runtime_api.h>
#include <linux/futex.h>
#include <sched.h>
#include <sys/syscall.h>
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

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// One per calling thread: a blocking call has at most one run outstanding.
// The caller spins on `remaining` for a short while (cfg.caller_spin_us), then
// sleeps on a futex word; the completer wakes only a sleeper, with one
// syscall and no lock (a mutex + condition variable cost ~2x per wake on a
// busy CPU share, and the completer wakes a batch's callers one by one).
struct BatchCore::Waiter {
  std::atomic<uint64_t> remaining{0};
  std::atomic<uint32_t> sleeping{0};  // the futex word: 1 while the caller sleeps (or is about to)
};

static void futex_wait(std::atomic<uint32_t>* a, uint32_t v) {
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(a), FUTEX_WAIT_PRIVATE, v, nullptr, nullptr, 0);
}
static void futex_wake(std::atomic<uint32_t>* a) {
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(a), FUTEX_WAKE_PRIVATE, 1, nullptr, nullptr, 0);
}

BatchCore::Waiter& BatchCore::my_waiter() {
  // never freed: the completer may still touch a waiter just after its
  // caller returned, and that caller's thread may be exiting
  thread_local Waiter* w = new Waiter;
  return *w;
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

static constexpr size_t kInBytes = 18;   // per op: key 8, value 8, op 1, cbf op 1
static constexpr size_t kOutBytes = 9;   // per op: value 8, status 1

enum : int { kFree = 0, kLaunched = 1, kExit = 2 };

BatchCore::BatchCore(uint32_t initial_depth, BatchingConfig cfg, uint64_t max_segments) : cfg_(cfg) {
  for (auto& c : fail_by_st_) c.store(0);
  pmdfc_cceh_config_t c{};
  c.initial_depth = initial_depth;
  c.max_batch = cfg.max_batch;
  c.max_segments = max_segments;
  c.device = cfg.device;
  c.flags = cfg.upsert ? PMDFC_CFG_UPSERT : 0u;
  CHK(hipSetDevice(cfg.device));
  abi(pmdfc_cceh_create(&c, &t_), "pmdfc_cceh_create");
  const size_t B = cfg.max_batch;
  // the ring holds 4 batches: callers run ahead of the launcher by that much
  uint64_t R = 1;
  while (R < 4 * (uint64_t)B) R <<= 1;
  ring_.resize(R);
  seq_.reset(new std::atomic<uint64_t>[R]);
  for (uint64_t i = 0; i < R; ++i) seq_[i].store(i, std::memory_order_relaxed);
  mask_ = R - 1;
  hipStream_t st;
  CHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  stream_ = st;
  for (Slot& s : slot_) {
    CHK(hipHostMalloc((void**)&s.h_in, B * kInBytes, hipHostMallocDefault));
    CHK(hipHostMalloc((void**)&s.h_out, B * kOutBytes, hipHostMallocDefault));
    CHK(hipHostGetDevicePointer((void**)&s.m_in, s.h_in, 0));
    CHK(hipHostGetDevicePointer((void**)&s.m_out, s.h_out, 0));
    CHK(hipMalloc((void**)&s.d_in, B * kInBytes));
    CHK(hipMalloc((void**)&s.d_out, B * kOutBytes));
    hipEvent_t e;
    CHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    s.ev = e;
    s.reqs.reserve(B);
  }
  CHK(hipMalloc((void**)&fa_dev_, 32));
  launch_th_ = std::thread(&BatchCore::launcher, this);
  cmpl_th_ = std::thread(&BatchCore::completer, this);
}

BatchCore::~BatchCore() {
  stop_.store(true);
  wake_launcher();
  if (launch_th_.joinable()) launch_th_.join();
  if (cmpl_th_.joinable()) cmpl_th_.join();
  (void)hipStreamSynchronize((hipStream_t)stream_);
  for (Slot& s : slot_) {
    if (s.h_in) (void)hipHostFree(s.h_in);
    if (s.h_out) (void)hipHostFree(s.h_out);
    if (s.d_in) (void)hipFree(s.d_in);
    if (s.d_out) (void)hipFree(s.d_out);
    if (s.ev) (void)hipEventDestroy((hipEvent_t)s.ev);
  }
  if (fa_dev_) (void)hipFree(fa_dev_);
  (void)hipStreamDestroy((hipStream_t)stream_);
  pmdfc_cceh_destroy(t_);
}

void BatchCore::set_error(const std::string& e) {
  std::lock_guard<std::mutex> lk(err_mu_);
  err_ = e;
}

BatchCore::PhaseTimes BatchCore::phase_times() const {
  std::lock_guard<std::mutex> lk(ph_mu_);
  return ph_;
}

std::string BatchCore::last_error() const {
  std::lock_guard<std::mutex> lk(err_mu_);
  return err_;
}

// ---------------------------------------------------------------- enqueue

// A worker that found nothing to do naps on its condition variable; whoever
// gives it work wakes it only then (the flag read is a shared, rarely written
// line).  The fences order "publish, then read the flag" against "set the
// flag, then re-check for work"; a miss costs at most the 1 ms nap timeout.
void BatchCore::wake_launcher() {
  std::atomic_thread_fence(std::memory_order_seq_cst);
  if (launcher_napping_.load(std::memory_order_relaxed)) {
    std::lock_guard<std::mutex> lk(nap_mu_);
    nap_cv_.notify_one();
  }
}

void BatchCore::wake_completer() {
  std::atomic_thread_fence(std::memory_order_seq_cst);
  if (completer_napping_.load(std::memory_order_relaxed)) {
    std::lock_guard<std::mutex> lk(cnap_mu_);
    cnap_cv_.notify_one();
  }
}

// Reserve n consecutive places (one atomic add: a run stays contiguous in the
// serial order), wait for each to be free (the ring is full only when the
// callers run 4 batches ahead of the GPU), write, publish.
void BatchCore::publish(const Req* r, uint64_t n) {
  if (stop_.load(std::memory_order_relaxed)) throw std::runtime_error("BatchCore: shut down");
  const uint64_t p0 = tail_.fetch_add(n, std::memory_order_relaxed);
  const double t = now_us();
  for (uint64_t k = 0; k < n; ++k) {
    const uint64_t p = p0 + k;
    std::atomic<uint64_t>& sq = seq_[p & mask_];
    for (uint32_t spin = 0; sq.load(std::memory_order_acquire) != p; ++spin) {
      if (spin > 1024) std::this_thread::yield();
      else cpu_relax();
    }
    ring_[p & mask_] = r[k];
    ring_[p & mask_].t_pub = t;
    sq.store(p + 1, std::memory_order_release);
  }
  wake_launcher();
}

// n places reserved only if they are free right now (places below head_ + ring
// size have been consumed by the launcher): the completion thread must never
// wait for a place, since only a batch it completes frees one.
bool BatchCore::try_publish(const Req* r, uint64_t n) {
  uint64_t t = tail_.load(std::memory_order_relaxed);
  do {
    if (t + n > head_.load(std::memory_order_acquire) + mask_ + 1) return false;
  } while (!tail_.compare_exchange_weak(t, t + n, std::memory_order_relaxed));
  const double now = now_us();
  for (uint64_t k = 0; k < n; ++k) {
    const uint64_t p = t + k;
    std::atomic<uint64_t>& sq = seq_[p & mask_];
    while (sq.load(std::memory_order_acquire) != p) cpu_relax();  // (freed: the launcher's store is in flight)
    ring_[p & mask_] = r[k];
    ring_[p & mask_].t_pub = now;
    sq.store(p + 1, std::memory_order_release);
  }
  wake_launcher();
  return true;
}

// A completion callback runs on the completer thread, the only thread that
// completes batches: a blocking call from it would wait for itself.
bool BatchCore::on_completer() const { return std::this_thread::get_id() == cmpl_id_.load(); }

// An async op from a completion callback is held (in order) and published
// after the batch's callbacks, as places free up: publishing it in place
// could wait for a ring place that only this thread's next completion frees.
void BatchCore::publish_async(const Req& r) {
  if (on_completer()) {
    held_.push_back(r);
    return;
  }
  publish(&r, 1);
}

void BatchCore::drain_held() {
  while (held_head_ < held_.size()) {
    const uint64_t n = std::min<uint64_t>(held_.size() - held_head_, cfg_.max_batch);
    if (!try_publish(held_.data() + held_head_, n)) {
      if (n == 1 || !try_publish(held_.data() + held_head_, 1)) return;  // full: the next completion frees places
      held_head_ += 1;
      continue;
    }
    held_head_ += n;
  }
  held_.clear();
  held_head_ = 0;
}

bool BatchCore::enqueue(const Req* r, uint64_t n, Waiter* w) {
  if (on_completer()) {
    set_error("BatchCore: a blocking call from a completion callback (it would deadlock)");
    for (uint64_t i = 0; i < n; ++i) {
      if (r[i].st) *r[i].st = kBatchFailed;
      if (r[i].out) *r[i].out = 0;
    }
    failed_.fetch_add(n);
    fail_by_st_[kBatchFailed].fetch_add(n);
    return false;
  }
  w->remaining.store(n);
  publish(r, n);
  const double t0 = now_us();
  const double spin = cfg_.caller_spin_us;
  while (w->remaining.load() != 0) {
    if (now_us() - t0 > spin) {
      // announce the sleep, then re-check: the completer zeroes `remaining`
      // before it reads `sleeping` (both seq_cst), so one of us sees the other
      for (;;) {
        w->sleeping.store(1);
        if (w->remaining.load() == 0) break;
        futex_wait(&w->sleeping, 1);
      }
      w->sleeping.store(0);
      break;
    }
    cpu_relax();
  }
  return true;
}

uint8_t BatchCore::Insert(uint64_t key, uint64_t value, bool count_bf) {
  uint8_t st = 0;
  Waiter& w = my_waiter();
  Req r{PMDFC_OP_INSERT, (uint8_t)(count_bf ? 1 : 0), key, value, nullptr, &st, &w, nullptr, nullptr};
  enqueue(&r, 1, &w);
  return st;
}

uint8_t BatchCore::Get(uint64_t key, uint64_t* value) {
  uint8_t st = 0;
  uint64_t v = 0;
  Waiter& w = my_waiter();
  Req r{PMDFC_OP_GET, 0, key, 0, &v, &st, &w, nullptr, nullptr};
  enqueue(&r, 1, &w);
  if (value) *value = v;
  return st;
}

void BatchCore::InsertAsync(uint64_t key, uint64_t value, OpCallback cb, void* ctx, bool count_bf) {
  const Req r{PMDFC_OP_INSERT, (uint8_t)(count_bf ? 1 : 0), key, value, nullptr, nullptr, nullptr, cb, ctx};
  publish_async(r);
}

void BatchCore::GetAsync(uint64_t key, OpCallback cb, void* ctx) {
  const Req r{PMDFC_OP_GET, 0, key, 0, nullptr, nullptr, nullptr, cb, ctx};
  publish_async(r);
}

uint64_t BatchCore::InsertRun(const uint64_t* keys, const uint64_t* values, uint8_t* status, uint64_t n,
                              bool count_bf) {
  if (n == 0) return 0;
  Waiter& w = my_waiter();
  std::vector<Req> rs(n);
  for (uint64_t i = 0; i < n; ++i)
    rs[i] = Req{PMDFC_OP_INSERT, (uint8_t)(count_bf ? 1 : 0), keys[i], values[i], nullptr, &status[i], &w,
                nullptr, nullptr};
  enqueue(rs.data(), n, &w);
  uint64_t bad = 0;
  for (uint64_t i = 0; i < n; ++i) bad += is_failure(PMDFC_OP_INSERT, status[i]);
  return bad;
}

uint64_t BatchCore::GetRun(const uint64_t* keys, uint64_t* values, uint8_t* status, uint64_t n) {
  if (n == 0) return 0;
  Waiter& w = my_waiter();
  std::vector<Req> rs(n);
  for (uint64_t i = 0; i < n; ++i)
    rs[i] = Req{PMDFC_OP_GET, 0, keys[i], 0, &values[i], &status[i], &w, nullptr, nullptr};
  enqueue(rs.data(), n, &w);
  uint64_t bad = 0;
  for (uint64_t i = 0; i < n; ++i) bad += is_failure(PMDFC_OP_GET, status[i]);
  return bad;
}

bool BatchCore::flush() {
  if (on_completer()) {  // (the ops queued before the callback cannot complete before it returns)
    set_error("BatchCore: a blocking call from a completion callback (it would deadlock); refused");
    return false;
  }
  const uint64_t target = tail_.load();
  const double t0 = now_us();
  while (done_seq_.load() < target) {
    if (now_us() - t0 > 200.0) std::this_thread::sleep_for(std::chrono::microseconds(20));
    else cpu_relax();
  }
  return true;
}

// ---------------------------------------------------------------- workers

// spin for a while, then nap; `ready` is re-checked after every nap
template <class F>
static void wait_for(F ready, std::atomic<bool>* napping, std::mutex* mu, std::condition_variable* cv) {
  const double t0 = now_us();
  while (!ready()) {
    if (now_us() - t0 < 100.0) {
      cpu_relax();
      continue;
    }
    std::unique_lock<std::mutex> lk(*mu);
    napping->store(true, std::memory_order_relaxed);
    std::atomic_thread_fence(std::memory_order_seq_cst);
    if (!ready()) cv->wait_for(lk, std::chrono::milliseconds(1));
    napping->store(false, std::memory_order_relaxed);
  }
}

void BatchCore::launcher() {
  int i = 0;
  for (;;) {
    Slot& s = slot_[i];
    // a free slot, then at least one published op (or shutdown with the ring drained)
    wait_for([&] { return s.state.load(std::memory_order_acquire) == kFree; }, &launcher_napping_, &nap_mu_,
             &nap_cv_);
    uint64_t h = head_.load(std::memory_order_relaxed);
    const auto published = [&](uint64_t p) {
      return seq_[p & mask_].load(std::memory_order_acquire) == p + 1;
    };
    wait_for([&] { return published(h) || (stop_.load() && tail_.load() == h); }, &launcher_napping_, &nap_mu_,
             &nap_cv_);
    if (!published(h)) break;  // stopped and drained
    if (cfg_.linger_us) {  // optional: wait for more ops before a partial batch
      const double t0 = now_us();
      while (tail_.load() - h < cfg_.max_batch && now_us() - t0 < cfg_.linger_us) cpu_relax();
    }
    // the longest published prefix: an op reserved but not yet written ends
    // the batch (the next one starts with it), so ring order is kept
    s.reqs.clear();
    while (s.reqs.size() < cfg_.max_batch && published(h)) {
      s.reqs.push_back(ring_[h & mask_]);
      seq_[h & mask_].store(h + mask_ + 1, std::memory_order_release);  // free for the next lap
      ++h;
    }
    head_.store(h, std::memory_order_relaxed);
    s.t_take = now_us();
    s.t_pub = s.t_take;
    for (const Req& q : s.reqs) s.t_pub = std::min(s.t_pub, q.t_pub);
    s.failed = false;
    try {
      stage(s);
    } catch (const std::exception& e) {
      set_error(e.what());
      s.failed = true;
    } catch (...) {
      set_error("unknown exception while staging a batch");
      s.failed = true;
    }
    s.t_launch = now_us();
    s.state.store(kLaunched, std::memory_order_release);
    wake_completer();
    i ^= 1;
  }
  // the completer drains what was launched, then exits at this slot
  Slot& s = slot_[i];
  wait_for([&] { return s.state.load(std::memory_order_acquire) == kFree; }, &launcher_napping_, &nap_mu_,
           &nap_cv_);
  s.state.store(kExit, std::memory_order_release);
  wake_completer();
}

void BatchCore::stage(Slot& s) {
  const uint64_t n = s.reqs.size();
  uint64_t* h_keys = reinterpret_cast<uint64_t*>(s.h_in);
  uint64_t* h_vin = h_keys + n;
  uint8_t* h_ops = reinterpret_cast<uint8_t*>(h_vin + n);
  uint8_t* h_cbf = h_ops + n;
  bool any_ins = false, any_get = false, any_cbf = false;
  for (uint64_t i = 0; i < n; ++i) {
    const Req& r = s.reqs[i];
    h_keys[i] = r.key;
    h_vin[i] = r.value;
    h_ops[i] = r.op;
    h_cbf[i] = (r.op == PMDFC_OP_INSERT && r.cbf) ? PMDFC_OP_INSERT : PMDFC_OP_GET;
    any_ins |= r.op == PMDFC_OP_INSERT;
    any_get |= r.op != PMDFC_OP_INSERT;
    any_cbf |= h_cbf[i] == PMDFC_OP_INSERT;
  }
  // a small batch (the blocking callers' usual ~14-32 ops) needs no copies:
  // its one kernel (k_mixed_small) reads the pinned staging block through its
  // device mapping and writes the results straight back into it
  const bool zc = n <= cfg_.zero_copy_max;
  uint8_t* in = zc ? s.m_in : s.d_in;
  uint64_t* d_keys = reinterpret_cast<uint64_t*>(in);
  uint64_t* d_vin = d_keys + n;
  uint8_t* d_ops = reinterpret_cast<uint8_t*>(d_vin + n);
  uint8_t* d_cbf = d_ops + n;
  uint64_t* d_vout = reinterpret_cast<uint64_t*>(zc ? s.m_out : s.d_out);
  uint8_t* d_st = reinterpret_cast<uint8_t*>(d_vout + n);
  std::lock_guard<std::mutex> lk(dev_mu_);
  hipStream_t st = (hipStream_t)stream_;
  if (zc) {
    abi(pmdfc_cceh_mixed(t_, d_ops, d_keys, d_vin, d_vout, d_st, n, st), "pmdfc_cceh_mixed");
    if (bf_ && any_cbf) abi(pmdfc_cbf_insert_ops(bf_, d_cbf, d_keys, n, st), "pmdfc_cbf_insert_ops");
    CHK(hipEventRecord((hipEvent_t)s.ev, st));
    launched_.fetch_add(1);
    return;
  }
  // one copy in: the keys alone for a Get batch, else everything
  const size_t in_bytes = any_ins ? n * kInBytes : n * 8;
  CHK(hipMemcpyAsync(s.d_in, s.h_in, in_bytes, hipMemcpyHostToDevice, st));
  // a batch of one kind takes its own entry point (no mixed-batch bookkeeping)
  if (!any_get) {
    abi(pmdfc_cceh_insert(t_, d_keys, d_vin, d_st, n, st), "pmdfc_cceh_insert");
  } else if (!any_ins) {
    abi(pmdfc_cceh_get(t_, d_keys, d_vout, d_st, n, st), "pmdfc_cceh_get");
  } else {
    abi(pmdfc_cceh_mixed(t_, d_ops, d_keys, d_vin, d_vout, d_st, n, st), "pmdfc_cceh_mixed");
  }
  if (bf_ && any_cbf) abi(pmdfc_cbf_insert_ops(bf_, d_cbf, d_keys, n, st), "pmdfc_cbf_insert_ops");
  // one copy out: statuses, and the values before them when there are Gets
  if (any_get)
    CHK(hipMemcpyAsync(s.h_out, s.d_out, n * kOutBytes, hipMemcpyDeviceToHost, st));
  else
    CHK(hipMemcpyAsync(s.h_out + 8 * n, d_st, n, hipMemcpyDeviceToHost, st));
  CHK(hipEventRecord((hipEvent_t)s.ev, st));
  launched_.fetch_add(1);
}

void BatchCore::completer() {
  cmpl_id_.store(std::this_thread::get_id());
  int i = 0;
  for (;;) {
    Slot& s = slot_[i];
    // (held async ops go out as places free: if the ring is full, the
    // launcher has work and a batch will come back to this loop)
    wait_for(
        [&] {
          if (held_head_ < held_.size()) drain_held();
          return s.state.load(std::memory_order_acquire) != kFree;
        },
        &completer_napping_, &cnap_mu_, &cnap_cv_);
    if (s.state.load() == kExit) return;
    if (!s.failed) {
      // poll (a blocking event wait can add tens of microseconds of wake-up)
      hipError_t e;
      const double t0 = now_us();
      while ((e = hipEventQuery((hipEvent_t)s.ev)) == hipErrorNotReady) {
        if (now_us() - t0 > 2000.0) sched_yield();
        else cpu_relax();
      }
      if (e != hipSuccess) {
        set_error(std::string("hipEventQuery: ") + hipGetErrorString(e));
        s.failed = true;
      }
    }
    const double t_done = now_us();
    complete(s);
    const uint64_t nops = s.reqs.size();
    const double t_pub = s.t_pub, t_take = s.t_take, t_launch = s.t_launch;
    // the slot is free before the sleepers are woken (one syscall each): the
    // launcher can stage the next batch meanwhile
    s.state.store(kFree, std::memory_order_release);
    wake_launcher();
    for (Waiter* w : wake_list_) futex_wake(&w->sleeping);
    wake_list_.clear();
    if (held_head_ < held_.size()) drain_held();  // what this batch's callbacks queued
    {
      const double t_end = now_us();
      std::lock_guard<std::mutex> lk(ph_mu_);
      ph_.batches += 1;
      ph_.ops += nops;
      ph_.queue_us += t_take - t_pub;
      ph_.stage_us += t_launch - t_take;
      ph_.gpu_us += t_done - t_launch;
      ph_.deliver_us += t_end - t_done;
    }
    i ^= 1;
  }
}

void BatchCore::complete(Slot& s) {
  const uint64_t n = s.reqs.size();
  const uint64_t* h_vout = reinterpret_cast<const uint64_t*>(s.h_out);
  const uint8_t* h_st = s.h_out + 8 * n;
  uint64_t bad = 0;
  for (uint64_t i = 0; i < n; ++i) {
    const Req& r = s.reqs[i];
    const uint8_t st = s.failed ? kBatchFailed : h_st[i];
    const uint64_t v = (!s.failed && st == PMDFC_ST_HIT) ? h_vout[i] : 0;
    if (r.st) *r.st = st;
    if (r.out) *r.out = v;
    if (is_failure(r.op, st)) {
      ++bad;
      fail_by_st_[st].fetch_add(1);
      const uint32_t bit = 1u << (st < 31 ? st : 31);
      if (!(logged_.fetch_or(bit) & bit))
        fprintf(stderr, "[pmdfc] %s op of key %llu failed with status %u (%s)%s%s\n",
                r.op == PMDFC_OP_INSERT ? "Insert" : "Get", (unsigned long long)r.key, st, status_name(st),
                st == kBatchFailed ? ": " : "", st == kBatchFailed ? last_error().c_str() : "");
      if (cfg_.fatal_on_error) {
        fprintf(stderr, "[pmdfc] fatal_on_error: aborting\n");
        abort();
      }
    }
    if (r.cb) r.cb(r.ctx, st, v);
  }
  if (bad) failed_.fetch_add(bad);
  done_seq_.fetch_add(n);
  // wake each blocking caller once, when the last of its ops in this batch is done
  for (uint64_t i = 0; i < n;) {
    Waiter* w = s.reqs[i].w;
    uint64_t j = i;
    while (j < n && s.reqs[j].w == w) ++j;
    if (w && w->remaining.fetch_sub(j - i) == j - i && w->sleeping.exchange(0) == 1) wake_list_.push_back(w);
    i = j;
  }
}

// ---------------------------------------------------------------- filter, stats

void BatchCore::attach_counting_bf(pmdfc_cbf_t* f) {
  if (!flush()) return;
  std::lock_guard<std::mutex> lk(dev_mu_);
  bf_ = f;
}

int BatchCore::pack_counting_bf() {
  if (!flush()) return PMDFC_ERR_STATE;
  std::lock_guard<std::mutex> lk(dev_mu_);
  if (!bf_) return PMDFC_ERR_STATE;
  int rc = pmdfc_cbf_pack(bf_, stream_);
  if (rc != PMDFC_OK) return rc;
  return hipStreamSynchronize((hipStream_t)stream_) == hipSuccess ? PMDFC_OK : PMDFC_ERR_HIP;
}

double BatchCore::Utilization() {
  if (!flush()) return -1.0;
  double u = 0;
  abi(pmdfc_cceh_utilization(t_, &u), "pmdfc_cceh_utilization");
  return u;
}

// CCEH::FindAnyway (CCEH_hybrid.cpp:482-496): after every op enqueued so far,
// one key through pmdfc_cceh_find_anyway on the core's stream (diagnostic, so
// synchronous and unbatched; a small device block allocated once)
uint8_t BatchCore::FindAnyway(uint64_t key, uint64_t* value) {
  if (!flush()) return kBatchFailed;
  std::lock_guard<std::mutex> lk(dev_mu_);
  hipStream_t st = (hipStream_t)stream_;
  uint64_t* d = fa_dev_;  // key, value, status
  uint8_t* ds = reinterpret_cast<uint8_t*>(fa_dev_ + 2);
  uint8_t status = kBatchFailed;
  uint64_t v = 0;
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
  return status;
}

uint64_t BatchCore::Capacity() {
  if (!flush()) return 0;
  pmdfc_cceh_stats_t s{};
  abi(pmdfc_cceh_stats(t_, &s), "pmdfc_cceh_stats");
  return s.capacity;
}

}  // namespace pmdfc_host
