// batch_core.cpp -- MPSC batching front-end over the C-ABI (batch_core.h).
#include "batch_core.h"

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>

namespace pmdfc_host {

#define CHK(x)                                                                                \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) throw std::runtime_error(std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

static void abi(int rc, const char* what) {
  if (rc != PMDFC_OK) throw std::runtime_error(std::string(what) + ": " + pmdfc_last_error());
}

// one per calling thread: a blocking call has at most one run outstanding
struct BatchCore::Waiter {
  std::mutex m;
  std::condition_variable cv;
  uint64_t remaining = 0;
};

BatchCore::Waiter& BatchCore::my_waiter() {
  thread_local Waiter w;
  return w;
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
  hipStream_t st;
  CHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  stream_ = st;
  for (Slot& s : slot_) {
    CHK(hipHostMalloc((void**)&s.h_ops, B, hipHostMallocDefault));
    CHK(hipHostMalloc((void**)&s.h_cbf, B, hipHostMallocDefault));
    CHK(hipHostMalloc((void**)&s.h_st, B, hipHostMallocDefault));
    CHK(hipHostMalloc((void**)&s.h_keys, B * 8, hipHostMallocDefault));
    CHK(hipHostMalloc((void**)&s.h_vin, B * 8, hipHostMallocDefault));
    CHK(hipHostMalloc((void**)&s.h_vout, B * 8, hipHostMallocDefault));
    CHK(hipMalloc((void**)&s.d_ops, B));
    CHK(hipMalloc((void**)&s.d_cbf, B));
    CHK(hipMalloc((void**)&s.d_st, B));
    CHK(hipMalloc((void**)&s.d_keys, B * 8));
    CHK(hipMalloc((void**)&s.d_vin, B * 8));
    CHK(hipMalloc((void**)&s.d_vout, B * 8));
    hipEvent_t e;
    CHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    s.ev = e;
    s.reqs.reserve(B);
  }
  launch_th_ = std::thread(&BatchCore::launcher, this);
  cmpl_th_ = std::thread(&BatchCore::completer, this);
}

BatchCore::~BatchCore() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_work_.notify_all();
  cv_slot_.notify_all();
  if (launch_th_.joinable()) launch_th_.join();
  cv_cmpl_.notify_all();
  if (cmpl_th_.joinable()) cmpl_th_.join();
  (void)hipStreamSynchronize((hipStream_t)stream_);
  for (Slot& s : slot_) {
    for (void* p : {(void*)s.h_ops, (void*)s.h_cbf, (void*)s.h_st, (void*)s.h_keys, (void*)s.h_vin, (void*)s.h_vout})
      if (p) (void)hipHostFree(p);
    for (void* p : {(void*)s.d_ops, (void*)s.d_cbf, (void*)s.d_st, (void*)s.d_keys, (void*)s.d_vin, (void*)s.d_vout})
      if (p) (void)hipFree(p);
    if (s.ev) (void)hipEventDestroy((hipEvent_t)s.ev);
  }
  (void)hipStreamDestroy((hipStream_t)stream_);
  pmdfc_cceh_destroy(t_);
}

void BatchCore::set_error(const std::string& e) {
  std::lock_guard<std::mutex> lk(err_mu_);
  err_ = e;
}

std::string BatchCore::last_error() const {
  std::lock_guard<std::mutex> lk(err_mu_);
  return err_;
}

// ---------------------------------------------------------------- enqueue

void BatchCore::enqueue(Req* r, uint64_t n, Waiter* w) {
  {
    std::lock_guard<std::mutex> lw(w->m);
    w->remaining = n;
  }
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (stop_) throw std::runtime_error("BatchCore: shut down");
    for (uint64_t i = 0; i < n; ++i) q_.push_back(r[i]);
    enq_seq_ += n;
  }
  cv_work_.notify_one();
  std::unique_lock<std::mutex> lw(w->m);
  w->cv.wait(lw, [&] { return w->remaining == 0; });
}

uint8_t BatchCore::Insert(uint64_t key, uint64_t value, bool count_bf) {
  uint8_t st = 0;
  Waiter& w = my_waiter();
  Req r{PMDFC_OP_INSERT, (uint8_t)(count_bf ? 1 : 0), key, value, nullptr, &st, &w};
  enqueue(&r, 1, &w);
  return st;
}

uint8_t BatchCore::Get(uint64_t key, uint64_t* value) {
  uint8_t st = 0;
  uint64_t v = 0;
  Waiter& w = my_waiter();
  Req r{PMDFC_OP_GET, 0, key, 0, &v, &st, &w};
  enqueue(&r, 1, &w);
  if (value) *value = v;
  return st;
}

uint64_t BatchCore::InsertRun(const uint64_t* keys, const uint64_t* values, uint8_t* status, uint64_t n,
                              bool count_bf) {
  if (n == 0) return 0;
  Waiter& w = my_waiter();
  std::vector<Req> rs(n);
  for (uint64_t i = 0; i < n; ++i)
    rs[i] = Req{PMDFC_OP_INSERT, (uint8_t)(count_bf ? 1 : 0), keys[i], values[i], nullptr, &status[i], &w};
  enqueue(rs.data(), n, &w);
  uint64_t bad = 0;
  for (uint64_t i = 0; i < n; ++i) bad += is_failure(PMDFC_OP_INSERT, status[i]);
  return bad;
}

uint64_t BatchCore::GetRun(const uint64_t* keys, uint64_t* values, uint8_t* status, uint64_t n) {
  if (n == 0) return 0;
  Waiter& w = my_waiter();
  std::vector<Req> rs(n);
  for (uint64_t i = 0; i < n; ++i) rs[i] = Req{PMDFC_OP_GET, 0, keys[i], 0, &values[i], &status[i], &w};
  enqueue(rs.data(), n, &w);
  uint64_t bad = 0;
  for (uint64_t i = 0; i < n; ++i) bad += is_failure(PMDFC_OP_GET, status[i]);
  return bad;
}

void BatchCore::flush() {
  std::unique_lock<std::mutex> lk(mu_);
  const uint64_t target = enq_seq_;
  cv_flush_.wait(lk, [&] { return done_seq_.load() >= target; });
}

// ---------------------------------------------------------------- workers

void BatchCore::launcher() {
  int i = 0;
  for (;;) {
    Slot& s = slot_[i];
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_slot_.wait(lk, [&] { return stop_ || !s.busy; });
      cv_work_.wait(lk, [&] { return stop_ || !q_.empty(); });
      if (q_.empty()) break;  // stop_ and drained
      if (q_.size() < cfg_.max_batch && cfg_.linger_us && !stop_) {
        // linger so concurrent callers share one device batch
        cv_work_.wait_for(lk, std::chrono::microseconds(cfg_.linger_us),
                          [&] { return stop_ || q_.size() >= cfg_.max_batch; });
      }
      if (s.busy) cv_slot_.wait(lk, [&] { return !s.busy; });
      const size_t m = std::min<size_t>(q_.size(), cfg_.max_batch);
      s.reqs.assign(q_.begin(), q_.begin() + m);
      q_.erase(q_.begin(), q_.begin() + m);
      s.busy = true;
    }
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
    {
      std::lock_guard<std::mutex> lk(mu_);
      cmpl_.push_back(i);
    }
    cv_cmpl_.notify_one();
    i ^= 1;
  }
  {
    std::lock_guard<std::mutex> lk(mu_);
    cmpl_.push_back(-1);  // the completer drains what was launched, then exits
  }
  cv_cmpl_.notify_one();
}

void BatchCore::stage(Slot& s) {
  const uint64_t n = s.reqs.size();
  bool any_ins = false, any_get = false, any_cbf = false;
  for (uint64_t i = 0; i < n; ++i) {
    const Req& r = s.reqs[i];
    s.h_ops[i] = r.op;
    s.h_keys[i] = r.key;
    s.h_vin[i] = r.value;
    s.h_cbf[i] = (r.op == PMDFC_OP_INSERT && r.cbf) ? PMDFC_OP_INSERT : PMDFC_OP_GET;
    any_ins |= r.op == PMDFC_OP_INSERT;
    any_get |= r.op != PMDFC_OP_INSERT;
    any_cbf |= s.h_cbf[i] == PMDFC_OP_INSERT;
  }
  std::lock_guard<std::mutex> lk(dev_mu_);
  hipStream_t st = (hipStream_t)stream_;
  CHK(hipMemcpyAsync(s.d_keys, s.h_keys, n * 8, hipMemcpyHostToDevice, st));
  if (any_ins) {
    CHK(hipMemcpyAsync(s.d_vin, s.h_vin, n * 8, hipMemcpyHostToDevice, st));
  }
  // a batch of one kind takes its own entry point (no mixed-batch bookkeeping)
  if (!any_get) {
    abi(pmdfc_cceh_insert(t_, s.d_keys, s.d_vin, s.d_st, n, st), "pmdfc_cceh_insert");
  } else if (!any_ins) {
    abi(pmdfc_cceh_get(t_, s.d_keys, s.d_vout, s.d_st, n, st), "pmdfc_cceh_get");
  } else {
    CHK(hipMemcpyAsync(s.d_ops, s.h_ops, n, hipMemcpyHostToDevice, st));
    abi(pmdfc_cceh_mixed(t_, s.d_ops, s.d_keys, s.d_vin, s.d_vout, s.d_st, n, st), "pmdfc_cceh_mixed");
  }
  if (bf_ && any_cbf) {
    CHK(hipMemcpyAsync(s.d_cbf, s.h_cbf, n, hipMemcpyHostToDevice, st));
    abi(pmdfc_cbf_insert_ops(bf_, s.d_cbf, s.d_keys, n, st), "pmdfc_cbf_insert_ops");
  }
  if (any_get) {
    CHK(hipMemcpyAsync(s.h_vout, s.d_vout, n * 8, hipMemcpyDeviceToHost, st));
  }
  CHK(hipMemcpyAsync(s.h_st, s.d_st, n, hipMemcpyDeviceToHost, st));
  CHK(hipEventRecord((hipEvent_t)s.ev, st));
  launched_.fetch_add(1);
}

void BatchCore::completer() {
  for (;;) {
    int i;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_cmpl_.wait(lk, [&] { return !cmpl_.empty(); });
      i = cmpl_.front();
      cmpl_.pop_front();
    }
    if (i < 0) return;
    Slot& s = slot_[i];
    if (!s.failed) {
      const hipError_t e = hipEventSynchronize((hipEvent_t)s.ev);
      if (e != hipSuccess) {
        set_error(std::string("hipEventSynchronize: ") + hipGetErrorString(e));
        s.failed = true;
      }
    }
    complete(s);
    {
      std::lock_guard<std::mutex> lk(mu_);
      s.busy = false;
    }
    cv_slot_.notify_one();
  }
}

void BatchCore::complete(Slot& s) {
  const uint64_t n = s.reqs.size();
  for (uint64_t i = 0; i < n; ++i) {
    const Req& r = s.reqs[i];
    const uint8_t st = s.failed ? kBatchFailed : s.h_st[i];
    *r.st = st;
    if (r.out) *r.out = (!s.failed && st == PMDFC_ST_HIT) ? s.h_vout[i] : 0;
  }
  note_failures(s);
  {
    std::lock_guard<std::mutex> lk(mu_);
    done_seq_.fetch_add(n);
  }
  cv_flush_.notify_all();
  // wake each caller once, when the last of its ops in this batch is done
  for (uint64_t i = 0; i < n;) {
    Waiter* w = s.reqs[i].w;
    uint64_t j = i;
    while (j < n && s.reqs[j].w == w) ++j;
    bool wake;
    {
      std::lock_guard<std::mutex> lw(w->m);
      w->remaining -= j - i;
      wake = w->remaining == 0;
    }
    if (wake) w->cv.notify_one();
    i = j;
  }
}

void BatchCore::note_failures(const Slot& s) {
  uint64_t bad = 0;
  for (const Req& r : s.reqs) {
    const uint8_t st = *r.st;
    if (!is_failure(r.op, st)) continue;
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
  if (bad) failed_.fetch_add(bad);
}

// ---------------------------------------------------------------- filter, stats

void BatchCore::attach_counting_bf(pmdfc_cbf_t* f) {
  flush();
  std::lock_guard<std::mutex> lk(dev_mu_);
  bf_ = f;
}

int BatchCore::pack_counting_bf() {
  flush();
  std::lock_guard<std::mutex> lk(dev_mu_);
  if (!bf_) return PMDFC_ERR_STATE;
  int rc = pmdfc_cbf_pack(bf_, stream_);
  if (rc != PMDFC_OK) return rc;
  return hipStreamSynchronize((hipStream_t)stream_) == hipSuccess ? PMDFC_OK : PMDFC_ERR_HIP;
}

double BatchCore::Utilization() {
  flush();
  double u = 0;
  abi(pmdfc_cceh_utilization(t_, &u), "pmdfc_cceh_utilization");
  return u;
}

uint64_t BatchCore::Capacity() {
  flush();
  pmdfc_cceh_stats_t s{};
  abi(pmdfc_cceh_stats(t_, &s), "pmdfc_cceh_stats");
  return s.capacity;
}

}  // namespace pmdfc_host
