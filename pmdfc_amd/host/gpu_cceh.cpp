// gpu_cceh.cpp -- IHash adapter + MPSC batching front-end over the C-ABI.
#include "gpu_cceh.h"

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <stdexcept>
#include <string>
#include <strings.h>

namespace pmdfc_host {

#define CHK(x)                                                                         \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) throw std::runtime_error(std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

static void abi(int rc, const char* what) {
  if (rc != PMDFC_OK) throw std::runtime_error(std::string(what) + ": " + pmdfc_last_error());
}

GpuCCEH::GpuCCEH(size_t initCap, bool hybrid, BatchingConfig cfg, uint64_t max_segments)
    : cfg_(cfg) {
  pmdfc_cceh_config_t c{};
  c.initial_depth = hybrid ? pmdfc_depth_for_hybrid(initCap) : pmdfc_depth_for_src(initCap);
  c.max_batch = cfg.max_batch;
  c.max_segments = max_segments;
  c.device = cfg.device;
  CHK(hipSetDevice(cfg.device));
  abi(pmdfc_cceh_create(&c, &t_), "pmdfc_cceh_create");
  const size_t B = cfg.max_batch;
  CHK(hipHostMalloc((void**)&h_ops_, B, hipHostMallocDefault));
  CHK(hipHostMalloc((void**)&h_st_, B, hipHostMallocDefault));
  CHK(hipHostMalloc((void**)&h_keys_, B * 8, hipHostMallocDefault));
  CHK(hipHostMalloc((void**)&h_vin_, B * 8, hipHostMallocDefault));
  CHK(hipHostMalloc((void**)&h_vout_, B * 8, hipHostMallocDefault));
  CHK(hipMalloc((void**)&d_ops_, B));
  CHK(hipMalloc((void**)&d_st_, B));
  CHK(hipMalloc((void**)&d_keys_, B * 8));
  CHK(hipMalloc((void**)&d_vin_, B * 8));
  CHK(hipMalloc((void**)&d_vout_, B * 8));
  hipStream_t s;
  CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  stream_ = s;
  th_ = std::thread(&GpuCCEH::worker, this);
}

GpuCCEH::~GpuCCEH() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_work_.notify_all();
  if (th_.joinable()) th_.join();
  (void)hipStreamSynchronize((hipStream_t)stream_);
  (void)hipStreamDestroy((hipStream_t)stream_);
  (void)hipHostFree(h_ops_);
  (void)hipHostFree(h_st_);
  (void)hipHostFree(h_keys_);
  (void)hipHostFree(h_vin_);
  (void)hipHostFree(h_vout_);
  (void)hipFree(d_ops_);
  (void)hipFree(d_st_);
  (void)hipFree(d_keys_);
  (void)hipFree(d_vin_);
  (void)hipFree(d_vout_);
  pmdfc_cceh_destroy(t_);
}

// host batch through the pinned staging buffers (n <= max_batch)
int GpuCCEH::mixed_host(const uint8_t* ops, const uint64_t* keys, const uint64_t* vin,
                        uint64_t* vout, uint8_t* st, uint64_t n) {
  std::lock_guard<std::mutex> lk(dev_mu_);
  hipStream_t s = (hipStream_t)stream_;
  std::copy(ops, ops + n, h_ops_);
  std::copy(keys, keys + n, h_keys_);
  std::copy(vin, vin + n, h_vin_);
  CHK(hipMemcpyAsync(d_ops_, h_ops_, n, hipMemcpyHostToDevice, s));
  CHK(hipMemcpyAsync(d_keys_, h_keys_, n * 8, hipMemcpyHostToDevice, s));
  CHK(hipMemcpyAsync(d_vin_, h_vin_, n * 8, hipMemcpyHostToDevice, s));
  int rc = pmdfc_cceh_mixed(t_, d_ops_, d_keys_, d_vin_, d_vout_, d_st_, n, s);
  if (rc != PMDFC_OK) return rc;
  if (bf_ && (rc = pmdfc_cbf_insert_ops(bf_, d_ops_, d_keys_, n, s)) != PMDFC_OK) return rc;
  CHK(hipMemcpyAsync(h_vout_, d_vout_, n * 8, hipMemcpyDeviceToHost, s));
  CHK(hipMemcpyAsync(h_st_, d_st_, n, hipMemcpyDeviceToHost, s));
  CHK(hipStreamSynchronize(s));
  std::copy(h_vout_, h_vout_ + n, vout);
  std::copy(h_st_, h_st_ + n, st);
  ++launched_;
  return PMDFC_OK;
}

int GpuCCEH::run_batch(std::vector<Req*>& reqs) {
  const uint64_t n = reqs.size();
  std::vector<uint8_t> ops(n), st(n);
  std::vector<uint64_t> k(n), v(n), out(n);
  for (uint64_t i = 0; i < n; ++i) {
    ops[i] = reqs[i]->op;
    k[i] = reqs[i]->key;
    v[i] = reqs[i]->value;
  }
  int rc = mixed_host(ops.data(), k.data(), v.data(), out.data(), st.data(), n);
  for (uint64_t i = 0; i < n; ++i) {
    reqs[i]->out = out[i];
    reqs[i]->st = rc == PMDFC_OK ? st[i] : 0xFF;
  }
  return rc;
}

void GpuCCEH::worker() {
  std::vector<Req*> batch;
  for (;;) {
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_work_.wait(lk, [&] { return stop_ || !q_.empty(); });
      if (stop_ && q_.empty()) return;
      // linger briefly so concurrent callers share one device batch
      if (q_.size() < cfg_.max_batch && cfg_.linger_us) {
        cv_work_.wait_for(lk, std::chrono::microseconds(cfg_.linger_us),
                          [&] { return stop_ || q_.size() >= cfg_.max_batch; });
      }
      const size_t m = std::min<size_t>(q_.size(), cfg_.max_batch);
      batch.assign(q_.begin(), q_.begin() + m);
      q_.erase(q_.begin(), q_.begin() + m);
    }
    run_batch(batch);
    {
      std::lock_guard<std::mutex> lk(mu_);
      for (Req* r : batch) r->done = true;
    }
    cv_done_.notify_all();
  }
}

uint8_t GpuCCEH::submit(uint8_t op, uint64_t key, uint64_t value, uint64_t* out) {
  Req r;
  r.op = op;
  r.key = key;
  r.value = value;
  {
    std::lock_guard<std::mutex> lk(mu_);
    q_.push_back(&r);
  }
  cv_work_.notify_one();
  std::unique_lock<std::mutex> lk(mu_);
  cv_done_.wait(lk, [&] { return r.done; });
  if (out) *out = r.out;
  return r.st;
}

Key_t GpuCCEH::Insert(Key_t& key, Value_t value) {
  submit(PMDFC_OP_INSERT, key, reinterpret_cast<uint64_t>(value), nullptr);
  return (Key_t)-1;  // CCEH never evicts (src/cceh.cpp:152)
}

Value_t GpuCCEH::Get(Key_t& key) {
  uint64_t v = 0;
  const uint8_t st = submit(PMDFC_OP_GET, key, 0, &v);
  return st == PMDFC_ST_HIT ? reinterpret_cast<Value_t>(v) : NONE;
}

// src/cceh.cpp:309-331: power-of-two sub-extent decomposition, restated with
// the reference's integer widths (ffs on int, __builtin_ctz on unsigned int,
// x86 masking of the 64-bit shift count).
void GpuCCEH::Insert_extent(Key_t key, uint64_t cluster, uint64_t len, Value_t value) {
  std::vector<uint64_t> ks;
  while (len > 0) {
    const uint64_t cur = key + cluster;
    ks.push_back(cur);
    if (len == 1) break;
    uint64_t sub;
    if (cur % 2 == 1) {
      sub = 1;
    } else if (cur != 0) {
      const uint64_t order = (uint64_t)(int64_t)(ffs((int)cur) - 1);
      const uint64_t lim = std::min<uint64_t>(len, 1ULL << (order & 63));
      const unsigned l32 = (unsigned)lim;  // ctz(0) is undefined: 32 (as extent.hip)
      sub = 1ULL << (l32 ? __builtin_ctz(l32) : 32);
    } else {
      sub = len / 2;
    }
    cluster += sub;
    len -= sub;
  }
  std::vector<uint64_t> vs(ks.size(), reinterpret_cast<uint64_t>(value));
  std::vector<uint8_t> st(ks.size());
  for (size_t off = 0; off < ks.size(); off += cfg_.max_batch) {
    const uint64_t m = std::min<uint64_t>(cfg_.max_batch, ks.size() - off);
    std::vector<uint8_t> ops(m, PMDFC_OP_INSERT);
    std::vector<uint64_t> out(m);
    abi(mixed_host(ops.data(), ks.data() + off, vs.data() + off, out.data(), st.data() + off, m),
        "insert_extent");
  }
}

// src/cceh.cpp:381-391: the loop returns on its first iteration
Value_t GpuCCEH::Get_extent(Key_t& key, uint64_t cluster) {
  Key_t cur = key + cluster;
  return Get(cur);
}

int GpuCCEH::pack_counting_bf() {
  if (!bf_) return PMDFC_ERR_STATE;
  std::lock_guard<std::mutex> lk(dev_mu_);
  int rc = pmdfc_cbf_pack(bf_, stream_);
  if (rc != PMDFC_OK) return rc;
  CHK(hipStreamSynchronize((hipStream_t)stream_));
  return PMDFC_OK;
}

double GpuCCEH::Utilization(void) {
  double u = 0;
  abi(pmdfc_cceh_utilization(t_, &u), "utilization");
  return u;
}

size_t GpuCCEH::Capacity(void) {
  pmdfc_cceh_stats_t s{};
  abi(pmdfc_cceh_stats(t_, &s), "stats");
  return s.capacity;
}

int GpuCCEH::InsertBatch(const uint64_t* keys, const uint64_t* values, uint8_t* status, uint64_t n) {
  for (uint64_t off = 0; off < n; off += cfg_.max_batch) {
    const uint64_t m = std::min<uint64_t>(cfg_.max_batch, n - off);
    std::vector<uint8_t> ops(m, PMDFC_OP_INSERT);
    std::vector<uint64_t> out(m);
    int rc = mixed_host(ops.data(), keys + off, values + off, out.data(), status + off, m);
    if (rc) return rc;
  }
  return PMDFC_OK;
}

int GpuCCEH::GetBatch(const uint64_t* keys, uint64_t* values, uint8_t* status, uint64_t n) {
  for (uint64_t off = 0; off < n; off += cfg_.max_batch) {
    const uint64_t m = std::min<uint64_t>(cfg_.max_batch, n - off);
    std::vector<uint8_t> ops(m, PMDFC_OP_GET);
    std::vector<uint64_t> vin(m, 0);
    int rc = mixed_host(ops.data(), keys + off, vin.data(), values + off, status + off, m);
    if (rc) return rc;
  }
  return PMDFC_OK;
}

#if !defined(PMDFC_USE_REFERENCE_IHASH)
GpuCCEHHybrid::GpuCCEHHybrid(size_t initCap, BatchingConfig cfg, uint64_t max_segments)
    : t_(initCap, /*hybrid=*/true, cfg, max_segments) {}

// CCEH_hybrid.cpp:90-105 (tail recursion unrolled; widths as extent.hip)
void GpuCCEHHybrid::Insert_extent(Key_t key, Value_t value, uint64_t len) {
  std::vector<uint64_t> ks;
  uint64_t head = key;
  while (len > 0) {
    ks.push_back(head);
    if (len == 1) break;
    const unsigned f = (unsigned)ffs((int)head);
    unsigned cover = f ? (unsigned)(1ULL << (f - 1)) : 0u;
    if (cover == 0) cover = 1u << 30;  // EXTENT_MAX_HEIGHT
    while (cover > len) cover >>= 1;
    head += cover;
    len -= cover;
  }
  std::vector<uint64_t> vs(ks.size(), reinterpret_cast<uint64_t>(value));
  std::vector<uint8_t> st(ks.size());
  abi(t_.InsertBatch(ks.data(), vs.data(), st.data(), ks.size()), "Insert_extent");
}

// CCEH_hybrid.cpp:330-341: the first nonzero Get(key - key % 2^h), h < 30
Value_t GpuCCEHHybrid::Get_extent(Key_t& key) {
  uint64_t ts[30], vs[30];
  uint8_t st[30];
  for (int h = 0; h < 30; ++h) ts[h] = key - key % (1ULL << h);
  abi(t_.GetBatch(ts, vs, st, 30), "Get_extent");
  for (int h = 0; h < 30; ++h)
    if (st[h] == PMDFC_ST_HIT && vs[h]) return reinterpret_cast<Value_t>(vs[h]);
  return NONE;
}
#endif

}  // namespace pmdfc_host
