// gpu_cceh.h -- drop-in IHash backend over the MI355X batched CCEH engine.
//
// Replaces `hash = new CCEH(size)` in server/KV.cpp:63-79 (add a -DGPUCCEH
// branch there).  Per-op calls from the server's concurrent
// threads (RDMA poll threads, server/rdma_svr.cpp:755-835; harness threads,
// server/test_KV.cpp:231-258) are aggregated by an MPSC batching front-end
// into device batches (pmdfc_cceh_mixed, include/pmdfc_cceh.h) and complete
// when their batch does.  The order in which ops enter the queue is the serial
// order the batch applies, a valid linearisation of the concurrent reference
// (CCEH_hybrid.cpp:107-298 is internally synchronised, unordered).
#pragma once
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/pmdfc_cceh.h"
#include "ihash_compat.h"

namespace pmdfc_host {

struct BatchingConfig {
  uint32_t max_batch = 1 << 16;      // ops per device batch
  uint32_t linger_us = 20;           // wait for more ops before launching a partial batch
  int device = 0;
};

class GpuCCEH : public IHash {
 public:
  // src/cceh.cpp CCEH(initCap): depth = floor(log2(initCap / 1024)) -- what KV
  // links (server/KV.cpp:67-68); `hybrid` = true for CCEH_hybrid(initCap).
  explicit GpuCCEH(size_t initCap, bool hybrid = false, BatchingConfig cfg = {},
                   uint64_t max_segments = 0);
  ~GpuCCEH();

  // ---- IHash (server/IHash.h:13-21)
  Key_t Insert(Key_t& key, Value_t value) override;            // returns (Key_t)-1, src/cceh.cpp:152
  void Insert_extent(Key_t key, uint64_t cluster, uint64_t len, Value_t value) override;
  bool Delete(Key_t& key) override { (void)key; return false; }  // CCEH_hybrid.cpp:322-324 stub
  Value_t Get(Key_t& key) override;                             // NONE on miss
  Value_t Get_extent(Key_t& key, uint64_t cluster) override;
  Value_t FindAnyway(Key_t& key) override { return Get(key); }
  double Utilization(void) override;
  size_t Capacity(void) override;
  bool Recovery(void) override { return false; }               // volatile device index

  // ---- whole-batch entry points (no queueing), host arrays
  int InsertBatch(const uint64_t* keys, const uint64_t* values, uint8_t* status, uint64_t n);
  int GetBatch(const uint64_t* keys, uint64_t* values, uint8_t* status, uint64_t n);

  // KV's server bloom filter (server/KV.cpp:113-121): every Insert op of a
  // device batch also increments this counting BF, on the batch's stream.
  // The filter must live on the same device and outlive the adapter's use.
  void attach_counting_bf(pmdfc_cbf_t* f) { bf_ = f; }
  // ToOrdinaryBloomFilter on the batch stream (rdma_svr.cpp:256-264), waits for it
  int pack_counting_bf();

  pmdfc_cceh_t* engine() { return t_; }
  uint64_t batches_launched() const { return launched_; }

 private:
  struct Req {
    uint8_t op;
    uint64_t key, value;
    uint64_t out = 0;
    uint8_t st = 0;
    bool done = false;
  };
  void worker();
  uint8_t submit(uint8_t op, uint64_t key, uint64_t value, uint64_t* out);
  int run_batch(std::vector<Req*>& reqs);
  int mixed_host(const uint8_t* ops, const uint64_t* keys, const uint64_t* vin, uint64_t* vout,
                 uint8_t* st, uint64_t n);

  pmdfc_cceh_t* t_ = nullptr;
  pmdfc_cbf_t* bf_ = nullptr;
  BatchingConfig cfg_;
  std::mutex mu_;
  std::condition_variable cv_work_, cv_done_;
  std::deque<Req*> q_;
  bool stop_ = false;
  std::thread th_;
  uint64_t launched_ = 0;
  std::mutex dev_mu_;
  // pinned staging + device buffers of max_batch
  uint8_t *h_ops_ = nullptr, *h_st_ = nullptr, *d_ops_ = nullptr, *d_st_ = nullptr;
  uint64_t *h_keys_ = nullptr, *h_vin_ = nullptr, *h_vout_ = nullptr;
  uint64_t *d_keys_ = nullptr, *d_vin_ = nullptr, *d_vout_ = nullptr;
  void* stream_ = nullptr;
};

// ICCEH (server/ICCEH.h:9-27), CCEH_hybrid's interface as NUMA_KV binds it
// (server/NuMA_KV.cpp:85-155): CCEH_hybrid(initCap) geometry, the hybrid
// extent variant (CCEH_hybrid.cpp:90-105,330-341), and the NUMA statistics
// the reference never fills (CCEH_hybrid.cpp:447-478: NUM_NUMA = 2 entries).
// Only available where ICCEH is declared (the compat header, or a TU built
// with -DPMDFC_USE_REFERENCE_ICCEH).
#if !defined(PMDFC_USE_REFERENCE_IHASH)
class GpuCCEHHybrid : public ICCEH {
 public:
  explicit GpuCCEHHybrid(size_t initCap, BatchingConfig cfg = {}, uint64_t max_segments = 0);
  int GetNodeID(Key_t&) override { return 0; }  // CCEH_hybrid.cpp:326-328
  void Insert_extent(Key_t key, Value_t value, uint64_t len) override;
  void Insert(Key_t& key, Value_t value) override { t_.Insert(key, value); }
  bool Delete(Key_t& key) override { return t_.Delete(key); }
  Value_t Get(Key_t& key) override { return t_.Get(key); }
  Value_t Get_extent(Key_t& key) override;
  Value_t FindAnyway(Key_t& key) override { return t_.Get(key); }
  double Utilization(void) override { return t_.Utilization(); }
  size_t Capacity(void) override { return t_.Capacity(); }
  bool Recovery(void) override { return false; }
  std::vector<unsigned> Freqs(void) override { return std::vector<unsigned>(2, 0); }
  std::vector<size_t> SegmentLoads(void) override { return std::vector<size_t>(2, 0); }
  std::vector<double> Metrics(void) override { return std::vector<double>(2, 0.0); }
  GpuCCEH& base() { return t_; }

 private:
  GpuCCEH t_;
};
#endif

}  // namespace pmdfc_host
