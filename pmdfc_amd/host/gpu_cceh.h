// gpu_cceh.h -- GpuCCEH : IHash, the drop-in index backend of KV.
//
// Replaces `hash = new CCEH(size)` in server/KV.cpp:63-79 (a -DGPUCCEH branch
// of the backend switch; integration/KV.cpp.gpucceh.patch).
// Header-only and thin: every method forwards to the BatchCore (batch_core.h,
// libpmdfc_gpucceh.so), so this class is compiled against whichever IHash the
// including translation unit sees -- the reference's own server/IHash.h under
// -DPMDFC_REFERENCE_HEADERS, else iface_compat.h.
#pragma once
#include <algorithm>
#include <strings.h>
#include <vector>

#include "batch_core.h"

#if defined(PMDFC_REFERENCE_HEADERS) || defined(PMDFC_USE_REFERENCE_IHASH)
#include "IHash.h"
#else
#include "iface_compat.h"
#endif

namespace pmdfc_host {

// src/cceh.cpp:309-331: power-of-two sub-extent decomposition, restated with
// the reference's integer widths (ffs on int, __builtin_ctz on unsigned int,
// x86 masking of the 64-bit shift count).  Heads of the sub-extents in order.
inline std::vector<uint64_t> extent_heads_src(uint64_t key, uint64_t cluster, uint64_t len) {
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
  return ks;
}

class GpuCCEH : public IHash {
 public:
  // src/cceh.cpp CCEH(initCap): depth = floor(log2(initCap / 1024)) -- what KV
  // links (server/KV.cpp:67-68); `hybrid` = true for CCEH_hybrid(initCap).
  explicit GpuCCEH(size_t initCap, bool hybrid = false, BatchingConfig cfg = {}, uint64_t max_segments = 0)
      : core_(hybrid ? pmdfc_depth_for_hybrid(initCap) : pmdfc_depth_for_src(initCap), cfg, max_segments) {}

  // ---- IHash (server/IHash.h:13-21)
  // CCEH never evicts: (Key_t)-1 always (src/cceh.cpp:152).  KV::Insert reads
  // any other value as an evicted key and deletes it from its counting BF
  // (server/KV.cpp:104-120), so a failed op is reported through the core's
  // counters (failed_ops(), failure_count(), last_error()) or fatal_on_error.
  Key_t Insert(Key_t& key, Value_t value) override {
    core_.Insert(key, reinterpret_cast<uint64_t>(value));
    return (Key_t)-1;
  }
  // KV::InsertExtent (server/KV.cpp:129-143): the heads go through the queue
  // as one contiguous run, and not into the counting BF
  void Insert_extent(Key_t key, uint64_t cluster, uint64_t len, Value_t value) override {
    const std::vector<uint64_t> ks = extent_heads_src(key, cluster, len);
    std::vector<uint64_t> vs(ks.size(), reinterpret_cast<uint64_t>(value));
    std::vector<uint8_t> st(ks.size());
    core_.InsertRun(ks.data(), vs.data(), st.data(), ks.size(), /*count_bf=*/false);
  }
  bool Delete(Key_t& key) override {  // CCEH_hybrid.cpp:322-324 stub
    (void)key;
    return false;
  }
  Value_t Get(Key_t& key) override {  // NONE on a miss (and on a failed op)
    uint64_t v = 0;
    return core_.Get(key, &v) == PMDFC_ST_HIT ? reinterpret_cast<Value_t>(v) : NONE;
  }
  // src/cceh.cpp:381-391: the loop returns on its first iteration
  Value_t Get_extent(Key_t& key, uint64_t cluster) override {
    Key_t cur = key + cluster;
    return Get(cur);
  }
  // CCEH_hybrid.cpp:482-496 (src/cceh.cpp:457-471): first copy in slot order
  Value_t FindAnyway(Key_t& key) override {
    uint64_t v = 0;
    return core_.FindAnyway(key, &v) == PMDFC_ST_HIT ? reinterpret_cast<Value_t>(v) : NONE;
  }
  double Utilization(void) override { return core_.Utilization(); }
  size_t Capacity(void) override { return core_.Capacity(); }
  bool Recovery(void) override { return false; }  // volatile device index

  // ---- whole-batch entry points (host arrays, through the queue in order)
  int InsertBatch(const uint64_t* keys, const uint64_t* values, uint8_t* status, uint64_t n) {
    return core_.InsertRun(keys, values, status, n) ? PMDFC_ERR_STATE : PMDFC_OK;
  }
  int GetBatch(const uint64_t* keys, uint64_t* values, uint8_t* status, uint64_t n) {
    return core_.GetRun(keys, values, status, n) ? PMDFC_ERR_STATE : PMDFC_OK;
  }

  // KV's server counting BF (server/KV.cpp:113-121): every per-op Insert of a
  // device batch also increments it, on the batch's stream
  void attach_counting_bf(pmdfc_cbf_t* f) { core_.attach_counting_bf(f); }
  int pack_counting_bf() { return core_.pack_counting_bf(); }

  BatchCore& core() { return core_; }
  pmdfc_cceh_t* engine() { return core_.engine(); }
  uint64_t batches_launched() const { return core_.batches_launched(); }
  uint64_t failed_ops() const { return core_.failed_ops(); }

 private:
  BatchCore core_;
};

}  // namespace pmdfc_host
