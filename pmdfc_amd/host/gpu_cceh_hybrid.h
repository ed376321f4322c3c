// gpu_cceh_hybrid.h -- GpuCCEHHybrid : ICCEH, the drop-in index of NUMA_KV.
//
// ICCEH (server/ICCEH.h:9-27) is CCEH_hybrid's interface as NUMA_KV binds it
// (`cceh{new CCEH(initCap)}`, server/NuMA_KV.cpp:48-51; calls :85-155):
// CCEH_hybrid(initCap) geometry, the hybrid extent variant
// (CCEH_hybrid.cpp:90-105,330-341), and the NUMA statistics the reference
// never fills (CCEH_hybrid.cpp:447-478, NUM_NUMA = 2 entries).  Header-only
// over the BatchCore, like gpu_cceh.h; under -DPMDFC_REFERENCE_HEADERS it is
// compiled against the reference's own server/ICCEH.h (which shares IHash.h's
// include guard, so this header never includes IHash.h).
#pragma once
#include <strings.h>
#include <vector>

#include "batch_core.h"

#if defined(PMDFC_REFERENCE_HEADERS) || defined(PMDFC_USE_REFERENCE_ICCEH)
#include "ICCEH.h"
#else
#include "iface_compat.h"
#endif

namespace pmdfc_host {

// CCEH_hybrid.cpp:90-105 (tail recursion unrolled; widths as extent.hip)
inline std::vector<uint64_t> extent_heads_hybrid(uint64_t key, uint64_t len) {
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
  return ks;
}

class GpuCCEHHybrid : public ICCEH {
 public:
  explicit GpuCCEHHybrid(size_t initCap, BatchingConfig cfg = {}, uint64_t max_segments = 0)
      : core_(pmdfc_depth_for_hybrid(initCap), cfg, max_segments) {}

  int GetNodeID(Key_t&) override { return 0; }  // CCEH_hybrid.cpp:326-328
  void Insert_extent(Key_t key, Value_t value, uint64_t len) override {
    const std::vector<uint64_t> ks = extent_heads_hybrid(key, len);
    std::vector<uint64_t> vs(ks.size(), reinterpret_cast<uint64_t>(value));
    std::vector<uint8_t> st(ks.size());
    core_.InsertRun(ks.data(), vs.data(), st.data(), ks.size(), /*count_bf=*/false);
  }
  void Insert(Key_t& key, Value_t value) override { core_.Insert(key, reinterpret_cast<uint64_t>(value)); }
  bool Delete(Key_t&) override { return false; }  // CCEH_hybrid.cpp:322-324 stub
  Value_t Get(Key_t& key) override {
    uint64_t v = 0;
    return core_.Get(key, &v) == PMDFC_ST_HIT ? reinterpret_cast<Value_t>(v) : NONE;
  }
  // CCEH_hybrid.cpp:330-341: the first nonzero Get(key - key % 2^h), h < 30,
  // the 30 probes as one contiguous run
  Value_t Get_extent(Key_t& key) override {
    uint64_t ts[30], vs[30];
    uint8_t st[30];
    for (int h = 0; h < 30; ++h) ts[h] = key - key % (1ULL << h);
    core_.GetRun(ts, vs, st, 30);
    for (int h = 0; h < 30; ++h)
      if (st[h] == PMDFC_ST_HIT && vs[h]) return reinterpret_cast<Value_t>(vs[h]);
    return NONE;
  }
  // CCEH_hybrid.cpp:482-496 (src/cceh.cpp:457-471): first copy in slot order
  Value_t FindAnyway(Key_t& key) override {
    uint64_t v = 0;
    return core_.FindAnyway(key, &v) == PMDFC_ST_HIT ? reinterpret_cast<Value_t>(v) : NONE;
  }
  double Utilization(void) override { return core_.Utilization(); }
  size_t Capacity(void) override { return core_.Capacity(); }
  bool Recovery(void) override { return false; }
  std::vector<unsigned> Freqs(void) override { return std::vector<unsigned>(2, 0); }
  std::vector<size_t> SegmentLoads(void) override { return std::vector<size_t>(2, 0); }
  std::vector<double> Metrics(void) override { return std::vector<double>(2, 0.0); }

  BatchCore& core() { return core_; }

 private:
  BatchCore core_;
};

}  // namespace pmdfc_host
