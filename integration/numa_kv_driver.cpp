// numa_kv_driver.cpp -- drives the reference's NUMA_KV front-end
// (server/NuMA_KV.{h,cpp}, built with integration/NuMA_KV.cpp.gpucceh.patch
// and -DGPUCCEH) over the GpuCCEHHybrid : ICCEH backend, in the pattern of
// server/test_KV.cpp:204-308: T pinned threads call NUMA_KV::Insert(key,
// value, uid, node) per op (server/NuMA_KV.cpp:85-98), then T threads call
// NUMA_KV::Get(key, node) (:118-132); pass = "0 failedSearch".  It then
// checks NUMA_KV::InsertExtent / GetExtent (:69-116) page by page.
//
// The reference ships no driver for NUMA_KV (its only target, `make oneside`,
// cannot link), so this file defines the harness globals that
// NuMA_KV.cpp declares extern (server/variables.h, test_KV.cpp:20-31).
// The queued Get(key, uid, node) (:136-151) is not driven: its per-node
// queues are never allocated by the reference (NuMA_KV.h:90).
//
// Usage: numa_kv_gpu [n_keys] [threads] [first_cpu]
#include <pthread.h>
#include <sched.h>

#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "NuMA_KV.h"

size_t initialTableSize = 32 * 1024;
size_t numData = 0;
size_t numKVThreads = 0;
size_t numNetworkThreads = 0;
size_t numPollThreads = 0;
bool numa_on = false;
bool verbose_flag = false;
bool bf_flag = false;
struct bitmask* netcpubuf;
struct bitmask* kvcpubuf;
struct bitmask* pollcpubuf;
int putcnt = 0;
int getcnt = 0;

static uint64_t splitmix(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

static void pin(std::thread& t, int cpu) {
  cpu_set_t set;
  CPU_ZERO(&set);
  CPU_SET(cpu, &set);
  pthread_setaffinity_np(t.native_handle(), sizeof(set), &set);
}

int main(int argc, char** argv) {
  const size_t n = argc > 1 ? strtoull(argv[1], 0, 0) : 200000;
  const int T = argc > 2 ? atoi(argv[2]) : 8;
  const int cpu0 = argc > 3 ? atoi(argv[3]) : 0;
  numData = n;
  std::vector<Key_t> keys(n);
  for (size_t i = 0; i < n; ++i) {
    keys[i] = splitmix(i + (91ULL << 40));
    if (keys[i] >= (uint64_t)-2 || keys[i] == 0) keys[i] = 0x3333333333333333ULL + i;
  }
  // NUMA_KV(initCap) -> CCEH_hybrid(initCap): 2^14 segments, test_KV's depth
  NUMA_KV* kv = new NUMA_KV(16384);
  const size_t chunk = n / T;
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t) {
    th.emplace_back([&, t] {
      const size_t to = t == T - 1 ? n : chunk * (t + 1);
      for (size_t i = chunk * t; i < to; ++i) kv->Insert(keys[i], reinterpret_cast<Value_t>(keys[i]), (int)i, 0);
    });
    pin(th.back(), cpu0 + t);
  }
  for (auto& x : th) x.join();
  th.clear();
  std::vector<int> failed(T, 0);
  for (int t = 0; t < T; ++t) {
    th.emplace_back([&, t] {
      const size_t to = t == T - 1 ? n : chunk * (t + 1);
      for (size_t i = chunk * t; i < to; ++i)
        if (kv->Get(keys[i], 0) != reinterpret_cast<Value_t>(keys[i])) failed[t]++;
    });
    pin(th.back(), cpu0 + t);
  }
  for (auto& x : th) x.join();
  int failedSearch = 0;
  for (int f : failed) failedSearch += f;
  // extents: NUMA_KV::InsertExtent stores an Extent* and GetExtent returns
  // value + 4096 * (key - extent key) (server/NuMA_KV.cpp:69-116)
  int ext_bad = 0;
  const uint64_t ek[2] = {(7ULL << 32) + 64, (9ULL << 32)};
  const uint64_t el[2] = {100, 4097};
  for (int e = 0; e < 2; ++e) {
    Key_t k = ek[e];
    kv->InsertExtent(k, reinterpret_cast<Value_t>(0x10000000ULL * (e + 1)), el[e]);
  }
  for (int e = 0; e < 2; ++e)
    for (uint64_t d = 0; d < el[e]; d += (e ? 13 : 1)) {
      Key_t k = ek[e] + d;
      ext_bad += kv->GetExtent(k) != reinterpret_cast<Value_t>(0x10000000ULL * (e + 1) + 4096 * d);
    }
  Key_t below = ek[0] - 1;
  ext_bad += kv->GetExtent(below) != NONE;
  printf("%d failedSearch\n", failedSearch);
  printf("extent_bad %d\n", ext_bad);
  printf("Util =%.3f\t Capa =%zu\n", kv->Utilization(), kv->Capacity());
  return failedSearch == 0 && ext_bad == 0 ? 0 : 1;
}
