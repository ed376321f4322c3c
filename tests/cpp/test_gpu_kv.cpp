// test_gpu_kv.cpp -- the reference harness pattern (server/test_KV.cpp:204-308)
// against the drop-in backends, outside the reference tree (iface_compat.h):
// T threads call per-op IHash::Insert concurrently (value = key), then T
// threads call IHash::Get; pass means "0 failedSearch".  Also checked: the
// counting BF sees per-op Inserts but not extent heads (server/KV.cpp:113-143),
// per-op failures are counted (not lost), upsert mode is last-writer-wins,
// and the ICCEH facade's hybrid extents.  Usage: test_gpu_kv [n_keys] [threads]
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <string>
#include <cstdlib>
#include <thread>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "../../pmdfc_amd/host/gpu_cceh.h"
#include "../../pmdfc_amd/host/gpu_cceh_hybrid.h"

static uint64_t splitmix(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

// callbacks that queue more async ops (each completion queues up to 4) with
// a 64-op batch, so the 256-place ring is full while they run: they must be
// held and published as places free, never wait for a place themselves
struct Chain {
  pmdfc_host::BatchCore* core = nullptr;
  const std::vector<uint64_t>* keys = nullptr;
  uint64_t total = 0;
  std::atomic<uint64_t> next{0}, done{0}, bad{0};
};
static void chain_cb(void* x, uint8_t st, uint64_t) {
  Chain* c = static_cast<Chain*>(x);
  if (st != PMDFC_ST_INSERTED) c->bad++;
  c->done++;
  for (int r = 0; r < 4; ++r) {
    const uint64_t i = c->next.fetch_add(1);
    if (i >= c->total) break;
    c->core->InsertAsync((*c->keys)[i], (*c->keys)[i] ^ 9, chain_cb, c);
  }
}

#define STEP(x) (fprintf(stderr, "[step] %s\n", x), fflush(stderr))

int main(int argc, char** argv) {
  const size_t n = argc > 1 ? strtoull(argv[1], 0, 0) : 200000;
  const int T = argc > 2 ? atoi(argv[2]) : 8;
  std::vector<uint64_t> keys(n);
  for (size_t i = 0; i < n; ++i) {
    keys[i] = splitmix(i + (77ULL << 40));
    if (keys[i] >= (uint64_t)-2 || keys[i] == 0) keys[i] = 0x5555555555555555ULL + i;
  }
  pmdfc_host::BatchingConfig cfg;
  cfg.max_batch = 1 << 14;
  cfg.linger_us = 50;
  // KV(10GiB*10/4096) -> src/cceh CCEH(26214400) -> depth 14 (server/test_KV.cpp:180-181)
  pmdfc_host::GpuCCEH kv(26214400, false, cfg, 1 << 15);
  STEP("created");
  // KV's server counting BF (server/KV.cpp:113-121), k=4 as the client's
  const uint64_t nbits = 10000019;
  pmdfc_cbf_t* bf = nullptr;
  if (pmdfc_cbf_create(nbits, 4, 0, &bf) != PMDFC_OK) return 2;
  kv.attach_counting_bf(bf);
  const size_t chunk = n / T;
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t)
    th.emplace_back([&, t] {
      const size_t to = t == T - 1 ? n : chunk * (t + 1);
      for (size_t i = chunk * t; i < to; ++i) kv.Insert(keys[i], reinterpret_cast<Value_t>(keys[i]));
    });
  for (auto& x : th) x.join();
  th.clear();
  STEP("inserted");
  std::vector<int> failed(T, 0);
  for (int t = 0; t < T; ++t)
    th.emplace_back([&, t] {
      const size_t to = t == T - 1 ? n : chunk * (t + 1);
      for (size_t i = chunk * t; i < to; ++i)
        if (kv.Get(keys[i]) != reinterpret_cast<Value_t>(keys[i])) failed[t]++;
    });
  for (auto& x : th) x.join();
  int failedSearch = 0;
  for (int f : failed) failedSearch += f;
  STEP("searched");
  // whole-batch path: absent keys miss
  std::vector<uint64_t> absent(1000), vals(1000);
  std::vector<uint8_t> st(1000);
  for (size_t i = 0; i < 1000; ++i) absent[i] = splitmix(i + (78ULL << 40));
  kv.GetBatch(absent.data(), vals.data(), st.data(), 1000);
  int false_hits = 0;
  for (auto s : st) false_hits += s != PMDFC_ST_MISS;
  // pack and probe the bitmap: every inserted key is positive (QueryBitBloom)
  int bf_neg = 0;
  {
    if (kv.pack_counting_bf() != PMDFC_OK) return 3;
    uint64_t* d_keys = nullptr;
    uint8_t* d_out = nullptr;
    if (hipMalloc((void**)&d_keys, n * 8) != hipSuccess || hipMalloc((void**)&d_out, n) != hipSuccess) return 4;
    (void)hipMemcpy(d_keys, keys.data(), n * 8, hipMemcpyHostToDevice);
    if (pmdfc_cbf_query_bits(bf, d_keys, d_out, n, nullptr) != PMDFC_OK) return 5;
    std::vector<uint8_t> pos(n);
    (void)hipMemcpy(pos.data(), d_out, n, hipMemcpyDeviceToHost);
    for (auto p : pos) bf_neg += p == 0;
    (void)hipFree(d_keys);
    (void)hipFree(d_out);
  }
  STEP("bf packed");
  // extent heads do not touch the counting BF (KV::InsertExtent, server/KV.cpp:129-143)
  int ext_cbf_changed = 0;
  {
    std::vector<uint8_t> c0(nbits), c1(nbits);
    if (pmdfc_cbf_get_counters_host(bf, c0.data(), nbits) != PMDFC_OK) return 6;
    kv.Insert_extent(1ULL << 40, 0, 1000, reinterpret_cast<Value_t>(0x7777ULL));
    kv.core().flush();
    if (pmdfc_cbf_get_counters_host(bf, c1.data(), nbits) != PMDFC_OK) return 7;
    for (uint64_t i = 0; i < nbits; ++i) ext_cbf_changed += c0[i] != c1[i];
    Key_t e = 1ULL << 40;  // src variant: Get(key + cluster), a sub-extent head (src/cceh.cpp:381-391)
    ext_cbf_changed += kv.Get_extent(e, 0) != reinterpret_cast<Value_t>(0x7777ULL);
  }
  STEP("extents");
  // ICCEH flavour (NUMA_KV's binding): hybrid extents cover their pages
  int ext_bad = 0;
  {
    pmdfc_host::GpuCCEHHybrid h(1024, cfg, 4096);
    h.Insert_extent(64, reinterpret_cast<Value_t>(0x1111ULL), 100);
    h.Insert_extent(1ULL << 32, reinterpret_cast<Value_t>(0x2222ULL), 4097);
    for (uint64_t k = 64; k < 164; ++k) ext_bad += h.Get_extent(k) != reinterpret_cast<Value_t>(0x1111ULL);
    for (uint64_t k = (1ULL << 32); k < (1ULL << 32) + 4097; k += 7)
      ext_bad += h.Get_extent(k) != reinterpret_cast<Value_t>(0x2222ULL);
    Key_t below = 63;
    ext_bad += h.Get_extent(below) != NONE;
    ext_bad += h.GetNodeID(below) != 0 || h.Freqs().size() != 2;
  }
  STEP("hybrid extents");
  // per-op failures are reported, not lost: a table of 8 segments at most
  // runs out (CAPACITY), a reserved key is rejected (RESERVED_KEY)
  int fail_bad = 0;
  {
    pmdfc_host::GpuCCEH small(2, true, cfg, 8);  // CCEH_hybrid(2): depth 1
    for (size_t i = 0; i < 20000; ++i) small.Insert(keys[i], reinterpret_cast<Value_t>(keys[i]));
    Key_t inv = INVALID;
    small.Insert(inv, reinterpret_cast<Value_t>(1));
    const auto& c = small.core();
    fail_bad += c.failure_count(PMDFC_ST_CAPACITY) == 0;
    fail_bad += c.failure_count(PMDFC_ST_RESERVED_KEY) != 1;
    fail_bad += c.failed_ops() != c.failure_count(PMDFC_ST_CAPACITY) + 1;
    printf("small table: %llu failed ops (%llu CAPACITY)\n", (unsigned long long)c.failed_ops(),
           (unsigned long long)c.failure_count(PMDFC_ST_CAPACITY));
  }
  STEP("failures");
  // upsert mode (last-writer-wins): the second Insert of a key overwrites
  int upsert_bad = 0;
  {
    pmdfc_host::BatchingConfig uc = cfg;
    uc.upsert = true;
    pmdfc_host::GpuCCEH u(1024, true, uc, 1 << 12);
    for (size_t i = 0; i < 5000; ++i) u.Insert(keys[i], reinterpret_cast<Value_t>(keys[i]));
    for (size_t i = 0; i < 5000; i += 2) u.Insert(keys[i], reinterpret_cast<Value_t>(keys[i] ^ 0xABCDULL));
    for (size_t i = 0; i < 5000; ++i) {
      const uint64_t want = i % 2 ? keys[i] : keys[i] ^ 0xABCDULL;
      upsert_bad += u.Get(keys[i]) != reinterpret_cast<Value_t>(want);
    }
    upsert_bad += u.failed_ops() != 0;
  }
  STEP("upsert");
  // a completion callback must not block on its core: such a call fails at
  // once (kBatchFailed, last_error) instead of deadlocking the completion thread
  int cb_bad = 0;
  {
    pmdfc_host::GpuCCEH cbt(1024, true, cfg, 1 << 12);
    struct Ctx {
      pmdfc_host::BatchCore* core;
      std::atomic<int> st{-1};
    } cx;
    cx.core = &cbt.core();
    cbt.core().InsertAsync(keys[1], keys[1], [](void* x, uint8_t, uint64_t) {
      Ctx* c = static_cast<Ctx*>(x);
      uint64_t v = 0;
      c->st = c->core->Get(12345, &v);
    }, &cx);
    cbt.core().flush();
    cb_bad += cx.st.load() != pmdfc_host::kBatchFailed;
    cb_bad += cbt.core().last_error().find("completion callback") == std::string::npos;
    cb_bad += cbt.Get(keys[1]) != reinterpret_cast<Value_t>(keys[1]);  // the core still serves
  }
  STEP("callback block");
  int chain_bad = 0;
  {
    pmdfc_host::BatchingConfig sc = cfg;
    sc.max_batch = 64;
    sc.linger_us = 0;
    pmdfc_host::GpuCCEH ch(1024, true, sc, 1 << 12);
    Chain c;
    c.core = &ch.core();
    c.keys = &keys;
    c.total = std::min<uint64_t>(20000, n);
    for (int r = 0; r < 300; ++r) {  // more than the ring holds: the main thread waits for places
      const uint64_t i = c.next.fetch_add(1);
      ch.core().InsertAsync(keys[i], keys[i] ^ 9, chain_cb, &c);
    }
    for (int ms = 0; c.done.load() < c.total && ms < 30000; ++ms) std::this_thread::sleep_for(std::chrono::milliseconds(1));
    chain_bad += c.done.load() != c.total;
    chain_bad += c.bad.load() != 0;
    for (uint64_t i = 0; i < c.total && !chain_bad; i += 7)
      chain_bad += ch.Get(keys[i]) != reinterpret_cast<Value_t>(keys[i] ^ 9);
    Key_t k0 = keys[0];
    chain_bad += ch.FindAnyway(k0) != reinterpret_cast<Value_t>(keys[0] ^ 9);
    printf("callback chain: %llu of %llu async ops done\n", (unsigned long long)c.done.load(),
           (unsigned long long)c.total);
  }
  STEP("callback chain");
  // an async flood (more unanswered ops than BatchingConfig::flood_ops): the
  // control thread serves them as engine batches with the wave stopped; ring
  // order still holds, so each thread's Get after its own Insert of a key sees
  // the value, and every op completes with the right status
  int flood_bad = 0;
  {
    pmdfc_host::BatchingConfig fc = cfg;
    fc.max_batch = 1 << 16;
    pmdfc_host::GpuCCEH fl(1024, true, fc, 1 << 14);
    struct FCtx {
      std::atomic<uint64_t> done{0}, bad{0};
    } fx;
    struct Op {
      FCtx* f;
      uint64_t want;  // Get: the value; Insert: ~0
    };
    const int FT = 4;
    const size_t per = std::min<size_t>(n / FT, 20000);
    std::vector<Op> ops(2 * per * FT);
    auto fcb = [](void* c, uint8_t st, uint64_t v) {
      Op* o = static_cast<Op*>(c);
      const bool ok = o->want == ~0ULL ? st == PMDFC_ST_INSERTED : (st == PMDFC_ST_HIT && v == o->want);
      if (!ok) o->f->bad++;
      o->f->done++;
    };
    std::vector<std::thread> ft;
    for (int t = 0; t < FT; ++t)
      ft.emplace_back([&, t] {
        for (size_t j = 0; j < per; ++j) {
          const size_t i = t * per + j;
          ops[2 * i] = Op{&fx, ~0ULL};
          fl.core().InsertAsync(keys[i], keys[i] ^ 0x5A, fcb, &ops[2 * i]);
          ops[2 * i + 1] = Op{&fx, keys[i] ^ 0x5A};
          fl.core().GetAsync(keys[i], fcb, &ops[2 * i + 1]);
        }
      });
    for (auto& x : ft) x.join();
    fl.core().flush();
    const auto ph = fl.core().phase_times();
    flood_bad += fx.done.load() != 2 * per * FT;
    flood_bad += fx.bad.load() != 0;
    for (size_t i = 0; i < per * FT; i += 101) flood_bad += fl.Get(keys[i]) != reinterpret_cast<Value_t>(keys[i] ^ 0x5A);
    printf("flood: %llu ops, %llu flood batches (%llu ops), %llu bad\n", (unsigned long long)fx.done.load(),
           (unsigned long long)ph.flood_batches, (unsigned long long)ph.flood_ops, (unsigned long long)fx.bad.load());
  }
  STEP("flood");
  // FindAnyway (CCEH_hybrid.cpp:482-496) through both facades: after the
  // queued ops, the stored value of present keys, NONE for absent ones
  int findany_bad = 0;
  for (size_t i = 0; i < n; i += n / 64 + 1) {
    Key_t k = keys[i];
    findany_bad += kv.FindAnyway(k) != reinterpret_cast<Value_t>(keys[i]);
  }
  {
    Key_t a = absent[0];
    findany_bad += kv.FindAnyway(a) != NONE;
    pmdfc_host::GpuCCEHHybrid h(1024, cfg, 4096);
    for (size_t i = 0; i < 3000; ++i) h.Insert(keys[i], reinterpret_cast<Value_t>(keys[i] ^ 0x3ULL));
    for (size_t i = 0; i < 3000; i += 97) {
      Key_t k = keys[i];
      findany_bad += h.FindAnyway(k) != reinterpret_cast<Value_t>(keys[i] ^ 0x3ULL);
    }
    findany_bad += h.FindAnyway(a) != NONE;
  }
  Key_t d = keys[0];
  printf("%d failedSearch\n", failedSearch);
  printf("findany_bad %d\n", findany_bad);
  printf("false_hits %d\n", false_hits);
  printf("bf_negatives %d\n", bf_neg);
  printf("extent_cbf_changed %d\n", ext_cbf_changed);
  printf("extent_bad %d\n", ext_bad);
  printf("failure_report_bad %d\n", fail_bad);
  printf("upsert_bad %d\n", upsert_bad);
  printf("callback_block_bad %d\n", cb_bad);
  printf("callback_chain_bad %d\n", chain_bad);
  printf("flood_bad %d\n", flood_bad);
  printf("failed_ops %llu\n", (unsigned long long)kv.failed_ops());
  printf("Util =%.3f\t Capa =%zu\n", kv.Utilization(), kv.Capacity());
  printf("batches %llu for %zu per-op calls\n", (unsigned long long)kv.batches_launched(), 2 * n);
  printf("delete %d recovery %d\n", (int)kv.Delete(d), (int)kv.Recovery());
  pmdfc_cbf_destroy(bf);
  return (failedSearch == 0 && false_hits == 0 && bf_neg == 0 && ext_cbf_changed == 0 && ext_bad == 0 &&
          fail_bad == 0 && upsert_bad == 0 && cb_bad == 0 && chain_bad == 0 && flood_bad == 0 && findany_bad == 0 &&
          kv.failed_ops() == 0)
             ? 0
             : 1;
}
