// ref_driver.cpp -- golden-vector generator that runs the REFERENCE's own
// CCEH_hybrid.cpp (or src/cceh.cpp with -DUSE_SRC_CCEH) and its util/hash.h /
// util/counting_bloom_filter.h, compiled from /root/reference by
// oracle/Makefile into oracle/_ref/ (git-ignored build output; it travels to
// the GPU box with the tree, where only the drop-in tests run its siblings).
//
// TEST INFRASTRUCTURE ONLY.  This file is our own driver; it includes the
// reference headers where they lie and is the only code that touches them.
//
// Modes (all little-endian binary files, written by oracle/gen_golden.py):
//   hash  IN OUT   IN: u64 n, u64 keys[n]
//                  OUT: per key: u64 h(key) (util/hash.h:252), u32 murmur2(key,8,s) s=0..3
//   cceh  IN OUT   IN: u64 initCap, u64 n, u64 keys[n], u64 values[n], u8 ops[n]
//                  (op 1 = Insert, 0 = Get; run serially in order)
//                  OUT: u64 depth, u64 nseg, per seg {u64 local_depth, u64 prefix},
//                       u64 keys[nseg*1024], u64 values[nseg*1024] (0 where key INVALID),
//                       u64 get_values[n], double utilization, u64 capacity
//   cbf   IN OUT   IN: u64 k, u64 m, u64 n_insert, u64 keys[n_insert], u64 n_query,
//                      u64 queries[n_query], u64 n_delete, u64 deletes[n_delete]
//                  OUT: u8 query[n_query], u8 querybb[n_query], u64 bitmap[(m+63)/64]
//                       (after deletes: u8 query2[n_query], u64 bitmap2[(m+63)/64])
//   cbfseq IN OUT  IN: u64 k, u64 m, u64 n_insert, u64 keys[n_insert], u64 n_delete,
//                      u64 deletes[n_delete]  (Insert all, then Delete in order)
//                  OUT: u8 counters[m] after the inserts, u8 deleted[n_delete],
//                       u8 counters[m] after the deletes, u64 bitmap[(m+63)/64]
//                       (ToOrdinaryBloomFilter after the deletes)
//   findany IN OUT the cceh-mode stream, then u64 nq, queries[nq]
//                  OUT: u64 FindAnyway[nq], u64 Get[nq] (after the stream)
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cmath>
#include <functional>
#include <iostream>
#include <set>
#include <sstream>
#include <string>
#include <vector>
#include <mutex>
#include <bitset>
#include <thread>
#include <unordered_map>
#include <pthread.h>
#include <time.h>
#include <openssl/sha.h>

size_t perfCounter = 0;

#define private public
#ifdef USE_SRC_CCEH
#include "src/cceh.h"
#else
#include "CCEH_hybrid.h"
#endif
#undef private
#include "util/hash.h"
#include "util/counting_bloom_filter.h"

static std::vector<uint8_t> read_file(const char* path) {
  FILE* f = fopen(path, "rb");
  if (!f) { perror(path); exit(2); }
  fseek(f, 0, SEEK_END);
  long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  std::vector<uint8_t> buf((size_t)n);
  if (n && fread(buf.data(), 1, (size_t)n, f) != (size_t)n) { perror("read"); exit(2); }
  fclose(f);
  return buf;
}

struct Reader {
  const uint8_t* p;
  template <class T> T get() { T v; memcpy(&v, p, sizeof(T)); p += sizeof(T); return v; }
  template <class T> void arr(T* out, size_t n) { memcpy(out, p, n * sizeof(T)); p += n * sizeof(T); }
};

struct Writer {
  FILE* f;
  template <class T> void put(T v) { fwrite(&v, sizeof(T), 1, f); }
  template <class T> void arr(const T* a, size_t n) { fwrite(a, sizeof(T), n, f); }
};

static int mode_hash(const char* in, const char* out) {
  auto buf = read_file(in);
  Reader r{buf.data()};
  uint64_t n = r.get<uint64_t>();
  std::vector<uint64_t> keys(n);
  r.arr(keys.data(), n);
  FILE* f = fopen(out, "wb");
  Writer w{f};
  for (uint64_t i = 0; i < n; ++i) {
    Key_t k = keys[i];
    w.put<uint64_t>(h(&k, sizeof(Key_t)));
    for (uint32_t s = 0; s < 4; ++s) w.put<uint32_t>((uint32_t)murmur2(&k, sizeof(Key_t), s));
  }
  fclose(f);
  return 0;
}

static void dump_table(CCEH* t, Writer& w) {
  Directory* d = t->dir;
  uint64_t depth = d->depth;
  uint64_t cap = d->capacity;
  std::vector<Segment*> segs;
  std::vector<uint64_t> ld, prefix;
  for (uint64_t x = 0; x < cap; ++x) {
    Segment* s = d->_[x];
    uint64_t l = s->local_depth;
    if ((x & ((1ULL << (depth - l)) - 1)) == 0) {
      segs.push_back(s);
      ld.push_back(l);
      prefix.push_back(x >> (depth - l));
    }
  }
  w.put<uint64_t>(depth);
  w.put<uint64_t>(segs.size());
  for (size_t i = 0; i < segs.size(); ++i) { w.put<uint64_t>(ld[i]); w.put<uint64_t>(prefix[i]); }
  for (Segment* s : segs)
    for (size_t j = 0; j < Segment::kNumSlot; ++j) w.put<uint64_t>(s->_[j].key);
  for (Segment* s : segs)
    for (size_t j = 0; j < Segment::kNumSlot; ++j)
      w.put<uint64_t>(s->_[j].key == INVALID ? 0 : reinterpret_cast<uint64_t>(s->_[j].value));
}

static int mode_cceh(const char* in, const char* out) {
  auto buf = read_file(in);
  Reader r{buf.data()};
  uint64_t init_cap = r.get<uint64_t>();
  uint64_t n = r.get<uint64_t>();
  std::vector<uint64_t> keys(n), values(n), results(n, 0);
  std::vector<uint8_t> ops(n);
  r.arr(keys.data(), n);
  r.arr(values.data(), n);
  r.arr(ops.data(), n);
  CCEH* t = new CCEH(init_cap);
  for (uint64_t i = 0; i < n; ++i) {
    Key_t k = keys[i];
    if (ops[i] == 1) {
      t->Insert(k, reinterpret_cast<Value_t>(values[i]));
    } else {
      results[i] = reinterpret_cast<uint64_t>(t->Get(k));
    }
  }
  FILE* f = fopen(out, "wb");
  Writer w{f};
  dump_table(t, w);
  w.arr(results.data(), n);
  w.put<double>(t->Utilization());
  w.put<uint64_t>(t->Capacity());
  fclose(f);
  return 0;
}

static int mode_cbf(const char* in, const char* out) {
  auto buf = read_file(in);
  Reader r{buf.data()};
  uint64_t k = r.get<uint64_t>(), m = r.get<uint64_t>();
  uint64_t ni = r.get<uint64_t>();
  std::vector<uint64_t> ins(ni);
  r.arr(ins.data(), ni);
  uint64_t nq = r.get<uint64_t>();
  std::vector<uint64_t> qs(nq);
  r.arr(qs.data(), nq);
  uint64_t nd = r.get<uint64_t>();
  std::vector<uint64_t> dels(nd);
  r.arr(dels.data(), nd);
  auto* bf = new CountingBloomFilter<Key_t>((uint8_t)k, m);
  for (auto key : ins) bf->Insert(key);
  bf->ToOrdinaryBloomFilter();
  FILE* f = fopen(out, "wb");
  Writer w{f};
  for (auto q : qs) w.put<uint8_t>(bf->Query(q) ? 1 : 0);
  for (auto q : qs) w.put<uint8_t>(bf->QueryBitBloom(q) ? 1 : 0);
  const uint64_t* bm = reinterpret_cast<const uint64_t*>(bf->GetBoolBitArray());
  w.arr(bm, bf->GetNumLongs());
  for (auto key : dels) bf->Delete(key);
  bf->ToOrdinaryBloomFilter();
  for (auto q : qs) w.put<uint8_t>(bf->Query(q) ? 1 : 0);
  w.arr(bm, bf->GetNumLongs());
  fclose(f);
  return 0;
}

static int mode_cbfseq(const char* in, const char* out) {
  auto buf = read_file(in);
  Reader r{buf.data()};
  uint64_t k = r.get<uint64_t>(), m = r.get<uint64_t>();
  uint64_t ni = r.get<uint64_t>();
  std::vector<uint64_t> ins(ni);
  r.arr(ins.data(), ni);
  uint64_t nd = r.get<uint64_t>();
  std::vector<uint64_t> dels(nd);
  r.arr(dels.data(), nd);
  auto* bf = new CountingBloomFilter<Key_t>((uint8_t)k, m);
  for (auto key : ins) bf->Insert(key);
  FILE* f = fopen(out, "wb");
  Writer w{f};
  const uint8_t* cnt = reinterpret_cast<const uint8_t*>(bf->GetBaseAddr());
  w.arr(cnt, m);
  for (auto key : dels) w.put<uint8_t>(bf->Delete(key) ? 1 : 0);
  w.arr(cnt, m);
  bf->ToOrdinaryBloomFilter();
  w.arr(reinterpret_cast<const uint64_t*>(bf->GetBoolBitArray()), bf->GetNumLongs());
  fclose(f);
  return 0;
}

// extent: the index's own extent API.  IN: u64 initCap, u64 n, keys[n],
// clusters[n], lens[n], values[n], u64 nq, qkeys[nq], qclusters[nq].
// hybrid: Insert_extent(key, value, len) (CCEH_hybrid.cpp:90-105), Get_extent(key)
// (:330-341); src: Insert_extent(key, cluster, len, value) (src/cceh.cpp:308-330),
// Get_extent(key, cluster) (:381-391).  OUT: the cceh-mode table dump, then
// u64 results[nq].
static int mode_extent(const char* in, const char* out) {
  auto buf = read_file(in);
  Reader r{buf.data()};
  uint64_t init_cap = r.get<uint64_t>();
  uint64_t n = r.get<uint64_t>();
  std::vector<uint64_t> keys(n), cl(n), lens(n), vals(n);
  r.arr(keys.data(), n);
  r.arr(cl.data(), n);
  r.arr(lens.data(), n);
  r.arr(vals.data(), n);
  uint64_t nq = r.get<uint64_t>();
  std::vector<uint64_t> qk(nq), qc(nq), res(nq, 0);
  r.arr(qk.data(), nq);
  r.arr(qc.data(), nq);
  CCEH* t = new CCEH(init_cap);
  for (uint64_t i = 0; i < n; ++i) {
#ifdef USE_SRC_CCEH
    t->Insert_extent(keys[i], cl[i], lens[i], reinterpret_cast<Value_t>(vals[i]));
#else
    t->Insert_extent(keys[i], reinterpret_cast<Value_t>(vals[i]), lens[i]);
#endif
  }
  for (uint64_t i = 0; i < nq; ++i) {
    Key_t k = qk[i];
#ifdef USE_SRC_CCEH
    res[i] = reinterpret_cast<uint64_t>(t->Get_extent(k, qc[i]));
#else
    res[i] = reinterpret_cast<uint64_t>(t->Get_extent(k));
#endif
  }
  FILE* f = fopen(out, "wb");
  Writer w{f};
  dump_table(t, w);
  w.arr(res.data(), nq);
  fclose(f);
  return 0;
}

// findany: the reference's FindAnyway (CCEH_hybrid.cpp:482-496; src/cceh.cpp:
// 457-471) next to Get.  IN: the cceh-mode stream (run serially), then u64 nq,
// queries[nq].  OUT: u64 find[nq], u64 get[nq] (FindAnyway prints its
// diagnostics to std::cout; they go to a discarded buffer).
static int mode_findany(const char* in, const char* out) {
  auto buf = read_file(in);
  Reader r{buf.data()};
  uint64_t init_cap = r.get<uint64_t>();
  uint64_t n = r.get<uint64_t>();
  std::vector<uint64_t> keys(n), values(n);
  std::vector<uint8_t> ops(n);
  r.arr(keys.data(), n);
  r.arr(values.data(), n);
  r.arr(ops.data(), n);
  uint64_t nq = r.get<uint64_t>();
  std::vector<uint64_t> qk(nq), fa(nq), gv(nq);
  r.arr(qk.data(), nq);
  CCEH* t = new CCEH(init_cap);
  for (uint64_t i = 0; i < n; ++i) {
    Key_t k = keys[i];
    if (ops[i] == 1) t->Insert(k, reinterpret_cast<Value_t>(values[i]));
    else (void)t->Get(k);
  }
  std::ostringstream sink;
  std::streambuf* old = std::cout.rdbuf(sink.rdbuf());
  for (uint64_t i = 0; i < nq; ++i) {
    Key_t k = qk[i];
    fa[i] = reinterpret_cast<uint64_t>(t->FindAnyway(k));
    gv[i] = reinterpret_cast<uint64_t>(t->Get(k));
  }
  std::cout.rdbuf(old);
  FILE* f = fopen(out, "wb");
  Writer w{f};
  w.arr(fa.data(), nq);
  w.arr(gv.data(), nq);
  fclose(f);
  return 0;
}

// bench N T INITCAP SEED: the reference's own CCEH_hybrid, test_KV's thread
// pattern (server/test_KV.cpp:204-303, without the sleep(1)): T threads insert
// contiguous chunks of N splitmix64 keys (value = key), then T threads Get
// them.  Prints "insert_s get_s failed".
static uint64_t splitmix(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

static double now_s() {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static int mode_bench(int argc, char** argv) {
  const size_t n = strtoull(argv[2], 0, 0);
  const int T = atoi(argv[3]);
  const size_t cap = strtoull(argv[4], 0, 0);
  const uint64_t seed = argc > 5 ? strtoull(argv[5], 0, 0) : 1000;
  std::vector<Key_t> keys(n);
  for (size_t i = 0; i < n; ++i) {
    uint64_t ctr = i + (seed << 40);
    uint64_t k = splitmix(ctr);
    if (k == 0 || k >= (uint64_t)-2) k = 0x5555555555555555ULL + ctr;
    keys[i] = k;
  }
  CCEH* t = new CCEH(cap);
  const size_t chunk = n / T;
  std::vector<std::thread> th;
  double t0 = now_s();
  for (int i = 0; i < T; ++i)
    th.emplace_back([&, i] {
      size_t to = i == T - 1 ? n : chunk * (i + 1);
      for (size_t j = chunk * i; j < to; ++j) t->Insert(keys[j], reinterpret_cast<Value_t>(keys[j]));
    });
  for (auto& x : th) x.join();
  double t1 = now_s();
  th.clear();
  std::vector<size_t> failed(T, 0);
  for (int i = 0; i < T; ++i)
    th.emplace_back([&, i] {
      size_t to = i == T - 1 ? n : chunk * (i + 1);
      size_t f = 0;
      for (size_t j = chunk * i; j < to; ++j)
        if (t->Get(keys[j]) != reinterpret_cast<Value_t>(keys[j])) ++f;
      failed[i] = f;
    });
  for (auto& x : th) x.join();
  double t2 = now_s();
  size_t fs = 0;
  for (auto f : failed) fs += f;
  printf("%.6f %.6f %zu\n", t1 - t0, t2 - t1, fs);
  return 0;
}

int main(int argc, char** argv) {
  if (argc >= 5 && std::string(argv[1]) == "bench") return mode_bench(argc, argv);
  if (argc != 4) {
    fprintf(stderr, "usage: %s hash|cceh|cbf IN OUT\n", argv[0]);
    return 2;
  }
  std::string m = argv[1];
  if (m == "hash") return mode_hash(argv[2], argv[3]);
  if (m == "cceh") return mode_cceh(argv[2], argv[3]);
  if (m == "cbf") return mode_cbf(argv[2], argv[3]);
  if (m == "cbfseq") return mode_cbfseq(argv[2], argv[3]);
  if (m == "extent") return mode_extent(argv[2], argv[3]);
  if (m == "findany") return mode_findany(argv[2], argv[3]);
  fprintf(stderr, "unknown mode %s\n", argv[1]);
  return 2;
}
