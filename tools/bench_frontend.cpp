// bench_frontend.cpp -- per-op throughput of the batching front-end at
// server concurrency: the reference calls its index per op from up to
// NUM_CLIENT x NUM_QUEUES = 4 x 8 = 32 RDMA poll threads
// (server/rdma_svr.h:17-18, server/rdma_svr.cpp:755-835).  T threads, each
// pinned to its own CPU of this process's affinity set, call GpuCCEH (the
// IHash facade KV binds, server/KV.cpp:100-158) per op: an Insert phase
// (value = key), then a Get phase; then a 50/50 mixed phase of fresh Inserts
// and Gets of stored keys.  Blocking calls keep one op per thread in flight;
// then the same three phases through the async calls (InsertAsync /
// GetAsync), each thread keeping up to `window` ops outstanding, as an RDMA
// poll thread that posts its reply from the completion would.  Prints one
// JSON line.
// Usage: bench_frontend [threads=32] [ops_per_thread=65536] [window=256] [max_batch=65536] [spin_us=10]
//                       [serve_waves=1] [delivery_threads=1]
#include <pthread.h>
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <string>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "../pmdfc_amd/host/gpu_cceh.h"

static uint64_t splitmix(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

static double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const int T = argc > 1 ? atoi(argv[1]) : 32;
  const size_t per = argc > 2 ? strtoull(argv[2], 0, 0) : 65536;
  const int W = argc > 3 ? atoi(argv[3]) : 256;
  pmdfc_host::BatchingConfig cfg;
  cfg.max_batch = argc > 4 ? (uint32_t)atoi(argv[4]) : 65536;
  if (argc > 5) cfg.caller_spin_us = (uint32_t)atoi(argv[5]);
  if (argc > 6) cfg.serve_waves = (uint32_t)atoi(argv[6]);  // serving waves (rings by hash prefix)
  if (argc > 7) cfg.delivery_threads = (uint32_t)atoi(argv[7]);  // threads running the async callbacks
  const size_t n = per * T;
  std::vector<uint64_t> keys(4 * n);
  for (size_t i = 0; i < 4 * n; ++i) {
    keys[i] = splitmix(i + (55ULL << 40));
    if (keys[i] >= (uint64_t)-2 || keys[i] == 0) keys[i] = 0x5555555555555555ULL + i;
  }
  cpu_set_t aff;
  sched_getaffinity(0, sizeof(aff), &aff);
  std::vector<int> cpus;
  for (int c = 0; c < CPU_SETSIZE; ++c)
    if (CPU_ISSET(c, &aff)) cpus.push_back(c);
  // KV(10GiB*10/4096) -> src/cceh CCEH(26214400): depth 14 (test_KV's table)
  pmdfc_host::GpuCCEH kv(26214400, false, cfg, 0);
  // an op's round trip by phase, per op, over one phase of the run
  // (BatchCore::phase_times: queue = waiting for a ring place, gpu = published
  // -> result seen, deliver = seen -> returned); batches = device chunks
  std::string phases;
  auto phase_json = [&](const char* name, const pmdfc_host::BatchCore::PhaseTimes& a,
                        const pmdfc_host::BatchCore::PhaseTimes& b) {
    const double nb = (double)std::max<uint64_t>(1, b.batches - a.batches);
    const double no = (double)std::max<uint64_t>(1, b.ops - a.ops);
    char buf[800];
    snprintf(buf, sizeof buf, "%s\"%s\": {\"batches\": %llu, \"ops_per_batch\": %.1f, \"queue_us_per_op\": %.2f, "
             "\"gpu_us_per_op\": %.2f, \"deliver_us_per_op\": %.2f, \"chunk_read_us\": %.2f, \"chunk_cbf_us\": %.2f, "
             "\"chunk_apply_us\": %.2f, \"chunk_answer_us\": %.2f, \"wave_life_us\": %.0f, \"empty_polls\": %llu, "
             "\"wave_starts\": %llu, \"flood_batches\": %llu, \"flood_ops\": %llu, \"flood_us\": %.0f, \"stop_us\": %.0f}", phases.empty() ? "" : ", ", name,
             (unsigned long long)(b.batches - a.batches), (b.ops - a.ops) / nb, (b.queue_us - a.queue_us) / no,
             (b.gpu_us - a.gpu_us) / no, (b.deliver_us - a.deliver_us) / no, (b.dev_read_us - a.dev_read_us) / nb,
             (b.dev_cbf_us - a.dev_cbf_us) / nb, (b.dev_apply_us - a.dev_apply_us) / nb,
             (b.dev_answer_us - a.dev_answer_us) / nb, b.dev_life_us - a.dev_life_us,
             (unsigned long long)(b.dev_empty_polls - a.dev_empty_polls),
             (unsigned long long)(b.wave_starts - a.wave_starts),
             (unsigned long long)(b.flood_batches - a.flood_batches), (unsigned long long)(b.flood_ops - a.flood_ops),
             b.flood_us - a.flood_us, b.stop_us - a.stop_us);
    phases += buf;
  };
  auto run = [&](auto body) {
    std::vector<std::thread> th;
    const double t0 = now_s();
    for (int t = 0; t < T; ++t) {
      th.emplace_back([&, t] { body(t); });
      cpu_set_t one;
      CPU_ZERO(&one);
      CPU_SET(cpus[t % cpus.size()], &one);
      pthread_setaffinity_np(th.back().native_handle(), sizeof(one), &one);
    }
    for (auto& x : th) x.join();
    return now_s() - t0;
  };
  const uint64_t b0 = kv.batches_launched();
  auto p0 = kv.core().phase_times();
  const double ti = run([&](int t) {
    for (size_t i = per * t; i < per * (t + 1); ++i) kv.Insert(keys[i], reinterpret_cast<Value_t>(keys[i]));
  });
  const uint64_t b1 = kv.batches_launched();
  auto p1 = kv.core().phase_times();
  phase_json("insert", p0, p1);
  std::vector<size_t> failed(T, 0);
  const double tg = run([&](int t) {
    size_t f = 0;
    for (size_t i = per * t; i < per * (t + 1); ++i) f += kv.Get(keys[i]) != reinterpret_cast<Value_t>(keys[i]);
    failed[t] = f;
  });
  const uint64_t b2 = kv.batches_launched();
  auto p2 = kv.core().phase_times();
  phase_json("get", p1, p2);
  const double tm = run([&](int t) {
    size_t f = 0;
    for (size_t j = 0; j < per; ++j) {
      const size_t i = per * t + j;
      if (j & 1) {
        f += kv.Get(keys[i]) != reinterpret_cast<Value_t>(keys[i]);
      } else {
        kv.Insert(keys[n + i], reinterpret_cast<Value_t>(keys[n + i]));
      }
    }
    failed[t] += f;
  });
  const uint64_t b3 = kv.batches_launched();
  auto p3 = kv.core().phase_times();
  phase_json("mixed", p2, p3);
  // ---- async: each thread keeps up to W ops outstanding
  // a caller's window: ops it queued (its own word) and ops completed (one
  // line per caller, no false sharing between callers).  The callbacks all
  // run on the index's one control thread (batch_core.h), so the completed
  // count is a single-writer word: a plain store, not a locked add on a line
  // the caller keeps reading (FE_CB=rmw: a locked add, A/B)
  struct alignas(64) Win {
    uint64_t queued = 0;
    alignas(64) std::atomic<uint64_t> done{0};
    std::atomic<size_t> bad{0};
  };
  std::vector<Win> win(T);
  struct Ctx {
    Win* w;
    uint64_t want;  // expected Get value, or ~0 for an Insert
  };
  std::vector<Ctx> ctx(2 * n);
  // (several delivery threads run callbacks concurrently: a locked add then)
  static const bool cb_rmw = (getenv("FE_CB") && std::string(getenv("FE_CB")) == "rmw") || cfg.delivery_threads > 1 ||
                             getenv("PMDFC_DELIVERY_THREADS");
  auto cb = [](void* c, uint8_t st, uint64_t v) {
    Ctx* x = static_cast<Ctx*>(c);
    if (x->want == ~0ULL ? (st != PMDFC_ST_INSERTED) : (st != PMDFC_ST_HIT || v != x->want)) x->w->bad++;
    if (cb_rmw) x->w->done.fetch_add(1, std::memory_order_release);
    else x->w->done.store(x->w->done.load(std::memory_order_relaxed) + 1, std::memory_order_release);
  };
  auto& core = kv.core();
  // a thread with its window full waits as an RDMA poll thread waiting on its
  // completion channel would: a short spin, then short sleeps (the GPU box
  // grants this process a 16-CPU quota: 32 callers spinning through it get
  // every thread of the process throttled, the index's control thread
  // included), and once full it resumes when `hyst` places are free again
  // (FE_SPIN / FE_HYST: A/B knobs)
  const int spin_max = getenv("FE_SPIN") ? atoi(getenv("FE_SPIN")) : 64;
  const uint64_t hyst = getenv("FE_HYST") ? (uint64_t)atoi(getenv("FE_HYST")) : 32;
  auto wait_until = [&](auto pred) {
    for (int spin = 0; !pred(); ++spin) {
      if (spin < spin_max) __builtin_ia32_pause();
      else std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
  };
  auto wait_room = [&](Win& w) {
    if (w.queued - w.done.load(std::memory_order_acquire) < (uint64_t)W) return;
    wait_until([&] { return w.queued - w.done.load(std::memory_order_acquire) <= (uint64_t)W - hyst; });
  };
  auto drain = [&](Win& w) { wait_until([&] { return w.done.load(std::memory_order_acquire) >= w.queued; }); };
  const uint64_t b4 = kv.batches_launched();
  auto p4 = kv.core().phase_times();
  const double tai = run([&](int t) {
    Win& w = win[t];
    for (size_t i = 2 * n + per * t; i < 2 * n + per * (t + 1); ++i) {
      wait_room(w);
      w.queued++;
      ctx[i - 2 * n] = Ctx{&w, ~0ULL};
      core.InsertAsync(keys[i], keys[i], cb, &ctx[i - 2 * n]);
    }
    drain(w);
  });
  const uint64_t b5 = kv.batches_launched();
  auto p5 = kv.core().phase_times();
  phase_json("async_insert", p4, p5);
  const double tag = run([&](int t) {
    Win& w = win[t];
    for (size_t i = 2 * n + per * t; i < 2 * n + per * (t + 1); ++i) {
      wait_room(w);
      w.queued++;
      ctx[i - 2 * n] = Ctx{&w, keys[i]};
      core.GetAsync(keys[i], cb, &ctx[i - 2 * n]);
    }
    drain(w);
  });
  const uint64_t b6 = kv.batches_launched();
  auto p6 = kv.core().phase_times();
  phase_json("async_get", p5, p6);
  const double tam = run([&](int t) {
    Win& w = win[t];
    for (size_t j = 0; j < per; ++j) {
      const size_t i = 2 * n + per * t + j;
      wait_room(w);
      w.queued++;
      if (j & 1) {
        ctx[i - 2 * n] = Ctx{&w, keys[i]};
        core.GetAsync(keys[i], cb, &ctx[i - 2 * n]);
      } else {
        ctx[n + i - 2 * n] = Ctx{&w, ~0ULL};
        core.InsertAsync(keys[n + i], keys[n + i], cb, &ctx[n + i - 2 * n]);
      }
    }
    drain(w);
  });
  const uint64_t b7 = kv.batches_launched();
  phase_json("async_mixed", p6, kv.core().phase_times());
  size_t fs = 0, afs = 0;
  for (auto f : failed) fs += f;
  for (auto& w : win) afs += w.bad.load();
  printf("{\"threads\": %d, \"serve_waves\": %u, \"ops_per_thread\": %zu, \"max_batch\": %u, \"window\": %d, "
         "\"insert_mops\": %.3f, \"get_mops\": %.3f, \"mixed_mops\": %.3f, "
         "\"insert_avg_batch\": %.1f, \"get_avg_batch\": %.1f, \"mixed_avg_batch\": %.1f, "
         "\"async_insert_mops\": %.3f, \"async_get_mops\": %.3f, \"async_mixed_mops\": %.3f, "
         "\"async_insert_avg_batch\": %.1f, \"async_get_avg_batch\": %.1f, \"async_mixed_avg_batch\": %.1f, "
         "\"failedSearch\": %zu, \"async_failed\": %zu, \"failed_ops\": %llu, \"cpus_available\": %zu, "
         "\"phases\": {%s}}\n",
         T, kv.core().serve_waves(), per, cfg.max_batch, W, n / ti / 1e6, n / tg / 1e6, n / tm / 1e6, (double)n / (double)(b1 - b0),
         (double)n / (double)(b2 - b1), (double)n / (double)(b3 - b2), n / tai / 1e6, n / tag / 1e6, n / tam / 1e6,
         (double)n / (double)(b5 - b4), (double)n / (double)(b6 - b5), (double)n / (double)(b7 - b6), fs, afs,
         (unsigned long long)kv.failed_ops(), cpus.size(), phases.c_str());
  return fs == 0 && afs == 0 && kv.failed_ops() == 0 ? 0 : 1;
}
