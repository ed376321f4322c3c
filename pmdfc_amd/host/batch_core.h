// batch_core.h -- the per-op front-end of the drop-in index backends.
//
// The reference server calls its index per op, concurrently, from up to 32
// RDMA poll threads (server/rdma_svr.h:17-18, server/rdma_svr.cpp:755-835)
// through KV (server/KV.cpp:100-158) or NUMA_KV (server/NuMA_KV.cpp:85-155).
// BatchCore serves those calls on the GPU.  It carries no reference type: the
// IHash and ICCEH facades (gpu_cceh.h, gpu_cceh_hybrid.h) are thin inline
// adapters over it, each in a header of its own, because the reference's
// IHash.h and ICCEH.h share one include guard and never meet in
// one translation unit.
//
// Served mode (no launcher, no completion thread in an op's path):
//   * a caller reserves places in a ring of requests in coherent pinned host
//     memory with one atomic add (a run of n ops reserves n consecutive
//     places), writes each op and then its sequence word;
//   * persistent device waves (k_serve, include/pmdfc_cceh.h
//     pmdfc_cceh_serve_start_n) poll the rings, each wave its own: it takes
//     the longest published prefix (at most 64 ops) in ring order, applies it
//     exactly as the serial reference would (the engine's one-wave
//     small-batch path), and writes each op's {value, status} into a
//     response ring, then its sequence word;
//   * the caller spins on that word (briefly, then sleeping) and reads its
//     result itself.
// With W = BatchingConfig::serve_waves rings, an op goes to the ring of its
// key's hash prefix (the top log2 W bits, i.e. the directory buckets that
// ring's wave owns), so one key -- and one segment -- always meets the same
// ring.  Each ring's order is the serial order of its keys, and ops of
// different rings touch disjoint segments and commute: the device applies a
// valid linearisation of the concurrent reference (CCEH_hybrid.cpp:107-298
// is internally synchronised and unordered).  One control thread beats a
// heartbeat (the waves exit if the host stops beating), runs the callbacks of
// the async calls in ring order, and frees ring places once their results
// are read.
//
// Blocking per-op calls are bounded by the callers' concurrency: 32 callers
// keep at most 32 ops in flight, so throughput is 32 / round-trip time.  A
// server whose poll threads need not block on each op (an RDMA handler can
// post its reply from a completion) uses InsertAsync / GetAsync: the op is
// queued and a callback runs on the control thread when its result is back.
//
// Calls that need the whole engine (Utilization, Capacity, FindAnyway, the
// counting-BF pack and attach) wait for every op queued before them, stop
// the device wave, run on the engine's stream, and start it again.
//
// Errors never escape a call: a failed HIP or engine call fails the ops it
// concerns with status kBatchFailed (0xFF) and records a sticky message
// (last_error()).  Per-op failures reported by the engine (CAPACITY,
// UNSPLITTABLE, DEPTH_LIMIT, RESERVED_KEY, ...) are counted per status
// (failure_count()) and the first of each kind is logged;
// BatchingConfig::fatal_on_error aborts instead, for a server that must not
// lose a write silently.
#pragma once
#include <atomic>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/pmdfc_cceh.h"

namespace pmdfc_host {

constexpr uint8_t kBatchFailed = 0xFF;  // status of an op that could not be served

// completion callback of the async calls: status (PMDFC_ST_*, or kBatchFailed)
// and the Get value (0 for inserts and misses); runs on the control thread
typedef void (*OpCallback)(void* ctx, uint8_t status, uint64_t value);

struct BatchingConfig {
  uint32_t max_batch = 1 << 16;  // the engine's largest batch (its workspaces)
  uint32_t linger_us = 0;        // (unused in served mode; kept for source compatibility)
  int device = 0;
  bool upsert = false;           // last-writer-wins Insert (PMDFC_CFG_UPSERT)
  bool fatal_on_error = false;   // abort() on the first failed op instead of counting it
  // a blocked caller spins this long on its result word, then sleeps until the
  // control thread sees answers arrive (a host with fewer CPUs than callers,
  // such as the GPU box's 16-CPU share under 32 callers, cannot afford every
  // caller spinning through a round trip)
  uint32_t caller_spin_us = 10;
  uint32_t zero_copy_max = 64;   // (unused in served mode)
  uint32_t ring_size = 1 << 13;  // request / response ring places (a power of two)
  // a backlog of this many unanswered places (async floods: callers with
  // hundreds of ops in flight each) is served by the control thread as large
  // batches through the engine's batch path (the wave stopped meanwhile);
  // 0: never.  Blocking callers (one op in flight each) never reach it.
  uint32_t flood_ops = 1024;
  // serving waves, each owning a hash-prefix range of the directory buckets
  // with a ring of its own (a power of two, clamped to the table's starting
  // bucket count).  32 blocking callers on the GPU box's 16-CPU share: 1
  // wave 1.63 Mops/s mixed, 8 waves 2.33, 16 waves 2.59 (bench config 8)
  uint32_t serve_waves = 8;
  // threads that run the async callbacks and free ring places: the control
  // thread and delivery_threads - 1 more, ring g's on thread g % delivery_threads
  // (at most serve_waves).  1: every callback on the control thread, one at a
  // time; more: the callbacks of different rings run concurrently (a
  // callback then must not assume it is alone)
  uint32_t delivery_threads = 1;
};

class BatchCore {
 public:
  // initial_depth: pmdfc_depth_for_src / _hybrid of the reference's initCap
  BatchCore(uint32_t initial_depth, BatchingConfig cfg, uint64_t max_segments);
  ~BatchCore();
  BatchCore(const BatchCore&) = delete;
  BatchCore& operator=(const BatchCore&) = delete;

  // ---- per-op calls (any thread, blocking until the op is applied)
  // count_bf: the op also increments the attached counting BF (KV::Insert's
  // bf->Insert, server/KV.cpp:113-114); extent heads do not (KV::InsertExtent,
  // server/KV.cpp:129-143, never touches the filter)
  uint8_t Insert(uint64_t key, uint64_t value, bool count_bf = true);
  uint8_t Get(uint64_t key, uint64_t* value);

  // ---- runs: n ops enqueued contiguously per ring (in this order, no op of
  // another thread in between within a ring; a run longer than half a ring
  // goes in such pieces), one wait for all of them.  Returns the number of
  // ops whose status is a failure (see is_failure).
  uint64_t InsertRun(const uint64_t* keys, const uint64_t* values, uint8_t* status, uint64_t n,
                     bool count_bf = true);
  uint64_t GetRun(const uint64_t* keys, uint64_t* values, uint8_t* status, uint64_t n);
  // interleaved Inserts and Gets (ops[i]: PMDFC_OP_INSERT / PMDFC_OP_GET), one
  // run like the two above; places (nullable) receives each op's ring place
  // | ring << 48, i.e. its position in the serial order of its ring
  uint64_t MixedRun(const uint8_t* ops, const uint64_t* keys, const uint64_t* values_in, uint64_t* values_out,
                    uint8_t* status, uint64_t n, uint64_t* places = nullptr, bool count_bf = true);

  // ---- asynchronous per-op calls: queue the op and return; cb(ctx, status,
  // value) runs on the control thread (or the delivery thread of the op's
  // ring, BatchingConfig::delivery_threads) once its result is back.  Ops queued by
  // one thread apply in the order it queued them.  A callback may queue more
  // async ops: they are held on the control thread and published after the
  // callbacks of the round, as ring places free up (never waiting for a
  // place, which only the control thread frees).  A callback must not make a
  // blocking call (Insert, Get, the runs, flush, the introspection calls):
  // such a call fails at once (kBatchFailed / an error value, last_error())
  // instead of deadlocking.
  void InsertAsync(uint64_t key, uint64_t value, OpCallback cb, void* ctx, bool count_bf = true);
  void GetAsync(uint64_t key, OpCallback cb, void* ctx);
  // either of the two; returns the op's ring place | ring << 48 (its
  // position in its ring's serial order), or ~0 when queued from a callback
  // (placed later)
  uint64_t SubmitAsync(uint8_t op, uint64_t key, uint64_t value, OpCallback cb, void* ctx, bool count_bf = true);

  // wait until every op enqueued before this call has completed (false, and
  // no wait, from a completion callback)
  bool flush();

  // ---- counting BF of KV (server/KV.cpp:113-121).  The filter must live on
  // the same device and outlive the core's use of it.
  void attach_counting_bf(pmdfc_cbf_t* f);
  // ToOrdinaryBloomFilter after the ops enqueued so far (rdma_svr.cpp:256-264)
  int pack_counting_bf();

  // ---- introspection (synchronous; from a completion callback they fail:
  // Utilization -1, FindAnyway kBatchFailed, Capacity 0)
  double Utilization();
  // CCEH::FindAnyway after every op enqueued so far: PMDFC_ST_HIT / _MISS
  // (kBatchFailed on a HIP failure); the first copy in slot order
  uint8_t FindAnyway(uint64_t key, uint64_t* value);
  uint64_t Capacity();
  // pmdfc_cceh_stats / pmdfc_cceh_dump after every op enqueued so far
  int Stats(pmdfc_cceh_stats_t* out);
  // Dump: sized and filled under one stop of the waves.  dir_cap: entries
  // dir_canon holds; seg_cap: segments local_depth / prefix hold (keys /
  // values: seg_cap * 1024).  *nseg_out / *ndir_out receive the sizes; a
  // table larger than the buffers returns PMDFC_ERR_SIZE with nothing written
  int Dump(uint64_t dir_cap, uint64_t seg_cap, uint32_t* dir_canon, uint32_t* local_depth, uint64_t* prefix,
           uint64_t* keys, uint64_t* values, uint64_t* nseg_out, uint64_t* ndir_out);
  // chunks after which a serving wave reloaded its LDS copy of the headers
  uint64_t header_reloads() const;
  uint32_t serve_waves() const { return W_; }
  pmdfc_cceh_t* engine() { return t_; }
  uint64_t batches_launched() const;  // device chunks served by the wave + flood batches
  uint64_t ops_completed() const;
  uint64_t failed_ops() const { return failed_.load(); }
  uint64_t failure_count(uint8_t status) const { return fail_by_st_[status].load(); }
  std::string last_error() const;
  static bool is_failure(uint8_t op, uint8_t status);
  // where an op's round trip goes, summed over the ops so far (us): queue =
  // reserve -> published (waiting for a free ring place); gpu = published ->
  // its result word seen (the device wave's polling, the chunk before it and
  // its own); deliver = seen -> returned (reading the result; for an async op
  // its callback).  stage: 0 (nothing is staged).  batches: device chunks.
  // dev_*: the device wave's own time per chunk phase, summed over chunks
  // (us): reading the requests from the ring, counting the BF, applying,
  // answering (results, sequence words, head).
  struct PhaseTimes {
    uint64_t batches = 0, ops = 0;
    double queue_us = 0, stage_us = 0, gpu_us = 0, deliver_us = 0;
    double dev_read_us = 0, dev_cbf_us = 0, dev_apply_us = 0, dev_answer_us = 0;
    double dev_life_us = 0;          // the waves' lifetimes
    uint64_t dev_empty_polls = 0;    // polls of the ring that found no op
    uint64_t wave_starts = 0;        // launches of the device wave
    uint64_t flood_batches = 0, flood_ops = 0;  // places served as large batches (BatchingConfig::flood_ops)
    double flood_us = 0, stop_us = 0;           // time in those batches; in stopping the wave
  };
  PhaseTimes phase_times() const;

 private:
  struct Async {
    OpCallback cb;  // null: a blocking op (its caller reads the result)
    void* ctx;
    uint8_t op;
    uint64_t key;
    double t_pub;
  };
  struct Op {
    uint8_t op, cbf;
    uint64_t key, value;
    OpCallback cb;  // async ops
    void* ctx;
  };
  // one serving wave's ring: its ops are those whose directory bucket it
  // owns (ring_of), so its order is the serial order of its keys
  struct Ring {
    pmdfc_serve_req* req = nullptr;    // views into the shared pinned allocations
    pmdfc_serve_resp* resp = nullptr;
    pmdfc_serve_ctl* ctl = nullptr;
    std::unique_ptr<std::atomic<uint64_t>[]> read;  // per place: p + 1 once a blocking caller read it
    std::unique_ptr<std::atomic<uint8_t>[]> asleep;  // per place: its caller sleeps on gen_
    std::vector<Async> async;                        // per place: the op's callback (cb null: blocking)
    alignas(64) std::atomic<uint64_t> tail{0};     // places reserved
    std::atomic<uint64_t> queue_ns{0};             // (the publishers' phase time: in tail's line, which they own anyway)
    // the blocking callers' phase times (per ring: one shared line for 32
    // callers bounced between them on every op)
    alignas(64) std::atomic<uint64_t> ph_ops{0}, ph_gpu_ns{0}, ph_deliver_ns{0};
    alignas(64) std::atomic<uint64_t> reclaim{0};  // places completed and read (all before it)
    uint64_t c = 0;       // (control thread) next place to free
    uint64_t seen = 0;    // (control thread) places answered, as far as it has looked
    // async ops queued by callbacks (of any delivery thread), in order;
    // published by the ring's delivery thread
    std::mutex held_mu;
    std::vector<Op> held;
    size_t held_head = 0;
    std::atomic<uint64_t> held_n{0};  // held.size() - held_head (read without the lock)
  };
  // one scan of a delivery thread's rings
  struct Scan {
    bool progress = false, pending = false, held_left = false, flood = false, wait_ops = false;
    uint64_t n_cb = 0, gpu_ns = 0;
    int nwake = 0;
  };

  void init(uint32_t initial_depth, uint64_t max_segments);  // (constructor body)
  void release();  // frees every allocation made so far (destructor; a constructor that throws)
  bool on_control() const;
  uint32_t ring_of(uint64_t key) const;
  // reserve n consecutive places of ring g, write, publish; returns the first place
  uint64_t publish(uint32_t g, const Op* r, uint64_t n, double* t_pub);
  bool try_publish(uint32_t g, const Op* r, uint64_t n);  // (control thread) only if n places are free now
  void write_place(Ring& q, uint64_t p, const Op& r, double t_pub);
  void drain_held(uint32_t g);
  // wait for the results of places [p0, p0 + n) of ring g (ops r[k] / outputs
  // at idx[k], or k when idx is null), store them, mark them read; returns
  // the failures among them
  uint64_t await(uint32_t g, uint64_t p0, uint64_t n, const Op* r, const uint64_t* idx, uint8_t* status,
                 uint64_t* values, double t_pub);
  uint64_t run(const Op* rs, uint64_t n, uint8_t* status, uint64_t* values,
               uint64_t* places = nullptr);  // publish + await, in pieces
  void control();
  void deliver(uint32_t d);  // delivery thread d >= 1: rings g with g % D_ == d
  void scan_ring(uint32_t g, double t_scan, Scan& o);
  void finish_scan(const Scan& o, double t_scan);
  void count_failure(uint8_t op, uint8_t st, uint64_t key);
  void set_error(const std::string& e);
  bool serve_flood(uint32_t g);  // (control thread, srv_mu_ held, no wave) one large batch from ring g
  bool start_server();   // launch the device waves (srv_mu_ held)
  bool stop_server();    // stop them and wait for them (srv_mu_ held)
  template <class F>
  bool with_engine(F f);  // flush, stop the waves, f(stream), start them again

  pmdfc_cceh_t* t_ = nullptr;
  pmdfc_cbf_t* bf_ = nullptr;
  BatchingConfig cfg_;
  void* stream_ = nullptr;  // the device waves' stream
  void* sync_ = nullptr;    // the synchronous calls' stream

  pmdfc_serve_req* req_ = nullptr;    // pinned, coherent, device-mapped: W rings of R places
  pmdfc_serve_resp* resp_ = nullptr;
  pmdfc_serve_ctl* ctl_ = nullptr;    // W control blocks
  uint64_t R_ = 0, mask_ = 0;
  uint32_t W_ = 1, lw_ = 0;           // serving waves (rings), log2
  std::vector<std::unique_ptr<Ring>> rings_;

  std::atomic<bool> stop_{false};
  std::thread ctl_th_;
  uint32_t D_ = 1;                 // delivery threads (the control thread is thread 0)
  std::vector<std::thread> dl_th_;
  std::mutex srv_mu_;             // starts / stops of the device waves
  std::atomic<bool> running_{false};  // (changed under srv_mu_) the waves were launched and not yet stopped
  std::atomic<uint64_t> chunks_base_{0};  // chunks of the waves before the current ones
  std::atomic<uint64_t> reloads_base_{0};  // header reloads of the waves before the current ones
  std::atomic<uint64_t> prof_base_[6] = {};  // ctl->prof of the waves before the current ones
  std::atomic<uint64_t> starts_{0};
  // blocked callers past their spin sleep on gen_ (futex); the control thread
  // bumps it and wakes the sleepers when answers arrived for sleeping callers
  alignas(64) std::atomic<uint32_t> gen_{0};
  std::atomic<int32_t> sleepers_{0};
  // publishers waiting for free ring places sleep on rgen_ (bumped and woken
  // by the control thread when it frees places)
  alignas(64) std::atomic<uint32_t> rgen_{0};
  std::atomic<int32_t> rwaiters_{0};
  uint64_t* fa_dev_ = nullptr;    // FindAnyway: device {key, value, status}
  // flood batches: pinned staging (keys, values, ops, cbf ops | values, statuses) and device copies
  uint64_t fl_cap_ = 0;
  uint8_t *fl_h_in_ = nullptr, *fl_h_out_ = nullptr, *fl_d_in_ = nullptr, *fl_d_out_ = nullptr;
  std::atomic<uint64_t> fl_batches_{0}, fl_ops_{0}, fl_ns_{0}, stop_ns_{0};

  std::atomic<uint64_t> failed_{0};
  std::atomic<uint64_t> fail_by_st_[256];
  std::atomic<uint32_t> logged_{0};  // statuses already logged (bit per status < 32)
  std::atomic<uint64_t> ph_ops_{0};
  std::atomic<uint64_t> ph_queue_ns_{0}, ph_gpu_ns_{0}, ph_deliver_ns_{0};
  mutable std::mutex err_mu_;
  std::string err_;
};

}  // namespace pmdfc_host
