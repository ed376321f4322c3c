// batch_core.h -- the batching front-end of the drop-in index backends.
//
// The reference server calls its index per op, concurrently, from up to 32
// RDMA poll threads (server/rdma_svr.h:17-18, server/rdma_svr.cpp:755-835)
// through KV (server/KV.cpp:100-158) or NUMA_KV (server/NuMA_KV.cpp:85-155).
// BatchCore turns those calls into device batches of the C-ABI
// (pmdfc_cceh_mixed, include/pmdfc_cceh.h) and completes every call when its
// batch does.  It carries no reference type: the IHash and ICCEH facades
// (gpu_cceh.h, gpu_cceh_hybrid.h) are thin inline adapters over it, each in a
// header of its own, because the reference's IHash.h and ICCEH.h share one
// include guard and never meet in one translation unit.
//
// Pipeline: callers reserve places in a bounded ring with one atomic add (a
// run of n ops reserves n consecutive places) and publish each op with a
// per-place sequence number -- no lock, no per-op wake-up.  A launcher thread
// takes the longest published prefix (up to max_batch ops) into one of two
// staging slots (pinned host + device buffers) as soon as a slot is free (no
// lingering by default: while one batch runs on the GPU the next one
// accumulates by itself) and enqueues one H2D copy, the batch and one D2H copy
// on the core's stream; a completion thread polls the slot's event, hands the
// results to the callers and frees the slot.  Batch i+1 is staged while batch
// i runs.  Ring order is the serial order the device applies, a valid
// linearisation of the concurrent reference (CCEH_hybrid.cpp:107-298 is
// internally synchronised and unordered).  The worker threads spin while
// there is work and nap when idle; a caller wakes a napping launcher only
// then.  Only the callers of a finished batch are woken (one waiter object
// per calling thread, which spins briefly before it sleeps).
//
// Blocking per-op calls are bounded by the callers' concurrency: 32 callers
// keep at most 32 ops in flight, so throughput is 32 / round-trip time.  A
// server whose poll threads need not block on each op (an RDMA handler can
// post its reply from a completion) uses InsertAsync / GetAsync: the op is
// queued and a callback runs on the completion thread when its batch is done.
//
// Errors never escape the worker threads: a failed HIP call or engine call
// marks every op of its batch with status kBatchFailed (0xFF), records a
// sticky message (last_error()) and the core keeps serving.  Per-op failures
// reported by the engine (CAPACITY, UNSPLITTABLE, DEPTH_LIMIT, RESERVED_KEY,
// SPLIT_LOST, ...) are counted per status (failure_count()) and the first of
// each kind is logged; BatchingConfig::fatal_on_error aborts instead, for a
// server that must not lose a write silently.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/pmdfc_cceh.h"

namespace pmdfc_host {

constexpr uint8_t kBatchFailed = 0xFF;  // status of an op whose whole batch failed

// completion callback of the async calls: status (PMDFC_ST_*, or kBatchFailed)
// and the Get value (0 for inserts and misses); runs on the completion thread
typedef void (*OpCallback)(void* ctx, uint8_t status, uint64_t value);

struct BatchingConfig {
  uint32_t max_batch = 1 << 16;  // ops per device batch
  uint32_t linger_us = 0;        // wait up to this long for more ops before launching a partial batch
  int device = 0;
  bool upsert = false;           // last-writer-wins Insert (PMDFC_CFG_UPSERT)
  bool fatal_on_error = false;   // abort() on the first failed op instead of counting it
  // a blocked caller spins this long, then sleeps until its batch completes.
  // Short by default: many callers spinning through a batch round trip
  // (tens of us) starve the launcher and completion threads, and on a
  // CPU-quota'd host get the whole process throttled.
  uint32_t caller_spin_us = 10;
  // batches of at most this many ops skip both copies: the engine's one-launch
  // small-batch kernel reads and writes the pinned staging block directly
  // (each of its blocks reads every key of the batch, so the cut stays small)
  uint32_t zero_copy_max = 64;
};

class BatchCore {
 public:
  // initial_depth: pmdfc_depth_for_src / _hybrid of the reference's initCap
  BatchCore(uint32_t initial_depth, BatchingConfig cfg, uint64_t max_segments);
  ~BatchCore();
  BatchCore(const BatchCore&) = delete;
  BatchCore& operator=(const BatchCore&) = delete;

  // ---- per-op calls (any thread, blocking until the op's batch completes)
  // count_bf: the op also increments the attached counting BF (KV::Insert's
  // bf->Insert, server/KV.cpp:113-114); extent heads do not (KV::InsertExtent,
  // server/KV.cpp:129-143, never touches the filter)
  uint8_t Insert(uint64_t key, uint64_t value, bool count_bf = true);
  uint8_t Get(uint64_t key, uint64_t* value);

  // ---- runs: n ops enqueued contiguously (in this order, no op of another
  // thread in between), one wait for all of them.  Returns the number of ops
  // whose status is a failure (see is_failure).
  uint64_t InsertRun(const uint64_t* keys, const uint64_t* values, uint8_t* status, uint64_t n,
                     bool count_bf = true);
  uint64_t GetRun(const uint64_t* keys, uint64_t* values, uint8_t* status, uint64_t n);

  // ---- asynchronous per-op calls: queue the op and return; cb(ctx, status,
  // value) runs on the completion thread once its batch is done.  Ops queued
  // by one thread apply in the order it queued them.  A callback may queue
  // more async ops: they are held on the completion thread and published
  // after the batch's callbacks, as ring places free up (never waiting for a
  // place, which only the completion thread can free).  A callback must not
  // make a blocking call (Insert, Get, the runs, flush, the introspection
  // calls): only the completion thread completes batches.  Such a call fails
  // at once (kBatchFailed / an error value, last_error()) instead of
  // deadlocking.
  void InsertAsync(uint64_t key, uint64_t value, OpCallback cb, void* ctx, bool count_bf = true);
  void GetAsync(uint64_t key, OpCallback cb, void* ctx);

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
  pmdfc_cceh_t* engine() { return t_; }
  uint64_t batches_launched() const { return launched_.load(); }
  uint64_t ops_completed() const { return done_seq_.load(); }
  uint64_t failed_ops() const { return failed_.load(); }
  uint64_t failure_count(uint8_t status) const { return fail_by_st_[status].load(); }
  std::string last_error() const;
  static bool is_failure(uint8_t op, uint8_t status);
  // where a batch's round trip goes, summed over the batches so far (us):
  // queue = its first op published -> the launcher takes the batch (waiting
  // for a free slot); stage = staging + the engine's launch calls; gpu =
  // launched -> the completer sees its event (device time + queueing behind
  // the other slot's batch); deliver = results handed out and callers woken
  struct PhaseTimes {
    uint64_t batches = 0, ops = 0;
    double queue_us = 0, stage_us = 0, gpu_us = 0, deliver_us = 0;
  };
  PhaseTimes phase_times() const;

 private:
  struct Waiter;
  struct Req {
    uint8_t op, cbf;
    uint64_t key, value;
    uint64_t* out;   // Get value (may be null)
    uint8_t* st;     // status (null for async ops)
    Waiter* w;       // blocking ops: the caller's waiter; async ops: null
    OpCallback cb;   // async ops
    void* ctx;
    double t_pub;    // when it was published (us; phase_times)
  };
  // staging of one batch: one pinned host block and one device block, each
  // laid out [keys n][values n][ops n][cbf n] in and [values n][status n] out,
  // so a batch costs one H2D and one D2H copy
  struct Slot {
    uint8_t* h_in = nullptr;
    uint8_t* h_out = nullptr;
    uint8_t* d_in = nullptr;
    uint8_t* d_out = nullptr;
    uint8_t* m_in = nullptr;    // device mappings of h_in / h_out (zero-copy batches)
    uint8_t* m_out = nullptr;
    void* ev = nullptr;
    std::vector<Req> reqs;
    double t_pub = 0, t_take = 0, t_launch = 0;  // phase stamps of the batch in the slot (us)
    std::atomic<int> state{0};  // kFree, kLaunched (the completer's), kExit
    bool failed = false;        // launch failed: the completion thread fails the ops
  };

  bool enqueue(const Req* r, uint64_t n, Waiter* w);  // blocking: waits for the ops (false: refused)
  bool on_completer() const;
  void publish(const Req* r, uint64_t n);               // reserve, write, publish
  void publish_async(const Req& r);                     // async op: publish, or hold it (completion thread)
  bool try_publish(const Req* r, uint64_t n);           // only if n places are free now (no waiting)
  void drain_held();                                    // (completion thread) publish what fits of held_
  void launcher();
  void completer();
  void stage(Slot& s);      // throws on HIP / engine failure
  void complete(Slot& s);
  void set_error(const std::string& e);
  void wake_launcher();
  void wake_completer();
  static Waiter& my_waiter();

  pmdfc_cceh_t* t_ = nullptr;
  pmdfc_cbf_t* bf_ = nullptr;
  BatchingConfig cfg_;
  void* stream_ = nullptr;
  Slot slot_[2];

  // the ring: place p holds an op when seq_[p & mask] == p + 1; it is free
  // for the op of place p when seq_[p & mask] == p (Vyukov's bounded queue)
  std::vector<Req> ring_;
  std::unique_ptr<std::atomic<uint64_t>[]> seq_;
  uint64_t mask_ = 0;
  alignas(64) std::atomic<uint64_t> tail_{0};  // places reserved
  alignas(64) std::atomic<uint64_t> head_{0};  // places taken by the launcher
  alignas(64) std::atomic<bool> launcher_napping_{false};
  std::mutex nap_mu_;
  std::condition_variable nap_cv_;
  alignas(64) std::atomic<bool> completer_napping_{false};
  std::mutex cnap_mu_;
  std::condition_variable cnap_cv_;
  std::atomic<bool> stop_{false};
  std::thread launch_th_, cmpl_th_;
  std::atomic<std::thread::id> cmpl_id_{};
  std::vector<Waiter*> wake_list_;      // (completer thread) sleepers of the batch just completed
  std::vector<Req> held_;               // (completer thread) async ops queued by callbacks, in order
  size_t held_head_ = 0;                // first of held_ not yet published
  uint64_t* fa_dev_ = nullptr;          // FindAnyway: device {key, value, status}
  std::mutex dev_mu_;                   // the stream (launcher vs pack_counting_bf)

  std::atomic<uint64_t> done_seq_{0};   // ops completed (batches complete in order)
  std::atomic<uint64_t> launched_{0};
  std::atomic<uint64_t> failed_{0};
  std::atomic<uint64_t> fail_by_st_[256];
  std::atomic<uint32_t> logged_{0};     // statuses already logged (bit per status < 32)
  mutable std::mutex ph_mu_;
  PhaseTimes ph_;                       // (completer thread)
  mutable std::mutex err_mu_;
  std::string err_;
};

}  // namespace pmdfc_host
