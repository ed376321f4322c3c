// cceh_engine.hip -- host side of the MI355X batched CCEH engine and the
// C-ABI declared in include/pmdfc_cceh.h.
//
// The engine owns its HBM (segment arena, occupancy bitmaps, local depths,
// bucketed directory, batch workspaces) and drives the kernels of
// cceh_kernels.hip / bucket.hip.  Every batched entry point only ENQUEUES work
// on the caller's stream; nothing on the Insert/Get/mixed path reads device
// state back (bucket.hip has the details of every pass):
//   Insert : k_part -> k_apply_fast (first pass; requests and reserves its
//            splits) -> k_split -> k_apply_parked -> k_bucket (final pass)
//   mixed  : k_mixed_prep -> k_mixed_get -> k_part -> the
//            same bucket passes (gated insert-only / mixed variants) ->
//            k_mixed_verify
//   <= 64 ops : k_mixed_tiny; <= 256: k_mixed_small (1 launch)
//   <= 8192   : k_part (one block) -> k_medium (2 launches)
//   Get    : k_get_u (1 launch; k_flatten first after inserts)
// Splits and directory growth are decided and done on the device (per-bucket
// sub-directories), so a batch never needs a host decision; only a table
// still coarser than its bucket resolution syncs once per sub-batch.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/pmdfc_cceh.h"
#include "cceh_device.h"
#include "cceh_kernels.h"

using namespace pmdfc;

namespace {

thread_local std::string g_err;

int fail(int code, const char* what, hipError_t e = hipSuccess) {
  char buf[512];
  if (e != hipSuccess)
    snprintf(buf, sizeof buf, "%s: %s", what, hipGetErrorString(e));
  else
    snprintf(buf, sizeof buf, "%s", what);
  g_err = buf;
  return code;
}

#define HIPCHK(x)                                   \
  do {                                              \
    hipError_t e_ = (x);                            \
    if (e_ != hipSuccess) return fail(PMDFC_ERR_HIP, #x, e_); \
  } while (0)

uint32_t ceil_log2(uint64_t v) {
  uint32_t b = 0;
  while ((1ULL << b) < v) ++b;
  return b;
}

struct DevGuard {
  int prev = -1;
  explicit DevGuard(int d) {
    (void)hipGetDevice(&prev);
    if (prev != d) (void)hipSetDevice(d);
  }
  ~DevGuard() {
    int cur;
    (void)hipGetDevice(&cur);
    if (prev >= 0 && cur != prev) (void)hipSetDevice(prev);
  }
};

// Per-class kernel time from HIP events on the launching stream.  Consecutive
// intervals share their boundary event (begin() closes the open interval), and
// events skip the system-scope fence, so timing perturbs the stream as little
// as possible.
struct Timing {
  bool on = false;
  struct Rec {
    int cls;
    hipEvent_t a, b;
  };
  std::vector<Rec> recs;
  std::vector<hipEvent_t> pool;
  hipEvent_t open = nullptr;
  int open_cls = -1;
  double ms[PMDFC_K_COUNT] = {0};
  uint64_t launches[PMDFC_K_COUNT] = {0};

  hipEvent_t ev() {
    if (!pool.empty()) {
      hipEvent_t e = pool.back();
      pool.pop_back();
      return e;
    }
    hipEvent_t e;
    (void)hipEventCreateWithFlags(&e, hipEventDisableSystemFence);
    return e;
  }
  void begin(int cls, hipStream_t s) {
    if (!on) return;
    hipEvent_t e = ev();
    (void)hipEventRecord(e, s);
    if (open) recs.push_back({open_cls, open, e});
    open = e;
    open_cls = cls;
    if (recs.size() > 4096) flush_closed();
  }
  // an interval on another stream (the partition stream of insert_batches):
  // its own event pair, the open interval is untouched
  hipEvent_t span_begin(hipStream_t s) {
    if (!on) return nullptr;
    hipEvent_t e = ev();
    (void)hipEventRecord(e, s);
    return e;
  }
  void span_end(int cls, hipEvent_t a, hipStream_t s) {
    if (!on || !a) return;
    hipEvent_t e = ev();
    (void)hipEventRecord(e, s);
    recs.push_back({cls, a, e});
    if (recs.size() > 4096) flush_closed();
  }
  void end(hipStream_t s) {
    if (!on || !open) return;
    hipEvent_t e = ev();
    (void)hipEventRecord(e, s);
    recs.push_back({open_cls, open, e});
    open = nullptr;
  }
  void flush_closed() {
    // an event may close one interval and open the next: recycle it once
    std::vector<hipEvent_t> done;
    for (auto& r : recs) {
      (void)hipEventSynchronize(r.b);
      float t = 0;
      (void)hipEventElapsedTime(&t, r.a, r.b);
      ms[r.cls] += t;
      launches[r.cls] += 1;
      done.push_back(r.a);
      done.push_back(r.b);
    }
    recs.clear();
    std::sort(done.begin(), done.end());
    done.erase(std::unique(done.begin(), done.end()), done.end());
    for (auto e : done)
      if (e != open) pool.push_back(e);
  }
  ~Timing() {
    flush_closed();
    if (open) pool.push_back(open);
    for (auto e : pool) (void)hipEventDestroy(e);
  }
};

}  // namespace

// partition record buffers (records, cursors, k_part overflow slots): the
// pipelined insert path keeps up to three batches in flight
// record buffers: pmdfc_cceh_insert_batches partitions groups of up to
// kRecBufs / 2 batches ahead (pipe_group); the per-batch pipeline of the
// routed loop (pipe_batch) reuses a buffer kRecBufs batches later
#ifndef PMDFC_RECBUFS
#define PMDFC_RECBUFS 16  // (A/B builds)
#endif
constexpr uint32_t kRecBufs = PMDFC_RECBUFS;
// segments per directory bucket past which the first pass takes its wide
// variant, and past which k_apply_fb is launched for the buckets it declines
// (sub-directories past 128 entries)
constexpr uint32_t kWideSegs = 20;
constexpr uint32_t kFbSegs = 64;
constexpr uint32_t kHintMixed = 6;  // h_hint word: the tag of the last mixed batch whose mixed passes ran (k_apply<true>)
constexpr uint32_t kHintMixIns = 7;  // h_hint word: the inserts of the last mixed batch (the next batch's mode)

struct pmdfc_cceh {
  pmdfc_cceh_config_t cfg{};
  int dev = 0;
  uint32_t D0 = 1, sbits = 0, shard = 0;
  uint32_t p1 = 0;        // directory bucket bits (grows to p1max as the table deepens)
  uint32_t p1_init = 0, p1max = 0;
  uint32_t sbb = 0;       // of which sub-bucket bits (partition buckets = 2^(p1 - sbb)); per batch (batch_geometry)
  uint32_t cp = 0;        // this batch uses the coarse partition (sbb == kCpSbb, k_apply_fast_cp)
  uint32_t g_wide = 0, g_fb = 0;  // this batch's lean pass variant (batch_geometry)
  uint32_t clean_sbb = ~0u;  // the current record buffer's cursors are zero for this geometry (~0: all zero)
  size_t cblk = 0;        // cursor block per record buffer, sized for p1max
  uint64_t* hdr_tmp = nullptr;  // re-bucketing: the old headers
  uint32_t* h_depth = nullptr;  // pinned: k_min_ldep's result
  uint32_t* h_hint = nullptr;   // pinned, coherent: the segment count as k_apply_parked last set it (a hint)
  uint32_t* d_hint = nullptr;   // its device mapping
  uint32_t* minld = nullptr;     // device word: the smallest live local depth
  uint64_t rebuckets = 0;
  uint32_t parity = 0;    // batch parity: the bucket passes' per-batch words (grant shards, worklists)
  uint32_t rb = 0;        // record buffer of the next batch (0..kRecBufs-1): records, cursors, k_part overflow
  uint64_t max_segs = 0;
  uint32_t max_batch = 0;
  uint32_t chunk = 0;     // ops per k_bucket chunk (0 = kernel default)
  uint32_t upsert = 0;    // PMDFC_CFG_UPSERT: last-writer-wins Insert
  uint16_t* upos = nullptr;  // upsert: pre-batch slot of each op's key (max_batch)

  ulonglong2* pairs = nullptr;
  uint32_t* occ = nullptr;
  uint8_t* ldep = nullptr;
  uint64_t* hdr = nullptr;    // 2^p1 bucket headers (room for 2^p1max)
  uint32_t* pool = nullptr;   // sub-directories
  uint64_t pool_cap = 0;      // entries
  uint64_t seq = 0;             // mixed batch epoch
  uint64_t* iset = nullptr;     // mixed: the batch's inserted keys (2^k >= 2 max_batch slots)
  uint64_t imask = 0;
  uint32_t* ipos = nullptr;     // mixed: per set slot, the key's insert position (valid if single)
  uint32_t* islot = nullptr;    // mixed: per op, its insert's set slot (~0: none) -- the verify pass clears it
  uint32_t* icnt = nullptr;     // mixed: per set slot, 1 if the key is inserted more than once
  uint32_t* icount = nullptr;   // mixed: per 256-op block, the set slots its joining Gets claimed (k_mixed_get -> k_mixed_join -> ctl->ins_total)
  uint32_t* jbits = nullptr;    // mixed: the joining Gets' filter, one per set replica (kJoinWords)
  uint64_t last_mixed_n = 0;    // mixed: the last batch's size (with the pinned insert count: mixed_join_mode)
  uint8_t* early = nullptr;     // mixed: per op, 1 early single-copy hit, 2 linked to its insert
  uint32_t* elink = nullptr;    // mixed: per op, the linked insert's position (early 2) or the
                                // pre-batch segment's local depth (early 1)
  uint32_t* loss0 = nullptr;    // mixed: ctl->loss_events before the batch

  DevCtl* ctl = nullptr;
  DevCtl* hctl = nullptr;  // pinned mirror (stats / dump only)

  // partition records
  uint32_t cap = 0;  // record slots per partition bucket region
  ulonglong2* rkv = nullptr;   // records {key, value}
  uint32_t* rop = nullptr;
  uint16_t* robk = nullptr;    // overflow records' bucket
  uint64_t nrec = 0;           // record slots per record buffer
  uint32_t* cursor = nullptr;  // 2 x (2^(p1 - sbb) region cursors + 1 overflow cursor), by batch parity
  uint64_t* wstat = nullptr;   // per directory bucket counters (summed by stats())
  ulonglong2* wl_kv = nullptr; // parked ops per directory bucket (apply -> final pass)
  uint32_t* wl_op = nullptr;
  uint32_t* wl_n = nullptr;
  // split rounds: requests per bucket, grants, the sharded request lists
  uint2* req = nullptr;
  uint32_t* reqop = nullptr;  // batch position of each request's insert (the drop log's trigger)
  ulonglong2* drops = nullptr;  // mixed batches: the drop log (kDropLog entries)
  uint32_t* need = nullptr;
  uint32_t* gbase = nullptr;
  uint32_t* ngrant = nullptr;
  uint32_t* newoff = nullptr;
  uint64_t* gsh = nullptr;  // [2][kGShards] grant shard words, kGStride apart
  uint4* gsplit = nullptr;  // [2][kGShards][gcap] the requested splits
  uint32_t gcap = 0;
  uint32_t* act = nullptr;  // buckets with requests (k_split -> k_apply_parked)
  uint32_t* touched = nullptr;  // medium batches: partition buckets that received ops ([0]: count)
  uint32_t* povf = nullptr;     // k_part: [parity][tile][partition bucket] overflow slots
  // worklist: final-pass buckets by parity
  uint32_t* fin = nullptr;
  uint32_t* fbl = nullptr;    // [2^p1max] buckets the lean first pass declined (bit 0) and decline counts

  uint32_t* partials = nullptr;
  unsigned long long* popc = nullptr;
  uint8_t* srv_st = nullptr;     // serving wave: a chunk's statuses (64) and Get values (64)
  uint64_t* srv_vout = nullptr;
  uint64_t* stamps = nullptr;  // debug (PMDFC_STAMPS=1): [0, 8*nb) k_bucket, then k_part
  // (PMDFC_STAMP_ROT=R: R stamp sets, batch i writing set i % R, for a
  // timeline of consecutive pipelined batches; stamp_cur: this batch's)
  uint64_t* stamp_cur = nullptr;
  uint32_t stamp_rot = 1, stamp_seq = 0;

  // insert_batches: batch i+1 is partitioned on pstream while batch i is
  // applied on the caller's stream
  hipStream_t pstream = nullptr;
  hipEvent_t ev_in = nullptr, ev_part[kRecBufs] = {}, ev_done[kRecBufs] = {};
  hipEvent_t ev_gpart[2] = {}, ev_gdone[2] = {};  // pipe_group: a group's partitions / passes done
  hipEvent_t ev_minld = nullptr;  // the last rebucket_now depth copy
  bool minld_pending = false;
  bool iset_dirty = false;        // a mixed batch's prep ran without its verify pass (an error return)

  uint64_t batches = 0;
  uint64_t last_get_n = 0, last_get_blocks = 0;
  bool last_get_counted = false;
  bool count_lines = false;
  Timing timing;
  std::mutex mu;

  uint32_t* gflat = nullptr;       // flattened directory (pure Gets), 2^kFlatMaxBits entries
  uint32_t* gflat_bits = nullptr;  // its physical depth (device)
  bool flat_valid = false;         // host: no insert since the last flatten
  uint32_t flat_max = kFlatMaxBits;  // deeper directories skip the flat copy (PMDFC_FLAT_MAX)

  Geo geo() const { return Geo{hdr, pool, p1, sbits, shard, nullptr, nullptr}; }
  Geo geo_flat() const { return Geo{hdr, pool, p1, sbits, shard, gflat, gflat_bits}; }
};

struct pmdfc_bloom {
  int dev = 0;
  uint64_t nbits = 0, nwords = 0;
  uint32_t k = 0;
  uint64_t* bm = nullptr;
};

struct pmdfc_cbf {
  int dev = 0;
  uint64_t nbits = 0, nwords = 0, padded = 0;
  uint32_t k = 0;
  uint8_t* cnt = nullptr;   // padded to kCbfChunk, padding stays zero
  uint64_t* bm = nullptr;   // nwords, MSB-first
  uint32_t* flag = nullptr; // delete-batch conflict flag
};

struct pmdfc_trace {
  int dev = 0;
  // grow-only scratch
  uint64_t cap_bytes = 0, cap_lines = 0;
  size_t temp_bytes = 0;
  uint64_t* nl = nullptr;        // newline positions
  TraceLine* lines = nullptr;
  uint64_t* pages = nullptr;
  uint64_t* cum = nullptr;
  uint64_t* small = nullptr;     // [0] newline count, [1] first bad, [2..6] info
  uint64_t* tile_cnt = nullptr;  // newlines per 16 KiB text tile
  uint64_t* tile_off = nullptr;  // their inclusive scan
  void* temp = nullptr;
};

// ------------------------------------------------------------------ helpers

static int read_ctl(pmdfc_cceh* t, hipStream_t s) {
  HIPCHK(hipMemcpyAsync(t->hctl, t->ctl, sizeof(DevCtl), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  return PMDFC_OK;
}

// per parity: kPartSubs cursors per partition bucket + the overflow cursor,
// padded to 256 B so both blocks are aligned (one fill kernel per memset)
static size_t cursor_block(uint32_t npb) { return ((size_t)npb * kPartSubs + 1 + 63) & ~(size_t)63; }

// Directory bucket geometry for p1 bits: the partition buckets and their
// record regions (a sub-region holds twice its mean share plus 16).  k_part
// block b writes sub-region b % kPartSubs, so a sub-region takes the records
// of ceil(tiles / kPartSubs) whole tiles: a batch of fewer than kPartSubs
// tiles puts a full tile's share in each (an engine whose max_batch is below
// kPartSubs * kPartTile would otherwise overflow into the shared area, which
// sends every bucket of the batch past the lean first pass).
static uint32_t part_cap(uint32_t max_batch, uint32_t p1, uint32_t sbb) {
  const uint64_t npb = 1ULL << (p1 - sbb);
  const uint64_t tiles = ((uint64_t)max_batch + kPartTile - 1) / kPartTile;
  const uint64_t sub_ops = (tiles + kPartSubs - 1) / kPartSubs * kPartTile;
  const uint64_t per_sub = (sub_ops + npb - 1) / npb;
  return (uint32_t)((2 * per_sub + 16) * kPartSubs);
}

static void set_geometry(pmdfc_cceh* t, uint32_t p1) {
  t->p1 = p1;
  t->sbb = p1 > kMaxPartBits ? p1 - kMaxPartBits : 0;
  t->cap = part_cap(t->max_batch, p1, t->sbb);
  t->cp = 0;
}

// A/B knob: PMDFC_CP=0 keeps the fine partition for every batch
static bool cp_enabled() {
  static const bool on = [] {
    const char* e = getenv("PMDFC_CP");
    return !(e && e[0] == '0');
  }();
  return on;
}

// The partition geometry of ONE batch, chosen before its launches are filled:
// insert-only, non-upsert batches of a table at its bucket resolution whose
// lean pass is the narrow one take the coarse partition (2^(p1 - 3)
// partition buckets of 8 directory buckets: k_part writes runs of ~8 records
// per tile and bucket instead of ~1, k_apply_fast_cp stages them per
// workgroup); the rest the fine one.  A batch whose record buffer's cursors
// were zeroed for another geometry (the previous batch clears the next
// buffer's cursors at its own positions) zeroes them all on `s` first
// (s == null: the caller zeroes them itself).
static int batch_geometry(pmdfc_cceh* t, bool insert_only, uint64_t n, hipStream_t s, bool zero_cursors = true) {
  const uint32_t spb = __atomic_load_n(t->h_hint, __ATOMIC_RELAXED) >> t->p1;  // segments per bucket
  t->g_wide = spb > kWideSegs ? 1u : 0u;
  t->g_fb = spb > kFbSegs ? 1u : 0u;
  // records per (partition bucket, sub-region): a sub-region takes the
  // records of ceil(tiles / kPartSubs) tiles; the staging holds kCpPre, so
  // the mean must stay near 2/3 of it (1M ops at p1 = 13: 128)
  const uint64_t tiles = (n + kPartTile - 1) / kPartTile;
  const uint64_t per_sub = t->p1 > kCpSbb ? (((tiles + kPartSubs - 1) / kPartSubs) * kPartTile) >> (t->p1 - kCpSbb) : ~0ull;
  const bool cp = insert_only && !t->upsert && !t->g_wide && t->p1 == t->p1max && per_sub <= 128 && cp_enabled() &&
                  fast_first_pass();
  const uint32_t sbb = cp ? kCpSbb : (t->p1 > kMaxPartBits ? t->p1 - kMaxPartBits : 0);
  t->cp = cp ? 1u : 0u;
  t->sbb = sbb;
  t->cap = part_cap(t->max_batch, t->p1, sbb);
  if (zero_cursors && t->clean_sbb != ~0u && t->clean_sbb != sbb)
    HIPCHK(hipMemsetAsync(t->cursor + (size_t)t->rb * t->cblk, 0, t->cblk * sizeof(uint32_t), s));
  return PMDFC_OK;
}

// A table created small (CCEH_hybrid(2): 2 segments, so 2 directory buckets)
// gets finer buckets as it deepens.  While p1 < p1max, batches run as
// sub-batches of about 1,024 ops per directory bucket (A/B on CCEH_hybrid(2)
// config 2: 128 -> 5.12-5.15 Gops/s, 512 -> 5.54, 1,024 -> 5.65, 2,048 ->
// 5.48, 4,096 -> 5.27: fewer host round trips against longer final passes
// over oversized buckets) (a sub-batch sequence is
// the same serial op stream), and before each one the host reads the smallest
// live local depth (k_min_ldep) and, once every segment is at least
// sbits + p1' deep, rebuilds the bucket headers for p1' (k_rebucket: the
// sub-directories stay where they are).  The depth is the one an earlier
// call's copy left in pinned memory: the host waits for that copy only (one
// sub-batch back), so the stream keeps a sub-batch queued instead of
// draining.  Local depths only grow, so a value one sub-batch old is still a
// lower bound (init_state seeds it with the initial depth after a
// device-wide sync, so no copy of an earlier table is in flight).  A table
// at p1max pays nothing.
static int rebucket_now(pmdfc_cceh* t, hipStream_t s) {
  if (t->p1 >= t->p1max) return PMDFC_OK;
  if (t->minld_pending) HIPCHK(hipEventSynchronize(t->ev_minld));
  const uint32_t minL = __atomic_load_n(&t->h_depth[1], __ATOMIC_ACQUIRE);
  HIPCHK(hipMemsetAsync(t->minld, 0xFF, sizeof(uint32_t), s));
  launch_min_ldep(t->ldep, t->ctl, (uint32_t)t->max_segs, t->minld, s);
  HIPCHK(hipMemcpyAsync(&t->h_depth[1], t->minld, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  HIPCHK(hipEventRecord(t->ev_minld, s));
  t->minld_pending = true;
  if (minL <= t->sbits || minL > kMaxDepth) return PMDFC_OK;
  const uint32_t target = std::min<uint32_t>(t->p1max, minL - t->sbits);
  if (target <= t->p1) return PMDFC_OK;
  HIPCHK(hipMemcpyAsync(t->hdr_tmp, t->hdr, sizeof(uint64_t) << t->p1, hipMemcpyDeviceToDevice, s));
  launch_rebucket(t->hdr_tmp, t->hdr, t->p1, target, s);
  HIPCHK(hipGetLastError());
  set_geometry(t, target);
  t->flat_valid = false;
  t->rebuckets += 1;
  return PMDFC_OK;
}

// ops per sub-batch while the table is still coarser than p1max
// (PMDFC_RAMP_OPS per directory bucket, at least PMDFC_RAMP_MIN: tuning knobs)
static uint64_t ramp_batch(const pmdfc_cceh* t, uint64_t n) {
  if (t->p1 >= t->p1max) return n;
  static const uint64_t per = [] {
    const char* e = getenv("PMDFC_RAMP_OPS");
    return e && atoi(e) > 0 ? (uint64_t)atoi(e) : 1024ULL;
  }();
  static const uint64_t lo = [] {
    const char* e = getenv("PMDFC_RAMP_MIN");
    return e && atoi(e) > 0 ? (uint64_t)atoi(e) : 4096ULL;
  }();
  return std::min<uint64_t>(n, std::max<uint64_t>(per << t->p1, lo));
}

static int init_state(pmdfc_cceh* t, hipStream_t s) {
  const uint32_t n0 = 1u << (t->D0 - t->sbits);
  // (no earlier rebucket_now copy may land after the seed below: the event
  // is recorded right after that copy -- a device-wide sync would also wait
  // for every other stream, a serving wave included)
  if (t->minld_pending) HIPCHK(hipEventSynchronize(t->ev_minld));
  __atomic_store_n(&t->h_depth[1], t->D0, __ATOMIC_RELEASE);
  t->minld_pending = false;
  // the mixed batches' key set is empty between batches (each batch's verify
  // pass empties the slots it used), so a reset leaves it alone -- unless it
  // is not known empty (a new engine, or a batch that stopped between its prep
  // and verify passes): then emptied here (32 MB of fills at 1M-op batches,
  // ~20 us of a reset the bench pays every step)
  if (t->iset_dirty) {
    HIPCHK(hipMemsetAsync(t->iset, 0xFF, (t->imask + 1) * sizeof(uint64_t), s));
    HIPCHK(hipMemsetAsync(t->icnt, 0, (t->imask + 1) * sizeof(uint32_t), s));
    HIPCHK(hipMemsetAsync(t->ipos, 0xFF, (t->imask + 1) * sizeof(uint32_t), s));
    HIPCHK(hipMemsetAsync(t->jbits, 0, kJoinWords * sizeof(uint32_t), s));
    t->iset_dirty = false;
  }
  set_geometry(t, t->p1_init);
  const uint32_t region = kFixedSlot << t->p1max;  // the fixed slots come first in the pool
  const uint32_t db0 = t->D0 - t->sbits - t->p1;
  const uint32_t fixed = (t->p1 == t->p1max && db0 <= kFixedBits) ? 1u : 0u;
  // the segments, the passes' per-bucket words and the control block with
  // the hint, in ONE kernel on s: a reset queues behind the work before it
  // without a host sync (the bench resets the table at every step)
  InitZero z{};
  z.p[0] = t->cursor;
  z.n[0] = (uint64_t)kRecBufs * t->cblk;
  z.p[1] = reinterpret_cast<uint32_t*>(t->wstat);
  z.n[1] = (2ULL * kWStat) << t->p1max;
  z.p[2] = t->wl_n;
  z.n[2] = 1ULL << t->p1max;
  z.p[3] = t->fbl;
  z.n[3] = 1ULL << t->p1max;
  z.p[4] = t->ngrant;
  z.n[4] = 1ULL << t->p1max;
  z.p[5] = reinterpret_cast<uint32_t*>(t->gsh);
  z.n[5] = 2ULL * 2 * kGShards * kGStride;
  launch_init_segments(t->pairs, t->occ, t->ldep, t->pool, t->hdr, n0, t->D0, t->p1, fixed, region, z, t->ctl,
                       region + (fixed ? 0u : n0), t->d_hint, s);
  t->clean_sbb = ~0u;
  t->batches = 0;
  t->parity = 0;
  t->rb = 0;
  t->flat_valid = false;
  return PMDFC_OK;
}

static void fill_bucket_launch(pmdfc_cceh* t, BucketLaunch& L, uint64_t n, uint8_t* st,
                               uint64_t* vout, bool mixed) {
  const uint32_t npb = 1u << (t->p1 - t->sbb);
  const uint32_t p = t->rb;
  L.n = n;
  L.rkv = t->rkv + p * t->nrec;
  L.rop = t->rop + p * t->nrec;
  L.robk = t->robk + (size_t)p * t->max_batch;
  L.chunk = t->chunk;
  L.cap = t->cap;
  L.cursor = t->cursor + (size_t)p * t->cblk;
  L.ovf = L.cursor + (size_t)npb * kPartSubs;
  L.cursor_next = t->cursor + (size_t)((p + 1) % kRecBufs) * t->cblk;
  L.ovf_next = L.cursor_next + (size_t)npb * kPartSubs;
  L.clear_next = 1;
  L.hdr = t->hdr;
  L.pool = t->pool;
  L.pool_cap = (uint32_t)t->pool_cap;
  L.p1 = t->p1;
  L.sbb = t->sbb;
  L.sbits = t->sbits;
  L.shard = t->shard;
  L.pfix = t->p1 == t->p1max ? 1u : 0u;
  L.pairs = t->pairs;
  L.occ = t->occ;
  L.ldep = t->ldep;
  L.vout = vout;
  L.st = st;
  L.mixed = mixed ? 1u : 0u;
  L.upsert = t->upsert;
  L.upos = t->upos;
  L.max_segments = (uint32_t)t->max_segs;
  L.ctl = t->ctl;
  L.wstat = t->wstat;
  L.wl_kv = t->wl_kv;
  L.wl_op = t->wl_op;
  L.wl_n = t->wl_n;
  L.stamps = t->stamp_cur;
  L.req = t->req;
  L.reqop = t->reqop;
  L.drops = nullptr;  // (mixed batches with early answers set it)
  L.need = t->need;
  L.gbase = t->gbase;
  L.ngrant = t->ngrant;
  L.newoff = t->newoff;
  L.gsh = t->gsh;
  L.gsplit = t->gsplit;
  L.gcap = t->gcap;
  L.act = t->act;
  L.fin = t->fin;
  L.fbl = t->fbl;
  L.par = t->parity;
  // the lean first pass in its wide variant once the table has more segments
  // per bucket than the narrow one's 32-entry sub-directories hold (about 20:
  // a bucket's deepest segment sits ~1.5 levels below the mean).  The count is
  // a hint the device leaves in pinned memory (k_apply_parked), read without
  // a sync, so it may lag the batches in flight: either variant is exact, and
  // each hands the buckets it cannot take to k_apply_fb.
  L.hint = t->d_hint;
  L.wide = t->g_wide;  // (batch_geometry)
  L.fb = t->g_fb;
  L.cp = t->cp;
  L.split_stamps = t->stamp_cur ? t->stamp_cur + (16ULL << t->p1max) + 8ULL * part_blocks(t->max_batch) : nullptr;
  // the larger grids of the passes after the first while the table ramps,
  // or is still small for the batch (more than 32 ops per segment: windows
  // fill within the batch, the final pass has work): the CCEH_hybrid(2)
  // ramp 5.11 -> 5.75 Gops/s with them after p1max too, config 2 (16 ops per
  // segment at its start) 12.56 against 12.41 without (profiles/r05/grids/)
  {
    const uint64_t segs = __atomic_load_n(t->h_hint, __ATOMIC_RELAXED);
    L.ramp = (t->p1 < t->p1max || n > 32ull * std::max<uint64_t>(segs, 1)) ? 1u : 0u;
  }
}

static uint64_t stamp_words(const pmdfc_cceh* t) {
  return 16ULL * (1ULL << t->p1max) + 8ULL * part_blocks(t->max_batch) + 8ULL * kSplitStamps;
}

static void fill_part_launch(pmdfc_cceh* t, PartLaunch& L, const uint8_t* ops, const uint64_t* keys,
                             const uint64_t* vin, uint8_t* st, uint64_t n) {
  L.keys = keys;
  L.vin = vin;
  L.kvs = 1;
  L.ops = ops;
  L.st = st;
  L.n = n;
  L.sbits = t->sbits;
  L.shard = t->shard;
  L.p1 = t->p1;
  L.sbb = t->sbb;
  L.cap = t->cap;
  const uint32_t p = t->rb, npb = 1u << (t->p1 - t->sbb);
  L.rkv = t->rkv + p * t->nrec;
  L.rop = t->rop + p * t->nrec;
  L.robk = t->robk + (size_t)p * t->max_batch;
  L.cursor = t->cursor + (size_t)p * t->cblk;
  L.ovf = L.cursor + (size_t)npb * kPartSubs;
  L.povf = t->povf + (size_t)p * part_blocks(t->max_batch) * (1u << kMaxPartBits);
  // (each batch's partition comes first: it takes the batch's stamp set)
  t->stamp_cur = t->stamps ? t->stamps + (uint64_t)(t->stamp_seq++ % t->stamp_rot) * stamp_words(t) : nullptr;
  L.stamps = t->stamp_cur ? t->stamp_cur + (16ULL << t->p1max) : nullptr;
}

// The bucket passes of one insert / mixed batch, all on the stream: a first
// apply pass, then kSplitRounds x {split round, apply pass over the parked
// ops (it commits the round's splits first)}, then the final pass for
// whatever is still parked -- ops whose segment needs a second split in the
// same batch, rare enough that one pipelined round measured best (an empty
// round costs ~15 us of launches).
static constexpr int kSplitRounds = 1;  // (a batch's grant shards hold one round of requests)

static void run_bucket_passes(pmdfc_cceh* t, const BucketLaunch& B, hipStream_t s) {
  t->timing.begin(PMDFC_K_PROCESS, s);
  launch_apply(B, 0, s);
  // the general first pass over the buckets the lean one declined: its own
  // launch (k_apply_fb, requesting splits for the split round) only where
  // declines are expected, a table past the wide pass's 128-entry
  // sub-directories; otherwise the rare declined bucket takes its first pass
  // in k_apply_parked (an empty k_apply_fb launch costs ~3.2 us a batch)
  if (B.fb) {
    t->timing.begin(PMDFC_K_FINAL, s);  // (the fallback first pass is timed with the final pass)
    launch_apply_fallback(B, s);
  }
  for (int r = 0; r < kSplitRounds; ++r) {
    t->timing.begin(PMDFC_K_SPLIT, s);
    launch_split_round(B, s);
    t->timing.begin(PMDFC_K_PARKED, s);
    launch_apply(B, r + 1 < kSplitRounds ? 1 : 2, s);  // the last one requests nothing
  }
  t->timing.begin(PMDFC_K_FINAL, s);
  launch_final(B, s);
}

// ------------------------------------------------------------------- C-ABI

extern "C" {

int pmdfc_abi_version(void) { return PMDFC_ABI_VERSION; }
const char* pmdfc_last_error(void) { return g_err.c_str(); }

uint32_t pmdfc_depth_for_hybrid(uint64_t init_cap) {
  return (uint32_t)(size_t)std::log2((double)init_cap);  // CCEH_hybrid.cpp:80
}

uint32_t pmdfc_depth_for_src(uint64_t init_cap) {
  return (uint32_t)(size_t)std::log2((double)(init_cap / kSlots));  // src/cceh.cpp:82
}

int pmdfc_cceh_create(const pmdfc_cceh_config_t* cfg, pmdfc_cceh_t** out) {
  if (!cfg || !out) return fail(PMDFC_ERR_ARG, "null argument");
  *out = nullptr;
  if (cfg->initial_depth < 1 || cfg->initial_depth > kMaxDepth)
    return fail(PMDFC_ERR_ARG, "initial_depth must be in [1, 30] (CCEH(initCap) needs initCap >= 2)");
  if (cfg->shard_bits > cfg->initial_depth || cfg->shard_bits > 16)
    return fail(PMDFC_ERR_ARG, "shard_bits must be <= initial_depth (and <= 16)");
  if (cfg->shard_bits && cfg->shard_id >= (1u << cfg->shard_bits))
    return fail(PMDFC_ERR_ARG, "shard_id out of range");
  if (cfg->max_batch == 0) return fail(PMDFC_ERR_ARG, "max_batch must be > 0");
  if (cfg->flags & ~PMDFC_CFG_UPSERT) return fail(PMDFC_ERR_ARG, "unknown flags");
  if ((uint64_t)cfg->max_batch > (uint64_t)kMaxPartBlocks * kPartTile)
    return fail(PMDFC_ERR_ARG, "max_batch must be <= 4194304");
  DevGuard g(cfg->device);
  auto* t = new pmdfc_cceh();
  t->cfg = *cfg;
  t->dev = cfg->device;
  t->D0 = cfg->initial_depth;
  t->sbits = cfg->shard_bits;
  t->shard = cfg->shard_id;
  t->max_batch = cfg->max_batch;
  t->upsert = (cfg->flags & PMDFC_CFG_UPSERT) ? 1u : 0u;
  const uint32_t Dl0 = t->D0 - t->sbits;
  const uint64_t n0 = 1ULL << Dl0;
  // directory buckets: about 128 ops each at max_batch (half a wave chunk),
  // never finer than the initial directory (a segment must not span two);
  // (64-op buckets measured slower: twice the waves, same latency per wave)
  // (floor: a routed engine's max_batch is 2^shard_bits padded owner blocks,
  // ~1.07x the ops it actually receives per batch)
  const uint32_t lgb = cfg->max_batch ? 31u - (uint32_t)__builtin_clz(cfg->max_batch) : 0u;
  uint32_t p1t = lgb > 7 ? lgb - 7 : 0;
  if (const char* e = getenv("PMDFC_P1MAX")) p1t = (uint32_t)atoi(e);  // A/B (capped at kMaxP1 below)
  // never finer than the initial directory at first (a segment must not
  // span two buckets); rebucket_now refines up to p1max as segments deepen
  t->p1max = std::min<uint32_t>(p1t, kMaxP1);
  t->p1_init = std::min<uint32_t>(t->p1max, Dl0);
  // k_part partitions into at most 2^kMaxPartBits buckets; finer directory
  // buckets share a partition bucket (sub-buckets)
  set_geometry(t, t->p1_init);
  if (const char* e = getenv("PMDFC_CHUNK")) t->chunk = (uint32_t)atoi(e);
  if (const char* e = getenv("PMDFC_FLAT_MAX")) t->flat_max = std::min<uint32_t>((uint32_t)atoi(e), kFlatMaxBits);
  uint64_t ms = cfg->max_segments;
  if (ms == 0) {
    size_t fr = 0, tot = 0;
    (void)hipMemGetInfo(&fr, &tot);
    ms = std::min<uint64_t>((uint64_t)(fr * 0.5) / (kSlots * 16 + 160), 1ULL << 22);
  }
  ms = std::max<uint64_t>(ms, n0 + 1);
  if (ms > kMaxSegments) ms = kMaxSegments;  // 26-bit segment ids in directory entries
  t->max_segs = ms;
  // sub-directory pool: the live directory is ~2 entries per segment; every
  // growth leaks the old region (like the reference's directory doubling)
  t->pool_cap = std::min<uint64_t>(std::max<uint64_t>(n0 * 4, 8ULL << ceil_log2(ms)) + 4096 +
                                        ((uint64_t)kFixedSlot << t->p1max), 0xFFFFFFF0ULL);
  // every per-bucket array is sized for p1max
  const uint64_t nb = 1ULL << t->p1max;
  uint64_t nrec = 0;
  for (uint32_t q = t->p1_init; q <= t->p1max; ++q) {
    const uint32_t sq = q > kMaxPartBits ? q - kMaxPartBits : 0;
    nrec = std::max<uint64_t>(nrec, ((uint64_t)part_cap(t->max_batch, q, sq) << (q - sq)) + t->max_batch);
    if (q > kCpSbb)  // (the coarse partition of batch_geometry)
      nrec = std::max<uint64_t>(nrec, ((uint64_t)part_cap(t->max_batch, q, kCpSbb) << (q - kCpSbb)) + t->max_batch);
  }
  t->nrec = nrec;
  {
    const uint32_t sq = t->p1max > kMaxPartBits ? t->p1max - kMaxPartBits : 0;
    t->cblk = cursor_block(1u << (t->p1max - sq));
  }
  const uint64_t nblk = part_blocks(t->max_batch);
  hipError_t e;
#define ALLOC(p, bytes)                                                   \
  do {                                                                    \
    e = hipMalloc(&(p), (bytes));                                         \
    if (e != hipSuccess) {                                                \
      pmdfc_cceh_destroy(t);                                              \
      return fail(PMDFC_ERR_NOMEM, "hipMalloc " #p, e);                   \
    }                                                                     \
  } while (0)
  ALLOC(t->pairs, ms * kSlots * sizeof(ulonglong2));
  ALLOC(t->occ, ms * 32 * sizeof(uint32_t));
  ALLOC(t->ldep, ms);
  {
    // the mixed batches' key set: kJoinReps replicas (k_mixed_get), each at
    // load <= 1/2 for its blocks' joining keys (>= 8192 slots: a replica takes
    // whole 256-op blocks, so a small batch may put one block in one replica)
    uint64_t isl = 8192;
    while (isl < 2 * (uint64_t)t->max_batch) isl <<= 1;
    t->imask = isl - 1;
    ALLOC(t->iset, isl * sizeof(uint64_t));
    ALLOC(t->ipos, isl * sizeof(uint32_t));
    ALLOC(t->icnt, isl * sizeof(uint32_t));
    ALLOC(t->early, t->max_batch);
    ALLOC(t->islot, t->max_batch * sizeof(uint32_t));
    ALLOC(t->icount, (t->max_batch / 256 + 1) * sizeof(uint32_t));
    ALLOC(t->jbits, kJoinWords * sizeof(uint32_t));
    ALLOC(t->elink, t->max_batch * sizeof(uint32_t));
    ALLOC(t->loss0, 256);
  }
  if (t->upsert) ALLOC(t->upos, (uint64_t)t->max_batch * sizeof(uint16_t));
  ALLOC(t->hdr, nb * sizeof(uint64_t));
  ALLOC(t->pool, t->pool_cap * sizeof(uint32_t));
  ALLOC(t->ctl, sizeof(DevCtl));
  // records, their overflow tags and cursors: kRecBufs sets, so a batch's
  // partition can run while the two batches before it are applied
  ALLOC(t->rkv, kRecBufs * nrec * sizeof(ulonglong2));
  ALLOC(t->rop, kRecBufs * nrec * sizeof(uint32_t));
  ALLOC(t->robk, kRecBufs * (uint64_t)t->max_batch * sizeof(uint16_t));
  ALLOC(t->cursor, kRecBufs * t->cblk * sizeof(uint32_t));
  ALLOC(t->hdr_tmp, nb * sizeof(uint64_t));
  ALLOC(t->minld, sizeof(uint32_t));
  ALLOC(t->wstat, nb * kWStat * sizeof(uint64_t));
  ALLOC(t->wl_kv, nb * kChunkWave * sizeof(ulonglong2));
  ALLOC(t->wl_op, nb * kChunkWave * sizeof(uint32_t));
  ALLOC(t->wl_n, nb * sizeof(uint32_t));
  ALLOC(t->gflat, (sizeof(uint32_t) << kFlatMaxBits));
  ALLOC(t->gflat_bits, sizeof(uint32_t));
  ALLOC(t->req, nb * kSplitCap * sizeof(uint2));
  ALLOC(t->reqop, nb * kSplitCap * sizeof(uint32_t));
  ALLOC(t->drops, (uint64_t)kDropLog * sizeof(ulonglong2));
  // bucket w requests in shard w % 8, at most kSplitCap splits
  t->gcap = (uint32_t)((nb + kGShards - 1) / kGShards) * kSplitCap;
  ALLOC(t->gsh, 2 * kGShards * kGStride * sizeof(uint64_t));
  ALLOC(t->gsplit, 2 * kGShards * (uint64_t)t->gcap * sizeof(uint4));
  ALLOC(t->act, nb * sizeof(uint32_t));
  ALLOC(t->touched, (nb + 1) * sizeof(uint32_t));
  ALLOC(t->povf, kRecBufs * (uint64_t)part_blocks(t->max_batch) * (1u << kMaxPartBits) * sizeof(uint32_t));
  ALLOC(t->need, nb * sizeof(uint32_t));
  ALLOC(t->gbase, nb * sizeof(uint32_t));
  ALLOC(t->ngrant, nb * sizeof(uint32_t));
  ALLOC(t->newoff, nb * sizeof(uint32_t));
  ALLOC(t->fin, 2 * nb * sizeof(uint32_t));
  ALLOC(t->fbl, nb * sizeof(uint32_t));
  ALLOC(t->partials, ((uint64_t)t->max_batch / 64 + 2) * sizeof(uint32_t));
  ALLOC(t->popc, sizeof(unsigned long long));
  ALLOC(t->srv_st, 64);
  ALLOC(t->srv_vout, 64 * sizeof(uint64_t));
  if (const char* ev = getenv("PMDFC_STAMPS"))
    if (ev[0] == '1') {
      const char* r = getenv("PMDFC_STAMP_ROT");
      t->stamp_rot = r && atoi(r) > 1 ? (uint32_t)atoi(r) : 1u;
      ALLOC(t->stamps, t->stamp_rot * (16 * nb + 8 * nblk + 8ULL * kSplitStamps) * sizeof(uint64_t));
      HIPCHK(hipMemset(t->stamps, 0, t->stamp_rot * (16 * nb + 8 * nblk + 8ULL * kSplitStamps) * sizeof(uint64_t)));
      t->stamp_cur = t->stamps;
    }
#undef ALLOC
  {
    // the partition stream at high priority: a batch's k_part is dispatched
    // ahead of the previous batch's remaining bucket waves (PMDFC_PSTREAM_PRIO=0: default priority, A/B)
    int lo = 0, hi = 0;
    const char* pe = getenv("PMDFC_PSTREAM_PRIO");
    if (!(pe && pe[0] == '0') && hipDeviceGetStreamPriorityRange(&lo, &hi) == hipSuccess)
      e = hipStreamCreateWithPriority(&t->pstream, hipStreamNonBlocking, hi);
    else
      e = hipStreamCreateWithFlags(&t->pstream, hipStreamNonBlocking);
  }
  if (e == hipSuccess) e = hipEventCreateWithFlags(&t->ev_in, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&t->ev_minld, hipEventDisableTiming);
  for (int i = 0; i < 2 && e == hipSuccess; ++i) {
    e = hipEventCreateWithFlags(&t->ev_gpart[i], hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&t->ev_gdone[i], hipEventDisableTiming);
  }
  for (int i = 0; i < (int)kRecBufs && e == hipSuccess; ++i) {
    e = hipEventCreateWithFlags(&t->ev_part[i], hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&t->ev_done[i], hipEventDisableTiming);
  }
  if (e == hipSuccess) e = hipHostMalloc((void**)&t->h_depth, 32 * sizeof(uint32_t), hipHostMallocDefault);
  if (e != hipSuccess) {
    pmdfc_cceh_destroy(t);
    return fail(PMDFC_ERR_HIP, "stream/event create", e);
  }
  // (coherent: the device's system-scope store reaches host memory without a
  // fence of the stream)
  if (e == hipSuccess) e = hipHostMalloc((void**)&t->h_hint, 64, hipHostMallocCoherent | hipHostMallocMapped);
  if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&t->d_hint, t->h_hint, 0);
  if (e != hipSuccess) {
    pmdfc_cceh_destroy(t);
    return fail(PMDFC_ERR_HIP, "hint word", e);
  }
  memset(t->h_hint, 0, 64);
  e = hipHostMalloc(&t->hctl, sizeof(DevCtl), hipHostMallocDefault);
  if (e != hipSuccess) {
    pmdfc_cceh_destroy(t);
    return fail(PMDFC_ERR_NOMEM, "hipHostMalloc", e);
  }
  t->iset_dirty = true;  // (fresh allocations: init_state empties the key set)
  int rc = init_state(t, (hipStream_t)0);
  if (rc == PMDFC_OK && hipStreamSynchronize((hipStream_t)0) != hipSuccess) rc = fail(PMDFC_ERR_HIP, "init");
  if (rc) {
    pmdfc_cceh_destroy(t);
    return rc;
  }
  *out = t;
  return PMDFC_OK;
}

int pmdfc_cceh_destroy(pmdfc_cceh_t* t) {
  if (!t) return PMDFC_OK;
  DevGuard g(t->dev);
  (void)hipDeviceSynchronize();
  t->timing.flush_closed();
  void* ptrs[] = {t->upos, t->pairs, t->occ, t->ldep, t->iset, t->ipos, t->islot, t->icnt, t->icount, t->jbits, t->early, t->elink, t->loss0, t->hdr, t->pool, t->ctl, t->rkv,
                  t->rop, t->robk, t->cursor, t->wstat, t->wl_kv, t->wl_op, t->wl_n, t->partials, t->popc, t->stamps,
                  t->req, t->reqop, t->drops, t->gsh, t->gsplit, t->act, t->touched, t->povf, t->gflat, t->gflat_bits, t->need, t->gbase, t->ngrant, t->newoff, t->fin, t->fbl, t->hdr_tmp, t->minld, t->srv_st, t->srv_vout};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  if (t->hctl) (void)hipHostFree(t->hctl);
  if (t->h_depth) (void)hipHostFree(t->h_depth);
  if (t->h_hint) (void)hipHostFree(t->h_hint);
  for (hipEvent_t ev : {t->ev_in, t->ev_minld, t->ev_gpart[0], t->ev_gpart[1], t->ev_gdone[0], t->ev_gdone[1]})
    if (ev) (void)hipEventDestroy(ev);
  for (uint32_t i = 0; i < kRecBufs; ++i) {
    if (t->ev_part[i]) (void)hipEventDestroy(t->ev_part[i]);
    if (t->ev_done[i]) (void)hipEventDestroy(t->ev_done[i]);
  }
  if (t->pstream) (void)hipStreamDestroy(t->pstream);
  delete t;
  return PMDFC_OK;
}

int pmdfc_cceh_reset(pmdfc_cceh_t* t, void* stream) {
  if (!t) return fail(PMDFC_ERR_ARG, "null engine");
  std::lock_guard<std::mutex> lk(t->mu);
  DevGuard g(t->dev);
  return init_state(t, (hipStream_t)stream);
}

static int do_get(pmdfc_cceh_t* t, const uint64_t* keys, uint64_t* vout, uint8_t* st, uint64_t n,
                  void* stream) {
  if (n == 0) return PMDFC_OK;
  std::lock_guard<std::mutex> lk(t->mu);
  DevGuard g(t->dev);
  hipStream_t s = (hipStream_t)stream;
  const bool count = t->count_lines && n <= t->max_batch;
  if (!t->flat_valid) {  // first Get after inserts: flatten the directory
    launch_flatten(t->hdr, t->pool, t->p1, t->gflat, t->gflat_bits, t->flat_max, s);
    t->flat_valid = true;
  }
  t->timing.begin(PMDFC_K_GET, s);
  launch_get(count, keys, vout, st, n, t->geo_flat(), t->pairs, t->partials, s);
  t->timing.end(s);
  t->last_get_n = n;
  t->last_get_counted = count;
  {
    const char* e = getenv("PMDFC_GET_UNROLL");
    int U = e ? atoi(e) : 2;
    if (U != 1 && U != 2 && U != 4) U = 2;
    t->last_get_blocks = ((n + U - 1) / U + 63) / 64;
  }
  HIPCHK(hipGetLastError());
  return PMDFC_OK;
}

int pmdfc_cceh_get(pmdfc_cceh_t* t, const uint64_t* keys, uint64_t* vout, uint8_t* st, uint64_t n,
                   void* stream) {
  if (!t || (n && (!keys || !vout || !st))) return fail(PMDFC_ERR_ARG, "null argument");
  return do_get(t, keys, vout, st, n, stream);
}

// Get batches [bounds[0], bounds[nb]): Get batches change nothing, so
// consecutive ones are one launch over their union -- the same results per op,
// without a kernel boundary (and its ramp and tail) between batches.
int pmdfc_cceh_get_batches(pmdfc_cceh_t* t, const uint64_t* keys, uint64_t* vout, uint8_t* st,
                           const uint64_t* bounds, uint32_t nbatches, void* stream) {
  if (!t || !bounds || (nbatches && (!keys || !vout || !st))) return fail(PMDFC_ERR_ARG, "null argument");
  for (uint32_t i = 0; i < nbatches; ++i)
    if (bounds[i + 1] < bounds[i]) return fail(PMDFC_ERR_ARG, "bounds must be non-decreasing");
  if (nbatches == 0) return PMDFC_OK;
#ifdef PMDFC_GETB_PER_BATCH  // (A/B builds: one launch per batch)
  for (uint32_t i = 0; i < nbatches; ++i)
    if (int rc = do_get(t, keys + bounds[i], vout + bounds[i], st + bounds[i], bounds[i + 1] - bounds[i], stream))
      return rc;
  return PMDFC_OK;
#else
  const uint64_t o = bounds[0];
  return do_get(t, keys + o, vout + o, st + o, bounds[nbatches] - o, stream);
#endif
}

int pmdfc_cceh_find_anyway(pmdfc_cceh_t* t, const uint64_t* keys, uint64_t* vout, uint8_t* st, uint64_t n,
                           void* stream) {
  if (!t || (n && (!keys || !vout || !st))) return fail(PMDFC_ERR_ARG, "null argument");
  if (n == 0) return PMDFC_OK;
  std::lock_guard<std::mutex> lk(t->mu);
  DevGuard g(t->dev);
  launch_find_anyway(keys, vout, st, n, t->geo(), t->pairs, (hipStream_t)stream);
  HIPCHK(hipGetLastError());
  return PMDFC_OK;
}

int pmdfc_cceh_get_records(pmdfc_cceh_t* t, const uint64_t* keys, uint64_t* resp, uint64_t n, void* stream) {
  if (!t || (n && (!keys || !resp))) return fail(PMDFC_ERR_ARG, "null argument");
  return do_get(t, keys, resp, nullptr, n, stream);
}

// A batch of at most kChunkWave ops takes one launch (k_mixed_small) instead
// of the ~12 of the general pipeline; its results are the serial reference's
// exactly.  PMDFC_SMALL_MAX lowers the cut (0: never; A/B and tests).
static uint64_t small_max() {
  static const uint64_t v = [] {
    const char* e = getenv("PMDFC_SMALL_MAX");
    return e ? std::min<uint64_t>(strtoull(e, nullptr, 0), kChunkWave) : (uint64_t)kChunkWave;
  }();
  return v;
}

static int small_one(pmdfc_cceh_t* t, const uint8_t* ops, const uint64_t* keys, const uint64_t* vin,
                     uint64_t* vout, uint8_t* st, uint64_t n, hipStream_t s) {
  int rc = rebucket_now(t, s);  // (a table coarser than p1max: one sync, as the general path)
  if (rc) return rc;
  if ((rc = batch_geometry(t, false, n, s, false))) return rc;  // (no records)
  BucketLaunch B{};
  fill_bucket_launch(t, B, n, st, vout, true);
  t->timing.begin(PMDFC_K_PROCESS, s);
  launch_mixed_small(B, ops, keys, vin, s);
  t->timing.end(s);
  t->batches += 1;
  t->flat_valid = false;
  HIPCHK(hipGetLastError());
  return PMDFC_OK;
}

// A batch of at most kPartTile ops at full bucket resolution takes two
// launches: its one-block partition (k_part, statuses initialized there, the
// touched buckets listed) and k_medium, the final pass over every touched
// bucket with its records in batch order.  Exact serial results (no early
// answers).  PMDFC_MEDIUM_MAX lowers the cut (0: never).
static uint64_t medium_max() {
  static const uint64_t v = [] {
    const char* e = getenv("PMDFC_MEDIUM_MAX");
    return e ? std::min<uint64_t>(strtoull(e, nullptr, 0), kPartTile) : (uint64_t)kPartTile;
  }();
  return v;
}

static int medium_one(pmdfc_cceh_t* t, const uint8_t* ops, const uint64_t* keys, const uint64_t* vin, uint32_t kvs,
                      uint64_t* vout, uint8_t* st, uint64_t n, hipStream_t s) {
  int rc = batch_geometry(t, false, n, s);
  if (rc) return rc;
  PartLaunch P{};
  fill_part_launch(t, P, ops, keys, vin, st, n);
  P.kvs = kvs;
  P.init = ops ? 1u : 0u;
  P.vout = vout;
  P.touched = t->touched;
  BucketLaunch B{};
  fill_bucket_launch(t, B, n, st, vout, ops != nullptr);
  t->timing.begin(PMDFC_K_PROCESS, s);
  launch_part(P, s);
  launch_medium(B, t->touched, s);
  t->timing.end(s);
  // the batch parity stays: k_medium (the final pass, splits inline) never
  // touches the per-batch words (grant shards, worklists), and only a general
  // batch's first pass clears the other parity's -- flipping here would hand
  // the next general batch the stale words of the one before this
  t->rb = (t->rb + 1) % kRecBufs;
  t->clean_sbb = t->sbb;  // (k_medium zeroed the next buffer's cursors at its positions)
  t->batches += 1;
  t->flat_valid = false;
  HIPCHK(hipGetLastError());
  return PMDFC_OK;
}

static int insert_one(pmdfc_cceh_t* t, const uint64_t* keys, const uint64_t* vin, uint32_t kvs, uint8_t* st,
                      uint64_t n, hipStream_t s) {
  int rc = batch_geometry(t, true, n, s);
  if (rc) return rc;
  PartLaunch P{};
  fill_part_launch(t, P, nullptr, keys, vin, st, n);
  P.kvs = kvs;
  BucketLaunch B{};
  fill_bucket_launch(t, B, n, st, nullptr, false);
  t->timing.begin(PMDFC_K_ROUTE, s);
  // upsert: the lean first pass probes each window itself; the pre-batch
  // probe serves the general pass only when the lean one is off
  const bool probe = t->upsert && !fast_first_pass();
  if (probe) launch_upsert_probe(keys, kvs, nullptr, n, t->geo(), t->pairs, t->upos, s);
  else B.upos = nullptr;
  launch_part(P, s);
  run_bucket_passes(t, B, s);
  t->timing.end(s);
  t->parity ^= 1;
  t->rb = (t->rb + 1) % kRecBufs;
  t->clean_sbb = t->sbb;  // (its first pass zeroed the next buffer's cursors at its positions)
  t->flat_valid = false;
  HIPCHK(hipGetLastError());
  return PMDFC_OK;
}

// one insert batch, as sub-batches while the table is coarser than p1max
static int insert_ramped(pmdfc_cceh_t* t, const uint64_t* keys, const uint64_t* vin, uint32_t kvs, uint8_t* st,
                         uint64_t n, hipStream_t s) {
  for (uint64_t o = 0; o < n;) {
    int rc = rebucket_now(t, s);
    if (rc) return rc;
    const uint64_t m = ramp_batch(t, n - o);
    rc = insert_one(t, keys + o * kvs, vin + o * kvs, kvs, st + o, m, s);
    if (rc) return rc;
    o += m;
  }
  t->batches += 1;
  return PMDFC_OK;
}

static int do_insert(pmdfc_cceh_t* t, const uint64_t* keys, const uint64_t* vin, uint32_t kvs, uint8_t* st,
                     uint64_t n, void* stream) {
  if (n == 0) return PMDFC_OK;
  if (n > t->max_batch) return fail(PMDFC_ERR_ARG, "n exceeds max_batch");
  std::lock_guard<std::mutex> lk(t->mu);
  DevGuard g(t->dev);
  if (kvs == 1 && n <= small_max()) return small_one(t, nullptr, keys, vin, nullptr, st, n, (hipStream_t)stream);
  if (n <= medium_max() && t->p1 >= t->p1max)
    return medium_one(t, nullptr, keys, vin, kvs, nullptr, st, n, (hipStream_t)stream);
  return insert_ramped(t, keys, vin, kvs, st, n, (hipStream_t)stream);
}

int pmdfc_cceh_insert(pmdfc_cceh_t* t, const uint64_t* keys, const uint64_t* vin, uint8_t* st,
                      uint64_t n, void* stream) {
  if (!t || (n && (!keys || !vin || !st))) return fail(PMDFC_ERR_ARG, "null argument");
  return do_insert(t, keys, vin, 1, st, n, stream);
}

int pmdfc_cceh_insert_records(pmdfc_cceh_t* t, const uint64_t* records, uint8_t* st, uint64_t n,
                              void* stream) {
  if (!t || (n && (!records || !st))) return fail(PMDFC_ERR_ARG, "null argument");
  return do_insert(t, records, records + 1, 2, st, n, stream);
}

// Pipelined insert batches (t->mu held, table at p1max): batch k of a run
// partitions on the partition stream while the bucket passes of batch k - 1
// (or k - 2) run on the caller's stream.  pipe_begin: the partition stream
// starts after everything already on s; pipe_batch: one batch (input_ready,
// if given: an event the partition waits for first -- the routed loop's
// received rows); pipe_end: the next buffer's cursors zeroed for the
// one-batch entry points.
static int pipe_begin(pmdfc_cceh_t* t, hipStream_t s) {
  HIPCHK(hipEventRecord(t->ev_in, s));
  HIPCHK(hipStreamWaitEvent(t->pstream, t->ev_in, 0));
  return PMDFC_OK;
}

static int pipe_batch(pmdfc_cceh_t* t, const uint64_t* keys, const uint64_t* vin, uint32_t kvs, uint8_t* st,
                      uint64_t n, hipStream_t s, uint32_t k, hipEvent_t input_ready,
                      hipEvent_t output_free = nullptr) {
  hipStream_t P = t->pstream;
  const uint32_t p = t->rb;
  // record buffer p's records and cursors were last read by the batch
  // kRecBufs back: with three buffers the partition of batch k + 1 may start
  // as soon as batch k - 2 is applied, so it runs under the bucket passes of
  // batch k - 1 or k instead of waiting for their end
  if (k >= kRecBufs) HIPCHK(hipStreamWaitEvent(P, t->ev_done[p], 0));
  if (input_ready) HIPCHK(hipStreamWaitEvent(P, input_ready, 0));
  if (output_free) HIPCHK(hipStreamWaitEvent(P, output_free, 0));  // (the partition writes the statuses)
  HIPCHK(hipMemsetAsync(t->cursor + p * t->cblk, 0, t->cblk * sizeof(uint32_t), P));
  int rc = batch_geometry(t, true, n, nullptr, false);  // (its cursors: zeroed just above)
  if (rc) return rc;
  PartLaunch PL{};
  fill_part_launch(t, PL, nullptr, keys, vin, st, n);
  PL.kvs = kvs;
  hipEvent_t e0 = t->timing.span_begin(P);
  const bool probe = t->upsert && !fast_first_pass();  // (as insert_one)
  if (probe) {  // the probe reads the table: after the previous batch (ev_done)
    if (k >= 1) HIPCHK(hipStreamWaitEvent(P, t->ev_done[(p + kRecBufs - 1) % kRecBufs], 0));
    launch_upsert_probe(keys, kvs, nullptr, n, t->geo(), t->pairs, t->upos, P);
  }
  launch_part(PL, P);
  t->timing.span_end(PMDFC_K_ROUTE, e0, P);
  HIPCHK(hipEventRecord(t->ev_part[p], P));
  HIPCHK(hipStreamWaitEvent(s, t->ev_part[p], 0));
  BucketLaunch B{};
  fill_bucket_launch(t, B, n, st, nullptr, false);
  B.clear_next = 0;  // the next batch's cursors may already be in use
  if (!probe) B.upos = nullptr;
  run_bucket_passes(t, B, s);
  t->timing.end(s);
  HIPCHK(hipEventRecord(t->ev_done[p], s));
  t->batches += 1;
  t->parity ^= 1;
  t->rb = (t->rb + 1) % kRecBufs;
  t->flat_valid = false;
  return PMDFC_OK;
}

// Groups of G consecutive batches (pmdfc_cceh_insert_batches): the group's
// partitions on the partition stream, then its bucket passes on s behind ONE
// event -- instead of an event record and a cross-stream wait per batch,
// each a packet the engine stream stops at between the passes of consecutive
// batches.  Group g's records reuse group g - 2's buffers (kRecBufs = 2 G_max),
// so its partitions wait for that group's passes only; they run under group
// g - 1's passes.  Each batch keeps the geometry its partition chose.
static uint32_t pipe_group_size() {
  static const uint32_t g = [] {
    const char* e = getenv("PMDFC_PIPE_GROUP");  // A/B: 1 = an event pair per batch
    const int v = e ? atoi(e) : 8;
    return (uint32_t)std::min<int>(std::max<int>(v, 1), (int)kRecBufs / 2);
  }();
  return g;
}

static int pipe_group(pmdfc_cceh_t* t, const uint64_t* keys, const uint64_t* vin, uint8_t* st,
                      const uint64_t* bounds, const uint32_t* idx, uint32_t m, hipStream_t s, uint32_t gi) {
  hipStream_t P = t->pstream;
  struct Geo1 {
    uint32_t rb, sbb, cap, cp, wide, fb;
    uint64_t* stamps;
  } geo[kRecBufs / 2 > 0 ? kRecBufs / 2 : 1];
  if (gi >= 2) HIPCHK(hipStreamWaitEvent(P, t->ev_gdone[gi & 1u], 0));
  hipEvent_t e0 = t->timing.span_begin(P);
  for (uint32_t j = 0; j < m; ++j) {
    const uint64_t o = bounds[idx[j]], n = bounds[idx[j] + 1] - o;
    const uint32_t p = t->rb;
    HIPCHK(hipMemsetAsync(t->cursor + p * t->cblk, 0, t->cblk * sizeof(uint32_t), P));
    if (int rc = batch_geometry(t, true, n, nullptr, false)) return rc;  // (its cursors: zeroed just above)
    PartLaunch PL{};
    fill_part_launch(t, PL, nullptr, keys + o, vin + o, st + o, n);
    launch_part(PL, P);
    geo[j] = {p, t->sbb, t->cap, t->cp, t->g_wide, t->g_fb, t->stamp_cur};
    t->rb = (p + 1) % kRecBufs;
  }
  t->timing.span_end(PMDFC_K_ROUTE, e0, P);
  HIPCHK(hipEventRecord(t->ev_gpart[gi & 1u], P));
  HIPCHK(hipStreamWaitEvent(s, t->ev_gpart[gi & 1u], 0));
  const uint32_t rb_next = t->rb;
  for (uint32_t j = 0; j < m; ++j) {
    const uint64_t o = bounds[idx[j]], n = bounds[idx[j] + 1] - o;
    t->rb = geo[j].rb;
    t->sbb = geo[j].sbb;
    t->cap = geo[j].cap;
    t->cp = geo[j].cp;
    t->g_wide = geo[j].wide;
    t->g_fb = geo[j].fb;
    t->stamp_cur = geo[j].stamps;
    BucketLaunch B{};
    fill_bucket_launch(t, B, n, st + o, nullptr, false);
    B.clear_next = 0;  // the next batch's cursors may already be in use
    B.upos = nullptr;
    run_bucket_passes(t, B, s);
    t->timing.end(s);
    t->batches += 1;
    t->parity ^= 1;
    t->flat_valid = false;
  }
  t->rb = rb_next;
  HIPCHK(hipEventRecord(t->ev_gdone[gi & 1u], s));
  HIPCHK(hipGetLastError());
  return PMDFC_OK;
}

static int pipe_end(pmdfc_cceh_t* t, hipStream_t s) {
  HIPCHK(hipMemsetAsync(t->cursor + t->rb * t->cblk, 0, t->cblk * sizeof(uint32_t), s));
  t->clean_sbb = ~0u;
  HIPCHK(hipGetLastError());
  return PMDFC_OK;
}

int pmdfc_cceh_insert_batches(pmdfc_cceh_t* t, const uint64_t* keys, const uint64_t* vin, uint8_t* st,
                              const uint64_t* bounds, uint32_t nbatches, void* stream) {
  if (!t || !bounds || (nbatches && (!keys || !vin || !st))) return fail(PMDFC_ERR_ARG, "null argument");
  for (uint32_t i = 0; i < nbatches; ++i) {
    if (bounds[i + 1] < bounds[i]) return fail(PMDFC_ERR_ARG, "bounds must be non-decreasing");
    if (bounds[i + 1] - bounds[i] > t->max_batch) return fail(PMDFC_ERR_ARG, "a batch exceeds max_batch");
  }
  if (nbatches == 0) return PMDFC_OK;
  std::lock_guard<std::mutex> lk(t->mu);
  DevGuard g(t->dev);
  hipStream_t s = (hipStream_t)stream;
  // a table still coarser than p1max: its first batches one by one, ramped
  uint32_t i0 = 0;
  for (; i0 < nbatches && t->p1 < t->p1max; ++i0) {
    const int rc = insert_ramped(t, keys + bounds[i0], vin + bounds[i0], 1, st + bounds[i0],
                                 bounds[i0 + 1] - bounds[i0], s);
    if (rc) return rc;
  }
  // the partition stream starts after everything already on the caller's
  // stream (the inputs, and every earlier batch)
  int rc = pipe_begin(t, s);
  if (t->upsert && !fast_first_pass()) {  // (the upsert probe reads the table: batch by batch)
    uint32_t k = 0;
    for (uint32_t i = i0; i < nbatches && rc == PMDFC_OK; ++i) {
      const uint64_t o = bounds[i], n = bounds[i + 1] - bounds[i];
      if (n == 0) continue;
      rc = pipe_batch(t, keys + o, vin + o, 1, st + o, n, s, k++, nullptr);
    }
    return rc ? rc : pipe_end(t, s);
  }
  const uint32_t G = pipe_group_size();
  uint32_t idx[kRecBufs / 2 > 0 ? kRecBufs / 2 : 1], m = 0, gi = 0;
  for (uint32_t i = i0; i <= nbatches && rc == PMDFC_OK; ++i) {
    if (i < nbatches && bounds[i + 1] > bounds[i]) idx[m++] = i;
    if (m == G || (i == nbatches && m)) {
      rc = pipe_group(t, keys, vin, st, bounds, idx, m, s, gi++);
      m = 0;
    }
  }
  return rc ? rc : pipe_end(t, s);
}

// PMDFC_MIXED_SMALL=0: the mixed passes of gated batches always on full grids (A/B)
static bool mixed_small_off() {
  static const bool v = [] {
    const char* e = getenv("PMDFC_MIXED_SMALL");
    return e && e[0] == '0';
  }();
  return v;
}

// A mixed batch tells its Gets whether the batch inserts their key through
// the JOIN (the Gets that need it claim their keys, the inserts look them up)
// when the last mixed batch inserted more than 1/8 of its ops, else through
// the INSERT set (every insert claims its key): ~500k random CASes fewer per
// half-insert config-4 batch, while a config-3 batch (5 % inserts) keeps the
// cheaper insert set (cceh_kernels.hip).  The count is a hint the device
// leaves in pinned memory, read without a sync: either mode is exact.
// PMDFC_MIXED_JOIN=0 / 1 forces one (A/B, tests).
static bool mixed_join_mode(pmdfc_cceh* t, uint64_t n) {
  static const int force = [] {
    const char* e = getenv("PMDFC_MIXED_JOIN");
    return e ? atoi(e) : -1;
  }();
  if (force >= 0) return force != 0;
  (void)n;
  const uint64_t last = __atomic_load_n(t->h_hint + kHintMixIns, __ATOMIC_RELAXED);
  return t->last_mixed_n && last * 8 > t->last_mixed_n;
}

static int mixed_one(pmdfc_cceh_t* t, const uint8_t* ops, const uint64_t* keys, const uint64_t* vin,
                     uint64_t* vout, uint8_t* st, uint64_t n, hipStream_t s) {
  const uint64_t seq = ++t->seq;
  if (t->iset_dirty) {  // an earlier batch stopped between its prep and verify passes: start the set empty
    HIPCHK(hipMemsetAsync(t->iset, 0xFF, (t->imask + 1) * sizeof(uint64_t), s));
    HIPCHK(hipMemsetAsync(t->icnt, 0, (t->imask + 1) * sizeof(uint32_t), s));
    HIPCHK(hipMemsetAsync(t->ipos, 0xFF, (t->imask + 1) * sizeof(uint32_t), s));
    HIPCHK(hipMemsetAsync(t->jbits, 0, kJoinWords * sizeof(uint32_t), s));
  }
  t->iset_dirty = true;  // (until the verify pass that empties the set is enqueued)
  if (int rc = batch_geometry(t, false, n, s)) return rc;
  // statuses + early answers + the joining Gets (k_mixed_get), then the
  // inserts' side of the join (k_mixed_join, timed as the pre-pass class);
  // k_part resolves the joining Gets
  const uint32_t tag = (uint32_t)seq;
  const bool join = mixed_join_mode(t, n);
  uint32_t* const hint_ins = t->d_hint + kHintMixIns;
  if (join) {
    t->timing.begin(PMDFC_K_MIXED_GET, s);
    launch_mixed_get(ops, keys, st, vout, n, t->geo(), t->pairs, t->early, t->islot, t->jbits, t->ctl, t->loss0, tag,
                     t->icount, t->upsert ? 1u : 0u, s);
    t->timing.begin(PMDFC_K_PREP, s);
    launch_mixed_join(ops, keys, st, n, t->iset, t->imask, t->ipos, t->icnt, t->islot, t->jbits, t->ctl, tag,
                      t->icount, hint_ins, s);
  } else {
    t->timing.begin(PMDFC_K_PREP, s);
    launch_mixed_prep(ops, keys, st, vout, n, t->geo(), t->iset, t->imask, t->ipos, t->icnt, t->early, t->islot,
                      t->ctl, t->loss0, t->icount, s);
    t->timing.begin(PMDFC_K_MIXED_GET, s);
    launch_mixed_get_iset(ops, keys, st, vout, n, t->geo(), t->pairs, t->iset, t->imask, t->ipos, t->icnt, t->early,
                          t->elink, t->ctl, tag, t->icount, t->upsert ? 1u : 0u, hint_ins, s);
  }
  t->last_mixed_n = n;
  PartLaunch P{};
  fill_part_launch(t, P, ops, keys, vin, st, n);
  P.iset = t->iset;
  P.imask = t->imask;
  P.icnt = t->icnt;
  P.ipos = t->ipos;
  P.early = t->early;
  P.elink = t->elink;
  P.ctl = t->ctl;
  P.tag = tag;
  P.vout = vout;
  BucketLaunch B{};
  fill_bucket_launch(t, B, n, st, vout, true);
  // when k_mixed_get answered every Get, the insert-only apply passes run
  // (upsert batches always take the mixed ones)
  B.gate_tag = t->upsert ? 0u : tag;
  // the mixed passes on small grids unless a mixed batch of the last 64 ran
  // them (the word may lag the batches in flight: either grid is exact)
  B.mseen = t->d_hint + kHintMixed;
  {
    const uint32_t last = __atomic_load_n(t->h_hint + kHintMixed, __ATOMIC_RELAXED);
    B.mixed_small = (last != 0 && tag - last < 64u) || mixed_small_off() ? 0u : 1u;
  }
  B.drops = t->drops;  // splits log what they drop, for k_mixed_verify
  t->timing.begin(PMDFC_K_ROUTE, s);
  if (t->upsert) launch_upsert_probe(keys, 1, ops, n, t->geo(), t->pairs, t->upos, s);
  launch_part(P, s);
  run_bucket_passes(t, B, s);
  launch_mixed_verify(ops, keys, vin, st, vout, n, t->geo(), t->pairs, t->early, t->elink, t->ctl, t->loss0, t->drops,
                      t->iset, t->icnt, t->ipos, t->islot, t->imask, join ? t->jbits : nullptr, s);
  t->timing.end(s);
  t->parity ^= 1;
  t->rb = (t->rb + 1) % kRecBufs;
  t->clean_sbb = t->sbb;
  t->flat_valid = false;
  HIPCHK(hipGetLastError());
  t->iset_dirty = false;
  return PMDFC_OK;
}

int pmdfc_cceh_mixed(pmdfc_cceh_t* t, const uint8_t* ops, const uint64_t* keys, const uint64_t* vin,
                     uint64_t* vout, uint8_t* st, uint64_t n, void* stream) {
  if (!t || (n && (!ops || !keys || !vin || !vout || !st))) return fail(PMDFC_ERR_ARG, "null argument");
  if (n == 0) return PMDFC_OK;
  if (n > t->max_batch) return fail(PMDFC_ERR_ARG, "n exceeds max_batch");
  std::lock_guard<std::mutex> lk(t->mu);
  DevGuard g(t->dev);
  hipStream_t s = (hipStream_t)stream;
  if (n <= small_max()) return small_one(t, ops, keys, vin, vout, st, n, s);
  if (n <= medium_max() && t->p1 >= t->p1max) return medium_one(t, ops, keys, vin, 1, vout, st, n, s);
  for (uint64_t o = 0; o < n;) {  // sub-batches while the table is coarser than p1max
    int rc = rebucket_now(t, s);
    if (rc) return rc;
    const uint64_t m = ramp_batch(t, n - o);
    rc = mixed_one(t, ops + o, keys + o, vin + o, vout + o, st + o, m, s);
    if (rc) return rc;
    o += m;
  }
  t->batches += 1;
  return PMDFC_OK;
}

// Batch after batch through the one-batch path.  (Running batch i + 1's
// pre-pass beside batch i -- double-buffered key sets, the pre-pass on a
// stream of its own -- measured slower: DESIGN.md, round 5.)
int pmdfc_cceh_mixed_batches(pmdfc_cceh_t* t, const uint8_t* ops, const uint64_t* keys, const uint64_t* vin,
                             uint64_t* vout, uint8_t* st, const uint64_t* bounds, uint32_t nbatches, void* stream) {
  if (!t || !bounds || (nbatches && (!ops || !keys || !vin || !vout || !st)))
    return fail(PMDFC_ERR_ARG, "null argument");
  for (uint32_t i = 0; i < nbatches; ++i) {
    if (bounds[i + 1] < bounds[i]) return fail(PMDFC_ERR_ARG, "bounds must be non-decreasing");
    if (bounds[i + 1] - bounds[i] > t->max_batch) return fail(PMDFC_ERR_ARG, "a batch exceeds max_batch");
  }
  for (uint32_t i = 0; i < nbatches; ++i) {
    const uint64_t o = bounds[i], n = bounds[i + 1] - bounds[i];
    if (n == 0) continue;
    if (int rc = pmdfc_cceh_mixed(t, ops + o, keys + o, vin + o, vout + o, st + o, n, stream)) return rc;
  }
  return PMDFC_OK;
}

static int serve_start(pmdfc_cceh_t* t, uint32_t nwaves, pmdfc_serve_req* req, pmdfc_serve_resp* resp,
                       pmdfc_serve_ctl* ctl, uint64_t ring_size, uint64_t head0, pmdfc_cbf_t* cbf, void* stream);

int pmdfc_cceh_serve_start(pmdfc_cceh_t* t, pmdfc_serve_req* req, pmdfc_serve_resp* resp, pmdfc_serve_ctl* ctl,
                           uint64_t ring_size, uint64_t head0, pmdfc_cbf_t* cbf, void* stream) {
  return serve_start(t, 1, req, resp, ctl, ring_size, head0, cbf, stream);
}

uint32_t pmdfc_cceh_serve_waves_max(pmdfc_cceh_t* t) {
  if (!t) return 0;
  std::lock_guard<std::mutex> lk(t->mu);
  return std::min<uint32_t>(1u << t->p1, kServeWavesMax);
}

int pmdfc_cceh_serve_start_n(pmdfc_cceh_t* t, uint32_t nwaves, pmdfc_serve_req* req, pmdfc_serve_resp* resp,
                             pmdfc_serve_ctl* ctl, uint64_t ring_size, pmdfc_cbf_t* cbf, void* stream) {
  if (!t || nwaves == 0 || (nwaves & (nwaves - 1)) || nwaves > kServeWavesMax)
    return fail(PMDFC_ERR_ARG, "serve_start_n: nwaves must be a power of two <= 64");
  {
    std::lock_guard<std::mutex> lk(t->mu);
    if (nwaves > (1u << t->p1)) return fail(PMDFC_ERR_ARG, "serve_start_n: more waves than directory buckets");
  }
  return serve_start(t, nwaves, req, resp, ctl, ring_size, 0, cbf, stream);
}

static int serve_start(pmdfc_cceh_t* t, uint32_t nwaves, pmdfc_serve_req* req, pmdfc_serve_resp* resp,
                       pmdfc_serve_ctl* ctl, uint64_t ring_size, uint64_t head0, pmdfc_cbf_t* cbf, void* stream) {
  if (!t || !req || !resp || !ctl || ring_size < 64 || ring_size > (1ull << 25) ||
      (ring_size & (ring_size - 1)))
    return fail(PMDFC_ERR_ARG, "serve_start: rings and a power-of-two ring_size in [64, 2^25]");
  if (cbf && cbf->dev != t->dev) return fail(PMDFC_ERR_ARG, "serve_start: counting BF on another device");
  std::lock_guard<std::mutex> lk(t->mu);
  DevGuard g(t->dev);
  hipStream_t s = (hipStream_t)stream;
  int rc = rebucket_now(t, s);  // (the wave keeps the bucket geometry it starts with)
  if (rc) return rc;
  void *dq = nullptr, *dr = nullptr, *dc = nullptr;
  HIPCHK(hipHostGetDevicePointer(&dq, req, 0));
  HIPCHK(hipHostGetDevicePointer(&dr, resp, 0));
  HIPCHK(hipHostGetDevicePointer(&dc, ctl, 0));
  if ((rc = batch_geometry(t, false, 64, s, false))) return rc;  // (no records)
  BucketLaunch B{};
  fill_bucket_launch(t, B, 64, t->srv_st, t->srv_vout, true);
  ServeLaunch V{};
  V.req = (const pmdfc_serve_req*)dq;
  V.resp = (pmdfc_serve_resp*)dr;
  V.ctl = (pmdfc_serve_ctl*)dc;
  V.ring_size = ring_size;
  V.head0 = head0;
  V.cbf = cbf ? cbf->cnt : nullptr;
  V.cbf_m = cbf ? cbf->nbits : 0;
  V.cbf_k = cbf ? cbf->k : 0;
  V.nwaves = nwaves;
  launch_serve(B, V, s);
  HIPCHK(hipGetLastError());
  t->flat_valid = false;
  return PMDFC_OK;
}

int pmdfc_cceh_mixed_host(pmdfc_cceh_t* t, const uint8_t* ops, const uint64_t* keys,
                          const uint64_t* vin, uint64_t* vout, uint8_t* st, uint64_t n) {
  if (!t) return fail(PMDFC_ERR_ARG, "null engine");
  DevGuard g(t->dev);
  for (uint64_t off = 0; off < n; off += t->max_batch) {
    const uint64_t m = std::min<uint64_t>(t->max_batch, n - off);
    uint8_t *d_ops = nullptr, *d_st = nullptr;
    uint64_t *d_keys = nullptr, *d_vin = nullptr, *d_vout = nullptr;
    HIPCHK(hipMalloc(&d_ops, m));
    HIPCHK(hipMalloc(&d_st, m));
    HIPCHK(hipMalloc(&d_keys, m * 8));
    HIPCHK(hipMalloc(&d_vin, m * 8));
    HIPCHK(hipMalloc(&d_vout, m * 8));
    HIPCHK(hipMemcpy(d_ops, ops + off, m, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(d_keys, keys + off, m * 8, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(d_vin, vin + off, m * 8, hipMemcpyHostToDevice));
    int rc = pmdfc_cceh_mixed(t, d_ops, d_keys, d_vin, d_vout, d_st, m, nullptr);
    if (rc == PMDFC_OK) {
      HIPCHK(hipMemcpy(vout + off, d_vout, m * 8, hipMemcpyDeviceToHost));
      HIPCHK(hipMemcpy(st + off, d_st, m, hipMemcpyDeviceToHost));
    }
    (void)hipFree(d_ops);
    (void)hipFree(d_st);
    (void)hipFree(d_keys);
    (void)hipFree(d_vin);
    (void)hipFree(d_vout);
    if (rc) return rc;
  }
  return PMDFC_OK;
}

int pmdfc_cceh_stats(pmdfc_cceh_t* t, pmdfc_cceh_stats_t* out) {
  if (!t || !out) return fail(PMDFC_ERR_ARG, "null argument");
  std::lock_guard<std::mutex> lk(t->mu);
  DevGuard g(t->dev);
  HIPCHK(hipDeviceSynchronize());
  int rc = read_ctl(t, (hipStream_t)0);
  if (rc) return rc;
  const DevCtl& c = *t->hctl;
  std::vector<uint64_t> ws((size_t)kWStat << t->p1max);  // (slots of every bucket geometry so far)
  HIPCHK(hipMemcpy(ws.data(), t->wstat, ws.size() * 8, hipMemcpyDeviceToHost));
  uint64_t sum[kWStat] = {0};
  uint32_t max_rounds = 0, max_ld = c.max_ld;
  for (size_t i = 0; i < ws.size(); ++i) {
    const int k = (int)(i % kWStat);
    if (k == 6) {
      max_rounds = std::max<uint32_t>(max_rounds, (uint32_t)(ws[i] & 0xFFFF));
      max_ld = std::max<uint32_t>(max_ld, (uint32_t)((ws[i] >> 16) & 0xFF));
      sum[6] += ws[i] >> 32;
    } else {
      sum[k] += ws[i];
    }
  }
  std::vector<uint64_t> hd(1ULL << t->p1);
  HIPCHK(hipMemcpy(hd.data(), t->hdr, hd.size() * 8, hipMemcpyDeviceToHost));
  uint32_t maxdb = 0;
  for (auto v : hd) maxdb = std::max(maxdb, hdr_db(v));
  const uint64_t nsegs = std::min<uint64_t>(c.nsegs, t->max_segs);
  out->depth = std::max(t->D0, max_ld);
  out->phys_depth = t->sbits + t->p1 + maxdb;
  out->segments = nsegs;
  out->capacity = nsegs * kSlots;
  out->max_segments = t->max_segs;
  out->splits = sum[2];
  out->doublings = sum[6];
  out->split_loss = sum[3] + c.split_loss;
  out->insert_passes = sum[5];
  out->batches = t->batches;
  out->segment_runs = sum[4];
  out->deferred_ops = sum[1];
  out->bucket_bits = t->p1;
  out->max_rounds = max_rounds;
  out->insert_lines = sum[0];
  out->error_flags = c.err;
  {
    std::vector<uint32_t> fb(1ULL << t->p1max);
    HIPCHK(hipMemcpy(fb.data(), t->fbl, fb.size() * 4, hipMemcpyDeviceToHost));
    uint64_t nd = 0;
    for (auto v : fb) nd += v >> 1;
    out->fast_declined = (uint32_t)std::min<uint64_t>(nd, 0xFFFFFFFFu);
  }
  return PMDFC_OK;
}

int pmdfc_cceh_utilization(pmdfc_cceh_t* t, double* out) {
  if (!t || !out) return fail(PMDFC_ERR_ARG, "null argument");
  std::lock_guard<std::mutex> lk(t->mu);
  DevGuard g(t->dev);
  HIPCHK(hipDeviceSynchronize());
  int rc = read_ctl(t, (hipStream_t)0);
  if (rc) return rc;
  const uint64_t nsegs = std::min<uint64_t>(t->hctl->nsegs, t->max_segs);
  HIPCHK(hipMemset(t->popc, 0, sizeof(unsigned long long)));
  launch_popcount(t->occ, nsegs * 32, t->popc, (hipStream_t)0);
  unsigned long long c = 0;
  HIPCHK(hipMemcpy(&c, t->popc, sizeof c, hipMemcpyDeviceToHost));
  *out = (double)c / ((double)nsegs * kSlots) * 100.0;
  return PMDFC_OK;
}

int pmdfc_cceh_dump(pmdfc_cceh_t* t, uint32_t* dir_canon, uint32_t* local_depth, uint64_t* prefix,
                    uint64_t* keys, uint64_t* values, uint64_t* nseg_out) {
  if (!t) return fail(PMDFC_ERR_ARG, "null engine");
  std::lock_guard<std::mutex> lk(t->mu);
  DevGuard g(t->dev);
  HIPCHK(hipDeviceSynchronize());
  int rc = read_ctl(t, (hipStream_t)0);
  if (rc) return rc;
  uint32_t max_ld = t->hctl->max_ld;
  {
    std::vector<uint64_t> ws((size_t)kWStat << t->p1max);
    HIPCHK(hipMemcpy(ws.data(), t->wstat, ws.size() * 8, hipMemcpyDeviceToHost));
    for (size_t i = 6; i < ws.size(); i += kWStat) max_ld = std::max<uint32_t>(max_ld, (uint32_t)((ws[i] >> 16) & 0xFF));
  }
  const uint32_t D = std::max(t->D0, max_ld);  // logical global depth
  const uint32_t Dl = D - t->sbits;
  const uint64_t nlog = 1ULL << Dl;
  std::vector<uint64_t> hd(1ULL << t->p1);
  HIPCHK(hipMemcpy(hd.data(), t->hdr, hd.size() * 8, hipMemcpyDeviceToHost));
  std::vector<uint32_t> pl(std::min<uint64_t>(t->hctl->pool_cur, t->pool_cap));
  HIPCHK(hipMemcpy(pl.data(), t->pool, pl.size() * 4, hipMemcpyDeviceToHost));
  const uint32_t nsub = Dl - t->p1;  // logical index bits below the bucket
  std::vector<uint32_t> order;
  uint32_t cur = 0;
  for (uint64_t x = 0; x < nlog; ++x) {
    const uint64_t hb = hd[x >> nsub];
    const uint32_t db = hdr_db(hb);
    const uint64_t sub = (x & ((1ULL << nsub) - 1)) >> (nsub - db);
    const uint32_t e = pl[hdr_off(hb) + sub];
    const uint32_t sid = de_seg(e);
    const uint32_t L = de_ld(e);
    const uint32_t Ll = L - t->sbits;
    if ((x & ((1ULL << (Dl - Ll)) - 1)) == 0) {
      cur = (uint32_t)order.size();
      order.push_back(sid);
      if (local_depth) local_depth[cur] = L;
      if (prefix) prefix[cur] = ((uint64_t)t->shard << Ll) | (x >> (Dl - Ll));
    }
    if (dir_canon) dir_canon[x] = cur;
  }
  if (nseg_out) *nseg_out = order.size();
  if (keys || values) {
    std::vector<ulonglong2> buf(kSlots);
    for (size_t i = 0; i < order.size(); ++i) {
      HIPCHK(hipMemcpy(buf.data(), t->pairs + (size_t)order[i] * kSlots, kSlots * 16,
                       hipMemcpyDeviceToHost));
      for (uint32_t j = 0; j < kSlots; ++j) {
        if (keys) keys[i * kSlots + j] = buf[j].x;
        if (values) values[i * kSlots + j] = buf[j].x == kInvalid ? 0 : buf[j].y;
      }
    }
  }
  return PMDFC_OK;
}

int pmdfc_cceh_timing_enable(pmdfc_cceh_t* t, int on) {
  if (!t) return fail(PMDFC_ERR_ARG, "null engine");
  std::lock_guard<std::mutex> lk(t->mu);
  t->timing.on = (on & 1) != 0;
  t->count_lines = (on & 2) != 0;
  return PMDFC_OK;
}

int pmdfc_cceh_timing_read(pmdfc_cceh_t* t, double* ms_out, uint64_t* launches_out, int reset) {
  if (!t) return fail(PMDFC_ERR_ARG, "null engine");
  std::lock_guard<std::mutex> lk(t->mu);
  DevGuard g(t->dev);
  t->timing.flush_closed();
  for (int i = 0; i < PMDFC_K_COUNT; ++i) {
    if (ms_out) ms_out[i] = t->timing.ms[i];
    if (launches_out) launches_out[i] = t->timing.launches[i];
    if (reset) {
      t->timing.ms[i] = 0;
      t->timing.launches[i] = 0;
    }
  }
  return PMDFC_OK;
}

int pmdfc_cceh_debug_stamps(pmdfc_cceh_t* t, uint64_t* out, uint64_t n, uint32_t* nbuckets) {
  if (!t || !out) return fail(PMDFC_ERR_ARG, "null argument");
  if (!t->stamps) return fail(PMDFC_ERR_STATE, "stamps are off (create with PMDFC_STAMPS=1)");
  std::lock_guard<std::mutex> lk(t->mu);
  DevGuard g(t->dev);
  HIPCHK(hipDeviceSynchronize());
  // the last batch's set, or every set when n holds them all (PMDFC_STAMP_ROT)
  const uint64_t tot = stamp_words(t), all = tot * t->stamp_rot;
  const bool every = t->stamp_rot > 1 && n >= all;
  const uint64_t* src = every ? t->stamps : (t->stamp_cur ? t->stamp_cur : t->stamps);
  HIPCHK(hipMemcpy(out, src, std::min(n, every ? all : tot) * 8, hipMemcpyDeviceToHost));
  if (nbuckets) *nbuckets = 1u << t->p1max;  // (the stamp rows are laid out for p1max)
  return PMDFC_OK;
}

int pmdfc_cceh_last_get_lines(pmdfc_cceh_t* t, uint64_t* lines) {
  if (!t || !lines) return fail(PMDFC_ERR_ARG, "null argument");
  std::lock_guard<std::mutex> lk(t->mu);
  if (!t->last_get_counted) return fail(PMDFC_ERR_STATE, "last get was not counted (enable timing)");
  DevGuard g(t->dev);
  HIPCHK(hipDeviceSynchronize());
  const uint64_t nb = t->last_get_blocks;
  std::vector<uint32_t> p(nb);
  HIPCHK(hipMemcpy(p.data(), t->partials, nb * 4, hipMemcpyDeviceToHost));
  uint64_t sum = 0;
  for (auto v : p) sum += v;
  *lines = sum;
  return PMDFC_OK;
}

int pmdfc_hash64(const uint64_t* keys, uint64_t* out, uint64_t n, void* stream) {
  if (n && (!keys || !out)) return fail(PMDFC_ERR_ARG, "null argument");
  launch_hash(keys, out, n, (hipStream_t)stream);
  HIPCHK(hipGetLastError());
  return PMDFC_OK;
}

int pmdfc_gen_keys(uint64_t seed, uint64_t start, uint64_t* out, uint64_t n, void* stream) {
  if (n && !out) return fail(PMDFC_ERR_ARG, "null argument");
  launch_gen_keys(seed, start, out, n, (hipStream_t)stream);
  HIPCHK(hipGetLastError());
  return PMDFC_OK;
}

int pmdfc_route_by_shard(const uint64_t* keys, uint64_t n, uint32_t shard_bits, uint32_t* perm,
                         uint64_t* h_counts, int device, void* stream) {
  if (shard_bits > 16 || (n && (!keys || !perm || !h_counts))) return fail(PMDFC_ERR_ARG, "bad argument");
  DevGuard g(device);
  hipStream_t s = (hipStream_t)stream;
  const uint32_t G = 1u << shard_bits;
  if (n == 0) {
    for (uint32_t i = 0; i < G; ++i) h_counts[i] = 0;
    return PMDFC_OK;
  }
  uint32_t *own = nullptr, *own2 = nullptr, *idx = nullptr;
  uint64_t* starts = nullptr;
  void* tmp = nullptr;
  size_t bytes = 0;
  HIPCHK(hipMallocAsync((void**)&own, n * 4, s));
  HIPCHK(hipMallocAsync((void**)&own2, n * 4, s));
  HIPCHK(hipMallocAsync((void**)&idx, n * 4, s));
  HIPCHK(hipMallocAsync((void**)&starts, (G + 1) * 8, s));
  if (shard_bits == 0) {
    launch_owner(keys, n, 0, own, perm, s);  // own unused
    h_counts[0] = n;
  } else {
    launch_owner(keys, n, shard_bits, own, idx, s);
    HIPCHK(rocprim::radix_sort_pairs(nullptr, bytes, own, own2, idx, perm, (size_t)n, 0u, shard_bits, s));
    HIPCHK(hipMallocAsync(&tmp, bytes + 16, s));
    HIPCHK(rocprim::radix_sort_pairs(tmp, bytes, own, own2, idx, perm, (size_t)n, 0u, shard_bits, s));
    launch_bounds(own2, n, G, starts, s);
    std::vector<uint64_t> st(G + 1);
    HIPCHK(hipMemcpyAsync(st.data(), starts, (G + 1) * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    for (uint32_t i = 0; i < G; ++i) h_counts[i] = st[i + 1] - st[i];
    HIPCHK(hipFreeAsync(tmp, s));
  }
  HIPCHK(hipFreeAsync(own, s));
  HIPCHK(hipFreeAsync(own2, s));
  HIPCHK(hipFreeAsync(idx, s));
  HIPCHK(hipFreeAsync(starts, s));
  HIPCHK(hipStreamSynchronize(s));
  return PMDFC_OK;
}

struct pmdfc_router {
  pmdfc_router_config cfg;
  uint32_t G = 1;
  uint64_t rows = 0;
  uint32_t parity = 0;      // carry buffer the next pack reads
  uint32_t last_width = 0;  // width of the carried records (fixed while the carry is non-empty)
  uint32_t* tile_cnt = nullptr;
  uint32_t* cnt = nullptr;  // [2][G] carry counts
  uint32_t* ovf = nullptr;  // sticky count of ops dropped on a full carry
  uint64_t* crec = nullptr; // [2][G][carry_cap][kCarryWords]
  uint32_t* cpos = nullptr; // [2][G][carry_cap]
};

int pmdfc_router_create(const pmdfc_router_config* c, pmdfc_router_t** out) {
  if (!c || !out) return fail(PMDFC_ERR_ARG, "router_create: null argument");
  *out = nullptr;
  const uint32_t G = 1u << c->shard_bits;
  if (c->shard_bits > 4 || c->max_batch == 0 || c->cap == 0 || c->flags)
    return fail(PMDFC_ERR_ARG, "router_create: shard_bits <= 4, max_batch > 0, cap > 0, flags 0");
  if (c->cap * G >= 0xFFFFFFFFULL) return fail(PMDFC_ERR_ARG, "router_create: cap * 2^shard_bits < 2^32");
  DevGuard g(c->device);
  auto* r = new pmdfc_router();
  r->cfg = *c;
  if (!r->cfg.carry_cap) r->cfg.carry_cap = c->max_batch;
  r->G = G;
  r->rows = c->cap * G;
  const uint64_t cc = r->cfg.carry_cap;
  hipError_t e = hipSuccess;
  auto A = [&](void** p, size_t bytes) {
    if (e == hipSuccess) e = hipMalloc(p, bytes);
  };
  A((void**)&r->tile_cnt, (size_t)route_tiles(c->max_batch) * G * 4 + 4);
  A((void**)&r->cnt, 2 * G * 4);
  A((void**)&r->ovf, 4);
  A((void**)&r->crec, 2 * G * cc * kCarryWords * 8);
  A((void**)&r->cpos, 2 * G * cc * 4);
  if (e == hipSuccess) e = hipMemset(r->cnt, 0, 2 * G * 4);
  if (e == hipSuccess) e = hipMemset(r->ovf, 0, 4);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    pmdfc_router_destroy(r);
    return fail(PMDFC_ERR_HIP, "router_create", e);
  }
  *out = r;
  return PMDFC_OK;
}

int pmdfc_router_destroy(pmdfc_router_t* r) {
  if (!r) return PMDFC_OK;
  DevGuard g(r->cfg.device);
  for (void* p : {(void*)r->tile_cnt, (void*)r->cnt, (void*)r->ovf, (void*)r->crec, (void*)r->cpos})
    if (p) (void)hipFree(p);
  delete r;
  return PMDFC_OK;
}

uint64_t pmdfc_router_rows(const pmdfc_router_t* r) { return r ? r->rows : 0; }

static int router_pack(pmdfc_router_t* r, const uint64_t* keys, const uint64_t* values, const uint8_t* ops,
                       const uint8_t* keep, uint64_t n, uint32_t width, uint32_t base, uint64_t* send,
                       uint32_t* rowpos, uint64_t* values_out, uint8_t* status_out, void* stream, uint32_t self_g,
                       uint64_t* self_dst);

int pmdfc_router_pack(pmdfc_router_t* r, const uint64_t* keys, const uint64_t* values, const uint8_t* ops,
                      const uint8_t* keep, uint64_t n, uint32_t width, uint32_t base, uint64_t* send,
                      uint32_t* rowpos, uint64_t* values_out, uint8_t* status_out, void* stream) {
  return router_pack(r, keys, values, ops, keep, n, width, base, send, rowpos, values_out, status_out, stream, 0,
                     nullptr);
}

// (self_dst: owner self_g's block goes there instead of into send -- the
// native loop packs the local block straight into its receive slot)
static int router_pack(pmdfc_router_t* r, const uint64_t* keys, const uint64_t* values, const uint8_t* ops,
                       const uint8_t* keep, uint64_t n, uint32_t width, uint32_t base, uint64_t* send,
                       uint32_t* rowpos, uint64_t* values_out, uint8_t* status_out, void* stream, uint32_t self_g,
                       uint64_t* self_dst) {
  if (!r || width < 1 || width > 3 || !send || !rowpos || (n && (!keys || !status_out)) ||
      (width >= 2 && n && !values) || (width == 3 && n && !ops))
    return fail(PMDFC_ERR_ARG, "router_pack: bad argument (width 1..3)");
  if (n > r->cfg.max_batch) return fail(PMDFC_ERR_ARG, "router_pack: n > max_batch");
  if ((uint64_t)base + n >= kRouteNone) return fail(PMDFC_ERR_ARG, "router_pack: base + n >= 2^32 - 1");
  if (r->last_width && r->last_width != width)
    return fail(PMDFC_ERR_STATE, "router_pack: carried records have another width (finish or reset the call)");
  DevGuard g(r->cfg.device);
  const uint64_t cc = r->cfg.carry_cap, G = r->G;
  const uint32_t pi = r->parity, po = pi ^ 1u;
  RouteArgs a{keys, values, ops, keep, n, r->cfg.shard_bits, width, r->cfg.cap, cc, base, send, rowpos,
              values_out, status_out, r->tile_cnt, r->cnt + pi * G, r->cnt + po * G,
              r->crec + pi * G * cc * kCarryWords, r->crec + po * G * cc * kCarryWords, r->cpos + pi * G * cc,
              r->cpos + po * G * cc, r->ovf, self_g, self_dst};
  launch_route_pack(a, (hipStream_t)stream);
  HIPCHK(hipGetLastError());
  r->parity = po;
  r->last_width = width;
  return PMDFC_OK;
}

int pmdfc_router_unpack(pmdfc_router_t* r, const void* back, uint32_t resp_width, const uint32_t* rowpos,
                        uint64_t* values_out, uint8_t* status_out, void* stream) {
  if (!r || resp_width > 1 || !back || !rowpos || !status_out) return fail(PMDFC_ERR_ARG, "router_unpack: bad argument");
  DevGuard g(r->cfg.device);
  launch_route_unpack(back, resp_width, rowpos, r->rows, values_out, status_out, (hipStream_t)stream);
  HIPCHK(hipGetLastError());
  return PMDFC_OK;
}

int pmdfc_router_carried(pmdfc_router_t* r, uint64_t* d_out, void* stream) {
  if (!r || !d_out) return fail(PMDFC_ERR_ARG, "router_carried: bad argument");
  DevGuard g(r->cfg.device);
  launch_route_carried(r->cnt + r->parity * r->G, r->G, d_out, (hipStream_t)stream);
  HIPCHK(hipGetLastError());
  return PMDFC_OK;
}

int pmdfc_router_end_call(pmdfc_router_t* r) {
  if (!r) return fail(PMDFC_ERR_ARG, "router_end_call: null router");
  r->last_width = 0;
  return PMDFC_OK;
}

int pmdfc_router_overflow_count(pmdfc_router_t* r, uint64_t* h_out, void* stream) {
  if (!r || !h_out) return fail(PMDFC_ERR_ARG, "router_overflow_count: bad argument");
  DevGuard g(r->cfg.device);
  uint32_t v = 0;
  HIPCHK(hipMemcpyAsync(&v, r->ovf, 4, hipMemcpyDeviceToHost, (hipStream_t)stream));
  HIPCHK(hipStreamSynchronize((hipStream_t)stream));
  *h_out = v;
  return PMDFC_OK;
}

int pmdfc_router_reset(pmdfc_router_t* r, void* stream) {
  if (!r) return fail(PMDFC_ERR_ARG, "router_reset: null router");
  DevGuard g(r->cfg.device);
  HIPCHK(hipMemsetAsync(r->cnt, 0, 2 * r->G * 4, (hipStream_t)stream));
  HIPCHK(hipMemsetAsync(r->ovf, 0, 4, (hipStream_t)stream));
  r->parity = 0;
  r->last_width = 0;
  return PMDFC_OK;
}

int pmdfc_router_dedupe(pmdfc_router_t* r, const uint64_t* keys, const uint8_t* keep_in, uint64_t n, uint32_t base,
                        uint8_t* keep_out, uint32_t* lead_out, void* stream) {
  if (!r || (n && (!keys || !keep_out || !lead_out))) return fail(PMDFC_ERR_ARG, "router_dedupe: bad argument");
  if (n > r->cfg.max_batch) return fail(PMDFC_ERR_ARG, "router_dedupe: n > max_batch");
  if ((uint64_t)base + n >= kRouteNone) return fail(PMDFC_ERR_ARG, "router_dedupe: base + n >= 2^32 - 1");
  if (!n) return PMDFC_OK;
  DevGuard g(r->cfg.device);
  launch_route_dedupe(keys, keep_in, n, base, keep_out, lead_out, (hipStream_t)stream);
  HIPCHK(hipGetLastError());
  return PMDFC_OK;
}

int pmdfc_router_fill(const uint32_t* lead, uint64_t n, uint64_t* values_out, uint8_t* status_out, int device,
                      void* stream) {
  if (n && (!lead || !status_out)) return fail(PMDFC_ERR_ARG, "router_fill: bad argument");
  DevGuard g(device);
  launch_route_fill(lead, n, values_out, status_out, (hipStream_t)stream);
  HIPCHK(hipGetLastError());
  return PMDFC_OK;
}

int pmdfc_route_split(const uint64_t* recv, uint64_t rows, uint32_t width, uint64_t* keys, uint64_t* values,
                      uint8_t* ops, int device, void* stream) {
  if (width < 1 || width > 3 || (rows && (!recv || !keys || (width >= 2 && !values) || (width == 3 && !ops))))
    return fail(PMDFC_ERR_ARG, "route_split: bad argument");
  DevGuard g(device);
  launch_route_split(recv, rows, width, keys, values, ops, (hipStream_t)stream);
  HIPCHK(hipGetLastError());
  return PMDFC_OK;
}

int pmdfc_route_respond(const uint64_t* values, const uint8_t* status, uint64_t rows, uint64_t* resp,
                        int device, void* stream) {
  if (rows && (!values || !status || !resp)) return fail(PMDFC_ERR_ARG, "route_respond: bad argument");
  DevGuard g(device);
  launch_route_resp(values, status, rows, resp, (hipStream_t)stream);
  HIPCHK(hipGetLastError());
  return PMDFC_OK;
}

int pmdfc_ubench_gather64(const void* buf, uint64_t nlines, const uint32_t* table, uint32_t tmask,
                          uint64_t n_ops, uint64_t seed, uint64_t* out, void* stream) {
  if (!buf || !out || nlines == 0) return fail(PMDFC_ERR_ARG, "bad argument");
  launch_gather64(buf, nlines, table, tmask, n_ops, seed, out, (hipStream_t)stream);
  HIPCHK(hipGetLastError());
  return PMDFC_OK;
}

int pmdfc_ubench_gather(const void* buf, uint64_t nbytes, uint32_t line, uint32_t depth, const uint32_t* table,
                        uint32_t tmask, uint64_t n_ops, uint64_t seed, uint64_t* out, uint64_t omask, void* stream) {
  if (!buf || !out || (omask & (omask + 1))) return fail(PMDFC_ERR_ARG, "bad argument (omask + 1: a power of two)");
  if (n_ops % depth) return fail(PMDFC_ERR_ARG, "n_ops must be a multiple of depth");
  if (launch_gather(buf, nbytes, line, depth, table, tmask, n_ops, seed, out, omask, (hipStream_t)stream))
    return fail(PMDFC_ERR_ARG, "line 64|128, depth 1|2|4, nbytes >= line");
  HIPCHK(hipGetLastError());
  return PMDFC_OK;
}

int pmdfc_ubench_scatter16(void* buf, uint64_t nbytes, uint32_t depth, uint64_t n_ops, uint64_t seed,
                           void* stream) {
  if (!buf) return fail(PMDFC_ERR_ARG, "bad argument");
  if (launch_scatter16(buf, nbytes, depth, n_ops, seed, (hipStream_t)stream))
    return fail(PMDFC_ERR_ARG, "depth 1|4, n_ops a multiple of depth, nbytes >= 16");
  HIPCHK(hipGetLastError());
  return PMDFC_OK;
}

// ------------------------------------------------------------------- bloom

int pmdfc_bloom_create(uint64_t nbits, uint32_t k, int device, pmdfc_bloom_t** out) {
  if (!out || nbits == 0 || k == 0 || k > 64 || nbits >= (1ULL << 32))
    return fail(PMDFC_ERR_ARG, "bloom: need 0 < nbits < 2^32 (unsigned int index, bloom_filter.c:87) and 0 < k <= 64");
  DevGuard g(device);
  auto* b = new pmdfc_bloom();
  b->dev = device;
  b->nbits = nbits;
  b->nwords = (nbits + 63) / 64;
  b->k = k;
  hipError_t e = hipMalloc(&b->bm, b->nwords * 8);
  if (e != hipSuccess) {
    delete b;
    return fail(PMDFC_ERR_NOMEM, "bloom hipMalloc", e);
  }
  e = hipMemset(b->bm, 0, b->nwords * 8);
  if (e != hipSuccess) {
    (void)hipFree(b->bm);
    delete b;
    return fail(PMDFC_ERR_HIP, "bloom memset", e);
  }
  *out = b;
  return PMDFC_OK;
}

int pmdfc_bloom_destroy(pmdfc_bloom_t* b) {
  if (!b) return PMDFC_OK;
  DevGuard g(b->dev);
  (void)hipDeviceSynchronize();
  (void)hipFree(b->bm);
  delete b;
  return PMDFC_OK;
}

int pmdfc_bloom_clear(pmdfc_bloom_t* b, void* stream) {
  if (!b) return fail(PMDFC_ERR_ARG, "null bloom");
  DevGuard g(b->dev);
  HIPCHK(hipMemsetAsync(b->bm, 0, b->nwords * 8, (hipStream_t)stream));
  return PMDFC_OK;
}

int pmdfc_bloom_add(pmdfc_bloom_t* b, const uint64_t* keys, uint64_t n, void* stream) {
  if (!b || (n && !keys)) return fail(PMDFC_ERR_ARG, "null argument");
  DevGuard g(b->dev);
  launch_bloom_add(b->bm, b->nbits, b->k, keys, n, (hipStream_t)stream);
  HIPCHK(hipGetLastError());
  return PMDFC_OK;
}

int pmdfc_bloom_probe(pmdfc_bloom_t* b, const uint64_t* keys, uint8_t* out, uint64_t n, void* stream) {
  if (!b || (n && (!keys || !out))) return fail(PMDFC_ERR_ARG, "null argument");
  DevGuard g(b->dev);
  launch_bloom_probe(b->bm, b->nbits, b->k, keys, out, n, (hipStream_t)stream);
  HIPCHK(hipGetLastError());
  return PMDFC_OK;
}

int pmdfc_bloom_bitmap(pmdfc_bloom_t* b, uint64_t** d_bitmap, uint64_t* nwords) {
  if (!b || !d_bitmap || !nwords) return fail(PMDFC_ERR_ARG, "null argument");
  *d_bitmap = b->bm;
  *nwords = b->nwords;
  return PMDFC_OK;
}

int pmdfc_bloom_set_bitmap_host(pmdfc_bloom_t* b, const uint64_t* host, uint64_t nwords) {
  if (!b || !host || nwords != b->nwords) return fail(PMDFC_ERR_ARG, "bitmap size mismatch");
  DevGuard g(b->dev);
  HIPCHK(hipMemcpy(b->bm, host, nwords * 8, hipMemcpyHostToDevice));
  return PMDFC_OK;
}

int pmdfc_bloom_get_bitmap_host(pmdfc_bloom_t* b, uint64_t* host, uint64_t nwords) {
  if (!b || !host || nwords != b->nwords) return fail(PMDFC_ERR_ARG, "bitmap size mismatch");
  DevGuard g(b->dev);
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(host, b->bm, nwords * 8, hipMemcpyDeviceToHost));
  return PMDFC_OK;
}

int pmdfc_bloom_probe_then_get(pmdfc_bloom_t* b, pmdfc_cceh_t* t, const uint64_t* keys,
                               uint64_t* vout, uint8_t* st, uint64_t n, void* stream) {
  if (!b || !t || (n && (!keys || !vout || !st))) return fail(PMDFC_ERR_ARG, "null argument");
  if (b->dev != t->dev) return fail(PMDFC_ERR_ARG, "bloom and index on different devices");
  std::lock_guard<std::mutex> lk(t->mu);
  DevGuard g(t->dev);
  hipStream_t s = (hipStream_t)stream;
  t->timing.begin(PMDFC_K_BLOOM, s);
  launch_bloom_get(b->bm, b->nbits, b->k, keys, vout, st, n, t->geo(), t->pairs, s);
  t->timing.end(s);
  HIPCHK(hipGetLastError());
  return PMDFC_OK;
}

// ----------------------------------------------------- counting bloom filter

int pmdfc_cbf_create(uint64_t nbits, uint32_t k, int device, pmdfc_cbf_t** out) {
  if (!out || nbits == 0 || nbits >= (1ULL << 31) || k == 0 || k > 64)
    return fail(PMDFC_ERR_ARG, "cbf: need 0 < nbits < 2^31 (int index, counting_bloom_filter.h:252) and 0 < k <= 64");
  DevGuard g(device);
  auto* f = new pmdfc_cbf();
  f->dev = device;
  f->nbits = nbits;
  f->nwords = (nbits + 63) / 64;
  f->padded = (nbits + kCbfChunk - 1) / kCbfChunk * kCbfChunk;
  f->k = k;
  hipError_t e = hipMalloc(&f->cnt, f->padded);
  if (e == hipSuccess) e = hipMalloc(&f->bm, f->nwords * 8);
  if (e == hipSuccess) e = hipMalloc(&f->flag, 256);
  if (e == hipSuccess) e = hipMemset(f->cnt, 0, f->padded);
  if (e == hipSuccess) e = hipMemset(f->bm, 0, f->nwords * 8);
  if (e != hipSuccess) {
    (void)hipFree(f->cnt);
    (void)hipFree(f->bm);
    (void)hipFree(f->flag);
    delete f;
    return fail(PMDFC_ERR_NOMEM, "cbf hipMalloc", e);
  }
  *out = f;
  return PMDFC_OK;
}

int pmdfc_cbf_destroy(pmdfc_cbf_t* f) {
  if (!f) return PMDFC_OK;
  DevGuard g(f->dev);
  (void)hipDeviceSynchronize();
  (void)hipFree(f->cnt);
  (void)hipFree(f->bm);
  (void)hipFree(f->flag);
  delete f;
  return PMDFC_OK;
}

int pmdfc_cbf_clear(pmdfc_cbf_t* f, void* stream) {
  if (!f) return fail(PMDFC_ERR_ARG, "null cbf");
  DevGuard g(f->dev);
  HIPCHK(hipMemsetAsync(f->cnt, 0, f->padded, (hipStream_t)stream));
  HIPCHK(hipMemsetAsync(f->bm, 0, f->nwords * 8, (hipStream_t)stream));
  return PMDFC_OK;
}

int pmdfc_cbf_insert(pmdfc_cbf_t* f, const uint64_t* keys, uint64_t n, void* stream) {
  if (!f || (n && !keys)) return fail(PMDFC_ERR_ARG, "null argument");
  DevGuard g(f->dev);
  launch_cbf_insert(f->cnt, f->nbits, f->k, keys, nullptr, n, (hipStream_t)stream);
  HIPCHK(hipGetLastError());
  return PMDFC_OK;
}

int pmdfc_cbf_insert_ops(pmdfc_cbf_t* f, const uint8_t* ops, const uint64_t* keys, uint64_t n,
                         void* stream) {
  if (!f || (n && (!keys || !ops))) return fail(PMDFC_ERR_ARG, "null argument");
  DevGuard g(f->dev);
  launch_cbf_insert(f->cnt, f->nbits, f->k, keys, ops, n, (hipStream_t)stream);
  HIPCHK(hipGetLastError());
  return PMDFC_OK;
}

int pmdfc_cbf_delete(pmdfc_cbf_t* f, const uint64_t* keys, uint8_t* deleted, uint64_t n,
                     void* stream) {
  if (!f || (n && (!keys || !deleted))) return fail(PMDFC_ERR_ARG, "null argument");
  DevGuard g(f->dev);
  launch_cbf_delete(f->cnt, f->nbits, f->k, keys, deleted, n, f->flag, (hipStream_t)stream);
  HIPCHK(hipGetLastError());
  return PMDFC_OK;
}

int pmdfc_cbf_query(pmdfc_cbf_t* f, const uint64_t* keys, uint8_t* out, uint64_t n, void* stream) {
  if (!f || (n && (!keys || !out))) return fail(PMDFC_ERR_ARG, "null argument");
  DevGuard g(f->dev);
  launch_cbf_query(f->cnt, f->nbits, f->k, keys, out, n, (hipStream_t)stream);
  HIPCHK(hipGetLastError());
  return PMDFC_OK;
}

int pmdfc_cbf_pack(pmdfc_cbf_t* f, void* stream) {
  if (!f) return fail(PMDFC_ERR_ARG, "null cbf");
  DevGuard g(f->dev);
  launch_cbf_pack(f->cnt, f->nbits, f->bm, (hipStream_t)stream);
  HIPCHK(hipGetLastError());
  return PMDFC_OK;
}

int pmdfc_cbf_query_bits(pmdfc_cbf_t* f, const uint64_t* keys, uint8_t* out, uint64_t n,
                         void* stream) {
  if (!f || (n && (!keys || !out))) return fail(PMDFC_ERR_ARG, "null argument");
  DevGuard g(f->dev);
  launch_bloom_probe(f->bm, f->nbits, f->k, keys, out, n, (hipStream_t)stream);
  HIPCHK(hipGetLastError());
  return PMDFC_OK;
}

int pmdfc_cbf_export(pmdfc_cbf_t* f, pmdfc_bloom_t* b, void* stream) {
  if (!f || !b) return fail(PMDFC_ERR_ARG, "null argument");
  if (b->nbits != f->nbits) return fail(PMDFC_ERR_ARG, "cbf and bloom differ in nbits");
  DevGuard g(f->dev);
  HIPCHK(hipMemcpyAsync(b->bm, f->bm, f->nwords * 8, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return PMDFC_OK;
}

int pmdfc_cbf_counters(pmdfc_cbf_t* f, uint8_t** d_counters, uint64_t** d_bitmap, uint64_t* nwords) {
  if (!f || !d_counters || !d_bitmap || !nwords) return fail(PMDFC_ERR_ARG, "null argument");
  *d_counters = f->cnt;
  *d_bitmap = f->bm;
  *nwords = f->nwords;
  return PMDFC_OK;
}

int pmdfc_cbf_get_counters_host(pmdfc_cbf_t* f, uint8_t* host, uint64_t nbits) {
  if (!f || !host || nbits != f->nbits) return fail(PMDFC_ERR_ARG, "counter size mismatch");
  DevGuard g(f->dev);
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(host, f->cnt, nbits, hipMemcpyDeviceToHost));
  return PMDFC_OK;
}

int pmdfc_cbf_get_bitmap_host(pmdfc_cbf_t* f, uint64_t* host, uint64_t nwords) {
  if (!f || !host || nwords != f->nwords) return fail(PMDFC_ERR_ARG, "bitmap size mismatch");
  DevGuard g(f->dev);
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(host, f->bm, nwords * 8, hipMemcpyDeviceToHost));
  return PMDFC_OK;
}

// ----------------------------------------------------------- trace ingestion

int pmdfc_trace_create(int device, pmdfc_trace_t** out) {
  if (!out) return fail(PMDFC_ERR_ARG, "null argument");
  DevGuard g(device);
  auto* t = new pmdfc_trace();
  t->dev = device;
  hipError_t e = hipMalloc(&t->small, 64);
  if (e != hipSuccess) {
    delete t;
    return fail(PMDFC_ERR_NOMEM, "trace hipMalloc", e);
  }
  *out = t;
  return PMDFC_OK;
}

static void trace_free(pmdfc_trace* t) {
  (void)hipFree(t->nl);
  (void)hipFree(t->lines);
  (void)hipFree(t->pages);
  (void)hipFree(t->cum);
  (void)hipFree(t->temp);
  (void)hipFree(t->tile_cnt);
  (void)hipFree(t->tile_off);
  t->tile_cnt = nullptr;
  t->tile_off = nullptr;
  t->nl = nullptr;
  t->lines = nullptr;
  t->pages = t->cum = nullptr;
  t->temp = nullptr;
  t->cap_bytes = t->cap_lines = 0;
  t->temp_bytes = 0;
}

int pmdfc_trace_destroy(pmdfc_trace_t* t) {
  if (!t) return PMDFC_OK;
  DevGuard g(t->dev);
  (void)hipDeviceSynchronize();
  trace_free(t);
  (void)hipFree(t->small);
  delete t;
  return PMDFC_OK;
}

int pmdfc_trace_parse(pmdfc_trace_t* t, const char* text, uint64_t nbytes, uint64_t num_data,
                      uint8_t* ops, uint64_t* keys, uint64_t* info, void* stream) {
  if (!t || !info || (nbytes && !text) || (num_data && (!ops || !keys)))
    return fail(PMDFC_ERR_ARG, "null argument");
  DevGuard g(t->dev);
  hipStream_t s = (hipStream_t)stream;
  const uint64_t cap_lines = nbytes + 1;
  if (nbytes > t->cap_bytes || cap_lines > t->cap_lines) {
    HIPCHK(hipStreamSynchronize(s));
    trace_free(t);
    const uint64_t tiles = std::max<uint64_t>(trace_nl_tiles(nbytes), 1);
    const size_t tb = std::max(trace_scan_temp_bytes(tiles), trace_scan_temp_bytes(cap_lines));
    hipError_t e = hipMalloc(&t->nl, std::max<uint64_t>(nbytes, 1) * 8);
    if (e == hipSuccess) e = hipMalloc(&t->tile_cnt, tiles * 8);
    if (e == hipSuccess) e = hipMalloc(&t->tile_off, tiles * 8);
    if (e == hipSuccess) e = hipMalloc(&t->lines, cap_lines * sizeof(TraceLine));
    if (e == hipSuccess) e = hipMalloc(&t->pages, cap_lines * 8);
    if (e == hipSuccess) e = hipMalloc(&t->cum, cap_lines * 8);
    if (e == hipSuccess) e = hipMalloc(&t->temp, std::max<size_t>(tb, 256));
    if (e != hipSuccess) {
      trace_free(t);
      return fail(PMDFC_ERR_NOMEM, "trace scratch", e);
    }
    t->cap_bytes = nbytes;
    t->cap_lines = cap_lines;
    t->temp_bytes = std::max<size_t>(tb, 256);
  }
  uint64_t h[2] = {0, 0};
  HIPCHK(hipMemsetAsync(t->small, 0, 16, s));
  HIPCHK(hipMemsetAsync(t->small + 1, 0xFF, 8, s));  // first bad = ~0
  if (nbytes)
    HIPCHK(launch_trace_newlines(text, nbytes, t->nl, t->small, t->tile_cnt, t->tile_off, t->temp,
                                 t->temp_bytes, s));
  char last = '\n';
  HIPCHK(hipMemcpyAsync(h, t->small, 8, hipMemcpyDeviceToHost, s));
  if (nbytes) HIPCHK(hipMemcpyAsync(&last, text + nbytes - 1, 1, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  const uint64_t nnl = h[0];
  const uint64_t nlines = nnl + (last != '\n' ? 1 : 0);  // getline: a last unterminated line
  HIPCHK(launch_trace_lines(text, nbytes, t->nl, nnl, nlines, t->lines, t->pages, t->cum,
                            (unsigned long long*)(t->small + 1), num_data, t->small + 2, t->temp,
                            t->temp_bytes, s));
  HIPCHK(hipMemcpyAsync(info, t->small + 2, 5 * 8, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  if (info[4] != ~0ull && info[4] <= info[3])
    return fail(PMDFC_ERR_ARG, "trace: malformed line before the replay's stop line (replay_KV.cpp:222-238 would throw)");
  if (info[0] < num_data)
    return fail(PMDFC_ERR_ARG, "trace: fewer ops than num_data (replay_KV.cpp:264-266 would read past its vectors)");
  launch_trace_expand(t->lines, t->cum, t->pages, nlines, info[0], ops, keys, s);
  HIPCHK(hipGetLastError());
  return PMDFC_OK;
}

// ------------------------------------------------------------------ extents

int pmdfc_cceh_insert_extent(pmdfc_cceh_t* t, int convention, const uint64_t* keys,
                             const uint64_t* cl, const uint64_t* lens, const uint64_t* vals, uint64_t n,
                             uint64_t* n_entries, void* stream) {
  if (!t || (n && (!keys || !lens || !vals)) || (convention != 0 && convention != 1))
    return fail(PMDFC_ERR_ARG, "bad argument");
  if (n_entries) *n_entries = 0;
  if (n == 0) return PMDFC_OK;
  const bool src = convention == 1;
  hipStream_t s = (hipStream_t)stream;
  uint64_t total = 0;
  uint64_t *cnt = nullptr, *cum = nullptr, *ok = nullptr, *ov = nullptr;
  uint8_t* st = nullptr;
  {
    DevGuard g(t->dev);
    HIPCHK(hipMallocAsync((void**)&cnt, n * 8, s));
    HIPCHK(hipMallocAsync((void**)&cum, n * 8, s));
    HIPCHK(launch_extent_count(src, keys, cl, lens, n, cnt, cum, s));
    HIPCHK(hipMemcpyAsync(&total, cum + n - 1, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    HIPCHK(hipMallocAsync((void**)&ok, total * 8, s));
    HIPCHK(hipMallocAsync((void**)&ov, total * 8, s));
    HIPCHK(hipMallocAsync((void**)&st, std::min<uint64_t>(total, t->max_batch), s));
    launch_extent_expand(src, keys, cl, lens, vals, n, cum, ok, ov, s);
    HIPCHK(hipGetLastError());
  }
  int rc = PMDFC_OK;
  for (uint64_t off = 0; off < total && rc == PMDFC_OK; off += t->max_batch)
    rc = do_insert(t, ok + off, ov + off, 1, st, std::min<uint64_t>(t->max_batch, total - off), s);
  DevGuard g(t->dev);
  (void)hipFreeAsync(cnt, s);
  (void)hipFreeAsync(cum, s);
  (void)hipFreeAsync(ok, s);
  (void)hipFreeAsync(ov, s);
  (void)hipFreeAsync(st, s);
  if (n_entries) *n_entries = total;
  return rc;
}

int pmdfc_cceh_get_extent(pmdfc_cceh_t* t, int convention, const uint64_t* keys, const uint64_t* cl,
                          uint64_t* vout, uint8_t* st, uint64_t n, void* stream) {
  if (!t || (n && (!keys || !vout || !st)) || (convention != 0 && convention != 1))
    return fail(PMDFC_ERR_ARG, "bad argument");
  if (n == 0) return PMDFC_OK;
  const uint32_t per = extent_targets_per_key(convention == 1);
  hipStream_t s = (hipStream_t)stream;
  uint64_t *tk = nullptr, *tv = nullptr;
  uint8_t* ts = nullptr;
  {
    DevGuard g(t->dev);
    HIPCHK(hipMallocAsync((void**)&tk, n * per * 8, s));
    HIPCHK(hipMallocAsync((void**)&tv, n * per * 8, s));
    HIPCHK(hipMallocAsync((void**)&ts, n * per, s));
    launch_extent_targets(keys, cl, n, per, tk, s);
    HIPCHK(hipGetLastError());
  }
  int rc = do_get(t, tk, tv, ts, n * per, stream);
  DevGuard g(t->dev);
  if (rc == PMDFC_OK) {
    launch_extent_pick(tv, ts, n, per, vout, st, s);
    HIPCHK(hipGetLastError());
  }
  (void)hipFreeAsync(tk, s);
  (void)hipFreeAsync(tv, s);
  (void)hipFreeAsync(ts, s);
  return rc;
}

}  // extern "C"

// ------------------------------------------------------- native routed batches
//
// The loop of pmdfc_amd.dist.BlockRouter._call_body in C++ with RCCL called
// directly: per batch one pack (route.hip), one equal-split all-to-all of the
// owner blocks, the owner's engine on the received rows, one all-to-all of
// the responses and one unpack.  Two streams joined by events: the
// communicator's (packs and both exchanges) and the caller's (the engine and
// the unpacks), so batch i+1's pack and request exchange and batch i-1's
// response exchange run while batch i is applied.  Buffers: requests and
// responses double-buffered, row positions triple-buffered (pack i+3 waits
// for unpack i).
#include <rccl/rccl.h>

struct pmdfc_comm {
  ncclComm_t comm = nullptr;
  int nranks = 1, rank = 0, device = 0;
  hipStream_t cs = nullptr;  // the exchanges' stream
  hipEvent_t ev[14] = {};
  // host-staged transport (pmdfc_comm_create_host): the exchanges go
  // through the caller's functions on pinned host copies instead of RCCL
  pmdfc_host_exchange_fn xchg = nullptr;
  pmdfc_host_allreduce_fn amax = nullptr;
  void* xctx = nullptr;
  uint8_t* hbuf = nullptr;  // [send | recv] staging, 2 * hcap bytes
  size_t hcap = 0;
};

namespace {
int nccl_fail(const char* what, ncclResult_t r) {
  char buf[256];
  snprintf(buf, sizeof buf, "%s: %s", what, ncclGetErrorString(r));
  return fail(PMDFC_ERR_HIP, buf);
}
}  // namespace

#define NCCLCHK(x)                                   \
  do {                                               \
    ncclResult_t r_ = (x);                           \
    if (r_ != ncclSuccess) return nccl_fail(#x, r_); \
  } while (0)

static_assert(sizeof(ncclUniqueId) == PMDFC_COMM_ID_BYTES, "RCCL unique id size");

int pmdfc_comm_id(uint8_t* id_out) {
  if (!id_out) return fail(PMDFC_ERR_ARG, "comm_id: null output");
  ncclUniqueId id;
  NCCLCHK(ncclGetUniqueId(&id));
  memcpy(id_out, &id, sizeof id);
  return PMDFC_OK;
}

int pmdfc_comm_create(const uint8_t* id, int nranks, int rank, int device, pmdfc_comm_t** out) {
  if (!id || !out || nranks < 1 || rank < 0 || rank >= nranks) return fail(PMDFC_ERR_ARG, "comm_create: bad argument");
  *out = nullptr;
  DevGuard g(device);
  auto* c = new pmdfc_comm();
  c->nranks = nranks;
  c->rank = rank;
  c->device = device;
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof uid);
  ncclResult_t nr = ncclCommInitRank(&c->comm, nranks, uid, rank);
  if (nr != ncclSuccess) {
    delete c;
    return nccl_fail("ncclCommInitRank", nr);
  }
  hipError_t e = hipStreamCreateWithFlags(&c->cs, hipStreamNonBlocking);
  for (auto& ev : c->ev)
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  if (e != hipSuccess) {
    pmdfc_comm_destroy(c);
    return fail(PMDFC_ERR_HIP, "comm_create", e);
  }
  *out = c;
  return PMDFC_OK;
}

int pmdfc_comm_create_host(int nranks, int rank, int device, pmdfc_host_exchange_fn xchg,
                           pmdfc_host_allreduce_fn amax, void* ctx, pmdfc_comm_t** out) {
  if (!out || !xchg || !amax || nranks < 1 || rank < 0 || rank >= nranks)
    return fail(PMDFC_ERR_ARG, "comm_create_host: bad argument");
  *out = nullptr;
  DevGuard g(device);
  auto* c = new pmdfc_comm();
  c->nranks = nranks;
  c->rank = rank;
  c->device = device;
  c->xchg = xchg;
  c->amax = amax;
  c->xctx = ctx;
  hipError_t e = hipStreamCreateWithFlags(&c->cs, hipStreamNonBlocking);
  for (auto& ev : c->ev)
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  if (e != hipSuccess) {
    pmdfc_comm_destroy(c);
    return fail(PMDFC_ERR_HIP, "comm_create_host", e);
  }
  *out = c;
  return PMDFC_OK;
}

int pmdfc_comm_destroy(pmdfc_comm_t* c) {
  if (!c) return PMDFC_OK;
  DevGuard g(c->device);
  if (c->cs) (void)hipStreamSynchronize(c->cs);
  if (c->hbuf) (void)hipHostFree(c->hbuf);
  if (c->comm) (void)ncclCommDestroy(c->comm);
  for (auto& ev : c->ev)
    if (ev) (void)hipEventDestroy(ev);
  if (c->cs) (void)hipStreamDestroy(c->cs);
  delete c;
  return PMDFC_OK;
}

// width 1: Get, 2: Insert, 3: mixed (ops; the received rows are split into
// the engine's key / value / op arrays, applied by pmdfc_cceh_mixed and
// answered as 16-B responses, as BlockRouter._run_mixed does)
static int route_batches(pmdfc_router_t* r, pmdfc_cceh_t* t, pmdfc_comm_t* c, uint32_t width, const uint8_t* ops,
                         const uint64_t* keys, const uint64_t* values, const uint64_t* bounds, uint64_t nb,
                         uint32_t dedupe, uint64_t* vout, uint8_t* st, void* stream);

int pmdfc_route_batches(pmdfc_router_t* r, pmdfc_cceh_t* t, pmdfc_comm_t* c, uint32_t width, const uint64_t* keys,
                        const uint64_t* values, const uint64_t* bounds, uint64_t nb, uint32_t dedupe,
                        uint64_t* vout, uint8_t* st, void* stream) {
  if (width != 1 && width != 2) return fail(PMDFC_ERR_ARG, "route_batches: bad argument (width 1: Get, 2: Insert)");
  return route_batches(r, t, c, width, nullptr, keys, values, bounds, nb, dedupe, vout, st, stream);
}

int pmdfc_route_mixed_batches(pmdfc_router_t* r, pmdfc_cceh_t* t, pmdfc_comm_t* c, const uint8_t* ops,
                              const uint64_t* keys, const uint64_t* values, const uint64_t* bounds, uint64_t nb,
                              uint64_t* vout, uint8_t* st, void* stream) {
  if (!ops) return fail(PMDFC_ERR_ARG, "route_mixed_batches: null ops");
  return route_batches(r, t, c, 3, ops, keys, values, bounds, nb, 0, vout, st, stream);
}

static int route_batches(pmdfc_router_t* r, pmdfc_cceh_t* t, pmdfc_comm_t* c, uint32_t width, const uint8_t* ops,
                         const uint64_t* keys, const uint64_t* values, const uint64_t* bounds, uint64_t nb,
                         uint32_t dedupe, uint64_t* vout, uint8_t* st, void* stream) {
  if (!r || !t || !c || width < 1 || width > 3 || !bounds || !nb || !st || (width != 2 && !vout) ||
      (width >= 2 && !values) || (width == 3 && !ops) || !keys)
    return fail(PMDFC_ERR_ARG, "route_batches: bad argument (width 1: Get, 2: Insert, 3: mixed)");
  if ((int)r->G != c->nranks) return fail(PMDFC_ERR_ARG, "route_batches: 2^shard_bits != communicator ranks");
  if (r->rows > t->max_batch) return fail(PMDFC_ERR_ARG, "route_batches: engine max_batch < router rows");
  if (r->last_width) return fail(PMDFC_ERR_STATE, "route_batches: the router holds another call's carry");
  const uint64_t total = bounds[nb] - bounds[0];
  for (uint64_t i = 0; i < nb; ++i)
    if (bounds[i + 1] < bounds[i] || bounds[i + 1] - bounds[i] > r->cfg.max_batch)
      return fail(PMDFC_ERR_ARG, "route_batches: a batch is empty-negative or past the router's max_batch");
  if (total >= kRouteNone) return fail(PMDFC_ERR_ARG, "route_batches: more than 2^32 - 2 ops");
  DevGuard g(c->device);
  hipStream_t S = (hipStream_t)stream, C = c->cs;
  // PMDFC_ROUTE_DIRECT=0: the pack / exchange / unpack path even on one rank
  // (its per-batch cost, measured where no peer exists; A/B and tests)
  static const bool direct_ok = [] {
    const char* e = getenv("PMDFC_ROUTE_DIRECT");
    return !(e && e[0] == '0');
  }();
  if (direct_ok && c->nranks == 1 && r->cfg.cap >= r->cfg.max_batch) {
    // One rank: every op's owner is this rank, its block never moves and
    // holds a whole batch (cap >= max_batch: no carry can form), so the
    // routed call IS the direct call in batch order -- the engine runs on
    // the caller's arrays with call-global outputs (no pack, no exchange, no
    // unpack; a Get-only batch needs no dedupe).  Inserts go through the
    // engine's partition pipeline as pmdfc_cceh_insert_batches.
    int e = PMDFC_OK;
    if (width == 2) {
      std::vector<uint64_t> rb(nb + 1);
      for (uint64_t i = 0; i <= nb; ++i) rb[i] = bounds[i] - bounds[0];
      e = pmdfc_cceh_insert_batches(t, keys + bounds[0], values + bounds[0], st, rb.data(), (uint32_t)nb, S);
    } else if (width == 3) {
      std::vector<uint64_t> rb(nb + 1);
      for (uint64_t i = 0; i <= nb; ++i) rb[i] = bounds[i] - bounds[0];
      e = pmdfc_cceh_mixed_batches(t, ops + bounds[0], keys + bounds[0], values + bounds[0], vout, st, rb.data(),
                                   (uint32_t)nb, S);
    } else {
      std::vector<uint64_t> rb(nb + 1);
      for (uint64_t i = 0; i <= nb; ++i) rb[i] = bounds[i] - bounds[0];
      e = pmdfc_cceh_get_batches(t, keys + bounds[0], vout, st, rb.data(), (uint32_t)nb, S);
    }
    return e;
  }
  const uint64_t rows = r->rows, cap = r->cfg.cap;
  const bool dd = dedupe && width == 1;
  const size_t req_b = rows * width * 8, resp_b = width == 2 ? rows : rows * 16;
  // call buffers (stream-ordered allocations, freed at the end)
  void* buf = nullptr;
  const size_t off_recv = 2 * req_b, off_rs = 4 * req_b, off_rb = off_rs + 3 * resp_b, off_pos = off_rb + 2 * resp_b;
  const size_t off_keep = off_pos + 3 * rows * 4, off_lead = off_keep + ((r->cfg.max_batch + 255) & ~255ull);
  const size_t off_car = off_lead + (dd ? ((total * 4 + 255) & ~255ull) : 0), off_mix = off_car + 256;
  // mixed: the engine's arrays for one batch of received rows (keys, values,
  // values out, statuses, ops)
  const size_t mix_b = width == 3 ? rows * 26 + 1024 : 0, all_b = off_mix + mix_b;
  HIPCHK(hipMallocAsync(&buf, all_b, S));
  uint8_t* B8 = static_cast<uint8_t*>(buf);
  uint64_t* send[2] = {(uint64_t*)B8, (uint64_t*)(B8 + req_b)};
  uint64_t* recv[2] = {(uint64_t*)(B8 + off_recv), (uint64_t*)(B8 + off_recv + req_b)};
  uint8_t* rsend[3] = {B8 + off_rs, B8 + off_rs + resp_b, B8 + off_rs + 2 * resp_b};  // (read by unpack i: i % 3)
  uint8_t* rback[2] = {B8 + off_rb, B8 + off_rb + resp_b};
  uint32_t* rowpos[3] = {(uint32_t*)(B8 + off_pos), (uint32_t*)(B8 + off_pos + rows * 4),
                         (uint32_t*)(B8 + off_pos + 2 * rows * 4)};
  uint8_t* keep = B8 + off_keep;
  uint32_t* lead = (uint32_t*)(B8 + off_lead);
  uint64_t* car = (uint64_t*)(B8 + off_car);
  uint64_t* mk = (uint64_t*)(B8 + off_mix);
  uint64_t* mv = mk + rows;
  uint64_t* mvo = mv + rows;
  uint8_t* mst = (uint8_t*)(mvo + rows);
  uint8_t* mop = mst + ((rows + 255) & ~255ull);
  hipEvent_t* evPack = c->ev;      // [2]
  hipEvent_t* evReq = c->ev + 2;   // [2]
  hipEvent_t* evRun = c->ev + 4;   // [2]
  hipEvent_t* evResp = c->ev + 6;  // [2]
  hipEvent_t evCar = c->ev[8], evCarDone = c->ev[9];
  hipEvent_t* evFin = c->ev + 10;  // [3]: unpack i done (pack i + 3 reuses its row positions)
  hipEvent_t evJoin = c->ev[13];
  (void)evPack;
  int rc = PMDFC_OK;
  // an all-to-all of equal blocks of `bytes` without the local block (it
  // never moves): grouped point-to-point sends and receives over RCCL
  auto exchange = [&](const void* sb, void* rb, uint64_t bytes) -> int {
    if (c->nranks == 1) return PMDFC_OK;
    if (c->xchg) {  // host-staged: the blocks through pinned host memory and the caller's transport
      const size_t tot = (size_t)c->nranks * bytes;
      if (tot > c->hcap) {
        if (c->hbuf) HIPCHK(hipHostFree(c->hbuf));
        c->hbuf = nullptr;
        HIPCHK(hipHostMalloc((void**)&c->hbuf, 2 * tot, hipHostMallocDefault));
        c->hcap = tot;
      }
      uint8_t* hs = c->hbuf;
      uint8_t* hr = c->hbuf + c->hcap;
      HIPCHK(hipMemcpyAsync(hs, sb, tot, hipMemcpyDeviceToHost, C));
      HIPCHK(hipStreamSynchronize(C));
      if (c->xchg(c->xctx, hs, hr, bytes) != 0) return fail(PMDFC_ERR_HIP, "route_batches: host exchange failed");
      for (int p = 0; p < c->nranks; ++p)  // (the local block never moves)
        if (p != c->rank)
          HIPCHK(hipMemcpyAsync(static_cast<uint8_t*>(rb) + (uint64_t)p * bytes, hr + (uint64_t)p * bytes, bytes,
                                hipMemcpyHostToDevice, C));
      HIPCHK(hipStreamSynchronize(C));  // (the staging is reused by the next exchange)
      return PMDFC_OK;
    }
    NCCLCHK(ncclGroupStart());
    for (int p = 0; p < c->nranks; ++p) {
      if (p == c->rank) continue;
      NCCLCHK(ncclSend(static_cast<const uint8_t*>(sb) + (uint64_t)p * bytes, bytes, ncclUint8, p, c->comm, C));
      NCCLCHK(ncclRecv(static_cast<uint8_t*>(rb) + (uint64_t)p * bytes, bytes, ncclUint8, p, c->comm, C));
    }
    NCCLCHK(ncclGroupEnd());
    return PMDFC_OK;
  };
  // the caller's stream holds the inputs' producers: the exchanges' stream
  // starts after them
  HIPCHK(hipEventRecord(evJoin, S));
  HIPCHK(hipStreamWaitEvent(C, evJoin, 0));
  auto pack = [&](uint64_t i) -> int {
    const uint64_t n = i < nb ? bounds[i + 1] - bounds[i] : 0;
    const uint64_t o = i < nb ? bounds[i] - bounds[0] : 0;
    const uint64_t* k = n ? keys + bounds[i] : nullptr;
    const uint64_t* v = n && width >= 2 ? values + bounds[i] : nullptr;
    const uint8_t* op = n && width == 3 ? ops + bounds[i] : nullptr;
    const uint8_t* kp = nullptr;
    if (i >= 3) HIPCHK(hipStreamWaitEvent(C, evFin[i % 3], 0));
    if (dd && n) {
      const int e = pmdfc_router_dedupe(r, k, nullptr, n, (uint32_t)o, keep, lead, C);
      if (e) return e;
      kp = keep;
    }
    // the local block goes straight into its receive slot; only peer blocks travel
    const int e = router_pack(r, k, v, op, kp, n, width, (uint32_t)o, send[i & 1], rowpos[i % 3],
                              width != 2 ? vout : nullptr, st, C, (uint32_t)c->rank,
                              recv[i & 1] + (uint64_t)c->rank * cap * width);
    if (e) return e;
    if ((rc = exchange(send[i & 1], recv[i & 1], cap * width * 8))) return rc;
    HIPCHK(hipEventRecord(evReq[i & 1], C));
    return PMDFC_OK;
  };
  // inserts at p1max go through the engine's pipeline (the partition of
  // batch i + 1 on the engine's partition stream, right after its rows
  // arrive, under batch i's bucket passes); a coarser table ramps batch by
  // batch first
  // (PMDFC_ROUTE_PIPE=1; measured slower on one rank: the partitions ran at
  // ~100 us beside the packs instead of ~40 us inline)
  static const bool pipe_inserts = [] {
    const char* e = getenv("PMDFC_ROUTE_PIPE");
    return e && atoi(e) != 0;
  }();
  uint32_t piped = 0;
  auto run = [&](uint64_t i) -> int {
    int e = PMDFC_OK;
    if (pipe_inserts && width == 2 && t->p1 >= t->p1max) {
      std::lock_guard<std::mutex> lk(t->mu);
      if (piped == 0) e = pipe_begin(t, S);
      // (the statuses buffer's last reader: the unpack of batch i - 3)
      if (!e)
        e = pipe_batch(t, recv[i & 1], recv[i & 1] + 1, 2, rsend[i % 3], rows, S, piped++, evReq[i & 1],
                       i >= 3 ? evFin[i % 3] : nullptr);
    } else {
      if (piped) {  // (cannot happen: a table never gets coarser)
        std::lock_guard<std::mutex> lk(t->mu);
        e = pipe_end(t, S);
        piped = 0;
      }
      HIPCHK(hipStreamWaitEvent(S, evReq[i & 1], 0));
      if (!e && width == 3) {
        launch_route_split(recv[i & 1], rows, 3, mk, mv, mop, S);
        e = pmdfc_cceh_mixed(t, mop, mk, mv, mvo, mst, rows, S);
        if (!e) launch_route_resp(mvo, mst, rows, rsend[i % 3], S);
        if (!e && hipGetLastError() != hipSuccess) e = fail(PMDFC_ERR_HIP, "route_batches: split / respond");
      } else if (!e) {
        e = width == 2 ? pmdfc_cceh_insert_records(t, recv[i & 1], rsend[i % 3], rows, S)
                       : pmdfc_cceh_get_records(t, recv[i & 1], (uint64_t*)rsend[i % 3], rows, S);
      }
    }
    if (e) return e;
    HIPCHK(hipEventRecord(evRun[i & 1], S));
    HIPCHK(hipStreamWaitEvent(C, evRun[i & 1], 0));
    if ((rc = exchange(rsend[i % 3], rback[i & 1], width == 2 ? cap : cap * 16))) return rc;
    HIPCHK(hipEventRecord(evResp[i & 1], C));
    return PMDFC_OK;
  };
  auto finish = [&](uint64_t i) -> int {
    HIPCHK(hipStreamWaitEvent(S, evResp[i & 1], 0));
    // (the local block's responses are read where the engine wrote them)
    launch_route_unpack(rback[i & 1], width == 2 ? 0u : 1u, rowpos[i % 3], rows, width != 2 ? vout : nullptr, st, S,
                        rsend[i % 3], (uint64_t)c->rank * cap, (uint64_t)(c->rank + 1) * cap);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(evFin[i % 3], S));
    return PMDFC_OK;
  };
  rc = pack(0);
  uint64_t i = 0, pend = 0;
  bool pending = false;
  while (rc == PMDFC_OK) {
    if (i + 1 < nb && (rc = pack(i + 1))) break;
    if ((rc = run(i))) break;
    if (pending && (rc = finish(pend))) break;
    pending = true;
    pend = i;
    if (++i < nb) continue;
    // drain: every rank exchanges until no rank carries ops (the counts come
    // from the last pack, on the exchanges' stream)
    if (hipEventRecord(evJoin, C) != hipSuccess || hipStreamWaitEvent(S, evJoin, 0) != hipSuccess) {
      rc = fail(PMDFC_ERR_HIP, "route_batches: join");
      break;
    }
    if ((rc = pmdfc_router_carried(r, car, S))) break;
    if (c->nranks > 1) {
      if (hipEventRecord(evCar, S) != hipSuccess || hipStreamWaitEvent(C, evCar, 0) != hipSuccess) {
        rc = fail(PMDFC_ERR_HIP, "route_batches: carried event");
        break;
      }
      if (c->amax) {  // host-staged transport
        uint64_t hv = 0;
        if (hipMemcpyAsync(&hv, car, 8, hipMemcpyDeviceToHost, C) != hipSuccess || hipStreamSynchronize(C) != hipSuccess ||
            c->amax(c->xctx, &hv) != 0 || hipMemcpyAsync(car, &hv, 8, hipMemcpyHostToDevice, C) != hipSuccess ||
            hipStreamSynchronize(C) != hipSuccess) {
          rc = fail(PMDFC_ERR_HIP, "route_batches: host all-reduce failed");
          break;
        }
      } else {
        const ncclResult_t nr = ncclAllReduce(car, car, 1, ncclUint64, ncclMax, c->comm, C);
        if (nr != ncclSuccess) {
          rc = nccl_fail("ncclAllReduce", nr);
          break;
        }
      }
      if (hipEventRecord(evCarDone, C) != hipSuccess || hipStreamWaitEvent(S, evCarDone, 0) != hipSuccess) {
        rc = fail(PMDFC_ERR_HIP, "route_batches: carried event");
        break;
      }
    }
    uint64_t h = 0;
    if (hipMemcpyAsync(&h, car, 8, hipMemcpyDeviceToHost, S) != hipSuccess || hipStreamSynchronize(S) != hipSuccess) {
      rc = fail(PMDFC_ERR_HIP, "route_batches: carried count");
      break;
    }
    if (h == 0) break;
    rc = pack(i);  // a drain exchange (no new ops)
  }
  if (rc == PMDFC_OK && pending) rc = finish(pend);
  if (rc == PMDFC_OK && piped) {
    std::lock_guard<std::mutex> lk(t->mu);
    rc = pipe_end(t, S);
  }
  if (rc == PMDFC_OK && (hipEventRecord(evJoin, C) != hipSuccess || hipStreamWaitEvent(S, evJoin, 0) != hipSuccess))
    rc = fail(PMDFC_ERR_HIP, "route_batches: join");
  if (rc == PMDFC_OK) rc = pmdfc_router_end_call(r);
  if (rc == PMDFC_OK && dd) rc = pmdfc_router_fill(lead, total, vout, st, c->device, S);
  if (rc != PMDFC_OK) {
    const std::string err = g_err;  // (the reset below must not hide the first error)
    (void)hipStreamSynchronize(C);
    (void)pmdfc_router_reset(r, S);
    (void)hipFreeAsync(buf, S);
    g_err = err;
    return rc;
  }
  HIPCHK(hipFreeAsync(buf, S));
  return PMDFC_OK;
}
