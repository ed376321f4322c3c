// bucket.hip -- the batched Insert / mixed path.
//
// A batch runs as a fixed launch sequence on the caller's stream, no host
// round trip:
//
// 1. k_part: partition of the batch's pending ops into 2^(p1 - sbb) partition
//    buckets by the top local hash bits.  Each 8192-op tile counts its ops per
//    bucket with LDS atomics and reserves one contiguous run per non-empty
//    bucket in its XCD's sub-region (blockIdx & 7) of that bucket's record
//    region (one global atomic per (tile, bucket), all of a thread's issued
//    back to back); a run that does not fit spills into a shared overflow
//    area, tagged with its bucket.  Records (SoA): {key, value}, rop = op
//    index | sub-bucket << 22 | Get << 31; order inside a bucket is not batch
//    order (the passes sort by op index).
// 2. the first apply pass, ONE WAVE PER DIRECTORY BUCKET: k_apply_fast (the
//    lean insert-only pass: parallel claims, fast_claim) or bucket_body's
//    general pass.  A directory bucket owns its sub-directory (cceh_device.h
//    "Bucketed directory") and every segment in it, so the wave applies its
//    ops with no one to coordinate with (CCEH splits are segment-local,
//    CCEH_hybrid.cpp:171-297): each insert takes the first free slot of its
//    32-slot window in batch order (CCEH_hybrid.cpp:143-168); a segment whose
//    window is full requests a split and parks the rest of its ops; the
//    bucket reserves its child ids and grown sub-directory with sharded
//    atomics (request_splits).
// 3. k_split: one wave per requested split (cluster replay below), global ids
//    from the shard offsets.
// 4. k_apply_parked: the requesting buckets commit their splits (directory
//    stride update, sub-directory growth, CCEH_hybrid.cpp:208-286) and apply
//    their parked ops.
// 5. k_bucket, the final pass: whatever is still parked, oversized buckets
//    (records walked tile by tile in batch order), rounds with inline splits
//    until nothing is pending (depth is capped at 30, so it terminates).
// Small batches skip the pipeline: k_mixed_tiny (<= 64 ops), k_mixed_small
// (<= 256) and k_part + k_medium (<= 8192) run the final pass's ordered runs
// directly.
#include <algorithm>
#include <cstdlib>
#include <cstddef>

#include "cceh_device.h"
#include "cceh_kernels.h"

namespace pmdfc {

constexpr int kPartThreads = 1024;
constexpr int kPartPer = (int)kPartTile / kPartThreads;  // ops per thread

constexpr int kCW = (int)kChunkWave;  // ops per wave chunk (LDS, register sort)
constexpr int kPer = kCW / 64;        // chunk slots per lane
constexpr int kBmLanes = 30;          // lanes with an LDS occupancy bitmap at a time (LDS: 4 waves/SIMD)
constexpr int kRoundGuard = 64;

constexpr uint32_t kGetBit = 0x80000000u;
constexpr uint32_t kOpMask = (1u << 22) - 1;

// k_bucket sort key: [segment:25 @39][op index:22 @17][chunk slot:9 @8][home line:8 @0].
// Ordering is (segment, batch index); the home line rides along so the
// per-run loop needs neither the key nor a hash.
__device__ __forceinline__ uint64_t sk_make(uint32_t seg, uint32_t op, uint32_t i, uint32_t home) {
  return ((uint64_t)seg << 39) | ((uint64_t)op << 17) | ((uint64_t)i << 8) | home;
}
__device__ __forceinline__ uint32_t sk_seg(uint64_t k) { return (uint32_t)(k >> 39); }
__device__ __forceinline__ uint32_t sk_op(uint64_t k) { return (uint32_t)(k >> 17) & kOpMask; }
__device__ __forceinline__ uint32_t sk_item(uint64_t k) { return (uint32_t)(k >> 8) & 511u; }
__device__ __forceinline__ uint32_t sk_home(uint64_t k) { return (uint32_t)k & 0xFFu; }

// --------------------------------------------------------------- partition

struct PartArgs {
  const uint64_t* keys;
  const uint64_t* vin;
  const uint8_t* ops;   // null: insert-only batch (k_part resolves statuses itself)
  uint8_t* st;
  uint64_t n;
  uint32_t kvs;         // u64 words from one op's key (value) to the next: 1, or 2 for {key, value} records
  uint32_t sbits, shard, p1, sbb;  // p1: partition bucket bits; sbb: sub-bucket bits
  uint32_t cap;         // record slots per bucket region
  uint32_t capx;        // ... per sub-region (cap / kPartSubs)
  uint64_t ovf_base;    // first overflow record slot
  ulonglong2* rkv;      // records: {key, value}
  uint32_t* rop;        // records: op index | sub-bucket << 22 | Get << 31
  uint16_t* robk;       // bucket of each overflow record
  uint32_t* cursor;     // this batch's cursors, [sub-region][bucket] (zero on entry)
  uint32_t* ovf;        // this batch's overflow cursor (zero on entry)
  uint32_t* povf;       // [tile][bucket] overflow slot of a run that does not fit its sub-region
  uint64_t* stamps;     // debug: 8 wall-clock stamps per block, or null
  uint32_t init;        // medium batch: statuses set here (PartLaunch::init)
  uint64_t* vout;
  uint32_t* touched;
  uint32_t delay;       // measurement knob (PMDFC_PART_DELAY_US): each block spins this many 100-MHz ticks at its end
  // general mixed batches: the joining Gets' resolution (PartLaunch)
  const uint64_t* iset;
  uint64_t imask;
  const uint32_t* icnt;
  const uint32_t* ipos;
  uint8_t* early;
  uint32_t* elink;
  DevCtl* ctl;
  uint32_t tag;
};

// A joining Get of a mixed batch (kStJoin, cceh_kernels.hip k_mixed_get),
// once k_mixed_join put the batch's inserts of its key into the set (count,
// first position): no insert -- its probe result stands (vout, early 1 for a
// hit); a miss whose key the batch inserts once -- a miss before that insert,
// linked to it after; else pending, for the ordered passes.  The set probe
// loads each slot's key, count and first position together (one round trip:
// the first slot almost always holds the key or is empty).  Returns the Get's
// new status.
__device__ __forceinline__ uint8_t join_resolve(const PartArgs& a, uint64_t p, uint64_t key, uint64_t h) {
  uint64_t sl = iset_slot(h, a.imask);
  const uint8_t c = a.early[p];
  uint32_t ic = 0, ps = 0;
  for (;; sl = (sl + 1) & a.imask) {
    const uint64_t v = a.iset[sl];
    const uint32_t ic1 = a.icnt[sl], ps1 = a.ipos[sl];
    if (v == kInvalid) break;  // no insert of the key
    if (v == key) {
      ic = ic1;
      ps = ps1;
      break;
    }
  }
  uint8_t s;
  if (ic == 0) {
    s = c ? 1 : 0;  // PMDFC_ST_HIT / PMDFC_ST_NOT_FOUND
  } else if (c == 0 && ic == 1) {
    if ((uint64_t)ps > p) {
      s = 0;
    } else {
      s = kStLinked;  // the insert's outcome after the batch (k_mixed_verify)
      a.early[p] = 2;
      a.elink[p] = ps;
    }
  } else {
    s = kStPending;
    a.early[p] = 0;
    a.vout[p] = 0;
    a.ctl->pget = a.tag;  // every writer stores the same word
  }
  a.st[p] = s;
  return s;
}

#define PART_STAMP(ph) \
  if (a.stamps && threadIdx.x == 0) a.stamps[(size_t)blockIdx.x * 8 + (ph)] = wall_clock64()

__global__ __launch_bounds__(kPartThreads) void k_part(PartArgs a) {
  // 64 KB of LDS: a block fits beside a CU's share of the apply pass, which
  // it overlaps in pipelined insert batches (the overflow slot of a run that
  // does not fit its sub-region, rare, goes through global memory: a.povf)
  __shared__ uint32_t s_cnt[1u << kMaxPartBits];  // ops of the tile per bucket
  __shared__ uint32_t s_reg[1u << kMaxPartBits];  // region slot of the bucket's run
  PART_STAMP(0);
  const uint32_t nb = 1u << a.p1;
  for (uint32_t i = threadIdx.x; i < nb; i += kPartThreads) s_cnt[i] = 0;
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x * kPartTile;
  uint64_t kk[kPartPer], vv[kPartPer];
  uint32_t bk[kPartPer], rk[kPartPer], ro[kPartPer];
#pragma unroll
  for (int k = 0; k < kPartPer; ++k) {
    const uint64_t p = base + (uint64_t)k * kPartThreads + threadIdx.x;
    kk[k] = p < a.n ? a.keys[p * a.kvs] : kInvalid;
  }
#pragma unroll
  for (int k = 0; k < kPartPer; ++k) {
    const uint64_t p = base + (uint64_t)k * kPartThreads + threadIdx.x;
    bool part = false;
    bk[k] = 0xFFFFFFFFu;
    vv[k] = 0;
    ro[k] = (uint32_t)p;
    if (p < a.n) {
      const uint64_t key = kk[k];
      const uint64_t h = hash64(key);
      if (!a.ops) {
        uint8_t code = 2;  // PMDFC_ST_INSERTED (k_bucket rewrites the rare failures)
        if (reserved_key(key)) code = 3;
        else if (wrong_shard(h, a.sbits, a.shard)) code = 8;
        a.st[p] = code;
        part = code == 2;
      } else {
        if (a.init) {  // (k_mixed_prep's rule)
          const uint8_t code = reserved_key(key) ? 3 : wrong_shard(h, a.sbits, a.shard) ? 8 : kStPending;
          a.st[p] = code;
          a.vout[p] = 0;
          part = code == kStPending;
        } else {
          uint8_t s0 = a.st[p];
          if (s0 == kStJoin) s0 = join_resolve(a, p, key, h);
          part = s0 == kStPending;
        }
        if (part && a.ops[p] != 1) ro[k] |= kGetBit;  // anything but PMDFC_OP_INSERT is a Get
        // inserts: PMDFC_ST_INSERTED unless a pass rewrites it (the
        // insert-only apply passes, which a gated mixed batch may take,
        // never write it)
        else if (part) a.st[p] = 2;
      }
      if (part) {
        const uint32_t b2 = bucket_of(h, a.sbits, a.p1 + a.sbb);  // directory bucket
        bk[k] = b2 >> a.sbb;
        ro[k] |= (b2 & ((1u << a.sbb) - 1)) << 22;
        if (!(ro[k] & kGetBit)) vv[k] = a.vin[p * a.kvs];
        rk[k] = atomicAdd(&s_cnt[bk[k]], 1u);
      }
    }
  }
  __syncthreads();
  PART_STAMP(1);
  if (a.touched) {  // one block (medium batch): the partition buckets that received ops
    __shared__ uint32_t s_nt;
    if (threadIdx.x == 0) s_nt = 0;
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < nb; b += kPartThreads)
      if (s_cnt[b]) a.touched[1 + atomicAdd(&s_nt, 1u)] = b;
    __syncthreads();
    if (threadIdx.x == 0) a.touched[0] = s_nt;
  }
  // one run per non-empty bucket: reserve it in this block's sub-region; the
  // part past the sub-region's capacity goes to the overflow area.  A
  // thread's cursor atomics are issued together (one round trip, not one per
  // bucket)
  {
    constexpr int kRes = (1 << kMaxPartBits) / kPartThreads;
    const uint32_t xs = blockIdx.x & (kPartSubs - 1);
    uint32_t cb[kRes], pos[kRes];
#pragma unroll
    for (int r = 0; r < kRes; ++r) {
      const uint32_t b = threadIdx.x + (uint32_t)r * kPartThreads;
      cb[r] = b < nb ? s_cnt[b] : 0u;
    }
#pragma unroll
    for (int r = 0; r < kRes; ++r) {
      const uint32_t b = threadIdx.x + (uint32_t)r * kPartThreads;
      pos[r] = cb[r] ? atomicAdd(&a.cursor[xs * nb + b], cb[r]) : 0u;  // XCD-private cursor lines
    }
#pragma unroll
    for (int r = 0; r < kRes; ++r) {
      const uint32_t b = threadIdx.x + (uint32_t)r * kPartThreads;
      const uint32_t c = cb[r];
      if (!c) continue;
      const uint32_t fit = pos[r] < a.capx ? min(c, a.capx - pos[r]) : 0u;
      s_reg[b] = b * a.cap + xs * a.capx + pos[r];
      s_cnt[b] = fit;
      if (fit < c) a.povf[(size_t)blockIdx.x * nb + b] = atomicAdd(a.ovf, c - fit);
    }
  }
  __syncthreads();
  PART_STAMP(2);
#pragma unroll
  for (int k = 0; k < kPartPer; ++k) {
    const uint32_t b = bk[k];
    if (b == 0xFFFFFFFFu) continue;
    uint64_t dst;
    const uint32_t fit = s_cnt[b];
    if (rk[k] < fit) {
      dst = (uint64_t)s_reg[b] + rk[k];
    } else {
      const uint32_t o = a.povf[(size_t)blockIdx.x * nb + b] + (rk[k] - fit);
      a.robk[o] = (uint16_t)b;
      dst = a.ovf_base + o;
    }
    a.rkv[dst] = make_ulonglong2(kk[k], vv[k]);
    a.rop[dst] = ro[k];
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  PART_STAMP(3);
  if (a.delay && threadIdx.x == 0) {
    const uint64_t t0 = wall_clock64();
    while (wall_clock64() - t0 < a.delay) __builtin_amdgcn_s_sleep(2);
  }
}

// ------------------------------------------------------------------ helpers

// s_waitcnt vmcnt(N) with the other counters left alone (gfx9 encoding)
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

__device__ __forceinline__ uint64_t umin64(uint64_t x, uint64_t y) { return x < y ? x : y; }
__device__ __forceinline__ uint64_t umax64(uint64_t x, uint64_t y) { return x < y ? y : x; }

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m) {
  const int lo = __shfl_xor((int)(uint32_t)v, m);
  const int hi = __shfl_xor((int)(uint32_t)(v >> 32), m);
  return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}

__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, uint32_t* total) {
  const uint32_t lane = __lane_id() & 63u;
  uint32_t incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = (uint32_t)__shfl_up((int)incl, o);
    if (lane >= (uint32_t)o) incl += t;
  }
  *total = (uint32_t)__shfl((int)incl, 63);
  return incl - v;
}

// Ascending bitonic sort, by one wave, of s[0..nvalid) padded with ~0 to n
// (a power of two <= kCW); s[0..n) holds the result.  Element e lives in
// lane e/8, register e%8: partner distances j < 8 stay in the lane, larger
// ones are cross-lane shuffles (j/8 <= 32).  Elements >= n only meet each
// other, so every lane runs the same network.
__device__ __forceinline__ void wave_sort8(uint64_t* s, uint32_t n, uint32_t nvalid) {
  const uint32_t lane = __lane_id() & 63u;
  uint64_t v[kPer];
#pragma unroll
  for (int q = 0; q < kPer; ++q) v[q] = (kPer * lane + q < nvalid) ? s[kPer * lane + q] : ~0ULL;
  for (uint32_t k = 2; k <= n; k <<= 1) {
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      if (j >= (uint32_t)kPer) {
        const int m = (int)(j / kPer);
#pragma unroll
        for (int q = 0; q < kPer; ++q) {
          const uint32_t e = kPer * lane + q;
          const uint64_t pv = shfl_xor64(v[q], m);
          const bool up = (e & k) == 0, lower = (e & j) == 0;
          v[q] = (lower == up) ? umin64(v[q], pv) : umax64(v[q], pv);
        }
      } else {
        // in-lane partners: dispatch on j so every register index is static
        // (a runtime v[q + j] would put v[] in scratch memory)
#pragma unroll
        for (int jj = kPer / 2; jj >= 1; jj >>= 1) {
          if ((int)j != jj) continue;
#pragma unroll
          for (int q = 0; q < kPer; ++q) {
            if (q & jj) continue;
            const uint32_t e = kPer * lane + q;
            const bool up = (e & k) == 0;
            const uint64_t x = v[q], y = v[q + jj];
            v[q] = up ? umin64(x, y) : umax64(x, y);
            v[q + jj] = up ? umax64(x, y) : umin64(x, y);
          }
        }
      }
    }
  }
#pragma unroll
  for (int q = 0; q < kPer; ++q)
    if (kPer * lane + q < n) s[kPer * lane + q] = v[q];
  __builtin_amdgcn_wave_barrier();
}

// Ascending bitonic sort of 32-bit keys held in registers: position
// KP*lane + q in v[q], n a power of two <= 64*KP, positions >= n hold ~0.
template <int KP>
__device__ __forceinline__ void wave_sort32(uint32_t (&v)[KP], uint32_t n) {
  const uint32_t lane = __lane_id() & 63u;
  for (uint32_t k = 2; k <= n; k <<= 1) {
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      if (j >= (uint32_t)KP) {
        const int m = (int)(j / KP);
#pragma unroll
        for (int q = 0; q < KP; ++q) {
          const uint32_t e = KP * lane + q;
          const uint32_t pv = (uint32_t)__shfl_xor((int)v[q], m);
          const bool up = (e & k) == 0, lower = (e & j) == 0;
          v[q] = (lower == up) ? min(v[q], pv) : max(v[q], pv);
        }
      } else {
#pragma unroll
        for (int jj = KP / 2; jj >= 1; jj >>= 1) {
          if ((int)j != jj) continue;
#pragma unroll
          for (int q = 0; q < KP; ++q) {
            if (q & jj) continue;
            const uint32_t e = KP * lane + q;
            const bool up = (e & k) == 0;
            const uint32_t x = v[q], y = v[q + jj];
            v[q] = up ? min(x, y) : max(x, y);
            v[q + jj] = up ? max(x, y) : min(x, y);
          }
        }
      }
    }
  }
}

// Positions < n of a 32-bit key array in LDS, sorted in place by one wave
// (KP keys per lane; p2 = n rounded up to a power of two, <= 64 * KP).
template <int KP>
__device__ __forceinline__ void wave_sort32_lds(uint32_t* buf, uint32_t n, uint32_t p2) {
  const uint32_t lane = __lane_id() & 63u;
  uint32_t v[KP];
#pragma unroll
  for (int q = 0; q < KP; ++q) v[q] = KP * lane + q < n ? buf[KP * lane + q] : ~0u;
  __builtin_amdgcn_wave_barrier();
  wave_sort32<KP>(v, p2);
#pragma unroll
  for (int q = 0; q < KP; ++q)
    if (KP * lane + q < n) buf[KP * lane + q] = v[q];
  __builtin_amdgcn_wave_barrier();
}

// ---------------------------------------------------------------- splitting
//
// Segment::Split (non-INPLACE, CCEH_hybrid.cpp:47-66): walk the parent in slot
// order 0..1023; each entry goes to child (hash bit 63-L) at the first free
// slot of its own 32-slot window, or is dropped if that window is full.
//
// Cluster decomposition (exact).  Nothing is ever deleted, so an
// entry at parent slot s with window start w has every slot of [w, s]
// occupied: it lies in one CLUSTER (maximal run of occupied
// parent slots).  Replaying in slot order, every entry lands in [w, s]: all
// entries before it landed at or before their own slots.  So clusters replay
// independently, each by one lane with its two child bitmaps in registers.
// The one exception is the cluster that wraps past slot 1023: the reference
// walks its head [0, b] first, so its tail entries can be pushed past 1023
// into wrapped slots <= 30 (or dropped); that cluster, plus every cluster
// starting at <= 30, is one unit replayed by one lane in slot order.  A fully
// occupied parent or a wrap unit wider than 128 slots takes the slower
// generic replay (wave_replay).  The other clusters are replayed as a sweep
// over positions (no drops are possible outside the wrap unit; see the
// comment at the sweep).
constexpr uint32_t kSplitScratch = 2080;  // u32 words per splitting wave

__device__ __forceinline__ uint32_t occ_end(const uint32_t* s_occ, uint32_t a) {
  uint32_t w = a >> 5;
  uint32_t bits = ~s_occ[w] & (~0u << (a & 31u));
  while (bits == 0) {
    if (++w == 32) return kSlots;
    bits = ~s_occ[w];
  }
  return w * 32u + (uint32_t)__builtin_ctz(bits);
}

__device__ __forceinline__ uint32_t ext32(uint64_t lo, uint64_t hi, uint32_t r) {
  if (r >= 128) return 0;
  if (r >= 64) return (uint32_t)(hi >> (r - 64));
  return (uint32_t)((lo >> r) | (r ? (hi << (64 - r)) : 0ULL));
}

// Replay parent slots [x, y) for ONE child c into a 128-bit map relative to
// origin o (the unit's first slot): only the child's entries are visited
// (a bit walk over the occupancy / child-1 words), in slot order.
__device__ __forceinline__ void unit_range(const uint16_t* s_inf, const uint32_t* s_occ, const uint32_t* s_ch1,
                                           uint16_t* s_dst, uint64_t& lo, uint64_t& hi, uint32_t c, uint32_t o,
                                           uint32_t x, uint32_t y, uint32_t* loss, bool* bad) {
  for (uint32_t wd = x >> 5; wd * 32u < y; ++wd) {
    const uint32_t ch = s_ch1[wd];
    uint32_t b = c ? ch : (s_occ[wd] & ~ch);
    if (wd == (x >> 5)) b &= ~0u << (x & 31u);
    if (y - wd * 32u < 32u) b &= (1u << (y - wd * 32u)) - 1u;
    while (b) {
      const uint32_t s = wd * 32u + (uint32_t)__builtin_ctz(b);
      b &= b - 1u;
      const uint32_t e = s_inf[s];
      const uint32_t rw = ((e & 0xFFu) * 4u - o) & (kSlots - 1);
      const uint32_t fr = ~ext32(lo, hi, rw);
      if (fr == 0) {
        ++*loss;  // window full: Insert4split drops the entry (CCEH_hybrid.cpp:24-27)
        continue;
      }
      const uint32_t q = rw + (uint32_t)__builtin_ctz(fr);
      if (q >= 128) {
        *bad = true;
        continue;
      }
      if (q < 64) lo |= 1ULL << q;
      else hi |= 1ULL << (q - 64);
      s_dst[s] = (uint16_t)((c << 10) | ((o + q) & (kSlots - 1)));
    }
  }
}

__device__ __forceinline__ void unit_flush(uint32_t* s_cb, uint64_t lo, uint64_t hi, uint32_t c,
                                           uint32_t o) {
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const uint64_t src = m < 2 ? lo : hi;
    const uint32_t chunk = (uint32_t)(src >> (32 * (m & 1)));
    if (!chunk) continue;
    const uint32_t slot = (o + 32u * m) & (kSlots - 1);
    const uint32_t wi = slot >> 5, sh = slot & 31u;
    atomicOr(&s_cb[c * 32u + wi], chunk << sh);
    if (sh) atomicOr(&s_cb[c * 32u + ((wi + 1u) & 31u)], chunk >> (32u - sh));
  }
}

// Generic replay (wave_replay) for the rare parents the cluster path does not
// take; reads the slot descriptors from s_inf, leaves the placements in s_dst
// and the child bitmaps in s_cb.  Returns this lane's dropped entries.
__device__ __noinline__ uint32_t split_slow(const uint16_t* s_inf, uint16_t* s_dst, uint32_t* s_cb,
                                            uint32_t* s_rep) {
  const uint32_t lane = __lane_id() & 63u;
  uint32_t inf[16], dest[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const uint32_t e = s_inf[j * 64 + lane];
    inf[j] = ((e & 0x8000u) ? 0x80000000u : 0u) | (e & 0x1FFu);
  }
  s_rep[lane] = 0;
  __builtin_amdgcn_wave_barrier();
  const uint32_t loss = wave_replay(inf, dest, s_rep, s_rep + 64, s_rep + 128);
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int j = 0; j < 16; ++j) s_dst[j * 64 + lane] = dest[j] == 0xFFFFFFFFu ? 0xFFFF : (uint16_t)dest[j];
  s_cb[lane] = s_rep[lane];
  __builtin_amdgcn_wave_barrier();
  return loss;
}

// Split `seg` (local depth L) into seg (child 0, the parent's storage) and c1
// with a team of NW waves (1, or 4 of one workgroup: k_split when the split
// list is short -- a split is then a chain of dependent phases, and four waves
// quarter its loads and stores).  Wave v of the team loads, hashes and later
// stores the slot groups [v * 16 / NW, (v + 1) * 16 / NW) (group g = slots
// 64g..64g+63); the replay in between (cluster sweep / wave_replay) is wave
// 0's.  Returns dropped entries (the team's total, on every wave); *bad_out
// is set if an internal assumption failed (reported as a sticky device
// error).  NW = 4 needs every wave of the workgroup (barriers).
#define SP_STAMP(k) \
  if (stamp && lane == 0 && v == 0) stamp[k] = wall_clock64()
// drops != null (mixed batches): each dropped entry is logged as {key, trig},
// trig = the batch position of the insert whose full window split `seg`.
template <int NW>
__device__ __forceinline__ uint32_t split_team(ulonglong2* __restrict__ pairs, uint32_t* __restrict__ occ,
                                               uint8_t* __restrict__ ldep, uint32_t seg, uint32_t c1, uint32_t L,
                                               uint32_t* scr, bool* bad_out, uint64_t* stamp, ulonglong2* drops,
                                               uint32_t* drop_n, uint32_t trig, uint32_t v) {
  static_assert(NW == 1 || NW == 4, "team of 1 or 4 waves");
  constexpr int G = 16 / NW;  // slot groups per wave
  const auto team_barrier = [] {
    if constexpr (NW == 1) __builtin_amdgcn_wave_barrier();
    else __syncthreads();
  };
  const uint32_t lane = __lane_id() & 63u;
  uint16_t* s_inf = reinterpret_cast<uint16_t*>(scr);          // 1024 x u16
  uint16_t* s_dst = reinterpret_cast<uint16_t*>(scr + 512);    // 1024 x u16
  uint32_t* s_occ = scr + 1024;                                // 32 words
  uint32_t* s_cb = scr + 1056;                                 // 64 words: child bitmaps
  uint32_t* s_ch1 = scr + 1120;                                // 32 words: parent slots of child 1
  uint32_t* s_tm = scr + 1152;                                 // team words: [0] far | bad, [1] loss
  uint32_t* s_rep = scr + 1376;                                // 3 x 64 words (fallback)
  uint32_t* s_E = scr + 1568;                                  // 2 x 256 words: per child and home line,
                                                               // the entries' slots relative to 4 * line
  ulonglong2* sp = pairs + (size_t)seg * kSlots;
  ulonglong2* s1 = pairs + (size_t)c1 * kSlots;
  const int g0 = (int)v * G;
  // keys only: the pairs are re-read (L2-hot) after placement, before the
  // first store, so nothing is live across the replay
  uint64_t pk[G];
#ifndef PMDFC_SPLIT_NT
#define PMDFC_SPLIT_NT 0  // (A/B builds) 1: the first read of the parent with non-temporal loads
#endif
#pragma unroll
  for (int j = 0; j < G; ++j) {
    // a plain load: the parent's lines stay in L2 for the reload below (a
    // non-temporal first read let them go: the reload then came from HBM,
    // ~14 us of a ~35 us split in the heaviest batches)
    if constexpr (PMDFC_SPLIT_NT)
      pk[j] = __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(sp + (g0 + j) * 64 + lane));
    else
      pk[j] = reinterpret_cast<const uint64_t*>(sp + (g0 + j) * 64 + lane)[0];
  }
  for (uint32_t t = v * 64u + lane; t < 512u; t += 64u * NW) s_E[t] = 0;
  if (v == 0) {
    s_cb[lane] = 0;
    if (lane < 2) s_tm[lane] = 0;
  }
  team_barrier();
  bool far = false;  // an entry more than 31 slots past its window start (cannot happen)
#pragma unroll
  for (int j = 0; j < G; ++j) {
    const int g = g0 + j;
    const bool valid = pk[j] != kInvalid;
    const uint64_t kh = hash64(pk[j]);
    if (valid) {
      const uint32_t sl = (uint32_t)g * 64u + lane, hl = (uint32_t)(kh & 0xFF);
      const uint32_t rel = (sl - 4u * hl) & (kSlots - 1);
      far |= rel > 31u;
      atomicOr(&s_E[((uint32_t)((kh >> (63 - L)) & 1u) << 8) | hl], 1u << (rel & 31u));
    }
    // bit 15 valid, bit 8 child (hash bit 63-L, CCEH_hybrid.cpp:52-55), bits 0-7 home line
    s_inf[g * 64 + lane] = (uint16_t)((valid ? 0x8000u : 0u) | ((uint32_t)((kh >> (63 - L)) & 1u) << 8) |
                                      (uint32_t)(kh & 0xFF));
    s_dst[g * 64 + lane] = 0xFFFF;
    const uint64_t m = __ballot(valid);
    const uint64_t m1 = __ballot(valid && ((kh >> (63 - L)) & 1u));
    if (lane == 0) {
      s_occ[2 * g] = (uint32_t)m;
      s_ch1[2 * g] = (uint32_t)m1;
    }
    if (lane == 1) {
      s_occ[2 * g + 1] = (uint32_t)(m >> 32);
      s_ch1[2 * g + 1] = (uint32_t)(m1 >> 32);
    }
  }
  if (NW > 1 && __ballot(far) && lane == 0) atomicOr(&s_tm[0], 1u);
  team_barrier();
  SP_STAMP(0);
  uint32_t loss = 0;
  if (v == 0) {
    bool bad = far || (NW > 1 && (s_tm[0] & 1u));
    // ---- clusters.  Lane l replays child c = l >> 5 for the clusters that
    // START in slots [32w, 32w + 32), w = l & 31 (so a long cluster costs one
    // lane per child, and both children run in parallel).
    const uint32_t c = lane >> 5, wl = lane & 31u;
    const uint32_t ow = s_occ[wl];
    const uint32_t pw = wl ? s_occ[wl - 1] : 0u;
    const uint32_t stw = ow & ~((ow << 1) | (pw >> 31));  // cluster starts in my word
    const bool all_full = __ballot(ow != ~0u) == 0;
    const bool cyclic = !all_full && (s_occ[0] & 1u) && (s_occ[31] >> 31);
    // the cluster holding slot 1023 starts at the last start overall
    const uint64_t nzw = __ballot(lane < 32 && stw != 0);
    const int tl = nzw ? 63 - __builtin_clzll(nzw) : 0;
    const uint32_t tail = (uint32_t)__shfl((int)(tl * 32 + (stw ? 31 - __builtin_clz(stw) : 0)), tl);
    const uint32_t head_end = cyclic ? occ_end(s_occ, 0) : 0u;
    SP_STAMP(1);
    bool wide = false;  // a unit outgrew the 128-bit window
    if (!all_full) {
      if (cyclic && wl == 0) {
        // the wrap unit in the reference's slot order: head, clusters starting
        // at <= 30, then the tail (which may push entries into wrapped slots)
        uint64_t lo = 0, hi = 0;
        unit_range(s_inf, s_occ, s_ch1, s_dst, lo, hi, c, tail, 0, head_end, &loss, &wide);
        uint32_t mb = stw & ~1u;
        while (mb) {
          const uint32_t a0 = (uint32_t)__builtin_ctz(mb);
          mb &= mb - 1;
          if (a0 <= 30u) unit_range(s_inf, s_occ, s_ch1, s_dst, lo, hi, c, tail, a0, occ_end(s_occ, a0), &loss, &wide);
        }
        unit_range(s_inf, s_occ, s_ch1, s_dst, lo, hi, c, tail, tail, kSlots, &loss, &wide);
        unit_flush(s_cb, lo, hi, c, tail);
      }
      if (stamp && lane == 0) stamp[7] = wall_clock64();
      // The other clusters: a sweep over positions, each 32-slot word by its
      // own lane.  Outside the wrap unit an entry at parent slot s with window
      // start w lands at some x in [w, s] of its child (the slots [w, s) hold at
      // most s - w earlier entries of it), so nothing is dropped, and replayed
      // in slot order the child's position x goes to the waiting entry with the
      // smallest s among those with w <= x (an earlier entry that could take x
      // would have, when x was still free).  So: M's bit k = the entry at slot
      // x + k is waiting; at x = 4h the entries of home line h join (s_E, bits
      // relative to 4h, all within 32); x takes M's lowest bit.
      // Words in parallel: the number waiting, P, follows P -> max(P + A - 4, 0)
      // over a home line with A arrivals, and these maps compose as
      // P -> max(P + alpha, beta), so a 32-lane scan gives P at every word
      // start.  P = 0 means nothing waits (M = 0): a lane replays from the last
      // word start at or before its own where P = 0 (usually its own or the
      // one before), recording only its own word's placements.
      {
        const uint32_t* Ec = s_E + c * 256u;
        uint32_t U = 0, T = kSlots;  // [U, T): the positions outside the wrap unit
        if (cyclic) {
          const uint32_t o0 = s_occ[0];
          const uint32_t st0 = o0 & ~(o0 << 1) & 0x7FFFFFFEu;  // cluster starts 1..30
          U = max(head_end, st0 ? occ_end(s_occ, 31u - (uint32_t)__builtin_clz(st0)) : 0u);
          T = tail;
        }
        const uint4* E4 = reinterpret_cast<const uint4*>(Ec);
        const auto line8 = [&](uint32_t vv, uint32_t (&e)[8]) {  // the 8 home lines of word vv
          const uint4 p = E4[2u * vv], q = E4[2u * vv + 1u];
          e[0] = p.x, e[1] = p.y, e[2] = p.z, e[3] = p.w, e[4] = q.x, e[5] = q.y, e[6] = q.z, e[7] = q.w;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const uint32_t x = vv * 32u + 4u * (uint32_t)j;
            if (x < U || x >= T) e[j] = 0u;  // the wrap unit's (replayed above)
          }
        };
        uint32_t e8[8];
        line8(wl, e8);
        int sa = 0, sb = 0;  // my word's map
        uint32_t anyw = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int a1 = __builtin_popcount(e8[j]) - 4;
          sa += a1;
          sb = max(sb + a1, 0);
          anyw |= e8[j];
        }
        // inclusive scan (composition) over my child's words 0..wl
        for (int o = 1; o < 32; o <<= 1) {
          const int pa = __shfl_up(sa, o, 32), pb = __shfl_up(sb, o, 32);
          if (wl >= (uint32_t)o) {
            sb = max(pb + sa, sb);
            sa += pa;
          }
        }
        const int pend = max(sa, sb);  // waiting after my word
        int pst = __shfl_up(pend, 1, 32);
        if (wl == 0) pst = 0;
        const uint32_t zb = (uint32_t)(__ballot(pst == 0) >> (32u * c)) & (wl == 31u ? ~0u : (2u << wl) - 1u);
        const uint32_t w0 = 31u - (uint32_t)__builtin_clz(zb);
        uint32_t M = 0;
        for (uint32_t vv = pst > 0 ? w0 : wl; vv < wl; ++vv) {  // catch up, recording nothing
          uint32_t ev[8];
          line8(vv, ev);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            M |= ev[j];
#pragma unroll
            for (int t = 0; t < 4; ++t) M = (M & (M - 1u)) >> 1;
          }
        }
        if (pst > 0 || anyw) {
          const uint32_t base = wl * 32u;
          uint32_t occw = 0;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            M |= e8[j];
#pragma unroll
            for (int t = 0; t < 4; ++t) {
              if (M) {
                const uint32_t x = base + 4u * (uint32_t)j + (uint32_t)t;
                s_dst[(x + (uint32_t)__builtin_ctz(M)) & (kSlots - 1)] = (uint16_t)((c << 10) | x);
                occw |= 1u << (4 * j + t);
                M &= M - 1u;
              }
              M >>= 1;
            }
          }
          if (occw) atomicOr(&s_cb[c * 32u + wl], occw);
        }
        bad |= __builtin_popcount(M) != pend;  // cannot happen: the replay agrees with the scan
      }
      __builtin_amdgcn_wave_barrier();
    }
    const bool fast = !all_full && __ballot(wide) == 0;
    if (stamp && lane == 0) stamp[6] = fast ? 1 : 2;
    if (!fast) {
      // a full parent or a unit wider than 128 slots: the generic replay
      // rewrites every placement and both child bitmaps
      loss = split_slow(s_inf, s_dst, s_cb, s_rep);
    }
    for (int o = 32; o > 0; o >>= 1) loss += (uint32_t)__shfl_down((int)loss, o);
    loss = (uint32_t)__shfl((int)loss, 0);
    bad = __ballot(bad) != 0;
    if (NW > 1 && lane == 0) {
      s_tm[1] = loss;
      if (bad) s_tm[0] |= 2u;
    }
    if (NW == 1) *bad_out = bad;
  }
  SP_STAMP(2);
  // every child slot is written exactly once: an entry or INVALID.  Child 0
  // is the parent's storage, so every parent pair is reloaded (L2-hot) into
  // registers before the first store (of any wave of the team); the stores
  // go group by group.
  __asm__ volatile("" ::: "memory");  // no reload hoisted across the replay
  team_barrier();
  ulonglong2 r[G];
#ifndef PMDFC_SPLIT_RELOAD
#define PMDFC_SPLIT_RELOAD 0  // (A/B builds) 1: the reload with plain loads instead of non-temporal ones
#endif
#pragma unroll
  for (int j = 0; j < G; ++j) {
    if constexpr (PMDFC_SPLIT_RELOAD) r[j] = sp[(g0 + j) * 64 + lane];
    else r[j] = ld_pair_l2(sp + (g0 + j) * 64 + lane);
  }
  wait_vmcnt<0>();  // every parent pair is in registers: no store waits below
  if constexpr (NW > 1) {
    team_barrier();  // (another wave's stores may land in my groups)
    loss = s_tm[1];
    *bad_out = (s_tm[0] & 2u) != 0;
  }
  SP_STAMP(3);
#pragma unroll
  for (int j = 0; j < G; ++j) {
    const uint32_t slot = (uint32_t)(g0 + j) * 64u + lane;
    const uint32_t d = s_dst[slot];
    if (d != 0xFFFFu) ((d >> 10) ? s1 : sp)[d & 1023u] = r[j];
#pragma unroll
    for (int c = 0; c < 2; ++c)
      if (!((s_cb[c * 32u + (slot >> 5)] >> (slot & 31u)) & 1u)) (c ? s1 : sp)[slot] = make_ulonglong2(kInvalid, 0ULL);
  }
  if (drops && loss) {
    // a valid parent entry with no placement was dropped (rare path)
#pragma unroll
    for (int j = 0; j < G; ++j) {
      const uint32_t slot = (uint32_t)(g0 + j) * 64u + lane;
      if (s_dst[slot] == 0xFFFFu && r[j].x != kInvalid) {
        const uint32_t k = atomicAdd(drop_n, 1u);
        if (k < kDropLog) drops[k] = make_ulonglong2(r[j].x, trig);
      }
    }
  }
  if (v == 0) {
    const uint32_t bw = s_cb[lane];  // lanes 0-31 child-0 words, 32-63 child-1 words
    if (lane < 32) occ[(size_t)seg * 32u + lane] = bw;
    else occ[(size_t)c1 * 32u + (lane - 32)] = bw;
    if (lane == 0) {
      ldep[seg] = (uint8_t)(L + 1);
      ldep[c1] = (uint8_t)(L + 1);
    }
  }
  SP_STAMP(4);  // the stores may still be in flight (callers wait when they re-read)
  if constexpr (NW > 1) team_barrier();  // (the scratch is reused by the team's next split)
  return loss;
}

__device__ __forceinline__ uint32_t wave_split(ulonglong2* __restrict__ pairs, uint32_t* __restrict__ occ,
                                               uint8_t* __restrict__ ldep, uint32_t seg, uint32_t c1, uint32_t L,
                                               uint32_t* scr, bool* bad_out, uint64_t* stamp,
                                               ulonglong2* drops = nullptr, uint32_t* drop_n = nullptr,
                                               uint32_t trig = 0) {
  return split_team<1>(pairs, occ, ldep, seg, c1, L, scr, bad_out, stamp, drops, drop_n, trig, 0u);
}

// ------------------------------------------------------------------ bucket

struct BucketArgs {
  const ulonglong2* rkv;
  const uint32_t* rop;
  const uint16_t* robk;
  uint64_t n;            // batch size (op indices are < n)
  uint32_t chunk;        // ops per wave chunk (<= kCW)
  uint32_t cap;          // records per bucket region
  uint32_t capx;         // ... per sub-region (kPartSubs of them)
  uint64_t ovf_base;
  const uint32_t* cursor;  // this batch's cursors (kPartSubs per bucket) / overflow count
  const uint32_t* ovf;
  uint32_t* cursor_next;   // cleared here for the next batch (clear_next)
  uint32_t* ovf_next;
  uint32_t clear_next;     // 0 when the next batch is already being partitioned
  uint64_t* hdr;
  uint32_t* pool;
  uint32_t pool_cap;
  uint32_t p1, sbb, sbits, shard;
  uint32_t pfix;         // small sub-directories in fixed slots (cceh_kernels.h kFixedBits)
  ulonglong2* pairs;
  uint32_t* occ;
  uint8_t* ldep;
  uint64_t* vout;        // mixed only
  uint8_t* st;
  uint32_t mixed;
  uint32_t upsert;       // last-writer-wins Insert
  const uint16_t* upos;  // upsert: pre-batch key slots (k_upsert_probe)
  uint32_t max_segments;
  DevCtl* ctl;
  uint64_t* wstat;       // per directory bucket: kWStat cumulative counters
  ulonglong2* wl_kv;     // per directory bucket: kCW parked {key, value}
  uint32_t* wl_op;       // ... and their rop words
  uint32_t* wl_n;        // per directory bucket: parked count, or kBigBucket
  uint64_t* stamps;      // debug: 16 wall-clock stamps per wave, or null
  uint2* req;            // per directory bucket: kSplitCap split requests
  uint32_t* reqop;       // ... and the batch position of each request's insert
  ulonglong2* drops;     // mixed batches with early answers: the drop log (else null)
  uint32_t* need;
  uint32_t* gbase;
  uint32_t* ngrant;
  uint32_t* newoff;
  uint64_t* gsh;           // grant shard words, gsplit their requested splits (cceh_kernels.h)
  uint4* gsplit;
  uint32_t gcap;
  uint32_t* act;
  uint32_t* fbl;         // per bucket: bit 0 k_apply_fast declined it (-> k_apply_fb), bits 1+ declines so far
  uint32_t* hint;        // host-mapped: the segment count after this batch's grants (k_apply_parked)
  uint32_t mode;         // k_apply: 0 first pass, 1 parked-op pass, 2 parked-op pass without
                         // split requests (the last before the final pass)
  uint32_t* fin;         // k_bucket's worklist of this batch (count: ctl->nfin[par])
  uint32_t par;
  // mixed batches: both apply variants are launched and exactly one runs.
  // gate 1 (MIXED kernels) runs iff ctl->pget == gate_tag (k_mixed_get left
  // a Get pending), gate 2 (the insert-only kernels) iff not; 0: always
  uint32_t gate, gate_tag;
  uint32_t* mseen;       // host-mapped: k_apply<true> stores gate_tag when it runs (BucketLaunch::mseen)
};

struct ServeArgs {
  BucketArgs a;                 // the engine at launch (st / vout: 64-entry device scratch)
  const pmdfc_serve_req* req;   // device mappings of the host rings (wave w: places w * ring_size ...)
  pmdfc_serve_resp* resp;
  pmdfc_serve_ctl* ctl;         // one per wave
  uint64_t ring_size, head0;    // head0: one wave's first place; several waves start at their ctl->head
  uint32_t nwaves;
  uint8_t* cbf;                 // counting BF counters, or null
  uint64_t cbf_m;
  uint32_t cbf_k;
};
constexpr uint32_t kServeHdrMax = 1024;  // directory buckets the serving wave caches in LDS (8 KB)
constexpr uint64_t kServeWatchdog = 100000000ull;  // wall_clock64 ticks (100 MHz): ~1 s without a heartbeat
constexpr uint64_t kServeIdle = 100000ull;         // ~1 ms without ops: raise ctl->idle (callers on a CPU-
                                                   // quota'd host pause for longer than 100 us at times)

// 0 start, 1 collected, 2 round-0 sorted, 3 round-0 applied, 7 end (first
// k_apply pass); 8..13 the same for the final pass (12: round-0 splits done)
#define BK_STAMP(ph) \
  if (a.stamps && lane == 0) a.stamps[(size_t)w * 16 + (ph)] = wall_clock64()

constexpr uint32_t kBmWords = kBmLanes * 33;
constexpr uint32_t kUnionWords = kBmWords > kSplitScratch ? kBmWords : kSplitScratch;

// Collect this wave's ops of the batch into LDS (records of its region, read
// coalesced, then its records in the overflow area).  Stores up to kCW;
// returns how many matched.
__device__ __forceinline__ uint32_t collect(const BucketArgs& a, uint32_t pb, uint32_t sub,
                                            uint32_t csub, uint32_t novf, ulonglong2* s_kv,
                                            uint32_t* s_op) {
  const uint32_t lane = __lane_id() & 63u;
  const uint64_t lt = (1ULL << lane) - 1;
  const uint32_t sbm = (1u << a.sbb) - 1;
  uint32_t m = 0;
  for (uint32_t xs = 0; xs < kPartSubs; ++xs) {  // csub: lane xs holds sub-region xs's count
  const uint32_t cnt = (uint32_t)__shfl((int)csub, (int)xs);
  const uint64_t rb = (uint64_t)pb * a.cap + (uint64_t)xs * a.capx;
  for (uint32_t j0 = 0; j0 < cnt; j0 += 128) {
    // plain scalars, all loads issued before any use (a conditionally set
    // ulonglong2[] lands in scratch memory and serializes the loads)
    uint32_t r[2];
    uint64_t kx[2], vx[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const uint32_t j = min(j0 + u * 64 + lane, cnt - 1);
      r[u] = a.rop[rb + j];
      const ulonglong2 kv = a.rkv[rb + j];
      kx[u] = kv.x;
      vx[u] = kv.y;
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const uint32_t j = j0 + u * 64 + lane;
      const bool match = j < cnt && ((r[u] >> 22) & sbm) == sub;
      const uint64_t bal = __ballot(match);
      const uint32_t idx = m + (uint32_t)__popcll(bal & lt);
      if (match && idx < (uint32_t)kCW) {
        s_kv[idx] = make_ulonglong2(kx[u], vx[u]);
        s_op[idx] = r[u];
      }
      m += (uint32_t)__popcll(bal);
    }
  }
  }
  for (uint32_t j0 = 0; j0 < novf; j0 += 64) {
    const uint32_t j = j0 + lane;
    bool match = false;
    uint32_t r = 0;
    if (j < novf && a.robk[j] == pb) {
      r = a.rop[a.ovf_base + j];
      match = ((r >> 22) & sbm) == sub;
    }
    const uint64_t bal = __ballot(match);
    const uint32_t idx = m + (uint32_t)__popcll(bal & lt);
    if (match && idx < (uint32_t)kCW) {
      s_kv[idx] = a.rkv[a.ovf_base + j];
      s_op[idx] = r;
    }
    m += (uint32_t)__popcll(bal);
  }
  __builtin_amdgcn_wave_barrier();
  return m;
}

// ---- big buckets (final pass): more ops than one chunk.  Chunks must follow
// batch order (per segment), and k_part wrote each (tile, bucket) as ONE
// contiguous run in the region plus at most one in the overflow area, where a
// tile is kPartTile consecutive ops.  So one scan finds every tile's runs, and
// the chunks walk the tiles in order: whole tiles while they fit, and a tile
// larger than a chunk through a map of its ops by in-tile index.  Linear in
// the bucket's records.
struct BigLds {
  uint32_t rs[kMaxPartBlocks], re[kMaxPartBlocks];  // region run of each tile
  uint32_t os[kMaxPartBlocks], oe[kMaxPartBlocks];  // overflow run of each tile
  uint16_t map[kPartTile];                          // in-tile op -> record of the tile
};
__device__ __forceinline__ BigLds* big_lds() {
  __shared__ BigLds s;
  return &s;
}

__device__ __forceinline__ uint32_t tile_of(uint32_t rop) { return (rop & kOpMask) / kPartTile; }

__device__ void big_index(const BucketArgs& a, BigLds* L, uint32_t pb, uint32_t csub, uint32_t novf,
                          uint32_t ntile) {
  const uint32_t lane = __lane_id() & 63u;
  for (uint32_t t = lane; t < ntile; t += 64) L->rs[t] = L->re[t] = L->os[t] = L->oe[t] = 0;
  __builtin_amdgcn_wave_barrier();
  // tile t's region run lies in sub-region t % kPartSubs (k_part block t);
  // rs/re are offsets inside that sub-region
  for (uint32_t xs = 0; xs < kPartSubs; ++xs) {
    const uint32_t cnt = (uint32_t)__shfl((int)csub, (int)xs);
    const uint64_t rb = (uint64_t)pb * a.cap + (uint64_t)xs * a.capx;
    for (uint32_t j = lane; j < cnt; j += 64) {
      const uint32_t t = tile_of(a.rop[rb + j]);
      if (j == 0 || tile_of(a.rop[rb + j - 1]) != t) L->rs[t] = j;
      if (j + 1 == cnt || tile_of(a.rop[rb + j + 1]) != t) L->re[t] = j + 1;
    }
  }
  for (uint32_t j = lane; j < novf; j += 64) {
    if (a.robk[j] != pb) continue;
    const uint32_t t = tile_of(a.rop[a.ovf_base + j]);
    if (j == 0 || a.robk[j - 1] != pb || tile_of(a.rop[a.ovf_base + j - 1]) != t) L->os[t] = j;
    if (j + 1 == novf || a.robk[j + 1] != pb || tile_of(a.rop[a.ovf_base + j + 1]) != t) L->oe[t] = j + 1;
  }
  __builtin_amdgcn_wave_barrier();
}

// record slot of entry k of tile t's runs (region first, then overflow)
__device__ __forceinline__ uint64_t big_rec(const BucketArgs& a, const BigLds* L, uint64_t rb, uint32_t t,
                                            uint32_t k) {
  const uint32_t rl = L->re[t] - L->rs[t];
  return k < rl ? rb + (uint64_t)(t % kPartSubs) * a.capx + L->rs[t] + k : a.ovf_base + L->os[t] + (k - rl);
}

// Next chunk of a big bucket into s_kv/s_op: ops of tiles [t, ...) in batch
// order, at most C.  (t, mp) is the walk position (mp > 0: inside tile t's map).
__device__ uint32_t big_chunk(const BucketArgs& a, BigLds* L, uint32_t pb, uint32_t sub, uint32_t ntile,
                              uint32_t C, uint32_t& t, uint32_t& mp, ulonglong2* s_kv, uint32_t* s_op) {
  const uint32_t lane = __lane_id() & 63u;
  const uint64_t lt = (1ULL << lane) - 1;
  const uint32_t sbm = (1u << a.sbb) - 1;
  const uint64_t rb = (uint64_t)pb * a.cap;
  uint32_t m = 0;
  while (t < ntile) {
    const uint32_t ct = (L->re[t] - L->rs[t]) + (L->oe[t] - L->os[t]);
    if (ct == 0) {
      ++t;
      continue;
    }
    if (mp == 0 && m + ct <= C) {  // the whole tile joins the chunk
      for (uint32_t k0 = 0; k0 < ct; k0 += 64) {
        const uint32_t k = k0 + lane;
        bool match = false;
        uint64_t rs = 0;
        uint32_t r = 0;
        if (k < ct) {
          rs = big_rec(a, L, rb, t, k);
          r = a.rop[rs];
          match = ((r >> 22) & sbm) == sub;
        }
        const uint64_t bal = __ballot(match);
        const uint32_t idx = m + (uint32_t)__popcll(bal & lt);
        if (match) {
          s_kv[idx] = a.rkv[rs];
          s_op[idx] = r;
        }
        m += (uint32_t)__popcll(bal);
      }
      ++t;
      continue;
    }
    if (mp == 0 && m > 0) break;  // a big tile starts its own chunk
    if (mp == 0) {
      for (uint32_t k = lane; k < kPartTile; k += 64) L->map[k] = 0xFFFF;
      __builtin_amdgcn_wave_barrier();
      for (uint32_t k = lane; k < ct; k += 64) {
        const uint32_t r = a.rop[big_rec(a, L, rb, t, k)];
        if (((r >> 22) & sbm) == sub) L->map[(r & kOpMask) % kPartTile] = (uint16_t)k;
      }
      __builtin_amdgcn_wave_barrier();
    }
    // walk the map from mp, taking ops in batch order until the chunk is full
    while (mp < kPartTile && m < C) {
      const uint32_t e = mp + lane < kPartTile ? L->map[mp + lane] : 0xFFFFu;
      const bool v = e != 0xFFFFu;
      const uint64_t bal = __ballot(v);
      const uint32_t room = C - m, nv = (uint32_t)__popcll(bal);
      const uint32_t idx = (uint32_t)__popcll(bal & lt);
      if (v && idx < room) {
        const uint64_t rs = big_rec(a, L, rb, t, e);
        s_kv[m + idx] = a.rkv[rs];
        s_op[m + idx] = a.rop[rs];
      }
      if (nv > room) {
        // stop just past the room-th valid entry of this group
        uint64_t b = bal;
        for (uint32_t q = 0; q + 1 < room; ++q) b &= b - 1;
        mp += (uint32_t)__builtin_ctzll(b) + 1;
        m = C;
      } else {
        mp += 64;
        m += nv;
      }
    }
    if (mp >= kPartTile) {  // tile done (its tail may hold no op of ours)
      mp = 0;
      ++t;
    }
    if (m >= C) break;  // else room is left: go on with the next tiles
  }
  __builtin_amdgcn_wave_barrier();
  return m;
}

// The rare full-window path of a run (out of line: keeps the run loop's
// registers small).  The window may hold the run's deferred inserts: write
// those out first (the store pass writes them again, identically), then test
// whether all 32 window entries carry the new key's full hash.
__device__ __noinline__ bool window_all_same(uint32_t mixed, ulonglong2* sp, const uint64_t* s_sk,
                                             const uint16_t* s_pos, const ulonglong2* s_kv,
                                             uint32_t q0, uint32_t q, uint32_t i, uint32_t w0) {
  if (!mixed) {
    for (uint32_t qq = q0; qq < q; ++qq) {
      const uint32_t i2 = sk_item(s_sk[qq]);
      const uint32_t p2 = s_pos[i2];
      if (p2 != 0xFFFFu) sp[p2] = s_kv[i2];
    }
    __builtin_amdgcn_s_waitcnt(0);
  }
  const uint64_t h = hash64(s_kv[i].x);
  for (uint32_t t0 = 0; t0 < kWindow; t0 += 4) {
    ulonglong2 w4[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) w4[t] = ld_pair_l2(sp + ((w0 + t0 + t) & (kSlots - 1)));
    bool same = true;
#pragma unroll
    for (int t = 0; t < 4; ++t) same = same && hash64(w4[t].x) == h;
    if (!same) return false;
  }
  return true;
}

// The same test for the insert-only apply passes, whose pairs live in
// registers until the store pass: a window slot claimed by an earlier op of
// the run holds that op's key (s_pos / s_key), any other slot its key in
// memory.
__device__ __noinline__ bool window_all_same_reg(const ulonglong2* sp, const uint64_t* s_sk, const uint16_t* s_pos,
                                                 const uint64_t* s_key, uint32_t q0, uint32_t q, uint32_t i,
                                                 uint32_t w0) {
  const uint64_t h = hash64(s_key[i]);
  for (uint32_t t = 0; t < kWindow; ++t) {
    const uint32_t slot = (w0 + t) & (kSlots - 1);
    bool claimed = false;
    uint64_t k = kInvalid;
    for (uint32_t qq = q0; qq < q; ++qq) {
      const uint32_t i2 = sk_item(s_sk[qq]);
      if (s_pos[i2] == slot) {
        k = s_key[i2];
        claimed = true;
      }
    }
    if (!claimed) k = ld_pair_l2(sp + slot).x;
    if (hash64(k) != h) return false;
  }
  return true;
}

struct RunCtx {  // what one run needs (passed by value: no kernarg copies)
  ulonglong2* pairs;
  uint32_t* occ;
  uint64_t* vout;
  uint8_t* st;
  DevCtl* ctl;
  uint2* req;       // this bucket's split requests (k_apply)
  uint32_t* reqop;  // ... their inserts' batch positions
  uint32_t mixed, max_segments, full, noreq;
  uint64_t* stamp;  // debug: this wave's stamp row (first apply pass), or null
  uint32_t sbits, p1, db;  // geometry of the request's sub-index
  uint32_t upsert;  // last-writer-wins Insert
  const uint16_t* upos;  // upsert, first apply pass: pre-batch key slots by op index, else null
};

// Upsert (last-writer-wins, CCEH_hybrid.cpp:153's overwrite clause enabled):
// the slot of `key` in its window if the key is stored there, else -1.  The
// probe walks the occupied prefix of the window (the bitmap marks claims of
// this run too; their slots still read INVALID in memory, which never
// matches), one 64-B line at a time with its 4 pairs loaded together.  With no
// deletes no stored entry sits past the window's first free slot,
// so the first free slot ends the probe, as in the reference's claim order.
__device__ __forceinline__ int upsert_find(const ulonglong2* sp, const uint32_t* bm, uint32_t wi0, uint64_t key) {
  for (uint32_t l = 0; l < kLines; ++l) {
    const uint32_t s0 = (wi0 + 4u * l) & (kSlots - 1);  // line aligned: its 4 bits share a word
    const uint32_t occ4 = (bm[s0 >> 5] >> (s0 & 31u)) & 0xFu;
    if (occ4 == 0) return -1;
    ulonglong2 p4[4];
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q) p4[q] = ld_pair_l2(sp + s0 + q);
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q) {
      if (!((occ4 >> q) & 1u)) return -1;
      if (p4[q].x == key) return (int)(s0 + q);
    }
  }
  return -1;
}

// One segment run (ops q0..q1 of the sorted chunk, one segment), by one lane,
// against an LDS copy of the segment's occupancy bitmap.  A full window stops
// the run: k_apply requests a split (granted at the end of the pass, done by
// k_split) and parks the rest of the run; the final pass splits inline.
template <bool FINAL, bool MIXED>
__device__ __forceinline__ uint2 apply_run(RunCtx a, const uint64_t* s_sk, uint32_t q0, uint32_t q1,
                                        const uint8_t* s_L, const ulonglong2* s_kv, const uint64_t* s_key,
                                        const uint32_t* s_op,
                                        uint16_t* s_pos, uint8_t* s_pend, uint64_t* s_split,
                                        uint32_t* s_nsplit, uint32_t* s_nreq, uint32_t* s_need, uint32_t* bm,
                                        ulonglong2* wl_kv, uint32_t* wl_op, bool pre) {
  // REG: the insert-only apply passes keep each op's pair in its owner lane's
  // registers; the run sees the keys (s_key) only
  constexpr bool REG = !FINAL && !MIXED;
  const auto key_of = [&](uint32_t i) -> uint64_t {
    if constexpr (REG) return s_key[i];
    else return s_kv[i].x;
  };
  const uint32_t lbase = a.sbits + a.p1;
  uint32_t lines = 0, waited = 0;
    const uint64_t sk0 = s_sk[q0];
    const uint32_t seg = sk_seg(sk0);
    const uint32_t L = s_L[sk_item(sk0)] & 31u;
    if (!pre) {  // (the apply pass prefetches the bitmaps of its first kBmLanes runs)
      const uint32_t* og = a.occ + (size_t)seg * 32u;
      uint4 bv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) bv[j] = ld_u4_l2(og + 4 * j);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        bm[4 * j] = bv[j].x;
        bm[4 * j + 1] = bv[j].y;
        bm[4 * j + 2] = bv[j].z;
        bm[4 * j + 3] = bv[j].w;
      }
    }
    ulonglong2* sp = a.pairs + (size_t)seg * kSlots;
    bool dirty = false;
    uint32_t qs = q0;
    if constexpr (!FINAL) {
      // the apply passes' common case: a wave-uniform loop (exit by ballot)
      // with a branch-free body that only claims slots; it stops a lane at
      // its first full window -- or, in a mixed batch, at its first Get --
      // where the general loop below takes over (upsert batches take the
      // general loop: an insert first looks for its key)
      bool go = !a.upsert;
      uint64_t skn = s_sk[q0];
      for (uint32_t q = q0;; ++q) {
        const bool act = go && q < q1;
        if (__ballot(act) == 0) break;
        if (act) {
          const uint64_t skq = skn;
          skn = s_sk[min(q + 1u, (uint32_t)kCW - 1u)];  // read ahead
          const uint32_t wi0 = sk_home(skq) * 4u;
          const uint32_t wi = wi0 >> 5, wn = (wi + 1u) & 31u;
          const uint32_t lo = bm[wi], hi = bm[wn];
          const uint32_t fr = ~__builtin_amdgcn_alignbit(hi, lo, wi0 & 31u);
          bool ok = fr != 0;
          if constexpr (MIXED) ok = ok && !(s_L[sk_item(skq)] & 0x80u);  // a Get: the general loop
          const uint32_t t = (uint32_t)__builtin_ctz(fr | (ok ? 0u : 1u));
          const uint32_t b = ok ? 1u << ((wi0 + t) & 31u) : 0u;
          const bool in_lo = (wi0 & 31u) + t < 32u;
          bm[wi] = lo | (in_lo ? b : 0u);  // both words written: no divergent branch
          bm[wn] = hi | (in_lo ? 0u : b);
          if (ok) s_pos[sk_item(skq)] = (uint16_t)((wi0 + t) & (kSlots - 1));
          lines += ok ? (t >> 2) + 1 : 0u;
          qs = ok ? q + 1 : qs;
          go = ok;
        }
      }
      dirty = qs > q0;
      if constexpr (MIXED) {
        // the general loop goes on (a Get, or a full window it inspects): it
        // reads the segment, so the claims made so far are stored first
        if (qs > q0 && qs < q1) {
          for (uint32_t qq = q0; qq < qs; ++qq) {
            const uint64_t sk = s_sk[qq];
            const uint32_t i2 = sk_item(sk);
            sp[s_pos[i2]] = s_kv[i2];
            a.st[sk_op(sk)] = 2;  // PMDFC_ST_INSERTED
            s_pos[i2] = 0xFFFF;
          }
        }
      }
      if (a.stamp && (__lane_id() & 63u) == 0) a.stamp[14] = wall_clock64();
    }
    uint64_t nxt = qs < q1 ? s_sk[qs] : 0ULL;
    uint64_t memo_k = kInvalid, memo_v = 0;  // mixed: last Get probe of this run
    uint8_t memo_s = 0;
    for (uint32_t q = qs; q < q1; ++q) {
      const uint64_t skq = nxt;
      if (q + 1 < q1) nxt = s_sk[q + 1];  // prefetch the next op's key
      const uint32_t i = sk_item(skq);
      const uint32_t op = sk_op(skq);
      if (MIXED && (s_L[i] & 0x80u)) {
        // a Get sees the run's earlier inserts only through its own key
        // (others just fill empty slots past or instead of the probe's end),
        // so repeated Gets of one key reuse the last probe until that key
        // is inserted (hot keys of skewed batches)
        const uint64_t key = s_kv[i].x;
        if (key != memo_k) {
          memo_v = 0;
          memo_s = lane_probe(sp, key, hash64(key), &memo_v);
          memo_k = key;
        }
        a.vout[op] = memo_v;
        a.st[op] = memo_s;
        s_pend[i] = 0;
        continue;
      }
      const uint32_t wi0 = sk_home(skq) * 4u;
      const uint32_t wi = wi0 >> 5;
      if (a.upsert) {
        // last-writer-wins: the key's own slot takes the pair if it has one --
        // a claim of this run not yet stored (insert-only batches store after
        // the run loop; the earlier claim is dropped, this op writes the slot),
        // else the window in memory
        // (s_pos: the slot each op of the round took, kept by mixed batches
        // too, so a claim of the key earlier in this run is found here)
        const uint64_t key = key_of(i);
        int upos = -1;
        for (uint32_t qq = q0; qq < q; ++qq) {
          const uint32_t i2 = sk_item(s_sk[qq]);
          if (s_pos[i2] != 0xFFFFu && key_of(i2) == key) {
            upos = s_pos[i2];
            s_pos[i2] = 0xFFFF;
          }
        }
        if (upos < 0) {
          if (a.upos) {  // first pass: the pre-batch probe (no split of this batch yet)
            const uint32_t u = a.upos[op];
            upos = u == 0xFFFFu ? -1 : (int)u;
          } else {
            upos = upsert_find(sp, bm, wi0, key);
          }
        }
        if (upos >= 0) {
          s_pos[i] = (uint16_t)upos;
          if (MIXED) {
            if (key == memo_k) memo_k = kInvalid;
            sp[upos] = s_kv[i];
          }
          a.st[op] = 11;  // PMDFC_ST_UPDATED
          lines += ((((uint32_t)upos - wi0) & (kSlots - 1)) >> 2) + 1;
          s_pend[i] = 0;
          continue;
        }
      }
      const int pos = window_first_free(bm[wi], bm[(wi + 1) & 31u], wi0);
      if (pos >= 0) {
        bm[(uint32_t)pos >> 5] |= 1u << ((uint32_t)pos & 31u);
        dirty = true;
        if (MIXED) {
          if (s_kv[i].x == memo_k) memo_k = kInvalid;
          sp[pos] = s_kv[i];
          a.st[op] = 2;  // PMDFC_ST_INSERTED (insert-only batches: preset by k_part)
          if (a.upsert) s_pos[i] = (uint16_t)pos;  // a later insert of the key in this run updates it
        } else {
          s_pos[i] = (uint16_t)pos;
        }
        lines += ((((uint32_t)pos - wi0) & (kSlots - 1)) >> 2) + 1;
        s_pend[i] = 0;
        continue;
      }
      // window full.  The reference would split forever if all 32 entries
      // carry this key's full hash: UNSPLITTABLE.
      bool same;
      if constexpr (REG) same = window_all_same_reg(sp, s_sk, s_pos, s_key, q0, q, i, wi0);
      else same = window_all_same(MIXED, sp, s_sk, s_pos, s_kv, q0, q, i, wi0);
      if (same || L + 1 > kMaxDepth) {
        a.st[op] = same ? 4 : 5;  // PMDFC_ST_UNSPLITTABLE / PMDFC_ST_DEPTH_LIMIT
        s_pend[i] = 0;
        continue;
      }
      if (!FINAL) {
        if (a.full) {  // a split round ran out of segment ids or pool
          a.st[op] = 6;  // PMDFC_ST_CAPACITY
          s_pend[i] = 0;
          continue;
        }
        // request the split; park the rest of the run (batch order is
        // restored by the next pass's sort), nothing of it runs ahead
        const uint32_t ri = a.noreq ? kSplitCap : atomicAdd(s_nreq, 1u);
        if (ri < kSplitCap) {
          const uint32_t x = sub_index(hash64(key_of(i)), a.sbits, a.p1, a.db);
          a.req[ri] = make_uint2(seg | (L << 27), x);
          a.reqop[ri] = op;
          atomicMax(s_need, L + 1 - lbase);
        }
        if constexpr (!REG) {
          const uint32_t k0 = atomicAdd(s_nsplit, q1 - q);
          for (uint32_t qq = q; qq < q1; ++qq) {
            const uint32_t i2 = sk_item(s_sk[qq]);
            wl_kv[k0 + (qq - q)] = s_kv[i2];
            wl_op[k0 + (qq - q)] = s_op[i2];
          }
        } else {  // the rest of the run stays pending; its owner lanes park it
          for (uint32_t qq = q; qq < q1; ++qq) s_pend[sk_item(s_sk[qq])] = 2;
        }
        waited += q1 - q;
        break;
      }
      const uint32_t si = atomicAdd(s_nsplit, 1u);
      if (si >= kSplitCap) {
        waited += q1 - q;  // split queue full: the run retries next round
        break;
      }
      const uint32_t c1 = atomicAdd(&a.ctl->nsegs, 1u);
      if (c1 >= a.max_segments) {
        s_split[si] = ~0ULL;
        a.st[op] = 6;  // PMDFC_ST_CAPACITY
        s_pend[i] = 0;
        continue;
      }
      s_split[si] = (uint64_t)i | ((uint64_t)L << 16) | ((uint64_t)c1 << 21);
      atomicMax(s_need, L + 1 - lbase);
      waited += q1 - q;
      break;  // the rest of the run waits for the split
    }
    if (dirty) {
      uint32_t* o = a.occ + (size_t)seg * 32u;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        *reinterpret_cast<uint4*>(o + 4 * j) = make_uint4(bm[4 * j], bm[4 * j + 1], bm[4 * j + 2], bm[4 * j + 3]);
    }
    if (a.stamp && (__lane_id() & 63u) == 0) a.stamp[15] = wall_clock64();
    return make_uint2(lines, waited);
}

// Sub-directory growth to `need` bits: a new pool region, new[i] = old[i >> k]
// (CCEH_hybrid.cpp:208-219 at bucket scale).  A fixed slot grows in place
// (no == off, at most kFixedSlot entries): every old entry is read into a
// register before any new one is stored.
__device__ __forceinline__ void grow_subdir(const BucketArgs& a, uint32_t w, uint32_t no, uint32_t need,
                                            uint32_t& off, uint32_t& db) {
  const uint32_t lane = __lane_id() & 63u;
  const uint32_t size = 1u << need, sh = need - db;
  if (size <= 128) {  // (a fixed slot holds up to 128 entries: all read before any store)
    const uint32_t v0 = lane < size ? ld_u32_l2(a.pool + off + (lane >> sh)) : 0u;
    const uint32_t v1 = lane + 64u < size ? ld_u32_l2(a.pool + off + ((lane + 64u) >> sh)) : 0u;
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    if (lane < size) a.pool[no + lane] = v0;
    if (lane + 64u < size) a.pool[no + lane + 64u] = v1;
  } else {  // (never in place)
    for (uint32_t t = lane; t < size; t += 64) a.pool[no + t] = ld_u32_l2(a.pool + off + (t >> sh));
  }
  __builtin_amdgcn_s_waitcnt(0);
  off = no;
  db = need;
  if (lane == 0) a.hdr[w] = hdr_make(no, need);
}

// Directory half of a split (CCEH_hybrid.cpp:243-286): the 2^(db - Lb) entries
// of the parent; the first half keeps child 0 (the parent's id), the second
// half gets child 1.  x: any sub-index of the parent at the current db.
__device__ __forceinline__ void dir_split(const BucketArgs& a, uint32_t off, uint32_t db, uint32_t x,
                                          uint32_t seg, uint32_t c1, uint32_t L) {
  const uint32_t lane = __lane_id() & 63u;
  const uint32_t Lb = L - a.sbits - a.p1;
  const uint32_t span = 1u << (db - Lb);
  const uint32_t xs = x & ~(span - 1u);
  for (uint32_t t = lane; t < span; t += 64) a.pool[off + xs + t] = de_make(t < span / 2 ? seg : c1, L + 1);
}

// Commit the splits granted to this bucket at the end of its last pass
// (k_split already moved the entries): grow the sub-directory if they need
// it, then point the children's directory entries at them.
__device__ __forceinline__ void commit_splits(const BucketArgs& a, uint32_t w, uint32_t& off, uint32_t& db,
                                              uint32_t& c_splits, uint32_t& c_grow, uint32_t& max_ld) {
  const uint32_t ng = a.ngrant[w];
  if (!ng) return;
  const uint32_t db0 = db;
  const uint32_t nd = a.need[w];
  if (nd > db) {
    grow_subdir(a, w, a.newoff[w], nd, off, db);
    ++c_grow;
  }
  const uint32_t cb = a.gbase[w];
  const uint2* rq = a.req + (size_t)w * kSplitCap;
  for (uint32_t i = 0; i < ng; ++i) {
    const uint2 r = rq[i];
    const uint32_t L = r.x >> 27;
    dir_split(a, off, db, r.y << (db - db0), r.x & ((1u << 27) - 1), cb + i, L);
    max_ld = max(max_ld, L + 1);
  }
  __builtin_amdgcn_s_waitcnt(0);
  c_splits += ng;
  if ((__lane_id() & 63u) == 0) a.ngrant[w] = 0;
}

// A bucket's split requests, at the end of the apply pass that made them:
// one atomic on its shard's segment word (cceh_kernels.h: kGShards) and, if
// its sub-directory must grow, one on the shard's pool word reserve its
// offsets among the shard's requested child segments and pool entries; each
// request is then recorded at its segment offset (k_split takes one per
// wave and turns the offsets into global grants).  (The grants used to be a
// prefix sum over all buckets in a single-workgroup kernel between the
// passes, a 12-20 us latency chain per batch with splits; one unsharded word
// serializes the ~8k requests of a split-heavy batch for ~100 us.)
// Wave-uniform call, after the wave's request stores.
__device__ __forceinline__ void request_splits(const BucketArgs& a, uint32_t w, uint32_t nr, uint32_t need) {
  const uint32_t lane = __lane_id() & 63u, x = w % kGShards;
  unsigned long long* sh = reinterpret_cast<unsigned long long*>(a.gsh + ((size_t)a.par * kGShards + x) * kGStride);
  uint64_t old = 0;
  if (lane == 0) old = atomicAdd(sh, (unsigned long long)nr | (1ULL << 32));
  if (lane == 1 && need && !(a.pfix && need <= kFixedBits)) old = atomicAdd(sh + 16, 1ULL << need);  // (else its fixed slot)
  __builtin_amdgcn_s_waitcnt(0);  // (this wave's request stores: read back below from L2)
  const uint32_t rw = lane < nr ? ld_u32_l2(reinterpret_cast<const uint32_t*>(a.req + (size_t)w * kSplitCap + lane)) : 0u;
  const uint64_t os = shfl64(old, 0), op = shfl64(old, 1);
  if (lane == 0) a.ctl->anyreq[a.par] = 1;
  // (a pool offset past 2^32 saturates: it is denied either way)
  if (lane < nr)
    a.gsplit[((size_t)a.par * kGShards + x) * a.gcap + (uint32_t)os + lane] =
        make_uint4(rw, w | (lane << 14) | ((uint32_t)(os >> 32) << 20), (uint32_t)min<uint64_t>(op, 0xFFFFFFFFULL),
                   nr | (need << 8));
}

// The batch's shard words, as prefixes over the shards: requesting buckets,
// splits and pool entries before shard x and the totals.  The per-shard
// prefixes live in lane x (< kGShards) and are read with a cross-lane read
// by the wave-uniform shard index: as arrays indexed at run time they went
// to scratch memory, 144 B per lane stored by every k_split wave (~19 MB of
// writes per launch of 2,048 waves) and reloaded per split.
struct GrantScan {
  uint32_t ce_l, cs_l;  // lane x: requesting buckets / splits before shard x
  uint64_t cp_l;        // lane x: pool entries before shard x
  uint32_t E, S;
  uint64_t P;
  __device__ __forceinline__ uint32_t ce(uint32_t x) const { return (uint32_t)__shfl((int)ce_l, (int)x); }
  __device__ __forceinline__ uint32_t cs(uint32_t x) const { return (uint32_t)__shfl((int)cs_l, (int)x); }
  __device__ __forceinline__ uint64_t cp(uint32_t x) const { return shfl64(cp_l, (int)x); }
};
__device__ __forceinline__ GrantScan grant_scan(const uint64_t* gsh, uint32_t par) {
  const uint32_t lane = __lane_id() & 63u;
  // lanes 0-7: the shards' segment words, lanes 8-15: their pool words
  const uint64_t mine = lane < 2 * kGShards
      ? __builtin_nontemporal_load(gsh + ((size_t)par * kGShards + (lane % kGShards)) * kGStride + (lane / kGShards) * 16)
      : 0ULL;
  GrantScan g;
  uint32_t e = 0, sg = 0;
  uint64_t p = 0;
  g.ce_l = g.cs_l = 0;
  g.cp_l = 0;
#pragma unroll
  for (uint32_t x = 0; x < kGShards; ++x) {
    const uint64_t v = shfl64(mine, (int)x), vp = shfl64(mine, (int)(x + kGShards));
    if (lane == x) {
      g.ce_l = e;
      g.cs_l = sg;
      g.cp_l = p;
    }
    e += (uint32_t)(v >> 32);
    sg += (uint32_t)v;
    p += vp;
  }
  g.E = e;
  g.S = sg;
  g.P = p;
  return g;
}
// split k of the batch (shard-major): its shard, the last x with cs(x) <= k
// (the prefixes are non-decreasing, so that is how many of shards 1..7 have
// cs <= k)
__device__ __forceinline__ uint32_t split_shard(const GrantScan& g, uint32_t k) {
  const uint32_t lane = __lane_id() & 63u;
  return (uint32_t)__popcll(__ballot(lane >= 1u && lane < kGShards && g.cs_l <= k));
}

// ---- parallel claims of the insert-only apply passes (fast_claim)
//
// Serial semantics (CCEH_hybrid.cpp:143-168): a segment's inserts, in batch
// order, each take the first free slot of their 32-slot window; the first one
// that finds its window full splits the segment, and it and every later insert
// of the segment wait for the split.  Two inserts of a segment interact only
// if their windows overlap -- home lines less than 8 apart (cyclic) -- since an
// insert only ever claims inside its own window.  So:
//   * an insert whose claim range -- home slot to the first free slot of its
//     window in the pre-pass bitmap -- meets no other insert's window (no
//     other insert of the segment homed from 7 lines before its home to the
//     line of that slot) is INDEPENDENT: nothing can claim inside that range
//     before it, and its claim is in nobody's window, so it takes that slot
//     whatever the batch order (lane per op, in parallel);
//   * the others (DEPENDENT, ~1/3 at the config-2 load) resolve in rounds, each
//     on its own lane: an insert whose earlier overlapping inserts (smaller op
//     index, same segment) have all resolved takes the first free slot of its
//     window in the pre-pass bitmap plus their claims.  The earliest unresolved
//     insert of every segment resolves in each round, so the rounds end; their
//     number is the longest chain of overlapping inserts (2-3 at config 2);
//   * the segment's split point is the smallest op index whose window is
//     full; inserts after it are parked, the one at it requests the split
//     (decisions taken after the split point are dropped with their insert).
//     If that insert fails instead of splitting (UNSPLITTABLE, DEPTH_LIMIT,
//     CAPACITY: later inserts go on past it), the sorted run loop takes over.
// Nothing is written until every decision is made, so a segment with more than
// kDepMax dependent inserts (tiny or skewed tables) hands the round back to the
// sorted run loop.  Checked against the serial rule on random bitmaps and home
// lines, and by the parity suite (configs 1 and 2 whole-table bit-exact).
constexpr uint32_t kFastBins = 32;  // segments (bins) of a bucket fast_claim handles (the general pass, k_apply_fast)
constexpr uint32_t kDepMax = 32;    // dependent inserts per segment it resolves
// LDS scratch (u32 words) of fast_claim for a dependent list of up to NL
// inserts on up to NB segments (bins) of the bucket (the apply pass's union
// area: NL = kCW; k_apply_fast: kFC; k_apply_wide: kFCW, 64 bins)
template <uint32_t NL, uint32_t NB = kFastBins>
struct FcLayout {
  static_assert(NB <= 64, "one lane per bin");
  static constexpr uint32_t Hm = 0;                      // [bin][8] home lines holding an insert
  static constexpr uint32_t Dm = Hm + NB * 8;            // [bin][8] home lines holding >= 2
  static constexpr uint32_t Cnt = Dm + NB * 8;           // [bin] dependent inserts
  static constexpr uint32_t Dst = Cnt + NB;              // [bin] their first list position
  static constexpr uint32_t Full = Dst + NB;             // [bin] op index of the segment's split (~0 none)
  static constexpr uint32_t Opk = Full + NB;             // dependent list [NL]: op << 8 | home
  static constexpr uint32_t Snap = Opk + NL;             // [NL] window occupancy before the pass
  static constexpr uint32_t Res = Snap + NL;             // [NL] u16 result (kFr*), 0 = unresolved
  static constexpr uint32_t Slot = Res + NL / 2;         // [NL] u8 insert slot (key index)
  static constexpr uint32_t Binp = Slot + NL / 4;        // [NL] u8 bin of the list entry
  static constexpr uint32_t Unres = Binp + NL / 4;       // [bin] entries still unresolved (bit q: entry dst + q)
  static constexpr uint32_t Words = Unres + NB;
};
static_assert(FcLayout<kCW>::Words <= kBmWords + 2 * kCW, "fast_claim scratch spans the bitmap rows and sort keys");
constexpr uint32_t kFrClaim = 0x8000u, kFrFail = 0x4000u, kFrSplit = 0x2000u, kFrPark = 0x1000u;
constexpr uint32_t kFrFull = 0x0800u;  // window full: the segment's split point if it is the first

// every slot of the window starting at wo holds a key of full hash h: the
// pre-pass pairs in memory, or the key of an earlier claim of this pass in the
// segment's dependent list [b0, b0 + n) -- the reference would split forever.
// 0 no, 1 yes, 2 undecided (a slot claimed this pass and no key array: the
// lean pass keeps no keys in LDS and hands such a bucket back)
__device__ __forceinline__ uint32_t fc_all_same(const ulonglong2* sp, uint64_t h, uint32_t wo, const uint16_t* res,
                                             const uint8_t* slot8, const uint64_t* s_key, uint32_t b0, uint32_t n) {
  for (uint32_t t = 0; t < kWindow; ++t) {
    const uint32_t sl = (wo + t) & (kSlots - 1);
    uint64_t k = kInvalid;
    bool claimed = false;
    for (uint32_t q = 0; q < n; ++q) {
      const uint32_t r = res[b0 + q];
      if ((r & kFrClaim) && (r & (kSlots - 1)) == sl) {
        if (!s_key) return 2u;
        k = s_key[slot8[b0 + q]];
        claimed = true;
      }
    }
    if (!claimed) k = ld_pair_l2(sp + sl).x;
    if (hash64(k) != h) return 0u;
  }
  return 1u;
}

// A full window: the insert fails (UNSPLITTABLE, DEPTH_LIMIT, CAPACITY) or
// splits its segment.  Returns kFrFail | status, or kFrSplit (kFrFail | 0:
// undecided, see fc_all_same).
__device__ __forceinline__ uint32_t fc_full(const BucketArgs& a, uint32_t full, uint32_t e, uint64_t key,
                                            uint32_t wo, const uint16_t* res, const uint8_t* slot8,
                                            const uint64_t* s_key, uint32_t b0, uint32_t n) {
  const uint32_t same = fc_all_same(a.pairs + (size_t)de_seg(e) * kSlots, hash64(key), wo, res, slot8, s_key, b0, n);
  if (same == 2u) return kFrFail;
  if (same || de_ld(e) + 1 > kMaxDepth) return kFrFail | (same ? 4u : 5u);  // UNSPLITTABLE / DEPTH_LIMIT
  if (full) return kFrFail | 6u;  // PMDFC_ST_CAPACITY: a split round ran out of ids or pool
  return kFrSplit;
}

// bin(j): insert j's bin, an index (< NB) of its segment within the bucket
// (one bin per segment); the caller defines it.
// UPS (last-writer-wins, the lean pass): upd[j] is the pre-batch slot of
// insert j's key in its window (0xFFFF: absent; the caller probed it, with
// no duplicate key in the bucket) and occw[2j], occw[2j+1] its two occupancy
// words (loaded by the caller for that probe).  An insert whose key is
// stored claims nothing: it overwrites its slot (PMDFC_ST_UPDATED) unless its
// segment splits before it in the batch, then it is parked like the others.
template <uint32_t NL, uint32_t NB, bool UPS = false, class BinF>
__device__ __forceinline__ bool fast_claim(const BucketArgs& a, uint32_t w, uint32_t* sc,
                                           const uint64_t* s_key, ulonglong2* wl_kv, uint32_t* wl_op,
                                           uint32_t* s_nsplit, uint32_t* s_nreq, uint32_t* s_need,
                                           const uint64_t (&rk)[kPer], const uint64_t (&rv)[kPer],
                                           const uint32_t (&rop)[kPer], const bool (&pq)[kPer],
                                           const uint32_t (&e8)[kPer], const uint32_t (&home8)[kPer],
                                           const uint32_t (&x8)[kPer], BinF bin, uint32_t& c_runs,
                                           uint32_t& c_lines, uint32_t& c_waited, uint64_t* stamp,
                                           const uint32_t* upd = nullptr, const uint32_t* occw = nullptr) {
  using FL = FcLayout<NL, NB>;
  const uint32_t lane = __lane_id() & 63u;
#define FC_STAMP(ph) \
  if (stamp && lane == 0) stamp[ph] = wall_clock64()
  const uint32_t lbase = a.sbits + a.p1;
  const uint32_t full = a.ctl->full;
  uint32_t* const hm = sc + FL::Hm;
  uint32_t* const dm = sc + FL::Dm;
  uint32_t* const cnt = sc + FL::Cnt;
  uint32_t* const dst = sc + FL::Dst;
  uint32_t* const bfull = sc + FL::Full;
  uint32_t* const opk = sc + FL::Opk;
  uint32_t* const snap = sc + FL::Snap;
  uint16_t* const res = reinterpret_cast<uint16_t*>(sc + FL::Res);
  uint8_t* const slot8 = reinterpret_cast<uint8_t*>(sc + FL::Slot);
  uint8_t* const binp = reinterpret_cast<uint8_t*>(sc + FL::Binp);
  uint32_t* const unres = sc + FL::Unres;
  // claimers: the inserts that take a slot (UPS: not those whose key is stored)
  bool pc[kPer];
#pragma unroll
  for (int j = 0; j < kPer; ++j) pc[j] = pq[j] && (!UPS || upd[j] == 0xFFFFu);
  // each insert's two occupancy words (its window), in flight during the LDS work
  uint32_t olo[kPer], ohi[kPer];
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    if (!pc[j]) continue;
    if constexpr (UPS) {
      olo[j] = occw[2 * j];
      ohi[j] = occw[2 * j + 1];
    } else {
      const uint32_t* og = a.occ + (size_t)de_seg(e8[j]) * 32u;
      const uint32_t wi = home8[j] >> 3;
      olo[j] = ld_u32_l2(og + wi);
      ohi[j] = ld_u32_l2(og + ((wi + 1u) & 31u));
    }
  }
#pragma unroll
  for (int t = 0; t < (int)(2 * NB * 8 / 64); ++t) hm[t * 64 + lane] = 0;  // hm and dm
  if (lane < NB) {
    cnt[lane] = 0;
    bfull[lane] = 0xFFFFFFFFu;
  }
  __builtin_amdgcn_wave_barrier();
  // 1. home lines per segment; a line taken twice is marked in dm
  uint32_t st[kPer];  // per insert: result (kFr* | slot or status) | list position << 16 | dependent << 24
#pragma unroll
  for (int j = 0; j < kPer; ++j)
    if (pc[j]) st[j] = atomicOr(&hm[bin(j) * 8u + (home8[j] >> 5)], 1u << (home8[j] & 31u));
#pragma unroll
  for (int j = 0; j < kPer; ++j)
    if (pc[j] && ((st[j] >> (home8[j] & 31u)) & 1u)) atomicOr(&dm[bin(j) * 8u + (home8[j] >> 5)], 1u << (home8[j] & 31u));
  __builtin_amdgcn_wave_barrier();
  FC_STAMP(4);
  if (stamp && lane == 0) stamp[2] = 0;  // (no sort stamp: phase_stamps.py tells the paths apart)
  // 2. independent inserts claim now; dependent ones are counted per segment
  constexpr uint32_t kDep = 1u << 24;
  uint64_t fk = 0;  // first window key of this lane's first independent full window
  int fkj = -1;
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    st[j] = 0;
    if (!pc[j]) continue;
    const uint32_t h = home8[j], xc = bin(j), base = xc * 8u, l0 = (h - 7u) & 255u;
    const uint32_t wo = h * 4u;
    const uint32_t win = __builtin_amdgcn_alignbit(ohi[j], olo[j], wo & 31u);  // bit t: slot wo + t taken
    // lines another insert's window may claim in: its home within 7 lines
    // before this one's, up to the line of this one's claim (the whole window
    // when it is full) -- outside that, neither claim can see the other
    const uint32_t cl = ~win ? (uint32_t)__builtin_ctz(~win) >> 2 : 7u;
    const uint32_t w0 = hm[base + (l0 >> 5)], w1 = hm[base + (((l0 >> 5) + 1u) & 7u)];
    // bit i: line h - 7 + i holds an insert; lines h-7..h+cl but h itself
    const uint32_t nb = __builtin_amdgcn_alignbit(w1, w0, l0 & 31u) & ((0x100u << cl) - 1u) & ~0x80u;
    const bool dup = (dm[base + (h >> 5)] >> (h & 31u)) & 1u;
    if (nb != 0 || dup) {
      const uint32_t r = atomicAdd(&cnt[xc], 1u);
      st[j] = kDep | (r << 16);
    } else if (~win) {
      st[j] = kFrClaim | ((wo + (uint32_t)__builtin_ctz(~win)) & (kSlots - 1));
    } else {
      st[j] = kFrFull;
      atomicMin(&bfull[xc], rop[j] & kOpMask);
      if (fkj < 0) {  // the window's first key, for the rarely true UNSPLITTABLE test below
        fk = ld_pair_l2(a.pairs + (size_t)de_seg(e8[j]) * kSlots + wo).x;
        fkj = j;
      }
    }
  }
  __builtin_amdgcn_wave_barrier();
  const uint32_t cb = lane < NB ? cnt[lane] : 0u;
  if (__ballot(cb > kDepMax)) return false;  // nothing written outside the scratch yet
  uint32_t ntot;
  const uint32_t ex = wave_excl_scan(cb, &ntot);
  if (lane < NB) dst[lane] = ex;
  uint32_t runs = 0;
  if (lane < NB) {
    uint32_t any = 0;
#pragma unroll
    for (int t = 0; t < 8; ++t) any |= hm[lane * 8u + t];
    runs = (uint32_t)__popcll(__ballot(any != 0));
  }
  __builtin_amdgcn_wave_barrier();
  FC_STAMP(5);
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    if (!(st[j] & kDep)) continue;
    const uint32_t xc = bin(j), p = dst[xc] + ((st[j] >> 16) & 0xFFu);
    st[j] = kDep | (p << 16);
    opk[p] = ((rop[j] & kOpMask) << 8) | home8[j];
    snap[p] = __builtin_amdgcn_alignbit(ohi[j], olo[j], (home8[j] * 4u) & 31u);  // the window before the pass
    res[p] = 0;
    slot8[p] = (uint8_t)((uint32_t)j * 64u + lane);
    binp[p] = (uint8_t)xc;
  }
  if (lane < NB) unres[lane] = cb >= 32 ? 0xFFFFFFFFu : (1u << cb) - 1u;
  __builtin_amdgcn_wave_barrier();
  // 3. dependent inserts resolve in rounds, one list entry per lane (the
  // list is usually shorter than a wave): first each entry's earlier
  // overlapping entries of its segment as a mask over the segment's list,
  // then rounds in which an entry whose mask is resolved decides
  constexpr int kLp = (int)NL / 64;
  uint32_t dmask[kLp], lres[kLp];
#pragma unroll
  for (int u = 0; u < kLp; ++u) {
    const uint32_t p = (uint32_t)u * 64u + lane;
    dmask[u] = 0;
    lres[u] = 1;  // (no entry: nothing to resolve)
    if (p >= ntot) continue;
    lres[u] = 0;
    const uint32_t v = opk[p], xc = binp[p], q0 = dst[xc], n = cnt[xc];
    const uint32_t op = v >> 8, h = v & 0xFFu;
    for (uint32_t q = 0; q < n; q += 4) {  // 4 independent LDS reads in flight
      uint32_t vq[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) vq[t] = q + t < n ? opk[q0 + q + t] : 0xFFFFFFFFu;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const uint32_t dl = ((vq[t] & 0xFFu) - h) & 0xFFu;
        if ((vq[t] >> 8) < op && (dl <= 7u || dl >= 249u)) dmask[u] |= 1u << (q + t);
      }
    }
  }
  FC_STAMP(10);
  uint32_t nrounds = 0;
  for (uint32_t round = 0; round <= kDepMax; ++round) {
    ++nrounds;
    bool blocked_any = false;
    uint32_t nr[kLp];
#pragma unroll
    for (int u = 0; u < kLp; ++u) {
      nr[u] = 0;
      const uint32_t p = (uint32_t)u * 64u + lane;
      if (lres[u]) continue;
      const uint32_t xc = binp[p];
      if (dmask[u] & unres[xc]) {
        blocked_any = true;
        continue;
      }
      const uint32_t v = opk[p], wo = (v & 0xFFu) * 4u, q0 = dst[xc];
      uint32_t occw = snap[p];
      bool park = false;
      for (uint32_t m = dmask[u]; m; m &= m - 1u) {
        const uint32_t rq = res[q0 + (uint32_t)__builtin_ctz(m)];
        const uint32_t ds = ((rq & (kSlots - 1)) - wo) & (kSlots - 1);
        park |= (rq & (kFrFull | kFrPark)) != 0;
        if ((rq & kFrClaim) && ds < kWindow) occw |= 1u << ds;
      }
      if (park) {  // behind an earlier full window of its segment: waits with it
        nr[u] = kFrPark;
      } else if (~occw) {
        nr[u] = kFrClaim | ((wo + (uint32_t)__builtin_ctz(~occw)) & (kSlots - 1));
      } else {
        nr[u] = kFrFull;
        atomicMin(&bfull[xc], v >> 8);
      }
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int u = 0; u < kLp; ++u) {
      if (!nr[u]) continue;
      const uint32_t p = (uint32_t)u * 64u + lane, xc = binp[p];
      res[p] = (uint16_t)nr[u];
      atomicAnd(&unres[xc], ~(1u << (p - dst[xc])));
      lres[u] = nr[u];
    }
    __builtin_amdgcn_wave_barrier();
    if (!__ballot(blocked_any)) break;
  }
  FC_STAMP(12);
  if (stamp && lane == 0) stamp[11] = nrounds | ((uint64_t)ntot << 16);
  // owners take their dependent results
#pragma unroll
  for (int j = 0; j < kPer; ++j)
    if (st[j] & kDep) st[j] |= res[(st[j] >> 16) & 0xFFu];
  // the first full window of a segment splits it -- unless the insert fails
  // instead (UNSPLITTABLE / DEPTH_LIMIT / CAPACITY, rare): then later inserts
  // go on past it, which the sorted run loop handles
  bool fails = false;
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    if (!pc[j] || (rop[j] & kOpMask) != bfull[bin(j)]) continue;
    const uint32_t xc = bin(j), q0 = (st[j] & kDep) ? dst[xc] : 0u, n = (st[j] & kDep) ? cnt[xc] : 0u;
    if (fkj == j && hash64(fk) != hash64(rk[j])) {  // not all one hash: splittable
      fails |= de_ld(e8[j]) + 1 > kMaxDepth || full;
      continue;
    }
    fails |= fc_full(a, full, e8[j], rk[j], home8[j] * 4u, res, slot8, s_key, q0, n) != kFrSplit;
  }
  if (__ballot(fails)) return false;  // still nothing written
  FC_STAMP(6);
  // 4. commit what precedes each segment's split, park the rest
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    if (!pq[j]) continue;
    const uint32_t op = rop[j] & kOpMask, bf = bfull[bin(j)];
    const uint32_t r = st[j] & 0xFFFFu;
    const uint32_t seg = de_seg(e8[j]);
    if (op >= bf || (r & kFrPark)) {
      if (op == bf) {  // this insert's full window splits the segment
        const uint32_t L = de_ld(e8[j]);
        const uint32_t ri = a.mode == 2 ? kSplitCap : atomicAdd(s_nreq, 1u);
        if (ri < kSplitCap) {
          a.req[(size_t)w * kSplitCap + ri] = make_uint2(seg | (L << 27), x8[j]);
          a.reqop[(size_t)w * kSplitCap + ri] = op;
          atomicMax(s_need, L + 1 - lbase);
        }
      }
      const uint32_t k = atomicAdd(s_nsplit, 1u);
      wl_kv[k] = make_ulonglong2(rk[j], rv[j]);
      wl_op[k] = rop[j];
      ++c_waited;
    } else if (r & kFrClaim) {
      const uint32_t sl = r & (kSlots - 1);
      a.pairs[(size_t)seg * kSlots + sl] = make_ulonglong2(rk[j], rv[j]);
      atomicOr(a.occ + (size_t)seg * 32u + (sl >> 5), 1u << (sl & 31u));
      c_lines += (((sl - home8[j] * 4u) & (kSlots - 1)) >> 2) + 1u;
    } else if (UPS && !pc[j]) {  // its key is stored: overwrite in place
      const uint32_t sl = upd[j];
      a.pairs[(size_t)seg * kSlots + sl] = make_ulonglong2(rk[j], rv[j]);
      a.st[op] = 11;  // PMDFC_ST_UPDATED
      c_lines += (((sl - home8[j] * 4u) & (kSlots - 1)) >> 2) + 1u;
    }
  }
  if (lane == 0) c_runs += runs;
  FC_STAMP(3);
#undef FC_STAMP
  return true;
}

// k_apply (FINAL = false, high occupancy, no split code): one round per
// directory bucket; a run blocked by a full window requests a split and parks
// the rest of the run.  mode 0 takes the bucket's records of the batch, mode 1
// its parked ops (after committing the last split round's splits).
// k_bucket (FINAL = true): buckets with parked ops, granted splits or too many
// ops for one chunk; loops rounds with inline splits until its ops are done.
constexpr uint32_t kBigBucket = 0xFFFFFFFFu;

constexpr uint32_t kLdsDir = 128;  // k_apply: sub-directories up to this size are read into LDS

// LDS of one bucket wave; the apply pass (no splits) carries no split state,
// which keeps its footprint, and so its occupancy, lower.
// The first apply pass of a batch (parity p) resets the previous batch's
// grant shards and final-pass count (parity p ^ 1): every pass that read
// them ran before it on the stream.
__device__ __forceinline__ void clear_other_parity(const BucketArgs& a) {
  const uint32_t lane = __lane_id() & 63u, q = a.par ^ 1u;
  if (lane < 2 * kGShards) a.gsh[((size_t)q * kGShards + (lane % kGShards)) * kGStride + (lane / kGShards) * 16] = 0;
  if (lane == 2 * kGShards) a.ctl->nfin[q] = 0;
  if (lane == 2 * kGShards + 1) a.ctl->anyreq[q] = 0;
  if (lane == 2 * kGShards + 2) a.ctl->anydecl[q] = 0;
}

template <bool FINAL, bool REG>
struct BucketLds {
  uint32_t u[FINAL ? kUnionWords : kBmWords];  // run phase: per-lane bitmaps; split phase: scratch
  uint64_t sk[kCW];       // sort keys of the pending ops
  ulonglong2 kv[REG ? 1 : kCW];   // {key, value} of each chunk slot (REG: in registers)
  uint64_t key[REG ? kCW : 1];    // REG: the key of each chunk slot
  uint32_t op[REG ? 1 : kCW];     // rop word of each chunk slot (REG: in registers)
  uint16_t pos[kCW];      // insert-only: slot claimed this round, 0xFFFF none
  uint16_t runq[kCW + 1];
  uint8_t L[kCW];         // local depth of the op's segment | Get << 7
  uint8_t pend[kCW];
  uint64_t split[FINAL ? kSplitCap : 1];
  uint32_t dir[FINAL ? 1 : kLdsDir];           // apply pass: the bucket's sub-directory
  uint32_t nsplit, nreq, need;
};
// the REG collect path stages kCW {key, value} pairs across u and sk
using BucketLdsReg = BucketLds<false, true>;
static_assert(offsetof(BucketLdsReg, sk) == sizeof(uint32_t) * kBmWords &&
                  sizeof(uint32_t) * kBmWords + sizeof(uint64_t) * kCW >= sizeof(ulonglong2) * kCW,
              "REG collect staging spans u and sk");


// pre_m (final pass only): the chunk's pre_m ops are already in S.kv / S.op
// (k_mixed_small); 0: the bucket's parked ops or its records
// Returns 0 (a bucket that needs the final pass is listed in fin).
template <bool FINAL, bool MIXED, bool FIRST>
__device__ __forceinline__ uint32_t bucket_body(const BucketArgs& a, const uint32_t w,  // w: directory bucket
                                            BucketLds<FINAL, !FINAL && !MIXED>& S,  // the kernel's LDS
                                            uint32_t pre_m = 0) {
  static_assert(!(FINAL && FIRST), "the final pass is never the first");
  // REG: the insert-only apply passes (k_apply / k_apply_parked) keep each
  // op's {key, value, rop} in its owner lane's registers (chunk slot j*64 +
  // lane); LDS holds only the keys.  3 KiB less LDS per wave: 4 waves per
  // SIMD instead of 3.
  constexpr bool REG = !FINAL && !MIXED;
  ulonglong2* const s_kv = S.kv;
  uint64_t* const s_key = S.key;
  uint32_t* const s_op = S.op;
  uint64_t* const s_sk = S.sk;
  uint16_t* const s_pos = S.pos;
  uint16_t* const s_runq = S.runq;
  uint8_t* const s_L = S.L;
  uint8_t* const s_pend = S.pend;
  uint64_t* const s_split = S.split;
  uint32_t* const s_u = S.u;
  uint32_t& s_nsplit = S.nsplit;
  uint32_t& s_nreq = S.nreq;
  uint32_t& s_need = S.need;

  const uint32_t lane = __lane_id() & 63u;  // (not threadIdx.x: callers may run several waves per workgroup)
  const uint32_t pb = w >> a.sbb, sub = w & ((1u << a.sbb) - 1);
  constexpr bool first = FIRST;  // k_apply (mode 0): the batch's records; else parked ops
  uint32_t nw = 0;
  if (!first) {
    nw = (FINAL && pre_m) ? pre_m : a.wl_n[w];
    if (nw == 0 && a.ngrant[w] == 0) return 0u;
    if (!FINAL && nw == kBigBucket) return 0u;  // the final pass takes it (listed by the first pass)
  }
  const bool big = FINAL && nw == kBigBucket;
  ulonglong2* const wl_kv = a.wl_kv + (size_t)w * kCW;
  uint32_t* const wl_op = a.wl_op + (size_t)w * kCW;
  if (first) BK_STAMP(0);
  if (FINAL) BK_STAMP(8);
  if (first && a.mode == 0 && a.clear_next) {  // the next batch's cursors start at zero
    if (sub == 0 && lane < kPartSubs) a.cursor_next[(lane << (a.p1 - a.sbb)) + pb] = 0;
    if (w == 0 && lane == 0) *a.ovf_next = 0;
  }
  if (first && a.mode == 0 && w == 0) clear_other_parity(a);
  // first pass: the first 32 records of each of the bucket's 8 sub-regions
  // and its stat slots are loaded before anything else is known (one round
  // trip with the header and cursor loads instead of three dependent ones)
  constexpr int kPre = 4;  // 4 x 64 = 256 records
  static_assert(kPre * 64 == 32 * kPartSubs, "prefetch: 32 records per sub-region");
  uint32_t pr_op[kPre];
  uint64_t pr_k[kPre], pr_v[kPre];
  const uint64_t rb0 = (uint64_t)pb * a.cap;
  // lane xs (< kPartSubs): sub-region xs's record count
  const uint32_t csub = lane < kPartSubs ? min(a.cursor[(lane << (a.p1 - a.sbb)) + pb], a.capx) : 0u;
  if (first) {
#pragma unroll
    for (int u = 0; u < kPre; ++u) {
      const uint32_t jj = (uint32_t)u * 64u + lane;  // sub-region jj / 32, record jj % 32
      const uint64_t j = rb0 + (uint64_t)(jj >> 5) * a.capx + min(jj & 31u, a.capx - 1u);
      pr_op[u] = a.rop[j];
      const ulonglong2 kv = a.rkv[j];
      pr_k[u] = kv.x;
      pr_v[u] = kv.y;
    }
  }
  const uint64_t wsv = lane < 7u ? a.wstat[(size_t)w * kWStat + lane] : 0ULL;
  uint32_t off, db;
  {
    const uint64_t hd = a.hdr[w];
    off = hdr_off(hd);
    db = hdr_db(hd);
  }
  uint32_t c_runs = 0, c_rounds = 0, c_waited = 0, c_lines = 0, c_splits = 0, c_loss = 0;
  uint32_t c_grow = 0, c_maxr = 0, c_bad = 0, my_max_ld = 0;
  if (!first) commit_splits(a, w, off, db, c_splits, c_grow, my_max_ld);
  const uint32_t C = a.chunk;
  const uint32_t full = FINAL ? 0u : a.ctl->full;
  // apply pass: a small sub-directory is read once into LDS (alongside the
  // record loads) instead of one dependent global load per op
  bool ldir = !FINAL && (1u << db) <= kLdsDir;
  uint32_t dirv0 = 0, dirv1 = 0;
  bool dirw = false;  // S.dir written
  if constexpr (!FINAL) {
    // loaded now, written to LDS at first use: the loads (which wait for the
    // header) overlap the record loads' wait and the hashing
    if (ldir) {
      if (lane < (1u << db)) dirv0 = ld_u32_l2(a.pool + off + lane);
      if (lane + 64u < (1u << db)) dirv1 = ld_u32_l2(a.pool + off + lane + 64u);
    }
  }
  if (lane == 0) {
    s_nsplit = 0;
    s_nreq = 0;
    s_need = db;
  }
  __builtin_amdgcn_wave_barrier();
  uint32_t cmax = csub;  // the largest sub-region count (the prefetch covers 32 of each)
#pragma unroll
  for (int o = 4; o > 0; o >>= 1) cmax = max(cmax, (uint32_t)__shfl_xor((int)cmax, o));
  cmax = (uint32_t)__shfl((int)cmax, 0);
  const uint32_t novf = *a.ovf;
  const uint32_t ntile = (uint32_t)((a.n + kPartTile - 1) / kPartTile);
  BigLds* BL = nullptr;
  uint32_t bt = 0, bmp = 0;  // big bucket walk position
  if constexpr (FINAL) {
    if (big) {
      BL = big_lds();
      big_index(a, BL, pb, csub, novf, ntile);
    }
  }
  bool first_chunk = true;
  uint64_t rk[kPer], rv[kPer];  // REG: the ops of chunk slots j*64 + lane
  uint32_t rop[kPer];
  bool rok[kPer];
#pragma unroll
  for (int j = 0; j < kPer; ++j) rok[j] = false;
  while (first || nw != 0) {
    uint32_t m = 0;
    if (first) {
      if (REG && cmax <= 32u && novf == 0) {
        // the prefetched records stay where they were loaded: chunk slot
        // u*64 + lane (sub-region u*2 + lane/32), holes where the record is
        // another sub-bucket's or past the sub-region's count
        const uint32_t sbm = (1u << a.sbb) - 1;
#pragma unroll
        for (int u = 0; u < kPre; ++u) {
          const uint32_t jj = (uint32_t)u * 64u + lane;
          const uint32_t cs = (uint32_t)__shfl((int)csub, (int)(jj >> 5));
          rok[u] = (jj & 31u) < cs && ((pr_op[u] >> 22) & sbm) == sub;
          rk[u] = pr_k[u];
          rv[u] = pr_v[u];
          rop[u] = pr_op[u];
          m += (uint32_t)__popcll(__ballot(rok[u]));
        }
      } else if (REG) {
        // collect compacts into the (still unused) sort scratch and sort
        // keys (contiguous: kCW pairs), the rop words into the key array,
        // then every lane takes chunk slots j*64 + lane into registers
        ulonglong2* stg = reinterpret_cast<ulonglong2*>(s_u);
        uint32_t* sop = reinterpret_cast<uint32_t*>(s_key);
        m = collect(a, pb, sub, csub, novf, stg, sop);
        if (m <= C) {
#pragma unroll
          for (int j = 0; j < kPer; ++j) {
            const uint32_t i = (uint32_t)j * 64u + lane;
            rok[j] = i < m;
            if (rok[j]) {
              const ulonglong2 kv = stg[i];
              rk[j] = kv.x;
              rv[j] = kv.y;
              rop[j] = sop[i];
            }
          }
        }
        __builtin_amdgcn_wave_barrier();
      } else if (cmax <= 32u && novf == 0) {
        const uint64_t lt = (1ULL << lane) - 1;
        const uint32_t sbm = (1u << a.sbb) - 1;
        m = 0;
#pragma unroll
        for (int u = 0; u < kPre; ++u) {
          const uint32_t jj = (uint32_t)u * 64u + lane;
          const uint32_t cs = (uint32_t)__shfl((int)csub, (int)(jj >> 5));
          const bool match = (jj & 31u) < cs && ((pr_op[u] >> 22) & sbm) == sub;
          const uint64_t bal = __ballot(match);
          const uint32_t idx = m + (uint32_t)__popcll(bal & lt);
          if (match && idx < (uint32_t)kCW) {
            s_kv[idx] = make_ulonglong2(pr_k[u], pr_v[u]);
            s_op[idx] = pr_op[u];
          }
          m += (uint32_t)__popcll(bal);
        }
      } else {
        m = collect(a, pb, sub, csub, novf, s_kv, s_op);
      }
      if (m > C) {
        if (lane == 0) {
          a.wl_n[w] = kBigBucket;  // too many for one chunk: final pass
          a.fin[(a.par << a.p1) + atomicAdd(&a.ctl->nfin[a.par], 1u)] = w;
        }
        return 0;
      }
    } else if (!big) {
      m = nw;
      if constexpr (REG) {
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
          const uint32_t i = (uint32_t)j * 64u + lane;
          rok[j] = i < m;
          if (rok[j]) {
            const ulonglong2 kv = wl_kv[i];
            rk[j] = kv.x;
            rv[j] = kv.y;
            rop[j] = wl_op[i];
          }
        }
      } else if (!(FINAL && pre_m)) {
        for (uint32_t i = lane; i < m; i += 64) {
          s_kv[i] = wl_kv[i];
          s_op[i] = wl_op[i];
        }
      }
      __builtin_amdgcn_wave_barrier();
    } else {
      if constexpr (FINAL) m = big_chunk(a, BL, pb, sub, ntile, C, bt, bmp, s_kv, s_op);
      if (m == 0) break;
    }
    if (first_chunk && (FINAL || first)) BK_STAMP(FINAL ? 9 : 1);
    if constexpr (REG) {
#pragma unroll
      for (int j = 0; j < kPer; ++j) {
        const uint32_t i = (uint32_t)j * 64u + lane;
        s_pend[i] = rok[j] ? 1 : 0;
        s_pos[i] = 0xFFFF;
        if (rok[j]) s_key[i] = rk[j];
      }
    } else {
      for (uint32_t i = lane; i < m; i += 64) {
        s_pend[i] = 1;
        s_pos[i] = 0xFFFF;
      }
    }
    __builtin_amdgcn_wave_barrier();
    uint32_t rounds = 0;
    // chunk slot of a lane's j-th op: strided in the apply pass (a half-full
    // chunk leaves whole j-iterations idle, skipped; REG: where the registers
    // hold it), blocked for the 64-bit register sort of the other paths
    const bool strided = REG || (!FINAL && ldir);
    for (uint32_t round = 0; m > 0; ++round) {
      // ---- a. sort keys of the pending ops
      uint64_t kk[kPer];
      uint32_t ro[kPer];
      bool pq[kPer];
      uint32_t cntp = 0;
#pragma unroll
      for (int j = 0; j < kPer; ++j) {
        const uint32_t i = strided ? (uint32_t)j * 64u + lane : kPer * lane + j;
        if constexpr (REG) {
          pq[j] = rok[j] && s_pend[i];
          kk[j] = rk[j];
          ro[j] = rop[j];
        } else {
          pq[j] = i < m && s_pend[i];
          if (pq[j]) {
            kk[j] = s_kv[i].x;
            ro[j] = s_op[i];
          }
        }
        cntp += pq[j];
      }
      uint32_t np;
      uint32_t at = wave_excl_scan(cntp, &np);
      if (np == 0) break;
      if (round >= kRoundGuard) {
        // cannot happen (depth is bounded); fail loudly rather than spin
#pragma unroll
        for (int j = 0; j < kPer; ++j)
          if (pq[j]) {
            a.st[ro[j] & kOpMask] = 6;
            s_pend[strided ? (uint32_t)j * 64u + lane : kPer * lane + j] = 0;
          }
        if (lane == 0) atomicOr(&a.ctl->err, 2u);
        break;
      }
      ++rounds;
      uint32_t e8[kPer], home8[kPer], x8[kPer];
#pragma unroll
      for (int j = 0; j < kPer; ++j)
        if (pq[j]) {
          const uint64_t h = hash64(kk[j]);
          home8[j] = (uint32_t)(h & 0xFF);
          x8[j] = sub_index(h, a.sbits, a.p1, db);
        }
      if constexpr (!FINAL) {
        if (ldir && !dirw) {
          if (lane < (1u << db)) S.dir[lane] = dirv0;
          if (lane + 64u < (1u << db)) S.dir[lane + 64u] = dirv1;
          __builtin_amdgcn_wave_barrier();
          dirw = true;
        }
      }
#pragma unroll
      for (int j = 0; j < kPer; ++j)
        if (pq[j]) {
          if constexpr (!FINAL) e8[j] = ldir ? S.dir[x8[j]] : ld_u32_l2(a.pool + off + x8[j]);
          else e8[j] = ld_u32_l2(a.pool + off + x8[j]);
        }
      if constexpr (REG) {
        // insert-only passes on a sub-directory of <= 32 entries: claims in
        // parallel (fast_claim); false = a segment with too many interacting
        // ops, nothing done yet: the sorted run loop below takes the round
        if ((1u << db) <= kFastBins && !a.upsert) {
          const uint32_t lbase = a.sbits + a.p1;
          // bin: the segment's first sub-index (< 32)
          const auto bin = [&](int j) -> uint32_t { return x8[j] & ~((1u << (db - (de_ld(e8[j]) - lbase))) - 1u); };
          if (fast_claim<kCW, kFastBins>(a, w, s_u, s_key, wl_kv, wl_op, &s_nsplit, &s_nreq, &s_need, rk, rv, rop, pq, e8,
                                         home8, x8, bin, c_runs, c_lines, c_waited,
                              (first && first_chunk && a.stamps) ? a.stamps + (size_t)w * 16 : nullptr))
            break;  // (an apply pass is one round)
        }
      }
      uint32_t nruns;
      // a 128-entry sub-directory (large tables): two bins per lane, and the
      // runs load their own bitmaps
      const bool wide = db > 6;
      const bool pre_bm = !FINAL && ldir && !wide;
      if (!FINAL && ldir) {
        // ---- segment runs without a 64-bit sort: the ops in batch order
        // (32-bit keys op << 8 | slot), then a stable counting sort by the
        // segment's first sub-directory index (< kLdsDir bins)
        uint32_t* hist = s_u;                                  // [128] ops per bin
        uint32_t* cur = s_u + 128;                             // [128] next position of the bin
        uint8_t* xcs = reinterpret_cast<uint8_t*>(s_u + 256);  // [kCW] bin of each slot
        uint32_t* bseg = s_u + 256 + kCW / 4;                  // [128] segment of each bin
        hist[lane] = 0;
        hist[lane + 64] = 0;
        __builtin_amdgcn_wave_barrier();
        const uint32_t lbase = a.sbits + a.p1;
#pragma unroll
        for (int j = 0; j < kPer; ++j)
          if (pq[j]) {
            const uint32_t i = (uint32_t)j * 64u + lane;
            const uint32_t L = de_ld(e8[j]);
            const uint32_t xc = x8[j] & ~((1u << (db - (L - lbase))) - 1u);
            xcs[i] = (uint8_t)xc;
            bseg[xc] = de_seg(e8[j]);
            atomicAdd(&hist[xc], 1u);
            s_sk[i] = sk_make(de_seg(e8[j]), ro[j] & kOpMask, i, home8[j]);  // by slot for now
            s_L[i] = (uint8_t)(L | ((ro[j] & kGetBit) ? 0x80u : 0u));
          }
        uint32_t p2 = 1;
        while (p2 < np) p2 <<= 1;
        __builtin_amdgcn_wave_barrier();
        // each non-empty bin's lane fetches its segment's bitmap now; the
        // loads land while the ops are sorted
        const uint32_t hv = hist[lane], hv2 = wide ? hist[lane + 64] : 0u;
        uint4 pbm[8];
        if (hv && !wide) {
          const uint32_t* og = a.occ + (size_t)bseg[lane] * 32u;
#pragma unroll
          for (int jj = 0; jj < 8; ++jj) pbm[jj] = ld_u4_l2(og + 4 * jj);
        }
        if (first_chunk && round == 0 && first) BK_STAMP(4);
        // batch order without a comparison sort: k_part tiles are 4096
        // consecutive ops, and a bucket holds ~0-2 ops per tile, so a
        // counting sort by the op's tile bin (256 bins) leaves only tiny bins
        // to order by op (insertion sort, one lane per bin)
        uint32_t* th = s_u + 448;     // [256] per-bin counts, then offsets
        uint32_t* o32 = s_u + 704;    // [kCW] keys (op << 8 | slot) in batch order
        static_assert(704 + kCW <= kBmWords, "sort scratch");
        {
          const uint32_t lgn = 32u - (uint32_t)__builtin_clz((uint32_t)max<uint64_t>(a.n - 1, 1));
          const uint32_t tsh = max(12u, lgn > 8u ? lgn - 8u : 0u);
#pragma unroll
          for (int t = 0; t < 4; ++t) th[4 * lane + t] = 0;
          __builtin_amdgcn_wave_barrier();
          uint32_t tb[kPer], tr[kPer];
#pragma unroll
          for (int j = 0; j < kPer; ++j)
            if (pq[j]) {
              tb[j] = min((ro[j] & kOpMask) >> tsh, 255u);
              tr[j] = atomicAdd(&th[tb[j]], 1u);
            }
          __builtin_amdgcn_wave_barrier();
          uint32_t c4[4], s4 = 0;
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            c4[t] = th[4 * lane + t];
            s4 += c4[t];
          }
          uint32_t tot;
          uint32_t ex = wave_excl_scan(s4, &tot);
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            th[4 * lane + t] = ex;
            ex += c4[t];
          }
          __builtin_amdgcn_wave_barrier();
#pragma unroll
          for (int j = 0; j < kPer; ++j)
            if (pq[j]) o32[th[tb[j]] + tr[j]] = ((ro[j] & kOpMask) << 8) | ((uint32_t)j * 64u + lane);
          __builtin_amdgcn_wave_barrier();
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            if (c4[t] < 2) continue;
            const uint32_t b0 = th[4 * lane + t], b1 = b0 + c4[t];
            for (uint32_t x = b0 + 1; x < b1; ++x) {  // insertion sort by (op, slot)
              const uint32_t v = o32[x];
              uint32_t y = x;
              while (y > b0 && o32[y - 1] > v) {
                o32[y] = o32[y - 1];
                --y;
              }
              o32[y] = v;
            }
          }
          __builtin_amdgcn_wave_barrier();
        }
        if (first_chunk && round == 0 && first) BK_STAMP(5);
        uint32_t rx;
        {  // bins: exclusive offsets; the non-empty ones are the runs
          uint32_t tot;
          const uint32_t ex = wave_excl_scan(hv + hv2, &tot);  // bins lane, lane + 64 in turn
          cur[lane] = ex;
          cur[lane + 64] = ex + hv;
          rx = wave_excl_scan((hv ? 1u : 0u) + (hv2 ? 1u : 0u), &nruns);
          if (hv) s_runq[rx] = (uint16_t)ex;
          if (hv2) s_runq[rx + (hv ? 1u : 0u)] = (uint16_t)(ex + hv);
          if (lane == 0) s_runq[nruns] = (uint16_t)np;
        }
        __builtin_amdgcn_wave_barrier();
        const uint64_t lt = (1ULL << lane) - 1;
        uint64_t skv[kPer];
        uint32_t dst[kPer];
#pragma unroll
        for (int j = 0; j < kPer; ++j) {  // positions j*64 + lane, in batch order
          const uint32_t q = (uint32_t)j * 64u + lane;
          const bool valid = q < np;
          const uint32_t i = valid ? (o32[q] & 0xFFu) : 0u;
          const uint32_t v = valid ? xcs[i] : 0u;
          uint64_t M = __ballot(valid);
#pragma unroll
          for (int b = 0; b < 7; ++b) {
            if (b == 6 && !wide) break;
            const bool bit = (v >> b) & 1u;
            const uint64_t bb = __ballot(bit);
            M &= bit ? bb : ~bb;
          }
          const uint32_t base = cur[v];
          dst[j] = base + (uint32_t)__popcll(M & lt);
          skv[j] = valid ? s_sk[i] : 0ULL;
          __builtin_amdgcn_wave_barrier();
          if (valid && lane == 63u - (uint32_t)__builtin_clzll(M)) cur[v] = base + (uint32_t)__popcll(M);
          __builtin_amdgcn_wave_barrier();
        }
#pragma unroll
        for (int j = 0; j < kPer; ++j)
          if ((uint32_t)j * 64u + lane < np) s_sk[dst[j]] = skv[j];
        // run rx's bitmap row (the sort scratch above is dead now)
        if (hv && !wide && rx < (uint32_t)kBmLanes) {
          uint32_t* row = s_u + rx * 33u;
#pragma unroll
          for (int jj = 0; jj < 8; ++jj) {
            row[4 * jj] = pbm[jj].x;
            row[4 * jj + 1] = pbm[jj].y;
            row[4 * jj + 2] = pbm[jj].z;
            row[4 * jj + 3] = pbm[jj].w;
          }
        }
        __builtin_amdgcn_wave_barrier();
      } else {
#pragma unroll
        for (int j = 0; j < kPer; ++j)
          if (pq[j]) {
            const uint32_t i = strided ? (uint32_t)j * 64u + lane : kPer * lane + j;
            s_sk[at++] = sk_make(de_seg(e8[j]), ro[j] & kOpMask, i, home8[j]);
            s_L[i] = (uint8_t)(de_ld(e8[j]) | ((ro[j] & kGetBit) ? 0x80u : 0u));
          }
        uint32_t p2 = 1;
        while (p2 < np) p2 <<= 1;
        __builtin_amdgcn_wave_barrier();
        if (p2 > 1) wave_sort8(s_sk, p2, np);
        // ---- runs: maximal stretches with one segment
        const uint32_t per_q = (np + 63) / 64;
        uint32_t rc = 0;
        for (uint32_t j = 0; j < per_q; ++j) {
          const uint32_t q = lane * per_q + j;
          if (q < np && (q == 0 || sk_seg(s_sk[q]) != sk_seg(s_sk[q - 1]))) ++rc;
        }
        uint32_t rat = wave_excl_scan(rc, &nruns);
        for (uint32_t j = 0; j < per_q; ++j) {
          const uint32_t q = lane * per_q + j;
          if (q < np && (q == 0 || sk_seg(s_sk[q]) != sk_seg(s_sk[q - 1]))) s_runq[rat++] = (uint16_t)q;
        }
        if (lane == 0) s_runq[nruns] = (uint16_t)np;
      }
      if (lane == 0 && FINAL) {
        s_nsplit = 0;
        s_need = db;
      }
      __builtin_amdgcn_wave_barrier();
      if (first_chunk && round == 0 && (FINAL || first)) BK_STAMP(FINAL ? 10 : 2);
      c_runs += lane == 0 ? nruns : 0;
      // ---- b. one lane per run, in batch order.  Insert-only batches only
      // DECIDE slots here (s_pos); the pairs are written by every lane below.
      // Mixed batches store at once: a later Get of the run must see them.
      {
        uint32_t* bm = s_u + (lane % kBmLanes) * 33u;
        const RunCtx rc{a.pairs, a.occ, a.vout, a.st, a.ctl, a.req + (size_t)w * kSplitCap,
                        a.reqop + (size_t)w * kSplitCap, a.mixed, a.max_segments, full, (uint32_t)(!FINAL && a.mode == 2),
                        (!FINAL && first && a.stamps) ? a.stamps + (size_t)w * 16 : nullptr,
                        a.sbits, a.p1, db, a.upsert, (first && a.upsert) ? a.upos : nullptr};
        for (uint32_t r0 = 0; r0 < nruns; r0 += kBmLanes) {
          const uint32_t r = r0 + lane;
          if (lane >= (uint32_t)kBmLanes || r >= nruns) continue;
          const uint2 cw = apply_run<FINAL, MIXED>(rc, s_sk, s_runq[r], s_runq[r + 1], s_L, s_kv, s_key, s_op, s_pos,
                                            s_pend, s_split, &s_nsplit, &s_nreq, &s_need, bm, wl_kv, wl_op,
                                            pre_bm && r < (uint32_t)kBmLanes);
          c_lines += cw.x;
          c_waited += cw.y;
        }
      }
      __builtin_amdgcn_wave_barrier();
      if (first_chunk && round == 0 && !FINAL && first) BK_STAMP(6);
      if constexpr (REG) {
        // ---- b'. each lane writes its own ops' claimed pairs from registers
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
          if (!pq[j]) continue;
          const uint32_t i = (uint32_t)j * 64u + lane;
          const uint32_t pos = s_pos[i];
          if (pos != 0xFFFFu) {
            a.pairs[(size_t)de_seg(e8[j]) * kSlots + pos] = make_ulonglong2(rk[j], rv[j]);
            s_pos[i] = 0xFFFF;
            s_pend[i] = 0;  // (the fast claim loop leaves it set)
          }
        }
      } else if (MIXED && !FINAL) {
        // ---- b'. mixed apply passes: the claims the run loops left unstored
        // (runs that never reached the general loop), with their status
        if (!a.upsert) {
          for (uint32_t q = lane; q < np; q += 64) {
            const uint64_t sk = s_sk[q];
            const uint32_t i = sk_item(sk);
            const uint32_t pos = s_pos[i];
            if (pos != 0xFFFFu) {
              a.pairs[(size_t)sk_seg(sk) * kSlots + pos] = s_kv[i];
              a.st[sk_op(sk)] = 2;  // PMDFC_ST_INSERTED
              s_pos[i] = 0xFFFF;
            }
          }
        }
      } else if (!MIXED) {
        // ---- b'. write the claimed pairs, all lanes (loads first, then stores)
        for (uint32_t q0 = 0; q0 < np; q0 += 256) {
          uint64_t kq[4], vq[4];
          uint32_t aq[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const uint32_t q = q0 + u * 64 + lane;
            aq[u] = 0xFFFFFFFFu;
            if (q < np) {
              const uint64_t sk = s_sk[q];
              const uint32_t i = sk_item(sk);
              const uint32_t pos = s_pos[i];
              if (pos != 0xFFFFu) {
                aq[u] = sk_seg(sk) * kSlots + pos;
                const ulonglong2 kv = s_kv[i];
                kq[u] = kv.x;
                vq[u] = kv.y;
                s_pos[i] = 0xFFFF;
              }
            }
          }
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if (aq[u] != 0xFFFFFFFFu) a.pairs[aq[u]] = make_ulonglong2(kq[u], vq[u]);
        }
      }
      if (FINAL) __builtin_amdgcn_s_waitcnt(0);  // the next round re-reads the segments
      __builtin_amdgcn_wave_barrier();
      if (first_chunk && round == 0 && (FINAL || first)) BK_STAMP(FINAL ? 11 : 3);
      if constexpr (REG) {
        // ---- e. park the ops a full window left pending (s_pend 2): their
        // owner lanes copy them to the bucket's wait list
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
          const uint32_t i = (uint32_t)j * 64u + lane;
          if (pq[j] && s_pend[i] == 2) {
            const uint32_t k = atomicAdd(&s_nsplit, 1u);
            wl_kv[k] = make_ulonglong2(rk[j], rv[j]);
            wl_op[k] = rop[j];
          }
        }
      }
      if (!FINAL) break;  // k_apply: one round; parked ops wait for the split round
      const uint32_t ns = min(s_nsplit, kSplitCap);
      if (ns == 0) continue;  // every pending op resolved (or failed) this round
      // ---- c. deepen the sub-directory if a child needs more bits
      const uint32_t need = s_need;
      if (need > db) {
        const uint32_t size = 1u << need;
        uint32_t no = 0;
        const bool fx = a.pfix && need <= kFixedBits;  // grows in place in its fixed slot
        if (lane == 0 && !fx) no = atomicAdd(&a.ctl->pool_cur, size);
        no = fx ? w * kFixedSlot : (uint32_t)__shfl((int)no, 0);
        if ((uint64_t)no + size > a.pool_cap) {
          // sub-directory pool exhausted: the blocked ops fail (CAPACITY)
          if (lane == 0) atomicOr(&a.ctl->err, 1u);
          for (uint32_t s = lane; s < ns; s += 64) {
            if (s_split[s] == ~0ULL) continue;
            const uint32_t i = (uint32_t)s_split[s] & 0xFFFFu;
            a.st[s_op[i] & kOpMask] = 6;
            s_pend[i] = 0;
          }
          __builtin_amdgcn_wave_barrier();
          continue;
        }
        grow_subdir(a, w, no, need, off, db);
        ++c_grow;
      }
      // ---- d. splits
      for (uint32_t s = 0; s < ns; ++s) {
        const uint64_t e = s_split[s];
        if (e == ~0ULL) continue;  // its child id ran out (CAPACITY)
        const uint32_t i = (uint32_t)e & 0xFFFFu;
        const uint32_t L = (uint32_t)(e >> 16) & 31u;
        const uint32_t c1 = (uint32_t)(e >> 21);
        const uint32_t x = sub_index(hash64(s_kv[i].x), a.sbits, a.p1, db);
        const uint32_t seg = de_seg(ld_u32_l2(a.pool + off + x));
        bool bad = false;
        uint32_t loss = 0;
        if constexpr (FINAL)
          loss = wave_split(a.pairs, a.occ, a.ldep, seg, c1, L, s_u, &bad, nullptr, a.drops, &a.ctl->drop_n,
                            s_op[i] & kOpMask);
        dir_split(a, off, db, x, seg, c1, L);
        __builtin_amdgcn_s_waitcnt(0);
        ++c_splits;
        c_loss += loss;
        c_bad += bad;
        my_max_ld = max(my_max_ld, L + 1);
      }
      __builtin_amdgcn_wave_barrier();
      if (first_chunk && round == 0) BK_STAMP(12);
    }
    c_rounds += rounds;
    c_maxr = max(c_maxr, rounds);
    first_chunk = false;
    if (!big) break;  // one chunk
  }
  uint32_t to_final = 0;
  if (!FINAL) {
    // the last parked-op pass requests nothing: what it parks is the final pass's
    to_final = (a.mode == 2 && s_nsplit) ? 1u : 0u;
    if (lane == 0) {
      a.wl_n[w] = s_nsplit;  // parked ops (0: done)
      if (to_final) a.fin[(a.par << a.p1) + atomicAdd(&a.ctl->nfin[a.par], 1u)] = w;
    }
  }
  if (!FINAL) {
    __builtin_amdgcn_wave_barrier();
    const uint32_t nr = min(s_nreq, kSplitCap);
    if (nr) request_splits(a, w, nr, s_need > db ? s_need : 0u);
  }
  // ---- counters: this bucket's own stat slot (no shared-line atomics: one
  // contended device atomic per wave costs more than the wave's work)
  for (int o = 32; o > 0; o >>= 1) {
    c_lines += (uint32_t)__shfl_down((int)c_lines, o);
    c_waited += (uint32_t)__shfl_down((int)c_waited, o);
  }
  {  // slot k by lane k, from the values prefetched at the start
    const uint32_t s0 = (uint32_t)__shfl((int)c_lines, 0), s1 = (uint32_t)__shfl((int)c_waited, 0);
    const uint32_t s3 = (uint32_t)__shfl((int)c_loss, 0), s4 = (uint32_t)__shfl((int)c_runs, 0);
    const uint32_t add = lane == 0 ? s0 : lane == 1 ? s1 : lane == 2 ? c_splits : lane == 3 ? s3
                       : lane == 4 ? s4 : lane == 5 ? c_rounds : 0u;
    uint64_t* ws = a.wstat + (size_t)w * kWStat;
    if (lane < 6u && add) ws[lane] = wsv + add;
    if (lane == 3u && s3) atomicAdd(&a.ctl->loss_events, 1u);  // never on the hot path: loss is rare
    // slot 6: max rounds (low 16 bits) | max local depth (bits 16-23) | growths << 32
    if (lane == 6u && (c_maxr || my_max_ld || c_grow)) {
      const uint64_t mr = max((uint32_t)(wsv & 0xFFFF), c_maxr);
      const uint64_t ml = max((uint32_t)((wsv >> 16) & 0xFF), my_max_ld);
      ws[6] = mr | (ml << 16) | (((wsv >> 32) + c_grow) << 32);
    }
    if (lane == 0 && c_bad) atomicOr(&a.ctl->err, 4u);
  }
  if (first) BK_STAMP(7);
  if (FINAL) BK_STAMP(13);
  return 0;
}

// insert-only and mixed batches get their own kernels: the run loop of an
// insert-only batch carries no Get / immediate-store paths
__device__ __forceinline__ bool gated_off(const BucketArgs& a) {
  if (a.gate == 0) return false;
  const bool pend = __builtin_nontemporal_load(&a.ctl->pget) == a.gate_tag;
  return a.gate == 1 ? !pend : pend;
}

template <bool MIXED>
__global__ __launch_bounds__(64, 2) void k_apply(BucketArgs a) {
  if (gated_off(a)) return;
  __shared__ BucketLds<false, !MIXED> S;
  if (MIXED && a.mseen && blockIdx.x == 0 && threadIdx.x == 0)
    __hip_atomic_store(a.mseen, a.gate_tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  bucket_body<false, MIXED, true>(a, blockIdx.x, S);
}
// The mixed first pass on a small grid looping over the buckets: launched
// when the host expects it gated off (BucketLaunch::mixed_small), so the exit
// of its few waves is cheap; exact on any grid (the loop needs more registers
// than k_apply's one bucket per wave, hence its own kernel)
__global__ __launch_bounds__(64, 2) void k_apply_mloop(BucketArgs a) {
  if (gated_off(a)) return;
  __shared__ BucketLds<false, false> S;
  if (a.mseen && blockIdx.x == 0 && threadIdx.x == 0)
    __hip_atomic_store(a.mseen, a.gate_tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  for (uint32_t w = blockIdx.x; w < (1u << a.p1); w += gridDim.x) {
    bucket_body<false, true, true>(a, w, S);
    __builtin_amdgcn_wave_barrier();
  }
}
// Hand out what k_split granted (wave 0 of the parked pass): a prefix of the
// requests in shard-major order -- all of them unless the arena or the pool
// ran out (plain stores: no other wave of k_apply_parked reads or allocates
// either counter).
__device__ __forceinline__ void handout(const BucketArgs& a) {
  const GrantScan g = grant_scan(a.gsh, a.par);
  const uint32_t seg0 = a.ctl->nsegs, pool0 = a.ctl->pool_cur;
  uint64_t ns = (uint64_t)seg0 + g.S, np = (uint64_t)pool0 + g.P;
  if (ns > a.max_segments || np > a.pool_cap) {
    ns = seg0;
    np = pool0;
    // rare: walk the buckets in shard-major order.  Segment ids are granted
    // as a prefix (a bucket denied for the pool leaves its ids unused);
    // pool regions too, since their offsets only grow (fixed slots take none)
    for (uint32_t k = 0; k < g.S;) {
      const uint32_t x = split_shard(g, k);
      const uint64_t cpx = g.cp(x);  // (every lane active)
      const uint4 el = a.gsplit[((size_t)a.par * kGShards + x) * a.gcap + (k - g.cs(x))];  // (a bucket's first split)
      const uint32_t nr = el.w & 0xFFu, need = el.w >> 8;
      const uint64_t gs = (uint64_t)seg0 + k + nr;
      if (gs > a.max_segments) break;
      ns = gs;
      if (need && !(a.pfix && need <= kFixedBits)) {
        const uint64_t gp = (uint64_t)pool0 + cpx + el.z + (1ULL << need);
        if (gp <= a.pool_cap) np = max(np, gp);
      }
      k += nr;
    }
  }
  if ((__lane_id() & 63u) == 0) {
    a.ctl->nsegs = (uint32_t)ns;
    a.ctl->pool_cur = (uint32_t)np;
    // the launch-time hint: a system-scope vector store into coherent
    // pinned host memory (the host reads it without a sync)
    if (a.hint) __hip_atomic_store(a.hint, (uint32_t)ns, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// the parked-op passes (mode 1 / 2): the same body under its own name, so
// kernel traces tell the two passes apart
// (over the worklist the grants built: the buckets with split requests)
template <bool MIXED>
__device__ __forceinline__ void parked_pass(const BucketArgs& a, BucketLds<false, !MIXED>& S) {
  const bool req = a.ctl->anyreq[a.par] != 0;
  const bool decl = !MIXED && a.ctl->anydecl[a.par] != 0;
  if (!req && !decl) return;  // no bucket requested a split or was declined: nothing is parked
  const uint32_t na = req ? a.ctl->nact[a.par] : 0u;
  if (req && blockIdx.x == 0) handout(a);
  for (uint32_t k = blockIdx.x; k < na; k += gridDim.x) {
    bucket_body<false, MIXED, false>(a, a.act[k], S);
    __builtin_amdgcn_wave_barrier();
  }
  if constexpr (!MIXED) {
    // the buckets the lean first pass declined, when no k_apply_fb ran for
    // them: their first pass here, after the split round -- buckets are
    // independent, and this pass requests no split (mode 2): what a full
    // window blocks goes to the final pass, which splits inline
    if (decl) {
      for (uint32_t w = blockIdx.x; w < (1u << a.p1); w += gridDim.x) {
        const uint32_t f = a.fbl[w];
        if (!(f & 1u)) continue;
        bucket_body<false, false, true>(a, w, S);
        if (threadIdx.x == 0) a.fbl[w] = f + 1u;  // pending bit off, count + 1
        __builtin_amdgcn_wave_barrier();
      }
    }
  }
}
template <bool MIXED>
__global__ __launch_bounds__(64, 3) void k_apply_parked(BucketArgs a) {
  if (gated_off(a)) return;
  __shared__ BucketLds<false, !MIXED> S;
  parked_pass<MIXED>(a, S);
}
// A gated mixed batch's parked pass as ONE launch (round 6; until then the
// insert-only and the mixed variant were both launched and one exited at
// once): the insert-only body unless k_mixed_get / k_part left a Get pending
// (ar: gate 2), else the mixed body (am: gate 1).  Both bodies fit the
// insert-only one's 3 waves per SIMD; the LDS is the larger of the two.
union ParkedLds {
  BucketLds<false, true> r;
  BucketLds<false, false> m;
};
__global__ __launch_bounds__(64, 3) void k_apply_parked_gated(BucketArgs ar, BucketArgs am) {
  __shared__ ParkedLds U;
  if (!gated_off(ar)) parked_pass<false>(ar, U.r);
  else parked_pass<true>(am, U.m);
}
// (over the buckets the earlier passes left to it)
template <bool MIXED>
__global__ __launch_bounds__(64, 1) void k_bucket(BucketArgs a) {
  __shared__ BucketLds<true, false> S;
  const uint32_t nf = a.ctl->nfin[a.par];
  for (uint32_t k = blockIdx.x; k < nf; k += gridDim.x) {
    bucket_body<true, MIXED, false>(a, a.fin[(a.par << a.p1) + k], S);
    __builtin_amdgcn_wave_barrier();
  }
}

// ------------------------------------------------------------- small batches
//
// k_mixed_small: a whole mixed (or insert-only: ops == null) batch of at most
// kCW ops in ONE launch, for the per-op front-end (host/batch_core.cpp: the
// reference's 32 poll threads calling KV::Insert / Get one op at a time,
// server/rdma_svr.cpp:755, batches of ~14-32 ops).  The general pipeline
// costs ~12 dependent launches per batch however small it is; here every
// block ranks the batch's ops by (directory bucket, batch index) itself and
// takes the blockIdx-th distinct bucket (blocks past the last one exit), so
// no partition pass and no grid-wide step is needed: the bucket's ops, in
// batch order, go straight into the final pass's LDS chunk and bucket_body's
// final pass applies them -- one round per split, splits and sub-directory
// growth inline -- with every Get answered in its segment's ordered run.  So
// results are the serial reference's exactly (no early answers, no
// SPLIT_LOST).  The inputs may be host-mapped (pinned) memory: a block reads
// the keys once for the ranking and its own ops' values.
__global__ __launch_bounds__(64, 1) void k_mixed_small(BucketArgs a, const uint8_t* __restrict__ ops,
                                                       const uint64_t* __restrict__ keys,
                                                       const uint64_t* __restrict__ vin) {
  __shared__ BucketLds<true, false> S;
  __shared__ uint32_t s_rank[kCW];  // (bucket << 8 | op) of the valid ops, ascending
  __shared__ uint32_t s_sel[2];     // this block's bucket, its first rank position
  const uint32_t lane = threadIdx.x, n = (uint32_t)a.n;
  static_assert(kCW <= 256, "op index in 8 bits");
  uint32_t v[kPer];
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    const uint32_t i = kPer * lane + q;  // wave_sort32's layout
    v[q] = ~0u;
    if (i < n) {
      const uint64_t key = keys[i];
      const uint64_t h = hash64(key);
      const uint8_t bad = reserved_key(key) ? 3 : wrong_shard(h, a.sbits, a.shard) ? 8 : 0;
      if (bad) {
        if (blockIdx.x == 0) {
          a.st[i] = bad;  // PMDFC_ST_RESERVED_KEY / PMDFC_ST_WRONG_SHARD
          if (a.vout) a.vout[i] = 0;  // (insert-only batches pass none)
        }
      } else {
        v[q] = (bucket_of(h, a.sbits, a.p1) << 8) | i;
      }
    }
  }
  wave_sort32<kPer>(v, kCW);
  // distinct buckets in ascending order; this block takes the blockIdx-th
  uint32_t starts = 0;
  const uint32_t prev_last = (uint32_t)__shfl_up((int)v[kPer - 1], 1);
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    const uint32_t pv = q ? v[q - 1] : (lane ? prev_last : ~0u);
    const bool st = v[q] != ~0u && (pv == ~0u || (pv >> 8) != (v[q] >> 8));
    starts |= st ? 1u << q : 0u;
    s_rank[kPer * lane + q] = v[q];
  }
  uint32_t tot;
  const uint32_t rk0 = wave_excl_scan((uint32_t)__builtin_popcount(starts), &tot);
  if (lane == 0) s_sel[0] = ~0u;
  __builtin_amdgcn_wave_barrier();
  if (blockIdx.x >= tot) return;
  {
    uint32_t r = rk0;
#pragma unroll
    for (int q = 0; q < kPer; ++q)
      if ((starts >> q) & 1u) {
        if (r == blockIdx.x) {
          s_sel[0] = v[q] >> 8;
          s_sel[1] = kPer * lane + q;
        }
        ++r;
      }
  }
  __builtin_amdgcn_wave_barrier();
  const uint32_t w = s_sel[0], e0 = s_sel[1];
  // the bucket's ops, in batch order, into the final pass's chunk
  uint32_t m = 0;
  for (uint32_t t0 = 0; e0 + t0 < kCW; t0 += 64) {
    const uint32_t t = t0 + lane;
    const uint32_t e = e0 + t < kCW ? s_rank[e0 + t] : ~0u;
    const bool mine = e != ~0u && (e >> 8) == w;
    const uint64_t bal = __ballot(mine);
    m += (uint32_t)__popcll(bal);
    if (mine) {
      const uint32_t i = e & 0xFFu;
      const bool ins = !ops || ops[i] == 1;  // PMDFC_OP_INSERT
      S.kv[t] = make_ulonglong2(keys[i], ins ? vin[i] : 0ULL);
      S.op[t] = i | (ins ? 0u : kGetBit);
      if (ins && a.vout) a.vout[i] = 0;
    }
    if (bal != ~0ULL) break;  // past the bucket
  }
  __builtin_amdgcn_wave_barrier();
  bucket_body<true, true, false>(a, w, S, m);
}

// k_mixed_tiny: a batch of at most 64 ops (the blocking front-end's usual
// 14-32) by ONE wave, a lane per op in batch order.  An op that is the only
// one of the batch on its segment is applied on its own lane at once: a Get
// probes the window (nothing of this batch changes that segment), an Insert
// takes the first free slot of its window -- exactly what the serial
// reference does, since nothing else of the batch touches the segment and a
// split of another segment never moves it.  The rest -- ops sharing a segment,
// an Insert whose window is full (it splits), every Insert in upsert mode --
// go through the final pass's ordered runs (bucket_body), one directory
// bucket at a time, in batch order within each: the same exact path as
// k_mixed_small.  Common case: key -> header -> sub-directory entry ->
// occupancy words or window line -> store, four dependent round trips in all.
// (the body, also the serving kernel's: lane i holds op i of the n <= 64 in
// registers; results go to a.st[i], a.vout[i])
// hdr_cache (nullable): the directory bucket headers in LDS (the serving
// wave's copy); returns whether the ordered path ran (it may have changed
// headers: the copy is stale then)
__device__ __forceinline__ bool tiny_batch(const BucketArgs& a, BucketLds<true, false>& S, uint32_t n, bool in,
                                           uint64_t key, bool ins, uint64_t val,
                                           const uint64_t* hdr_cache = nullptr) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t h = hash64(key);
  bool live = false;
  if (in) {
    const uint8_t bad = reserved_key(key) ? 3 : wrong_shard(h, a.sbits, a.shard) ? 8 : 0;
    if (bad) {
      a.st[lane] = bad;  // PMDFC_ST_RESERVED_KEY / PMDFC_ST_WRONG_SHARD
      if (a.vout) a.vout[lane] = 0;
    }
    live = !bad;
  }
  const uint32_t w = live ? bucket_of(h, a.sbits, a.p1) : 0u;
  uint32_t e = 0;
  if (live) {
    const uint64_t hd = hdr_cache ? hdr_cache[w] : a.hdr[w];
    e = ld_u32_l2(a.pool + hdr_off(hd) + sub_index(h, a.sbits, a.p1, hdr_db(hd)));
  }
  const uint32_t seg = de_seg(e);
  // another live op of the batch on my segment?
  const uint64_t lv = __ballot(live);
  bool shared = false;
  for (uint64_t m = lv; m; m &= m - 1) {
    const int j = __builtin_ctzll(m);
    const uint32_t sj = (uint32_t)__shfl((int)seg, j);  // (every lane: a shuffle reads active lanes only)
    shared |= (uint32_t)j != lane && sj == seg;
  }
  bool general = live && (shared || (ins && a.upsert));
  if (live && !general) {
    ulonglong2* sp = a.pairs + (size_t)seg * kSlots;
    if (!ins) {
      uint64_t v = 0;
      const uint8_t st = lane_probe(sp, key, h, &v);
      a.vout[lane] = v;
      a.st[lane] = st;
    } else {
      const uint32_t wi0 = (uint32_t)(h & 0xFF) * 4u, wi = wi0 >> 5, wn = (wi + 1u) & 31u;
      uint32_t* og = a.occ + (size_t)seg * 32u;
      const uint32_t lo = ld_u32_l2(og + wi), hi = ld_u32_l2(og + wn);
      const int pos = window_first_free(lo, hi, wi0);
      if (pos < 0) {
        general = true;  // full window: the ordered path splits
      } else {
        sp[pos] = make_ulonglong2(key, val);
        const uint32_t pw = (uint32_t)pos >> 5;
        og[pw] = (pw == wi ? lo : hi) | (1u << ((uint32_t)pos & 31u));
        a.st[lane] = 2;  // PMDFC_ST_INSERTED
        if (a.vout) a.vout[lane] = 0;
      }
    }
  }
  // the rest, bucket by bucket, in batch order within each
  const bool any_general = __ballot(general) != 0;
  for (uint64_t gm = __ballot(general); gm;) {
    const uint32_t wb = (uint32_t)__shfl((int)w, __builtin_ctzll(gm));
    const uint64_t mine = __ballot(general && w == wb);
    if (general && w == wb) {
      const uint32_t t = (uint32_t)__popcll(mine & ((1ULL << lane) - 1));
      S.kv[t] = make_ulonglong2(key, val);
      S.op[t] = lane | (ins ? 0u : kGetBit);
      if (ins && a.vout) a.vout[lane] = 0;
    }
    __builtin_amdgcn_s_waitcnt(0);  // (the direct stores land before the bucket's runs read)
    __builtin_amdgcn_wave_barrier();
    bucket_body<true, true, false>(a, wb, S, (uint32_t)__popcll(mine));
    __builtin_amdgcn_wave_barrier();
    gm &= ~mine;
  }
  return any_general;
}

__global__ __launch_bounds__(64, 1) void k_mixed_tiny(BucketArgs a, const uint8_t* __restrict__ ops,
                                                      const uint64_t* __restrict__ keys,
                                                      const uint64_t* __restrict__ vin) {
  __shared__ BucketLds<true, false> S;
  const uint32_t lane = threadIdx.x, n = (uint32_t)a.n;
  const bool in = lane < n;
  const uint64_t key = in ? keys[lane] : kInvalid;
  const bool ins = in && (!ops || ops[lane] == 1);  // PMDFC_OP_INSERT
  const uint64_t val = ins ? vin[lane] : 0ULL;
  tiny_batch(a, S, n, in, key, ins, val);
}

// ------------------------------------------------------------ serving kernel
//
// k_serve: the per-op front-end's device side (host/batch_core.cpp, served
// mode).  The server's caller threads (up to 32 RDMA poll threads calling
// KV::Insert / Get one op at a time, server/rdma_svr.cpp:755-835) publish
// their ops straight into a ring in coherent pinned host memory; ONE
// persistent wave takes the longest published prefix (at most 64 ops)
// in ring order, applies it exactly as k_mixed_tiny does (the serial
// reference, every Get in its ordered run), bumps the attached counting
// bloom filter for the inserts that count (KV::Insert's bf->Insert,
// server/KV.cpp:113-114), and writes each op's {value, status, sequence
// word} into the response ring: the caller that spins on that word reads its
// result without any host thread in between -- no launch, no completion
// event, no wake-up.
// After ~1 ms without ops it raises ctl->idle (and lowers it when ops come
// again): the host then stops it, so a device-wide synchronisation elsewhere
// in the process never waits on an idle wave.  It exits when the host sets
// ctl->stop, or when the host's heartbeat word has not moved for ~1 s (a host
// that died must not leave a spinning wave); either way it clears ctl->alive
// last.
__device__ __forceinline__ uint32_t sys_ld32(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t sys_ld64(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void sys_st32(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void sys_st64(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(64, 1) void k_serve(ServeArgs sa) {
  __shared__ BucketLds<true, false> S;
  const uint32_t lane = threadIdx.x;
  const uint64_t mask = sa.ring_size - 1;
  // several waves: wave w serves ring w, whose ops all fall in the directory
  // buckets with the top log2(nwaves) bucket bits == w (the host routes each
  // op by its hash): no two waves touch one segment, a sub-directory or a
  // header (splits take their ids and pool regions with atomics)
  if (sa.nwaves > 1) {
    sa.req += (size_t)blockIdx.x * sa.ring_size;
    sa.resp += (size_t)blockIdx.x * sa.ring_size;
    sa.ctl += blockIdx.x;
    sa.head0 = sys_ld64(&sa.ctl->head);
  }
  uint64_t head = sa.head0, chunks = 0, reloads = 0;
  uint64_t hb = sys_ld64(&sa.ctl->heartbeat);
  uint64_t t_hb = (uint64_t)wall_clock64(), t_last = t_hb;
  bool idle_set = false;
  uint64_t tp[5] = {0, 0, 0, 0, 0};  // ticks: read, count BF, apply, answer; empty polls
  const uint64_t t_start = t_hb;
  // head, chunks and the profile every 64 chunks and at exit (the host reads
  // head only to restart a wave that stopped)
  const auto put_prof = [&] {
    const uint64_t life = (uint64_t)wall_clock64() - t_start;
    if (lane < 6)
      sys_st64(&sa.ctl->prof[lane],
               lane == 0 ? tp[0] : lane == 1 ? tp[1] : lane == 2 ? tp[2] : lane == 3 ? tp[3] : lane == 4 ? tp[4] : life);
    if (lane == 6) sys_st64(&sa.ctl->head, head);
    if (lane == 7) sys_st64(&sa.ctl->chunks, chunks);
    if (lane == 8) sys_st64(&sa.ctl->reloads, reloads);
  };
  // results are staged in LDS (no device-memory round trip to read them back)
  __shared__ uint8_t s_st[64];
  __shared__ uint64_t s_vout[64];
  BucketArgs ab = sa.a;
  ab.st = s_st;
  ab.vout = s_vout;
  // the directory bucket headers in LDS (one dependent round trip less per
  // op), reloaded after a chunk whose ordered path may have changed them
  __shared__ uint64_t s_hdr[kServeHdrMax];
  const uint32_t nhdr = 1u << ab.p1;
  const uint64_t* hc = nhdr <= kServeHdrMax ? s_hdr : nullptr;
  const auto load_hdr = [&] {
    for (uint32_t b = lane; b < nhdr; b += 64u) s_hdr[b] = ab.hdr[b];
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
  };
  if (hc) load_hdr();
  bool hdr_stale = false;
  // the request ring through a buffer resource: 16-B loads at system scope
  // (sc0 sc1), both halves of 64 places and the stop word in one round trip
  const __amdgpu_buffer_rsrc_t rq =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<pmdfc_serve_req*>(sa.req), 0, 0x7fffffff, 0x00020000);
  u32x4_t qlo, qhi;
  uint32_t stop;
  const auto poll = [&](uint64_t h) {
    const uint32_t off = (uint32_t)(((h + lane) & mask) * sizeof(pmdfc_serve_req));
    stop = sys_ld32(&sa.ctl->stop);
    qlo = __builtin_amdgcn_raw_buffer_load_b128(rq, off, 0, 0x11);
    qhi = __builtin_amdgcn_raw_buffer_load_b128(rq, off + 16u, 0, 0x11);
  };
  poll(head);
  for (uint32_t idle = 0;;) {
    if (stop) break;
    const uint64_t p = head + lane;
    const uint32_t want = ((uint32_t)p + 1u) & 0x3FFFFFFFu;
    const bool ready = qlo.z == qhi.z && (qlo.z >> 2) == want;  // both halves of place p written
    const uint64_t rb = __ballot(ready);
    const uint32_t n = ~rb ? (uint32_t)__builtin_ctzll(~rb) : 64u;  // the published prefix
    if (n == 0) {
      ++tp[4];
      // idle: back off; every 64 polls check that the host still beats
      if ((++idle & 63u) == 0) {
        const uint64_t h2 = sys_ld64(&sa.ctl->heartbeat), now = (uint64_t)wall_clock64();
        if (h2 != hb) {
          hb = h2;
          t_hb = now;
        } else if (now - t_hb > kServeWatchdog) {
          break;
        }
        if (!idle_set && now - t_last > kServeIdle) {
          idle_set = true;
          if (lane == 0) sys_st32(&sa.ctl->idle, 1u);
        }
      }
      __builtin_amdgcn_s_sleep(4);
      poll(head);
      continue;
    }
    idle = 0;
    const uint64_t c0 = (uint64_t)wall_clock64();
    t_last = c0;
    if (idle_set) {
      idle_set = false;
      if (lane == 0) sys_st32(&sa.ctl->idle, 0u);
    }
    const bool in = lane < n;
    const uint64_t key = in ? ((uint64_t)qlo.y << 32) | qlo.x : kInvalid;
    const uint32_t op = in ? qlo.z & 3u : 0u;
    const bool ins = in && (op & 1u) == PMDFC_SERVE_INSERT;
    const uint64_t val = ins ? ((uint64_t)qhi.y << 32) | qhi.x : 0ULL;
    const uint64_t c1 = c0;
    // the earlier chunks rewrote table lines this CU may hold in its L1 (the
    // headers are read with plain loads): an acquire at agent scope drops them
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    if (hc && hdr_stale) {
      load_hdr();
      ++reloads;
    }
    if (sa.cbf && ins && (op & PMDFC_SERVE_CBF)) cbf_increment(sa.cbf, sa.cbf_m, sa.cbf_k, key);
    __builtin_amdgcn_s_waitcnt(0);
    const uint64_t c2 = (uint64_t)wall_clock64();
    hdr_stale = tiny_batch(ab, S, n, in, key, ins, val, hc);
    // the results in LDS (not the table stores: they complete under the next
    // poll, which the release below waits for anyway; this wave's later loads
    // of the same lines are ordered behind them)
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0) only (gfx9 encoding)
    __builtin_amdgcn_wave_barrier();
    const uint64_t c3 = (uint64_t)wall_clock64();
    // each answer is ONE 16-B store {value, status | seq << 32} (one bus
    // write per op)
    if (in) {
      const uint8_t st = s_st[lane];
      const uint64_t v = !ins && st == 1 ? s_vout[lane] : 0ULL;
      const u64x2_t w = {v, (uint64_t)st | ((uint64_t)(uint32_t)(p + 1) << 32)};
      __builtin_nontemporal_store(w, reinterpret_cast<u64x2_t*>(sa.resp + (p & mask)));
    }
    head += n;
    ++chunks;
    // the next chunk's poll travels with the answers (the release below waits
    // for both)
    poll(head);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // (system scope: the answers leave now)
    const uint64_t c4 = (uint64_t)wall_clock64();
    tp[0] += c1 - c0;
    tp[1] += c2 - c1;
    tp[2] += c3 - c2;
    tp[3] += c4 - c3;
    if ((chunks & 63u) == 0) put_prof();
  }
  put_prof();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  if (lane == 0) sys_st32(&sa.ctl->alive, 0u);
}

// k_medium: a mixed / insert batch of at most kPartTile ops after its
// one-block partition: block i takes the i-th partition bucket that received
// ops (blocks past the last exit) and runs each of its directory buckets
// through the final pass with every record walked in batch order (the
// oversized-bucket walk of bucket_body: chunks of whole tiles, here the one
// tile) -- rounds with inline splits, Gets answered in their ordered runs, so
// the serial reference's results exactly.  Two launches per batch instead of
// the general pipeline's ~12; the async front-end's batches of ~1-4k ops.
// The blocks also zero the other parity's cursors for the next batch.
template <bool MIXED>
__global__ __launch_bounds__(64, 1) void k_medium(BucketArgs a, const uint32_t* __restrict__ touched) {
  __shared__ BucketLds<true, false> S;
  const uint32_t lane = threadIdx.x, npb = 1u << (a.p1 - a.sbb);
  for (uint32_t i = blockIdx.x * 64u + lane; i < npb * kPartSubs; i += gridDim.x * 64u) a.cursor_next[i] = 0;
  if (blockIdx.x == 0 && lane == 0) *a.ovf_next = 0;
  const uint32_t nt = touched[0];
  for (uint32_t k = blockIdx.x; k < nt; k += gridDim.x) {
    const uint32_t pb = touched[1 + k];
    for (uint32_t sub = 0; sub < (1u << a.sbb); ++sub) {
      bucket_body<true, MIXED, false>(a, (pb << a.sbb) | sub, S, kBigBucket);
      __builtin_amdgcn_wave_barrier();
    }
  }
}

// ---------------------------------------------------------------- split round
//
// k_split: one wave per entry of the split list the apply pass granted (a
// fixed grid looping over ctl->nsplit[par] entries; denied entries are ~0).
struct SplitArgs {
  uint32_t par;        // the batch's parity: its grant shards
  uint32_t pfix;       // small sub-directories grow in their fixed slots
  uint64_t* stamps;
  const uint64_t* gsh;
  const uint4* gsplit;
  uint32_t gcap;
  uint32_t* act;       // out: the buckets with requests (k_apply_parked's worklist)
  uint32_t* gbase;     // out, per bucket: first child id, grants, pool offset, sub-directory bits
  uint32_t* ngrant;
  uint32_t* newoff;
  uint32_t* need;
  uint32_t max_segments, pool_cap;
  ulonglong2* pairs;
  uint32_t* occ;
  uint8_t* ldep;
  DevCtl* ctl;
  const uint32_t* reqop;  // batch position of each request's insert (drop log)
  ulonglong2* drops;      // the drop log, or null
  uint32_t team_max;      // split lists up to this long go by teams of four waves
};

constexpr uint32_t kSplitWaves = 4;      // waves per k_split workgroup
#ifndef PMDFC_SPLIT_GROUPS
#define PMDFC_SPLIT_GROUPS 512  // (A/B builds; 1024: two dispatch rounds at 2 waves/SIMD, 12.41-12.44 against 12.56 Gops/s)
#endif
constexpr uint32_t kSplitGroups = PMDFC_SPLIT_GROUPS;  // k_split grid (waves loop over the requested splits)
#ifndef PMDFC_SPLIT_GROUPS_RAMP
#define PMDFC_SPLIT_GROUPS_RAMP 1024
#endif
constexpr uint32_t kSplitGroupsRamp = PMDFC_SPLIT_GROUPS_RAMP;  // ... while the table ramps (p1 < p1max)

// One wave per requested split, in shard-major order: split k is request i of
// bucket w; its child id is the segment counter at the start of the pass + k
// (the shards' segment offsets are exactly the prefix sums of the requests)
// and the bucket's grown sub-directory, if any, sits at the pool counter + the
// pools of the shards before + its offset in its shard.  A bucket whose
// requests do not fit max_segments / the pool is denied whole (ctl->full: the
// parked pass fails its ops with CAPACITY); both offsets only grow in
// shard-major order, so the grants are a prefix (k_apply_parked then sets the
// counters).  The wave of a bucket's first request also grants it and lists
// it for the parked pass.
__global__ __launch_bounds__(64 * kSplitWaves, 2) void k_split(SplitArgs a) {
  if (a.ctl->anyreq[a.par] == 0) return;
  __shared__ uint32_t s_scr[kSplitWaves][kSplitScratch];
  const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const GrantScan g = grant_scan(a.gsh, a.par);
  const uint32_t seg0 = a.ctl->nsegs, pool0 = a.ctl->pool_cur;
  if (blockIdx.x == 0 && threadIdx.x == 0) a.ctl->nact[a.par] = g.E;
  // a short split list (by default at most one split per workgroup): the
  // workgroup's four waves split together (split_team<4>: a quarter of the
  // loads and stores each), else one wave per split
  const bool team = g.S <= a.team_max;
  uint32_t loss = 0, bad = 0;
  const uint32_t k0 = team ? blockIdx.x : blockIdx.x * kSplitWaves + wv;
  const uint32_t ks = team ? gridDim.x : gridDim.x * kSplitWaves;
  for (uint32_t k = k0; k < g.S; k += ks) {
    const uint32_t x = split_shard(g, k);
    // (the cross-lane reads with every lane active)
    const uint32_t csx = g.cs(x), cex = g.ce(x);
    const uint64_t cpx = g.cp(x);
    const uint4 el = a.gsplit[((size_t)a.par * kGShards + x) * a.gcap + (k - csx)];
    const uint32_t w = el.y & 0x3FFFu, i = (el.y >> 14) & 63u, nr = el.w & 0xFFu, need = el.w >> 8;
    const bool fx = a.pfix && need && need <= kFixedBits;  // grows in its fixed slot: no pool
    const uint64_t gs = (uint64_t)seg0 + k - i, gp = fx ? (uint64_t)w * kFixedSlot : (uint64_t)pool0 + cpx + el.z;
    const bool ok = gs + nr <= a.max_segments && (fx || gp + (need ? 1ULL << need : 0ULL) <= a.pool_cap);
    if (i == 0 && lane == 0 && (!team || wv == 0)) {
      a.gbase[w] = (uint32_t)gs;
      a.ngrant[w] = ok ? nr : 0u;
      a.newoff[w] = (uint32_t)gp;
      a.need[w] = need;
      a.act[cex + (el.y >> 20)] = w;
      if (!ok) a.ctl->full = 1;
    }
    if (!ok) continue;  // (uniform over a team: one k)
    bool b = false;
    uint64_t* stp = a.stamps && k < kSplitStamps ? a.stamps + (size_t)k * 8 : nullptr;
    if (stp && lane == 0 && (!team || wv == 0)) stp[5] = wall_clock64();
    const uint32_t trig = a.drops ? a.reqop[(size_t)w * kSplitCap + i] : 0u;
    const uint32_t ps = el.x & ((1u << 27) - 1), pl = el.x >> 27;
    if (team) {
      loss += split_team<4>(a.pairs, a.occ, a.ldep, ps, seg0 + k, pl, &s_scr[0][0], &b, stp, a.drops, &a.ctl->drop_n,
                            trig, wv);
    } else {
      // an opaque scratch offset per iteration: otherwise the split's LDS
      // addresses are hoisted out of the loop into ~60 VGPRs
      uint32_t so = wv * kSplitScratch;
      __asm__ volatile("" : "+v"(so));
      loss += wave_split(a.pairs, a.occ, a.ldep, ps, seg0 + k, pl, &s_scr[0][0] + so, &b, stp, a.drops,
                         &a.ctl->drop_n, trig);
    }
    bad |= b;
  }
  if (lane == 0 && (!team || wv == 0)) {  // (a team's total is on every wave: wave 0 reports it)
    if (loss) {
      atomicAdd(reinterpret_cast<unsigned long long*>(&a.ctl->split_loss), (unsigned long long)loss);
      atomicAdd(&a.ctl->loss_events, 1u);
    }
    if (bad) atomicOr(&a.ctl->err, 4u);
  }
}

// ---------------------------------------------------- lean first apply pass
//
// k_apply_fast: the first pass of an insert-only batch for the common bucket
// -- at most 64 records per sub-region (32 prefetched), no overflow, at most
// kFC inserts, a sub-directory of <= kFastBins entries -- with the parallel
// claims of fast_claim (see there for the rule and why it is exact), in a
// kernel of its own sized for OCCUPANCY: the pass is a chain of dependent
// memory round trips (records + header + fixed sub-directory slot, then each
// insert's two occupancy words, then the claims' stores) with ~6 % VALU busy,
// so its time is waves in flight.  Dense insert slots (the records compacted
// through LDS, kFP per lane), the sub-directory in a register (a shuffle per
// lookup), occupancy words straight from memory and claimed bits OR-ed back
// with global atomics (no bitmap rows in LDS), no key array (the rare
// UNSPLITTABLE check that needs a key claimed in this pass hands the bucket
// back): ~4.9 KB of LDS and no general path in the kernel, so 8 waves per SIMD
// instead of 4.  A bucket it does not take -- or whose claims hit a case
// fast_claim hands back -- is listed (nothing written yet) for k_apply_fb,
// bucket_body's general first pass, launched right after.
// The wide variant (k_apply_wide) takes the buckets of large tables -- a
// sub-directory of up to 128 entries (a 2^28-key table at 2^13 buckets has
// 64-128), read from its fixed slot in the first round trip (two entries
// per lane), at most kFCW inserts -- with the bins of fast_claim assigned
// densely to the segments the bucket's inserts touch (at most 64), and
// fewer insert slots per lane: 6.7 KB of LDS, 6 waves per SIMD.
template <bool WIDE>
struct FastCfg {
  static constexpr int FP = WIDE ? 2 : 3;               // dense insert slots per lane
  static constexpr uint32_t FC = 64u * (uint32_t)FP;    // inserts per bucket on the fast path
  static constexpr uint32_t NB = WIDE ? 64u : kFastBins; // segments (bins) per bucket
  static constexpr uint32_t MaxDb = WIDE ? 7u : 5u;     // sub-directory bits it takes
};

template <bool WIDE>
struct FastLds {
  using C = FastCfg<WIDE>;
  union {
    uint32_t sc[FcLayout<C::FC, C::NB>::Words];  // fast_claim's scratch
    struct {
      ulonglong2 kv[C::FC];
      uint32_t op[C::FC];
    } stage;  // record compaction (before the claims)
  };
  uint32_t seen[4];  // WIDE: the segments (first sub-index) the inserts touch
  uint32_t nsplit, nreq, need;
};

// 0: taken; else a bucket the fast path does not take (nothing written yet):
// 2 for a table-wide reason (sub-directory past MaxDb bits, partition overflow)
// UPS: last-writer-wins (PMDFC_CFG_UPSERT): a bucket with two inserts of one
// key goes to the general pass; otherwise each insert's window is probed for
// its key over the occupied prefix (a stored key lies before the window's
// first free slot: nothing is deleted) and a stored key is overwritten.
// The coarse-partition first pass (k_apply_fast_cp): k_part partitions into
// 2^(p1 - 3) buckets, each the records of 8 directory buckets, so a tile's run
// per partition bucket is ~8 records (whole 128-B lines, 1/8 of the reserve
// atomics) instead of ~1; the 8 waves of a workgroup -- one per directory
// bucket -- stage their partition bucket's records in LDS once (coalesced,
// kCpPre per sub-region) and each compacts its own from there.  The staging
// overlays the waves' claim scratch (4 workgroups per CU: 8 waves per SIMD).
constexpr uint32_t kCpWaves = 1u << kCpSbb;
constexpr uint32_t kCpPre = 192;  // records staged per sub-region (mean 128 at 1M ops / 1,024 buckets / 8 sub-regions)
struct CpLds {
  union {
    FastLds<false> w[kCpWaves];
    struct {
      ulonglong2 kv[kPartSubs * kCpPre];
      uint32_t op[kPartSubs * kCpPre];
      uint16_t idx[kCpWaves][FastCfg<false>::FC];  // each wave's records: staging slots
    } st;
  };
  uint32_t csub[kPartSubs];
};
static_assert(sizeof(CpLds) <= 40 * 1024, "4 workgroups of 8 waves per CU");

template <bool WIDE, bool UPS = false, bool CP = false>
__device__ __forceinline__ uint32_t apply_fast(const BucketArgs& a, FastLds<WIDE>& S, uint32_t w,
                                               CpLds* cpl = nullptr) {
  using C = FastCfg<WIDE>;
  static_assert(!CP || (!WIDE && !UPS), "the coarse-partition pass is the lean insert-only one");
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t pb = w >> a.sbb, sub = w & ((1u << a.sbb) - 1);
  uint64_t* const stamp = a.stamps ? a.stamps + (size_t)w * 16 : nullptr;
#define FS_STAMP(ph) \
  if (stamp && lane == 0) stamp[ph] = wall_clock64()
  FS_STAMP(0);
  if (a.clear_next) {  // the next batch's cursors start at zero
    if (sub == 0 && lane < kPartSubs) a.cursor_next[(lane << (a.p1 - a.sbb)) + pb] = 0;
    if (w == 0 && lane == 0) *a.ovf_next = 0;
  }
  if (w == 0) clear_other_parity(a);
  // one round trip: the first 32 records of each sub-region, the counts, the
  // header, the stat slots, the overflow count and the fixed sub-directory slot
  uint32_t pr_op[4];
  uint64_t pr_k[4], pr_v[4];
  const uint64_t rb0 = (uint64_t)pb * a.cap;
  constexpr int kCpLd = (int)(kPartSubs * kCpPre / (64 * kCpWaves));  // staging loads per thread
  if constexpr (CP) {
    // the workgroup stages kCpPre records of each sub-region (slot t of the
    // workgroup: sub-region t / kCpPre); a wave's loads land below
#pragma unroll
    for (int u = 0; u < kCpLd; ++u) {
      const uint32_t t = (uint32_t)u * 64u * kCpWaves + threadIdx.x;
      const uint64_t j = rb0 + (uint64_t)(t / kCpPre) * a.capx + min(t % kCpPre, a.capx - 1u);
      pr_op[u] = a.rop[j];
      const ulonglong2 kv = a.rkv[j];
      pr_k[u] = kv.x;
      pr_v[u] = kv.y;
    }
  } else {
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const uint32_t jj = (uint32_t)u * 64u + lane;  // sub-region jj / 32, record jj % 32
    const uint64_t j = rb0 + (uint64_t)(jj >> 5) * a.capx + min(jj & 31u, a.capx - 1u);
    pr_op[u] = a.rop[j];
    const ulonglong2 kv = a.rkv[j];
    pr_k[u] = kv.x;
    pr_v[u] = kv.y;
  }
  }
  const uint32_t csub = lane < kPartSubs ? min(a.cursor[(lane << (a.p1 - a.sbb)) + pb], a.capx) : 0u;
  const uint64_t wsv = lane < 7u ? a.wstat[(size_t)w * kWStat + lane] : 0ULL;
  const uint32_t* fslot = a.pool + (size_t)w * kFixedSlot;
  const uint32_t spec0 = (a.pfix && (WIDE || lane < 32u)) ? ld_u32_l2(fslot + lane) : 0u;
  const uint32_t spec1 = (WIDE && a.pfix) ? ld_u32_l2(fslot + 64u + lane) : 0u;
  const uint64_t hd = a.hdr[w];
  const uint32_t off = hdr_off(hd), db = hdr_db(hd);
  const uint32_t novf = *a.ovf;
  // the sub-directory, one (two) entries per lane (else loads that wait for the header)
  const bool fixed = a.pfix && off == w * kFixedSlot && db <= kFixedBits;
  uint32_t dv0, dv1 = 0u;
  if (fixed) {
    dv0 = lane < (1u << db) ? spec0 : 0u;
    dv1 = lane + 64u < (1u << db) ? spec1 : 0u;
  } else {
    dv0 = (db <= C::MaxDb && lane < (1u << db)) ? ld_u32_l2(a.pool + off + lane) : 0u;
    if (WIDE) dv1 = (db <= C::MaxDb && lane + 64u < (1u << db)) ? ld_u32_l2(a.pool + off + 64u + lane) : 0u;
  }
  uint32_t cmax = csub;
#pragma unroll
  for (int o = 4; o > 0; o >>= 1) cmax = max(cmax, (uint32_t)__shfl_xor((int)cmax, o));
  cmax = (uint32_t)__shfl((int)cmax, 0);
  bool pq[kPer];
  uint64_t rk[kPer], rv[kPer];
  uint32_t rop[kPer];
  if constexpr (CP) {
    // staged records -> LDS; then each wave lists its own (sub-bucket == its
    // bucket) and takes them into insert slots j * 64 + lane; the two
    // workgroup barriers are reached by every wave, declining or not
#pragma unroll
    for (int u = 0; u < kCpLd; ++u) {
      const uint32_t t = (uint32_t)u * 64u * kCpWaves + threadIdx.x;
      cpl->st.op[t] = pr_op[u];
      cpl->st.kv[t] = make_ulonglong2(pr_k[u], pr_v[u]);
    }
    __syncthreads();
    uint32_t dec = (db > C::MaxDb || novf != 0) ? 2u : cmax > kCpPre ? 2u : 0u;
    uint32_t m = 0;
    if (!dec) {
      const uint64_t lt = (1ULL << lane) - 1;
      const uint32_t v = w & (kCpWaves - 1);
      uint16_t* my = cpl->st.idx[v];
#pragma unroll 4
      for (uint32_t c = 0; c < kPartSubs * kCpPre / 64; ++c) {
        const uint32_t t = c * 64u + lane;
        const uint32_t cs = (uint32_t)__shfl((int)csub, (int)(t / kCpPre));
        const uint32_t r = cpl->st.op[t];
        const bool match = t % kCpPre < cs && ((r >> 22) & (kCpWaves - 1)) == v;
        const uint64_t bal = __ballot(match);
        const uint32_t idx = m + (uint32_t)__popcll(bal & lt);
        if (match && idx < C::FC) my[idx] = (uint16_t)t;
        m += (uint32_t)__popcll(bal);
      }
      if (m > C::FC) dec = 1u;
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int j = 0; j < kPer; ++j) {
        const uint32_t i = (uint32_t)j * 64u + lane;
        pq[j] = !dec && j < C::FP && i < m;
        rk[j] = rv[j] = 0;
        rop[j] = 0;
        if (pq[j]) {
          const uint32_t t = my[i];
          const ulonglong2 kv = cpl->st.kv[t];
          rk[j] = kv.x;
          rv[j] = kv.y;
          rop[j] = cpl->st.op[t];
        }
      }
    }
    __syncthreads();  // (the staging is dead: the waves' claim scratch overlays it)
    if (dec) return dec;
  } else {
  if (db > C::MaxDb || novf != 0) return 2u;
  if (cmax > C::FC) return 1u;
  // compact the bucket's records into insert slots j * 64 + lane, j < FP
  // (in sub-region order: records 0-31 of every sub-region, then 32-63 of
  // those with more, ... -- k_part's sub-regions are ~Poisson(16) at config 2,
  // so ~10 buckets a batch take the second load; a batch of fewer than
  // kPartSubs partition tiles fills fewer sub-regions, more deeply.  The order
  // of the slots does not matter, the claims are decided by op index)
  const uint32_t sbm = (1u << a.sbb) - 1;
  const uint64_t lt = (1ULL << lane) - 1;
  uint32_t m = 0;
  for (uint32_t half = 0; half * 32u < cmax; ++half) {
    if (half) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint32_t jj = (uint32_t)u * 64u + lane;
        const uint64_t j = rb0 + (uint64_t)(jj >> 5) * a.capx + min(half * 32u + (jj & 31u), a.capx - 1u);
        pr_op[u] = a.rop[j];
        const ulonglong2 kv = a.rkv[j];
        pr_k[u] = kv.x;
        pr_v[u] = kv.y;
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t jj = (uint32_t)u * 64u + lane;
      const uint32_t cs = (uint32_t)__shfl((int)csub, (int)(jj >> 5));
      const bool match = half * 32u + (jj & 31u) < cs && ((pr_op[u] >> 22) & sbm) == sub;
      const uint64_t bal = __ballot(match);
      const uint32_t idx = m + (uint32_t)__popcll(bal & lt);
      if (match && idx < C::FC) {
        S.stage.kv[idx] = make_ulonglong2(pr_k[u], pr_v[u]);
        S.stage.op[idx] = pr_op[u];
      }
      m += (uint32_t)__popcll(bal);
    }
  }
  if (m > C::FC) return 1u;
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const uint32_t i = (uint32_t)j * 64u + lane;
    pq[j] = j < C::FP && i < m;
    rk[j] = rv[j] = 0;
    rop[j] = 0;
    if (pq[j]) {
      const ulonglong2 kv = S.stage.kv[i];
      rk[j] = kv.x;
      rv[j] = kv.y;
      rop[j] = S.stage.op[i];
    }
  }
  __builtin_amdgcn_wave_barrier();  // (staging is dead: the claims' scratch overlays it)
  }
  if (lane == 0) {
    S.nsplit = 0;
    S.nreq = 0;
    S.need = db;
  }
  if (WIDE && lane < 4) S.seen[lane] = 0;
  uint32_t e8[kPer], home8[kPer], x8[kPer], bn[WIDE ? kPer : 1];
  (void)bn;
  const uint32_t lbase = a.sbits + a.p1;
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    home8[j] = x8[j] = 0;
    if (pq[j]) {
      const uint64_t h = hash64(rk[j]);
      home8[j] = (uint32_t)(h & 0xFF);
      x8[j] = sub_index(h, a.sbits, a.p1, db);
    }
    // (every lane: a shuffle reads active lanes only)
    const uint32_t lo = (uint32_t)__shfl((int)dv0, (int)(x8[j] & 63u));
    if (WIDE) {
      const uint32_t hi = (uint32_t)__shfl((int)dv1, (int)(x8[j] & 63u));
      e8[j] = x8[j] < 64u ? lo : hi;
    } else {
      e8[j] = lo;
    }
  }
  // bin: the segment's first sub-index; WIDE: the touched segments numbered
  // densely in sub-index order
  const auto first_sub = [&](int j) -> uint32_t { return x8[j] & ~((1u << (db - (de_ld(e8[j]) - lbase))) - 1u); };
  if constexpr (WIDE) {
#pragma unroll
    for (int j = 0; j < kPer; ++j) bn[j] = pq[j] ? first_sub(j) : 0u;
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int j = 0; j < kPer; ++j)
      if (pq[j]) atomicOr(&S.seen[bn[j] >> 5], 1u << (bn[j] & 31u));
    __builtin_amdgcn_wave_barrier();
    const uint32_t s0 = S.seen[0], s1 = S.seen[1], s2 = S.seen[2], s3 = S.seen[3];
    if (__builtin_popcount(s0) + __builtin_popcount(s1) + __builtin_popcount(s2) + __builtin_popcount(s3) > (int)C::NB)
      return 1u;  // (nothing written yet)
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const uint32_t x = bn[j], q = x >> 5, below = (1u << (x & 31u)) - 1u;
      uint32_t r = __builtin_popcount((q == 0 ? s0 : q == 1 ? s1 : q == 2 ? s2 : s3) & below);
      r += q > 0 ? __builtin_popcount(s0) : 0;
      r += q > 1 ? __builtin_popcount(s1) : 0;
      r += q > 2 ? __builtin_popcount(s2) : 0;
      bn[j] = r;
    }
  }
  uint32_t upd[UPS ? kPer : 1], occw[UPS ? 2 * kPer : 1];
  if constexpr (UPS) {
    // two inserts of one key: the general pass (equal keys have equal hashes;
    // a 32-bit hash collision only sends the bucket there too)
    uint32_t hv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) hv[q] = q < kPer && pq[q] ? (uint32_t)hash64(rk[q]) : 0xFFFFFFFFu;
    wave_sort32<4>(hv, 256);
    bool dup = false;
#pragma unroll
    for (int q = 0; q < 3; ++q) dup |= hv[q] != 0xFFFFFFFFu && hv[q] == hv[q + 1];
    const uint32_t nx = (uint32_t)__shfl_down((int)hv[0], 1);
    dup |= lane < 63u && hv[3] != 0xFFFFFFFFu && hv[3] == nx;
    if (__ballot(dup)) return 1u;
    // the window's occupancy words, then its occupied prefix, line by line
    // (the loads of all of a lane's inserts in flight together)
    uint32_t nl[kPer];
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      upd[j] = 0xFFFFu;
      occw[2 * j] = occw[2 * j + 1] = 0;
      if (!pq[j]) continue;
      const uint32_t* og = a.occ + (size_t)de_seg(e8[j]) * 32u;
      const uint32_t wi = home8[j] >> 3;
      occw[2 * j] = ld_u32_l2(og + wi);
      occw[2 * j + 1] = ld_u32_l2(og + ((wi + 1u) & 31u));
    }
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const uint32_t win = __builtin_amdgcn_alignbit(occw[2 * j + 1], occw[2 * j], (home8[j] * 4u) & 31u);
      const uint32_t ff = ~win ? (uint32_t)__builtin_ctz(~win) : 32u;  // first free slot of the window
      nl[j] = pq[j] ? (ff + 3u) >> 2 : 0u;
    }
    for (uint32_t t = 0;; ++t) {
      bool more = false;
#pragma unroll
      for (int j = 0; j < kPer; ++j) more |= t < nl[j] && upd[j] == 0xFFFFu;
      if (!__ballot(more)) break;
      uint64_t kq[kPer][4];
#pragma unroll
      for (int j = 0; j < kPer; ++j) {
        if (t >= nl[j] || upd[j] != 0xFFFFu) continue;
        const ulonglong2* ln = a.pairs + (size_t)de_seg(e8[j]) * kSlots + ((home8[j] + t) & 255u) * 4u;
#pragma unroll
        for (int q = 0; q < 4; ++q) kq[j][q] = reinterpret_cast<const uint64_t*>(ln + q)[0];
      }
#pragma unroll
      for (int j = 0; j < kPer; ++j) {
        if (t >= nl[j] || upd[j] != 0xFFFFu) continue;
#pragma unroll
        for (int q = 3; q >= 0; --q)
          if (kq[j][q] == rk[j]) upd[j] = ((home8[j] + t) * 4u + (uint32_t)q) & (kSlots - 1);
      }
    }
  }
  FS_STAMP(1);
  uint32_t c_runs = 0, c_lines = 0, c_waited = 0;
  const auto bin = [&](int j) -> uint32_t {
    if constexpr (WIDE) return bn[j];
    else return first_sub(j);
  };
  if (!fast_claim<C::FC, C::NB, UPS>(a, w, S.sc, nullptr, a.wl_kv + (size_t)w * kCW, a.wl_op + (size_t)w * kCW,
                                     &S.nsplit, &S.nreq, &S.need, rk, rv, rop, pq, e8, home8, x8, bin, c_runs, c_lines,
                                     c_waited, stamp, UPS ? upd : nullptr, UPS ? occw : nullptr))
    return 1u;
  if (lane == 0) a.wl_n[w] = S.nsplit;  // parked inserts (0: done)
  {
    __builtin_amdgcn_wave_barrier();
    const uint32_t nr = min(S.nreq, kSplitCap);
    if (nr) request_splits(a, w, nr, S.need > db ? S.need : 0u);
  }
  // this bucket's stat slots, as bucket_body's first pass keeps them
  for (int o = 32; o > 0; o >>= 1) {
    c_lines += (uint32_t)__shfl_down((int)c_lines, o);
    c_waited += (uint32_t)__shfl_down((int)c_waited, o);
  }
  {
    const uint32_t s0 = (uint32_t)__shfl((int)c_lines, 0), s1 = (uint32_t)__shfl((int)c_waited, 0);
    const uint32_t s4 = (uint32_t)__shfl((int)c_runs, 0);
    const uint32_t add = lane == 0 ? s0 : lane == 1 ? s1 : lane == 4 ? s4 : lane == 5 ? 1u : 0u;
    uint64_t* ws = a.wstat + (size_t)w * kWStat;
    if (lane < 6u && add) ws[lane] = wsv + add;
    if (lane == 6u) ws[6] = max((uint32_t)(wsv & 0xFFFF), 1u) | (((wsv >> 16) & 0xFF) << 16) | ((wsv >> 32) << 32);
  }
  FS_STAMP(7);
#undef FS_STAMP
  return 0u;
}

// a bucket the lean pass declined (nothing written): flagged for k_apply_fb,
// or, when none is launched, for k_apply_parked (anydecl: every decliner
// stores the same word, no read-modify-write)
__device__ __forceinline__ void declined(const BucketArgs& a, uint32_t w) {
  a.fbl[w] |= 1u;
  a.ctl->anydecl[a.par] = 1u;
}

__global__ __launch_bounds__(64, 8) void k_apply_fast(BucketArgs a) {
  if (gated_off(a)) return;
  __shared__ FastLds<false> S;
  // a declined bucket is flagged in its own word (bit 0; bits 1+ count the
  // declines for stats): no shared counter, since in a table whose every
  // bucket declines 8,192 atomics on one word would serialize (~88 per us)
  if (apply_fast<false>(a, S, blockIdx.x) != 0 && threadIdx.x == 0) declined(a, blockIdx.x);
}

// the coarse-partition lean first pass: a workgroup of 8 waves per partition
// bucket, wave v taking directory bucket (partition bucket << 3) | v
#ifndef PMDFC_CP_WPE
#define PMDFC_CP_WPE 8  // (A/B builds) minimum waves per SIMD: 8 caps it at 64 VGPRs
#endif
__global__ __launch_bounds__(64 * kCpWaves) __attribute__((amdgpu_waves_per_eu(PMDFC_CP_WPE, 8))) void k_apply_fast_cp(
    BucketArgs a) {
  if (gated_off(a)) return;
  __shared__ CpLds L;
  // (the wave's index through readfirstlane: wave-uniform, so w and every
  // address derived from it live in scalar registers)
  const uint32_t v = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), w = (blockIdx.x << kCpSbb) | v;
  if (apply_fast<false, false, true>(a, L.w[v], w, &L) != 0 && (threadIdx.x & 63u) == 0) declined(a, w);
}

// the lean first pass for large tables (the host picks it from the table's
// segments per bucket, pmdfc_cceh::wide): sub-directories up to 128 entries
__global__ __launch_bounds__(64, 6) void k_apply_wide(BucketArgs a) {
  if (gated_off(a)) return;
  __shared__ FastLds<true> S;
  if (apply_fast<true>(a, S, blockIdx.x) != 0 && threadIdx.x == 0) declined(a, blockIdx.x);
}

// the lean first passes in last-writer-wins mode (insert-only batches)
template <bool WIDE>
__global__ __launch_bounds__(64, 5) void k_apply_fast_ups(BucketArgs a) {
  __shared__ FastLds<WIDE> S;
  if (apply_fast<WIDE, true>(a, S, blockIdx.x) != 0 && threadIdx.x == 0) declined(a, blockIdx.x);
}

// the buckets k_apply_fast / k_apply_wide declined: bucket_body's general
// first pass, the same wave per bucket (the others exit after one load).  At
// config 2 it flags nothing and costs one empty launch.
__global__ __launch_bounds__(64, 2) void k_apply_fb(BucketArgs a) {
  if (gated_off(a)) return;
  const uint32_t w = blockIdx.x, f = a.fbl[w];
  if (!(f & 1u)) return;
  __shared__ BucketLds<false, true> S;
  bucket_body<false, false, true>(a, w, S);
  if (threadIdx.x == 0) a.fbl[w] = f + 1u;  // pending bit off, count + 1
}

// A/B knob: dynamic LDS added to each k_apply_fast wave (lowers its occupancy)
static uint32_t fast_lds_pad() {
  static const uint32_t pad = [] {
    const char* e = getenv("PMDFC_FAST_LDS_PAD");
    return e ? (uint32_t)atoi(e) : 0u;
  }();
  return pad;
}

bool fast_first_pass() {
  static const bool on = [] {
    const char* e = getenv("PMDFC_FAST_APPLY");  // A/B: 0 = the general first pass for every bucket
    return !(e && e[0] == '0');
  }();
  return on;
}

// ------------------------------------------------------------- launchers

#ifndef PMDFC_PARKED_GRID
#define PMDFC_PARKED_GRID 3072  // (A/B builds; 3 waves per SIMD since round 6: 2048 13.13-13.15 Gops/s against 13.22; 1024 12.25-12.30 in round 4)
#endif
#ifndef PMDFC_FINAL_GRID
#define PMDFC_FINAL_GRID 256  // (A/B builds; 1024 as above)
#endif
constexpr uint32_t kParkedGrid = PMDFC_PARKED_GRID;  // k_apply_parked waves (loop over the worklist)
constexpr uint32_t kFinalGrid = PMDFC_FINAL_GRID;    // k_bucket waves
#ifndef PMDFC_MIXED_SMALL_GRID
#define PMDFC_MIXED_SMALL_GRID 256  // (A/B builds) the mixed passes' grid when the host expects them gated off
#endif
constexpr uint32_t kMixedSmallGrid = PMDFC_MIXED_SMALL_GRID;
#ifndef PMDFC_PARKED_GRID_RAMP
#define PMDFC_PARKED_GRID_RAMP 4096
#endif
#ifndef PMDFC_FINAL_GRID_RAMP
#define PMDFC_FINAL_GRID_RAMP 1024
#endif
constexpr uint32_t kParkedGridRamp = PMDFC_PARKED_GRID_RAMP;  // while the table ramps (p1 < p1max)
constexpr uint32_t kFinalGridRamp = PMDFC_FINAL_GRID_RAMP;

uint32_t part_blocks(uint64_t n) { return (uint32_t)((n + kPartTile - 1) / kPartTile); }

void launch_part(const PartLaunch& L, hipStream_t s) {
  if (!L.n) return;
  PartArgs a;
  a.keys = L.keys;
  a.vin = L.vin;
  a.ops = L.ops;
  a.st = L.st;
  a.n = L.n;
  a.kvs = L.kvs ? L.kvs : 1u;
  a.sbits = L.sbits;
  a.shard = L.shard;
  a.p1 = L.p1 - L.sbb;
  a.sbb = L.sbb;
  a.cap = L.cap;
  a.capx = L.cap / kPartSubs;
  a.ovf_base = (uint64_t)L.cap << (L.p1 - L.sbb);
  a.rkv = L.rkv;
  a.rop = L.rop;
  a.robk = L.robk;
  a.cursor = L.cursor;
  a.ovf = L.ovf;
  a.stamps = L.stamps;
  a.init = L.init;
  a.vout = L.vout;
  a.touched = L.touched;
  static const uint32_t delay = [] {
    const char* e = getenv("PMDFC_PART_DELAY_US");
    return e ? (uint32_t)(atof(e) * 100.0) : 0u;
  }();
  a.delay = delay;
  a.povf = L.povf;
  a.iset = L.iset;
  a.imask = L.imask;
  a.icnt = L.icnt;
  a.ipos = L.ipos;
  a.early = L.early;
  a.elink = L.elink;
  a.ctl = L.ctl;
  a.tag = L.tag;
  hipLaunchKernelGGL(k_part, dim3(part_blocks(L.n)), dim3(kPartThreads), 0, s, a);
}

static BucketArgs bucket_args(const BucketLaunch& L) {
  BucketArgs a;
  a.rkv = L.rkv;
  a.rop = L.rop;
  a.robk = L.robk;
  a.n = L.n;
  a.chunk = (L.chunk == 0 || L.chunk > (uint32_t)kCW) ? (uint32_t)kCW : L.chunk;
  a.cap = L.cap;
  a.capx = L.cap / kPartSubs;
  a.ovf_base = (uint64_t)L.cap << (L.p1 - L.sbb);
  a.cursor = L.cursor;
  a.ovf = L.ovf;
  a.cursor_next = L.cursor_next;
  a.ovf_next = L.ovf_next;
  a.clear_next = L.clear_next;
  a.hdr = L.hdr;
  a.pool = L.pool;
  a.pool_cap = L.pool_cap;
  a.p1 = L.p1;
  a.sbb = L.sbb;
  a.sbits = L.sbits;
  a.shard = L.shard;
  a.pfix = L.pfix;
  a.pairs = L.pairs;
  a.occ = L.occ;
  a.ldep = L.ldep;
  a.vout = L.vout;
  a.st = L.st;
  a.mixed = L.mixed;
  a.upsert = L.upsert;
  a.upos = L.upos;
  a.max_segments = L.max_segments;
  a.ctl = L.ctl;
  a.wstat = L.wstat;
  a.wl_kv = L.wl_kv;
  a.wl_op = L.wl_op;
  a.wl_n = L.wl_n;
  a.stamps = L.stamps;
  a.req = L.req;
  a.reqop = L.reqop;
  a.drops = L.drops;
  a.need = L.need;
  a.gbase = L.gbase;
  a.ngrant = L.ngrant;
  a.newoff = L.newoff;
  a.gsh = L.gsh;
  a.gsplit = L.gsplit;
  a.gcap = L.gcap;
  a.act = L.act;
  a.fbl = L.fbl;
  a.hint = L.hint;
  a.mseen = L.mseen;
  a.mode = 0;
  a.fin = L.fin;
  a.par = L.par;
  a.gate = 0;
  a.gate_tag = L.gate_tag;
  return a;
}

void launch_apply(const BucketLaunch& L, uint32_t mode, hipStream_t s) {
  if (!L.n) return;
  BucketArgs a = bucket_args(L);
  a.mode = mode;
  const dim3 g(1u << L.p1);
  // a gated mixed batch launches the insert-only variant (taken when
  // k_mixed_get answered every Get) and then the mixed one
  const bool gated = L.mixed && L.gate_tag != 0;
  BucketArgs ar = a;
  if (gated) {
    ar.gate = 2;
    a.gate = 1;
  }
  if (mode == 0) {
    if (gated || !L.mixed) {
      if (L.upsert && !L.mixed && fast_first_pass()) {
        // last-writer-wins, insert-only: the lean pass probes each window
        if (L.wide) hipLaunchKernelGGL(k_apply_fast_ups<true>, g, dim3(64), 0, s, ar);
        else hipLaunchKernelGGL(k_apply_fast_ups<false>, g, dim3(64), 0, s, ar);
      } else if (!L.upsert && fast_first_pass()) {
        // the lean first pass (launch_apply_fallback: the general one over
        // the buckets it left), its wide variant for large tables
        if (L.cp) hipLaunchKernelGGL(k_apply_fast_cp, dim3(1u << (L.p1 - kCpSbb)), dim3(64 * kCpWaves), 0, s, ar);
        else if (L.wide) hipLaunchKernelGGL(k_apply_wide, g, dim3(64), 0, s, ar);
        else hipLaunchKernelGGL(k_apply_fast, g, dim3(64), fast_lds_pad(), s, ar);
      } else {
        hipLaunchKernelGGL(k_apply<false>, g, dim3(64), 0, s, ar);
      }
    }
    if (L.mixed && gated && L.mixed_small)
      hipLaunchKernelGGL(k_apply_mloop, dim3(std::min(1u << L.p1, kMixedSmallGrid)), dim3(64), 0, s, a);
    else if (L.mixed)
      hipLaunchKernelGGL(k_apply<true>, g, dim3(64), 0, s, a);
  } else {
    // worklist passes: a smaller grid (a ramping table's passes carry more work per batch)
    const dim3 gw(std::min(1u << L.p1, L.ramp ? kParkedGridRamp : kParkedGrid));
    if (gated) {  // (both variants as two launches: configs 3 / 4 7.17-7.25 / 6.04-6.06 against 7.31-7.34 / 6.12-6.15)
      hipLaunchKernelGGL(k_apply_parked_gated, gw, dim3(64), 0, s, ar, a);
    } else {
      if (gated || !L.mixed) hipLaunchKernelGGL(k_apply_parked<false>, gw, dim3(64), 0, s, ar);
      if (L.mixed)
        hipLaunchKernelGGL(k_apply_parked<true>, gated && L.mixed_small ? dim3(std::min(gw.x, kMixedSmallGrid)) : gw,
                           dim3(64), 0, s, a);
    }
  }
}

void launch_apply_fallback(const BucketLaunch& L, hipStream_t s) {
  if (!L.n || !fast_first_pass() || (L.upsert && L.mixed)) return;  // (no lean pass was launched)
  const bool gated = L.mixed && L.gate_tag != 0;
  if (L.mixed && !gated) return;
  BucketArgs a = bucket_args(L);
  if (gated) a.gate = 2;  // with the insert-only variant it follows
  hipLaunchKernelGGL(k_apply_fb, dim3(1u << L.p1), dim3(64), 0, s, a);
}

void launch_final(const BucketLaunch& L, hipStream_t s) {
  if (!L.n) return;
  const dim3 g(std::min(1u << L.p1, L.ramp ? kFinalGridRamp : kFinalGrid));
  if (L.mixed) hipLaunchKernelGGL(k_bucket<true>, g, dim3(64), 0, s, bucket_args(L));
  else hipLaunchKernelGGL(k_bucket<false>, g, dim3(64), 0, s, bucket_args(L));
}

void launch_mixed_small(const BucketLaunch& L, const uint8_t* ops, const uint64_t* keys, const uint64_t* vin,
                        hipStream_t s) {
  if (!L.n) return;
  BucketArgs a = bucket_args(L);
  a.stamps = nullptr;
  if (L.n <= 64) {
    hipLaunchKernelGGL(k_mixed_tiny, dim3(1), dim3(64), 0, s, a, ops, keys, vin);
    return;
  }
  const uint32_t grid = (uint32_t)std::min<uint64_t>(L.n, 1ULL << L.p1);  // >= the distinct buckets
  hipLaunchKernelGGL(k_mixed_small, dim3(grid), dim3(64), 0, s, a, ops, keys, vin);
}

void launch_serve(const BucketLaunch& L, const ServeLaunch& V, hipStream_t s) {
  ServeArgs sa;
  sa.a = bucket_args(L);
  sa.a.stamps = nullptr;
  sa.req = V.req;
  sa.resp = V.resp;
  sa.ctl = V.ctl;
  sa.ring_size = V.ring_size;
  sa.head0 = V.head0;
  sa.cbf = V.cbf;
  sa.cbf_m = V.cbf_m;
  sa.cbf_k = V.cbf_k;
  sa.nwaves = V.nwaves ? V.nwaves : 1u;
  hipLaunchKernelGGL(k_serve, dim3(sa.nwaves), dim3(64), 0, s, sa);
}

void launch_medium(const BucketLaunch& L, const uint32_t* touched, hipStream_t s) {
  if (!L.n) return;
  const uint32_t npb = 1u << (L.p1 - L.sbb);
  const dim3 g((uint32_t)std::min<uint64_t>(std::max<uint64_t>(L.n, 64), npb));  // >= the touched buckets
  if (L.mixed) hipLaunchKernelGGL(k_medium<true>, g, dim3(64), 0, s, bucket_args(L), touched);
  else hipLaunchKernelGGL(k_medium<false>, g, dim3(64), 0, s, bucket_args(L), touched);
}

void launch_split_round(const BucketLaunch& L, hipStream_t s) {
  if (!L.n) return;
  SplitArgs p;
  p.par = L.par;
  p.pfix = L.pfix;
  p.stamps = L.split_stamps;
  p.gsh = L.gsh;
  p.gsplit = L.gsplit;
  p.gcap = L.gcap;
  p.act = L.act;
  p.gbase = L.gbase;
  p.ngrant = L.ngrant;
  p.newoff = L.newoff;
  p.need = L.need;
  p.max_segments = L.max_segments;
  p.pool_cap = L.pool_cap;
  p.pairs = L.pairs;
  p.occ = L.occ;
  p.ldep = L.ldep;
  p.ctl = L.ctl;
  p.reqop = L.reqop;
  p.drops = L.drops;
  static const uint32_t team_max = [] {  // PMDFC_SPLIT_TEAM_MAX (A/B): the team-mode cut
    const char* e = getenv("PMDFC_SPLIT_TEAM_MAX");
    return e ? (uint32_t)strtoul(e, nullptr, 0) : kSplitGroups;
  }();
  p.team_max = team_max;
  hipLaunchKernelGGL(k_split, dim3(L.ramp ? kSplitGroupsRamp : kSplitGroups), dim3(64 * kSplitWaves), 0, s, p);
}

}  // namespace pmdfc
