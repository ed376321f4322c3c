// cceh_device.h -- layout constants, hashes and probe primitives shared by the
// MI355X CCEH kernels (gfx950, wave64).
//
// HBM layout (DESIGN.md "Data layout"):
//   pairs  : max_segments x 1024 x {u64 key, u64 value}   (16 KiB per segment,
//            64-B lines of 4 slots; a probe window is 8 lines = 512 B)
//   occ    : max_segments x 32 u32   occupancy bitmap, bit j of word i = slot 32i+j
//   ldep   : max_segments x u8       local depth (global hash bits)
//   dir    : 2^(phys_depth - shard_bits) x u32 segment ids
// Reference layout: server/CCEH_hybrid.h:14-19,27-100 (Segment = 1024 Pair +
// sema + local_depth; Directory = Segment*[2^depth]).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pmdfc {

constexpr uint32_t kSlots = 1024;        // Segment::kNumSlot
constexpr uint32_t kWindow = 32;         // kNumPairPerCacheLine * kNumCacheLine
constexpr uint32_t kLines = 8;           // 64-B lines per window
constexpr uint32_t kMaxDepth = 30;
constexpr uint64_t kInvalid = ~0ULL;     // server/util/pair.h:10
constexpr uint64_t kSentinel = ~0ULL - 1;  // server/util/pair.h:9
constexpr uint8_t kStPending = 0xFF;     // internal: not yet resolved
constexpr uint8_t kStLinked = 0xFE;      // internal (mixed batches): resolved after the batch from its one earlier insert
constexpr uint8_t kStJoin = 0xFD;        // internal (mixed batches): a Get whose answer waits for the join with the batch's inserts
// mixed batches: the joining Gets' filter (k_mixed_get / k_mixed_join), one
// per set replica (kJoinReps, by the claiming block's XCD), interleaved: word
// (bit >> 5) * kJoinReps + replica
constexpr uint32_t kJoinReps = 8;
constexpr uint32_t kJoinBits = 1u << 20;  // bits per replica (8 x 128 KiB)
constexpr uint64_t kJoinWords = (uint64_t)kJoinBits / 32 * kJoinReps;
// a key's first slot in a mixed batch's key set (or in one replica of it)
__host__ __device__ __forceinline__ uint64_t iset_slot(uint64_t h, uint64_t mask) {
  return (h ^ (h >> 29) ^ (h >> 47)) & mask;
}

// std::_Hash_bytes(&key, 8, 0xc70697) -- server/util/hash.h:7-10,252-254.
// libstdc++ hash_bytes.cc (64-bit size_t branch), one 8-byte block, no tail.
__host__ __device__ __forceinline__ uint64_t hash64(uint64_t key) {
  const uint64_t mul = 0xc6a4a7935bd1e995ULL;
  uint64_t h = 0xc70697ULL ^ (8ULL * mul);
  uint64_t d = key * mul;
  d = (d ^ (d >> 47)) * mul;
  h ^= d;
  h *= mul;
  h = (h ^ (h >> 47)) * mul;
  return h ^ (h >> 47);
}

// MurmurHash2 (32-bit) of the 8 key bytes -- server/util/hash.h:42-91,
// client/hash.h:48-97 (identical).
__host__ __device__ __forceinline__ uint32_t murmur2_u64(uint64_t key, uint32_t seed) {
  const uint32_t m = 0x5bd1e995u;
  uint32_t h = seed ^ 8u;
  uint32_t k = (uint32_t)key;
  k *= m; k ^= k >> 24; k *= m;
  h *= m; h ^= k;
  k = (uint32_t)(key >> 32);
  k *= m; k ^= k >> 24; k *= m;
  h *= m; h ^= k;
  h ^= h >> 13; h *= m; h ^= h >> 15;
  return h;
}

__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

__host__ __device__ __forceinline__ bool reserved_key(uint64_t k) {
  return k >= kSentinel;
}

// Directory entries pack the segment id and its local depth (so a walk over
// the directory never needs a dependent ldep[] load): bits 0-25 segment id,
// bits 26-31 local depth in global hash bits.
constexpr uint32_t kSegBits = 26;
constexpr uint32_t kSegMask = (1u << kSegBits) - 1;
constexpr uint64_t kMaxSegments = 1ULL << 25;  // k_bucket sort keys carry 25-bit segment ids
__host__ __device__ __forceinline__ uint32_t de_seg(uint32_t e) { return e & kSegMask; }
__host__ __device__ __forceinline__ uint32_t de_ld(uint32_t e) { return e >> kSegBits; }
__host__ __device__ __forceinline__ uint32_t de_make(uint32_t seg, uint32_t ld) {
  return seg | (ld << kSegBits);
}

// Bucketed directory.  The reference directory is one flat
// array of 2^depth segment pointers indexed by the top `depth` hash bits
// (CCEH_hybrid.cpp:119).  Here the top p1 local hash bits (after the shard
// prefix) pick a BUCKET; each bucket owns a sub-directory of 2^db entries,
// indexed by the next db bits, in a pool.  Logically it is the same directory
// (entry for prefix x = sub-directory entry of x's bucket at that bucket's
// depth), but every bucket grows on its own, so a workgroup that owns a bucket
// can split segments AND deepen its sub-directory without any global
// doubling (CCEH_hybrid.cpp:197-219).  p1 <= every local depth (minus shard
// bits), so a segment never spans two buckets.
//   hdr[b] : bits 0-31 pool offset of bucket b's sub-directory, 32-39 db
struct Geo {
  const uint64_t* hdr;   // 2^p1 bucket headers
  const uint32_t* pool;  // sub-directory entries (de_make format)
  uint32_t p1;           // bucket bits
  uint32_t sbits;        // shard prefix bits
  uint32_t shard;        // shard prefix value
  // pure-Get batches: the directory flattened to one level (k_flatten), or
  // null; *flat_bits > kFlatMaxBits means "too deep, use hdr/pool"
  const uint32_t* flat;
  const uint32_t* flat_bits;
};
constexpr uint32_t kFlatMaxBits = 20;  // 4 MiB of u32 entries: stays in L2

__host__ __device__ __forceinline__ uint32_t hdr_off(uint64_t hd) { return (uint32_t)hd; }
__host__ __device__ __forceinline__ uint32_t hdr_db(uint64_t hd) { return (uint32_t)(hd >> 32) & 0xFFu; }
__host__ __device__ __forceinline__ uint64_t hdr_make(uint32_t off, uint32_t db) {
  return (uint64_t)off | ((uint64_t)db << 32);
}

// bucket of a hash: top p1 bits after the shard prefix
__device__ __forceinline__ uint32_t bucket_of(uint64_t h, uint32_t sbits, uint32_t p1) {
  return p1 ? (uint32_t)((h << sbits) >> (64 - p1)) : 0u;
}
// index inside a bucket's sub-directory of depth db
__device__ __forceinline__ uint32_t sub_index(uint64_t h, uint32_t sbits, uint32_t p1, uint32_t db) {
  return db ? (uint32_t)((h << (sbits + p1)) >> (64 - db)) : 0u;
}

__device__ __forceinline__ uint32_t dir_entry(const Geo& g, uint64_t h) {
  if (g.flat) {  // one dependent load instead of two
    const uint32_t fb = *g.flat_bits;
    if (fb <= kFlatMaxBits) return g.flat[fb ? (uint32_t)((h << g.sbits) >> (64 - fb)) : 0u];
  }
  const uint64_t hd = g.hdr[bucket_of(h, g.sbits, g.p1)];
  return g.pool[hdr_off(hd) + sub_index(h, g.sbits, g.p1, hdr_db(hd))];
}

__device__ __forceinline__ bool wrong_shard(uint64_t h, uint32_t sbits, uint32_t shard) {
  return sbits != 0 && (uint32_t)(h >> (64 - sbits)) != shard;
}

// Loads of state that other waves of the same workgroup rewrite inside one
// launch (segment pairs, occupancy words, sub-directory entries): served by
// L2, never by a possibly stale L1 line (MI355X_MICROARCH.md, visibility).
typedef unsigned long long u64x2_t __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ ulonglong2 ld_pair_l2(const ulonglong2* p) {
  const u64x2_t v = __builtin_nontemporal_load(reinterpret_cast<const u64x2_t*>(p));
  return make_ulonglong2(v.x, v.y);
}
__device__ __forceinline__ uint4 ld_u4_l2(const uint32_t* p) {
  const u32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint32_t ld_u32_l2(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// first free slot of the 32-slot window starting at w (a multiple of 4) in a
// 1024-bit occupancy map, cyclic (CCEH_hybrid.cpp:143-156: (y+i) % kNumSlot);
// -1 if the window is full.
__device__ __forceinline__ int window_first_free(uint32_t lo, uint32_t hi, uint32_t w) {
  uint64_t win = (((uint64_t)hi << 32) | lo) >> (w & 31);
  uint32_t fr = ~(uint32_t)win;
  if (fr == 0) return -1;
  return (int)((w + (uint32_t)__builtin_ctz(fr)) & (kSlots - 1));
}

__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
  int lo = __shfl((int)(uint32_t)v, src);
  int hi = __shfl((int)(uint32_t)(v >> 32), src);
  return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}

// Quad-cooperative Get probe (4 lanes per key, one 16-B slot each, one 64-B
// line per step, early exit at the first empty slot -- SURVEY a5, equal to the
// reference's full scan CCEH_hybrid.cpp:372-382 because nothing is deleted).
// All 4 lanes of the quad must call it with the same key/h.  Returns HIT/MISS,
// *val valid on every lane of the quad, *lines = 64-B lines read.
// From an even window line, the next line is the other half of the same
// 128-B HBM line: both are loaded together (one round trip per two lines).
__device__ __forceinline__ uint8_t quad_probe(const ulonglong2* __restrict__ seg, uint64_t key,
                                              uint64_t h, uint32_t q, uint64_t* val,
                                              uint32_t* lines) {
  const uint32_t line0 = (uint32_t)(h & 0xFF);
  const uint32_t qbase = (__lane_id() & 63u) & ~3u;
  for (uint32_t t = 0; t < kLines;) {
    const uint32_t ln = (line0 + t) & 255u;
    const bool two = !(ln & 1u) && t + 1 < kLines;
    const ulonglong2 pa = seg[ln * 4u + q];
    const ulonglong2 pb = two ? seg[ln * 4u + 4u + q] : pa;
#pragma unroll
    for (uint32_t k = 0; k < 2; ++k) {
      if (k == 1 && !two) break;
      const ulonglong2 p = k ? pb : pa;
      const uint32_t mn = (uint32_t)(__ballot(p.x == key) >> qbase) & 0xFu;
      const uint32_t en = (uint32_t)(__ballot(p.x == kInvalid) >> qbase) & 0xFu;
      if (mn) {
        *val = shfl64(p.y, (int)(qbase + (uint32_t)__builtin_ctz(mn)));
        *lines = t + k + 1;
        return 1;  // PMDFC_ST_HIT
      }
      if (en) {
        *lines = t + k + 1;
        return 0;  // PMDFC_ST_MISS
      }
    }
    t += two ? 2u : 1u;
  }
  *lines = kLines;
  return 0;
}

// quad_probe that also tells a single copy of the key from several: scans
// on to the window's first empty slot (every copy of a key lies before it:
// slots are never freed, and an Insert takes the first free slot of its
// window, CCEH_hybrid.cpp:143-168; split replay keeps that).  Returns 0 miss,
// 1 hit with exactly one copy, 2 several copies.  Lines in pairs as above.
__device__ __forceinline__ uint8_t quad_probe_once(const ulonglong2* __restrict__ seg, uint64_t key,
                                                   uint64_t h, uint32_t q, uint64_t* val) {
  const uint32_t line0 = (uint32_t)(h & 0xFF);
  const uint32_t qbase = (__lane_id() & 63u) & ~3u;
  uint32_t copies = 0;
  for (uint32_t t = 0; t < kLines;) {
    const uint32_t ln = (line0 + t) & 255u;
    const bool two = !(ln & 1u) && t + 1 < kLines;
    const ulonglong2 pa = seg[ln * 4u + q];
    const ulonglong2 pb = two ? seg[ln * 4u + 4u + q] : pa;
    bool stop = false;
#pragma unroll
    for (uint32_t k = 0; k < 2; ++k) {
      if (k == 1 && !two) break;
      const ulonglong2 p = k ? pb : pa;
      const uint32_t mn = (uint32_t)(__ballot(p.x == key) >> qbase) & 0xFu;
      const uint32_t en = (uint32_t)(__ballot(p.x == kInvalid) >> qbase) & 0xFu;
      if (mn && copies == 0) *val = shfl64(p.y, (int)(qbase + (uint32_t)__builtin_ctz(mn)));
      copies += (uint32_t)__builtin_popcount(mn);
      if (en || copies > 1) {
        stop = true;
        break;
      }
    }
    if (stop) break;
    t += two ? 2u : 1u;
  }
  return copies == 0 ? 0 : copies == 1 ? 1 : 2;
}

// Single-lane probe used inside per-segment sequential processing (reads
// through L2: earlier inserts of this launch may have changed the lines).
__device__ __forceinline__ uint8_t lane_probe(const ulonglong2* __restrict__ seg, uint64_t key,
                                              uint64_t h, uint64_t* val) {
  const uint32_t line0 = (uint32_t)(h & 0xFF);
  // two lines per round trip (the window's slots in order: first match or
  // first empty slot decides, as one line at a time would)
  for (uint32_t t = 0; t < kLines; t += 2) {
    ulonglong2 ln[8];
#pragma unroll
    for (uint32_t q = 0; q < 8; ++q) ln[q] = ld_pair_l2(seg + ((line0 + t + (q >> 2)) & 255u) * 4u + (q & 3u));
#pragma unroll
    for (uint32_t q = 0; q < 8; ++q) {
      const ulonglong2 p = ln[q];
      if (p.x == key) {
        *val = p.y;
        return 1;
      }
      if (p.x == kInvalid) return 0;
    }
  }
  return 0;
}

// Exact parallel replay of Segment::Split's slot-order Insert4split loop
// (CCEH_hybrid.cpp:18-28,53-60) for one wave.  Slot s = 64*g + lane is
// described by inf[g]: bit 31 valid, bit 8 child, bits 0-7 home line.  The
// sequential rule: in slot order, each entry takes the first free slot of its
// 32-slot window in its child, or is dropped.
// Per group of 64 slots (one per lane) the wave iterates:
//   * each pending lane computes a tentative slot from the committed child
//     bitmaps: the (r+1)-th free slot of its window, r = number of earlier
//     pending lanes with the same (child, home);
//   * all tentative slots are posted to a claim map; a lane is SAFE if the
//     claims inside [home, tentative] are exactly its own r+1 (no other home
//     claims there, no two lanes on one slot) -- then its sequential result is
//     the tentative one, given that every earlier lane is exact;
//   * lanes before the first unsafe lane commit; the first pending lane always
//     commits (every earlier lane is already committed, r = 0).
// Returns the per-lane count of dropped entries; dest[g] = (child<<10)|slot or
// ~0u if dropped/invalid.  s_b (64 words) must hold the empty child bitmaps;
// s_cb / s_col (64 words each) are scratch.  All 64 lanes must be active.
__device__ __forceinline__ uint32_t wave_replay(const uint32_t (&inf)[16], uint32_t (&dest)[16],
                                                uint32_t* s_b, uint32_t* s_cb, uint32_t* s_col) {
  const uint32_t lane = __lane_id() & 63u;
  const uint64_t lt = (1ULL << lane) - 1;
  uint32_t loss = 0;
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    const uint32_t in = inf[g];
    const uint32_t c = (in >> 8) & 1u;
    const uint32_t home = in & 0xFFu;
    const uint32_t key = in & 0x1FFu;  // (child, home)
    const uint32_t w = home * 4u;
    const uint32_t wi = w >> 5, off = w & 31u;
    const uint32_t wlo = c * 32u + wi, whi = c * 32u + ((wi + 1u) & 31u);
    bool rem = (in >> 31) != 0;
    uint32_t d = 0xFFFFFFFFu;
    for (;;) {
      const uint64_t rm = __ballot(rem);
      if (!rm) break;
      const uint32_t f = (uint32_t)__builtin_ctzll(rm);
      uint64_t mm = rm;
#pragma unroll
      for (uint32_t bit = 0; bit < 9; ++bit) {
        const uint64_t bb = __ballot((key >> bit) & 1u);
        mm &= ((key >> bit) & 1u) ? bb : ~bb;
      }
      const uint32_t r = (uint32_t)__popcll(mm & lt);
      const uint64_t win = (((uint64_t)s_b[whi] << 32) | s_b[wlo]) >> off;
      const uint32_t fr = ~(uint32_t)win;
      uint32_t f2 = fr;
      for (uint32_t i = 0; i < r && f2; ++i) f2 &= f2 - 1;
      const bool lost = f2 == 0;
      const uint32_t t = lost ? 0u : (uint32_t)__builtin_ctz(f2);   // offset in window
      const uint32_t tpos = (w + t) & (kSlots - 1);
      s_cb[lane] = 0;
      s_col[lane] = 0;
      __builtin_amdgcn_wave_barrier();
      if (rem && !lost) {
        const uint32_t bit = 1u << (tpos & 31u);
        const uint32_t old = atomicOr(&s_cb[c * 32u + (tpos >> 5)], bit);
        if (old & bit) atomicOr(&s_col[c * 32u + (tpos >> 5)], bit);
      }
      __builtin_amdgcn_wave_barrier();
      const uint64_t cbw = (((uint64_t)s_cb[whi] << 32) | s_cb[wlo]) >> off;
      const uint64_t clw = (((uint64_t)s_col[whi] << 32) | s_col[wlo]) >> off;
      const uint32_t span = lost ? 32u : t + 1u;
      const uint32_t mask = span >= 32 ? 0xFFFFFFFFu : ((1u << span) - 1u);
      const uint32_t expect = lost ? (uint32_t)__popc(fr) : r + 1u;
      const bool safe = (uint32_t)__popc((uint32_t)cbw & mask) == expect && ((uint32_t)clw & mask) == 0;
      uint64_t um = __ballot(rem && !safe);
      um &= ~((2ULL << f) - 1);  // lanes <= f commit regardless
      const uint32_t P = um ? (uint32_t)__builtin_ctzll(um) : 64u;
      const bool commit = rem && lane < P;
      __builtin_amdgcn_wave_barrier();
      if (commit) {
        if (lost) {
          ++loss;
        } else {
          atomicOr(&s_b[c * 32u + (tpos >> 5)], 1u << (tpos & 31u));
          d = (c << 10) | tpos;
        }
        rem = false;
      }
      __builtin_amdgcn_wave_barrier();
    }
    dest[g] = d;
  }
  return loss;
}

// CountingBloomFilter<Key_t>::Insert of one key (server/util/counting_bloom_filter.h
// :109-118): saturating += 1 on the u8 counter of each of the k indices
// (int)(murmur2(&x, 8, seed=i) % m), m < 2^31; a per-byte CAS on its u32 word.
__device__ __forceinline__ void cbf_increment(uint8_t* cnt, uint64_t m, uint32_t k, uint64_t key) {
  for (uint32_t j = 0; j < k; ++j) {
    const uint64_t idx = (uint64_t)(murmur2_u64(key, j) % (uint32_t)m);
    uint32_t* w = reinterpret_cast<uint32_t*>(cnt + (idx & ~3ull));
    const uint32_t sh = 8u * (uint32_t)(idx & 3u);
    uint32_t o = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while (((o >> sh) & 0xFFu) != 0xFFu) {
      const uint32_t prev = atomicCAS(w, o, o + (1u << sh));
      if (prev == o) break;
      o = prev;
    }
  }
}

// Device-side control block (one per engine).  Nothing on the insert path
// reads it back: the host copies it only for stats/dump.
struct DevCtl {
  uint32_t nsegs;        // segment ids handed out (may overshoot max on CAPACITY)
  uint32_t pool_cur;     // sub-directory pool entries handed out (may overshoot the pool likewise)
  uint32_t max_ld;       // max local depth (global bits)
  uint32_t err;          // sticky: 1 pool exhausted, 2 round guard tripped
  uint32_t max_rounds;   // most split rounds one chunk needed
  uint32_t full;         // sticky: a grant ran out of segment ids or pool
  uint32_t anyreq[2];    // by batch parity: some bucket requested a split (the split round's early exit)
  uint32_t nact[2];      // by batch parity: buckets with requests (k_split -> k_apply_parked; list: act)
  uint64_t split_loss;   // entries dropped by split replay
  uint64_t splits;       // splits performed
  uint64_t runs;         // (segment, round) runs processed
  uint64_t rounds;       // (bucket chunk, round) iterations
  uint64_t waited;       // ops that waited for a split
  uint64_t growths;      // sub-directory growths
  uint64_t ins_lines;    // sum over inserts of 64-B lines from y to the claimed slot
  uint32_t depth_count[32];  // live segments per local depth
  uint32_t loss_events;  // splits that dropped entries (k_split, k_bucket): mixed-batch verify
  uint32_t nfin[2];      // -> k_bucket, by batch parity: buckets left for the final pass (list: fin)
  uint32_t pget;         // k_mixed_get -> bucket passes: tag of the last mixed batch that left a Get pending
  uint32_t drop_n;       // mixed batch: entries in the drop log (k_mixed_reset zeroes it)
  uint32_t anydecl[2];   // by batch parity: the lean first pass declined some bucket (k_apply_parked takes it)
  uint32_t ins_total;    // mixed batch: key-set slots its joining Gets claimed (k_mixed_join sums k_mixed_get's per-block counts)
  uint32_t njoin;        // k_mixed_get -> k_mixed_join: tag of the last mixed batch with a joining Get
};

// Drop log of a mixed batch (kDropLog x {key, op index of the insert whose
// split dropped it}): a split's Insert4split drops (CCEH_hybrid.cpp:24-27)
// are logged with the batch position of the insert that triggered the split,
// so k_mixed_verify can place a drop before or after an early-answered Get.
constexpr uint32_t kDropLog = 1u << 18;


}  // namespace pmdfc
