// bucket.hip -- the batched Insert / mixed path.
//
// Two launches per batch, no host round trip:
//
// 1. k_part: stable partition of the batch's pending ops into 2^p1 buckets by
//    the top p1 local hash bits.  Each 4096-op tile ranks its ops per bucket
//    in batch order (64-lane ballot matching) and appends one RUN per
//    (bucket, tile) to the bucket's record region (atomic cursor; overflow
//    runs go to a shared overflow area).  runpos[bucket][tile] records where
//    each run went, so the bucket kernel can walk a bucket's ops in batch
//    order without any global scan.  Records are SoA: key, value, op index
//    (bit 31 = Get).
//
// 2. k_bucket: ONE WORKGROUP PER BUCKET.  A bucket owns a contiguous range of
//    the directory (its sub-directory, cceh_device.h "Bucketed directory")
//    and every segment in it, so it can apply its ops, split full segments
//    and deepen its sub-directory without coordinating with anyone
//    (CCEH splits are segment-local, CCEH_hybrid.cpp:171-297).  Per chunk of
//    <= 1024 ops, in batch order, it loops rounds:
//      a. sort the pending ops by (segment, batch position) -- LDS bitonic;
//      b. one lane per segment run applies the run's ops in batch order
//         against the segment's occupancy bitmap (LDS copy): an Insert takes
//         the first free slot of its 32-slot window (CCEH_hybrid.cpp:143-168)
//         and stores the pair at once; a Get probes the segment, which already
//         holds the run's earlier inserts.  A full window stops the run: the
//         segment is queued for a split, the rest of the run waits;
//      c. if the queued splits need a deeper sub-directory, grow it (new pool
//         region, new[i] = old[i >> k], CCEH_hybrid.cpp:208-219);
//      d. one wave per queued segment: Segment::Split's slot-order replay
//         (CCEH_hybrid.cpp:18-66) and the directory stride update (:243-286).
//    until no op of the chunk is pending.  Every round either finishes ops or
//    deepens a segment, so it terminates (depth is capped at 30).
#include "cceh_device.h"
#include "cceh_kernels.h"

namespace pmdfc {

constexpr int kPartThreads = 256;
constexpr int kPartWaves = kPartThreads / 64;
constexpr int kPartPerWave = kPartTile / kPartWaves;  // 1024 consecutive ops per wave
constexpr int kPartSteps = kPartPerWave / 64;

constexpr int kBT = 256;              // threads per bucket workgroup
constexpr int kBW = kBT / 64;         // waves per bucket workgroup
constexpr int kChunk = 1024;          // ops per chunk (LDS)
constexpr int kRoundGuard = 64;

constexpr uint32_t kGetBit = 0x80000000u;

// --------------------------------------------------------------- partition

struct PartArgs {
  const uint64_t* keys;
  const uint64_t* vin;
  const uint8_t* ops;   // null: insert-only batch (k_part resolves statuses itself)
  uint8_t* st;
  uint64_t n;
  uint32_t sbits, shard, p1, nblk;
  uint32_t cap;         // record slots per bucket region
  uint64_t ovf_base;    // first overflow record slot
  uint64_t* rkey;
  uint64_t* rval;
  uint32_t* rop;
  uint32_t* cursor;     // per bucket, zero on entry (k_bucket resets it)
  uint2* runpos;        // [bucket][tile] = {first record, count}
  DevCtl* ctl;
};

__global__ __launch_bounds__(kPartThreads) void k_part(PartArgs a) {
  __shared__ uint16_t s_w[kPartWaves][1u << kMaxP1];  // per-wave running count, later exclusive offset
  __shared__ uint32_t s_base[1u << kMaxP1];
  const uint32_t nb = 1u << a.p1;
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  for (uint32_t i = threadIdx.x; i < kPartWaves * nb; i += kPartThreads) s_w[i / nb][i % nb] = 0;
  __syncthreads();
  const uint64_t lt = (1ULL << lane) - 1;
  const uint64_t base = (uint64_t)blockIdx.x * kPartTile + (uint64_t)wv * kPartPerWave;
  uint64_t kk[kPartSteps], vv[kPartSteps];
  uint32_t bk[kPartSteps], rk[kPartSteps], opw[kPartSteps];
  // issue every load of the tile first (16 independent 8-B loads per lane)
#pragma unroll
  for (int k = 0; k < kPartSteps; ++k) {
    const uint64_t p = base + (uint64_t)k * 64 + lane;
    kk[k] = p < a.n ? a.keys[p] : kInvalid;
  }
#pragma unroll
  for (int k = 0; k < kPartSteps; ++k) {
    const uint64_t p = base + (uint64_t)k * 64 + lane;
    bool part = false;
    uint32_t b = 0;
    opw[k] = (uint32_t)p;
    vv[k] = 0;
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
        part = a.st[p] == kStPending;
        if (part && a.ops[p] != 1) opw[k] |= kGetBit;  // anything but PMDFC_OP_INSERT is a Get
      }
      b = bucket_of(h, a.sbits, a.p1);
      if (part && !(opw[k] & kGetBit)) vv[k] = a.vin[p];
    }
    uint64_t mm = __ballot(part);
    for (uint32_t bit = 0; bit < a.p1; ++bit) {
      const uint64_t bb = __ballot((b >> bit) & 1u);
      mm &= ((b >> bit) & 1u) ? bb : ~bb;
    }
    uint32_t rank = 0;
    if (part) {
      rank = s_w[wv][b] + (uint32_t)__popcll(mm & lt);
      if ((mm >> lane) == 1ULL) s_w[wv][b] = (uint16_t)(s_w[wv][b] + __popcll(mm));
    }
    bk[k] = part ? b : 0xFFFFFFFFu;
    rk[k] = rank;
  }
  __syncthreads();
  // one run per non-empty bucket: reserve it, publish it, turn counts into offsets
  for (uint32_t b = threadIdx.x; b < nb; b += kPartThreads) {
    uint32_t c[kPartWaves], tot = 0;
#pragma unroll
    for (int w = 0; w < kPartWaves; ++w) {
      c[w] = s_w[w][b];
      tot += c[w];
    }
    uint64_t at = 0;
    if (tot) {
      const uint32_t pos = atomicAdd(&a.cursor[b], tot);
      if ((uint64_t)pos + tot <= a.cap) at = (uint64_t)b * a.cap + pos;
      else at = a.ovf_base + atomicAdd(&a.ctl->ovf_cur, tot);
    }
    a.runpos[(size_t)b * a.nblk + blockIdx.x] = make_uint2((uint32_t)at, tot);
    s_base[b] = (uint32_t)at;
    uint32_t acc = 0;
#pragma unroll
    for (int w = 0; w < kPartWaves; ++w) {
      s_w[w][b] = (uint16_t)acc;
      acc += c[w];
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kPartSteps; ++k) {
    const uint32_t b = bk[k];
    if (b == 0xFFFFFFFFu) continue;
    const uint64_t dst = (uint64_t)s_base[b] + s_w[wv][b] + rk[k];
    a.rkey[dst] = kk[k];
    a.rval[dst] = vv[k];
    a.rop[dst] = opw[k];
  }
}

// ------------------------------------------------------------------ helpers

// exclusive scan of one value per thread over the workgroup (kBT threads)
__device__ __forceinline__ uint32_t wg_excl_scan(uint32_t v, uint32_t* s_tmp, uint32_t* total) {
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  uint32_t incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = (uint32_t)__shfl_up((int)incl, o);
    if (lane >= (uint32_t)o) incl += t;
  }
  if (lane == 63) s_tmp[wv] = incl;
  __syncthreads();
  uint32_t before = 0, all = 0;
#pragma unroll
  for (int w = 0; w < kBW; ++w) {
    const uint32_t t = s_tmp[w];
    if ((uint32_t)w < wv) before += t;
    all += t;
  }
  __syncthreads();  // s_tmp reuse
  *total = all;
  return before + incl - v;
}

// ascending bitonic sort of s[0..n), n a power of two
__device__ __forceinline__ void wg_bitonic(uint64_t* s, uint32_t n) {
  for (uint32_t k = 2; k <= n; k <<= 1) {
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      for (uint32_t t = threadIdx.x; t < n / 2; t += kBT) {
        const uint32_t i = 2 * t - (t & (j - 1));
        const uint32_t l = i + j;
        const uint64_t x = s[i], y = s[l];
        const bool up = (i & k) == 0;
        if ((x > y) == up) {
          s[i] = y;
          s[l] = x;
        }
      }
      __syncthreads();
    }
  }
}

// Segment::Split (non-INPLACE, CCEH_hybrid.cpp:47-66) of `seg` at local depth
// L into seg (child 0, reusing the parent's storage) and c1, by one wave.
// Every lane holds 16 parent slots in registers; wave_replay computes the
// exact slot-order placement; then each child slot is written exactly once
// (an entry or INVALID).  Returns the number of dropped entries (lane 0).
__device__ uint32_t wave_split(ulonglong2* __restrict__ pairs, uint32_t* __restrict__ occ,
                               uint8_t* __restrict__ ldep, uint32_t seg, uint32_t c1, uint32_t L,
                               uint32_t* s_b, uint32_t* s_cb, uint32_t* s_col) {
  const uint32_t lane = __lane_id() & 63u;
  ulonglong2* sp = pairs + (size_t)seg * kSlots;
  ulonglong2* s1 = pairs + (size_t)c1 * kSlots;
  ulonglong2 pr[16];
  uint32_t inf[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) pr[j] = ld_pair_l2(sp + j * 64 + lane);
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const bool valid = pr[j].x != kInvalid;
    const uint64_t kh = hash64(pr[j].x);
    // bit 31 valid, bit 8 child (hash bit 63-L, CCEH_hybrid.cpp:52-55), bits 0-7 home line
    inf[j] = (valid ? 0x80000000u : 0u) | ((uint32_t)((kh >> (63 - L)) & 1u) << 8) |
             (uint32_t)(kh & 0xFF);
  }
  s_b[lane] = 0;
  __builtin_amdgcn_wave_barrier();
  uint32_t dest[16];
  uint32_t loss = wave_replay(inf, dest, s_b, s_cb, s_col);
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const uint32_t d = dest[j];
    if (d != 0xFFFFFFFFu) ((d >> 10) ? s1 : sp)[d & 1023u] = pr[j];
  }
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    ulonglong2* dst = c ? s1 : sp;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const uint32_t slot = (uint32_t)j * 64u + lane;
      const uint32_t w = s_b[c * 32u + (slot >> 5)];
      if (!((w >> (slot & 31u)) & 1u)) dst[slot] = make_ulonglong2(kInvalid, 0ULL);
    }
  }
  const uint32_t bw = s_b[lane];  // lanes 0-31 child-0 words, 32-63 child-1 words
  if (lane < 32) occ[(size_t)seg * 32u + lane] = bw;
  else occ[(size_t)c1 * 32u + (lane - 32)] = bw;
  if (lane == 0) {
    ldep[seg] = (uint8_t)(L + 1);
    ldep[c1] = (uint8_t)(L + 1);
  }
  for (int o = 32; o > 0; o >>= 1) loss += (uint32_t)__shfl_down((int)loss, o);
  return loss;
}

// ------------------------------------------------------------------ bucket

struct BucketArgs {
  const uint64_t* rkey;
  const uint64_t* rval;
  const uint32_t* rop;
  const uint2* runpos;
  uint32_t nblk;
  uint32_t chunk;       // ops per chunk (<= kChunk)
  uint32_t* cursor;
  uint64_t* hdr;
  uint32_t* pool;
  uint32_t pool_cap;
  uint32_t p1, sbits;
  ulonglong2* pairs;
  uint32_t* occ;
  uint8_t* ldep;
  uint64_t* vout;       // mixed only
  uint8_t* st;
  uint32_t mixed;
  uint32_t max_segments;
  DevCtl* ctl;
};

// run table of bucket b in tile (= batch) order: s_rpos[k] = first record of
// tile k's run, s_rpre[k] = ops in runs 0..k-1, s_rpre[nblk] = total
__device__ __forceinline__ uint32_t load_runs(const BucketArgs& a, uint32_t b, uint32_t* s_rpos,
                                              uint32_t* s_rpre, uint32_t* s_tmp) {
  const uint32_t tid = threadIdx.x;
  uint32_t lens[4] = {0, 0, 0, 0}, mysum = 0;
  const uint32_t per = (a.nblk + kBT - 1) / kBT;  // <= 4
  for (uint32_t j = 0; j < per; ++j) {
    const uint32_t k = tid * per + j;
    if (k < a.nblk) {
      const uint2 rp = a.runpos[(size_t)b * a.nblk + k];
      s_rpos[k] = rp.x;
      lens[j] = rp.y;
      mysum += rp.y;
    }
  }
  uint32_t total;
  uint32_t acc = wg_excl_scan(mysum, s_tmp, &total);
  for (uint32_t j = 0; j < per; ++j) {
    const uint32_t k = tid * per + j;
    if (k < a.nblk) s_rpre[k] = acc;
    acc += lens[j];
  }
  if (tid == 0) s_rpre[a.nblk] = total;
  __syncthreads();
  return total;
}

// LDS union, phase by phase: chunk gather (run table), run phase (one
// 33-word occupancy bitmap per lane), split phase (3 x 64 words per wave)
constexpr uint32_t kUnionWords = kBT * 33 > 2 * kMaxPartBlocks + 1 ? kBT * 33 : 2 * kMaxPartBlocks + 1;

__global__ __launch_bounds__(kBT, 2) void k_bucket(BucketArgs a) {
  __shared__ uint64_t s_key[kChunk];
  __shared__ uint64_t s_val[kChunk];
  __shared__ uint32_t s_op[kChunk];
  __shared__ uint64_t s_sk[kChunk];
  __shared__ uint64_t s_split[kChunk];
  __shared__ uint16_t s_runq[kChunk + 1];
  __shared__ uint8_t s_pend[kChunk];
  __shared__ uint32_t s_u[kUnionWords];
  __shared__ uint32_t s_tmp[kBW];
  __shared__ uint32_t s_off, s_db, s_nsplit, s_need, s_fail;
  uint32_t* const s_rpos = s_u;
  uint32_t* const s_rpre = s_u + kMaxPartBlocks;

  const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
  const uint32_t b = blockIdx.x;
  if (tid == 0) {
    a.cursor[b] = 0;  // partition cursors are consumed: ready for the next batch
    if (b == 0) a.ctl->ovf_cur = 0;
    const uint64_t hd = a.hdr[b];
    s_off = hdr_off(hd);
    s_db = hdr_db(hd);
  }
  const uint32_t total = load_runs(a, b, s_rpos, s_rpre, s_tmp);
  if (total == 0) return;

  uint32_t c_runs = 0, c_rounds = 0, c_waited = 0, c_lines = 0, c_splits = 0, c_loss = 0, c_grow = 0;
  uint32_t c_maxr = 0;
  uint32_t my_max_ld = 0;
  const uint32_t C = a.chunk;
  for (uint32_t cs = 0; cs < total; cs += C) {
    const uint32_t m = min(C, total - cs);
    if (cs) load_runs(a, b, s_rpos, s_rpre, s_tmp);  // the union was reused
    // ---- gather the chunk (records of consecutive runs, batch order)
    for (uint32_t i = tid; i < m; i += kBT) {
      const uint32_t g = cs + i;
      uint32_t lo = 0, hi = a.nblk;  // last k with s_rpre[k] <= g
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (s_rpre[mid] <= g) lo = mid;
        else hi = mid;
      }
      const uint64_t pos = (uint64_t)s_rpos[lo] + (g - s_rpre[lo]);
      s_key[i] = a.rkey[pos];
      s_val[i] = a.rval[pos];
      s_op[i] = a.rop[pos];
      s_pend[i] = 1;
    }
    __syncthreads();
    for (uint32_t round = 0;; ++round) {
      // ---- a. sort keys of the pending ops: (segment, L, chunk position)
      const uint32_t per_t = (m + kBT - 1) / kBT;
      uint32_t cnt = 0;
      for (uint32_t j = 0; j < per_t; ++j) {
        const uint32_t i = tid * per_t + j;
        if (i < m && s_pend[i]) ++cnt;
      }
      uint32_t np;
      uint32_t at = wg_excl_scan(cnt, s_tmp, &np);
      if (np == 0) break;
      if (round >= kRoundGuard) {
        // cannot happen (depth is bounded); fail loudly rather than spin
        for (uint32_t i = tid; i < m; i += kBT)
          if (s_pend[i]) {
            a.st[s_op[i] & ~kGetBit] = 6;
            s_pend[i] = 0;
          }
        if (tid == 0) atomicOr(&a.ctl->err, 2u);
        __syncthreads();
        break;
      }
      ++c_rounds;
      const uint32_t off = s_off, db = s_db;
      for (uint32_t j = 0; j < per_t; ++j) {
        const uint32_t i = tid * per_t + j;
        if (i < m && s_pend[i]) {
          const uint64_t h = hash64(s_key[i]);
          const uint32_t e = ld_u32_l2(a.pool + off + sub_index(h, a.sbits, a.p1, db));
          s_sk[at++] = ((uint64_t)de_seg(e) << 21) | ((uint64_t)de_ld(e) << 16) | i;
        }
      }
      uint32_t p2 = 1;
      while (p2 < np) p2 <<= 1;
      for (uint32_t j = np + tid; j < p2; j += kBT) s_sk[j] = ~0ULL;
      __syncthreads();
      if (p2 > 1) wg_bitonic(s_sk, p2);
      // ---- runs: maximal stretches with one segment
      const uint32_t per_q = (np + kBT - 1) / kBT;
      uint32_t rc = 0;
      for (uint32_t j = 0; j < per_q; ++j) {
        const uint32_t q = tid * per_q + j;
        if (q < np && (q == 0 || (s_sk[q] >> 21) != (s_sk[q - 1] >> 21))) ++rc;
      }
      uint32_t nruns;
      uint32_t rat = wg_excl_scan(rc, s_tmp, &nruns);
      for (uint32_t j = 0; j < per_q; ++j) {
        const uint32_t q = tid * per_q + j;
        if (q < np && (q == 0 || (s_sk[q] >> 21) != (s_sk[q - 1] >> 21))) s_runq[rat++] = (uint16_t)q;
      }
      if (tid == 0) {
        s_runq[nruns] = (uint16_t)np;
        s_nsplit = 0;
        s_need = db;
        s_fail = 0;
      }
      __syncthreads();
      c_runs += (tid == 0) ? nruns : 0;
      // ---- b. one lane per run, in batch order
      uint32_t* bm = s_u + tid * 33u;
      for (uint32_t r = tid; r < nruns; r += kBT) {
        const uint32_t q0 = s_runq[r], q1 = s_runq[r + 1];
        const uint64_t sk0 = s_sk[q0];
        const uint32_t seg = (uint32_t)(sk0 >> 21);
        const uint32_t L = (uint32_t)(sk0 >> 16) & 31u;
        const uint32_t* og = a.occ + (size_t)seg * 32u;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint4 v = ld_u4_l2(og + 4 * j);
          bm[4 * j] = v.x;
          bm[4 * j + 1] = v.y;
          bm[4 * j + 2] = v.z;
          bm[4 * j + 3] = v.w;
        }
        ulonglong2* sp = a.pairs + (size_t)seg * kSlots;
        bool dirty = false;
        for (uint32_t q = q0; q < q1; ++q) {
          const uint32_t i = (uint32_t)s_sk[q] & 0xFFFFu;
          const uint64_t key = s_key[i];
          const uint32_t ow = s_op[i];
          const uint32_t op = ow & ~kGetBit;
          const uint64_t h = hash64(key);
          if (ow & kGetBit) {
            uint64_t val = 0;
            const uint8_t s = lane_probe(sp, key, h, &val);
            a.vout[op] = val;
            a.st[op] = s;
            s_pend[i] = 0;
            continue;
          }
          const uint32_t w = (uint32_t)(h & 0xFF) * 4u;
          const uint32_t wi = w >> 5;
          const int pos = window_first_free(bm[wi], bm[(wi + 1) & 31u], w);
          if (pos >= 0) {
            bm[(uint32_t)pos >> 5] |= 1u << ((uint32_t)pos & 31u);
            dirty = true;
            sp[pos] = make_ulonglong2(key, s_val[i]);
            if (a.mixed) a.st[op] = 2;  // PMDFC_ST_INSERTED (insert-only batches: preset by k_part)
            c_lines += ((((uint32_t)pos - w) & (kSlots - 1)) >> 2) + 1;
            s_pend[i] = 0;
            continue;
          }
          // window full.  The reference would split forever if all 32 entries
          // carry this key's full hash: UNSPLITTABLE.
          bool same = true;
          for (uint32_t t = 0; t < kWindow && same; ++t)
            same = hash64(ld_pair_l2(sp + ((w + t) & (kSlots - 1))).x) == h;
          uint8_t code = 0;
          uint32_t c1 = 0;
          if (same) {
            code = 4;  // PMDFC_ST_UNSPLITTABLE
          } else if (L + 1 > kMaxDepth) {
            code = 5;  // PMDFC_ST_DEPTH_LIMIT
          } else {
            c1 = atomicAdd(&a.ctl->nsegs, 1u);
            if (c1 >= a.max_segments) code = 6;  // PMDFC_ST_CAPACITY
          }
          if (code) {
            a.st[op] = code;
            s_pend[i] = 0;
            continue;
          }
          const uint32_t si = atomicAdd(&s_nsplit, 1u);
          s_split[si] = (uint64_t)i | ((uint64_t)L << 16) | ((uint64_t)c1 << 21);
          atomicMax(&s_need, L + 1 - a.sbits - a.p1);
          c_waited += q1 - q;
          break;  // the rest of the run waits for the split
        }
        if (dirty) {
          uint32_t* o = a.occ + (size_t)seg * 32u;
#pragma unroll
          for (int j = 0; j < 8; ++j)
            *reinterpret_cast<uint4*>(o + 4 * j) = make_uint4(bm[4 * j], bm[4 * j + 1], bm[4 * j + 2], bm[4 * j + 3]);
        }
      }
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
      const uint32_t ns = s_nsplit;
      if (ns == 0) continue;  // every pending op resolved (or failed) this round
      // ---- c. deepen the sub-directory if a child needs more bits
      if (s_need > db) {
        const uint32_t nd = s_need;
        const uint32_t size = 1u << nd;
        if (tid == 0) {
          const uint32_t no = atomicAdd(&a.ctl->pool_cur, size);
          if ((uint64_t)no + size > a.pool_cap) {
            s_fail = 1;
            atomicOr(&a.ctl->err, 1u);
          } else {
            s_tmp[0] = no;
          }
        }
        __syncthreads();
        if (s_fail) {
          // sub-directory pool exhausted: the blocked ops fail (CAPACITY)
          for (uint32_t s = tid; s < ns; s += kBT) {
            const uint32_t i = (uint32_t)s_split[s] & 0xFFFFu;
            a.st[s_op[i] & ~kGetBit] = 6;
            s_pend[i] = 0;
          }
          __syncthreads();
          continue;
        }
        const uint32_t no = s_tmp[0];
        const uint32_t sh = nd - db;
        for (uint32_t t = tid; t < size; t += kBT) a.pool[no + t] = ld_u32_l2(a.pool + off + (t >> sh));
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
        if (tid == 0) {
          s_off = no;
          s_db = nd;
          a.hdr[b] = hdr_make(no, nd);
          ++c_grow;
        }
        __syncthreads();
      }
      // ---- d. splits, one wave per queued segment
      {
        const uint32_t off2 = s_off, db2 = s_db;
        uint32_t* scr = s_u + wv * 192u;
        for (uint32_t s = wv; s < ns; s += kBW) {
          const uint64_t e = s_split[s];
          const uint32_t i = (uint32_t)e & 0xFFFFu;
          const uint32_t L = (uint32_t)(e >> 16) & 31u;
          const uint32_t c1 = (uint32_t)(e >> 21);
          const uint64_t h = hash64(s_key[i]);
          const uint32_t x = sub_index(h, a.sbits, a.p1, db2);
          const uint32_t seg = de_seg(ld_u32_l2(a.pool + off2 + x));
          const uint32_t loss = wave_split(a.pairs, a.occ, a.ldep, seg, c1, L, scr, scr + 64, scr + 128);
          // directory: the 2^(db-Lb) entries of the parent; first half keeps
          // child 0 (the parent's id), second half gets child 1
          const uint32_t Lb = L - a.sbits - a.p1;
          const uint32_t span = 1u << (db2 - Lb);
          const uint32_t xs = x & ~(span - 1u);
          for (uint32_t t = lane; t < span; t += 64)
            a.pool[off2 + xs + t] = de_make(t < span / 2 ? seg : c1, L + 1);
          if (lane == 0) {
            ++c_splits;
            c_loss += loss;
            my_max_ld = max(my_max_ld, L + 1);
            atomicSub(&a.ctl->depth_count[L], 1u);
            atomicAdd(&a.ctl->depth_count[L + 1], 2u);
          }
        }
      }
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
    }
    c_maxr = max(c_maxr, c_rounds);
    __syncthreads();
  }
  // ---- counters (one atomic per wave)
  for (int o = 32; o > 0; o >>= 1) {
    c_lines += (uint32_t)__shfl_down((int)c_lines, o);
    c_waited += (uint32_t)__shfl_down((int)c_waited, o);
    c_splits += (uint32_t)__shfl_down((int)c_splits, o);
    c_loss += (uint32_t)__shfl_down((int)c_loss, o);
    my_max_ld = max(my_max_ld, (uint32_t)__shfl_down((int)my_max_ld, o));
  }
  if (lane == 0) {
    if (c_lines) atomicAdd((unsigned long long*)&a.ctl->ins_lines, (unsigned long long)c_lines);
    if (c_waited) atomicAdd((unsigned long long*)&a.ctl->waited, (unsigned long long)c_waited);
    if (c_splits) atomicAdd((unsigned long long*)&a.ctl->splits, (unsigned long long)c_splits);
    if (c_loss) atomicAdd((unsigned long long*)&a.ctl->split_loss, (unsigned long long)c_loss);
    if (my_max_ld) atomicMax(&a.ctl->max_ld, my_max_ld);
  }
  if (tid == 0) {
    atomicAdd((unsigned long long*)&a.ctl->runs, (unsigned long long)c_runs);
    atomicAdd((unsigned long long*)&a.ctl->rounds, (unsigned long long)c_rounds);
    if (c_grow) atomicAdd((unsigned long long*)&a.ctl->growths, (unsigned long long)c_grow);
    atomicMax(&a.ctl->max_rounds, c_maxr);
  }
}

// ------------------------------------------------------------- launchers

uint32_t part_blocks(uint64_t n) { return (uint32_t)((n + kPartTile - 1) / kPartTile); }

void launch_part(const PartLaunch& L, hipStream_t s) {
  if (!L.n) return;
  PartArgs a;
  a.keys = L.keys;
  a.vin = L.vin;
  a.ops = L.ops;
  a.st = L.st;
  a.n = L.n;
  a.sbits = L.sbits;
  a.shard = L.shard;
  a.p1 = L.p1;
  a.nblk = part_blocks(L.n);
  a.cap = L.cap;
  a.ovf_base = (uint64_t)L.cap << L.p1;
  a.rkey = L.rkey;
  a.rval = L.rval;
  a.rop = L.rop;
  a.cursor = L.cursor;
  a.runpos = L.runpos;
  a.ctl = L.ctl;
  hipLaunchKernelGGL(k_part, dim3(a.nblk), dim3(kPartThreads), 0, s, a);
}

void launch_bucket(const BucketLaunch& L, hipStream_t s) {
  if (!L.n) return;
  BucketArgs a;
  a.rkey = L.rkey;
  a.rval = L.rval;
  a.rop = L.rop;
  a.runpos = L.runpos;
  a.nblk = part_blocks(L.n);
  a.chunk = (L.chunk == 0 || L.chunk > (uint32_t)kChunk) ? (uint32_t)kChunk : L.chunk;
  a.cursor = L.cursor;
  a.hdr = L.hdr;
  a.pool = L.pool;
  a.pool_cap = L.pool_cap;
  a.p1 = L.p1;
  a.sbits = L.sbits;
  a.pairs = L.pairs;
  a.occ = L.occ;
  a.ldep = L.ldep;
  a.vout = L.vout;
  a.st = L.st;
  a.mixed = L.mixed;
  a.max_segments = L.max_segments;
  a.ctl = L.ctl;
  hipLaunchKernelGGL(k_bucket, dim3(1u << L.p1), dim3(kBT), 0, s, a);
}

}  // namespace pmdfc
