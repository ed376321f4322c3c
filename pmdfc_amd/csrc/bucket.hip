// bucket.hip -- single-launch batched insert/mixed path (the fast path).
//
// 1. k_part_hist / exclusive scan / k_part_scatter: stable partition of the
//    pending ops into 2^P1 buckets by the top P1 local hash bits.  With P1 <=
//    (min local depth - shard bits) every segment lies inside one bucket, so a
//    bucket is an independent sub-problem (CCEH splits are segment-local,
//    CCEH_hybrid.cpp:171-297).
// 2. k_bucket: one workgroup per bucket.  It keeps the bucket's directory
//    slice in LDS and walks the bucket's ops in batch order, chunk by chunk;
//    per round: stable LDS counting sort of the pending ops by directory
//    index, one lane per segment run applies inserts in batch order on the
//    segment's occupancy bitmap (LDS), Gets are resolved against the pre-round
//    image plus earlier inserts of the run, slots are written, and full
//    segments are split in place by a whole wave (slot-order replay,
//    CCEH_hybrid.cpp:18-67) with the directory slice updated -- no host round
//    trip.  Only a split that needs a global directory doubling defers the rest
//    of that segment's ops to the host-driven pass (engine).
#include "cceh_device.h"
#include "cceh_kernels.h"

namespace pmdfc {

constexpr int kPartThreads = 256;
constexpr int kPartItems = 16;
constexpr int kPartTile = kPartThreads * kPartItems;  // 4096 ops per partition block
constexpr int kMaxP1 = 12;                            // <= 4096 buckets

constexpr int kBT = 128;                              // k_bucket threads (2 waves)
constexpr int kChunk = 512;                           // ops per chunk
constexpr int kMaxBins = 1024;                        // directory slice per bucket

__device__ __forceinline__ uint32_t bucket_of(uint64_t h, uint32_t sbits, uint32_t p1) {
  return (uint32_t)((h << sbits) >> (64 - p1));
}

__device__ __forceinline__ uint64_t ld_sc1_u64(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_sc1_u32(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------- partition

__device__ __forceinline__ bool part_item(uint64_t p, uint64_t npend, const uint32_t* pend,
                                          const uint8_t* st, uint32_t* op) {
  if (p >= npend) return false;
  *op = pend ? pend[p] : (uint32_t)p;
  return st[*op] == kStPending;
}

__global__ __launch_bounds__(kPartThreads) void k_part_hist(
    const uint32_t* __restrict__ pend, const uint32_t* __restrict__ npend_dev, uint64_t npend_host,
    const uint8_t* __restrict__ st, const uint64_t* __restrict__ hbuf, uint32_t sbits, uint32_t p1,
    uint32_t nblk, uint32_t* __restrict__ hist) {
  __shared__ uint32_t s_h[1 << kMaxP1];
  const uint32_t nb = 1u << p1;
  for (uint32_t i = threadIdx.x; i < nb; i += kPartThreads) s_h[i] = 0;
  __syncthreads();
  const uint64_t npend = npend_dev ? *npend_dev : npend_host;
  const uint64_t base = (uint64_t)blockIdx.x * kPartTile;
  for (int k = 0; k < kPartItems; ++k) {
    const uint64_t p = base + (uint64_t)k * kPartThreads + threadIdx.x;
    uint32_t op;
    if (part_item(p, npend, pend, st, &op)) atomicAdd(&s_h[bucket_of(hbuf[op], sbits, p1)], 1u);
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < nb; i += kPartThreads) hist[(size_t)i * nblk + blockIdx.x] = s_h[i];
}

// Stable scatter: each wave ranks a contiguous quarter of the tile in order
// (64-lane match by ballots over the bucket bits + a per-wave running count in
// LDS), then adds the counts of the earlier waves of the block.
__global__ __launch_bounds__(kPartThreads) void k_part_scatter(
    const uint32_t* __restrict__ pend, const uint32_t* __restrict__ npend_dev, uint64_t npend_host,
    const uint8_t* __restrict__ st, const uint64_t* __restrict__ hbuf, uint32_t sbits, uint32_t p1,
    uint32_t nblk, const uint32_t* __restrict__ hist, const uint32_t* __restrict__ inc,
    uint64_t* __restrict__ ph, uint32_t* __restrict__ pop) {
  __shared__ uint16_t s_w[4][1 << kMaxP1];  // per-wave running count per bucket
  const uint32_t nb = 1u << p1;
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  for (uint32_t i = threadIdx.x; i < 4 * nb; i += kPartThreads) s_w[i / nb][i % nb] = 0;
  __syncthreads();
  const uint64_t npend = npend_dev ? *npend_dev : npend_host;
  const uint64_t base = (uint64_t)blockIdx.x * kPartTile + (uint64_t)wv * (kPartTile / 4);
  const uint64_t lt = (1ULL << lane) - 1;
  uint32_t bk[kPartItems], rk[kPartItems], opv[kPartItems];
#pragma unroll
  for (int k = 0; k < kPartItems; ++k) {
    const uint64_t p = base + (uint64_t)k * 64 + lane;
    uint32_t op = 0;
    const bool v = part_item(p, npend, pend, st, &op);
    const uint32_t b = v ? bucket_of(hbuf[op], sbits, p1) : 0xFFFFu;
    uint64_t mm = __ballot(v);
    for (uint32_t bit = 0; bit < p1; ++bit) {
      const uint64_t bb = __ballot((b >> bit) & 1u);
      mm &= ((b >> bit) & 1u) ? bb : ~bb;
    }
    uint32_t r = 0;
    if (v) {
      r = s_w[wv][b] + (uint32_t)__popcll(mm & lt);
      // the highest matching lane updates the running count (no other lane of
      // this wave touches bucket b in this step)
      if ((mm >> lane) == 1ULL) s_w[wv][b] = (uint16_t)(s_w[wv][b] + __popcll(mm));
    }
    bk[k] = b;
    rk[k] = r;
    opv[k] = op;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kPartItems; ++k) {
    const uint32_t b = bk[k];
    if (b == 0xFFFFu) continue;
    uint32_t add = 0;
    for (uint32_t w = 0; w < wv; ++w) add += s_w[w][b];
    const size_t hi = (size_t)b * nblk + blockIdx.x;
    const uint32_t dst = inc[hi] - hist[hi] + add + rk[k];
    ph[dst] = hbuf[opv[k]];
    pop[dst] = opv[k];
  }
}

// ------------------------------------------------------------- wave split
// Segment::Split (non-INPLACE, CCEH_hybrid.cpp:47-66) by one full wave.  Reads
// the parent with L1-bypassing loads (this workgroup may have just written it),
// replays slots 0..1023 in order into two child bitmaps held in one VGPR
// (lanes 0-31 child 0, 32-63 child 1), then scatters the entries to their
// child slots and fills the rest with INVALID: every child slot is written
// exactly once.  Child 0 reuses the parent's storage.  Returns entries lost.
__device__ uint32_t wave_split(ulonglong2* __restrict__ pairs, uint32_t* __restrict__ occ,
                               uint8_t* __restrict__ ldep, uint32_t seg, uint32_t c1, uint32_t L) {
  const uint32_t lane = __lane_id();
  const uint64_t* src = reinterpret_cast<const uint64_t*>(pairs + (size_t)seg * kSlots);
  uint64_t pk[16], pv[16];
  uint32_t inf[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const uint32_t slot = (uint32_t)j * 64u + lane;
    pk[j] = ld_sc1_u64(src + 2 * slot);
    pv[j] = ld_sc1_u64(src + 2 * slot + 1);
  }
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const uint64_t kh = hash64(pk[j]);
    inf[j] = (pk[j] != kInvalid ? 0x80000000u : 0u) | ((uint32_t)((kh >> (63 - L)) & 1u) << 8) |
             (uint32_t)(kh & 0xFF);
  }
  uint32_t b = 0, loss = 0;
  uint32_t dest[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    uint32_t d = 0xFFFFFFFFu;
    uint64_t vm = __ballot((inf[j] & 0x80000000u) != 0);
    while (vm) {
      const int l = __builtin_ctzll(vm);
      vm &= vm - 1;
      const uint32_t si = (uint32_t)__builtin_amdgcn_readlane((int)inf[j], l);
      const uint32_t c = (si >> 8) & 1u;
      const uint32_t w = (si & 0xFFu) * 4u;
      const uint32_t wi = w >> 5;
      const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)b, (int)(c * 32u + wi));
      const uint32_t hi =
          (uint32_t)__builtin_amdgcn_readlane((int)b, (int)(c * 32u + ((wi + 1u) & 31u)));
      const int pos = window_first_free(lo, hi, w);
      if (pos < 0) {
        ++loss;
        continue;
      }
      const uint32_t wsel = (uint32_t)pos >> 5;
      const uint32_t nw = ((wsel == wi) ? lo : hi) | (1u << ((uint32_t)pos & 31u));
      b = (lane == c * 32u + wsel) ? nw : b;
      d = (lane == (uint32_t)l) ? ((c << 10) | (uint32_t)pos) : d;
    }
    dest[j] = d;
  }
  ulonglong2* c0p = pairs + (size_t)seg * kSlots;
  ulonglong2* c1p = pairs + (size_t)c1 * kSlots;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const uint32_t d = dest[j];
    if (d != 0xFFFFFFFFu) ((d >> 10) ? c1p : c0p)[d & 1023u] = make_ulonglong2(pk[j], pv[j]);
  }
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    ulonglong2* cp = c ? c1p : c0p;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const uint32_t slot = (uint32_t)j * 64u + lane;
      const uint32_t word = (uint32_t)__shfl((int)b, (int)(c * 32u + (slot >> 5)));
      if (!((word >> (slot & 31u)) & 1u)) cp[slot] = make_ulonglong2(kInvalid, 0ULL);
    }
  }
  if (lane < 32) occ[(size_t)seg * 32u + lane] = b;
  else occ[(size_t)c1 * 32u + (lane - 32)] = b;
  if (lane == 0) {
    ldep[seg] = (uint8_t)(L + 1);
    ldep[c1] = (uint8_t)(L + 1);
  }
  return loss;
}

// ---------------------------------------------------------------- bucket

struct BucketArgs {
  const uint64_t* ph;
  const uint32_t* pop;
  const uint32_t* offs;      // inclusive scan of the bucket-major partition histogram
  uint32_t nblk;             // partition blocks (offs row length)
  uint32_t p1, bbits;        // bucket bits, directory-slice bits
  uint32_t gdepth, sbits;
  const uint8_t* ops;        // null: all inserts
  const uint64_t* keys;
  const uint64_t* vin;
  uint64_t* vout;
  uint8_t* st;
  ulonglong2* pairs;
  uint32_t* occ;
  uint8_t* ldep;
  uint32_t* dir;
  uint8_t* deferred;         // host-pass flags
  DevCtl* ctl;
  uint32_t max_segments;
  unsigned long long* stamps;  // diagnostic: per-block phase cycles (null = off)
};

// result codes kept per chunk position in s_res
constexpr uint16_t kResPend = 0xFFFF;   // not handled yet
constexpr uint16_t kResGet = 0xFFFE;    // Get inside a processed run prefix
constexpr uint16_t kResDone = 0xFFFD;   // resolved (status written)
constexpr uint16_t kResOvf = 0xFFFC;    // insert that found its window full

__global__ __launch_bounds__(kBT) void k_bucket(BucketArgs a) {
  __shared__ uint32_t s_dir[kMaxBins];
  __shared__ uint8_t s_ld[kMaxBins];
  __shared__ uint8_t s_frozen[kMaxBins];
  __shared__ uint32_t s_base[kMaxBins];    // bin -> start in sorted order
  __shared__ uint32_t s_run[kMaxBins];     // running count per bin (sort)
  __shared__ uint32_t s_w0[kMaxBins];      // wave-0 count per bin, round-stamped
  __shared__ uint64_t s_h[kChunk];
  __shared__ uint32_t s_op[kChunk];
  __shared__ uint16_t s_res[kChunk];
  __shared__ uint16_t s_sorted[kChunk];
  __shared__ uint16_t s_runq[kBT + 1];     // run start (sorted index); [nr] = end
  __shared__ uint16_t s_ovq[kBT];          // overflow sorted index per run (0xFFFF none)
  __shared__ uint8_t s_code[kChunk];
  __shared__ uint32_t s_bm[kBT][33];
  __shared__ uint32_t s_cnt[4];
  __shared__ uint32_t s_defer;
  __shared__ uint32_t s_runs;

  const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
  const uint32_t b = blockIdx.x;
  // diagnostic phase stamps (thread 0): 0 load, 1 sort, 2 runs, 3 seq, 4 gets,
  // 5 writes, 6 split, 7 rounds
  unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long st_last = (a.stamps && tid == 0) ? __builtin_amdgcn_s_memtime() : 0;
#define STAMP(k)                                                      \
  do {                                                                \
    if (a.stamps && tid == 0) {                                       \
      const unsigned long long t_ = __builtin_amdgcn_s_memtime();     \
      st_acc[k] += t_ - st_last;                                      \
      st_last = t_;                                                   \
    }                                                                 \
  } while (0)
  const uint32_t nbins = 1u << a.bbits;
  // a.offs is the INCLUSIVE scan of the bucket-major partition histogram
  const uint64_t beg = b ? a.offs[(size_t)b * a.nblk - 1] : 0;
  const uint64_t end = a.offs[(size_t)(b + 1) * a.nblk - 1];
  if (beg >= end) return;
  const uint32_t xbase = b << a.bbits;
  const uint32_t Dl = a.gdepth - a.sbits;

  for (uint32_t x = tid; x < nbins; x += kBT) {
    s_dir[x] = a.dir[xbase + x];
    s_frozen[x] = 0;
    s_w0[x] = 0;
  }
  if (tid == 0) {
    s_defer = 0;
    s_runs = 0;
  }
  __syncthreads();
  for (uint32_t x = tid; x < nbins; x += kBT) s_ld[x] = a.ldep[s_dir[x]];
  __syncthreads();

  // sort key of chunk position i: the first directory bin of its segment, so
  // that a stable sort keeps every segment's ops in batch order (a segment
  // spans 2^(gdepth - L) consecutive bins)
  auto seg_bin = [&](uint32_t i) -> uint32_t {
    const uint32_t bin = (uint32_t)((s_h[i] << a.sbits) >> (64 - Dl)) & (nbins - 1);
    const uint32_t sb = a.gdepth - s_ld[bin];
    return (bin >> sb) << sb;
  };

  for (uint64_t cs = beg; cs < end; cs += kChunk) {
    const uint32_t m = (uint32_t)min<uint64_t>(kChunk, end - cs);
    uint32_t stamp = 0;
    for (uint32_t x = tid; x < nbins; x += kBT) s_w0[x] = 0;
    for (uint32_t i = tid; i < kChunk; i += kBT) {
      if (i < m) {
        const uint32_t op = a.pop[cs + i];
        s_op[i] = op;
        s_h[i] = a.ph[cs + i];
        s_code[i] = a.ops ? a.ops[op] : (uint8_t)1;
        s_res[i] = kResPend;
      } else {
        s_res[i] = kResDone;
      }
    }
    __syncthreads();

    for (;;) {
      STAMP(0);
      if (a.stamps && tid == 0) st_acc[7] += 1;
      // ---- frozen segments (waiting for a directory doubling): defer
      for (uint32_t i = tid; i < m; i += kBT) {
        if (s_res[i] != kResPend) continue;
        const uint32_t bin = (uint32_t)((s_h[i] << a.sbits) >> (64 - Dl)) & (nbins - 1);
        if (s_frozen[bin]) {
          a.deferred[s_op[i]] = 1;
          s_res[i] = kResDone;
          atomicAdd(&s_defer, 1u);
        }
      }
      // ---- stable counting sort of pending positions by directory bin
      for (uint32_t x = tid; x < nbins; x += kBT) s_run[x] = 0;
      if (tid < 4) s_cnt[tid] = 0;
      __syncthreads();
      for (uint32_t i = tid; i < m; i += kBT)
        if (s_res[i] == kResPend) atomicAdd(&s_run[seg_bin(i)], 1u);
      __syncthreads();
      // exclusive scan of s_run into s_base (one wave, nbins <= 1024)
      if (wv == 0) {
        uint32_t carry = 0;
        for (uint32_t x0 = 0; x0 < nbins; x0 += 64) {
          const uint32_t x = x0 + lane;
          const uint32_t v = x < nbins ? s_run[x] : 0;
          uint32_t inc = v;
          for (int o = 1; o < 64; o <<= 1) {
            const uint32_t t = (uint32_t)__shfl_up((int)inc, o);
            if (lane >= (uint32_t)o) inc += t;
          }
          if (x < nbins) s_base[x] = carry + inc - v;
          carry += (uint32_t)__shfl((int)inc, 63);
        }
        if (lane == 0) s_cnt[0] = carry;  // pending count
      }
      __syncthreads();
      const uint32_t npend = s_cnt[0];
      if (npend == 0) break;
      for (uint32_t x = tid; x < nbins; x += kBT) s_run[x] = 0;
      __syncthreads();
      for (uint32_t r0 = 0; r0 < kChunk; r0 += kBT) {
        const uint32_t i = r0 + tid;
        const bool v = i < m && s_res[i] == kResPend;
        const uint32_t bin = v ? seg_bin(i) : 0u;
        uint64_t mm = __ballot(v);
        for (uint32_t bit = 0; bit < a.bbits; ++bit) {
          const uint64_t bb = __ballot((bin >> bit) & 1u);
          mm &= ((bin >> bit) & 1u) ? bb : ~bb;
        }
        const uint32_t lower = (uint32_t)__popcll(mm & ((1ULL << lane) - 1));
        const bool leader = v && (mm >> lane) == 1ULL;  // highest lane of its bin
        ++stamp;
        if (wv == 0 && leader) s_w0[bin] = (stamp << 16) | (uint32_t)__popcll(mm);
        __syncthreads();
        uint32_t rank = 0;
        if (v) {
          rank = s_run[bin] + lower;
          if (wv == 1) {
            const uint32_t w0 = s_w0[bin];
            if ((w0 >> 16) == (stamp & 0xFFFFu)) rank += w0 & 0xFFFFu;
          }
          s_sorted[s_base[bin] + rank] = (uint16_t)i;
        }
        __syncthreads();
        if (leader) atomicAdd(&s_run[bin], (uint32_t)__popcll(mm));
        __syncthreads();
      }
      STAMP(1);
      // ---- runs: sorted positions with the same segment (first kBT runs only)
      if (tid == 0) s_cnt[1] = 0;
      __syncthreads();
      for (uint32_t q0 = 0; q0 < npend; q0 += kBT) {
        const uint32_t q = q0 + tid;
        bool start = false;
        if (q < npend) {
          const uint32_t pi = s_sorted[q];
          const uint32_t seg = s_dir[(uint32_t)((s_h[pi] << a.sbits) >> (64 - Dl)) & (nbins - 1)];
          if (q == 0) {
            start = true;
          } else {
            const uint32_t pp = s_sorted[q - 1];
            start = s_dir[(uint32_t)((s_h[pp] << a.sbits) >> (64 - Dl)) & (nbins - 1)] != seg;
          }
        }
        const uint64_t sm = __ballot(start);
        if (lane == 0) s_cnt[2 + wv] = (uint32_t)__popcll(sm);
        __syncthreads();
        const uint32_t ridx = s_cnt[1] + (wv ? s_cnt[2] : 0u) +
                              (uint32_t)__popcll(sm & ((1ULL << lane) - 1));
        if (start && ridx <= (uint32_t)kBT) s_runq[ridx] = (uint16_t)q;
        __syncthreads();
        if (tid == 0) s_cnt[1] += s_cnt[2] + s_cnt[3];
        __syncthreads();
      }
      const uint32_t nruns_all = s_cnt[1];
      const uint32_t nr = min(nruns_all, (uint32_t)kBT);
      if (tid == 0 && nruns_all <= (uint32_t)kBT) s_runq[nr] = (uint16_t)npend;
      if (tid == 0) s_runs += nr;
      __syncthreads();

      STAMP(2);
      // ---- one lane per run: inserts in batch order on the LDS bitmap
      if (tid < nr) {
        const uint32_t q0 = s_runq[tid], q1 = s_runq[tid + 1];
        const uint32_t p0 = s_sorted[q0];
        const uint32_t seg = s_dir[(uint32_t)((s_h[p0] << a.sbits) >> (64 - Dl)) & (nbins - 1)];
        uint32_t* bm = s_bm[tid];
        const uint32_t* og = a.occ + (size_t)seg * 32u;
#pragma unroll
        for (int j = 0; j < 32; ++j) bm[j] = ld_sc1_u32(og + j);
        uint16_t ov = 0xFFFF;
        bool dirty = false;
        for (uint32_t q = q0; q < q1; ++q) {
          const uint32_t pi = s_sorted[q];
          if (s_code[pi] != 1) {
            s_res[pi] = kResGet;
            continue;
          }
          const uint64_t h = s_h[pi];
          const uint32_t w = (uint32_t)(h & 0xFF) * 4u;
          const uint32_t wi = w >> 5;
          const int pos = window_first_free(bm[wi], bm[(wi + 1) & 31u], w);
          if (pos < 0) {
            s_res[pi] = kResOvf;
            ov = (uint16_t)q;
            break;
          }
          bm[(uint32_t)pos >> 5] |= 1u << ((uint32_t)pos & 31u);
          s_res[pi] = (uint16_t)pos;
          dirty = true;
        }
        s_ovq[tid] = ov;
        if (dirty) {
          uint32_t* o = a.occ + (size_t)seg * 32u;
#pragma unroll
          for (int j = 0; j < 32; ++j) o[j] = bm[j];
        }
      }
      __syncthreads();

      STAMP(3);
      // ---- Gets of processed run prefixes: pre-round image + earlier inserts
      if (a.ops) {
        for (uint32_t r = 0; r < nr; ++r) {
          const uint32_t q0 = s_runq[r];
          const uint32_t q1 = (s_ovq[r] != 0xFFFF) ? s_ovq[r] : s_runq[r + 1];
          for (uint32_t q = q0 + tid; q < q1; q += kBT) {
            const uint32_t pi = s_sorted[q];
            if (s_res[pi] != kResGet) continue;
            const uint32_t op = s_op[pi];
            const uint64_t h = s_h[pi];
            const uint64_t key = a.keys[op];
            const uint32_t seg = s_dir[(uint32_t)((h << a.sbits) >> (64 - Dl)) & (nbins - 1)];
            const uint32_t y = (uint32_t)(h & 0xFF) * 4u;
            const uint64_t* sp = reinterpret_cast<const uint64_t*>(a.pairs + (size_t)seg * kSlots);
            uint32_t best = kWindow;  // probe index of the first match
            uint64_t val = 0;
            for (uint32_t i = 0; i < kWindow; ++i) {
              const uint32_t slot = (y + i) & (kSlots - 1);
              const uint64_t k = ld_sc1_u64(sp + 2 * slot);
              if (k == key) {
                best = i;
                val = ld_sc1_u64(sp + 2 * slot + 1);
                break;
              }
              if (k == kInvalid) break;
            }
            // inserts of this run before this Get fill slots that were empty
            for (uint32_t qq = q0; qq < q; ++qq) {
              const uint32_t pj = s_sorted[qq];
              const uint16_t rs = s_res[pj];
              if (s_code[pj] != 1 || rs >= kResOvf) continue;
              const uint32_t opj = s_op[pj];
              if (a.keys[opj] != key) continue;
              const uint32_t pidx = ((uint32_t)rs - y) & (kSlots - 1);
              if (pidx < best) {
                best = pidx;
                val = a.vin[opj];
              }
            }
            a.vout[op] = (best < kWindow) ? val : 0;
            a.st[op] = (best < kWindow) ? 1 : 0;
          }
        }
        __syncthreads();
        for (uint32_t i = tid; i < m; i += kBT)
          if (s_res[i] == kResGet) s_res[i] = kResDone;
      }
      __syncthreads();

      STAMP(4);
      // ---- slot writes of the claimed inserts
      for (uint32_t i = tid; i < m; i += kBT) {
        const uint16_t rs = s_res[i];
        if (rs >= kResOvf) continue;
        const uint32_t op = s_op[i];
        const uint32_t seg = s_dir[(uint32_t)((s_h[i] << a.sbits) >> (64 - Dl)) & (nbins - 1)];
        a.pairs[(size_t)seg * kSlots + rs] = make_ulonglong2(a.keys[op], a.vin[op]);
        a.st[op] = 2;
        if (a.vout) a.vout[op] = 0;
        s_res[i] = kResDone;
      }
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();

      STAMP(5);
      // ---- overflow: split in place (one wave per run), or freeze / status
      for (uint32_t r = wv; r < nr; r += 2) {
        const uint16_t oq = s_ovq[r];
        if (oq == 0xFFFF) continue;
        const uint32_t pi = s_sorted[oq];
        const uint32_t op = s_op[pi];
        const uint64_t h = s_h[pi];
        const uint32_t bin = (uint32_t)((h << a.sbits) >> (64 - Dl)) & (nbins - 1);
        const uint32_t seg = s_dir[bin];
        const uint32_t L = s_ld[bin];
        // the reference would split forever if the window holds 32 copies of
        // this key's hash
        const uint32_t y = (uint32_t)(h & 0xFF) * 4u;
        bool same = true;
        if (lane < kWindow) {
          const uint64_t k = ld_sc1_u64(reinterpret_cast<const uint64_t*>(
              a.pairs + (size_t)seg * kSlots + ((y + lane) & (kSlots - 1))));
          same = hash64(k) == h;
        }
        const bool unsplittable = __ballot(!same) == 0;
        uint8_t code = 0;
        if (unsplittable) code = 4;
        else if (L + 1 > kMaxDepth) code = 5;
        if (code) {
          if (lane == 0) {
            a.st[op] = code;
            s_res[pi] = kResDone;
          }
          continue;
        }
        if (L >= a.gdepth) {
          // needs a directory doubling: freeze the segment's bins; its ops go
          // to the host pass (in batch order, behind this one)
          const uint32_t span = 1u << (a.gdepth - L);
          const uint32_t x0 = bin & ~(span - 1);
          for (uint32_t x = lane; x < span; x += 64) s_frozen[x0 + x] = 1;
          if (lane == 0) {
            atomicOr(&a.ctl->need_double, 1u);
            s_res[pi] = kResPend;
          }
          continue;
        }
        uint32_t c1 = 0;
        if (lane == 0) c1 = atomicAdd(&a.ctl->nsegs, 1u);
        c1 = (uint32_t)__shfl((int)c1, 0);
        if (c1 >= a.max_segments) {
          if (lane == 0) {
            a.st[op] = 6;
            s_res[pi] = kResDone;
          }
          continue;
        }
        const uint32_t loss = wave_split(a.pairs, a.occ, a.ldep, seg, c1, L);
        // directory: second half of the segment's range -> child 1
        const uint32_t span = 1u << (a.gdepth - L);
        const uint32_t x0 = bin & ~(span - 1);
        for (uint32_t x = lane; x < span; x += 64) {
          if (x >= span / 2) {
            s_dir[x0 + x] = c1;
            a.dir[xbase + x0 + x] = c1;
          }
          s_ld[x0 + x] = (uint8_t)(L + 1);
        }
        if (lane == 0) {
          atomicMax(&a.ctl->max_ld, L + 1);
          atomicAdd((unsigned long long*)&a.ctl->splits, 1ULL);
          if (loss) atomicAdd((unsigned long long*)&a.ctl->split_loss, (unsigned long long)loss);
        }
        s_res[pi] = kResPend;  // the overflowing insert retries in the child
      }
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
      // overflowed-run remainders are still kResPend; loop
      STAMP(6);
    }
  }
  __syncthreads();
  STAMP(0);
  if (a.stamps && tid == 0)
    for (int k = 0; k < 8; ++k) atomicAdd(&a.stamps[k], st_acc[k]);
#undef STAMP
  if (tid == 0) {
    if (s_defer) atomicAdd(&a.ctl->n_deferred, s_defer);
    atomicAdd((unsigned long long*)&a.ctl->reserved[0], (unsigned long long)s_runs);
  }
}

// ------------------------------------------------------------- launchers

#define GRID(n, per) dim3((unsigned)(((n) + (per)-1) / (per)))

uint32_t part_blocks(uint64_t n) { return (uint32_t)((n + kPartTile - 1) / kPartTile); }

void launch_part_hist(const uint32_t* pend, const uint32_t* npend_dev, uint64_t npend_host,
                      uint64_t nmax, const uint8_t* st, const uint64_t* hbuf, uint32_t sbits,
                      uint32_t p1, uint32_t* hist, hipStream_t s) {
  const uint32_t nblk = part_blocks(nmax);
  hipLaunchKernelGGL(k_part_hist, dim3(nblk), dim3(kPartThreads), 0, s, pend, npend_dev, npend_host,
                     st, hbuf, sbits, p1, nblk, hist);
}

void launch_part_scatter(const uint32_t* pend, const uint32_t* npend_dev, uint64_t npend_host,
                         uint64_t nmax, const uint8_t* st, const uint64_t* hbuf, uint32_t sbits,
                         uint32_t p1, const uint32_t* hist, const uint32_t* inc, uint64_t* ph,
                         uint32_t* pop, hipStream_t s) {
  const uint32_t nblk = part_blocks(nmax);
  hipLaunchKernelGGL(k_part_scatter, dim3(nblk), dim3(kPartThreads), 0, s, pend, npend_dev,
                     npend_host, st, hbuf, sbits, p1, nblk, hist, inc, ph, pop);
}

void launch_bucket(const BucketLaunch& L, hipStream_t s) {
  BucketArgs a;
  a.ph = L.ph;
  a.pop = L.pop;
  a.offs = L.offs;
  a.nblk = part_blocks(L.nmax);
  a.p1 = L.p1;
  a.bbits = L.bbits;
  a.gdepth = L.gdepth;
  a.sbits = L.sbits;
  a.ops = L.ops;
  a.keys = L.keys;
  a.vin = L.vin;
  a.vout = L.vout;
  a.st = L.st;
  a.pairs = L.pairs;
  a.occ = L.occ;
  a.ldep = L.ldep;
  a.dir = L.dir;
  a.deferred = L.deferred;
  a.ctl = L.ctl;
  a.max_segments = L.max_segments;
  a.stamps = L.stamps;
  hipLaunchKernelGGL(k_bucket, dim3(1u << L.p1), dim3(kBT), 0, s, a);
}

}  // namespace pmdfc
