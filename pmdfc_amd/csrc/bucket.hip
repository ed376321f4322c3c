// bucket.hip -- the batched insert/mixed fast path.
//
// 1. k_part_hist / inclusive scan / k_part_scatter: stable partition of the
//    batch's pending ops into 2^P1 buckets by the top P1 local hash bits, one
//    packed u64 record per op (op index | directory bin | home line).  With
//    P1 <= min local depth every segment lies inside one bucket, so buckets are
//    independent (CCEH splits are segment-local, CCEH_hybrid.cpp:171-297).
// 2. k_bucket: ONE WAVE per bucket.  It keeps the bucket's directory slice in
//    LDS, and per chunk of <= kChunk ops: gathers the ops' keys/values into LDS,
//    stable-sorts the pending ops by segment (ballot matching, no global sort),
//    and gives every segment run to one lane, which applies the run's ops in
//    batch order against the segment's occupancy bitmap (LDS): inserts claim
//    the first free slot of the 32-slot window (CCEH_hybrid.cpp:143-168) and
//    store the pair at once; Gets probe the segment, which already holds the
//    lane's earlier inserts.  A run whose window is full stops there: the
//    segment is queued for splitting and the rest of the run (and every later
//    op of that segment in this pass) waits for the next pass.
// 3. k_split_q: one wave per queued segment (slot-order replay, k_split's
//    algorithm), grid-stride over the device-side queue of that pass.
// Passes 0..kPasses-1 run back to back with no host round trip; whatever is
// still pending after the last pass (or needs a global directory doubling)
// goes to the host-driven generic path (engine).
#include "cceh_device.h"
#include "cceh_kernels.h"

namespace pmdfc {

constexpr int kPartThreads = 256;
constexpr int kPartItems = 16;
constexpr int kPartTile = kPartThreads * kPartItems;  // 4096 ops per partition block
constexpr int kMaxP1 = 12;                            // <= 4096 buckets

constexpr int kChunk = 256;                           // ops per k_bucket chunk
constexpr int kMaxBins = 512;                         // directory slice per bucket

constexpr uint8_t kPsDone = 0xFF;   // partition-position state: resolved
// other values: the bucket pass the op is pending in

__device__ __forceinline__ uint32_t bucket_of(uint64_t h, uint32_t sbits, uint32_t p1) {
  return (uint32_t)((h << sbits) >> (64 - p1));
}

// record: bits 0-31 op index, 32-41 directory bin inside the bucket, 42-49 home line
__device__ __forceinline__ uint32_t rec_op(uint64_t r) { return (uint32_t)r; }
__device__ __forceinline__ uint32_t rec_bin(uint64_t r) { return (uint32_t)(r >> 32) & 1023u; }
__device__ __forceinline__ uint32_t rec_home(uint64_t r) { return (uint32_t)(r >> 42) & 255u; }

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
    uint32_t bbits, uint32_t nblk, const uint32_t* __restrict__ hist,
    const uint32_t* __restrict__ inc, uint64_t* __restrict__ rec) {
  __shared__ uint16_t s_w[4][1 << kMaxP1];  // per-wave running count per bucket
  const uint32_t nb = 1u << p1;
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  for (uint32_t i = threadIdx.x; i < 4 * nb; i += kPartThreads) s_w[i / nb][i % nb] = 0;
  __syncthreads();
  const uint64_t npend = npend_dev ? *npend_dev : npend_host;
  const uint64_t base = (uint64_t)blockIdx.x * kPartTile + (uint64_t)wv * (kPartTile / 4);
  const uint64_t lt = (1ULL << lane) - 1;
  const uint32_t dl = p1 + bbits;
  uint32_t bk[kPartItems], rk[kPartItems];
  uint64_t rv[kPartItems];
#pragma unroll
  for (int k = 0; k < kPartItems; ++k) {
    const uint64_t p = base + (uint64_t)k * 64 + lane;
    uint32_t op = 0;
    const bool v = part_item(p, npend, pend, st, &op);
    uint32_t b = 0xFFFFu;
    uint64_t r = 0;
    if (v) {
      const uint64_t h = hbuf[op];
      const uint64_t xl = (h << sbits) >> (64 - dl);
      b = (uint32_t)(xl >> bbits);
      r = (uint64_t)op | ((xl & ((1ULL << bbits) - 1)) << 32) | ((h & 0xFFULL) << 42);
    }
    uint64_t mm = __ballot(v);
    for (uint32_t bit = 0; bit < p1; ++bit) {
      const uint64_t bb = __ballot((b >> bit) & 1u);
      mm &= ((b >> bit) & 1u) ? bb : ~bb;
    }
    uint32_t rank = 0;
    if (v) {
      rank = s_w[wv][b] + (uint32_t)__popcll(mm & lt);
      // the highest matching lane updates the running count
      if ((mm >> lane) == 1ULL) s_w[wv][b] = (uint16_t)(s_w[wv][b] + __popcll(mm));
    }
    bk[k] = b;
    rk[k] = rank;
    rv[k] = r;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kPartItems; ++k) {
    const uint32_t b = bk[k];
    if (b == 0xFFFFu) continue;
    uint32_t add = 0;
    for (uint32_t w = 0; w < wv; ++w) add += s_w[w][b];
    const size_t hi = (size_t)b * nblk + blockIdx.x;
    rec[inc[hi] - hist[hi] + add + rk[k]] = rv[k];
  }
}

// ---------------------------------------------------------------- bucket

struct BucketArgs {
  const uint64_t* rec;
  const uint32_t* inc;       // inclusive scan of the bucket-major partition histogram
  uint32_t nblk;             // partition blocks (row length of inc)
  uint32_t p1, bbits;        // bucket bits, directory-slice bits
  uint32_t gdepth, sbits;
  uint32_t pass, last;       // this pass; last pass defers to the host instead of splitting
  const uint8_t* ops;        // null: all inserts
  const uint64_t* keys;
  const uint64_t* vin;
  uint64_t* vout;
  uint8_t* st;
  ulonglong2* pairs;
  uint32_t* occ;
  const uint32_t* dir;
  uint8_t* pstate;           // per partition position
  uint8_t* bwork;            // per bucket: bit k = ops pending in pass k
  uint8_t* hostdef;          // per op: deferred to the host generic pass
  uint32_t* split_list;      // this pass's queue, 2 u32 per entry
  DevCtl* ctl;
  uint32_t max_segments;
};

__global__ __launch_bounds__(64) void k_bucket(BucketArgs a) {
  __shared__ uint32_t s_dir[kMaxBins];
  __shared__ uint8_t s_blk[kMaxBins];  // segment blocked for the rest of the pass: 1 next pass, 2 host
  __shared__ uint32_t s_base[kMaxBins];
  __shared__ uint32_t s_run[kMaxBins];
  __shared__ uint64_t s_rec[kChunk];
  __shared__ uint64_t s_key[kChunk];
  __shared__ uint64_t s_val[kChunk];
  __shared__ uint8_t s_code[kChunk];
  __shared__ uint16_t s_sorted[kChunk];
  __shared__ uint16_t s_runq[kChunk + 1];
  __shared__ uint32_t s_bm[64][33];

  const uint32_t lane = threadIdx.x;
  const uint32_t b = blockIdx.x;
  if (a.pass > 0 && !((a.bwork[b] >> a.pass) & 1u)) return;
  const uint64_t beg = b ? a.inc[(size_t)b * a.nblk - 1] : 0;
  const uint64_t end = a.inc[(size_t)(b + 1) * a.nblk - 1];
  if (beg >= end) return;
  const uint32_t nbins = 1u << a.bbits;
  const uint32_t xbase = b << a.bbits;
  for (uint32_t x = lane; x < nbins; x += 64) {
    s_dir[x] = a.dir[xbase + x];
    s_blk[x] = 0;
  }
  __syncthreads();
  // first bin of the segment owning bin x (a segment spans 2^(gdepth-L) bins)
  auto seg_start = [&](uint32_t x) -> uint32_t {
    const uint32_t sb = a.gdepth - de_ld(s_dir[x]);
    return (x >> sb) << sb;
  };

  const uint64_t lt = (1ULL << lane) - 1;
  uint32_t n_next = 0, n_host = 0, n_runs = 0;
  for (uint64_t cs = beg; cs < end; cs += kChunk) {
    const uint32_t m = (uint32_t)min<uint64_t>(kChunk, end - cs);
    if (cs != beg) {
      // same-segment ops in the previous chunk were applied by other lanes of
      // this wave: make their stores visible to this CU's loads
      __builtin_amdgcn_s_waitcnt(0);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    // ---- load the chunk: records, then keys/values/opcodes of pending ops
    for (uint32_t i = lane; i < kChunk; i += 64) {
      uint64_t r = ~0ULL;
      if (i < m && a.pstate[cs + i] == a.pass) r = a.rec[cs + i];
      s_rec[i] = r;
    }
    __syncthreads();
    for (uint32_t i = lane; i < m; i += 64) {
      const uint64_t r = s_rec[i];
      if (r == ~0ULL) continue;
      const uint32_t op = rec_op(r);
      const uint8_t code = a.ops ? a.ops[op] : (uint8_t)1;
      s_code[i] = code;
      s_key[i] = a.keys[op];
      s_val[i] = code == 1 ? a.vin[op] : 0;
    }
    // ---- stable counting sort of pending positions by segment start bin
    for (uint32_t x = lane; x < nbins; x += 64) s_run[x] = 0;
    __syncthreads();
    for (uint32_t i = lane; i < m; i += 64)
      if (s_rec[i] != ~0ULL) atomicAdd(&s_run[seg_start(rec_bin(s_rec[i]))], 1u);
    __syncthreads();
    uint32_t carry = 0;
    for (uint32_t x0 = 0; x0 < nbins; x0 += 64) {
      const uint32_t x = x0 + lane;
      const uint32_t v = x < nbins ? s_run[x] : 0;
      uint32_t incl = v;
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = (uint32_t)__shfl_up((int)incl, o);
        if (lane >= (uint32_t)o) incl += t;
      }
      if (x < nbins) {
        s_base[x] = carry + incl - v;
        s_run[x] = 0;
      }
      carry += (uint32_t)__shfl((int)incl, 63);
    }
    const uint32_t npend = carry;
    __syncthreads();
    if (npend == 0) continue;
    for (uint32_t r0 = 0; r0 < m; r0 += 64) {
      const uint32_t i = r0 + lane;
      const bool v = i < m && s_rec[i] != ~0ULL;
      const uint32_t key = v ? seg_start(rec_bin(s_rec[i])) : 0u;
      uint64_t mm = __ballot(v);
      for (uint32_t bit = 0; bit < a.bbits; ++bit) {
        const uint64_t bb = __ballot((key >> bit) & 1u);
        mm &= ((key >> bit) & 1u) ? bb : ~bb;
      }
      if (v) s_sorted[s_base[key] + s_run[key] + (uint32_t)__popcll(mm & lt)] = (uint16_t)i;
      __syncthreads();
      if (v && (mm >> lane) == 1ULL) s_run[key] += (uint32_t)__popcll(mm);
      __syncthreads();
    }
    // ---- runs: maximal stretches of the sorted order with one segment
    uint32_t nruns = 0;
    for (uint32_t q0 = 0; q0 < npend; q0 += 64) {
      const uint32_t q = q0 + lane;
      bool start = false;
      if (q < npend) {
        const uint32_t k = seg_start(rec_bin(s_rec[s_sorted[q]]));
        start = q == 0 || seg_start(rec_bin(s_rec[s_sorted[q - 1]])) != k;
      }
      const uint64_t sm = __ballot(start);
      if (start) s_runq[nruns + (uint32_t)__popcll(sm & lt)] = (uint16_t)q;
      nruns += (uint32_t)__popcll(sm);
    }
    if (lane == 0) s_runq[nruns] = (uint16_t)npend;
    __syncthreads();
    n_runs += nruns;

    // ---- one lane per run
    for (uint32_t rg = 0; rg < nruns; rg += 64) {
      const uint32_t r = rg + lane;
      if (r >= nruns) continue;
      const uint32_t q0 = s_runq[r], q1 = s_runq[r + 1];
      const uint32_t x0 = seg_start(rec_bin(s_rec[s_sorted[q0]]));
      const uint32_t e = s_dir[x0];
      const uint32_t seg = de_seg(e);
      const uint32_t L = de_ld(e);
      const uint8_t blk = s_blk[x0];
      if (blk) {
        // segment waits for a split (1) or a directory doubling (2)
        for (uint32_t q = q0; q < q1; ++q) {
          const uint32_t pi = s_sorted[q];
          if (blk == 1) {
            a.pstate[cs + pi] = (uint8_t)(a.pass + 1);
            ++n_next;
          } else {
            a.pstate[cs + pi] = kPsDone;
            a.hostdef[rec_op(s_rec[pi])] = 1;
            ++n_host;
          }
        }
        continue;
      }
      uint32_t* bm = s_bm[lane];
      const uint4* og = reinterpret_cast<const uint4*>(a.occ + (size_t)seg * 32u);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint4 v = og[j];
        bm[4 * j] = v.x;
        bm[4 * j + 1] = v.y;
        bm[4 * j + 2] = v.z;
        bm[4 * j + 3] = v.w;
      }
      ulonglong2* sp = a.pairs + (size_t)seg * kSlots;
      bool dirty = false;
      for (uint32_t q = q0; q < q1; ++q) {
        const uint32_t pi = s_sorted[q];
        const uint64_t rr = s_rec[pi];
        const uint32_t op = rec_op(rr);
        const uint32_t home = rec_home(rr);
        const uint64_t key = s_key[pi];
        if (s_code[pi] != 1) {
          uint64_t val = 0;
          const uint8_t s = lane_probe(sp, key, home, &val);
          a.vout[op] = val;
          a.st[op] = s;
          a.pstate[cs + pi] = kPsDone;
          continue;
        }
        const uint32_t w = home * 4u;
        const uint32_t wi = w >> 5;
        const int pos = window_first_free(bm[wi], bm[(wi + 1) & 31u], w);
        if (pos >= 0) {
          bm[(uint32_t)pos >> 5] |= 1u << ((uint32_t)pos & 31u);
          dirty = true;
          sp[pos] = make_ulonglong2(key, s_val[pi]);
          a.st[op] = 2;  // PMDFC_ST_INSERTED
          if (a.vout) a.vout[op] = 0;
          a.pstate[cs + pi] = kPsDone;
          continue;
        }
        // window full.  The reference would split forever if all 32 entries
        // carry this key's full hash: UNSPLITTABLE.
        const uint64_t h = hash64(key);
        bool same = true;
        for (uint32_t i = 0; i < kWindow && same; ++i)
          same = hash64(sp[(w + i) & (kSlots - 1)].x) == h;
        uint8_t code = 0;
        if (same) code = 4;
        else if (L + 1 > kMaxDepth) code = 5;
        uint32_t c1 = 0;
        uint8_t dest = 0;  // 1: next pass after a queued split, 2: host
        if (!code) {
          if (L >= a.gdepth || a.last) {
            dest = 2;  // needs a directory doubling, or no pass left
            if (L >= a.gdepth) atomicOr(&a.ctl->need_double, 1u);
          } else {
            c1 = atomicAdd(&a.ctl->nsegs, 1u);
            if (c1 >= a.max_segments) code = 6;
            else dest = 1;
          }
        }
        if (code) {
          a.st[op] = code;
          if (a.vout) a.vout[op] = 0;
          a.pstate[cs + pi] = kPsDone;
          continue;
        }
        if (dest == 1) {
          const uint32_t si = atomicAdd(&a.ctl->pass_split[a.pass], 1u);
          a.split_list[2 * si] = seg;
          a.split_list[2 * si + 1] = c1;
        }
        // this op and the rest of the run wait; so do later chunks' ops of
        // this segment (s_blk)
        for (uint32_t qq = q; qq < q1; ++qq) {
          const uint32_t pj = s_sorted[qq];
          if (dest == 1) {
            a.pstate[cs + pj] = (uint8_t)(a.pass + 1);
            ++n_next;
          } else {
            a.pstate[cs + pj] = kPsDone;
            a.hostdef[rec_op(s_rec[pj])] = 1;
            ++n_host;
          }
        }
        const uint32_t span = 1u << (a.gdepth - L);
        for (uint32_t x = 0; x < span; ++x) s_blk[x0 + x] = dest;
        break;
      }
      if (dirty) {
        uint4* o = reinterpret_cast<uint4*>(a.occ + (size_t)seg * 32u);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = make_uint4(bm[4 * j], bm[4 * j + 1], bm[4 * j + 2], bm[4 * j + 3]);
      }
    }
    __syncthreads();
  }
  // wave reductions of the per-lane counters
  for (int o = 32; o > 0; o >>= 1) {
    n_next += (uint32_t)__shfl_down((int)n_next, o);
    n_host += (uint32_t)__shfl_down((int)n_host, o);
  }
  if (lane == 0) {
    if (n_next) a.bwork[b] |= (uint8_t)(1u << (a.pass + 1));
    if (n_host) atomicAdd(&a.ctl->n_deferred, n_host);
    atomicAdd((unsigned long long*)&a.ctl->runs, (unsigned long long)n_runs);
  }
}

// ---------------------------------------------------------- queued splits
// Segment::Split (non-INPLACE, CCEH_hybrid.cpp:47-66) + directory update
// (:243-286) for every segment queued by bucket pass `pass`; one wave per
// segment, grid-stride over the device-side count.
__global__ __launch_bounds__(64) void k_split_q(const uint32_t* __restrict__ split_list,
                                                const uint32_t* __restrict__ count,
                                                ulonglong2* __restrict__ pairs,
                                                uint32_t* __restrict__ occ,
                                                uint8_t* __restrict__ ldep, uint32_t* __restrict__ dir,
                                                uint32_t gdepth, uint32_t sbits,
                                                DevCtl* __restrict__ ctl) {
  __shared__ ulonglong2 s_par[kSlots];
  __shared__ uint16_t s_inv[2][kSlots];
  __shared__ uint32_t s_b[64], s_cb[64], s_col[64];
  const uint32_t lane = threadIdx.x;
  const uint32_t n = *count;
  for (uint32_t it = blockIdx.x; it < n; it += gridDim.x) {
    const uint32_t seg = split_list[2 * it];
    const uint32_t c1 = split_list[2 * it + 1];
    const uint32_t L = ldep[seg];
    ulonglong2* sp = pairs + (size_t)seg * kSlots;
    uint32_t inf[16];
    uint64_t any_h = 0;
    bool have = false;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const uint32_t slot = (uint32_t)j * 64u + lane;
      const ulonglong2 p = sp[slot];
      s_par[slot] = p;
      s_inv[0][slot] = 0;
      s_inv[1][slot] = 0;
      const bool valid = p.x != kInvalid;
      const uint64_t kh = hash64(p.x);
      if (valid && !have) {
        have = true;
        any_h = kh;
      }
      inf[j] = (valid ? 0x80000000u : 0u) | ((uint32_t)((kh >> (63 - L)) & 1u) << 8) |
               (uint32_t)(kh & 0xFF);
    }
    s_b[lane] = 0;
    __builtin_amdgcn_wave_barrier();
    uint32_t dest[16];
    uint32_t loss = wave_replay(inf, dest, s_b, s_cb, s_col);
    for (int o = 32; o > 0; o >>= 1) loss += (uint32_t)__shfl_down((int)loss, o);
    const uint32_t bw = s_b[lane];  // lanes 0-31 child 0 words, 32-63 child 1 words
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const uint32_t d = dest[j];
      if (d != 0xFFFFFFFFu) s_inv[d >> 10][d & 1023u] = (uint16_t)(j * 64 + lane + 1);
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      ulonglong2* dst = pairs + (size_t)(c ? c1 : seg) * kSlots;
#pragma unroll 4
      for (int j = 0; j < 16; ++j) {
        const uint32_t slot = (uint32_t)j * 64u + lane;
        const uint32_t src = s_inv[c][slot];
        dst[slot] = src ? s_par[src - 1] : make_ulonglong2(kInvalid, 0ULL);
      }
    }
    if (lane < 32) occ[(size_t)seg * 32u + lane] = bw;
    else occ[(size_t)c1 * 32u + (lane - 32)] = bw;
    if (lane == 0) {
      ldep[seg] = (uint8_t)(L + 1);
      ldep[c1] = (uint8_t)(L + 1);
      atomicMax(&ctl->max_ld, L + 1);
      atomicAdd((unsigned long long*)&ctl->splits, 1ULL);
      if (loss) atomicAdd((unsigned long long*)&ctl->split_loss, (unsigned long long)loss);
    }
    const uint64_t vmask = __ballot(have);
    const int src = vmask ? __builtin_ctzll(vmask) : 0;
    const uint64_t h0 = shfl64(any_h, src);
    const uint32_t Ll = L - sbits;
    const uint32_t Dl = gdepth - sbits;
    const uint64_t prefix = Ll ? ((h0 >> (64 - L)) & ((1ULL << Ll) - 1)) : 0;
    const uint64_t stride = 1ULL << (Dl - Ll);
    const uint64_t xb = prefix << (Dl - Ll);
    for (uint64_t i = lane; i < stride; i += 64) dir[xb + i] = de_make(i < stride / 2 ? seg : c1, L + 1);
    __syncthreads();  // s_par / s_inv reuse by the next iteration
  }
}

// ------------------------------------------------------------- launchers

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
                         uint32_t p1, uint32_t bbits, const uint32_t* hist, const uint32_t* inc,
                         uint64_t* rec, hipStream_t s) {
  const uint32_t nblk = part_blocks(nmax);
  hipLaunchKernelGGL(k_part_scatter, dim3(nblk), dim3(kPartThreads), 0, s, pend, npend_dev,
                     npend_host, st, hbuf, sbits, p1, bbits, nblk, hist, inc, rec);
}

void launch_bucket(const BucketLaunch& L, hipStream_t s) {
  BucketArgs a;
  a.rec = L.rec;
  a.inc = L.inc;
  a.nblk = part_blocks(L.nmax);
  a.p1 = L.p1;
  a.bbits = L.bbits;
  a.gdepth = L.gdepth;
  a.sbits = L.sbits;
  a.pass = L.pass;
  a.last = L.last;
  a.ops = L.ops;
  a.keys = L.keys;
  a.vin = L.vin;
  a.vout = L.vout;
  a.st = L.st;
  a.pairs = L.pairs;
  a.occ = L.occ;
  a.dir = L.dir;
  a.pstate = L.pstate;
  a.bwork = L.bwork;
  a.hostdef = L.hostdef;
  a.split_list = L.split_list;
  a.ctl = L.ctl;
  a.max_segments = L.max_segments;
  hipLaunchKernelGGL(k_bucket, dim3(1u << L.p1), dim3(64), 0, s, a);
}

void launch_split_q(const uint32_t* split_list, const uint32_t* count, ulonglong2* pairs,
                    uint32_t* occ, uint8_t* ldep, uint32_t* dir, uint32_t gdepth, uint32_t sbits,
                    DevCtl* ctl, uint32_t grid, hipStream_t s) {
  hipLaunchKernelGGL(k_split_q, dim3(grid), dim3(64), 0, s, split_list, count, pairs, occ, ldep,
                     dir, gdepth, sbits, ctl);
}

}  // namespace pmdfc
