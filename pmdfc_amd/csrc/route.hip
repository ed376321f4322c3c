// route.hip -- fixed-capacity shard routing for the multi-GPU path.
//
// The key space shards by the top shard_bits of h(key), the bits CCEH indexes
// its directory with (CCEH_hybrid.cpp:119), so each op has exactly one owner
// GPU.  A batch is exchanged with equal-split RCCL all-to-alls: every rank
// sends every owner a block of `cap` records, the owner's ops first, the rest
// padded with key INVALID (server/util/pair.h:10), which the engine answers
// with RESERVED_KEY and never stores.  Equal splits mean the exchange needs no
// counts on the host, so a routed batch has no host sync.
//
// No op is dropped: an owner block that fills up leaves the rest of that
// owner's ops in a per-owner FIFO carry (device memory), and the next pack
// sends the carry first, then its own ops.  Each (rank, owner) stream of ops
// therefore travels in order, cap ops per exchange; a call ends with drain
// exchanges until every rank's carry is empty (pmdfc_amd/dist.py).  Only an op
// that finds the carry itself full (carry_cap ops per owner waiting) comes
// back PMDFC_ST_ROUTE_OVERFLOW, counted in a sticky counter.
//
//   k_route_count   tile of 1024 ops -> per-owner counts
//   k_route_scatter one kernel, three kinds of blocks:
//                   tiles: slot = carried-in count + earlier tiles' counts +
//                   stable in-tile rank (ballot); slot < cap -> send row,
//                   else -> carry-out slot (slot - cap);
//                   carry: carried-in op j -> send row j, or carry-out j - cap;
//                   padding: rows past the owner's total get key INVALID, and
//                   the owner's carry-out count
//   rowpos[row]     the call-global output index of the op a row carries
//   k_route_split   received records -> engine key / value / op arrays
//   k_route_resp    engine (value, status) -> 16-B response records
//   k_route_unpack  returned response rows -> call-global outputs via rowpos
//   k_dedupe_tile   Get batches: one row per distinct key of each 1024-Get
//                   tile (its first Get); the others copy its result
//                   (k_route_fill)
// An optional keep mask (the replicated bloom filter's probe)
// keeps negatives home: they take no slot, never cross xGMI, and are reported
// PMDFC_ST_FILTERED.
#include <hip/hip_runtime.h>

#include "cceh_device.h"
#include "cceh_kernels.h"

namespace pmdfc {

namespace {

constexpr uint32_t kRT = 256;                     // threads per routing block
constexpr uint32_t kRPer = kRouteTile / kRT;      // ops per thread (4)
constexpr uint32_t kStOverflow = 9;               // PMDFC_ST_ROUTE_OVERFLOW
constexpr uint32_t kStFiltered = 7;               // PMDFC_ST_FILTERED
constexpr uint32_t kPadPer = 4;                   // padding blocks per owner in k_route_scatter
constexpr uint32_t kCarryPer = 8;                 // carry blocks per owner in k_route_scatter

__device__ __forceinline__ uint32_t owner_of(uint64_t key, uint32_t sbits) {
  return sbits ? (uint32_t)(hash64(key) >> (64 - sbits)) : 0u;
}

__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__global__ __launch_bounds__(kRT) void k_route_count(const uint64_t* __restrict__ keys,
                                                     const uint8_t* __restrict__ keep, uint64_t n,
                                                     uint32_t sbits, uint32_t* __restrict__ tile_cnt) {
  __shared__ uint32_t cnt[kRouteMaxOwners];
  const uint32_t G = 1u << sbits;
  if (threadIdx.x < G) cnt[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x * kRouteTile;
  uint32_t mine[kRouteMaxOwners];
#pragma unroll
  for (uint32_t g = 0; g < kRouteMaxOwners; ++g) mine[g] = 0;
#pragma unroll
  for (uint32_t j = 0; j < kRPer; ++j) {
    const uint64_t i = base + j * kRT + threadIdx.x;
    if (i < n && (!keep || keep[i])) {
      const uint32_t o = owner_of(keys[i], sbits);
#pragma unroll
      for (uint32_t g = 0; g < kRouteMaxOwners; ++g) mine[g] += (o == g);
    }
  }
  // wave sums, then one LDS add per wave and owner
#pragma unroll
  for (uint32_t g = 0; g < kRouteMaxOwners; ++g) {
    if (g < G) {
      uint32_t v = mine[g];
      for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off);
      if ((threadIdx.x & 63u) == 0) atomicAdd(&cnt[g], v);
    }
  }
  __syncthreads();
  if (threadIdx.x < G) tile_cnt[(size_t)blockIdx.x * G + threadIdx.x] = cnt[threadIdx.x];
}

__device__ __forceinline__ void put_row(const RouteArgs& a, uint32_t g, uint64_t slot, uint64_t k, uint64_t v,
                                        uint64_t op) {
  uint64_t* rec = a.self_dst && g == a.self_g ? a.self_dst + slot * a.width : a.send + (g * a.cap + slot) * a.width;
  if (a.width == 2) {  // 16-B record, one store
    *reinterpret_cast<ulonglong2*>(rec) = make_ulonglong2(k, v);
  } else {
    rec[0] = k;
    if (a.width > 2) {
      rec[1] = v;
      rec[2] = op;
    }
  }
}

__device__ __forceinline__ void put_carry(const RouteArgs& a, uint64_t at, uint64_t k, uint64_t v, uint64_t op,
                                          uint32_t gi) {
  uint64_t* rec = a.crec_out + at * kCarryWords;
  rec[0] = k;
  if (a.width > 1) rec[1] = v;
  if (a.width > 2) rec[2] = op;
  a.cpos_out[at] = gi;
}

__device__ __forceinline__ void not_sent(const RouteArgs& a, uint32_t gi, uint8_t st) {
  a.st_out[gi] = st;
  if (a.vals_out) a.vals_out[gi] = 0;
}

// padding blocks: owner g's rows past its total get key INVALID (0xFF.. values
// / ops, no memset) and rowpos kRouteNone; part 0 writes its carry-out count
__device__ __forceinline__ void route_pad(const RouteArgs& a, uint32_t tiles, uint32_t pb) {
  __shared__ uint32_t s_tot;
  const uint32_t G = 1u << a.sbits, g = pb / kPadPer, part = pb % kPadPer;
  if (threadIdx.x == 0) s_tot = 0;
  __syncthreads();
  uint32_t acc = 0;
  for (uint32_t t = threadIdx.x; t < tiles; t += kRT) acc += a.tile_cnt[(size_t)t * G + g];
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off);
  if ((threadIdx.x & 63u) == 0) atomicAdd(&s_tot, acc);
  __syncthreads();
  const uint64_t tot = (uint64_t)s_tot + a.cin[g];
  if (part == 0 && threadIdx.x == 0) a.cout[g] = tot > a.cap ? (uint32_t)min<uint64_t>(a.cc, tot - a.cap) : 0u;
  const uint64_t lo = min<uint64_t>(tot, a.cap);
  const uint64_t rows = a.cap - lo;
  const uint64_t chunk = (rows + kPadPer - 1) / kPadPer;
  const uint64_t r0 = lo + part * chunk, r1 = min<uint64_t>(a.cap, r0 + chunk);
  const uint64_t W = a.width;
  uint64_t* blk = a.self_dst && g == a.self_g ? a.self_dst : a.send + (uint64_t)g * a.cap * W;
  for (uint64_t e = r0 * W + threadIdx.x; e < r1 * W; e += kRT) blk[e] = ~0ULL;
  for (uint64_t r = r0 + threadIdx.x; r < r1; r += kRT) a.rowpos[(uint64_t)g * a.cap + r] = kRouteNone;
}

// carry blocks: owner g's carried-in ops, in FIFO order, ahead of this batch
__device__ __forceinline__ void route_carry(const RouteArgs& a, uint32_t cb) {
  const uint32_t g = cb / kCarryPer, part = cb % kCarryPer;
  const uint32_t c = a.cin[g];
  for (uint64_t j = (uint64_t)part * kRT + threadIdx.x; j < c; j += (uint64_t)kCarryPer * kRT) {
    const uint64_t at = (uint64_t)g * a.cc + j;
    const uint64_t* rec = a.crec_in + at * kCarryWords;
    const uint64_t k = rec[0], v = a.width > 1 ? rec[1] : 0, op = a.width > 2 ? rec[2] : 0;
    const uint32_t gi = a.cpos_in[at];
    if (j < a.cap) {
      put_row(a, g, j, k, v, op);
      a.rowpos[(uint64_t)g * a.cap + j] = gi;
    } else {
      put_carry(a, (uint64_t)g * a.cc + (j - a.cap), k, v, op, gi);
    }
  }
}

__global__ __launch_bounds__(kRT) void k_route_scatter(RouteArgs a, uint32_t tiles) {
  __shared__ uint32_t s_base[kRouteMaxOwners];         // running slot per owner
  __shared__ uint32_t s_wc[kRPer][kRT / 64][kRouteMaxOwners];  // per-wave counts of each chunk
  const uint32_t G = 1u << a.sbits;
  if (blockIdx.x >= tiles + G * kPadPer) {
    route_carry(a, blockIdx.x - tiles - G * kPadPer);
    return;
  }
  if (blockIdx.x >= tiles) {
    route_pad(a, tiles, blockIdx.x - tiles);
    return;
  }
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  // every op of the tile loaded up front (kRPer per thread: one round trip),
  // ranked per chunk by ballots, then placed: two workgroup barriers in all
  // (the chunks one after another, a barrier pair each, measured 33 us per
  // 1M-op batch)
  const uint64_t base = (uint64_t)blockIdx.x * kRouteTile;
  uint64_t key[kRPer], val[kRPer], opw[kRPer];
  uint32_t o[kRPer], r[kRPer];
  bool live[kRPer];
#pragma unroll
  for (uint32_t j = 0; j < kRPer; ++j) {
    const uint64_t i = base + j * kRT + threadIdx.x;
    const bool inb = i < a.n;
    live[j] = inb && (!a.keep || a.keep[i]);
    if (inb && !live[j]) not_sent(a, a.base + (uint32_t)i, (uint8_t)kStFiltered);
    key[j] = live[j] ? a.keys[i] : 0;
    val[j] = live[j] && a.width > 1 ? a.vals[i] : 0;
    opw[j] = live[j] && a.width > 2 ? (uint64_t)a.ops[i] : 0;
  }
  if (threadIdx.x < G) s_base[threadIdx.x] = a.cin[threadIdx.x];
  // slots taken by the tiles before this one: the (tile, owner) counts are
  // read as one flat array, element e belongs to owner e % G
  uint32_t acc = 0;
  {
    const uint32_t ne = blockIdx.x * G;  // G divides kRT, so e % G == threadIdx.x % G
    for (uint32_t e = threadIdx.x; e < ne; e += kRT) acc += a.tile_cnt[e];
    // lanes l and l + G, l + 2G, ... hold the same owner: fold them
    for (uint32_t off = 32; off >= G && off > 0; off >>= 1) acc += __shfl_down(acc, off);
  }
#pragma unroll
  for (uint32_t j = 0; j < kRPer; ++j) {
    o[j] = live[j] ? owner_of(key[j], a.sbits) : G;
    r[j] = 0;
#pragma unroll
    for (uint32_t g = 0; g < kRouteMaxOwners; ++g) {
      if (g < G) {
        const uint64_t m = __ballot(o[j] == g);
        if (o[j] == g) r[j] = lanes_below(m);
        if (lane == 0) s_wc[j][wave][g] = (uint32_t)__popcll(m);
      }
    }
  }
  __syncthreads();  // (s_base seeded, s_wc complete)
  if (lane < G) atomicAdd(&s_base[lane], acc);
  __syncthreads();
#pragma unroll
  for (uint32_t j = 0; j < kRPer; ++j) {
    if (!live[j]) continue;
    const uint32_t g = o[j];
    uint64_t slot = s_base[g] + r[j];
    for (uint32_t jj = 0; jj < j; ++jj)  // the chunks before, in batch order
      for (uint32_t w = 0; w < kRT / 64; ++w) slot += s_wc[jj][w][g];
    for (uint32_t w = 0; w < wave; ++w) slot += s_wc[j][w][g];
    const uint32_t gi = a.base + (uint32_t)(base + j * kRT + threadIdx.x);
    if (slot < a.cap) {
      put_row(a, g, slot, key[j], val[j], opw[j]);
      a.rowpos[(uint64_t)g * a.cap + slot] = gi;
    } else if (slot - a.cap < a.cc) {
      put_carry(a, (uint64_t)g * a.cc + (slot - a.cap), key[j], val[j], opw[j], gi);
    } else {
      not_sent(a, gi, (uint8_t)kStOverflow);
      atomicAdd(a.ovf, 1u);
    }
  }
}

__global__ __launch_bounds__(256) void k_route_split(const uint64_t* __restrict__ recv, uint64_t rows,
                                                     uint32_t W, uint64_t* __restrict__ keys,
                                                     uint64_t* __restrict__ vals,
                                                     uint8_t* __restrict__ ops) {
  const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (i >= rows) return;
  const uint64_t* rec = recv + i * W;
  keys[i] = rec[0];
  if (W > 1) vals[i] = rec[1];
  if (W > 2) ops[i] = (uint8_t)rec[2];
}

__global__ __launch_bounds__(256) void k_route_resp(const uint64_t* __restrict__ vals,
                                                    const uint8_t* __restrict__ st, uint64_t rows,
                                                    ulonglong2* __restrict__ resp) {
  const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (i >= rows) return;
  resp[i] = make_ulonglong2(vals[i], (unsigned long long)st[i]);
}

// lane per returned row: scatter into the call-global outputs
__global__ __launch_bounds__(256) void k_route_unpack(const void* __restrict__ back, uint32_t W,
                                                      const uint32_t* __restrict__ rowpos, uint64_t rows,
                                                      uint64_t* __restrict__ vals_out,
                                                      uint8_t* __restrict__ st_out, const void* __restrict__ back_self,
                                                      uint64_t self_lo, uint64_t self_hi) {
  const uint64_t r = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (r >= rows) return;
  const uint32_t p = rowpos[r];
  if (p == kRouteNone) return;
  const void* src = r >= self_lo && r < self_hi ? back_self : back;
  if (W == 0) {
    st_out[p] = ((const uint8_t*)src)[r];
  } else {
    const ulonglong2 x = ((const ulonglong2*)src)[r];
    if (vals_out) vals_out[p] = x.x;
    st_out[p] = (uint8_t)x.y;
  }
}

__global__ __launch_bounds__(64) void k_route_carried(const uint32_t* __restrict__ cnt, uint32_t G,
                                                      uint64_t* __restrict__ out) {
  uint64_t v = threadIdx.x < G ? cnt[threadIdx.x] : 0;
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off);
  if (threadIdx.x == 0) *out = v;
}

// Get dedupe: one 256-thread block per tile of kDedupTile Gets, an LDS
// open-addressing table {key, min index} at load 1/2.  A Zipf-hot key keeps
// one row per tile (1024 per 1M batch) instead of one per Get; the cost is one
// coalesced pass over the keys (a global table costs ~100 us per 1M in
// device-memory atomics).
constexpr uint32_t kDedupThreads = 256;
constexpr uint32_t kDedupTile = 1024;
constexpr uint32_t kDedupBits = 11;  // 2048 LDS slots: 16 KiB keys + 8 KiB indices
__global__ __launch_bounds__(kDedupThreads) void k_dedupe_tile(const uint64_t* __restrict__ keys,
                                                              const uint8_t* __restrict__ keep, uint64_t n,
                                                              uint32_t base, uint8_t* __restrict__ keep_out,
                                                              uint32_t* __restrict__ lead_out) {
  __shared__ unsigned long long tk[1u << kDedupBits];
  __shared__ uint32_t ti[1u << kDedupBits];
  for (uint32_t s = threadIdx.x; s < (1u << kDedupBits); s += kDedupThreads) {
    tk[s] = ~0ULL;
    ti[s] = ~0u;
  }
  __syncthreads();
  constexpr uint32_t kPer = kDedupTile / kDedupThreads;
  constexpr uint32_t mask = (1u << kDedupBits) - 1;
  const uint64_t t0 = (uint64_t)blockIdx.x * kDedupTile;
  uint32_t slot[kPer];
  bool kp[kPer];
#pragma unroll
  for (uint32_t j = 0; j < kPer; ++j) {
    const uint32_t r = j * kDedupThreads + threadIdx.x;  // index in the tile (coalesced)
    const uint64_t i = t0 + r;
    slot[j] = kRouteNone;
    kp[j] = i < n && (!keep || keep[i]);
    if (i >= n) continue;
    const uint64_t k = keys[i];
    if (!kp[j] || k == ~0ULL) continue;  // kept home / the empty marker: own leader
    uint32_t s = (uint32_t)(((k ^ (k >> 29)) * 0x9E3779B97F4A7C15ULL) >> (64 - kDedupBits));
    for (uint32_t step = 0; step <= mask; ++step, s = (s + 1) & mask) {
      unsigned long long cur = tk[s];
      if (cur == ~0ULL) cur = atomicCAS(&tk[s], ~0ULL, (unsigned long long)k);
      if (cur == ~0ULL || cur == k) {
        atomicMin(&ti[s], r);
        slot[j] = s;
        break;
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (uint32_t j = 0; j < kPer; ++j) {
    const uint32_t r = j * kDedupThreads + threadIdx.x;
    const uint64_t i = t0 + r;
    if (i >= n) continue;
    const uint32_t l = slot[j] == kRouteNone ? r : ti[slot[j]];
    keep_out[i] = (uint8_t)(l == r && kp[j]);
    lead_out[base + i] = base + (uint32_t)(t0 + l);
  }
}

__global__ __launch_bounds__(256) void k_route_fill(const uint32_t* __restrict__ lead, uint64_t n,
                                                    uint64_t* __restrict__ vals, uint8_t* __restrict__ st) {
  const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  const uint32_t l = lead[i];
  if (l == (uint32_t)i) return;
  if (vals) vals[i] = vals[l];
  st[i] = st[l];
}

inline dim3 grid_of(uint64_t n, uint32_t per) { return dim3((unsigned)((n + per - 1) / per)); }

}  // namespace

uint32_t route_tiles(uint64_t n) { return (uint32_t)((n + kRouteTile - 1) / kRouteTile); }

void launch_route_pack(const RouteArgs& a, hipStream_t s) {
  const uint32_t G = 1u << a.sbits;
  const uint32_t tiles = route_tiles(a.n);
  if (tiles)
    hipLaunchKernelGGL(k_route_count, dim3(tiles), dim3(kRT), 0, s, a.keys, a.keep, a.n, a.sbits, a.tile_cnt);
  hipLaunchKernelGGL(k_route_scatter, dim3(tiles + G * (kPadPer + kCarryPer)), dim3(kRT), 0, s, a, tiles);
}

void launch_route_split(const uint64_t* recv, uint64_t rows, uint32_t W, uint64_t* keys, uint64_t* vals,
                        uint8_t* ops, hipStream_t s) {
  if (rows) hipLaunchKernelGGL(k_route_split, grid_of(rows, 256), dim3(256), 0, s, recv, rows, W, keys, vals, ops);
}

void launch_route_resp(const uint64_t* vals, const uint8_t* st, uint64_t rows, void* resp, hipStream_t s) {
  if (rows)
    hipLaunchKernelGGL(k_route_resp, grid_of(rows, 256), dim3(256), 0, s, vals, st, rows, (ulonglong2*)resp);
}

void launch_route_unpack(const void* back, uint32_t W, const uint32_t* rowpos, uint64_t rows, uint64_t* vals_out,
                         uint8_t* st_out, hipStream_t s, const void* back_self, uint64_t self_lo, uint64_t self_hi) {
  if (rows)
    hipLaunchKernelGGL(k_route_unpack, grid_of(rows, 256), dim3(256), 0, s, back, W, rowpos, rows, vals_out,
                       st_out, back_self ? back_self : back, self_lo, self_hi);
}

void launch_route_carried(const uint32_t* cnt, uint32_t G, uint64_t* out, hipStream_t s) {
  hipLaunchKernelGGL(k_route_carried, dim3(1), dim3(64), 0, s, cnt, G, out);
}

void launch_route_dedupe(const uint64_t* keys, const uint8_t* keep_in, uint64_t n, uint32_t base, uint8_t* keep_out,
                         uint32_t* lead_out, hipStream_t s) {
  if (n)
    hipLaunchKernelGGL(k_dedupe_tile, grid_of(n, kDedupTile), dim3(kDedupThreads), 0, s, keys, keep_in, n, base,
                       keep_out, lead_out);
}

void launch_route_fill(const uint32_t* lead, uint64_t n, uint64_t* vals, uint8_t* st, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_route_fill, grid_of(n, 256), dim3(256), 0, s, lead, n, vals, st);
}

}  // namespace pmdfc
