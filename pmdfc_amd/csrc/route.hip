// route.hip -- fixed-capacity shard routing for the multi-GPU path.
//
// The key space shards by the top shard_bits of h(key), the bits CCEH indexes
// its directory with (CCEH_hybrid.cpp:119), so each op has exactly one owner
// GPU.  A batch is exchanged with equal-split RCCL all-to-alls: every rank
// sends every owner a block of `cap` records, the owner's ops first (in batch
// order), the rest padded with key INVALID (server/util/pair.h:10), which the
// engine answers with RESERVED_KEY and never stores.  Equal splits mean the
// exchange needs no counts on the host, so a routed batch has no host sync.
// Ops past `cap` for one owner (far outside the hash's binomial spread at the
// default slack) come back as PMDFC_ST_ROUTE_OVERFLOW and are not applied.
//
//   k_route_count   tile of 1024 ops -> per-owner counts
//   k_route_scatter tile offsets from the counts of the tiles before it (L2
//                   reads); stable in-tile ranks by ballot; records
//                   {key[, value[, op]]} to send[owner][slot];
//                   pos[i] = owner * cap + slot
//                   + kPadPer extra blocks per owner: key INVALID into the
//                   unused slots [total, cap) of its block (no memset)
//   k_route_split   received records -> engine key / value / op arrays
//   k_route_resp    engine (value, status) -> 16-B response records
//   k_route_unpack  returned responses -> batch order via pos
// An optional keep mask (the replicated bloom filter's probe)
// keeps negatives home: they take no slot, never cross xGMI, and unpack
// reports them PMDFC_ST_FILTERED.
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

__device__ __forceinline__ uint32_t owner_of(uint64_t key, uint32_t sbits) {
  return sbits ? (uint32_t)(hash64(key) >> (64 - sbits)) : 0u;
}

__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__global__ __launch_bounds__(kRT) void k_route_count(const uint64_t* __restrict__ keys,
                                                     const uint8_t* __restrict__ keep, uint64_t n,
                                                     uint32_t sbits, uint32_t* __restrict__ tile_cnt,
                                                     uint32_t* __restrict__ overflow) {
  __shared__ uint32_t cnt[kRouteMaxOwners];
  const uint32_t G = 1u << sbits;
  if (blockIdx.x == 0 && threadIdx.x == 0) *overflow = 0;  // k_route_scatter runs after this kernel
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

// blocks [0, tiles): one tile each; blocks [tiles, tiles + G * kPadPer): padding
__device__ __forceinline__ void route_pad(const RouteArgs& a, uint32_t tiles, uint32_t pb) {
  __shared__ uint32_t s_tot;
  const uint32_t G = 1u << a.sbits, g = pb / kPadPer, part = pb % kPadPer;
  if (threadIdx.x == 0) {
    s_tot = 0;
    if (tiles == 0 && pb == 0) *a.overflow = 0;  // empty batch: no k_route_count
  }
  __syncthreads();
  uint32_t acc = 0;
  for (uint32_t t = threadIdx.x; t < tiles; t += kRT) acc += a.tile_cnt[(size_t)t * G + g];
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off);
  if ((threadIdx.x & 63u) == 0) atomicAdd(&s_tot, acc);
  __syncthreads();
  const uint64_t lo = min<uint64_t>(s_tot, a.cap);
  const uint64_t words = (a.cap - lo) * a.width;
  const uint64_t chunk = (words + kPadPer - 1) / kPadPer;
  const uint64_t e0 = part * chunk, e1 = min<uint64_t>(words, e0 + chunk);
  uint64_t* blk = a.send + ((uint64_t)g * a.cap + lo) * a.width;
  for (uint64_t e = e0 + threadIdx.x; e < e1; e += kRT) blk[e] = ~0ULL;
}

__global__ __launch_bounds__(kRT) void k_route_scatter(RouteArgs a, uint32_t tiles) {
  __shared__ uint32_t s_base[kRouteMaxOwners];         // running slot per owner
  __shared__ uint32_t s_wc[kRT / 64][kRouteMaxOwners];  // per-wave counts of a chunk
  if (blockIdx.x >= tiles) {
    route_pad(a, tiles, blockIdx.x - tiles);
    return;
  }
  const uint32_t G = 1u << a.sbits;
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  if (threadIdx.x < G) s_base[threadIdx.x] = 0;
  __syncthreads();
  // slots taken by the tiles before this one: the (tile, owner) counts are
  // read as one flat array, element e belongs to owner e % G
  {
    const uint32_t ne = blockIdx.x * G;  // G divides kRT, so e % G == threadIdx.x % G
    uint32_t acc = 0;
    for (uint32_t e = threadIdx.x; e < ne; e += kRT) acc += a.tile_cnt[e];
    // lanes l and l + G, l + 2G, ... hold the same owner: fold them
    for (uint32_t off = 32; off >= G && off > 0; off >>= 1) acc += __shfl_down(acc, off);
    if (lane < G) atomicAdd(&s_base[lane], acc);
  }
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x * kRouteTile;
  const uint32_t W = a.width;
  for (uint32_t j = 0; j < kRPer; ++j) {
    const uint64_t i = base + j * kRT + threadIdx.x;
    const bool inb = i < a.n;
    const bool live = inb && (!a.keep || a.keep[i]);
    if (inb && !live) a.pos[i] = kRouteFiltered;
    const uint64_t key = live ? a.keys[i] : 0;
    const uint32_t o = live ? owner_of(key, a.sbits) : G;
    uint32_t r = 0;
#pragma unroll
    for (uint32_t g = 0; g < kRouteMaxOwners; ++g) {
      if (g < G) {
        const uint64_t m = __ballot(o == g);
        if (o == g) r = lanes_below(m);
        if (lane == 0) s_wc[wave][g] = (uint32_t)__popcll(m);
      }
    }
    __syncthreads();
    if (live) {
      uint32_t slot = s_base[o] + r;
      for (uint32_t w = 0; w < wave; ++w) slot += s_wc[w][o];
      if (slot < a.cap) {
        const size_t at = (size_t)o * a.cap + slot;
        uint64_t* rec = a.send + at * W;
        if (W == 2) {  // 16-B record, one store
          *reinterpret_cast<ulonglong2*>(rec) = make_ulonglong2(key, a.vals[i]);
        } else {
          rec[0] = key;
          if (W > 2) {
            rec[1] = a.vals[i];
            rec[2] = (uint64_t)a.ops[i];
          }
        }
        a.pos[i] = (uint32_t)at;
      } else {
        a.pos[i] = 0xFFFFFFFFu;
        atomicOr(a.overflow, 1u);
      }
    }
    __syncthreads();
    if (threadIdx.x < G) {
      uint32_t add = 0;
      for (uint32_t w = 0; w < kRT / 64; ++w) add += s_wc[w][threadIdx.x];
      s_base[threadIdx.x] += add;
    }
    __syncthreads();
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

__global__ __launch_bounds__(256) void k_route_unpack(const void* __restrict__ back, uint32_t W,
                                                      const uint32_t* __restrict__ pos, uint64_t n,
                                                      uint64_t* __restrict__ vals_out,
                                                      uint8_t* __restrict__ st_out) {
  const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  const uint32_t p = pos[i];
  if (p >= kRouteFiltered) {  // overflow, or kept home by the bloom filter
    if (vals_out) vals_out[i] = 0;
    st_out[i] = (uint8_t)(p == kRouteFiltered ? kStFiltered : kStOverflow);
    return;
  }
  if (W == 0) {
    st_out[i] = ((const uint8_t*)back)[p];
  } else {
    const ulonglong2 r = ((const ulonglong2*)back)[p];
    if (vals_out) vals_out[i] = r.x;
    st_out[i] = (uint8_t)r.y;
  }
}

inline dim3 grid_of(uint64_t n, uint32_t per) { return dim3((unsigned)((n + per - 1) / per)); }

}  // namespace

uint32_t route_tiles(uint64_t n) { return (uint32_t)((n + kRouteTile - 1) / kRouteTile); }

void launch_route_pack(const RouteArgs& a, hipStream_t s) {
  const uint32_t G = 1u << a.sbits;
  const uint32_t tiles = route_tiles(a.n);
  if (tiles)
    hipLaunchKernelGGL(k_route_count, dim3(tiles), dim3(kRT), 0, s, a.keys, a.keep, a.n, a.sbits, a.tile_cnt,
                       a.overflow);
  // + padding blocks: unused slots of every owner block get key INVALID (0xFF.. values / ops)
  hipLaunchKernelGGL(k_route_scatter, dim3(tiles + G * kPadPer), dim3(kRT), 0, s, a, tiles);
}

void launch_route_split(const uint64_t* recv, uint64_t rows, uint32_t W, uint64_t* keys, uint64_t* vals,
                        uint8_t* ops, hipStream_t s) {
  if (rows) hipLaunchKernelGGL(k_route_split, grid_of(rows, 256), dim3(256), 0, s, recv, rows, W, keys, vals, ops);
}

void launch_route_resp(const uint64_t* vals, const uint8_t* st, uint64_t rows, void* resp, hipStream_t s) {
  if (rows)
    hipLaunchKernelGGL(k_route_resp, grid_of(rows, 256), dim3(256), 0, s, vals, st, rows, (ulonglong2*)resp);
}

void launch_route_unpack(const void* back, uint32_t W, const uint32_t* pos, uint64_t n, uint64_t* vals_out,
                         uint8_t* st_out, hipStream_t s) {
  if (n)
    hipLaunchKernelGGL(k_route_unpack, grid_of(n, 256), dim3(256), 0, s, back, W, pos, n, vals_out, st_out);
}

}  // namespace pmdfc
