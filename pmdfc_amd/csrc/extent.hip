// extent.hip -- the index's extent API on the device.
//
// An extent (key, len) is stored as a chain of power-of-two sub-extents, one
// index entry per sub-extent head, all with the extent's value.  The two
// reference variants differ:
//   hybrid  CCEH_hybrid.cpp:90-105   Insert_extent(key, value, len):
//           cover = 1 << (ffs((int)head) - 1) as unsigned int (0 when the low
//           32 bits are 0 -> 1 << EXTENT_MAX_HEIGHT), halved while > len.
//           Get_extent(key) (:330-341): first nonzero Get(key - key % 2^h),
//           h = 0..EXTENT_MAX_HEIGHT-1.
//   src     src/cceh.cpp:308-330      Insert_extent(key, cluster, len, value):
//           odd head -> 1; else 1 << ctz(min(len, 1 << (ffs((int)head) - 1)))
//           (64-bit shift count masked as on x86); head 0 -> len / 2.
//           Get_extent(key, cluster) (:381-391) returns Get(key + cluster).
// Widths follow the reference (ffs on int, ctz on unsigned int, unsigned int
// cover); lens are < 2^31, beyond which the reference's int shifts overflow.
// Batches expand by count -> inclusive scan -> lane-per-extent expansion, and
// then run through the ordinary batched Insert, so a batch of extents equals
// the reference's Insert_extent calls in batch order.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "cceh_kernels.h"

namespace pmdfc {

constexpr uint32_t kExtentMaxHeight = 30;  // EXTENT_MAX_HEIGHT (CCEH_hybrid.cpp:13, src/cceh.cpp:13)

__device__ __forceinline__ uint32_t ffs32(uint64_t x) {  // ffs((int)x)
  const uint32_t lo = (uint32_t)x;
  return lo ? (uint32_t)__builtin_ctz(lo) + 1u : 0u;
}

// size of the sub-extent at `head` with `len` pages left (len >= 2)
__device__ __forceinline__ uint64_t sub_hybrid(uint64_t head, uint64_t len) {
  const uint32_t f = ffs32(head);
  uint32_t cover = f ? (uint32_t)(1ull << (f - 1)) : 0u;
  if (cover == 0) cover = 1u << kExtentMaxHeight;
  while ((uint64_t)cover > len) cover >>= 1;
  return cover;
}

__device__ __forceinline__ uint64_t sub_src(uint64_t cur, uint64_t len) {
  if (cur & 1ull) return 1;
  if (cur == 0) return len / 2;
  const uint64_t order = (uint64_t)((int64_t)ffs32(cur) - 1);
  const uint64_t lim = min(len, 1ull << (order & 63));
  const uint32_t l32 = (uint32_t)lim;
  return 1ull << (l32 ? __builtin_ctz(l32) : 32);
}

// hybrid: heads walk key, key + c0, ...; src: heads are key + cluster, ...
template <bool SRC>
__device__ __forceinline__ uint64_t walk(uint64_t key, uint64_t cl, uint64_t len, uint64_t* out_k,
                                         uint64_t* out_v, uint64_t v) {
  uint64_t cnt = 0;
  uint64_t head = SRC ? key + cl : key;
  while (len > 0) {
    if (out_k) {
      out_k[cnt] = head;
      out_v[cnt] = v;
    }
    ++cnt;
    if (len == 1) break;
    const uint64_t sub = SRC ? sub_src(head, len) : sub_hybrid(head, len);
    head += sub;
    len -= sub;
  }
  return cnt;
}

template <bool SRC>
__global__ __launch_bounds__(256) void k_extent_count(const uint64_t* __restrict__ keys,
                                                      const uint64_t* __restrict__ cl,
                                                      const uint64_t* __restrict__ lens, uint64_t n,
                                                      uint64_t* __restrict__ cnt) {
  const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  cnt[i] = walk<SRC>(keys[i], cl ? cl[i] : 0, lens[i], nullptr, nullptr, 0);
}

template <bool SRC>
__global__ __launch_bounds__(256) void k_extent_expand(const uint64_t* __restrict__ keys,
                                                       const uint64_t* __restrict__ cl,
                                                       const uint64_t* __restrict__ lens,
                                                       const uint64_t* __restrict__ vals, uint64_t n,
                                                       const uint64_t* __restrict__ cum,
                                                       uint64_t* __restrict__ out_k,
                                                       uint64_t* __restrict__ out_v) {
  const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  const uint64_t base = i ? cum[i - 1] : 0;
  walk<SRC>(keys[i], cl ? cl[i] : 0, lens[i], out_k + base, out_v + base, vals[i]);
}

// Get_extent targets: src -> one (key + cluster); hybrid -> key - key % 2^h
__global__ __launch_bounds__(256) void k_extent_targets(const uint64_t* __restrict__ keys,
                                                        const uint64_t* __restrict__ cl, uint64_t n,
                                                        uint32_t per, uint64_t* __restrict__ out) {
  const uint64_t j = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (j >= n * per) return;
  const uint64_t i = j / per;
  const uint32_t h = (uint32_t)(j - i * per);
  const uint64_t k = keys[i];
  out[j] = per == 1 ? k + (cl ? cl[i] : 0) : k - k % (1ull << h);
}

// first target whose Get returned a nonzero value ("if (result) return result")
__global__ __launch_bounds__(256) void k_extent_pick(const uint64_t* __restrict__ v,
                                                     const uint8_t* __restrict__ st, uint64_t n,
                                                     uint32_t per, uint64_t* __restrict__ vout,
                                                     uint8_t* __restrict__ sout) {
  const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  uint64_t r = 0;
  uint8_t s = 0;  // PMDFC_ST_MISS
  for (uint32_t h = 0; h < per; ++h) {
    const uint8_t sh = st[i * per + h];
    if (sh == 1 && v[i * per + h] != 0) {  // PMDFC_ST_HIT
      r = v[i * per + h];
      s = 1;
      break;
    }
    if (sh != 0 && sh != 1) {  // reserved key / wrong shard: report it
      s = sh;
      break;
    }
  }
  vout[i] = r;
  sout[i] = s;
}

#define GRID(n, per) dim3((unsigned)(((n) + (per)-1) / (per)))

hipError_t launch_extent_count(bool src, const uint64_t* keys, const uint64_t* cl, const uint64_t* lens,
                               uint64_t n, uint64_t* cnt, uint64_t* cum, hipStream_t s) {
  if (!n) return hipSuccess;
  if (src) hipLaunchKernelGGL(k_extent_count<true>, GRID(n, 256), dim3(256), 0, s, keys, cl, lens, n, cnt);
  else hipLaunchKernelGGL(k_extent_count<false>, GRID(n, 256), dim3(256), 0, s, keys, cl, lens, n, cnt);
  size_t tb = 0;
  hipError_t e = hipcub::DeviceScan::InclusiveSum(nullptr, tb, cnt, cum, n, s);
  if (e != hipSuccess) return e;
  void* temp = nullptr;
  e = hipMallocAsync(&temp, tb, s);
  if (e != hipSuccess) return e;
  e = hipcub::DeviceScan::InclusiveSum(temp, tb, cnt, cum, n, s);
  hipError_t e2 = hipFreeAsync(temp, s);
  return e != hipSuccess ? e : e2;
}

void launch_extent_expand(bool src, const uint64_t* keys, const uint64_t* cl, const uint64_t* lens,
                          const uint64_t* vals, uint64_t n, const uint64_t* cum, uint64_t* out_k,
                          uint64_t* out_v, hipStream_t s) {
  if (!n) return;
  if (src)
    hipLaunchKernelGGL(k_extent_expand<true>, GRID(n, 256), dim3(256), 0, s, keys, cl, lens, vals, n, cum,
                       out_k, out_v);
  else
    hipLaunchKernelGGL(k_extent_expand<false>, GRID(n, 256), dim3(256), 0, s, keys, cl, lens, vals, n,
                       cum, out_k, out_v);
}

uint32_t extent_targets_per_key(bool src) { return src ? 1u : kExtentMaxHeight; }

void launch_extent_targets(const uint64_t* keys, const uint64_t* cl, uint64_t n, uint32_t per,
                           uint64_t* out, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_extent_targets, GRID(n * per, 256), dim3(256), 0, s, keys, cl, n, per, out);
}

void launch_extent_pick(const uint64_t* v, const uint8_t* st, uint64_t n, uint32_t per, uint64_t* vout,
                        uint8_t* sout, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_extent_pick, GRID(n, 256), dim3(256), 0, s, v, st, n, per, vout, sout);
}

}  // namespace pmdfc
