// bloom.hip -- the client bloom filter (client/bloom_filter.c) as batched
// gfx950 kernels.  Bitmap = ceil(nbits/64) u64 words, bit (63 - idx%64) of
// word idx/64 (MSB-first, bloom_filter.c:71-74,100-103), idx =
// murmur2(&key, 8, i) % nbits for i < k (bloom_filter.c:69,93).
#include "cceh_device.h"
#include "cceh_kernels.h"

namespace pmdfc {

__device__ __forceinline__ uint64_t bloom_idx(uint64_t key, uint32_t i, uint64_t nbits) {
  return (uint64_t)murmur2_u64(key, i) % nbits;
}

// bloom_filter_add (bloom_filter.c:61-80); atomicOr makes concurrent adds safe
__global__ __launch_bounds__(256) void k_bloom_add(uint64_t* __restrict__ bm, uint64_t nbits,
                                                   uint32_t k, const uint64_t* __restrict__ keys,
                                                   uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  const uint64_t key = keys[i];
  for (uint32_t j = 0; j < k; ++j) {
    const uint64_t idx = bloom_idx(key, j, nbits);
    atomicOr((unsigned long long*)&bm[idx >> 6], 1ULL << (63 - (idx & 63)));
  }
}

// bloom_filter_check (bloom_filter.c:82-117): probes in order, stops at the
// first clear bit.  One lane per key.
__global__ __launch_bounds__(256) void k_bloom_probe(const uint64_t* __restrict__ bm,
                                                     uint64_t nbits, uint32_t k,
                                                     const uint64_t* __restrict__ keys,
                                                     uint8_t* __restrict__ out, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  const uint64_t key = keys[i];
  uint8_t r = 1;
  for (uint32_t j = 0; j < k; ++j) {
    const uint64_t idx = bloom_idx(key, j, nbits);
    if (!((bm[idx >> 6] >> (63 - (idx & 63))) & 1ULL)) {
      r = 0;
      break;
    }
  }
  out[i] = r;
}

// Fused client path (client/rdpma.c:1050-1061 then the server Get): one quad
// per key.  Lane q tests hash q (q, q+4, ... for k > 4) in parallel; a negative
// key is FILTERED without touching the index, a positive one runs the
// quad-cooperative CCEH probe.
__global__ __launch_bounds__(256) void k_bloom_get(const uint64_t* __restrict__ bm,
                                                   uint64_t nbits, uint32_t k,
                                                   const uint64_t* __restrict__ keys,
                                                   uint64_t* __restrict__ vout,
                                                   uint8_t* __restrict__ st, uint64_t n, Geo g,
                                                   const ulonglong2* __restrict__ pairs) {
  const uint64_t op = ((uint64_t)blockIdx.x * 256u + threadIdx.x) >> 2;
  const uint32_t q = threadIdx.x & 3u;
  if (op >= n) return;
  const uint64_t key = keys[op];
  bool ok = true;
  for (uint32_t j = q; j < k; j += 4) {
    const uint64_t idx = bloom_idx(key, j, nbits);
    ok = ok && ((bm[idx >> 6] >> (63 - (idx & 63))) & 1ULL);
  }
  const uint32_t qbase = (__lane_id() & 63u) & ~3u;
  const bool pos = (((uint32_t)(__ballot(!ok) >> qbase)) & 0xFu) == 0;
  uint64_t val = 0;
  uint8_t s;
  if (!pos) {
    s = 7;  // PMDFC_ST_FILTERED
  } else {
    const uint64_t h = hash64(key);
    if (reserved_key(key)) {
      s = 3;
    } else if (wrong_shard(h, g.sbits, g.shard)) {
      s = 8;
    } else {
      uint32_t lines;
      const uint32_t seg = de_seg(dir_entry(g, h));
      s = quad_probe(pairs + (size_t)seg * kSlots, key, h, q, &val, &lines);
    }
  }
  if (q == 0) {
    vout[op] = val;
    st[op] = s;
  }
}

#define GRID(n, per) dim3((unsigned)(((n) + (per)-1) / (per)))

void launch_bloom_add(uint64_t* bitmap, uint64_t nbits, uint32_t k, const uint64_t* keys,
                      uint64_t n, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_bloom_add, GRID(n, 256), dim3(256), 0, s, bitmap, nbits, k, keys, n);
}

void launch_bloom_probe(const uint64_t* bitmap, uint64_t nbits, uint32_t k, const uint64_t* keys,
                        uint8_t* out, uint64_t n, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_bloom_probe, GRID(n, 256), dim3(256), 0, s, bitmap, nbits, k, keys, out, n);
}

void launch_bloom_get(const uint64_t* bitmap, uint64_t nbits, uint32_t k, const uint64_t* keys,
                      uint64_t* vout, uint8_t* st, uint64_t n, Geo g, const ulonglong2* pairs,
                      hipStream_t s) {
  if (n)
    hipLaunchKernelGGL(k_bloom_get, GRID(n, 64), dim3(256), 0, s, bitmap, nbits, k, keys, vout, st,
                       n, g, pairs);
}

}  // namespace pmdfc
