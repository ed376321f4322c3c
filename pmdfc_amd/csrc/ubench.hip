// ubench.hip -- random 64-B line gather ceiling (measurement tool for the
// roofline of k_get; SURVEY §8d "measured random-64 B-gather ceiling").
// Same access shape as k_get: 4 lanes per op, one 16-B load each from a
// 64-B-aligned line chosen by a hash of the op index; with `dep` the line
// index first goes through a u32 table (like the CCEH directory).
#include "cceh_device.h"
#include "cceh_kernels.h"

namespace pmdfc {

template <bool DEP>
__global__ __launch_bounds__(256) void k_gather64(const ulonglong2* __restrict__ buf, uint64_t nlines,
                                                  const uint32_t* __restrict__ table, uint32_t tmask,
                                                  uint64_t nops, uint64_t seed,
                                                  uint64_t* __restrict__ out) {
  const uint64_t op = ((uint64_t)blockIdx.x * 256u + threadIdx.x) >> 2;
  const uint32_t q = threadIdx.x & 3u;
  if (op >= nops) return;
  const uint64_t h = hash64(op ^ seed);
  uint64_t line = h % nlines;
  if (DEP) line = ((uint64_t)table[(uint32_t)(h >> 40) & tmask] * 64u + (h & 63u)) % nlines;
  const ulonglong2 p = buf[line * 4u + q];
  uint64_t x = p.x ^ p.y;
  x ^= (uint64_t)__shfl_xor((int)x, 1) ^ (uint64_t)__shfl_xor((int)x, 2);
  if (q == 0) out[op] = x;
}

void launch_gather64(const void* buf, uint64_t nlines, const uint32_t* table, uint32_t tmask,
                     uint64_t nops, uint64_t seed, uint64_t* out, hipStream_t s) {
  const dim3 g((unsigned)((nops + 63) / 64));
  if (table)
    hipLaunchKernelGGL(k_gather64<true>, g, dim3(256), 0, s, (const ulonglong2*)buf, nlines, table,
                       tmask, nops, seed, out);
  else
    hipLaunchKernelGGL(k_gather64<false>, g, dim3(256), 0, s, (const ulonglong2*)buf, nlines, table,
                       tmask, nops, seed, out);
}

}  // namespace pmdfc
