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

// The same shape at full scale (the bench's gather ceiling): LINE-byte lines
// (64 or 128), LINE/16 lanes per line, DEPTH independent random lines per lane
// group with all loads issued before any use (DEPTH lines in flight per lane),
// optionally through the dependent table.  One xor-folded u64 per lane group
// lands in out[group & omask] so the loads cannot be elided.
template <int LINE, int DEPTH, bool DEP>
__global__ __launch_bounds__(256) void k_gather(const ulonglong2* __restrict__ buf, uint64_t nlines,
                                                const uint32_t* __restrict__ table, uint32_t tmask,
                                                uint64_t ngroups, uint64_t seed, uint64_t* __restrict__ out,
                                                uint64_t omask) {
  constexpr uint32_t L = LINE / 16;  // lanes per line
  const uint64_t g = ((uint64_t)blockIdx.x * 256u + threadIdx.x) / L;
  const uint32_t q = threadIdx.x % L;
  if (g >= ngroups) return;
  ulonglong2 p[DEPTH];
#pragma unroll
  for (int d = 0; d < DEPTH; ++d) {
    const uint64_t h = hash64((g * DEPTH + d) ^ seed);
    uint64_t line = h % nlines;
    if (DEP) line = ((uint64_t)table[(uint32_t)(h >> 40) & tmask] * 64u + (h & 63u)) % nlines;
    p[d] = buf[line * L + q];
  }
  uint64_t x = 0;
#pragma unroll
  for (int d = 0; d < DEPTH; ++d) x ^= p[d].x ^ p[d].y;
  for (uint32_t m = 1; m < L; m <<= 1) x ^= (uint64_t)(uint32_t)__shfl_xor((int)x, (int)m);
  if (q == 0) out[g & omask] = x;
}

template <int LINE, int DEPTH>
static void gather_launch(const void* buf, uint64_t nlines, const uint32_t* table, uint32_t tmask, uint64_t nops,
                          uint64_t seed, uint64_t* out, uint64_t omask, hipStream_t s) {
  const uint64_t ng = nops / DEPTH;
  const dim3 grid((unsigned)((ng * (LINE / 16) + 255) / 256));
  if (table)
    hipLaunchKernelGGL((k_gather<LINE, DEPTH, true>), grid, dim3(256), 0, s, (const ulonglong2*)buf, nlines,
                       table, tmask, ng, seed, out, omask);
  else
    hipLaunchKernelGGL((k_gather<LINE, DEPTH, false>), grid, dim3(256), 0, s, (const ulonglong2*)buf, nlines,
                       table, tmask, ng, seed, out, omask);
}

int launch_gather(const void* buf, uint64_t nbytes, uint32_t line, uint32_t depth, const uint32_t* table,
                  uint32_t tmask, uint64_t nops, uint64_t seed, uint64_t* out, uint64_t omask, hipStream_t s) {
  const uint64_t nlines = nbytes / line;
  if (!nlines) return -1;
#define GL(LN, D)                                                                     \
  if (line == LN && depth == D) {                                                     \
    gather_launch<LN, D>(buf, nlines, table, tmask, nops, seed, out, omask, s);      \
    return 0;                                                                         \
  }
  GL(64, 1) GL(64, 2) GL(64, 4) GL(128, 1) GL(128, 2) GL(128, 4)
#undef GL
  return -1;
}

// Random 16-B store ceiling (the shape of an insert's pair store: one lane
// writes one {key, value} pair into a random slot of a large arena): n_ops
// stores of 16 B at random 16-B-aligned offsets of buf, `depth` stores per
// lane, all issued back to back.
template <int DEPTH>
__global__ __launch_bounds__(256) void k_scatter16(ulonglong2* __restrict__ buf, uint64_t nslots, uint64_t nlanes,
                                                   uint64_t seed) {
  const uint64_t t = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (t >= nlanes) return;
#pragma unroll
  for (int d = 0; d < DEPTH; ++d) {
    const uint64_t h = hash64((t * DEPTH + d) ^ seed);
    buf[h % nslots] = make_ulonglong2(h, t);
  }
}

int launch_scatter16(void* buf, uint64_t nbytes, uint32_t depth, uint64_t nops, uint64_t seed, hipStream_t s) {
  const uint64_t nslots = nbytes / 16;
  if (!nslots || (depth != 1 && depth != 4) || nops % depth) return -1;
  const uint64_t nl = nops / depth;
  const dim3 grid((unsigned)((nl + 255) / 256));
  if (depth == 1)
    hipLaunchKernelGGL(k_scatter16<1>, grid, dim3(256), 0, s, (ulonglong2*)buf, nslots, nl, seed);
  else
    hipLaunchKernelGGL(k_scatter16<4>, grid, dim3(256), 0, s, (ulonglong2*)buf, nslots, nl, seed);
  return 0;
}

}  // namespace pmdfc
