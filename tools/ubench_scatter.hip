// Scattered store/load microbenchmark (measurement tool, not product code):
// n random granules of G bytes (G = 16, 64, 128) into a large buffer,
// written (or read) by G/16 consecutive lanes with 16-B accesses.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
  return x;
}

template <int G, bool STORE, bool NT>
__global__ __launch_bounds__(256) void k_scatter(uint4* buf, uint64_t nlines, uint64_t n, uint64_t seed, uint32_t* sink) {
  constexpr int LPG = G / 16;  // lanes per granule
  const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint64_t g = t / LPG;
  if (g >= n) return;
  const uint64_t line = mix(g + seed) % nlines;          // G-aligned granule index
  uint4* p = buf + line * LPG + (t % LPG);
  if (STORE) {
    const uint4 v = make_uint4((uint32_t)g, 1, 2, 3);
    if (NT) __builtin_nontemporal_store(v.x, &p->x), __builtin_nontemporal_store(v.y, &p->y),
            __builtin_nontemporal_store(v.z, &p->z), __builtin_nontemporal_store(v.w, &p->w);
    else *p = v;
  } else {
    const uint4 v = *p;
    if (v.x == 0xdeadbeef) sink[0] = v.y;
  }
}

template <int G, bool STORE, bool NT>
float run(uint4* buf, uint64_t bytes, uint64_t n, uint32_t* sink) {
  const uint64_t nlines = bytes / G;
  const uint64_t threads = n * (G / 16);
  dim3 grid((unsigned)((threads + 255) / 256));
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  hipLaunchKernelGGL((k_scatter<G, STORE, NT>), grid, dim3(256), 0, 0, buf, nlines, n, 1, sink);
  hipDeviceSynchronize();
  hipEventRecord(a);
  const int reps = 10;
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((k_scatter<G, STORE, NT>), grid, dim3(256), 0, 0, buf, nlines, n, r + 2, sink);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  return ms * 1000.f / reps;
}

int main() {
  const uint64_t bytes = 4ULL << 30, n = 1 << 20;
  uint4* buf; uint32_t* sink;
  hipMalloc(&buf, bytes); hipMalloc(&sink, 64);
  hipMemset(buf, 0, bytes);
  printf("1M granules over 4 GiB, us per launch\n");
  printf("load  16B %8.1f  64B %8.1f  128B %8.1f\n", run<16, false, false>(buf, bytes, n, sink),
         run<64, false, false>(buf, bytes, n, sink), run<128, false, false>(buf, bytes, n, sink));
  printf("store 16B %8.1f  64B %8.1f  128B %8.1f\n", run<16, true, false>(buf, bytes, n, sink),
         run<64, true, false>(buf, bytes, n, sink), run<128, true, false>(buf, bytes, n, sink));
  printf("ntst  16B %8.1f  64B %8.1f  128B %8.1f\n", run<16, true, true>(buf, bytes, n, sink),
         run<64, true, true>(buf, bytes, n, sink), run<128, true, true>(buf, bytes, n, sink));
  return 0;
}
