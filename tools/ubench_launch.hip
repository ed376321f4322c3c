// Empty-kernel launch cost vs grid size and LDS (measurement tool, not
// product code): back-to-back launches of a kernel whose waves exit after one
// load, as the bucket passes' empty launches do.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int LDS>
__global__ __launch_bounds__(64) void k_empty(const uint32_t* flag, uint32_t* out) {
  __shared__ uint32_t s[LDS / 4 + 1];
  if (flag[0] == 0) return;
  s[threadIdx.x] = threadIdx.x;
  __syncthreads();
  out[blockIdx.x] = s[(threadIdx.x + 1) & 63];
}

template <int LDS>
float run(uint32_t grid, const uint32_t* flag, uint32_t* out, int reps) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int r = 0; r < 10; ++r) hipLaunchKernelGGL(k_empty<LDS>, dim3(grid), dim3(64), 0, 0, flag, out);
  hipEventRecord(a);
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_empty<LDS>, dim3(grid), dim3(64), 0, 0, flag, out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1000.f / reps;
}

int main() {
  uint32_t *flag, *out;
  hipMalloc(&flag, 4);
  hipMalloc(&out, 1 << 20);
  hipMemset(flag, 0, 4);
  const uint32_t grids[] = {1, 8, 64, 256, 1024, 4096, 8192, 16384};
  printf("empty launches, us per launch (back to back, 2000 reps)\n");
  printf("%8s %10s %10s %10s\n", "grid", "lds0", "lds10k", "lds32k");
  for (uint32_t g : grids)
    printf("%8u %10.2f %10.2f %10.2f\n", g, run<4>(g, flag, out, 2000), run<10240>(g, flag, out, 2000),
           run<32768>(g, flag, out, 2000));
  // a graph of 4 empty kernels
  hipStream_t s;
  hipStreamCreate(&s);
  hipGraph_t gr;
  hipGraphExec_t ge;
  hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
  for (int k = 0; k < 4; ++k) hipLaunchKernelGGL(k_empty<4>, dim3(1024), dim3(64), 0, s, flag, out);
  hipStreamEndCapture(s, &gr);
  hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int r = 0; r < 10; ++r) hipGraphLaunch(ge, s);
  hipEventRecord(a, s);
  for (int r = 0; r < 500; ++r) hipGraphLaunch(ge, s);
  hipEventRecord(b, s);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  printf("graph of 4 empty kernels (grid 1024): %.2f us per kernel\n", ms * 1000.f / 500 / 4);
  return 0;
}
