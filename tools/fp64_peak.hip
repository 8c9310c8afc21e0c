// FP64 VALU peak microbenchmark (the local MI355X guide has no FP64 figure; the render
// kernel's arithmetic is IEEE fp64, so its issue roofline needs a measured peak).
// Every lane runs K independent v_fma_f64 chains (enough in flight to cover the FMA
// latency), grid >> 256 CUs. Prints FLOP/s (1 FMA = 2 FLOP) and the v_fma_f64 issue rate.
//   hipcc --offload-arch=gfx950 -O3 tools/fp64_peak.hip -o tools/fp64_peak && tools/fp64_peak
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int K = 8;
constexpr int ITERS = 4096;

__global__ void __launch_bounds__(256) fma_kernel(double* out, double a, double b) {
  double x[K];
#pragma unroll
  for (int i = 0; i < K; ++i) x[i] = threadIdx.x * 1e-9 + i;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < K; ++i) x[i] = __builtin_fma(x[i], a, b);
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < K; ++i) s += x[i];
  if (s == 12345.678) out[0] = s;  // keeps the chains alive; never true for these inputs
}

int main() {
  double* d;
  if (hipMalloc(&d, 8) != hipSuccess) { printf("{\"error\": \"hipMalloc\"}\n"); return 1; }
  hipDeviceProp_t pr;
  hipGetDeviceProperties(&pr, 0);
  const int blocks = pr.multiProcessorCount * 64, threads = 256;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int w = 0; w < 3; ++w) fma_kernel<<<blocks, threads>>>(d, 0.999999, 1e-7);
  hipDeviceSynchronize();
  const int reps = 10;
  hipEventRecord(e0);
  for (int r = 0; r < reps; ++r) fma_kernel<<<blocks, threads>>>(d, 0.999999, 1e-7);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  const double fmas = (double)blocks * threads * ITERS * K * reps;
  const double s = ms * 1e-3;
  printf("{\"kernel\": \"fp64_peak\", \"cus\": %d, \"blocks\": %d, \"threads\": %d, \"ms\": %.3f, "
         "\"fp64_tflops\": %.2f, \"fma_f64_per_s\": %.4e, \"fma_f64_per_clk_per_cu\": %.2f, \"clock_mhz_nominal\": %d}\n",
         pr.multiProcessorCount, blocks, threads, ms, 2 * fmas / s / 1e12, fmas / s,
         fmas / s / (pr.clockRate * 1e3) / pr.multiProcessorCount, pr.clockRate / 1000);
  hipFree(d);
  return 0;
}
