// Microbenchmark (not shipped): is the few-active-lanes issue penalty a
// property of the wave or of the SIMD?  256 workgroups x 512 threads (two
// waves per SIMD); waves 0-3 run a dependent fp64 FMA chain on k0 lanes,
// waves 4-7 on k1 lanes.
// Build: hipcc -O3 --offload-arch=gfx950 scripts/micro/lane_mix.hip -o _ab/lane_mix
#include <hip/hip_runtime.h>
#include <cstdio>
#pragma clang diagnostic ignored "-Wunused-result"

__global__ void __launch_bounds__(512) k(double* out, int k0, int k1, double s, unsigned long long* cyc) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int kact = w < 4 ? k0 : k1;
  double a = out[threadIdx.x] + s;
  unsigned long long t0 = __builtin_readcyclecounter();
  if (lane < kact) {
#pragma unroll 1
    for (int r = 0; r < 256; ++r) {
#pragma unroll
      for (int j = 0; j < 16; ++j) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(a) : "v"(s));
    }
  }
  unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * 512 + threadIdx.x] = a;
  if (lane == 0) cyc[blockIdx.x * 8 + w] = t1 - t0;
}

int main() {
  double* o;
  unsigned long long* c;
  hipMalloc(&o, 256 * 512 * sizeof(double));
  hipMemset(o, 0, 256 * 512 * sizeof(double));
  hipMalloc(&c, 256 * 8 * 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int cfg[][2] = {{64, 64}, {4, 4}, {64, 4}, {4, 64}, {64, 0}, {4, 0}, {16, 16}, {64, 64}};
  for (auto& p : cfg) {
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k, dim3(256), dim3(512), 0, 0, o, p[0], p[1], 1e-3, c);
    hipEventRecord(e0);
    for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(k, dim3(256), dim3(512), 0, 0, o, p[0], p[1], 1e-3, c);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long h[256 * 8];
    hipMemcpy(h, c, sizeof(h), hipMemcpyDeviceToHost);
    double a = 0, b = 0;
    for (int i = 0; i < 256; ++i)
      for (int w = 0; w < 8; ++w) (w < 4 ? a : b) += h[i * 8 + w];
    printf("waves0-3 k=%2d, waves4-7 k=%2d: %7.2f us per launch; mean cycle counter per wave %8.0f / %8.0f\n", p[0], p[1],
           ms * 1e3 / 10, a / 1024, b / 1024);
  }
  return 0;
}
