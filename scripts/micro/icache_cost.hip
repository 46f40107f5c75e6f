// Microbenchmark (not shipped): what cold instruction fetch costs a short
// launch on gfx950.  A kernel executes K VALU instructions once per wave,
// either as straight-line code (K distinct instructions, every line fetched
// cold after the dispatch's cache invalidation) or as a 64-instruction loop
// body run K/64 times (warm after the first pass).  Difference = fetch cost.
// One wave per SIMD (256 x 256 threads) and the 8-GPU strong share (32 x 256).
// Build: hipcc -O3 --offload-arch=gfx950 scripts/micro/icache_cost.hip -o _ab/icache_cost
#include <hip/hip_runtime.h>

#include <cstdio>


template <int K>
__global__ void __launch_bounds__(256) k_line(int* out) {
  int a = threadIdx.x, b = blockIdx.x;
  asm volatile(".rept %2\n v_add_u32 %0, %0, %1\n .endr" : "+v"(a) : "v"(b), "n"(K));
  if (a == -12345) out[0] = a;
}

template <int K>
__global__ void __launch_bounds__(256) k_loop(int* out) {
  int a = threadIdx.x, b = blockIdx.x;
#pragma unroll 1
  for (int r = 0; r < K / 64; ++r) {
    asm volatile(".rept 64\n v_add_u32 %0, %0, %1\n .endr" : "+v"(a) : "v"(b));
  }
  if (a == -12345) out[0] = a;
}

template <int K>
__global__ void __launch_bounds__(256) k_line64(int* out) {
  double a = threadIdx.x, b = blockIdx.x;
  asm volatile(".rept %2\n v_add_f64 %0, %0, %1\n .endr" : "+v"(a) : "v"(b), "n"(K));
  if (a == -12345.0) out[0] = 1;
}

template <int K>
__global__ void __launch_bounds__(256) k_loop64(int* out) {
  double a = threadIdx.x, b = blockIdx.x;
#pragma unroll 1
  for (int r = 0; r < K / 64; ++r) {
    asm volatile(".rept 64\n v_add_f64 %0, %0, %1\n .endr" : "+v"(a) : "v"(b));
  }
  if (a == -12345.0) out[0] = 1;
}

template <typename F>
float per_launch_us(F launch) {
  hipEvent_t s, e;
  hipEventCreate(&s);
  hipEventCreate(&e);
  for (int r = 0; r < 50; ++r) launch();
  hipDeviceSynchronize();
  const int reps = 1000;
  hipEventRecord(s);
  for (int r = 0; r < reps; ++r) launch();
  hipEventRecord(e);
  hipEventSynchronize(e);
  float ms;
  hipEventElapsedTime(&ms, s, e);
  return ms * 1e3f / reps;
}

template <int K>
void row(int* out) {
  for (int blocks : {256, 32}) {
    const float l = per_launch_us([&] { hipLaunchKernelGGL(k_line<K>, dim3(blocks), dim3(256), 0, 0, out); });
    const float p = per_launch_us([&] { hipLaunchKernelGGL(k_loop<K>, dim3(blocks), dim3(256), 0, 0, out); });
    const float l8 = per_launch_us([&] { hipLaunchKernelGGL(k_line64<K>, dim3(blocks), dim3(256), 0, 0, out); });
    const float p8 = per_launch_us([&] { hipLaunchKernelGGL(k_loop64<K>, dim3(blocks), dim3(256), 0, 0, out); });
    printf("K=%5d blocks=%3d  u32: line %7.2f loop %7.2f us (code %6d B) | f64: line %7.2f loop %7.2f us (code %6d B)\n",
           K, blocks, l, p, 4 * K, l8, p8, 8 * K);
  }
}

int main() {
  int* out;
  hipMalloc(&out, 64);
  row<64>(out);
  row<1024>(out);
  row<2048>(out);
  row<4096>(out);
  row<8192>(out);
  return 0;
}
