// Microbenchmark (not shipped): does the cost of a dependent fp64 chain depend
// on how many lanes of the wave are active?  256 workgroups x 256 threads (one
// wave per SIMD); in every wave lanes < k run the chain, the rest skip it.
// Build: hipcc -O3 --offload-arch=gfx950 scripts/micro/lane_count.hip -o _ab/lane_count
#include <hip/hip_runtime.h>
#include <cstdio>
#pragma clang diagnostic ignored "-Wunused-result"

template <int KIND>
__global__ void __launch_bounds__(256) k(double* out, int kact, double s) {
  const int lane = threadIdx.x & 63;
  double a = out[threadIdx.x] + s;
  float f = (float)a;
  double b2 = a + 1, c2 = a + 2, d2 = a + 3, e2 = a + 4, f2 = a + 5, g2 = a + 6, h2 = a + 7;
  if (lane < kact) {
#pragma unroll 1
    for (int r = 0; r < 256; ++r) {
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        if constexpr (KIND == 0) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(a) : "v"(s));
        if constexpr (KIND == 1) asm volatile("v_rcp_f64 %0, %0" : "+v"(a));
        if constexpr (KIND == 2) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(f) : "v"((float)s));
        if constexpr (KIND == 4) {  // 8 independent fp64 FMA chains (issue-bound, not latency-bound)
          asm volatile("v_fma_f64 %0, %0, %8, %8\n\tv_fma_f64 %1, %1, %8, %8\n\tv_fma_f64 %2, %2, %8, %8\n\tv_fma_f64 %3, %3, %8, %8\n\t"
                       "v_fma_f64 %4, %4, %8, %8\n\tv_fma_f64 %5, %5, %8, %8\n\tv_fma_f64 %6, %6, %8, %8\n\tv_fma_f64 %7, %7, %8, %8"
                       : "+v"(a), "+v"(b2), "+v"(c2), "+v"(d2), "+v"(e2), "+v"(f2), "+v"(g2), "+v"(h2) : "v"(s));
        }
        if constexpr (KIND == 3) {  // compare + select (VOPC to vcc, then cndmask)
          asm volatile("v_cmp_lt_f32 vcc, %0, %1\n\tv_cndmask_b32 %0, %1, %0, vcc" : "+v"(f) : "v"((float)s) : "vcc");
        }
      }
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = a + f + b2 + c2 + d2 + e2 + f2 + g2 + h2;
}

template <int KIND>
void run(const char* name) {
  double* o;
  hipMalloc(&o, 256 * 256 * sizeof(double));
  hipMemset(o, 0, 256 * 256 * sizeof(double));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int kact : {64, 1, 4, 8, 9, 16, 17, 32, 33, 48, 64}) {
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k<KIND>, dim3(256), dim3(256), 0, 0, o, kact, 1e-3);
    hipEventRecord(e0);
    for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(k<KIND>, dim3(256), dim3(256), 0, 0, o, kact, 1e-3);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    printf("%-16s k=%2d active lanes: %8.2f us per launch (4096 instr per chain)\n", name, kact, ms * 1e3 / 20);
  }
  hipFree(o);
}

int main() {
  run<4>("8 indep fma f64");
  run<0>("fma f64");
  run<1>("rcp f64");
  run<2>("fma f32");
  run<3>("cmp+cndmask f64");
  return 0;
}
