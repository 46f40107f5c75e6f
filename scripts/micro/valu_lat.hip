// Microbenchmark (not shipped): per-wave cycles of dependent / independent
// fp64 VALU chains on gfx950, one or two waves per SIMD.
// Build: hipcc -O3 --offload-arch=gfx950 scripts/micro/valu_lat.hip -o _ab/valu_lat
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ unsigned long long clk() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

template <int KIND>
__global__ void __launch_bounds__(64) k(double* out, unsigned long long* cyc, double s) {
  double a = out[threadIdx.x] + s, b = a + 1.0, c = a + 2.0, d = a + 3.0;
  const unsigned long long t0 = clk();
#pragma unroll 1
  for (int r = 0; r < 64; ++r) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      if (KIND == 0) {  // dependent fma f64
        asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(a) : "v"(s));
      } else if (KIND == 1) {  // 4 independent fma f64 chains
        asm volatile("v_fma_f64 %0, %0, %4, %4\n\tv_fma_f64 %1, %1, %4, %4\n\tv_fma_f64 %2, %2, %4, %4\n\tv_fma_f64 %3, %3, %4, %4"
                     : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(s));
      } else if (KIND == 2) {  // dependent add f64
        asm volatile("v_add_f64 %0, %0, %1" : "+v"(a) : "v"(s));
      } else if (KIND == 3) {  // dependent fma f32 (on the low word)
        float x = __builtin_bit_cast(float2, a).x;
        asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(x) : "v"((float)s));
        a = __builtin_bit_cast(double, make_float2(x, 0.f));
      } else if (KIND == 4) {  // 2 independent fma f64 chains
        asm volatile("v_fma_f64 %0, %0, %2, %2\n\tv_fma_f64 %1, %1, %2, %2" : "+v"(a), "+v"(b) : "v"(s));
      } else if (KIND == 5) {  // dependent rcp f64
        asm volatile("v_rcp_f64 %0, %0" : "+v"(a));
      } else if (KIND == 6) {  // dependent max f64
        asm volatile("v_max_f64 %0, %0, %1" : "+v"(a) : "v"(s));
      }
    }
  }
  const unsigned long long t1 = clk();
  out[threadIdx.x] = a + b + c + d;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int KIND>
void run(const char* name, int instr_per_iter, int blocks) {
  double* o; unsigned long long* c;
  hipMalloc(&o, 64 * sizeof(double)); hipMemset(o, 0, 64 * sizeof(double));
  hipMalloc(&c, blocks * 8);
  hipLaunchKernelGGL(k<KIND>, dim3(blocks), dim3(64), 0, 0, o, c, 1e-3);
  hipLaunchKernelGGL(k<KIND>, dim3(blocks), dim3(64), 0, 0, o, c, 1e-3);
  hipDeviceSynchronize();
  unsigned long long h[4096];
  hipMemcpy(h, c, blocks * 8, hipMemcpyDeviceToHost);
  double m = 0; for (int i = 0; i < blocks; ++i) m += h[i]; m /= blocks;
  // s_memtime counts at a fixed 100 MHz reference on gfx9? report raw and per-instr
  printf("%-28s waves %5d: %.1f memtime ticks per wave, %.4f ticks/instr\n", name, blocks, m, m / (64.0 * 16 * instr_per_iter));
  hipFree(o); hipFree(c);
}

int main() {
  for (int blocks : {1024, 2048}) {
    run<0>("dep fma f64", 1, blocks);
    run<1>("4 indep fma f64", 4, blocks);
    run<4>("2 indep fma f64", 2, blocks);
    run<2>("dep add f64", 1, blocks);
    run<3>("dep fma f32", 1, blocks);
    run<5>("dep rcp f64", 1, blocks);
    run<6>("dep max f64", 1, blocks);
  }
  // wall clock for the dep chain at 1024 waves -> cycles/instr at the real clock
  double* o; unsigned long long* c; hipMalloc(&o, 512); hipMalloc(&c, 4096 * 8);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int blocks : {1024, 2048}) {
    hipEventRecord(e0);
    for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(64), 0, 0, o, c, 1e-3);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    printf("dep fma f64 chain of 1024 instr, %d waves: %.2f us per launch\n", blocks, ms * 1e3 / 20);
    hipEventRecord(e0);
    for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(64), 0, 0, o, c, 1e-3);
    hipEventRecord(e1); hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    printf("4 indep fma f64 (4096 instr), %d waves: %.2f us per launch\n", blocks, ms * 1e3 / 20);
  }
  return 0;
}
