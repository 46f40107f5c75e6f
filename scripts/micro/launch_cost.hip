// Microbenchmark (not shipped): the DEVICE-side cost of a short launch on
// gfx950, i.e. what a kernel boundary costs when the host is not the
// bottleneck.  Every measurement queues a spin kernel first (it holds the
// queue for longer than the host needs to enqueue all launches behind it, as
// bench.py's _per_launch_ms does), then `reps` launches between one event
// pair: span / reps = the device time per launch including the dispatch gap
// to the next one.  The host-paced rate (no spin kernel ahead: what rounds 2-4
// quoted as the "launch floor") is printed beside it.
//
// Grids: the maze step (N = 65,536: 256 x 256 threads; the 8-GPU share
// 8,192: 32 x 256), the GC / HGC sampler at B = 1,024 (1,024 x 256), the
// powder light kernel (4,096 x 256) -- empty kernels, and a few bodies of
// the shapes the real kernels have (16-B load + store per lane, 256 VGPRs,
// LDS + barrier).  Run under `rocprofv3 --kernel-trace --stats` for the
// per-dispatch durations (scripts/gpu_r05_floor.sh).
// Build: hipcc -O3 --offload-arch=gfx950 scripts/micro/launch_cost.hip -o _ab/launch_cost
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

__global__ void spin_kernel(long long ticks) {
  // wall_clock64: the 100 MHz constant clock (s_memrealtime, a scalar read)
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

__global__ void __launch_bounds__(256) k_empty(double2* q, int n) {}

__global__ void __launch_bounds__(256) k_copy(const double2* __restrict__ a, double2* __restrict__ q, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) q[i] = make_double2(q[i].x + a[i].x, q[i].y + a[i].y);
}

__global__ void __launch_bounds__(256) k_bigvgpr(const double2* __restrict__ a, double2* __restrict__ q, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  asm volatile("" ::: "v250", "v251", "v252", "v253", "v254", "v255", "a0", "a1", "a2", "a3", "a20", "a21");
  if (i < n) q[i] = make_double2(q[i].x + a[i].x, q[i].y + a[i].y);
}

__global__ void __launch_bounds__(256) k_lds(const double2* __restrict__ a, double2* __restrict__ q, int n) {
  __shared__ double2 s[256];
  const int i = blockIdx.x * 256 + threadIdx.x;
  s[threadIdx.x] = i < n ? a[i] : make_double2(0, 0);
  __syncthreads();
  if (i < n) q[i] = s[255 - threadIdx.x];
}

template <typename F>
void measure(const char* name, int blocks, F launch) {
  hipEvent_t s, e;
  hipEventCreate(&s);
  hipEventCreate(&e);
  for (int r = 0; r < 50; ++r) launch();
  hipDeviceSynchronize();
  const int reps = 2000;
  // device-paced: a 40 ms spin holds the queue while the host enqueues
  hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, 0, 4000000LL);
  hipEventRecord(s);
  for (int r = 0; r < reps; ++r) launch();
  hipEventRecord(e);
  hipEventSynchronize(e);
  float dev_ms;
  hipEventElapsedTime(&dev_ms, s, e);
  // host-paced: no spin ahead (the rounds 2-4 measurement)
  hipDeviceSynchronize();
  hipEventRecord(s);
  for (int r = 0; r < reps; ++r) launch();
  hipEventRecord(e);
  hipEventSynchronize(e);
  float host_ms;
  hipEventElapsedTime(&host_ms, s, e);
  printf("%-14s blocks %5d  device-paced %6.2f us/launch   host-paced %6.2f us/launch\n", name, blocks,
         dev_ms * 1e3 / reps, host_ms * 1e3 / reps);
  hipEventDestroy(s);
  hipEventDestroy(e);
}

int main() {
  const int n = 1 << 20;
  double2 *q, *a;
  hipMalloc(&q, n * sizeof(double2));
  hipMalloc(&a, n * sizeof(double2));
  hipMemset(q, 0, n * sizeof(double2));
  hipMemset(a, 0, n * sizeof(double2));
  const dim3 b(256);
  struct Grid {
    const char* tag;
    int blocks;
  } grids[] = {{"maze65536", 256}, {"maze8192", 32}, {"gc1024", 1024}, {"pwlight4096", 4096}};
  for (const Grid& g : grids) {
    const int m = g.blocks * 256;
    char nm[64];
    snprintf(nm, sizeof nm, "empty/%s", g.tag);
    measure(nm, g.blocks, [&] { hipLaunchKernelGGL(k_empty, dim3(g.blocks), b, 0, 0, q, m); });
    snprintf(nm, sizeof nm, "copy/%s", g.tag);
    measure(nm, g.blocks, [&] { hipLaunchKernelGGL(k_copy, dim3(g.blocks), b, 0, 0, a, q, m); });
  }
  measure("bigvgpr/maze65536", 256, [&] { hipLaunchKernelGGL(k_bigvgpr, dim3(256), b, 0, 0, a, q, 65536); });
  measure("lds/gc1024", 1024, [&] { hipLaunchKernelGGL(k_lds, dim3(1024), b, 0, 0, a, q, 1024 * 256); });
  return 0;
}
