// Microbenchmark (not shipped): what a short launch of 65,536 lanes costs on
// gfx950 -- empty kernel, a 16-B load + store per lane, the same with a
// dependent read of a parameter block, with an LDS staging barrier, with a
// large VGPR allocation, and with byte flag stores.  Back-to-back launches
// (total / count) and event-pair medians.
// Build: hipcc -O3 --offload-arch=gfx950 scripts/micro/launch_cost.hip -o _ab/launch_cost
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

struct Params {
  int H, W;
  unsigned short nb[256];
};

__global__ void __launch_bounds__(256) k_empty(double2* q, int n) {}

__global__ void __launch_bounds__(256) k_copy(const double2* __restrict__ a, double2* __restrict__ q, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) q[i] = make_double2(q[i].x + a[i].x, q[i].y + a[i].y);
}

__global__ void __launch_bounds__(256) k_param(const Params* __restrict__ P, const double2* __restrict__ a,
                                               double2* __restrict__ q, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) {
    const double2 v = q[i];
    const int c = ((int)v.x & 7) * P->W + ((int)v.y & 7);
    q[i] = make_double2(v.x + a[i].x + P->nb[c & 255], v.y + a[i].y);
  }
}

__global__ void __launch_bounds__(256) k_lds(const Params* __restrict__ P, const double2* __restrict__ a,
                                             double2* __restrict__ q, int n) {
  __shared__ unsigned short nb[256];
  for (int t = threadIdx.x; t < P->H * P->W; t += 256) nb[t] = P->nb[t];
  __syncthreads();
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) {
    const double2 v = q[i];
    const int c = ((int)v.x & 7) * 8 + ((int)v.y & 7);
    q[i] = make_double2(v.x + a[i].x + nb[c], v.y + a[i].y);
  }
}

__global__ void __launch_bounds__(256) k_bigvgpr(const double2* __restrict__ a, double2* __restrict__ q, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  asm volatile("" ::: "v250", "v251", "v252", "v253", "v254", "v255", "a0", "a1", "a2", "a3", "a20", "a21");
  if (i < n) q[i] = make_double2(q[i].x + a[i].x, q[i].y + a[i].y);
}

__global__ void __launch_bounds__(256) k_flags(const double2* __restrict__ a, double2* __restrict__ q,
                                               float* rew, unsigned char* t0, unsigned char* t1,
                                               unsigned char* t2, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) {
    const double2 v = make_double2(q[i].x + a[i].x, q[i].y + a[i].y);
    q[i] = v;
    rew[i] = v.x > 0.0 ? 1.f : 0.f;
    t0[i] = v.x > 1.0;
    t1[i] = v.y > 1.0;
    t2[i] = v.y > 2.0;
  }
}

template <typename F>
void measure(const char* name, F launch) {
  hipEvent_t s, e;
  hipEventCreate(&s);
  hipEventCreate(&e);
  for (int r = 0; r < 50; ++r) launch();
  hipDeviceSynchronize();
  const int reps = 2000;
  hipEventRecord(s);
  for (int r = 0; r < reps; ++r) launch();
  hipEventRecord(e);
  hipEventSynchronize(e);
  float ms;
  hipEventElapsedTime(&ms, s, e);
  std::vector<hipEvent_t> ev(2 * 400);
  for (auto& x : ev) hipEventCreate(&x);
  for (int r = 0; r < 400; ++r) {
    hipEventRecord(ev[2 * r]);
    launch();
    hipEventRecord(ev[2 * r + 1]);
  }
  hipDeviceSynchronize();
  std::vector<float> t(400);
  for (int r = 0; r < 400; ++r) hipEventElapsedTime(&t[r], ev[2 * r], ev[2 * r + 1]);
  std::sort(t.begin(), t.end());
  printf("%-10s back-to-back %7.2f us/launch   event median %7.2f us\n", name, ms * 1e3 / reps, t[200] * 1e3);
  for (auto& x : ev) hipEventDestroy(x);
}

int main() {
  const int n = 65536;
  double2 *q, *a;
  float* rew;
  unsigned char* f;
  Params* P;
  hipMalloc(&q, n * sizeof(double2));
  hipMalloc(&a, n * sizeof(double2));
  hipMalloc(&rew, n * 4);
  hipMalloc(&f, 3 * n);
  hipMalloc(&P, sizeof(Params));
  hipMemset(q, 0, n * sizeof(double2));
  hipMemset(a, 0, n * sizeof(double2));
  Params hp{};
  hp.H = 8;
  hp.W = 8;
  hipMemcpy(P, &hp, sizeof(hp), hipMemcpyHostToDevice);
  const dim3 g(n / 256), b(256);
  measure("empty", [&] { hipLaunchKernelGGL(k_empty, g, b, 0, 0, q, n); });
  measure("copy", [&] { hipLaunchKernelGGL(k_copy, g, b, 0, 0, a, q, n); });
  measure("param", [&] { hipLaunchKernelGGL(k_param, g, b, 0, 0, P, a, q, n); });
  measure("lds", [&] { hipLaunchKernelGGL(k_lds, g, b, 0, 0, P, a, q, n); });
  measure("bigvgpr", [&] { hipLaunchKernelGGL(k_bigvgpr, g, b, 0, 0, a, q, n); });
  measure("flags", [&] { hipLaunchKernelGGL(k_flags, g, b, 0, 0, a, q, rew, f, f + n, f + 2 * n, n); });
  const dim3 g8(8192 / 256);
  measure("copy8k", [&] { hipLaunchKernelGGL(k_copy, g8, b, 0, 0, a, q, 8192); });
  measure("lds8k", [&] { hipLaunchKernelGGL(k_lds, g8, b, 0, 0, P, a, q, 8192); });
  return 0;
}
