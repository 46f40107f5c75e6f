// Microbenchmark (not shipped): relative error of v_rcp_f64 alone and with one
// or two Newton-Raphson refinements against the IEEE quotient 1.0 / d.
// Build: hipcc -O3 --offload-arch=gfx950 scripts/micro/rcp_err.hip -o _ab/rcp_err
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#pragma clang diagnostic ignored "-Wunused-result"

__global__ void k(const double* d, double* e0, double* e1, double* e2, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double x = d[i], q = 1.0 / x;
  double r = __builtin_amdgcn_rcp(x);
  e0[i] = fabs(r - q) / q;
  r = fma(r, fma(-x, r, 1.0), r);
  e1[i] = fabs(r - q) / q;
  r = fma(r, fma(-x, r, 1.0), r);
  e2[i] = fabs(r - q) / q;
}

int main() {
  const int n = 1 << 22;
  double* h = new double[n];
  unsigned long long s = 88172645463325252ull;
  for (int i = 0; i < n; ++i) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    h[i] = std::ldexp(1.0 + (s >> 11) * 0x1.0p-53, (int)(s % 40) - 20);  // [2^-20, 2^20)
  }
  double *d, *e[3];
  hipMalloc(&d, n * 8);
  for (auto& p : e) hipMalloc(&p, n * 8);
  hipMemcpy(d, h, n * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, d, e[0], e[1], e[2], n);
  const char* names[3] = {"v_rcp_f64", "+1 NR", "+2 NR"};
  for (int j = 0; j < 3; ++j) {
    hipMemcpy(h, e[j], n * 8, hipMemcpyDeviceToHost);
    double m = 0;
    for (int i = 0; i < n; ++i) m = h[i] > m ? h[i] : m;
    printf("%-10s max relative error %.3e (%.2f ulp of 2^-52)\n", names[j], m, m / 0x1.0p-52);
  }
  return 0;
}
