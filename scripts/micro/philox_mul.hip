// Microbenchmark (not shipped): Philox4x32-10 throughput on gfx950 with the
// round's two 32x32->64 products as v_mul_hi_u32 + v_mul_lo_u32 pairs (what
// LLVM emits for the plain C++ products) vs one v_mad_u64_u32 each (what
// common.h's philox4x32_10_wide issues).  Measured: 550 vs 583 G calls/s.
// Build: hipcc -O3 --offload-arch=gfx950 scripts/micro/philox_mul.hip -o _abx/philox_mul
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "../../ogbench_amd/csrc/common.h"

__device__ __forceinline__ uint64_t mad64(uint32_t a, uint32_t b) {
  uint64_t r, c;
  asm volatile("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(r), "=s"(c) : "v"(a), "v"(b));
  return r;
}

__device__ __forceinline__ ogbx::u32x4 philox_pair(ogbx::u32x4 c, uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(M0, c.x), lo0 = M0 * c.x, hi1 = __umulhi(M1, c.z), lo1 = M1 * c.z;
    ogbx::u32x4 n;
    n.x = hi1 ^ c.y ^ k0;
    n.y = lo1;
    n.z = hi0 ^ c.w ^ k1;
    n.w = lo0;
    c = n;
    k0 += W0;
    k1 += W1;
  }
  return c;
}

__device__ __forceinline__ ogbx::u32x4 philox_mad(ogbx::u32x4 c, uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = mad64(M0, c.x), p1 = mad64(M1, c.z);
    ogbx::u32x4 n;
    n.x = (uint32_t)(p1 >> 32) ^ c.y ^ k0;
    n.y = (uint32_t)p1;
    n.z = (uint32_t)(p0 >> 32) ^ c.w ^ k1;
    n.w = (uint32_t)p0;
    c = n;
    k0 += W0;
    k1 += W1;
  }
  return c;
}

template <int KIND>
__global__ void __launch_bounds__(256) k(uint32_t* out, int calls, uint32_t k0, uint32_t k1) {
  uint32_t acc = 0;
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
#pragma unroll 1
  for (int i = 0; i < calls; i += 2) {
    ogbx::u32x4 a, b;
    if (KIND == 0) {
      a = philox_pair({t, (uint32_t)i, 7u, 0u}, k0, k1);
      b = philox_pair({t, (uint32_t)i + 1, 7u, 0u}, k0, k1);
    } else {
      a = philox_mad({t, (uint32_t)i, 7u, 0u}, k0, k1);
      b = philox_mad({t, (uint32_t)i + 1, 7u, 0u}, k0, k1);
    }
    acc ^= a.x + a.y * 3u + a.z * 5u + a.w * 7u;
    acc ^= b.x + b.y * 3u + b.z * 5u + b.w * 7u;
  }
  out[t] = acc;
}

template <int KIND>
float run(uint32_t* o, int blocks, int calls, uint32_t* h, int n) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(k<KIND>, dim3(blocks), dim3(256), 0, 0, o, calls, 0x1234u, 0x5678u);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k<KIND>, dim3(blocks), dim3(256), 0, 0, o, calls, 0x1234u, 0x5678u);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  hipMemcpy(h, o, n * 4, hipMemcpyDeviceToHost);
  return ms / 5;
}

int main() {
  const int blocks = 4096, calls = 256, n = blocks * 256;
  uint32_t* o; hipMalloc(&o, n * 4);
  static uint32_t ha[4096 * 256], hb[4096 * 256];
  const float ta = run<0>(o, blocks, calls, ha, n);
  const float tb = run<1>(o, blocks, calls, hb, n);
  int diff = 0;
  for (int i = 0; i < n; ++i) diff += ha[i] != hb[i];
  const double g = (double)n * calls / 1e9;
  printf("mul_hi+mul_lo : %.3f ms  %.2f G Philox calls/s\n", ta, g / (ta * 1e-3));
  printf("v_mad_u64_u32 : %.3f ms  %.2f G Philox calls/s\n", tb, g / (tb * 1e-3));
  printf("outputs differ in %d of %d lanes\n", diff, n);
  return diff != 0;
}
