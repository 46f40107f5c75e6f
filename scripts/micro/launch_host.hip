// Microbenchmark (not shipped): the HOST cost of one kernel launch on ROCm,
// i.e. what bounds a Python env.step / GCDataset.sample(1024) call besides
// the Python itself.  A spin kernel holds the queue so that no launch waits
// on the device; the host time of `reps` launches / reps is printed for:
//   ggl12   hipLaunchKernelGGL, 12 pointer/int arguments (ogbx_maze_step's shape)
//   ggl_big hipLaunchKernelGGL with a 1,376-byte by-value struct (the sampler's
//           column table) + 6 scalars
//   mod12   hipModuleLaunchKernel of the same 12-argument kernel through a cached
//           hipFunction_t and one prepacked kernarg buffer (HIP_LAUNCH_PARAM_*)
//   mod_big the big-struct kernel the same way
//   setdev  hipSetDevice(0) alone; getlast hipGetLastError alone
// Build: hipcc -O3 --offload-arch=gfx950 scripts/micro/launch_host.hip -o _ab/launch_host
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>

__global__ void spin_kernel(long long ticks) {
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

__global__ void __launch_bounds__(256) k12(const void* a, const void* b, int n, void* c, void* d, void* e, void* f,
                                           void* g, void* h, int flag, unsigned k0, unsigned k1) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && flag == 12345) *(int*)c = n + k0 + k1;
}

struct Big {
  unsigned char b[1376];
};

__global__ void __launch_bounds__(256) kbig(Big cols, int ncols, long long total, int tile, unsigned k0, unsigned k1,
                                            void* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && ncols == 12345) *(int*)out = cols.b[total & 1023] + tile + k0 + k1;
}

#define CK(x)                                                         \
  do {                                                                \
    hipError_t _e = (x);                                              \
    if (_e != hipSuccess) {                                           \
      std::printf("%s: %s\n", #x, hipGetErrorString(_e));             \
      return 1;                                                       \
    }                                                                 \
  } while (0)

template <class F>
static double host_us(hipStream_t s, int reps, F&& f) {
  hipDeviceSynchronize();
  hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, s, (long long)(reps * 40e-6 * 1e8));  // 100 MHz
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < reps; ++i) f(i);
  const auto t1 = std::chrono::steady_clock::now();
  hipDeviceSynchronize();
  return std::chrono::duration<double, std::micro>(t1 - t0).count() / reps;
}

int main() {
  CK(hipSetDevice(0));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  void* buf;
  CK(hipMalloc(&buf, 1 << 20));
  Big big;
  std::memset(&big, 0, sizeof(big));
  hipFunction_t f12, fbig;
  CK(hipGetFuncBySymbol(&f12, reinterpret_cast<const void*>(k12)));
  CK(hipGetFuncBySymbol(&fbig, reinterpret_cast<const void*>(kbig)));
  const int reps = 2000;
  for (int round = 0; round < 3; ++round) {
    const double a = host_us(s, reps, [&](int i) {
      hipLaunchKernelGGL(k12, dim3(256), dim3(256), 0, s, buf, buf, 65536, buf, buf, buf, buf, buf, buf, 1, (unsigned)i,
                         2u);
    });
    const double b = host_us(s, reps, [&](int i) {
      hipLaunchKernelGGL(kbig, dim3(1024), dim3(256), 0, s, big, 9, (long long)1024, 1, (unsigned)i, 2u, buf);
    });
    struct __attribute__((packed, aligned(8))) A12 {
      const void *a, *b;
      int n, pad;
      void *c, *d, *e, *f, *g, *h;
      int flag;
      unsigned k0, k1;
    } a12{buf, buf, 65536, 0, buf, buf, buf, buf, buf, buf, 1, 0u, 2u};
    size_t sz12 = sizeof(a12);
    const double c = host_us(s, reps, [&](int i) {
      a12.k0 = (unsigned)i;
      void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &a12, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz12, HIP_LAUNCH_PARAM_END};
      hipModuleLaunchKernel(f12, 256, 1, 1, 256, 1, 1, 0, s, nullptr, cfg);
    });
    struct __attribute__((aligned(8))) ABig {
      Big cols;
      int ncols;
      int pad;
      long long total;
      int tile;
      unsigned k0, k1;
      int pad2;
      void* out;
    } ab{big, 9, 0, 1024, 1, 0u, 2u, 0, buf};
    size_t szb = sizeof(ab);
    const double d = host_us(s, reps, [&](int i) {
      ab.k0 = (unsigned)i;
      void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &ab, HIP_LAUNCH_PARAM_BUFFER_SIZE, &szb, HIP_LAUNCH_PARAM_END};
      hipModuleLaunchKernel(fbig, 1024, 1, 1, 256, 1, 1, 0, s, nullptr, cfg);
    });
    const double e = host_us(s, reps, [&](int) { (void)hipSetDevice(0); });
    const double g = host_us(s, reps, [&](int) { (void)hipGetLastError(); });
    std::printf("round %d: ggl12 %.2f us  ggl_big %.2f us  mod12 %.2f us  mod_big %.2f us  setdev %.3f us  getlast %.3f us\n",
                round, a, b, c, d, e, g);
  }
  CK(hipDeviceSynchronize());
  CK(hipGetLastError());
  return 0;
}
