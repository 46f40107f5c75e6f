// Microbenchmark (not shipped): latency of the contact path's pieces as
// dependent chains, one lane per state, states sampled near walls of
// pointmaze-large.  Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off
//   -I ogbench_amd/csrc scripts/micro/phys_micro.hip -o build/phys_micro
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>
#include "point_physics.h"

using namespace ogbx;

__global__ void k_collide(const PointModel* pmp, const uint16_t* nb_g, int H, int W, const double* xy, int n, int reps,
                          double* out) {
  const PointModel pm = *pmp;
  __shared__ uint16_t nb[256];
  for (int i = threadIdx.x; i < H * W; i += blockDim.x) nb[i] = nb_g[i];
  __syncthreads();
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double x = xy[2 * i], y = xy[2 * i + 1], acc = 0.0;
  for (int r = 0; r < reps; ++r) {
    Contacts c;
    collide_walls(pm, nb, H, W, x, y, c);
    const double s = c.s0.kp + c.s1.kp + c.s2.kp + c.s0.w * 1e-30 + c.s2.nx;
    acc += s;
    x += s * 1e-300;  // dependent chain
  }
  out[i] = acc + x;
}

__global__ void k_solve(const PointModel* pmp, const uint16_t* nb_g, int H, int W, const double* xy, int n, int reps,
                        double* out) {
  const PointModel pm = *pmp;
  __shared__ uint16_t nb[256];
  for (int i = threadIdx.x; i < H * W; i += blockDim.x) nb[i] = nb_g[i];
  __syncthreads();
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double x = xy[2 * i], y = xy[2 * i + 1];
  Contacts c;
  collide_walls(pm, nb, H, W, x, y, c);
  double vx = 0.3, vy = -0.2, wx = 0.0, wy = 0.0, ax, ay;
  for (int r = 0; r < reps; ++r) {
    solve_acc(pm, c, vx, vy, &ax, &ay, &wx, &wy);
    vx = vx + ax * 1e-6;
    vy = vy + ay * 1e-6;
  }
  out[i] = vx + vy;
}

__global__ void k_step(const PointModel* pmp, const uint16_t* nb_g, int H, int W, const double* xy, int n, int reps,
                       double* out) {
  const PointModel pm = *pmp;
  __shared__ uint16_t nb[256];
  for (int i = threadIdx.x; i < H * W; i += blockDim.x) nb[i] = nb_g[i];
  __syncthreads();
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double x = xy[2 * i], y = xy[2 * i + 1];
  for (int r = 0; r < reps; ++r) point_step(pm, nb, H, W, &x, &y);
  out[i] = x + y;
}

int main(int argc, char** argv) {
  // pointmaze-large map (maze.py:112-123), 1 = wall
  const char* m = "111111111111100001000001101101010101100000010001101111011101"
                  "100101000001110101010111100100010001111111111111";
  const int H = 9, W = 12;
  std::vector<uint16_t> nb(H * W);
  for (int i = 0; i < H; ++i)
    for (int j = 0; j < W; ++j) {
      uint16_t v = 0;
      for (int di = -1; di <= 1; ++di)
        for (int dj = -1; dj <= 1; ++dj) {
          int ii = i + di, jj = j + dj;
          bool wall = ii < 0 || ii >= H || jj < 0 || jj >= W || m[ii * W + jj] == '1';
          v |= (uint16_t)wall << (4 + 3 * di + dj);
        }
      nb[i * W + j] = v;
    }
  // PointModel as the library builds it: read from a file written by the host lib? keep in sync by hand:
  const PointModel pm = make_point_model(4.0, 4.0);
  const int n = argc > 1 ? atoi(argv[1]) : 5632;
  std::vector<double> xy(2 * n);
  srand(1);
  int k = 0;
  while (k < n) {  // states within the contact band of some wall
    int i = rand() % H, j = rand() % W;
    if (m[i * W + j] == '1') continue;
    double cx = j * 4.0 - 4.0, cy = i * 4.0 - 4.0;
    double ox = (rand() / (double)RAND_MAX) * 3.9 - 1.95, oy = (rand() / (double)RAND_MAX) * 3.9 - 1.95;
    if (std::fabs(ox) < 1.25 && std::fabs(oy) < 1.25) continue;
    xy[2 * k] = cx + ox;
    xy[2 * k + 1] = cy + oy;
    ++k;
  }
  PointModel* dpm; uint16_t* dnb; double *dxy, *dout;
  hipMalloc(&dpm, sizeof(pm)); hipMalloc(&dnb, nb.size() * 2); hipMalloc(&dxy, xy.size() * 8); hipMalloc(&dout, n * 8);
  hipMemcpy(dpm, &pm, sizeof(pm), hipMemcpyHostToDevice);
  hipMemcpy(dnb, nb.data(), nb.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(dxy, xy.data(), xy.size() * 8, hipMemcpyHostToDevice);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  const int reps = 200;
  auto run = [&](const char* name, auto kern, int rr) {
    hipLaunchKernelGGL(kern, dim3((n + 255) / 256), dim3(256), 0, 0, dpm, dnb, H, W, dxy, n, rr, dout);
    hipDeviceSynchronize();
    hipEventRecord(a);
    hipLaunchKernelGGL(kern, dim3((n + 255) / 256), dim3(256), 0, 0, dpm, dnb, H, W, dxy, n, rr, dout);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    printf("%-8s %8.3f ms  %8.1f ns/iter  (%d reps, n=%d)\n", name, ms, ms * 1e6 / rr, rr, n);
  };
  run("collide", k_collide, reps);
  run("solve", k_solve, reps);
  run("step", k_step, 10);
  return 0;
}
