// loader.hip -- device side of the dataset loader and the single-task /
// oracle-rep relabel pass.
//
// Reference (hliuson/ogbench):
//   load_dataset (compact / regular conversion)  ogbench/utils.py:14-96
//   relabel_dataset (maze branch)                ogbench/relabel_utils.py:4-31,111-113
//   add_oracle_reps (maze branch)                ogbench/relabel_utils.py:116-133,166
//
// The raw .npz columns are copied to HBM once; these kernels do the per-row
// work there: the compact terminals/valids rewrite, the regular-mode row
// compaction (a row gather by hipCUB-selected indices), and one pass over qpos
// producing rewards, masks and oracle_reps together.
#include <algorithm>

#include "common.h"

namespace ogbx {

// valids = 1 - t ; shifted = t[i+1] (1 past the end) ; terminals = min(t + shifted, 1)
__global__ void compact_terminals_kernel(const float* __restrict__ t, int64_t n, float* __restrict__ terms,
                                         float* __restrict__ valids, float* __restrict__ shifted) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float ti = t[i];
    const float nx = i + 1 < n ? t[i + 1] : 1.0f;
    if (valids) valids[i] = 1.0f - ti;
    if (shifted) shifted[i] = nx;
    if (terms) {
      const float s = ti + nx;
      terms[i] = s < 1.0f ? s : 1.0f;
    }
  }
}

// dst[k] = src[idx[k]] for rows of row_bytes (widest aligned unit per lane).
template <typename T>
__global__ void gather_rows_kernel(const T* __restrict__ src, int64_t units, const int64_t* __restrict__ idx,
                                   int64_t n, T* __restrict__ dst) {
  const int64_t total = units * n;
  for (int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; f < total;
       f += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = f / units, k = f - r * units;
    dst[f] = src[idx[r] * units + k];
  }
}

// One pass over qpos rows: success = ||qpos[:, 0:2] - goal|| <= tol in
// float64 (qpos upcast, plain sqrt(dx*dx + dy*dy) as np.linalg.norm(axis=-1)
// computes it for two columns); rewards = success - 1, masks = 1 - success
// (float32); oracle_reps = qpos[:, 0:2] as float32.
template <typename Q>
__global__ void relabel_maze_kernel(const Q* __restrict__ qpos, int64_t stride, int64_t n, double gx, double gy,
                                    double tol, float* __restrict__ rewards, float* __restrict__ masks,
                                    float* __restrict__ reps) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const Q qx = qpos[i * stride], qy = qpos[i * stride + 1];
    if (rewards || masks) {
      const double dx = (double)qx - gx, dy = (double)qy - gy;
      const double d = sqrt(dx * dx + dy * dy);
      const float s = d <= tol ? 1.0f : 0.0f;
      if (rewards) rewards[i] = s - 1.0f;
      if (masks) masks[i] = 1.0f - s;
    }
    if (reps) {
      reps[2 * i] = (float)qx;
      reps[2 * i + 1] = (float)qy;
    }
  }
}

inline uint32_t grid_for(int64_t n) {
  const int64_t b = (n + 255) / 256;
  return (uint32_t)std::max<int64_t>(1, std::min<int64_t>(b, 1 << 20));
}

}  // namespace ogbx

using namespace ogbx;

extern "C" {

ogbx_status ogbx_compact_terminals(const float* terminals_in, int64_t n, float* terminals_out,
                                   float* valids_out, float* shifted_out, void* stream) {
  OGBX_CHECK(terminals_in && n >= 0, OGBX_EINVAL, "ogbx_compact_terminals: bad argument");
  if (n == 0) return OGBX_OK;
  hipLaunchKernelGGL(compact_terminals_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream,
                     terminals_in, n, terminals_out, valids_out, shifted_out);
  OGBX_LAUNCHED("compact_terminals_kernel");
  return OGBX_OK;
}

ogbx_status ogbx_gather_rows(const void* src, int64_t row_bytes, const int64_t* idx, int64_t n, void* dst,
                             void* stream) {
  OGBX_CHECK(src && idx && dst && row_bytes > 0 && n >= 0, OGBX_EINVAL, "ogbx_gather_rows: bad argument");
  if (n == 0) return OGBX_OK;
  const uintptr_t a = (uintptr_t)src | (uintptr_t)dst;
  hipStream_t s = (hipStream_t)stream;
  auto launch = [&](auto tag) {
    using T = decltype(tag);
    const int64_t units = row_bytes / (int64_t)sizeof(T);
    const int64_t total = units * n;
    hipLaunchKernelGGL(gather_rows_kernel<T>, dim3((uint32_t)std::min<int64_t>((total + 255) / 256, 65536)),
                       dim3(256), 0, s, (const T*)src, units, idx, n, (T*)dst);
  };
  if (row_bytes % 16 == 0 && a % 16 == 0)
    launch(uint4{});
  else if (row_bytes % 8 == 0 && a % 8 == 0)
    launch(uint2{});
  else if (row_bytes % 4 == 0 && a % 4 == 0)
    launch(uint32_t{});
  else
    launch(uint8_t{});
  OGBX_LAUNCHED("gather_rows_kernel");
  return OGBX_OK;
}

ogbx_status ogbx_relabel_maze(const void* qpos, int32_t qpos_is_f64, int64_t num_rows, int64_t qpos_stride,
                              double goal_x, double goal_y, double goal_tol, float* rewards, float* masks,
                              float* oracle_reps, void* stream) {
  OGBX_CHECK(qpos && num_rows >= 0 && qpos_stride >= 2, OGBX_EINVAL, "ogbx_relabel_maze: bad argument");
  if (num_rows == 0) return OGBX_OK;
  hipStream_t s = (hipStream_t)stream;
  if (qpos_is_f64)
    hipLaunchKernelGGL(relabel_maze_kernel<double>, dim3(grid_for(num_rows)), dim3(256), 0, s,
                       (const double*)qpos, qpos_stride, num_rows, goal_x, goal_y, goal_tol, rewards, masks,
                       oracle_reps);
  else
    hipLaunchKernelGGL(relabel_maze_kernel<float>, dim3(grid_for(num_rows)), dim3(256), 0, s,
                       (const float*)qpos, qpos_stride, num_rows, goal_x, goal_y, goal_tol, rewards, masks,
                       oracle_reps);
  OGBX_LAUNCHED("relabel_maze_kernel");
  return OGBX_OK;
}

}  // extern "C"
