// eval.hip -- per-task episode counters for batched evaluation.
//
// Reference: impls/utils/evaluation.py:36-123 (evaluate: success of the final
// step of each episode, averaged per task) and impls/main.py:226-258 (per-task
// means, overall = mean over tasks).  Here every env of a batch runs its own
// task; at each step the envs whose episode ends (terminated | truncated) add
// their final success to counters[task-1] = {success_sum, episode_count}, until
// each env has contributed `remaining[env]` episodes.  The counters are the
// int64[num_tasks, 2] block that the ranks all-gather.
#include <algorithm>

#include "common.h"

namespace ogbx {

constexpr int kEvalMaxTasks = 64;

__global__ void __launch_bounds__(256) eval_accumulate_kernel(
    const uint8_t* __restrict__ success, const uint8_t* __restrict__ terminated,
    const uint8_t* __restrict__ truncated, const int32_t* __restrict__ task_id,
    int32_t* __restrict__ remaining, int64_t n, int32_t num_tasks,
    unsigned long long* __restrict__ counters) {
  __shared__ unsigned int s_cnt[kEvalMaxTasks][2];
  for (int i = threadIdx.x; i < num_tasks * 2; i += blockDim.x) s_cnt[i >> 1][i & 1] = 0;
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if ((terminated[i] | truncated[i]) && remaining[i] > 0) {
      const int t = task_id[i] - 1;
      if (t >= 0 && t < num_tasks) {
        atomicAdd(&s_cnt[t][0], success[i] ? 1u : 0u);
        atomicAdd(&s_cnt[t][1], 1u);
      }
      remaining[i] -= 1;
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < num_tasks * 2; i += blockDim.x) {
    const unsigned int v = s_cnt[i >> 1][i & 1];
    if (v) atomicAdd(&counters[i], (unsigned long long)v);
  }
}

}  // namespace ogbx

using namespace ogbx;

extern "C" {

ogbx_status ogbx_eval_accumulate(const uint8_t* success, const uint8_t* terminated,
                                 const uint8_t* truncated, const int32_t* task_id,
                                 int32_t* remaining, int64_t n, int32_t num_tasks, int64_t* counters,
                                 void* stream) {
  OGBX_CHECK(success && terminated && truncated && task_id && remaining && counters, OGBX_EINVAL,
             "ogbx_eval_accumulate: null argument");
  OGBX_CHECK(n >= 0 && num_tasks >= 1 && num_tasks <= kEvalMaxTasks, OGBX_EINVAL,
             "ogbx_eval_accumulate: bad n or num_tasks (1..64)");
  if (n == 0) return OGBX_OK;
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 1024);
  hipLaunchKernelGGL(eval_accumulate_kernel, dim3((uint32_t)blocks), dim3(256), 0, (hipStream_t)stream,
                     success, terminated, truncated, task_id, remaining, n, num_tasks,
                     reinterpret_cast<unsigned long long*>(counters));
  OGBX_LAUNCHED("eval_accumulate_kernel");
  return OGBX_OK;
}

}  // extern "C"
