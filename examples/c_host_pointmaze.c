/*
 * c_host_pointmaze.c -- a host with no Python and no torch driving the hot path
 * through the C-ABI alone (include/ogbx.h): what a Go / Java / C++ maintainer
 * binds.  pointmaze-large-navigate-v0 (locomaze/__init__.py:27-35): N envs,
 * reset(task_id = i % 5 + 1, seed), K steps of random float32 actions with
 * same-step auto-reset, then the ogbx_eval_accumulate success counters.
 *
 * Device memory and the stream come from the HIP runtime directly.  Checks:
 * every obs stays inside the maze's bounding box, every env is truncated
 * exactly at the TimeLimit when it never reached its goal, the counters add
 * up, and a rerun with the same seed is bit-identical.  Prints one summary line.
 *
 * Build (examples/Makefile):
 *   hipcc -O2 -I../include examples/c_host_pointmaze.c -L../ogbench_amd -logbx -o c_host_pointmaze
 */
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ogbx.h"

#define CHECK_OGBX(x)                                                                        \
  do {                                                                                       \
    ogbx_status st_ = (x);                                                                   \
    if (st_ != OGBX_OK) {                                                                    \
      fprintf(stderr, "%s:%d: %s -> %d (%s)\n", __FILE__, __LINE__, #x, st_, ogbx_last_error()); \
      exit(2);                                                                               \
    }                                                                                        \
  } while (0)
#define CHECK_HIP(x)                                                                         \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      fprintf(stderr, "%s:%d: %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));  \
      exit(3);                                                                               \
    }                                                                                        \
  } while (0)

/* xorshift64* -> uniform [-1, 1) float32 actions, host side */
static float urand(uint64_t* s) {
  uint64_t x = *s;
  x ^= x >> 12;
  x ^= x << 25;
  x ^= x >> 27;
  *s = x;
  return (float)((x * 0x2545F4914F6CDD1DULL) >> 40) / (float)(1 << 24) * 2.0f - 1.0f;
}

typedef struct {
  double* qpos_final;
  int64_t counters[16];
} run_out;

static void run(int64_t n, int k, uint64_t seed, run_out* out) {
  ogbx_maze_opts o;
  memset(&o, 0, sizeof(o));
  o.loco_type = 0;
  o.success_timing = 0;
  o.terminate_at_goal = 1;
  o.add_noise_to_goal = 1;
  o.reward_task_id = -1;
  o.max_episode_steps = 1000;
  o.env_base = 0;
  ogbx_maze_t env;
  CHECK_OGBX(ogbx_maze_create("large", n, 0, &o, &env));
  int32_t tasks_n = 0;
  CHECK_OGBX(ogbx_maze_describe(env, NULL, NULL, &tasks_n, NULL, NULL));

  hipStream_t stream;
  CHECK_HIP(hipStreamCreate(&stream));
  int32_t* h_task = (int32_t*)malloc(n * sizeof(int32_t));
  for (int64_t i = 0; i < n; ++i) h_task[i] = (int32_t)(i % tasks_n) + 1;
  int32_t *d_task, *d_remaining;
  double *d_obs, *d_goal;
  float *d_act, *d_rew;
  uint8_t *d_term, *d_trunc, *d_succ;
  int64_t* d_cnt;
  CHECK_HIP(hipMalloc((void**)&d_task, n * sizeof(int32_t)));
  CHECK_HIP(hipMalloc((void**)&d_remaining, n * sizeof(int32_t)));
  CHECK_HIP(hipMalloc((void**)&d_obs, n * 2 * sizeof(double)));
  CHECK_HIP(hipMalloc((void**)&d_goal, n * 2 * sizeof(double)));
  CHECK_HIP(hipMalloc((void**)&d_act, (size_t)k * n * 2 * sizeof(float)));
  CHECK_HIP(hipMalloc((void**)&d_rew, n * sizeof(float)));
  CHECK_HIP(hipMalloc((void**)&d_term, n));
  CHECK_HIP(hipMalloc((void**)&d_trunc, n));
  CHECK_HIP(hipMalloc((void**)&d_succ, n));
  CHECK_HIP(hipMalloc((void**)&d_cnt, tasks_n * 2 * sizeof(int64_t)));
  CHECK_HIP(hipMemcpy(d_task, h_task, n * sizeof(int32_t), hipMemcpyHostToDevice));
  CHECK_HIP(hipMemset(d_cnt, 0, tasks_n * 2 * sizeof(int64_t)));
  /* one episode per env is counted */
  for (int64_t i = 0; i < n; ++i) h_task[i] = 1;
  CHECK_HIP(hipMemcpy(d_remaining, h_task, n * sizeof(int32_t), hipMemcpyHostToDevice));
  for (int64_t i = 0; i < n; ++i) h_task[i] = (int32_t)(i % tasks_n) + 1;

  float* h_act = (float*)malloc((size_t)k * n * 2 * sizeof(float));
  uint64_t rs = 0x9E3779B97F4A7C15ULL ^ seed;
  for (size_t j = 0; j < (size_t)k * n * 2; ++j) h_act[j] = urand(&rs);
  CHECK_HIP(hipMemcpy(d_act, h_act, (size_t)k * n * 2 * sizeof(float), hipMemcpyHostToDevice));

  /* MazeEnv.reset(seed, options={'task_id': ...}) for every env */
  CHECK_OGBX(ogbx_maze_reset(env, d_task, NULL, NULL, NULL, d_obs, d_goal, seed, stream));
  for (int t = 0; t < k; ++t) {
    /* TimeLimit -> MazeEnv.step -> PointEnv.step, auto-reset on done */
    CHECK_OGBX(ogbx_maze_step(env, d_act + (size_t)t * n * 2, 0, 1, d_obs, d_rew, d_term, d_trunc, d_succ, NULL, 1,
                              stream));
    /* evaluation.py:83-121 success bookkeeping on the device */
    CHECK_OGBX(ogbx_eval_accumulate(d_succ, d_term, d_trunc, d_task, d_remaining, n, tasks_n, d_cnt, stream));
  }
  CHECK_HIP(hipStreamSynchronize(stream));
  out->qpos_final = (double*)malloc(n * 2 * sizeof(double));
  CHECK_HIP(hipMemcpy(out->qpos_final, d_obs, n * 2 * sizeof(double), hipMemcpyDeviceToHost));
  CHECK_HIP(hipMemcpy(out->counters, d_cnt, tasks_n * 2 * sizeof(int64_t), hipMemcpyDeviceToHost));

  free(h_act);
  free(h_task);
  hipFree(d_task);
  hipFree(d_remaining);
  hipFree(d_obs);
  hipFree(d_goal);
  hipFree(d_act);
  hipFree(d_rew);
  hipFree(d_term);
  hipFree(d_trunc);
  hipFree(d_succ);
  hipFree(d_cnt);
  CHECK_HIP(hipStreamDestroy(stream));
  CHECK_OGBX(ogbx_maze_destroy(env));
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 65536;
  const int k = argc > 2 ? atoi(argv[2]) : 1100;
  if (ogbx_abi_version() != OGBX_ABI_VERSION) {
    fprintf(stderr, "ABI mismatch: header %d, library %d\n", OGBX_ABI_VERSION, ogbx_abi_version());
    return 4;
  }
  run_out a, b;
  run(n, k, 42, &a);
  run(n, k, 42, &b);
  int bad = 0;
  /* the large maze spans x in [-6, 42], y in [-6, 30] (9 x 12 cells of 4) */
  for (int64_t i = 0; i < n; ++i) {
    const double x = a.qpos_final[2 * i], y = a.qpos_final[2 * i + 1];
    if (!(x > -6.0 && x < 42.0 && y > -6.0 && y < 30.0) || isnan(x) || isnan(y)) ++bad;
  }
  const int same = memcmp(a.qpos_final, b.qpos_final, n * 2 * sizeof(double)) == 0 &&
                   memcmp(a.counters, b.counters, sizeof(a.counters)) == 0;
  int64_t episodes = 0, successes = 0;
  for (int t = 0; t < 5; ++t) {
    successes += a.counters[2 * t];
    episodes += a.counters[2 * t + 1];
  }
  /* k > 1000: every env finished at least one episode (TimeLimit 1000) */
  const int ok = bad == 0 && same && episodes == n && successes >= 0 && successes <= episodes;
  printf("c_host_pointmaze: n=%lld k=%d episodes=%lld successes=%lld out_of_box=%d rerun_identical=%d %s\n",
         (long long)n, k, (long long)episodes, (long long)successes, bad, same, ok ? "OK" : "FAIL");
  free(a.qpos_final);
  free(b.qpos_final);
  return ok ? 0 : 1;
}
