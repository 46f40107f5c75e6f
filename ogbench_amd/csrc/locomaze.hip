// locomaze.hip -- batched pointmaze envs on gfx950: reset / step / physics kernels
// and their C-ABI (include/ogbx.h).
//
// Layout in HBM (one handle = one batch of N envs on one device):
//   qpos    f64[N,2]  (x, y interleaved: one 16-B load/store per lane)
//   goal    f64[N,2]
//   elapsed i32[N]    TimeLimit counter (gymnasium TimeLimit, max_episode_steps)
//   task    i32[N]    1-based task id of the running episode
//   episode u32[N]    per-env reset counter (Philox counter word)
// Static tables (map, tasks, teleports, model constants) travel as one by-value
// kernel argument; the map is staged into LDS at block start.
//
// Reference behaviour restated here (paths relative to hliuson/ogbench):
//   MazeEnv.reset   ogbench/locomaze/maze.py:373-431
//   MazeEnv.step    ogbench/locomaze/maze.py:433-466
//   compute_success ogbench/locomaze/maze.py:486-490
//   xy_to_ij / ij_to_xy / add_noise  maze.py:552-567
//   PointEnv.step   ogbench/locomaze/point.py:64-95
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <string>
#include <vector>

#include "common.h"
#include "point_physics.h"
#include "point_contact.h"


namespace ogbx {

constexpr int kMaxCells = 256;
constexpr int kMaxTasks = 8;

struct MazeParams {
  PointModel pm;
  int32_t H, W, num_tasks, loco_type;
  int32_t success_pre, terminate_at_goal, add_noise_to_goal, reward_task_id;
  int32_t max_steps, n_tp_in, n_tp_out, pad_;
  int64_t env_base;  // global index of env 0: Philox streams count global envs
  double goal_tol, tp_radius;
  double tp_in[2][2];
  double tp_out[3][2];
  int32_t tasks[kMaxTasks][4];  // init_i, init_j, goal_i, goal_j
  uint8_t wall[kMaxCells];
  uint16_t nbmask[kMaxCells];   // 3x3 wall mask per cell, bit (di+1)*3+(dj+1)
};

struct MazeState {
  double* qpos;
  double* goal;
  int32_t* elapsed;
  int32_t* task;
  uint32_t* episode;
};

}  // namespace ogbx

struct ogbx_maze_env {
  int32_t device = 0;
  int64_t n = 0;
  ogbx::MazeParams P;
  ogbx::MazeState S{};
  ogbx::MazeParams* Pd = nullptr;  // device copy of P (tables indexed per lane)
  int16_t* bfs = nullptr;  // [H*W goal cell][H*W cell] BFS distances (maze.py:517-536)
  uint64_t seed = 0;
  bool was_reset = false;
  double* body_qpos = nullptr;  // ant handles: f64[N,15] (antmaze.h)
  double* body_qvel = nullptr;  // ant handles: f64[N,14]
  int epw = 64;  // envs per 64-lane wave of the step/physics kernels
  int lds_pad = 0;  // dynamic LDS bytes requested per step/physics workgroup
  // outputs bound by ogbx_maze_bind_step for ogbx_maze_step_bound
  bool bound = false;
  double* b_obs = nullptr;
  float* b_reward = nullptr;
  uint8_t *b_term = nullptr, *b_trunc = nullptr, *b_succ = nullptr;
  double* b_final = nullptr;
  int32_t b_auto = 0;
};

namespace ogbx {

// ------------------------------------------------------------ device helpers

// The contact model is the same for every maze (P.pm == kPointModel, checked at
// create): the step kernels use the compile-time copy so its ~30 constants fold
// into the instructions instead of living in (spilled) SGPRs.
#define OGBX_POINT_MODEL(pm, P) constexpr PointModel pm = kPointModel

__device__ inline void stage_wall(const MazeParams& P, uint8_t* wall_s) {
  for (int t = threadIdx.x; t < P.H * P.W; t += blockDim.x) wall_s[t] = P.wall[t];
  __syncthreads();
}

__device__ inline void stage_nbmask(const MazeParams& P, uint16_t* nb_s) {
  for (int t = threadIdx.x; t < P.H * P.W; t += blockDim.x) nb_s[t] = P.nbmask[t];
  __syncthreads();
}

// The step/physics kernels run 256-thread blocks, one thread per entry of the
// kMaxCells-entry wall-mask table: each thread loads its entry straight from
// the table's address (no dependent read of H*W), issued together with the
// env's state and action loads so that the whole prologue is one HBM round
// trip; nbmask_commit stores it into LDS after them.
constexpr int kStepBlock = 256;
static_assert(kMaxCells == kStepBlock, "one wall-mask entry per thread of a step block");

__device__ __forceinline__ uint16_t nbmask_fetch(const MazeParams* Pp) { return Pp->nbmask[threadIdx.x]; }

__device__ __forceinline__ void nbmask_commit(uint16_t* nb_s, uint16_t v) {
  nb_s[threadIdx.x] = v;
  __syncthreads();
}

// np.linalg.norm(xy - goal) <= tol with the 1-D OpenBLAS ddot rounding:
// sqrt(fma(dy, dy, dx*dx)) (maze.py:487).
__device__ inline bool goal_reached(double x, double y, double gx, double gy, double tol) {
  double dx = x - gx, dy = y - gy;
  return sqrt(fma(dy, dy, dx * dx)) <= tol;
}

// The four uniform(-1, 1) reset draws of one env, in reference order
// (init x, init y, goal x, goal y).
__device__ inline void reset_draws(uint64_t i, uint32_t ep, uint32_t k0, uint32_t k1,
                                   double r[4]) {
  u32x4 a = philox4x32_10({(uint32_t)i, ep, 0u, (uint32_t)(i >> 32)}, k0, k1);
  u32x4 b = philox4x32_10({(uint32_t)i, ep, 1u, (uint32_t)(i >> 32)}, k0, k1);
  r[0] = -1.0 + 2.0 * u01_from(a.x, a.y);
  r[1] = -1.0 + 2.0 * u01_from(a.z, a.w);
  r[2] = -1.0 + 2.0 * u01_from(b.x, b.y);
  r[3] = -1.0 + 2.0 * u01_from(b.z, b.w);
}

__device__ inline int32_t draw_task(const MazeParams& P, uint64_t i, uint32_t ep, uint32_t k0,
                                    uint32_t k1) {
  u32x4 c = philox4x32_10({(uint32_t)i, ep, 2u, (uint32_t)(i >> 32)}, k0, k1);
  return 1 + (int32_t)bounded_u32(c.x, (uint32_t)P.num_tasks);
}

// MazeEnv.reset for one env: returns init (x, y) and goal (gx, gy).
// add_noise: xy + uniform(-1,1) * maze_unit / 4 (maze.py:564-567).
__device__ inline void reset_one(const MazeParams& P, int32_t task, const double* task_xy,
                                 const double r[4], double& x, double& y, double& gx,
                                 double& gy) {
  double ix, iy, bx, by;
  if (task_xy != nullptr) {
    ix = task_xy[0];
    iy = task_xy[1];
    bx = task_xy[2];
    by = task_xy[3];
  } else {
    const int32_t* t = P.tasks[task - 1];
    ix = t[1] * P.pm.unit - P.pm.off_x;
    iy = t[0] * P.pm.unit - P.pm.off_y;
    bx = t[3] * P.pm.unit - P.pm.off_x;
    by = t[2] * P.pm.unit - P.pm.off_y;
  }
  x = ix + r[0] * P.pm.unit / 4.0;
  y = iy + r[1] * P.pm.unit / 4.0;
  if (P.add_noise_to_goal) {
    gx = bx + r[2] * P.pm.unit / 4.0;
    gy = by + r[3] * P.pm.unit / 4.0;
  } else {
    gx = bx;
    gy = by;
  }
}

// ------------------------------------------------------------------ kernels

// Env index of this lane when each 64-lane wave carries only `epw` envs
// (epw in {8, 16, 32, 64}).  The contact path is a long fp64 dependency chain,
// so one full wave per SIMD leaves the SIMD idle; fewer envs per wave (more
// waves per SIMD) lets the SIMD interleave independent chains.  Returns -1 for
// idle lanes.  With kEpwReplicate the other lanes of the wave are not idle but
// copies: lane l steps env (l mod epw) of the wave's epw envs bit for bit (every
// choice of the contact path is per lane), and only lanes l < epw (*writer)
// store.  A wave then runs the union of the paths of only epw envs with all 64
// lanes active (gfx950 issues a dependent chain ~2x slower with few active
// lanes).
constexpr int kEpwReplicate = 0x100;

__device__ inline int64_t env_of_lane(int epw, bool* writer) {
  const int lane = threadIdx.x & 63;
  const int e = epw & 0xFF;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  *writer = lane < e;
  if (lane >= e && !(epw & kEpwReplicate)) return -1;
  return wave * e + (lane & (e - 1));
}

__global__ void __launch_bounds__(256) maze_reset_kernel(const MazeParams* __restrict__ Pp, MazeState S, int64_t n,
                                                         const int32_t* task_id,
                                                         const double* task_xy,
                                                         const uint8_t* mask, const double* noise,
                                                         double* obs, double* goal_out,
                                                         uint32_t k0, uint32_t k1) {
  const MazeParams& P = *Pp;
  const PointModel pm = P.pm;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (mask != nullptr && mask[i] == 0) return;
  uint32_t ep = S.episode[i] + 1u;
  const uint64_t gi = (uint64_t)(i + P.env_base);
  int32_t task;
  if (P.reward_task_id > 0) task = P.reward_task_id;
  else if (task_id != nullptr) task = task_id[i];
  else task = draw_task(P, gi, ep, k0, k1);
  if (task < 1 || task > P.num_tasks) task = 1;  // validated on the host
  double r[4];
  if (noise != nullptr) {
    r[0] = noise[4 * i + 0];
    r[1] = noise[4 * i + 1];
    r[2] = noise[4 * i + 2];
    r[3] = noise[4 * i + 3];
  } else {
    reset_draws(gi, ep, k0, k1, r);
  }
  double x, y, gx, gy;
  reset_one(P, task, task_xy ? task_xy + 4 * i : nullptr, r, x, y, gx, gy);
  S.qpos[2 * i] = x;
  S.qpos[2 * i + 1] = y;
  S.goal[2 * i] = gx;
  S.goal[2 * i + 1] = gy;
  S.elapsed[i] = 0;
  S.task[i] = task;
  S.episode[i] = ep;
  obs[2 * i] = x;
  obs[2 * i + 1] = y;
  goal_out[2 * i] = gx;
  goal_out[2 * i + 1] = gy;
}

// One launch = k_steps consecutive env steps of every env; state stays in
// registers across the k loop.  One lane per env.
// kUntilDone (no auto-reset): an env stops at the first step that ends its
// episode (terminated | truncated); its later rows are not written, its state
// is the state at that step, and steps_taken[i] counts the rows it wrote.  A
// wave leaves the k loop as soon as a ballot finds every lane done, so a batch
// of evaluation episodes costs the steps of its longest episode per wave, not
// k_steps.  Until then a done lane keeps stepping unobserved (as K single
// steps would), so the wave's contact-path choice -- and with it every written
// row -- is bit-identical to K calls of the single step.
#ifdef OGBX_WAVE_STAMPS
__device__ unsigned long long g_wave_stamps[4096 * 4];
#endif

typedef double f64x2 __attribute__((ext_vector_type(2)));  // 16-byte non-temporal stores

template <bool kF64, bool kUntilDone>
__global__ void __launch_bounds__(256) maze_step_kernel(
    const MazeParams* __restrict__ Pp, MazeState S, int64_t n, const void* __restrict__ action_v,
    int32_t k_steps,
    double* __restrict__ obs, float* __restrict__ reward, uint8_t* __restrict__ terminated,
    uint8_t* __restrict__ truncated, uint8_t* __restrict__ success,
    double* __restrict__ final_obs, int32_t auto_reset, uint32_t k0, uint32_t k1, int epw,
    int32_t* __restrict__ steps_taken) {
  const MazeParams& P = *Pp;
  OGBX_POINT_MODEL(pm, P);
  __shared__ uint16_t nb_s[kMaxCells];
#ifdef OGBX_WAVE_STAMPS
  const unsigned long long ws_t0 = wall_clock64(), ws_c0 = clock64();
#endif
  bool writer;
  const int64_t i = env_of_lane(epw, &writer);
  const bool live = i >= 0 && i < n;
  // one HBM round trip before the first barrier: the wall-mask entry, the
  // env's state and its first action
  const uint16_t nbv = nbmask_fetch(Pp);
  double2 q = make_double2(0.0, 0.0), g = q, a0d = q;
  float2 a0f = make_float2(0.0f, 0.0f);
  int32_t el = 0, task = 1;
  uint32_t ep = 0;
  if (live) {
    if (kF64) a0d = reinterpret_cast<const double2*>(action_v)[i];
    else a0f = reinterpret_cast<const float2*>(action_v)[i];
    q = reinterpret_cast<const double2*>(S.qpos)[i];
    g = reinterpret_cast<const double2*>(S.goal)[i];
    el = S.elapsed[i];
  }
  nbmask_commit(nb_s, nbv);
  if (!live) return;
  // task and episode counter are read only by an auto-reset or a teleport:
  // fetched here (their round trip hides under the physics) for the envs that
  // can end this step -- TimeLimit, or within goal_tol + 2 of the goal (a step
  // moves |0.2 a| <= 0.29 for actions in the action space) -- and lazily by
  // any other env that does end (an out-of-space action)
  bool have_te = k_steps > 1 || P.n_tp_in > 0 || el + 1 >= P.max_steps;
  {
    const double ddx = q.x - g.x, ddy = q.y - g.y, lim = P.goal_tol + 2.0;
    have_te |= ddx * ddx + ddy * ddy <= lim * lim;
  }
  if (have_te) {
    ep = S.episode[i];
    task = S.task[i];
  }
  const uint64_t gi = (uint64_t)(i + P.env_base);
  double x = q.x, y = q.y, gx = g.x, gy = g.y;
  bool reset_any = false;  // goal / episode change only on an auto-reset
  bool done = false;       // kUntilDone: this env's episode has ended
  int32_t taken = 0;
  double dx_ = x, dy_ = y;  // kUntilDone: the state at the end of the episode
  int32_t del_ = el;

  for (int32_t k = 0; k < k_steps; ++k) {
    if (kUntilDone) {
      if (__all(done)) break;  // wave-uniform early exit (ballot over live lanes)
    }
    const int64_t o = (int64_t)k * n + i;
    double dx, dy;
    if (kF64) {
      const double2 a = k == 0 ? a0d : reinterpret_cast<const double2*>(action_v)[o];
      dx = 0.2 * a.x;
      dy = 0.2 * a.y;
    } else {
      const float2 a = k == 0 ? a0f : reinterpret_cast<const float2*>(action_v)[o];
      dx = (double)(0.2f * a.x);  // float32 * weak python float stays float32 (NEP 50)
      dy = (double)(0.2f * a.y);
    }
    bool succ = false;
    if (P.success_pre) succ = goal_reached(x, y, gx, gy, P.goal_tol);
    x = x + dx;
    y = y + dy;
    point_step_as(pm, nb_s, P.H, P.W, &x, &y);
    if (!P.success_pre) succ = goal_reached(x, y, gx, gy, P.goal_tol);
    const double ox = x, oy = y;  // ob is taken before a teleport (maze.py:437-451)
    if (P.n_tp_in > 0) {
      for (int t = 0; t < P.n_tp_in; ++t) {
        if (goal_reached(x, y, P.tp_in[t][0], P.tp_in[t][1], P.tp_radius * 1.5)) {
          u32x4 c = philox4x32_10({(uint32_t)gi, ep, 0x100u + (uint32_t)el, (uint32_t)(gi >> 32)},
                                  k0 ^ kTagMazeTeleport, k1);
          int o_idx = (int)bounded_u32(c.x, (uint32_t)P.n_tp_out);
          x = P.tp_out[o_idx][0];
          y = P.tp_out[o_idx][1];
          break;
        }
      }
    }
    float rew = succ ? 1.0f : 0.0f;
    if (P.reward_task_id > 0) rew -= 1.0f;
    const bool term = succ && P.terminate_at_goal;
    el += 1;
    const bool trunc = el >= P.max_steps;
    const bool write = writer && (!kUntilDone || !done);
    if (write) {
      __builtin_nontemporal_store(rew, &reward[o]);
      __builtin_nontemporal_store((uint8_t)term, &terminated[o]);
      __builtin_nontemporal_store((uint8_t)trunc, &truncated[o]);
      __builtin_nontemporal_store((uint8_t)succ, &success[o]);
    }
    double wx = ox, wy = oy;
    if (auto_reset && (term || trunc)) {
      if (!have_te) {
        ep = S.episode[i];
        task = S.task[i];
        have_te = true;
      }
      if (final_obs != nullptr && writer) reinterpret_cast<double2*>(final_obs)[o] = make_double2(ox, oy);
      ep += 1u;
      reset_any = true;
      double r[4];
      reset_draws(gi, ep, k0, k1, r);
      reset_one(P, task, nullptr, r, x, y, gx, gy);
      el = 0;
      wx = x;
      wy = y;
    }
    if (write) __builtin_nontemporal_store(f64x2{wx, wy}, reinterpret_cast<f64x2*>(obs) + o);
    if (kUntilDone && !done) {
      taken = k + 1;
      done = term || trunc;
      dx_ = x;
      dy_ = y;
      del_ = el;
    }
  }
  if (kUntilDone) {
    x = dx_;
    y = dy_;
    el = del_;
    if (writer) steps_taken[i] = taken;
  }
  if (!writer) return;  // a copy lane (kEpwReplicate)
  // non-temporal stores for the state and the outputs (nothing in the launch
  // reads them back): 11.37 -> 11.29 us per launch at N = 65,536 (A/B,
  // four rounds), no change at 8,192
  __builtin_nontemporal_store(f64x2{x, y}, reinterpret_cast<f64x2*>(S.qpos) + i);
  __builtin_nontemporal_store(el, &S.elapsed[i]);
  if (reset_any) {
    reinterpret_cast<double2*>(S.goal)[i] = make_double2(gx, gy);
    S.episode[i] = ep;
  }
#ifdef OGBX_WAVE_STAMPS
  {
    const unsigned long long t1 = wall_clock64(), c1 = clock64();
    const int64_t w = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if ((threadIdx.x & 63) == 0 && w < 4096) {
      g_wave_stamps[4 * w + 0] = ws_t0;
      g_wave_stamps[4 * w + 1] = t1;
      g_wave_stamps[4 * w + 2] = c1 - ws_c0;
    }
  }
#endif
}

template <bool kF64>
__global__ void __launch_bounds__(256) point_physics_kernel(const MazeParams* __restrict__ Pp,
                                                            const double* qpos_in,
                                                            const void* action_v, int64_t n,
                                                            double* qpos_out,
                                                            uint8_t* contact_out, int epw) {
  OGBX_POINT_MODEL(pm, (*Pp));
  __shared__ uint16_t nb_s[kMaxCells];
  bool writer;
  const int64_t i = env_of_lane(epw, &writer);
  const bool live = i >= 0 && i < n;
  const uint16_t nbv = nbmask_fetch(Pp);
  double x = 0.0, y = 0.0, ax = 0.0, ay = 0.0;
  if (live) {
    x = qpos_in[2 * i];
    y = qpos_in[2 * i + 1];
    if (kF64) {
      const double* a = (const double*)action_v;
      ax = 0.2 * a[2 * i];
      ay = 0.2 * a[2 * i + 1];
    } else {
      const float* a = (const float*)action_v;
      ax = (double)(0.2f * a[2 * i]);
      ay = (double)(0.2f * a[2 * i + 1]);
    }
  }
  nbmask_commit(nb_s, nbv);
  if (!live) return;
  const MazeParams& P = *Pp;
  x = x + ax;
  y = y + ay;
  int c = point_step_as(pm, nb_s, P.H, P.W, &x, &y);
  if (!writer) return;  // a copy lane (kEpwReplicate)
  qpos_out[2 * i] = x;
  qpos_out[2 * i + 1] = y;
  if (contact_out) contact_out[i] = (uint8_t)c;
}

// xy_to_ij: i = int((y + off_y + 0.5*unit)/unit) with Python int() truncation
// toward zero (maze.py:552-556).
__global__ void xy_to_ij_kernel(const MazeParams* __restrict__ Pp, const double* xy, int64_t n, int32_t* ij) {
  const MazeParams& P = *Pp;
  const PointModel pm = P.pm;
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  double x = xy[2 * t], y = xy[2 * t + 1];
  double fi = (y + P.pm.off_y + 0.5 * P.pm.unit) / P.pm.unit;
  double fj = (x + P.pm.off_x + 0.5 * P.pm.unit) / P.pm.unit;
  fi = fmin(fmax(fi, -2147483648.0), 2147483647.0);
  fj = fmin(fmax(fj, -2147483648.0), 2147483647.0);
  ij[2 * t] = (int32_t)fi;
  ij[2 * t + 1] = (int32_t)fj;
}

__global__ void ij_to_xy_kernel(const MazeParams* __restrict__ Pp, const int32_t* ij, int64_t n, double* xy) {
  const MazeParams& P = *Pp;
  const PointModel pm = P.pm;
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  xy[2 * t] = ij[2 * t + 1] * P.pm.unit - P.pm.off_x;
  xy[2 * t + 1] = ij[2 * t] * P.pm.unit - P.pm.off_y;
}

__device__ inline int clamp_idx(double f, int hi) {
  f = fmin(fmax(f, -1.0), (double)hi);
  int v = (int)f;
  return v < 0 ? 0 : (v > hi - 1 ? hi - 1 : v);
}

// get_oracle_subgoal (maze.py:503-550) from the precomputed BFS table.
// get_oracle_subgoal (maze.py:503-550) for one (start, goal) pair from the
// precomputed BFS distance table (int16 [goal cell][cell], -1 unreachable).
__device__ inline void subgoal_of(const MazeParams& P, const uint8_t* wall_s, const int16_t* bfs, double x,
                                  double y, double gx, double gy, double* sx_out, double* sy_out) {
  const int H = P.H, W = P.W;
  const int si = clamp_idx((y + P.pm.off_y + 0.5 * P.pm.unit) / P.pm.unit, H);
  const int sj = clamp_idx((x + P.pm.off_x + 0.5 * P.pm.unit) / P.pm.unit, W);
  const int gi = clamp_idx((gy + P.pm.off_y + 0.5 * P.pm.unit) / P.pm.unit, H);
  const int gj = clamp_idx((gx + P.pm.off_x + 0.5 * P.pm.unit) / P.pm.unit, W);
  const int16_t* d = bfs + (int64_t)(gi * W + gj) * (H * W);
  int bi = si, bj = sj;
  const int di[4] = {-1, 0, 1, 0}, dj[4] = {0, -1, 0, 1};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int ni = si + di[k], nj = sj + dj[k];
    if (ni >= 0 && ni < H && nj >= 0 && nj < W && wall_s[ni * W + nj] == 0 && d[ni * W + nj] < d[bi * W + bj]) {
      bi = ni;
      bj = nj;
    }
  }
  *sx_out = bj * P.pm.unit - P.pm.off_x;
  *sy_out = bi * P.pm.unit - P.pm.off_y;
}

__global__ void oracle_subgoal_kernel(const MazeParams* __restrict__ Pp, const int16_t* bfs, const double* start_xy,
                                      const double* goal_xy, int64_t n, double* sub_xy) {
  const MazeParams& P = *Pp;
  __shared__ uint8_t wall_s[kMaxCells];
  stage_wall(P, wall_s);
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  subgoal_of(P, wall_s, bfs, start_xy[2 * t], start_xy[2 * t + 1], goal_xy[2 * t], goal_xy[2 * t + 1],
             &sub_xy[2 * t], &sub_xy[2 * t + 1]);
}

// Point-maze expert of data_gen_scripts/generate_locomaze.py:147-166 (the
// point actor returns the subgoal direction, :44-46):
//   dir = (subgoal - xy) / (||subgoal - xy|| + 1e-6),  ||v|| = sqrt(fma(vy, vy, vx*vx))
//   (np.linalg.norm of a 1-D pair goes through BLAS ddot), action =
//   clip(dir + normal, -1, 1) with normal = np.random.normal(0, noise, 2)
//   (injected, or noise * Box-Muller(Philox)).  float64 actions.
__global__ void expert_action_kernel(const MazeParams* __restrict__ Pp, const int16_t* bfs, const double* start_xy,
                                     const double* goal_xy, int64_t n, double noise, const double* normal,
                                     uint32_t k0, uint32_t k1, uint32_t call_lo, uint32_t call_hi,
                                     double* action) {
  const MazeParams& P = *Pp;
  __shared__ uint8_t wall_s[kMaxCells];
  stage_wall(P, wall_s);
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const double x = start_xy[2 * t], y = start_xy[2 * t + 1];
  double sx, sy;
  subgoal_of(P, wall_s, bfs, x, y, goal_xy[2 * t], goal_xy[2 * t + 1], &sx, &sy);
  const double dx = sx - x, dy = sy - y;
  const double den = sqrt(fma(dy, dy, dx * dx)) + 1e-6;
  const double ux = dx / den, uy = dy / den;
  double nx, ny;
  if (normal != nullptr) {
    nx = normal[2 * t];
    ny = normal[2 * t + 1];
  } else {
    const uint64_t gt = (uint64_t)(t + P.env_base);
    const u32x4 w = philox4x32_10({(uint32_t)gt, call_lo, 0x45u, (uint32_t)(gt >> 32) ^ call_hi}, k0, k1);
    const double u1 = 1.0 - u01_from(w.x, w.y);  // (0, 1]
    const double u2 = u01_from(w.z, w.w);
    const double r = sqrt(-2.0 * log(u1));
    const double a = 6.283185307179586 * u2;
    nx = 0.0 + noise * (r * cos(a));
    ny = 0.0 + noise * (r * sin(a));
  }
  double ax = ux + nx, ay = uy + ny;
  ax = ax < -1.0 ? -1.0 : (ax > 1.0 ? 1.0 : ax);
  ay = ay < -1.0 ? -1.0 : (ay > 1.0 ? 1.0 : ay);
  action[2 * t] = ax;
  action[2 * t + 1] = ay;
}

// MazeEnv.set_goal(goal_ij) (maze.py:492-501) for the envs with mask[i] != 0:
// goal = ij_to_xy(goal_ij) (+ add_noise: uniform(-1,1)*unit/4 per axis,
// injected or Philox).
__global__ void set_goal_kernel(const MazeParams* __restrict__ Pp, MazeState S, int64_t n, const int32_t* goal_ij,
                                const uint8_t* mask, const double* noise, uint32_t k0, uint32_t k1, uint32_t call_lo,
                                uint32_t call_hi) {
  const MazeParams& P = *Pp;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || (mask != nullptr && mask[i] == 0)) return;
  double gx = goal_ij[2 * i + 1] * P.pm.unit - P.pm.off_x;
  double gy = goal_ij[2 * i] * P.pm.unit - P.pm.off_y;
  if (P.add_noise_to_goal) {
    double r0, r1;
    if (noise != nullptr) {
      r0 = noise[2 * i];
      r1 = noise[2 * i + 1];
    } else {
      const uint64_t gi = (uint64_t)(i + P.env_base);
      const u32x4 w = philox4x32_10({(uint32_t)gi, call_lo, 0x47u, (uint32_t)(gi >> 32) ^ call_hi}, k0, k1);
      r0 = -1.0 + 2.0 * u01_from(w.x, w.y);
      r1 = -1.0 + 2.0 * u01_from(w.z, w.w);
    }
    gx = gx + r0 * P.pm.unit / 4.0;
    gy = gy + r1 * P.pm.unit / 4.0;
  }
  reinterpret_cast<double2*>(S.goal)[i] = make_double2(gx, gy);
}

}  // namespace ogbx

#include "antmaze.h"

namespace ogbx {

// ------------------------------------------------------------- host tables

struct MazeSpec {
  const char* name;
  int H, W;
  const char* rows;  // H*W chars '1'/'0'
  int ntasks;
  int tasks[5][4];
};

// Maps: maze.py:90-150.  Tasks: maze.py:310-345.
static const MazeSpec kMazes[] = {
    {"arena", 8, 8,
     "11111111"
     "10000001"
     "10000001"
     "10000001"
     "10000001"
     "10000001"
     "10000001"
     "11111111",
     1, {{1, 1, 6, 6}}},
    {"medium", 8, 8,
     "11111111"
     "10011001"
     "10010001"
     "11000111"
     "10010001"
     "10100101"
     "10001001"
     "11111111",
     5, {{1, 1, 6, 6}, {6, 1, 1, 6}, {5, 3, 4, 2}, {6, 5, 6, 1}, {2, 6, 1, 1}}},
    {"large", 9, 12,
     "111111111111"
     "100001000001"
     "101101010101"
     "100000010001"
     "101111011101"
     "100101000001"
     "110101010111"
     "100100010001"
     "111111111111",
     5, {{1, 1, 7, 10}, {5, 4, 7, 1}, {7, 4, 1, 10}, {3, 8, 5, 4}, {1, 1, 5, 4}}},
    {"giant", 12, 16,
     "1111111111111111"
     "1010000001100001"
     "1010110101001101"
     "1000100100010001"
     "1011101111110101"
     "1000100010000101"
     "1110101001010111"
     "1000100100010001"
     "1010101111110101"
     "1011100010001101"
     "1000001000100001"
     "1111111111111111",
     5, {{1, 1, 10, 14}, {1, 14, 10, 1}, {8, 14, 1, 1}, {8, 3, 5, 12}, {5, 9, 3, 8}}},
    {"teleport", 9, 12,
     "111111111111"
     "100000101001"
     "110100010011"
     "110111000001"
     "100001010101"
     "101101010101"
     "101101010101"
     "100001000101"
     "111111111111",
     5, {{1, 10, 7, 1}, {1, 1, 7, 10}, {5, 6, 7, 10}, {7, 1, 7, 10}, {5, 6, 7, 1}}},
};


static void build_bfs(const MazeParams& P, std::vector<int16_t>& out) {
  const int H = P.H, W = P.W, C = H * W;
  out.assign((size_t)C * C, -1);
  for (int g = 0; g < C; ++g) {
    int16_t* d = out.data() + (size_t)g * C;
    std::deque<int> qu;
    d[g] = 0;
    qu.push_back(g);
    const int di[4] = {-1, 0, 1, 0}, dj[4] = {0, -1, 0, 1};
    while (!qu.empty()) {
      int c = qu.front();
      qu.pop_front();
      int i = c / W, j = c % W;
      for (int k = 0; k < 4; ++k) {
        int ni = i + di[k], nj = j + dj[k];
        if (ni >= 0 && ni < H && nj >= 0 && nj < W && P.wall[ni * W + nj] == 0 &&
            d[ni * W + nj] == -1) {
          d[ni * W + nj] = (int16_t)(d[c] + 1);
          qu.push_back(ni * W + nj);
        }
      }
    }
  }
}

static inline uint32_t grid_for(int64_t n, int block) { return (uint32_t)((n + block - 1) / block); }

}  // namespace ogbx

using namespace ogbx;

extern "C" {

ogbx_status ogbx_maze_create(const char* maze_type, int64_t n_envs, int32_t device,
                             const ogbx_maze_opts* opts, ogbx_maze_t* out) {
  OGBX_CHECK(out != nullptr && maze_type != nullptr && opts != nullptr, OGBX_EINVAL,
             "ogbx_maze_create: null argument");
  *out = nullptr;
  OGBX_CHECK(n_envs > 0 && n_envs <= (int64_t)1 << 32, OGBX_EINVAL,
             "ogbx_maze_create: n_envs must be in [1, 2^32]");
  const MazeSpec* spec = nullptr;
  for (const auto& s : kMazes)
    if (std::strcmp(s.name, maze_type) == 0) spec = &s;
  OGBX_CHECK(spec != nullptr, OGBX_EINVAL, std::string("Unknown maze type: ") + maze_type);
  OGBX_CHECK(opts->loco_type >= 0 && opts->loco_type <= 2, OGBX_EINVAL,
             "Unknown locomotion environment type");
  OGBX_CHECK(opts->success_timing == 0 || opts->success_timing == 1, OGBX_EINVAL,
             "success_timing must be 'pre' or 'post'");
  OGBX_CHECK(opts->max_episode_steps > 0, OGBX_EINVAL, "max_episode_steps must be positive");
  OGBX_CHECK(opts->env_base >= 0, OGBX_EINVAL, "env_base must be >= 0");
  OGBX_CHECK(opts->reward_task_id <= spec->ntasks, OGBX_EINVAL,
             "Task ID must be in [1, " + std::to_string(spec->ntasks) + "].");
  ogbx_status st = use_device(device);
  if (st != OGBX_OK) return st;

  auto* e = new ogbx_maze_env();
  e->device = device;
  if (const char* v = std::getenv("OGBX_MAZE_LDS")) {  // diagnostic placement knob (A/B only)
    e->lds_pad = std::atoi(v);
    (void)hipFuncSetAttribute((const void*)maze_step_kernel<false, false>, hipFuncAttributeMaxDynamicSharedMemorySize, e->lds_pad);
    (void)hipFuncSetAttribute((const void*)maze_step_kernel<true, false>, hipFuncAttributeMaxDynamicSharedMemorySize, e->lds_pad);
    (void)hipFuncSetAttribute((const void*)maze_step_kernel<false, true>, hipFuncAttributeMaxDynamicSharedMemorySize, e->lds_pad);
    (void)hipFuncSetAttribute((const void*)maze_step_kernel<true, true>, hipFuncAttributeMaxDynamicSharedMemorySize, e->lds_pad);
    (void)hipFuncSetAttribute((const void*)point_physics_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, e->lds_pad);
    (void)hipFuncSetAttribute((const void*)point_physics_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, e->lds_pad);
  }
  e->n = n_envs;
  MazeParams& P = e->P;
  std::memset(&P, 0, sizeof(P));
  P.pm = kPointModel;
  P.H = spec->H;
  P.W = spec->W;
  P.num_tasks = spec->ntasks;
  P.loco_type = opts->loco_type;
  P.success_pre = opts->success_timing;
  P.terminate_at_goal = opts->terminate_at_goal;
  P.add_noise_to_goal = opts->add_noise_to_goal;
  P.reward_task_id = opts->reward_task_id == 0 ? 1 : opts->reward_task_id;  // maze.py:361-362
  if (opts->reward_task_id < 0) P.reward_task_id = -1;
  P.max_steps = opts->max_episode_steps;
  P.env_base = opts->env_base;
  P.goal_tol = opts->loco_type == 0 ? 1.0 : 0.5;  // maze.py:86
  for (int c = 0; c < spec->H * spec->W; ++c) P.wall[c] = spec->rows[c] == '1';
  for (int i = 0; i < spec->H; ++i)
    for (int j = 0; j < spec->W; ++j) {
      uint16_t m = 0;
      for (int di = -1; di <= 1; ++di)
        for (int dj = -1; dj <= 1; ++dj) {
          const int ii = i + di, jj = j + dj;
          if (ii >= 0 && ii < spec->H && jj >= 0 && jj < spec->W && P.wall[ii * spec->W + jj])
            m |= (uint16_t)(1u << ((di + 1) * 3 + (dj + 1)));
        }
      P.nbmask[i * spec->W + j] = m;
    }
  for (int t = 0; t < spec->ntasks; ++t)
    for (int k = 0; k < 4; ++k) P.tasks[t][k] = spec->tasks[t][k];
  if (std::strcmp(spec->name, "teleport") == 0) {  // maze.py:151-161
    const int in_ij[2][2] = {{4, 6}, {5, 1}};
    const int out_ij[3][2] = {{1, 7}, {6, 1}, {6, 10}};
    P.n_tp_in = 2;
    P.n_tp_out = 3;
    P.tp_radius = 1.0;
    for (int t = 0; t < 2; ++t) {
      P.tp_in[t][0] = in_ij[t][1] * 4.0 - 4.0;
      P.tp_in[t][1] = in_ij[t][0] * 4.0 - 4.0;
    }
    for (int t = 0; t < 3; ++t) {
      P.tp_out[t][0] = out_ij[t][1] * 4.0 - 4.0;
      P.tp_out[t][1] = out_ij[t][0] * 4.0 - 4.0;
    }
  }

  const size_t n = (size_t)n_envs;
  hipError_t herr = hipSuccess;
  herr = hipMalloc(&e->S.qpos, n * 2 * sizeof(double));
  if (herr == hipSuccess) herr = hipMalloc(&e->S.goal, n * 2 * sizeof(double));
  if (herr == hipSuccess) herr = hipMalloc(&e->S.elapsed, n * sizeof(int32_t));
  if (herr == hipSuccess) herr = hipMalloc(&e->S.task, n * sizeof(int32_t));
  if (herr == hipSuccess) herr = hipMalloc(&e->S.episode, n * sizeof(uint32_t));
  if (herr == hipSuccess && P.loco_type == 1) {
    herr = hipMalloc(&e->body_qpos, n * kAntNq * sizeof(double));
    if (herr == hipSuccess) herr = hipMalloc(&e->body_qvel, n * kAntNv * sizeof(double));
    if (herr == hipSuccess) herr = hipMemset(e->body_qpos, 0, n * kAntNq * sizeof(double));
    if (herr == hipSuccess) herr = hipMemset(e->body_qvel, 0, n * kAntNv * sizeof(double));
  }
  std::vector<int16_t> bfs;
  build_bfs(P, bfs);
  if (herr == hipSuccess) herr = hipMalloc(&e->Pd, sizeof(MazeParams));
  if (herr == hipSuccess) herr = hipMemcpy(e->Pd, &P, sizeof(MazeParams), hipMemcpyHostToDevice);
  if (herr == hipSuccess) herr = hipMalloc(&e->bfs, bfs.size() * sizeof(int16_t));
  if (herr == hipSuccess)
    herr = hipMemcpy(e->bfs, bfs.data(), bfs.size() * sizeof(int16_t), hipMemcpyHostToDevice);
  if (herr == hipSuccess) herr = hipMemset(e->S.qpos, 0, n * 2 * sizeof(double));
  if (herr == hipSuccess) herr = hipMemset(e->S.goal, 0, n * 2 * sizeof(double));
  if (herr == hipSuccess) herr = hipMemset(e->S.elapsed, 0, n * sizeof(int32_t));
  if (herr == hipSuccess) herr = hipMemset(e->S.task, 0, n * sizeof(int32_t));
  if (herr == hipSuccess) herr = hipMemset(e->S.episode, 0, n * sizeof(uint32_t));
  if (herr == hipSuccess) herr = hipDeviceSynchronize();
  if (herr != hipSuccess) {
    ogbx_maze_destroy(e);
    return hip_fail(herr, "ogbx_maze_create: device allocation");
  }
  *out = e;
  return OGBX_OK;
}

ogbx_status ogbx_maze_destroy(ogbx_maze_t e) {
  if (e == nullptr) return OGBX_OK;
  (void)hipSetDevice(e->device);
  (void)hipFree(e->S.qpos);
  (void)hipFree(e->S.goal);
  (void)hipFree(e->S.elapsed);
  (void)hipFree(e->S.task);
  (void)hipFree(e->S.episode);
  (void)hipFree(e->body_qpos);
  (void)hipFree(e->body_qvel);
  (void)hipFree(e->bfs);
  (void)hipFree(e->Pd);
  delete e;
  return OGBX_OK;
}

int64_t ogbx_maze_num_envs(ogbx_maze_t e) { return e ? e->n : 0; }

ogbx_status ogbx_maze_set_envs_per_wave(ogbx_maze_t e, int32_t epw) {
  OGBX_CHECK(e != nullptr, OGBX_EINVAL, "null handle");
  const int per = epw & ~kEpwReplicate;
  OGBX_CHECK((epw & ~(kEpwReplicate | 0xFF)) == 0 && (per == 8 || per == 16 || per == 32 || per == 64), OGBX_EINVAL,
             "envs per wave must be 8, 16, 32 or 64 (optionally | OGBX_EPW_REPLICATE)");
  e->epw = epw;
  return OGBX_OK;
}

#ifdef OGBX_WAVE_STAMPS
// Diagnostic build only: per-wave (start, end) wall clock (s_memrealtime,
// 100 MHz) and shader-clock cycles of the last maze_step_kernel launch.
ogbx_status ogbx_diag_wave_stamps(unsigned long long* out) {
  OGBX_HIP(hipDeviceSynchronize());
  OGBX_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wave_stamps), 4096 * 4 * sizeof(unsigned long long)));
  // slot 3: the path counters of point_physics.h g_wave_paths (then cleared)
  static unsigned long long paths[4096];
  OGBX_HIP(hipMemcpyFromSymbol(paths, HIP_SYMBOL(g_wave_paths), sizeof(paths)));
  for (int w = 0; w < 4096; ++w) out[4 * w + 3] = paths[w];
  static unsigned long long z[4096];
  OGBX_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_wave_paths), z, sizeof(z)));
  return OGBX_OK;
}
#endif

#ifdef OGBX_MASK_TRACE
// Diagnostic build only: the lean stages' start / settled masks of the last
// launch (point_contact.h g_mask_trace, 40 words per global thread).
ogbx_status ogbx_diag_mask_trace(uint32_t* out) {
  OGBX_HIP(hipDeviceSynchronize());
  OGBX_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_mask_trace), 65536 * 40 * sizeof(uint32_t)));
  return OGBX_OK;
}
#endif

#ifdef OGBX_STAGE_STAMPS
// Diagnostic build only: the per-wave lean-stage cycle parts of the last
// launch (point_contact.h g_wave_stages, 8 words per wave), then cleared.
ogbx_status ogbx_diag_wave_stages(unsigned long long* out) {
  OGBX_HIP(hipDeviceSynchronize());
  OGBX_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wave_stages), 4096 * 8 * sizeof(unsigned long long)));
  static unsigned long long z[4096 * 8];
  OGBX_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_wave_stages), z, sizeof(z)));
  return OGBX_OK;
}
#endif

#ifdef OGBX_PHYS_STATS
// Diagnostic build only: read and clear the 32 physics path counters.
ogbx_status ogbx_diag_phys_stats(unsigned long long* out16) {
  OGBX_HIP(hipDeviceSynchronize());
  OGBX_HIP(hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_phys_stats), 32 * sizeof(unsigned long long)));
  unsigned long long z[32] = {0};
  OGBX_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_phys_stats), z, sizeof(z)));
  return OGBX_OK;
}
#endif

ogbx_status ogbx_maze_static_tables(const char* maze_type, int32_t* map_h, int32_t* map_w,
                                    int32_t* num_tasks, int32_t* map_out, int32_t* tasks_out) {
  OGBX_CHECK(maze_type != nullptr, OGBX_EINVAL, "null maze_type");
  const MazeSpec* spec = nullptr;
  for (const auto& s : kMazes)
    if (std::strcmp(s.name, maze_type) == 0) spec = &s;
  OGBX_CHECK(spec != nullptr, OGBX_EINVAL, std::string("Unknown maze type: ") + maze_type);
  if (map_h) *map_h = spec->H;
  if (map_w) *map_w = spec->W;
  if (num_tasks) *num_tasks = spec->ntasks;
  if (map_out)
    for (int c = 0; c < spec->H * spec->W; ++c) map_out[c] = spec->rows[c] == '1';
  if (tasks_out)
    for (int t = 0; t < spec->ntasks; ++t)
      for (int k = 0; k < 4; ++k) tasks_out[4 * t + k] = spec->tasks[t][k];
  return OGBX_OK;
}

ogbx_status ogbx_maze_describe(ogbx_maze_t e, int32_t* map_h, int32_t* map_w, int32_t* num_tasks,
                               double* goal_tol, double* maze_unit) {
  OGBX_CHECK(e != nullptr, OGBX_EINVAL, "null handle");
  if (map_h) *map_h = e->P.H;
  if (map_w) *map_w = e->P.W;
  if (num_tasks) *num_tasks = e->P.num_tasks;
  if (goal_tol) *goal_tol = e->P.goal_tol;
  if (maze_unit) *maze_unit = e->P.pm.unit;
  return OGBX_OK;
}

ogbx_status ogbx_maze_tables(ogbx_maze_t e, int32_t* map_out, int32_t* tasks_out) {
  OGBX_CHECK(e != nullptr, OGBX_EINVAL, "null handle");
  if (map_out)
    for (int c = 0; c < e->P.H * e->P.W; ++c) map_out[c] = e->P.wall[c];
  if (tasks_out)
    for (int t = 0; t < e->P.num_tasks; ++t)
      for (int k = 0; k < 4; ++k) tasks_out[4 * t + k] = e->P.tasks[t][k];
  return OGBX_OK;
}

ogbx_status ogbx_maze_reset(ogbx_maze_t e, const int32_t* task_id, const double* task_xy,
                            const uint8_t* mask, const double* noise, double* obs, double* goal,
                            uint64_t seed, void* stream) {
  OGBX_CHECK(e != nullptr, OGBX_EINVAL, "null handle");
  OGBX_CHECK(obs != nullptr && goal != nullptr, OGBX_EINVAL, "ogbx_maze_reset: null output");
  OGBX_CHECK(e->P.loco_type != 1, OGBX_EINVAL, "ant handles reset through ogbx_antmaze_reset");
  OGBX_HIP(hipSetDevice(e->device));
  e->seed = seed;
  uint32_t k0, k1;
  seed_key(seed, kTagMazeReset, &k0, &k1);
  hipLaunchKernelGGL(maze_reset_kernel, dim3(grid_for(e->n, 256)), dim3(256), 0,
                     (hipStream_t)stream, e->Pd, e->S, e->n, task_id, task_xy, mask, noise, obs,
                     goal, k0, k1);
  OGBX_LAUNCHED("maze_reset_kernel");
  e->was_reset = true;
  return OGBX_OK;
}

}  // extern "C"

namespace {
// the launch of ogbx_maze_step / ogbx_maze_step_bound (arguments validated)
ogbx_status maze_step_launch(ogbx_maze_t e, const void* action, int32_t action_is_f64, int32_t k_steps, double* obs,
                             float* reward, uint8_t* terminated, uint8_t* truncated, uint8_t* success,
                             double* final_obs, int32_t auto_reset, void* stream) {
  OGBX_HIP(hipSetDevice(e->device));
  uint32_t k0, k1;
  seed_key(e->seed, kTagMazeReset, &k0, &k1);
  const int epw = e->epw;
  dim3 grid(grid_for(e->n * (64 / (epw & 0xFF)), kStepBlock)), block(kStepBlock);
  if (action_is_f64)
    hipLaunchKernelGGL((maze_step_kernel<true, false>), grid, block, e->lds_pad, (hipStream_t)stream, e->Pd, e->S,
                       e->n, action, k_steps, obs, reward, terminated, truncated, success,
                       final_obs, auto_reset, k0, k1, epw, nullptr);
  else
    hipLaunchKernelGGL((maze_step_kernel<false, false>), grid, block, e->lds_pad, (hipStream_t)stream, e->Pd, e->S,
                       e->n, action, k_steps, obs, reward, terminated, truncated, success,
                       final_obs, auto_reset, k0, k1, epw, nullptr);
  OGBX_LAUNCHED("maze_step_kernel");
  return OGBX_OK;
}
}  // namespace

extern "C" {

ogbx_status ogbx_maze_step(ogbx_maze_t e, const void* action, int32_t action_is_f64,
                           int32_t k_steps, double* obs, float* reward, uint8_t* terminated,
                           uint8_t* truncated, uint8_t* success, double* final_obs,
                           int32_t auto_reset, void* stream) {
  OGBX_CHECK(e != nullptr, OGBX_EINVAL, "null handle");
  OGBX_CHECK(e->was_reset, OGBX_ESTATE, "Cannot call env.step() before calling env.reset()");
  OGBX_CHECK(e->P.loco_type == 0, OGBX_EINVAL,
             "only the point-mass dynamics are implemented (ant/humanoid are wrapper-only)");
  OGBX_CHECK(action && obs && reward && terminated && truncated && success, OGBX_EINVAL,
             "ogbx_maze_step: null argument");
  OGBX_CHECK(k_steps >= 1, OGBX_EINVAL, "k_steps must be >= 1");
  return maze_step_launch(e, action, action_is_f64, k_steps, obs, reward, terminated, truncated, success, final_obs,
                          auto_reset, stream);
}

ogbx_status ogbx_maze_bind_step(ogbx_maze_t e, double* obs, float* reward, uint8_t* terminated, uint8_t* truncated,
                                uint8_t* success, double* final_obs, int32_t auto_reset) {
  OGBX_CHECK(e != nullptr, OGBX_EINVAL, "null handle");
  OGBX_CHECK(e->P.loco_type == 0 || e->P.loco_type == 1, OGBX_EINVAL,
             "ogbx_maze_bind_step: point handles (ogbx_maze_step_bound) or ant handles (ogbx_antmaze_step_bound)");
  OGBX_CHECK(obs && reward && terminated && truncated && success, OGBX_EINVAL, "ogbx_maze_bind_step: null output");
  e->b_obs = obs;
  e->b_reward = reward;
  e->b_term = terminated;
  e->b_trunc = truncated;
  e->b_succ = success;
  e->b_final = final_obs;
  e->b_auto = auto_reset;
  e->bound = true;
  return OGBX_OK;
}

ogbx_status ogbx_maze_step_bound(ogbx_maze_t e, const void* action, int32_t action_is_f64, void* stream) {
  OGBX_CHECK(e != nullptr && action != nullptr, OGBX_EINVAL, "ogbx_maze_step_bound: null argument");
  OGBX_CHECK(e->P.loco_type == 0, OGBX_EINVAL,
             "only the point-mass dynamics are implemented (ant/humanoid are wrapper-only)");
  OGBX_CHECK(e->bound, OGBX_ESTATE, "ogbx_maze_step_bound: no outputs bound (ogbx_maze_bind_step)");
  OGBX_CHECK(e->was_reset, OGBX_ESTATE, "Cannot call env.step() before calling env.reset()");
  return maze_step_launch(e, action, action_is_f64, 1, e->b_obs, e->b_reward, e->b_term, e->b_trunc, e->b_succ,
                          e->b_final, e->b_auto, stream);
}

ogbx_status ogbx_antmaze_state(ogbx_maze_t e, double** body_qpos, double** body_qvel) {
  OGBX_CHECK(e != nullptr, OGBX_EINVAL, "null handle");
  OGBX_CHECK(e->P.loco_type == 1, OGBX_EINVAL, "ogbx_antmaze_state: not an ant handle");
  if (body_qpos) *body_qpos = e->body_qpos;
  if (body_qvel) *body_qvel = e->body_qvel;
  return OGBX_OK;
}

ogbx_status ogbx_antmaze_reset(ogbx_maze_t e, const int32_t* task_id, const double* task_xy, const uint8_t* mask,
                               const double* noise, const double* body_draws, const double* goal_states,
                               double* obs, double* goal, double* goal_ob, uint64_t seed, void* stream) {
  OGBX_CHECK(e != nullptr, OGBX_EINVAL, "null handle");
  OGBX_CHECK(e->P.loco_type == 1, OGBX_EINVAL, "ogbx_antmaze_reset: not an ant handle");
  OGBX_CHECK(obs != nullptr && goal != nullptr, OGBX_EINVAL, "ogbx_antmaze_reset: null output");
  OGBX_HIP(hipSetDevice(e->device));
  e->seed = seed;
  uint32_t k0, k1;
  seed_key(seed, kTagMazeReset, &k0, &k1);
  hipLaunchKernelGGL(ant_reset_kernel, dim3(grid_for(e->n, 256)), dim3(256), 0, (hipStream_t)stream, e->Pd, e->S,
                     e->body_qpos, e->body_qvel, e->n, task_id, task_xy, mask, noise, body_draws, goal_states, obs,
                     goal, goal_ob, k0, k1);
  OGBX_LAUNCHED("ant_reset_kernel");
  e->was_reset = true;
  return OGBX_OK;
}

ogbx_status ogbx_antmaze_step_bound(ogbx_maze_t e, const double* qpos_post, const double* qvel_post,
                                    const double* reset_states, void* stream) {
  OGBX_CHECK(e != nullptr, OGBX_EINVAL, "null handle");
  OGBX_CHECK(e->bound, OGBX_ESTATE, "ogbx_antmaze_step_bound: no outputs bound (ogbx_maze_bind_step)");
  return ogbx_antmaze_step(e, qpos_post, qvel_post, e->b_obs, e->b_reward, e->b_term, e->b_trunc, e->b_succ,
                           e->b_final, e->b_auto, reset_states, stream);
}

ogbx_status ogbx_antmaze_step(ogbx_maze_t e, const double* qpos_post, const double* qvel_post, double* obs,
                              float* reward, uint8_t* terminated, uint8_t* truncated, uint8_t* success,
                              double* final_obs, int32_t auto_reset, const double* reset_states, void* stream) {
  OGBX_CHECK(e != nullptr, OGBX_EINVAL, "null handle");
  OGBX_CHECK(e->P.loco_type == 1, OGBX_EINVAL, "ogbx_antmaze_step: not an ant handle");
  OGBX_CHECK(e->was_reset, OGBX_ESTATE, "Cannot call env.step() before calling env.reset()");
  OGBX_CHECK(qpos_post && qvel_post && obs && reward && terminated && truncated && success, OGBX_EINVAL,
             "ogbx_antmaze_step: null argument");
  const bool qin = qpos_post == e->body_qpos, vin = qvel_post == e->body_qvel;
  OGBX_CHECK(qin == vin, OGBX_EINVAL, "ogbx_antmaze_step: qpos and qvel must both be (or both not be) the handle's state");
  OGBX_HIP(hipSetDevice(e->device));
  uint32_t k0, k1;
  seed_key(e->seed, kTagMazeReset, &k0, &k1);
  // 16-byte row words when every row pointer allows them
  const bool vec = ((reinterpret_cast<uintptr_t>(qpos_post) | reinterpret_cast<uintptr_t>(qvel_post) |
                     reinterpret_cast<uintptr_t>(obs) | reinterpret_cast<uintptr_t>(e->body_qpos) |
                     reinterpret_cast<uintptr_t>(e->body_qvel)) & 15u) == 0;
  hipLaunchKernelGGL(vec ? ant_step_kernel<true> : ant_step_kernel<false>, dim3(grid_for(e->n, kAntEnvs)),
                     dim3(kAntThreads), 0, (hipStream_t)stream, e->Pd, e->S, e->body_qpos, e->body_qvel, e->n,
                     qpos_post, qvel_post, (int32_t)qin, obs, reward, terminated, truncated, success, final_obs,
                     auto_reset, reset_states, k0, k1);
  OGBX_LAUNCHED("ant_step_kernel");
  return OGBX_OK;
}

ogbx_status ogbx_maze_rollout_until_done(ogbx_maze_t e, const void* action, int32_t action_is_f64,
                                         int32_t k_steps, double* obs, float* reward, uint8_t* terminated,
                                         uint8_t* truncated, uint8_t* success, int32_t* steps_taken,
                                         void* stream) {
  OGBX_CHECK(e != nullptr, OGBX_EINVAL, "null handle");
  OGBX_CHECK(e->was_reset, OGBX_ESTATE, "Cannot call env.step() before calling env.reset()");
  OGBX_CHECK(e->P.loco_type == 0, OGBX_EINVAL,
             "only the point-mass dynamics are implemented (ant/humanoid are wrapper-only)");
  OGBX_CHECK(action && obs && reward && terminated && truncated && success && steps_taken, OGBX_EINVAL,
             "ogbx_maze_rollout_until_done: null argument");
  OGBX_CHECK(k_steps >= 1, OGBX_EINVAL, "k_steps must be >= 1");
  OGBX_HIP(hipSetDevice(e->device));
  // Same Philox key as ogbx_maze_step: the teleport out-portal draw of a rollout row
  // must equal that of the single step it stands for.
  uint32_t k0, k1;
  seed_key(e->seed, kTagMazeReset, &k0, &k1);
  const int epw = e->epw;
  dim3 grid(grid_for(e->n * (64 / (epw & 0xFF)), kStepBlock)), block(kStepBlock);
  if (action_is_f64)
    hipLaunchKernelGGL((maze_step_kernel<true, true>), grid, block, e->lds_pad, (hipStream_t)stream, e->Pd, e->S,
                       e->n, action, k_steps, obs, reward, terminated, truncated, success, nullptr, 0, k0, k1,
                       epw, steps_taken);
  else
    hipLaunchKernelGGL((maze_step_kernel<false, true>), grid, block, e->lds_pad, (hipStream_t)stream, e->Pd, e->S,
                       e->n, action, k_steps, obs, reward, terminated, truncated, success, nullptr, 0, k0, k1,
                       epw, steps_taken);
  OGBX_LAUNCHED("maze_step_kernel");
  return OGBX_OK;
}

ogbx_status ogbx_maze_state(ogbx_maze_t e, double** qpos, double** goal_xy, int32_t** elapsed,
                            int32_t** task_id, uint32_t** episode) {
  OGBX_CHECK(e != nullptr, OGBX_EINVAL, "null handle");
  if (qpos) *qpos = e->S.qpos;
  if (goal_xy) *goal_xy = e->S.goal;
  if (elapsed) *elapsed = e->S.elapsed;
  if (task_id) *task_id = e->S.task;
  if (episode) *episode = e->S.episode;
  // A restore through these pointers counts as a reset.
  e->was_reset = true;
  return OGBX_OK;
}

ogbx_status ogbx_maze_set_seed(ogbx_maze_t e, uint64_t seed) {
  OGBX_CHECK(e != nullptr, OGBX_EINVAL, "null handle");
  e->seed = seed;
  return OGBX_OK;
}

ogbx_status ogbx_point_physics(ogbx_maze_t e, const double* qpos_in, const void* action,
                               int32_t action_is_f64, int64_t n, double* qpos_out,
                               uint8_t* contact_out, void* stream) {
  OGBX_CHECK(e != nullptr && qpos_in && action && qpos_out, OGBX_EINVAL, "null argument");
  if (n <= 0) return OGBX_OK;
  OGBX_HIP(hipSetDevice(e->device));
  const int epw = e->epw;
  dim3 grid(grid_for(n * (64 / (epw & 0xFF)), kStepBlock)), block(kStepBlock);
  if (action_is_f64)
    hipLaunchKernelGGL(point_physics_kernel<true>, grid, block, e->lds_pad, (hipStream_t)stream, e->Pd,
                       qpos_in, action, n, qpos_out, contact_out, epw);
  else
    hipLaunchKernelGGL(point_physics_kernel<false>, grid, block, e->lds_pad, (hipStream_t)stream, e->Pd,
                       qpos_in, action, n, qpos_out, contact_out, epw);
  OGBX_LAUNCHED("point_physics_kernel");
  return OGBX_OK;
}

ogbx_status ogbx_maze_xy_to_ij(ogbx_maze_t e, const double* xy, int64_t n, int32_t* ij,
                               void* stream) {
  OGBX_CHECK(e != nullptr && xy && ij, OGBX_EINVAL, "null argument");
  if (n <= 0) return OGBX_OK;
  OGBX_HIP(hipSetDevice(e->device));
  hipLaunchKernelGGL(xy_to_ij_kernel, dim3(grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream,
                     e->Pd, xy, n, ij);
  OGBX_LAUNCHED("xy_to_ij_kernel");
  return OGBX_OK;
}

ogbx_status ogbx_maze_ij_to_xy(ogbx_maze_t e, const int32_t* ij, int64_t n, double* xy,
                               void* stream) {
  OGBX_CHECK(e != nullptr && xy && ij, OGBX_EINVAL, "null argument");
  if (n <= 0) return OGBX_OK;
  OGBX_HIP(hipSetDevice(e->device));
  hipLaunchKernelGGL(ij_to_xy_kernel, dim3(grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream,
                     e->Pd, ij, n, xy);
  OGBX_LAUNCHED("ij_to_xy_kernel");
  return OGBX_OK;
}

ogbx_status ogbx_maze_oracle_subgoal(ogbx_maze_t e, const double* start_xy, const double* goal_xy,
                                     int64_t n, double* subgoal_xy, void* stream) {
  OGBX_CHECK(e != nullptr && start_xy && goal_xy && subgoal_xy, OGBX_EINVAL, "null argument");
  if (n <= 0) return OGBX_OK;
  OGBX_HIP(hipSetDevice(e->device));
  hipLaunchKernelGGL(oracle_subgoal_kernel, dim3(grid_for(n, 256)), dim3(256), 0,
                     (hipStream_t)stream, e->Pd, e->bfs, start_xy, goal_xy, n, subgoal_xy);
  OGBX_LAUNCHED("oracle_subgoal_kernel");
  return OGBX_OK;
}

ogbx_status ogbx_maze_expert_action(ogbx_maze_t e, const double* start_xy, const double* goal_xy, int64_t n,
                                   double noise, const double* normal, uint64_t seed, uint64_t call_index,
                                   double* action, void* stream) {
  OGBX_CHECK(e != nullptr && action, OGBX_EINVAL, "ogbx_maze_expert_action: null argument");
  OGBX_CHECK((start_xy && goal_xy) || n == e->n, OGBX_EINVAL,
             "ogbx_maze_expert_action: n must equal the batch size when reading the env state");
  if (n <= 0) return OGBX_OK;
  OGBX_HIP(hipSetDevice(e->device));
  uint32_t k0, k1;
  seed_key(seed, kTagMazeExpert, &k0, &k1);
  hipLaunchKernelGGL(expert_action_kernel, dim3(grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream, e->Pd,
                     e->bfs, start_xy ? start_xy : e->S.qpos, goal_xy ? goal_xy : e->S.goal, n, noise, normal, k0,
                     k1, (uint32_t)call_index, (uint32_t)(call_index >> 32), action);
  OGBX_LAUNCHED("expert_action_kernel");
  return OGBX_OK;
}

ogbx_status ogbx_maze_set_goal(ogbx_maze_t e, const int32_t* goal_ij, const uint8_t* mask, const double* noise,
                               uint64_t seed, uint64_t call_index, void* stream) {
  OGBX_CHECK(e != nullptr && goal_ij, OGBX_EINVAL, "ogbx_maze_set_goal: null argument");
  OGBX_HIP(hipSetDevice(e->device));
  uint32_t k0, k1;
  seed_key(seed, kTagMazeGoal, &k0, &k1);
  hipLaunchKernelGGL(set_goal_kernel, dim3(grid_for(e->n, 256)), dim3(256), 0, (hipStream_t)stream, e->Pd, e->S,
                     e->n, goal_ij, mask, noise, k0, k1, (uint32_t)call_index, (uint32_t)(call_index >> 32));
  OGBX_LAUNCHED("set_goal_kernel");
  return OGBX_OK;
}

}  // extern "C"
