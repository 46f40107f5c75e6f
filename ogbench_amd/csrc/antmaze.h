// antmaze.h -- the antmaze wrapper (loco_type 'ant') around caller-supplied
// ant physics: the maze layer of the reference's MazeEnv (ogbench/locomaze/
// maze.py:373-466) at the AntEnv state layout (ogbench/locomaze/ant.py:69-122),
// batched over N envs.  Included by locomaze.hip (MazeParams, MazeState,
// reset_draws, reset_one, goal_reached).
//
// State in HBM per env: body qpos f64[15] (free joint xyz + quat, 8 hinges)
// and qvel f64[14] (the ant's nq/nv, ant.xml), plus the maze state shared with
// the point env (goal, elapsed, task, episode, and xy = get_xy() after the last
// step, which 'pre' success timing reads).  The articulated dynamics
// (AntEnv.do_simulation -> mj_step x5) are NOT here: the caller's physics
// engine advances the body state and hands the post-physics state to
// ogbx_antmaze_step, which does everything MazeEnv.step + TimeLimit do with it:
//   ob = concat(qpos, qvel)                         (ant.py:97-101, before any teleport)
//   success = |qpos[:2] - goal| <= 0.5 (fma norm)   (maze.py:86,486-490; pre or post)
//   teleport: qpos[:2] := a Philox-drawn out-portal (maze.py:442-451)
//   terminated = success & terminate_at_goal; reward = success (-1 single-task)
//   truncated = (++elapsed >= max_episode_steps)    (gymnasium TimeLimit)
//   optional same-step auto-reset (below).
// Reset (maze.py:373-431 with AntEnv.reset_model, ant.py:103-111): the
// returned ob is the second reset's state, qpos = init_qpos + U(-0.1, 0.1)^15,
// qvel = 0.1 N(0,1)^14, then set_xy(init_xy) -- no physics.  info['goal'] is
// the goal OBSERVATION (maze.py:407-418): the body state after the first reset
// and 5 random-action physics steps, with set_xy(goal_xy).  Those steps are the
// caller's physics, so the caller hands that state in (goal_states [N,29]) and
// the kernel writes it with qpos[:2] := goal_xy; without it, the first
// reset_model state (Philox, its own counter slots) stands in for the stepped
// one.  The oracle representation (use_oracle_rep) is the goal xy.
// The body draws come from Philox (tag kTagAntBody) or from the caller:
// injected draws [N,29] (parity) or whole reset states [N,29] produced by the
// caller's own physics reset (auto-reset), whose xy is then set to init_xy.
#pragma once

namespace ogbx {

constexpr int kAntNq = 15, kAntNv = 14, kAntOb = kAntNq + kAntNv;
constexpr uint32_t kTagAntBody = 0x414E0001u;

// ant.xml qpos0: torso at (0, 0, 0.75), unit quaternion, hinges at 0.
__device__ __forceinline__ double ant_init_qpos(int c) {
  return c == 2 ? 0.75 : (c == 3 ? 1.0 : 0.0);
}

// The c-th body draw of env gi's episode ep: c < 15 -> uniform(-0.1, 0.1),
// c >= 15 -> standard normal (Box-Muller on two Philox uniforms).
// slot: 0x300 for the reset_model that sets the returned ob, 0x340 for the
// first (goal) reset_model of MazeEnv.reset.
__device__ inline double ant_body_draw(uint64_t gi, uint32_t ep, int c, uint32_t k0, uint32_t k1,
                                      uint32_t slot = 0x300u) {
  const u32x4 w = philox4x32_10({(uint32_t)gi, ep, slot + (uint32_t)c, (uint32_t)(gi >> 32)}, k0 ^ kTagAntBody, k1);
  const double u0 = u01_from(w.x, w.y), u1 = u01_from(w.z, w.w);
  if (c < kAntNq) return -0.1 + 0.2 * u0;
  const double r = sqrt(-2.0 * log1p(-u0));  // 1 - u0 in (0, 1]
  return r * cospi(2.0 * u1);
}

// One env's reset body state into q[15], v[14] with xy := (x, y).
// draws: injected [29] (uniform(-0.1,0.1) x15, N(0,1) x14) or NULL (Philox);
// states: a whole caller reset state [29] (qpos, qvel) or NULL.
__device__ inline void ant_reset_body(uint64_t gi, uint32_t ep, uint32_t k0, uint32_t k1, const double* draws,
                                      const double* states, double x, double y, double* q, double* v) {
  for (int c = 0; c < kAntNq; ++c)
    q[c] = states ? states[c] : ant_init_qpos(c) + (draws ? draws[c] : ant_body_draw(gi, ep, c, k0, k1));
  for (int c = 0; c < kAntNv; ++c) {
    const int d = kAntNq + c;
    v[c] = states ? states[d] : 0.0 + 0.1 * (draws ? draws[d] : ant_body_draw(gi, ep, d, k0, k1));
  }
  q[0] = x;  // set_xy(init_xy) (ant.py:118-122)
  q[1] = y;
}

// MazeEnv.reset for ant handles.  One lane per env; row writes are strided
// (reset is off the step path).
__global__ void __launch_bounds__(256) ant_reset_kernel(const MazeParams* __restrict__ Pp, MazeState S,
                                                        double* __restrict__ bq, double* __restrict__ bv, int64_t n,
                                                        const int32_t* task_id, const double* task_xy,
                                                        const uint8_t* mask, const double* noise,
                                                        const double* body_draws, const double* goal_states,
                                                        double* obs, double* goal_out, double* goal_ob,
                                                        uint32_t k0, uint32_t k1) {
  const MazeParams& P = *Pp;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (mask != nullptr && mask[i] == 0) return;
  const uint32_t ep = S.episode[i] + 1u;
  const uint64_t gi = (uint64_t)(i + P.env_base);
  int32_t task;
  if (P.reward_task_id > 0) task = P.reward_task_id;
  else if (task_id != nullptr) task = task_id[i];
  else task = draw_task(P, gi, ep, k0, k1);
  if (task < 1 || task > P.num_tasks) task = 1;
  double r[4];
  if (noise != nullptr) {
    for (int k = 0; k < 4; ++k) r[k] = noise[4 * i + k];
  } else {
    reset_draws(gi, ep, k0, k1, r);
  }
  double x, y, gx, gy;
  reset_one(P, task, task_xy ? task_xy + 4 * i : nullptr, r, x, y, gx, gy);
  double q[kAntNq], v[kAntNv];
  ant_reset_body(gi, ep, k0, k1, body_draws ? body_draws + (int64_t)kAntOb * i : nullptr, nullptr, x, y, q, v);
  for (int c = 0; c < kAntNq; ++c) {
    bq[kAntNq * i + c] = q[c];
    obs[kAntOb * i + c] = q[c];
  }
  for (int c = 0; c < kAntNv; ++c) {
    bv[kAntNv * i + c] = v[c];
    obs[kAntOb * i + kAntNq + c] = v[c];
  }
  S.qpos[2 * i] = x;
  S.qpos[2 * i + 1] = y;
  S.goal[2 * i] = gx;
  S.goal[2 * i + 1] = gy;
  S.elapsed[i] = 0;
  S.task[i] = task;
  S.episode[i] = ep;
  goal_out[2 * i] = gx;
  goal_out[2 * i + 1] = gy;
  if (goal_ob != nullptr) {
    // get_ob() after the goal reset's random steps and set_xy(goal_xy)
    double* g = goal_ob + (int64_t)kAntOb * i;
    const double* gs = goal_states ? goal_states + (int64_t)kAntOb * i : nullptr;
    for (int c = 0; c < kAntOb; ++c) {
      double val;
      if (gs) val = gs[c];
      else if (c < kAntNq) val = ant_init_qpos(c) + ant_body_draw(gi, ep, c, k0, k1, 0x340u);
      else val = 0.0 + 0.1 * ant_body_draw(gi, ep, c, k0, k1, 0x340u);
      g[c] = c == 0 ? gx : (c == 1 ? gy : val);
    }
  }
}

// Row kinds decided in phase A of ant_step_kernel.
constexpr uint8_t kRowPlain = 0, kRowTeleport = 1, kRowReset = 2;
// 64 envs per 256-thread block: phase A on the first wave, phase B's
// 64 x 29 elements spread over all four (8 per thread), so a launch at the
// 16,384 envs of one 8-GPU share has 1,024 waves with short streams.
constexpr int kAntEnvs = 64, kAntThreads = 256;
constexpr int kAntPer = (kAntEnvs * kAntOb + kAntThreads - 1) / kAntThreads;

// One wrapper step of kAntEnvs envs per block.
//   phase B (the block's [64 x 29] obs rows as one flat range): every row is
//     first written as the plain row -- ob = the post-physics (qpos, qvel)
//     row, coalesced, and the body state the same row unless the caller
//     stepped it in place -- as soon as its loads return, with no wait for
//     phase A;
//   phase A (one lane per env, first wave, meanwhile): success / teleport /
//     TimeLimit / reward and flags;
//   after one barrier the first wave overwrites the rows phase A changed:
//     a teleport's body xy, an auto-reset's whole rows (rare).  The barrier
//     orders those writes after the plain ones of the other waves.
// kVec (every row pointer 16-byte aligned, the host checks): phase B moves
// the block's qpos / qvel ranges as 16-byte words -- loads, and the body
// state stores straight from them -- and assembles the obs rows in LDS,
// stored as 16-byte words after the barrier; phase A runs before that
// barrier and leaves each env's row kind in LDS, so the plain obs stores
// skip the auto-reset rows and need no second barrier.
typedef double AntD2 __attribute__((ext_vector_type(2)));
// one 16-byte streaming store (p 16-byte aligned)
__device__ __forceinline__ void ant_nt_store2(double* p, double2 v) {
  const AntD2 w = {v.x, v.y};
  __builtin_nontemporal_store(w, reinterpret_cast<AntD2*>(p));
}

template <bool kVec>
__global__ void __launch_bounds__(kAntThreads) ant_step_kernel(
    const MazeParams* __restrict__ Pp, MazeState S, double* __restrict__ bq, double* __restrict__ bv, int64_t n,
    const double* __restrict__ qpost, const double* __restrict__ vpost, int32_t in_place,
    double* __restrict__ obs, float* __restrict__ reward, uint8_t* __restrict__ terminated,
    uint8_t* __restrict__ truncated, uint8_t* __restrict__ success, double* __restrict__ final_obs,
    int32_t auto_reset, const double* __restrict__ reset_states, uint32_t k0, uint32_t k1) {
  const MazeParams& P = *Pp;
  const int64_t base = (int64_t)blockIdx.x * kAntEnvs;
  const int nb = (int)(n - base < (int64_t)kAntEnvs ? n - base : (int64_t)kAntEnvs);
  const int tot = nb * kAntOb;
  // block-local rows (32-bit offsets from here on)
  const double* qb = qpost + kAntNq * base;
  const double* vb = vpost + kAntNv * base;
  double* ob = obs + kAntOb * base;
  double* bqb = bq + kAntNq * base;
  double* bvb = bv + kAntNv * base;
  double val[kAntPer];
  // kVec: word j of the block's qpos (qvel) range holds elements 2j, 2j + 1
  constexpr int kQW = (kAntEnvs * kAntNq / 2 + kAntThreads - 1) / kAntThreads;
  constexpr int kVW = (kAntEnvs * kAntNv / 2 + kAntThreads - 1) / kAntThreads;
  const int nq = nb * kAntNq, nv = nb * kAntNv;  // nv is even
  double2 qw[kQW], vw[kVW];
  __shared__ double rows[kAntEnvs * kAntOb];
  __shared__ uint8_t kinds[kAntEnvs];
  if constexpr (!kVec) {
#pragma unroll
    for (int r = 0; r < kAntPer; ++r) {
      const int f = (int)threadIdx.x + kAntThreads * r;
      const int e = f / kAntOb, c = f - e * kAntOb;
      val[r] = 0.0;
      if (f < tot) val[r] = c < kAntNq ? qb[kAntNq * e + c] : vb[kAntNv * e + (c - kAntNq)];
    }
  } else {
#pragma unroll
    for (int r = 0; r < kQW; ++r) {
      const int j = (int)threadIdx.x + kAntThreads * r;
      qw[r] = make_double2(0.0, 0.0);
      if (2 * j + 1 < nq)
        qw[r] = reinterpret_cast<const double2*>(qb)[j];
      else if (2 * j < nq)
        qw[r].x = qb[2 * j];
    }
#pragma unroll
    for (int r = 0; r < kVW; ++r) {
      const int j = (int)threadIdx.x + kAntThreads * r;
      vw[r] = make_double2(0.0, 0.0);
      if (2 * j < nv) vw[r] = reinterpret_cast<const double2*>(vb)[j];
    }
  }
  const int64_t i = base + threadIdx.x;
  const bool lane_a = threadIdx.x < kAntEnvs && i < n;
  // phase A's loads, issued before any of this thread's stores
  double2 g = make_double2(0.0, 0.0), pre = g;
  double px = 0.0, py = 0.0;
  int32_t el = 0;
  if (lane_a) {
    g = reinterpret_cast<const double2*>(S.goal)[i];
    px = qpost[kAntNq * i];
    py = qpost[kAntNq * i + 1];
    el = S.elapsed[i];
    // pre timing: the xy the previous step (or reset) left, kept in S.qpos
    // because an in-place physics engine has already overwritten the body
    pre = P.success_pre ? reinterpret_cast<const double2*>(S.qpos)[i] : make_double2(px, py);
  }
  // phase B: the plain rows
#pragma unroll
  for (int r = 0; r < (kVec ? 0 : kAntPer); ++r) {
    const int f = (int)threadIdx.x + kAntThreads * r;
    if (f >= tot) continue;
    const int e = f / kAntOb, c = f - e * kAntOb;
    // non-temporal: nothing in this launch reads the rows back, and streaming
    // stores leave less for the end-of-kernel write-back (A/B: 5.24 -> 4.78 us
    // per launch at 16,384 envs)
    __builtin_nontemporal_store(val[r], &ob[f]);
    if (in_place) continue;
    if (c < kAntNq)
      __builtin_nontemporal_store(val[r], &bqb[kAntNq * e + c]);
    else
      __builtin_nontemporal_store(val[r], &bvb[kAntNv * e + (c - kAntNq)]);
  }
  uint8_t kind = kRowPlain;
  double nx = px, ny = py;
  if (lane_a) {
    const bool succ = goal_reached(pre.x, pre.y, g.x, g.y, P.goal_tol);
    if (P.n_tp_in > 0) {
      for (int t = 0; t < P.n_tp_in; ++t) {
        if (goal_reached(px, py, P.tp_in[t][0], P.tp_in[t][1], P.tp_radius * 1.5)) {
          const uint64_t gi = (uint64_t)(i + P.env_base);
          const uint32_t ep = S.episode[i];
          const u32x4 c = philox4x32_10({(uint32_t)gi, ep, 0x100u + (uint32_t)el, (uint32_t)(gi >> 32)},
                                        k0 ^ kTagMazeTeleport, k1);
          const int o = (int)bounded_u32(c.x, (uint32_t)P.n_tp_out);
          nx = P.tp_out[o][0];
          ny = P.tp_out[o][1];
          kind = kRowTeleport;
          break;
        }
      }
    }
    float rew = succ ? 1.0f : 0.0f;
    if (P.reward_task_id > 0) rew -= 1.0f;
    const bool term = succ && P.terminate_at_goal;
    el += 1;
    const bool trunc = el >= P.max_steps;
    reward[i] = rew;
    terminated[i] = term;
    truncated[i] = trunc;
    success[i] = succ;
    if (auto_reset && (term || trunc)) kind = kRowReset;
  }
  if constexpr (kVec) {
    // body state from the loaded words; obs rows assembled in LDS
#pragma unroll
    for (int r = 0; r < kQW; ++r) {
      const int j = (int)threadIdx.x + kAntThreads * r;
      if (2 * j >= nq) continue;
      const bool two = 2 * j + 1 < nq;
      if (!in_place) {
        if (two)
          ant_nt_store2(&bqb[2 * j], qw[r]);
        else
          __builtin_nontemporal_store(qw[r].x, &bqb[2 * j]);
      }
      const int e0 = (2 * j) / kAntNq, c0 = 2 * j - e0 * kAntNq;
      rows[kAntOb * e0 + c0] = qw[r].x;
      if (two) {
        const int e1 = (2 * j + 1) / kAntNq, c1 = 2 * j + 1 - e1 * kAntNq;
        rows[kAntOb * e1 + c1] = qw[r].y;
      }
    }
#pragma unroll
    for (int r = 0; r < kVW; ++r) {
      const int j = (int)threadIdx.x + kAntThreads * r;
      if (2 * j >= nv) continue;
      if (!in_place) ant_nt_store2(&bvb[2 * j], vw[r]);
      const int e0 = (2 * j) / kAntNv, c0 = 2 * j - e0 * kAntNv;  // 2j, 2j + 1: one row (kAntNv even)
      rows[kAntOb * e0 + kAntNq + c0] = vw[r].x;
      rows[kAntOb * e0 + kAntNq + c0 + 1] = vw[r].y;
    }
    if (threadIdx.x < kAntEnvs) kinds[threadIdx.x] = kind;
    __syncthreads();  // rows and kinds complete; the body stores above precede the overwrites below
    // plain obs rows as 16-byte words (a word may span two rows: both must
    // be plain; the auto-reset rows are written whole below)
    for (int j = (int)threadIdx.x; 2 * j < tot; j += kAntThreads) {
      const int e0 = (2 * j) / kAntOb, e1 = (2 * j + 1) / kAntOb;
      const bool p0 = kinds[e0] != kRowReset, p1 = 2 * j + 1 < tot && kinds[e1] != kRowReset;
      if (p0 && p1)
        ant_nt_store2(&ob[2 * j], reinterpret_cast<const double2*>(rows)[j]);
      else {
        if (p0) __builtin_nontemporal_store(rows[2 * j], &ob[2 * j]);
        if (p1) __builtin_nontemporal_store(rows[2 * j + 1], &ob[2 * j + 1]);
      }
    }
  } else {
    __syncthreads();  // the plain rows above are written before the overwrites below
  }
  if (lane_a) {
    if (kind == kRowReset) {
      if (final_obs != nullptr) {  // the pre-reset observation
        for (int c = 0; c < kAntNq; ++c) final_obs[kAntOb * i + c] = qpost[kAntNq * i + c];
        for (int c = 0; c < kAntNv; ++c) final_obs[kAntOb * i + kAntNq + c] = vpost[kAntNv * i + c];
      }
      const uint64_t gi = (uint64_t)(i + P.env_base);
      const uint32_t ep = S.episode[i] + 1u;
      const int32_t task = S.task[i];
      double r[4];
      reset_draws(gi, ep, k0, k1, r);
      double x, y, gx, gy;
      reset_one(P, task, nullptr, r, x, y, gx, gy);
      double q[kAntNq], v[kAntNv];
      ant_reset_body(gi, ep, k0, k1, nullptr, reset_states ? reset_states + (int64_t)kAntOb * i : nullptr, x, y,
                     q, v);
      for (int c = 0; c < kAntNq; ++c) {
        bq[kAntNq * i + c] = q[c];
        obs[kAntOb * i + c] = q[c];
      }
      for (int c = 0; c < kAntNv; ++c) {
        bv[kAntNv * i + c] = v[c];
        obs[kAntOb * i + kAntNq + c] = v[c];
      }
      reinterpret_cast<double2*>(S.goal)[i] = make_double2(gx, gy);
      S.episode[i] = ep;
      el = 0;
      nx = x;
      ny = y;
    } else if (kind == kRowTeleport) {
      bq[kAntNq * i] = nx;  // set_xy on the body
      bq[kAntNq * i + 1] = ny;
    }
    reinterpret_cast<double2*>(S.qpos)[i] = make_double2(nx, ny);  // get_xy()
    S.elapsed[i] = el;
  }
}

}  // namespace ogbx
