/*
 * ogbx.h -- C-ABI of the MI355X-native OGBench hot path (libogbx.so, gfx950).
 *
 * This header is the drop-in boundary. Every entry point replaces one reference
 * interface; the reference file:line it stands in for is cited next to it
 * (paths relative to hliuson/ogbench).  Types are plain C: device pointers,
 * sizes, an opaque handle and a hipStream_t passed as `void*`.  No torch types
 * cross this boundary; the Python layer (ogbench_amd/) passes
 * `tensor.data_ptr()` and `torch.cuda.current_stream().cuda_stream`.
 *
 * Conventions (all entry points):
 *   - Every call returns an ogbx_status; on failure ogbx_last_error() holds a
 *     thread-local message.  Status codes never become exceptions here; the
 *     Python layer raises ValueError/AssertionError/RuntimeError exactly where
 *     the reference does (maze.py:29,163,347,379,384).
 *   - All I/O buffers are caller-owned DEVICE memory.  A handle owns only its
 *     static tables (maze map, task table, goal worlds), its per-env state and
 *     its RNG counters.
 *   - Calls are asynchronous on `stream`; nothing synchronises the host except
 *     the explicit *_sync / *_read_state helpers.
 *   - One handle per (device, stream) at a time; distinct handles are
 *     independent, so one process may drive several GPUs.
 *   - There is no CPU fallback: a handle can only be created on a visible
 *     gfx950 device, otherwise OGBX_EDEVICE.
 */
#ifndef OGBX_H
#define OGBX_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* History: 4 = rounds 1-3; 5 adds ogbx_gc_sample_ahead, ogbx_hgc_sample_ahead,
 * ogbx_maze_set_seed, ogbx_powder_set_seed, ogbx_stream_version,
 * ogbx_powder_state_view, ogbx_powder_state_written, ogbx_powder_set_phase
 * and the sampler plans ogbx_gc_plan_* (no entry point of 4 changed its
 * signature or meaning). */
#define OGBX_ABI_VERSION 5

typedef enum {
  OGBX_OK = 0,
  OGBX_EINVAL = -1,  /* bad argument (reference: ValueError / AssertionError) */
  OGBX_EDEVICE = -2, /* HIP runtime error or no gfx950 device */
  OGBX_ENOMEM = -3,  /* device allocation failed */
  OGBX_ESTATE = -4   /* handle used in the wrong state (e.g. step before reset) */
} ogbx_status;

/* Thread-local message describing the last failure of this thread. */
const char* ogbx_last_error(void);
/* OGBX_ABI_VERSION of the loaded library. */
int32_t ogbx_abi_version(void);

/* Version of the Philox random streams: which counter words feed which draw.
 * The same seed reproduces a run only between libraries with the same stream
 * version (tests/test_stream_pin_gpu.py pins the outputs of every Philox
 * consumer at this version).  History: 1 = rounds 1-2; 2 = powderworld
 * medium/hard rand fields from three Philox calls per group of four cells
 * (all 12 words used), where version 1 took one call per cell. */
#define OGBX_STREAM_VERSION 2
/* OGBX_STREAM_VERSION of the loaded library. */
int32_t ogbx_stream_version(void);
/* Name of the GPU architecture the library was built for ("gfx950"). */
const char* ogbx_build_arch(void);

/* ======================================================================
 * Locomaze (pointmaze) batched environment
 * ====================================================================== */

typedef struct ogbx_maze_env* ogbx_maze_t;

/* Static options of a batch of MazeEnv instances.
 * Reference: MazeEnv.__init__ kwargs, ogbench/locomaze/maze.py:37-86, and the
 * registry kwargs in ogbench/locomaze/__init__.py:10-13,16-35,248-275. */
typedef struct {
  int32_t loco_type;         /* 0 = point (PointEnv dynamics, point.py:64-95).
                                1 = ant, 2 = humanoid: wrapper only (goal/time/
                                reward logic, maze.py:433-466); dynamics are out
                                of scope and such handles reject step(). */
  int32_t success_timing;    /* 0 = 'post' (default, maze.py:43), 1 = 'pre'. */
  int32_t terminate_at_goal; /* maze.py:42, default 1. */
  int32_t add_noise_to_goal; /* maze.py:45, default 1 (0 for singletask). */
  int32_t reward_task_id;    /* -1 = goal-conditioned (None); 0 => default task 1
                                (maze.py:361-362); 1..num_tasks single-task. */
  int32_t max_episode_steps; /* TimeLimit, locomaze/__init__.py:20 (1000). */
  int64_t env_base;          /* Global index of env 0 of this handle.  Every
                                Philox stream (reset noise, task draws, teleport
                                out-portal, expert noise, set_goal noise) is
                                counted by the GLOBAL env index env_base + i, so
                                G ranks holding envs [r*N/G, (r+1)*N/G) with one
                                shared seed reproduce the single-GPU run of N
                                envs bit for bit.  0 = unsharded.
                                Any boundary works: every contact-solver choice
                                is made per env, so results do not depend on
                                which envs share a wavefront (multiples of 64
                                envs keep the wavefronts full;
                                ogbench_amd.sharding.shard aligns to 64). */
} ogbx_maze_opts;

/* Create a batch of `n_envs` maze envs on `device`.
 * maze_type: "arena" | "medium" | "large" | "giant" | "teleport"
 * (maze.py:90-163; anything else -> OGBX_EINVAL, reference ValueError at :163).
 * Replaces: make_maze_env(...) + gymnasium.make (maze.py:13-218). */
ogbx_status ogbx_maze_create(const char* maze_type, int64_t n_envs, int32_t device,
                             const ogbx_maze_opts* opts, ogbx_maze_t* out);
ogbx_status ogbx_maze_destroy(ogbx_maze_t env);
/* Number of envs of the handle. */
int64_t ogbx_maze_num_envs(ogbx_maze_t env);
/* Launch shape of the step/physics kernels: envs carried per 64-lane wave
 * (8, 16, 32 or 64; default 64), optionally | OGBX_EPW_REPLICATE: the wave's
 * other lanes then step copies of its epw envs (only the first copy stores)
 * instead of idling.  Performance knob only: every choice of the contact path
 * is made per lane, so results are bit-identical across layouts (DESIGN.md
 * section 4.1; tests/test_locomaze_gpu.py). */
#define OGBX_EPW_REPLICATE 0x100
ogbx_status ogbx_maze_set_envs_per_wave(ogbx_maze_t env, int32_t epw);

/* Static description: H, W of the map, number of tasks, goal_tol
 * (maze.py:86: 1.0 point / 0.5 ant+humanoid), maze_unit (4.0). */
ogbx_status ogbx_maze_describe(ogbx_maze_t env, int32_t* map_h, int32_t* map_w,
                               int32_t* num_tasks, double* goal_tol, double* maze_unit);
/* Copy the map (row-major int32 [H*W], 1 = wall) and the task table
 * (int32 [num_tasks*4] = init_i, init_j, goal_i, goal_j; maze.py:308-359)
 * to HOST buffers. Either pointer may be NULL. */
ogbx_status ogbx_maze_tables(ogbx_maze_t env, int32_t* map_out, int32_t* tasks_out);

/* Device-free query of the static maze tables (used by host-side checks):
 * map_h/map_w/num_tasks out; map_out int32[H*W] and tasks_out int32[num_tasks*4]
 * may be NULL (query sizes first).  Unknown maze_type -> OGBX_EINVAL. */
ogbx_status ogbx_maze_static_tables(const char* maze_type, int32_t* map_h, int32_t* map_w,
                                    int32_t* num_tasks, int32_t* map_out, int32_t* tasks_out);

/* Reset the envs selected by `mask` (device u8[N]; NULL = all).
 * Reference: MazeEnv.reset, maze.py:373-431 (+ PointEnv.set_xy point.py:111-115).
 *   task_id  device i32[N], values in 1..num_tasks; NULL = keep/draw: a single-
 *            task handle always uses reward_task_id; otherwise NULL draws a
 *            uniform task from the Philox stream (maze.py:391-394).
 *            Values are validated by the caller (the Python layer raises the
 *            reference AssertionError); out-of-range values fall back to 1.
 *   task_xy  device f64[N,4] (init_x, init_y, goal_x, goal_y) or NULL; when given
 *            it replaces the task table, i.e. options['task_info'] (maze.py:387-
 *            390) with the cell centres already converted by ij_to_xy.
 *   noise    device f64[N,4] = the four np.random.uniform(-1,1) draws in reset
 *            order (init x, init y, goal x, goal y; maze.py:402-405,564-567) or
 *            NULL = draw them from Philox4x32-10 keyed by (seed, env index,
 *            episode counter).
 *   obs      device f64[N,2] out (ob = init_xy), goal device f64[N,2] out
 *            (info['goal'] = goal_xy, maze.py:416-427).  Rows of masked-out envs
 *            are left untouched. */
ogbx_status ogbx_maze_reset(ogbx_maze_t env, const int32_t* task_id, const double* task_xy,
                            const uint8_t* mask, const double* noise, double* obs, double* goal,
                            uint64_t seed, void* stream);

/* Step all N envs `k_steps` times with actions device [k_steps, N, 2]
 * (float32 if action_is_f64 == 0, float64 otherwise) in ONE launch.
 * Reference per step: TimeLimit -> MazeEnv.step (maze.py:433-466) ->
 * PointEnv.step (point.py:64-95) -> mujoco.mj_step(nstep=5) (point.py:73).
 * Outputs are [k_steps, N] rows (obs [k_steps, N, 2]):
 *   obs f64, reward f32 (1/0, or -1/0 single-task), terminated/truncated/
 *   success u8.  final_obs (nullable) receives the pre-reset observation of envs
 *   that auto-reset at that step (gymnasium same-step autoreset).
 * auto_reset != 0: envs that end (terminated|truncated) are reset in the same
 *   step with Philox noise (seed given at the last ogbx_maze_reset) keeping
 *   their task; obs then holds the new initial observation. */
ogbx_status ogbx_maze_step(ogbx_maze_t env, const void* action, int32_t action_is_f64,
                           int32_t k_steps, double* obs, float* reward, uint8_t* terminated,
                           uint8_t* truncated, uint8_t* success, double* final_obs,
                           int32_t auto_reset, void* stream);

/* The steady per-step call of a host that reuses its output buffers (the
 * Gymnasium surface returns the same tensors every step): bind the outputs
 * and the auto-reset flag once, then step with the action and the stream
 * only.  ogbx_maze_step_bound(env, a, f64, s) == ogbx_maze_step(env, a, f64, 1,
 * <bound outputs>, s); a new bind replaces the old one.  Ant handles bind the
 * same way (obs f64[N,29]) for ogbx_antmaze_step_bound (below). */
ogbx_status ogbx_maze_bind_step(ogbx_maze_t env, double* obs, float* reward, uint8_t* terminated,
                                uint8_t* truncated, uint8_t* success, double* final_obs, int32_t auto_reset);
ogbx_status ogbx_maze_step_bound(ogbx_maze_t env, const void* action, int32_t action_is_f64, void* stream);

/* ---- antmaze wrapper (loco_type 1): the maze layer around caller-supplied
 * ant physics.  The ant's articulated dynamics (AntEnv.do_simulation ->
 * mujoco.mj_step x5, ogbench/locomaze/ant.py:69-95) are out of scope: the
 * caller's physics engine advances the body state; these entry points do what
 * MazeEnv.reset / MazeEnv.step + TimeLimit do around it (maze.py:373-466) at
 * the AntEnv layout (qpos f64[15], qvel f64[14], ob = concat(qpos, qvel) f64[29],
 * xy = qpos[:2], goal_tol 0.5; ant.py:97-122, maze.py:86).  Wrapper parity is
 * pinned by the reference's own methods (tests/golden/antmaze_golden.npz);
 * ant dynamics are unpinned and not implemented. */

/* The handle's body state: device f64[N,15] qpos and f64[N,14] qvel, the
 * buffers an in-place physics engine reads and overwrites each step. */
ogbx_status ogbx_antmaze_state(ogbx_maze_t env, double** body_qpos, double** body_qvel);

/* MazeEnv.reset for an ant handle (maze.py:373-431): task / init_xy / goal_xy
 * exactly as ogbx_maze_reset (same task_id, task_xy, mask, noise and seed
 * semantics); body = AntEnv.reset_model (ant.py:103-111): qpos = qpos0 +
 * uniform(-0.1, 0.1)^15, qvel = 0.1 * normal^14, then set_xy(init_xy).
 *   body_draws  device f64[N,29] = the 15 uniform(-0.1,0.1) and 14 standard
 *               normal draws in reset_model order, or NULL = Philox.
 *   goal_states device f64[N,29] (qpos, qvel) = the body state the caller's
 *               physics reached after the reference's goal reset and its 5
 *               random-action steps (maze.py:408-413), or NULL: the goal
 *               reset's reset_model state (Philox) stands in, unstepped.
 *   obs         device f64[N,29] out; goal device f64[N,2] out = the goal xy
 *               (cur_goal_xy; info['goal'] under use_oracle_rep, maze.py:482-484).
 *   goal_ob     device f64[N,29] out (nullable) = info['goal'], the goal
 *               observation: goal_states with qpos[:2] := goal xy
 *               (set_xy + get_ob, maze.py:416-418, ant.py:97-122). */
ogbx_status ogbx_antmaze_reset(ogbx_maze_t env, const int32_t* task_id, const double* task_xy,
                               const uint8_t* mask, const double* noise, const double* body_draws,
                               const double* goal_states, double* obs, double* goal, double* goal_ob,
                               uint64_t seed, void* stream);

/* MazeEnv.step + TimeLimit for an ant handle, given the post-physics state
 * qpos_post f64[N,15] / qvel_post f64[N,14] -- either the handle's own state
 * (ogbx_antmaze_state, stepped in place by the physics engine) or separate
 * buffers (copied into the handle's state).  Outputs [N]: obs f64[N,29] (the
 * post-physics ob, taken before a teleport), reward f32, terminated /
 * truncated / success u8; success on qpos[:2] (post, or the previous xy for
 * success_timing 'pre').  Teleport mazes move qpos[:2] as ogbx_maze_step does.
 * auto_reset != 0: envs that end are reset in the same step (Philox xy draws
 * with the seed of the last reset, task kept); their body is reset_states
 * f64[N,29] (the caller's own reset state rows, xy replaced by init_xy) or,
 * when NULL, the Philox reset_model draws; final_obs (nullable) f64[N,29]
 * receives their pre-reset ob. */
ogbx_status ogbx_antmaze_step(ogbx_maze_t env, const double* qpos_post, const double* qvel_post,
                              double* obs, float* reward, uint8_t* terminated, uint8_t* truncated,
                              uint8_t* success, double* final_obs, int32_t auto_reset,
                              const double* reset_states, void* stream);
/* ogbx_antmaze_step with the outputs and auto-reset flag of the last
 * ogbx_maze_bind_step (the steady per-step call: four arguments). */
ogbx_status ogbx_antmaze_step_bound(ogbx_maze_t env, const double* qpos_post, const double* qvel_post,
                                    const double* reset_states, void* stream);

/* Evaluation rollout without auto-reset: env i steps with actions device
 * [k_steps, N, 2] until the first step that ends its episode (terminated |
 * truncated) or k_steps, in ONE launch; rows k >= steps_taken[i] of the
 * outputs (same layout as ogbx_maze_step) are left untouched, and the env's
 * state is the state after its last step.  Replaces the reference's
 * evaluation episode loop `while not done: env.step(...)`
 * (impls/utils/evaluation.py:83-112) for a batch of episodes; a wave of 64
 * envs leaves the loop when a ballot finds all of them done.
 * Every written row equals what K calls of ogbx_maze_step (auto_reset 0)
 * produce. */
ogbx_status ogbx_maze_rollout_until_done(ogbx_maze_t env, const void* action, int32_t action_is_f64,
                                         int32_t k_steps, double* obs, float* reward, uint8_t* terminated,
                                         uint8_t* truncated, uint8_t* success, int32_t* steps_taken,
                                         void* stream);

/* Device pointers of the env-owned state (for checkpoint/restore and tests):
 * qpos f64[N,2], goal_xy f64[N,2], elapsed i32[N], task_id i32[N],
 * episode u32[N] (per-env reset counter = the Philox counter word of that
 * env's reset draws; zeroing it re-seeds the env: reset(seed=s) twice gives
 * the same episode, as gymnasium's reseeding does). */
ogbx_status ogbx_maze_state(ogbx_maze_t env, double** qpos, double** goal_xy, int32_t** elapsed,
                            int32_t** task_id, uint32_t** episode);

/* The seed later steps key their Philox draws with (auto-reset, noise), as
 * the last ogbx_maze_reset set it: a state restored through ogbx_maze_state
 * into another handle restores its seed with this (checkpoint/restore). */
ogbx_status ogbx_maze_set_seed(ogbx_maze_t env, uint64_t seed);

/* Free-standing physics: advance `n` point masses one PointEnv step without
 * any env bookkeeping: qpos_out = mj_step^5(qpos + 0.2*action).  Used by the
 * parity tests for arbitrary (qpos, action) pairs.  Replaces point.py:68-73. */
ogbx_status ogbx_point_physics(ogbx_maze_t env, const double* qpos_in, const void* action,
                               int32_t action_is_f64, int64_t n, double* qpos_out,
                               uint8_t* contact_out, void* stream);

/* Batched coordinate helpers (maze.py:552-562): xy f64[n,2] -> ij i32[n,2]
 * with Python int() truncation toward zero, and ij -> xy. */
ogbx_status ogbx_maze_xy_to_ij(ogbx_maze_t env, const double* xy, int64_t n, int32_t* ij,
                               void* stream);
ogbx_status ogbx_maze_ij_to_xy(ogbx_maze_t env, const int32_t* ij, int64_t n, double* xy,
                               void* stream);

/* Oracle subgoal (maze.py:503-550) for n (start_xy, goal_xy) pairs:
 * BFS next-hop from a device table built at create time.  subgoal f64[n,2]. */
ogbx_status ogbx_maze_oracle_subgoal(ogbx_maze_t env, const double* start_xy,
                                     const double* goal_xy, int64_t n, double* subgoal_xy,
                                     void* stream);

/* Point-maze expert action of data_gen_scripts/generate_locomaze.py:147-166
 * (+ the point actor, :44-46): dir = (subgoal - xy) / (||subgoal - xy|| +
 * 1e-6), action = clip(dir + normal, -1, 1), float64 [n,2].  start_xy /
 * goal_xy: device f64 [n,2], or both NULL to use the env's own qpos / goal
 * (then n must be the batch size).  normal: device f64 [n,2] draws of
 * np.random.normal(0, noise) (injected) or NULL = noise * Box-Muller(Philox
 * keyed by seed, counted by (row, call_index)). */
ogbx_status ogbx_maze_expert_action(ogbx_maze_t env, const double* start_xy, const double* goal_xy, int64_t n,
                                   double noise, const double* normal, uint64_t seed, uint64_t call_index,
                                   double* action, void* stream);

/* MazeEnv.set_goal(goal_ij) (maze.py:492-501) for the envs with mask != 0
 * (mask NULL = all): goal = ij_to_xy(goal_ij) plus, if add_noise_to_goal, the
 * add_noise draws (device f64 [N,2] uniform(-1,1) injected, or NULL = Philox).
 * goal_ij: device int32 [N,2].  Used by the 'navigate' data collection. */
ogbx_status ogbx_maze_set_goal(ogbx_maze_t env, const int32_t* goal_ij, const uint8_t* mask, const double* noise,
                               uint64_t seed, uint64_t call_index, void* stream);


/* ======================================================================
 * Offline replay: fused index-gather + hindsight goal relabel
 * (impls/utils/datasets.py: Dataset.get_random_idxs/get_subset :65-83,
 *  GCDataset.sample :213-294, GCDataset.sample_goals :296-327)
 * ====================================================================== */

/* One dataset column to gather into the batch. */
typedef struct {
  const void* src;   /* device, [num_rows, row_bytes] contiguous */
  void* dst;         /* device, [num_batches * batch, row_bytes] */
  int64_t row_bytes; /* bytes of one row (multiple of 4 uses dword copies) */
  int32_t select;    /* 0 = idxs, 1 = min(idxs+1, R-1) (next_observations,
                        datasets.py:82), 2 = value goal, 3 = actor goal */
  int32_t src_stride; /* bytes between consecutive source rows; 0 = row_bytes
                        (dense).  A larger stride lets several small columns
                        share one interleaved row record, so a sample's rows of
                        them come from one 128-B line instead of one line each. */
} ogbx_gc_column;

/* Static description of an HBM-resident trajectory buffer. */
typedef struct {
  int64_t num_rows;          /* R = Dataset.size (datasets.py:56)                */
  const int64_t* valid_idxs; /* device [num_valid] = nonzero(valids > 0) or NULL */
  int64_t num_valid;         /* (NULL -> randint(R), datasets.py:65-70)          */
  const int64_t* traj_end;   /* device [R]: terminal_locs[searchsorted(
                                terminal_locs, row)] (datasets.py:309)           */
  const int64_t* valid_traj_end; /* optional device [num_valid] =
                                traj_end[valid_idxs]: lets a drawn index and its
                                trajectory end load in parallel (NULL = two
                                dependent loads)                                  */
  const int64_t* valid_pairs; /* optional device [num_valid, 2] = (valid_idxs,
                                valid_traj_end) interleaved: the drawn index and
                                its trajectory end in ONE 16-B load (one line per
                                pick instead of two); used when non-NULL         */
  /* Optional closed form of the tables (0 = use them).  When the buffer is
   * num_rows / period equal trajectories whose pickable rows (valid_idxs, or
   * every row) are the first period_picks rows of each period and whose
   * trajectory end is row period_end of it, pick p of period q = p /
   * period_picks maps to idx = q period + p % period_picks and traj_end =
   * q period + period_end: no index load.  The caller guarantees equality
   * with valid_idxs / traj_end (ogbench_amd.datasets checks on the device);
   * the tables stay required for explicit idxs. */
  int64_t period;
  int64_t period_picks;
  int64_t period_end;
} ogbx_gc_buffer;

/* Goal-sampling configuration (GCDataset config keys, datasets.py:155-170).
 * *_traj_thresh = p_trajgoal / (1 - p_curgoal) computed by the caller in
 * float64 exactly as datasets.py:321.  *_cur_is_one = (p_curgoal == 1.0). */
typedef struct {
  double value_p_curgoal, value_traj_thresh, value_discount;
  double actor_p_curgoal, actor_traj_thresh, actor_discount;
  int32_t value_geom_sample, actor_geom_sample;
  int32_t value_cur_is_one, actor_cur_is_one;
  int32_t gc_negative;
  int32_t pad_;
} ogbx_gc_config;

/* Injected draws (parity mode).  Each pointer is device [num_batches*batch]
 * or NULL; a NULL pointer means "draw it from Philox".  The values are the
 * raw outputs of the reference's np.random calls in call order (datasets.py:
 * 67, 305, 312 or 316, 321, 325):
 *   pick      randint(len(valid_idxs)) for the sample indices
 *   v_pick / a_pick   randint(len(valid_idxs)) for random goals
 *   v_geom / a_geom   geometric(1 - discount) offsets (geom mode)
 *   v_dist / a_dist   rand() distances (uniform mode)
 *   v_u_traj, v_u_cur, a_u_traj, a_u_cur   the two rand() of the where()s. */
typedef struct {
  const int64_t* idxs;  /* explicit sample indices (sample(idxs=...)) or NULL */
  const int64_t* pick;
  const int64_t* v_pick;
  const int64_t* v_geom;
  const double* v_dist;
  const double* v_u_traj;
  const double* v_u_cur;
  const int64_t* a_pick;
  const int64_t* a_geom;
  const double* a_dist;
  const double* a_u_traj;
  const double* a_u_cur;
} ogbx_gc_draws;

/* Optional record of every draw the kernel used (same layout as
 * ogbx_gc_draws, all non-NULL device buffers) so a checker can replay it. */
typedef struct {
  int64_t* pick;
  int64_t* v_pick;
  int64_t* v_geom;
  double* v_dist;
  double* v_u_traj;
  double* v_u_cur;
  int64_t* a_pick;
  int64_t* a_geom;
  double* a_dist;
  double* a_u_traj;
  double* a_u_cur;
} ogbx_gc_draw_record;

/* Sample num_batches x batch transitions with value/actor goals in ONE launch.
 * Outputs: the columns (dst pointers), idxs_out / value_goal_out /
 * actor_goal_out (device int64 [nb*B], each nullable), masks / rewards
 * (device float64 [nb*B]: masks = 1 - (idxs == value_goal),
 *  rewards = (idxs == value_goal) - gc_negative, datasets.py:250-252).
 * Philox draws are keyed by (seed, stream tag) with counter (sample, call). */
ogbx_status ogbx_gc_sample(const ogbx_gc_buffer* buf, const ogbx_gc_config* cfg,
                           const ogbx_gc_column* cols, int32_t num_cols, int64_t batch,
                           int64_t num_batches, const ogbx_gc_draws* draws, uint64_t seed,
                           uint64_t call_index, int64_t* idxs_out, int64_t* value_goal_out,
                           int64_t* actor_goal_out, double* masks, double* rewards,
                           const ogbx_gc_draw_record* record, void* stream);

/* Look-ahead sampling for a steady stream of equal calls (same batch,
 * num_batches <= 1024 samples in total, Philox draws): the launch of call c
 * gathers its rows from the selectors the launch of call c-1 stored in
 * ahead_in (NULL: computed in this launch first) and, while it gathers,
 * computes call c+1's selectors (Philox counter call_index + 1) into
 * ahead_out (NULL: not computed), so a call's draw chain (Philox -> picks ->
 * goals) is off its own critical path.  ahead_in / ahead_out are caller-owned
 * device buffers of OGBX_GC_AHEAD_WORDS 8-byte words per sample, ordered on
 * `stream` (a launch on another stream needs a pair of its own: it would
 * overwrite selectors an in-flight launch still reads); ahead_in must hold
 * what the previous launch stored for exactly this (seed, call_index,
 * batch, num_batches, buffer, config), i.e. for call_index - 1's successor.  Every output
 * is bit-identical to ogbx_gc_sample's with the same seed and call_index.
 * Same reference as ogbx_gc_sample (datasets.py:213-327). */
#define OGBX_GC_AHEAD_WORDS 8
ogbx_status ogbx_gc_sample_ahead(const ogbx_gc_buffer* buf, const ogbx_gc_config* cfg,
                                 const ogbx_gc_column* cols, int32_t num_cols, int64_t batch,
                                 int64_t num_batches, uint64_t seed, uint64_t call_index,
                                 const int64_t* ahead_in, int64_t* ahead_out, int64_t* idxs_out,
                                 int64_t* value_goal_out, int64_t* actor_goal_out, double* masks,
                                 double* rewards, void* stream);

/* ---- HGCDataset (impls/utils/datasets.py:467-643) ------------------------
 * Static config of the hierarchical sampler.  Subgoal steps are the resolved
 * values of the reference's config (value/actor default to
 * high_subgoal_steps, itself defaulting to subgoal_steps).  The four tables
 * are device f64 arrays indexed by the clipped subgoal step count s in
 * [0, K] (K = value_subgoal_steps for hv_*, low_subgoal_steps for lv_*):
 * masks = 1 - (s < K), rewards = gc_negative ? -(1 - d^s)/(1 - d) : d^s (s < K),
 * precomputed on the host with the reference's own float64 power. */
typedef struct {
  int64_t value_subgoal_steps;
  int64_t low_subgoal_steps;
  int64_t actor_subgoal_steps;
  int32_t has_low_value_goals; /* config low_discount is not None */
  int32_t pad;
  double low_discount;
  const double* hv_mask_table;
  const double* hv_reward_table;
  const double* lv_mask_table;
  const double* lv_reward_table;
} ogbx_hgc_config;

/* Injected draws: the GC draws (pick, v_*, a_*) plus the low-level value goal
 * draws (l_*: randint pick, geometric, two rand) in the reference call order. */
typedef struct {
  ogbx_gc_draws gc;
  const int64_t* l_pick;
  const int64_t* l_geom;
  const double* l_u_traj;
  const double* l_u_cur;
} ogbx_hgc_draws;

typedef struct {
  ogbx_gc_draw_record gc;
  int64_t* l_pick;
  int64_t* l_geom;
  double* l_u_traj;
  double* l_u_cur;
} ogbx_hgc_draw_record;

/* Per-sample scalar outputs (device, [batch*num_batches]); index outputs
 * may be NULL. */
typedef struct {
  int64_t* idxs;
  int64_t* high_value_goal_idxs;
  int64_t* high_actor_goal_idxs;
  int64_t* low_value_goal_idxs;
  int64_t* high_value_offsets;      /* int64, goal - idx */
  int64_t* high_value_subgoal_steps;
  double* high_value_masks;
  double* high_value_rewards;
  int64_t* low_value_subgoal_steps;
  double* low_value_masks;
  double* low_value_rewards;
  double* masks;                    /* one-step: 1 - (idx == high value goal) */
  double* rewards;
} ogbx_hgc_outputs;

/* HGCDataset.sample in ONE launch.  Column `select` codes: 0 idx, 1 next
 * (min(idx+1, R-1)), 2 high value goal, 3 high actor goal, 4 high value next,
 * 5 low value next, 6 low value goal, 7 high actor next, 8 low actor goal
 * (min(idx + actor_subgoal_steps, final)), 9 low actor next. */
ogbx_status ogbx_hgc_sample(const ogbx_gc_buffer* buf, const ogbx_gc_config* cfg,
                            const ogbx_hgc_config* hcfg, const ogbx_gc_column* cols,
                            int32_t num_cols, int64_t batch, int64_t num_batches,
                            const ogbx_hgc_draws* draws, uint64_t seed, uint64_t call_index,
                            const ogbx_hgc_outputs* out, const ogbx_hgc_draw_record* record,
                            void* stream);

/* HGCDataset.sample with look-ahead: ogbx_gc_sample_ahead's scheme for
 * ogbx_hgc_sample (records of OGBX_HGC_AHEAD_WORDS words per sample: the ten
 * row selectors and the nine scalar outputs).  Bit-identical to
 * ogbx_hgc_sample with the same seed and call_index. */
#define OGBX_HGC_AHEAD_WORDS 20
ogbx_status ogbx_hgc_sample_ahead(const ogbx_gc_buffer* buf, const ogbx_gc_config* cfg,
                                  const ogbx_hgc_config* hcfg, const ogbx_gc_column* cols, int32_t num_cols,
                                  int64_t batch, int64_t num_batches, uint64_t seed, uint64_t call_index,
                                  const int64_t* ahead_in, int64_t* ahead_out, const ogbx_hgc_outputs* out,
                                  void* stream);

/* ---- Sampler plans: the steady sample(batch) call, prepared once ---------
 * A plan holds what every call of one GCDataset / HGCDataset repeats -- the
 * validated buffer and config, the Philox key of `seed`, the geometric log
 * terms -- plus up to OGBX_GC_PLAN_SLOTS prepared output batches and the
 * look-ahead state that ogbx_gc_sample_ahead leaves to its caller: one pair
 * of selector buffers per stream (owned by the plan, allocated on the
 * stream's first call, at most 8 streams; further streams run without
 * look-ahead) and the (stream, samples, call) the stored selectors belong
 * to.  So a host that calls ogbx_gc_plan_sample with increasing call indices
 * gets the look-ahead's latency without keeping its contract, and a call
 * whose index, size or stream does not match simply computes its own
 * selectors.  Every output is bit-identical to ogbx_gc_sample /
 * ogbx_hgc_sample with the same seed and call_index (whatever the slot,
 * stream or look-ahead setting).  hcfg NULL: GCDataset; else HGCDataset.
 * lookahead 0: every call launches the direct kernel. */
#define OGBX_GC_PLAN_SLOTS 8
typedef struct ogbx_gc_plan_s* ogbx_gc_plan_t;
ogbx_status ogbx_gc_plan_create(const ogbx_gc_buffer* buf, const ogbx_gc_config* cfg,
                                const ogbx_hgc_config* hcfg, uint64_t seed, int32_t lookahead,
                                ogbx_gc_plan_t* plan);
/* Prepare output batch `slot` (0..7): the columns (select codes as
 * ogbx_gc_sample / ogbx_hgc_sample), batch x num_batches samples, and the
 * scalar outputs (GC: idxs / goals may be NULL, masks and rewards not; HGC:
 * hgc_out, the GC scalars unused).  Overwrites the slot; launches already
 * issued keep their arguments. */
ogbx_status ogbx_gc_plan_set_batch(ogbx_gc_plan_t plan, int32_t slot, const ogbx_gc_column* cols,
                                   int32_t num_cols, int64_t batch, int64_t num_batches, int64_t* idxs_out,
                                   int64_t* value_goal_out, int64_t* actor_goal_out, double* masks,
                                   double* rewards, const ogbx_hgc_outputs* hgc_out);
/* One sample() call into the batch of `slot`, Philox counter call_index, on
 * `stream`: the look-ahead kernel (batch x num_batches <= 1024) or the direct
 * kernel. */
ogbx_status ogbx_gc_plan_sample(ogbx_gc_plan_t plan, int32_t slot, uint64_t call_index, void* stream);
/* Calls served from selectors a previous launch stored (diagnostic). */
int64_t ogbx_gc_plan_hits(ogbx_gc_plan_t plan);
/* Frees the plan and its look-ahead buffers (waits for launches in flight). */
ogbx_status ogbx_gc_plan_destroy(ogbx_gc_plan_t plan);

/* traj_end[r] = terminal_locs[searchsorted(terminal_locs, r, 'left')] for
 * r in [0, R): binary search per row over the sorted terminal_locs
 * (device int64 [num_terminals]).  datasets.py:186,309. */
ogbx_status ogbx_gc_traj_end(const int64_t* terminal_locs, int64_t num_terminals,
                             int64_t num_rows, int64_t* traj_end, void* stream);

/* out = nonzero(x > 0) for device float32 x[n] (stable order); *count is a
 * device int64.  Used for valid_idxs / terminal_locs (datasets.py:59-60,185). */
ogbx_status ogbx_nonzero_f32(const float* x, int64_t n, int64_t* out, int64_t* count,
                             void* stream);

/* ======================================================================
 * Powderworld (batched PowderworldEnv in 'task' mode; easy, medium, hard)
 * Reference: ogbench/powderworld/powderworld_env.py:21-476, sim.py:15-590,
 * registration ogbench/powderworld/__init__.py:3-8 (max_episode_steps 500).
 * One env = one world_size^2 grid; state stays in HBM between calls.
 * ====================================================================== */

typedef struct ogbx_powder_env* ogbx_powder_t;

typedef struct {
  int32_t world_size;        /* 32 or 64 (PowderworldEnv world_size, :24) */
  int32_t grid_size;         /* 4 (:25) */
  int32_t brush_size;        /* 4 (:26) */
  int32_t num_elems;         /* 2 = easy, 5 = medium, 8 = hard (:57-62) */
  int32_t max_episode_steps; /* TimeLimit (500 in the registry) */
  int32_t pad;
  int64_t env_base;          /* global index of env 0 (Philox counter; see
                                ogbx_maze_opts.env_base) */
} ogbx_powder_opts;

/* PowderworldEnv.__init__ (+ set_tasks, :81-282).  Easy: the goal world of
 * every task is replayed once on the device at create (its forward is
 * deterministic).  Medium/hard: the forward is stochastic, so every reset
 * replays its env's goal (powderworld_env.py:320-329) and keeps it per env. */
ogbx_status ogbx_powder_create(const ogbx_powder_opts* opts, int64_t n_envs, int32_t device,
                               ogbx_powder_t* out);
ogbx_status ogbx_powder_destroy(ogbx_powder_t env);
ogbx_status ogbx_powder_describe(ogbx_powder_t env, int32_t* world_size, int32_t* xy_action_size,
                                 int32_t* num_elems, int32_t* num_tasks, int32_t* tol);
/* Goal world element ids, host uint8 [num_tasks, H, W] (cur_goal_world, :329);
 * easy only (medium/hard goals: ogbx_powder_full_state). */
ogbx_status ogbx_powder_goal_worlds(ogbx_powder_t env, uint8_t* out);

/* PowderworldEnv.reset (:284-352) for envs with mask[e] != 0 (mask NULL = all).
 * task_id: device int32 [N] in 1..num_tasks, NULL = random task per env.
 * reset_action: device int32 [N,3] (elem index, x, y) of the random initial
 * semantic action (sample_semantic_action, :446-451), NULL = Philox draws.
 * rand (medium/hard): device float32 [N, rand_rows, 3, H, W], the three rand
 * fields (rand_movement, rand_interact, rand_element; sim.py:363-380) of each
 * forward: row s < len(task) = goal action s, row len(task) = the reset's
 * forward.  NULL = Philox.  Needs task_id, reset_action and rand_rows >=
 * longest task + 1.
 * obs, goal_obs: device uint8 [N, H, W, 6] (ob and info['goal']). */
ogbx_status ogbx_powder_reset(ogbx_powder_t env, const int32_t* task_id, const uint8_t* mask,
                              const int32_t* reset_action, const float* rand, int32_t rand_rows,
                              uint8_t* obs, uint8_t* goal_obs, uint64_t seed, void* stream);

/* k_steps x PowderworldEnv.step (:354-427) under TimeLimit.  action: device
 * int32 [k_steps, N]; an action outside the stage's range takes a random one
 * (np.random.randint, :358-377): draws[k, N] supplies those values, NULL =
 * Philox.  rand (medium/hard): device float32 [k_steps, N, 3, H, W] rand
 * fields of the forward of each third step, NULL = Philox (auto-resets always
 * draw from Philox).  Outputs per (k, env): obs uint8 [k,N,H,W,6], reward
 * float32, terminated/truncated/success uint8.  auto_reset != 0 resets done
 * envs in the same step (obs is then the new episode's first observation). */
ogbx_status ogbx_powder_step(ogbx_powder_t env, const int32_t* action, int32_t k_steps,
                             const int32_t* draws, const float* rand, uint8_t* obs, float* reward,
                             uint8_t* terminated, uint8_t* truncated, uint8_t* success,
                             int32_t auto_reset, void* stream);

/* Device pointers to the state: world uint8 [N, H*W] (id | GravityInter<<5 |
 * DidGravity<<6), ctrl int32 [N] (stage | elem<<2 | x<<8 | task<<16),
 * elapsed int32 [N], episode uint32 [N] (Philox counter word, as for
 * ogbx_maze_state).  Any argument may be NULL.  Writable (state restore):
 * medium/hard envs keep a render cache of the world's colours, and asking for
 * `world` marks it stale, so the next ogbx_powder_step renders from the state
 * (a write through a kept pointer after that step must be announced with
 * ogbx_powder_state_written; readers use ogbx_powder_state_view). */
ogbx_status ogbx_powder_state(ogbx_powder_t env, uint8_t** world, int32_t** ctrl,
                              int32_t** elapsed, uint32_t** episode);

/* Read-only views of the state (world as ogbx_powder_state; momentum,
 * velocity and goal ids as ogbx_powder_full_state, medium/hard only).  Unlike
 * those two, this hands out no writable pointer, so the render cache and the
 * phase guess stay valid: the accessor for readers that run every step
 * (PowderworldEnv.world_ids / world_full).  Any argument may be NULL. */
ogbx_status ogbx_powder_state_view(ogbx_powder_t env, const uint8_t** world, const int8_t** momentum,
                                   const float** velocity, const uint8_t** goal_ids);

/* The caller wrote the state through a pointer of ogbx_powder_state /
 * ogbx_powder_full_state (a restore, an edit): marks the render cache stale,
 * forgets the phase guess and allows stepping without a reset.  Needed when
 * the write comes after a step that followed the pointer's hand-out (a host
 * that keeps the pointers); harmless otherwise. */
ogbx_status ogbx_powder_state_written(ogbx_powder_t env);

/* Phase hint (medium/hard): every env steps in phase, `phase` steps after a
 * common all-env reset (what an unmasked ogbx_powder_reset sets to 0); -1 =
 * unknown (what ogbx_powder_state_written and masked resets set).  With it
 * the host skips the light kernel on steps where every in-phase env needs the
 * full kernel, and launches the full kernel in its sparse form (a few envs
 * per workgroup) on render-only steps.  A wrong hint only costs time: envs out
 * of the phase are stepped bit-identically either way.  For a host restoring
 * a checkpoint of envs it knows to be in phase. */
ogbx_status ogbx_powder_set_phase(ogbx_powder_t env, int64_t phase);

/* The seed of the steps' Philox draws (invalid-action replacements, rand
 * fields, auto-resets), as the last ogbx_powder_reset set it; restores it with
 * a state loaded through ogbx_powder_state (checkpoint/restore). */
ogbx_status ogbx_powder_set_seed(ogbx_powder_t env, uint64_t seed);

/* Medium/hard state: momentum int8 [N, H*W] (channel 6), velocity float32
 * [N, H*W, 2] (channels 3, 4), goal ids uint8 [N, H*W] (cur_goal_world).
 * Asking for `velocity` marks the render cache stale, as `world` does above. */
ogbx_status ogbx_powder_full_state(ogbx_powder_t env, int8_t** momentum, float** velocity,
                                   uint8_t** goal_ids);

/* `steps` x PWSim.forward (sim.py:363-380) on packed easy worlds, device
 * uint8 [n_worlds, H*W] in -> out (may alias). */
ogbx_status ogbx_powder_forward(ogbx_powder_t env, const uint8_t* world_in, int64_t n_worlds,
                                int32_t steps, uint8_t* world_out, void* stream);

/* `steps` x PWSim.forward with every rule (stone, gravity, sand, fluid, ice,
 * water, fire, plant, velocity; sim.py:284-308, 461-982) on worlds in the
 * reference's layout, device float32 [n_worlds, 9, H, W] in -> out.  rand:
 * device float32 [steps, n_worlds, 3, H, W] or NULL (Philox).  rgb_out
 * (optional): PWRenderer.render of the result, uint8 [n_worlds, H, W, 3]. */
ogbx_status ogbx_powder_forward_full(ogbx_powder_t env, const float* world_in, int64_t n_worlds,
                                     int32_t steps, const float* rand, float* world_out,
                                     uint8_t* rgb_out, void* stream);

/* Task table (host only, no device): semantic actions (elem index, x, y) of
 * task task_id (1-based) for num_elems 2/5/8 into seq [cap, 3], its length
 * and success tolerance (set_tasks, powderworld_env.py:81-282). */
ogbx_status ogbx_powder_task_table(int32_t num_elems, int32_t task_id, int32_t* seq, int32_t cap,
                                   int32_t* len, int32_t* tol);

/* ======================================================================
 * Dataset loader and relabel pass (ogbench/utils.py:14-96,
 * ogbench/relabel_utils.py).  Device buffers; rows are dense.
 * ====================================================================== */

/* Compact-dataset rewrite of the raw terminals t[n] (utils.py:65-76):
 * valids = 1 - t, shifted = t[i+1] (1.0 past the end),
 * terminals = min(t + shifted, 1).  Any output may be NULL. */
ogbx_status ogbx_compact_terminals(const float* terminals_in, int64_t n, float* terminals_out,
                                   float* valids_out, float* shifted_out, void* stream);

/* dst[k] = src[idx[k]] for rows of row_bytes bytes (k < n).  With idx from
 * ogbx_nonzero_f32 this is the regular-dataset mask compaction
 * (utils.py:77-94: observations[ob_mask], observations[next_ob_mask], ...). */
ogbx_status ogbx_gather_rows(const void* src, int64_t row_bytes, const int64_t* idx, int64_t n, void* dst,
                             void* stream);

/* Maze branch of relabel_dataset + add_oracle_reps in one pass over qpos
 * (float32 or float64 [num_rows, qpos_stride]): success = ||qpos[:,0:2] -
 * goal|| <= goal_tol in float64; rewards = success - 1, masks = 1 - success
 * (float32 [num_rows]); oracle_reps = float32(qpos[:, 0:2]) ([num_rows, 2]).
 * Any output may be NULL.  relabel_utils.py:17-31,116-127,166. */
ogbx_status ogbx_relabel_maze(const void* qpos, int32_t qpos_is_f64, int64_t num_rows, int64_t qpos_stride,
                              double goal_x, double goal_y, double goal_tol, float* rewards, float* masks,
                              float* oracle_reps, void* stream);

/* ======================================================================
 * Evaluation counters (impls/utils/evaluation.py:36-123, impls/main.py:226-258)
 * ====================================================================== */

/* For every env i whose episode ended at this step (terminated[i] |
 * truncated[i]) while remaining[i] > 0: counters[task_id[i]-1] += {success[i],
 * 1} and remaining[i] -= 1.  All pointers are device memory: success /
 * terminated / truncated u8[n] (a step's outputs), task_id i32[n] (1-based),
 * remaining i32[n] (in/out), counters int64[num_tasks, 2] = {success_sum,
 * episode_count} (accumulated, never cleared here; num_tasks <= 64).  The
 * counter block is what ranks all-gather at the end of evaluation. */
ogbx_status ogbx_eval_accumulate(const uint8_t* success, const uint8_t* terminated,
                                 const uint8_t* truncated, const int32_t* task_id,
                                 int32_t* remaining, int64_t n, int32_t num_tasks, int64_t* counters,
                                 void* stream);

/* ----------------------------------------------------------------------
 * Eval all-gather over RCCL (xGMI), for hosts without torch.distributed
 * (impls/main.py:226-258 gathers per-task success across workers).  One
 * communicator per (process, device): rank 0 calls ogbx_comm_unique_id and
 * ships the 128-byte id to every rank out of band (the cgo / JNI host's own
 * channel); every rank then calls ogbx_comm_create.  RCCL is resolved at
 * run time (the librccl.so.1 already in the process, e.g. PyTorch's, or the
 * system one), so libogbx.so has no link-time RCCL dependency.
 * ---------------------------------------------------------------------- */
typedef struct ogbx_comm* ogbx_comm_t;
#define OGBX_COMM_ID_BYTES 128

ogbx_status ogbx_comm_unique_id(uint8_t* id /* host [OGBX_COMM_ID_BYTES] */);
ogbx_status ogbx_comm_create(const uint8_t* id, int32_t world_size, int32_t rank, int32_t device,
                             ogbx_comm_t* out);
ogbx_status ogbx_comm_destroy(ogbx_comm_t comm);
/* all[r * count + i] = local_of_rank_r[i] for every rank r: device int64
 * local[count] (e.g. the int64[num_tasks, 2] counters) -> device int64
 * all[world_size * count].  Async on `stream`. */
ogbx_status ogbx_eval_allgather(ogbx_comm_t comm, const int64_t* local, int64_t count, int64_t* all,
                                void* stream);

#ifdef __cplusplus
}
#endif

#endif /* OGBX_H */
