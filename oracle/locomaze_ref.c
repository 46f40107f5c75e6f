/*
 * oracle/locomaze_ref.c -- TEST INFRASTRUCTURE ONLY (never shipped, never
 * called by the product path).  Plain-C restatement of the reference pointmaze
 * env, used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * as the checker for libogbx.
 *
 * Parity status (see DESIGN.md section "Oracle"):
 *   - maze tables, xy_to_ij/ij_to_xy, reset arithmetic, free-space step,
 *     success mask, reward/termination/truncation: PINNED by the reference code
 *     (known-answer tests derived from maze.py / point.py, golden tables in
 *     tests/golden/ extracted from the reference source).
 *   - wall-contact dynamics (inside mujoco.mj_step, point.py:73): pinned to
 *     MuJoCo's PUBLISHED FORMULATION by tests/mjmodel_np.py (independent
 *     enumeration model + closed forms, agreement 2e-16), NOT to MuJoCo's
 *     output: MuJoCo (pyproject.toml:12, mujoco >= 3.1.6, no lockfile) is not
 *     installed and no reference trajectories exist; this file restates the
 *     published MuJoCo soft-constraint algorithm with the defaults listed in
 *     DESIGN.md.  It is written independently of the HIP kernel: literal
 *     4-edge pyramids in acceleration space (floor included as 4 edges) and a
 *     Newton solver with Armijo backtracking, instead of the kernel's u-space,
 *     3-row, exact-line-search solver.
 *
 * Reference citations (hliuson/ogbench):
 *   maze maps/tasks       ogbench/locomaze/maze.py:90-163, 308-359
 *   reset                 ogbench/locomaze/maze.py:373-431, 564-567
 *   step / success        ogbench/locomaze/maze.py:433-466, 486-490
 *   xy_to_ij / ij_to_xy   ogbench/locomaze/maze.py:552-562
 *   PointEnv.step         ogbench/locomaze/point.py:64-95 (mj_step nstep=5)
 *   point model           ogbench/locomaze/assets/point.xml:4-40
 *   wall boxes            ogbench/locomaze/maze.py:225-239
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------ tables */
typedef struct {
  const char* name;
  int H, W, ntasks;
  const char* map;
  int tasks[5][4];
} orc_maze;

static const orc_maze ORC_MAZES[] = {
    {"arena", 8, 8, 1,
     "11111111100000011000000110000001100000011000000110000001"
     "11111111",
     {{1, 1, 6, 6}}},
    {"medium", 8, 8, 5,
     "11111111100110011001000111000111100100011010010110001001"
     "11111111",
     {{1, 1, 6, 6}, {6, 1, 1, 6}, {5, 3, 4, 2}, {6, 5, 6, 1}, {2, 6, 1, 1}}},
    {"large", 9, 12, 5,
     "111111111111100001000001101101010101100000010001101111011101"
     "100101000001110101010111100100010001111111111111",
     {{1, 1, 7, 10}, {5, 4, 7, 1}, {7, 4, 1, 10}, {3, 8, 5, 4}, {1, 1, 5, 4}}},
    {"giant", 12, 16, 5,
     "1111111111111111101000000110000110101101010011011000100100010001"
     "1011101111110101100010001000010111101010010101111000100100010001"
     "1010101111110101101110001000110110000010001000011111111111111111",
     {{1, 1, 10, 14}, {1, 14, 10, 1}, {8, 14, 1, 1}, {8, 3, 5, 12}, {5, 9, 3, 8}}},
    {"teleport", 9, 12, 5,
     "111111111111100000101001110100010011110111000001100001010101"
     "101101010101101101010101100001000101111111111111",
     {{1, 10, 7, 1}, {1, 1, 7, 10}, {5, 6, 7, 10}, {7, 1, 7, 10}, {5, 6, 7, 1}}},
};

static const orc_maze* find_maze(const char* name) {
  for (size_t k = 0; k < sizeof(ORC_MAZES) / sizeof(ORC_MAZES[0]); ++k)
    if (strcmp(ORC_MAZES[k].name, name) == 0) return &ORC_MAZES[k];
  return NULL;
}

int orc_maze_tables(const char* name, int* H, int* W, int* ntasks, int* map_out, int* tasks_out) {
  const orc_maze* mz = find_maze(name);
  if (!mz) return -1;
  *H = mz->H;
  *W = mz->W;
  *ntasks = mz->ntasks;
  if (map_out)
    for (int c = 0; c < mz->H * mz->W; ++c) map_out[c] = mz->map[c] == '1';
  if (tasks_out)
    for (int t = 0; t < mz->ntasks; ++t)
      for (int k = 0; k < 4; ++k) tasks_out[4 * t + k] = mz->tasks[t][k];
  return 0;
}

/* -------------------------------------------------- MuJoCo point constants */
/* point.xml: sphere r = 0.7, density 100, slide joints x/y, timestep 0.02 RK4;
 * default solref (0.02, 1), solimp (0.9, 0.95, 0.001, 0.5, 2), pyramidal cone,
 * friction (1, 0.5, 0.5), margin 0. */
#define ORC_PI 3.14159265358979323846
static const double R_SPH = 0.7;
static const double DT = 0.02;
static const double SOLIMP[5] = {0.9, 0.95, 0.001, 0.5, 2.0};
static const double MJMINVAL = 1e-15;
static const double UNIT = 4.0, OFFX = 4.0, OFFY = 4.0;

typedef struct {
  double m, K, B, tran;
} orc_consts;

static orc_consts consts(void) {
  orc_consts c;
  double vol = 4.0 / 3.0 * ORC_PI * R_SPH * R_SPH * R_SPH;
  c.m = 100.0 * vol;
  double tc = 0.02;
  if (tc < 2.0 * DT) tc = 2.0 * DT; /* refsafe */
  double dr = 1.0, dmax = SOLIMP[1];
  c.K = 1.0 / (dmax * dmax * tc * tc * dr * dr);
  c.B = 2.0 / (dmax * tc);
  /* body_invweight0[tran] = trace(J M^-1 J')/3 with J = [e_x e_y] (2 of 3 axes) */
  c.tran = (2.0 / c.m) / 3.0;
  return c;
}

static double get_imp(double pos) {
  double x = fabs(pos / SOLIMP[2]);
  if (x >= 1.0) return SOLIMP[1];
  if (x <= 0.0) return SOLIMP[0];
  double y;
  if (x <= SOLIMP[3])
    y = pow(x, SOLIMP[4]) / pow(SOLIMP[3], SOLIMP[4] - 1.0);
  else
    y = 1.0 - pow(1.0 - x, SOLIMP[4]) / pow(1.0 - SOLIMP[3], SOLIMP[4] - 1.0);
  return SOLIMP[0] + y * (SOLIMP[1] - SOLIMP[0]);
}

#define MAXE 32
typedef struct {
  int n;
  double jx[MAXE], jy[MAXE], aref[MAXE], D[MAXE];
} edges_t;

/* one condim-3 contact: 4 pyramid edges n +- mu*t1, n +- mu*t2 (mu = 1) */
static void push_contact(edges_t* E, const orc_consts* C, double dist, const double n[2],
                         const double t1[2], const double t2[2], double vx, double vy) {
  double imp = get_imp(dist);
  double diag = C->tran + 1.0 * 1.0 * C->tran;
  double R = (1.0 - imp) / imp * diag;
  if (R < MJMINVAL) R = MJMINVAL;
  const double* tt[2] = {t1, t2};
  for (int k = 0; k < 2; ++k)
    for (int sgn = 1; sgn >= -1; sgn -= 2) {
      if (E->n >= MAXE) return;
      double jx = n[0] + sgn * tt[k][0], jy = n[1] + sgn * tt[k][1];
      E->jx[E->n] = jx;
      E->jy[E->n] = jy;
      E->aref[E->n] = -C->B * (jx * vx + jy * vy) - C->K * imp * dist;
      E->D[E->n] = 1.0 / R;
      E->n++;
    }
}

static int build_edges(const orc_maze* mz, const orc_consts* C, double x, double y, double vx,
                       double vy, edges_t* E) {
  E->n = 0;
  /* floor plane: normal +z (J_n = 0), tangents e_y and -e_x, dist 0 */
  {
    double n[2] = {0, 0}, t1[2] = {0, 1}, t2[2] = {-1, 0};
    push_contact(E, C, 0.0, n, t1, t2, vx, vy);
  }
  int walls = 0;
  int ci = (int)floor((y + OFFY + 0.5 * UNIT) / UNIT);
  int cj = (int)floor((x + OFFX + 0.5 * UNIT) / UNIT);
  for (int i = ci - 1; i <= ci + 1; ++i)
    for (int j = cj - 1; j <= cj + 1; ++j) {
      if (i < 0 || i >= mz->H || j < 0 || j >= mz->W) continue;
      if (mz->map[i * mz->W + j] != '1') continue;
      /* box centre (j*4-4, i*4-4, 1), half sizes (2, 2, 1) */
      double bx = j * UNIT - OFFX, by = i * UNIT - OFFY, bz = 0.5 / 2 * UNIT;
      double hs[3] = {UNIT / 2, UNIT / 2, 0.5 / 2 * UNIT};
      double c3[3] = {x - bx, y - by, 0.7 - bz};
      double cl[3], t[3];
      for (int k = 0; k < 3; ++k) {
        cl[k] = c3[k] < -hs[k] ? -hs[k] : (c3[k] > hs[k] ? hs[k] : c3[k]);
        t[k] = cl[k] - c3[k];
      }
      double d = sqrt(t[0] * t[0] + t[1] * t[1] + t[2] * t[2]);
      if (d - R_SPH > 0.0) continue;
      walls++;
      if (d > MJMINVAL) {
        double n[2] = {-t[0] / d, -t[1] / d};
        double t1[2] = {-n[1], n[0]}, t2[2] = {0.0, 0.0};
        push_contact(E, C, d - R_SPH, n, t1, t2, vx, vy);
      } else {
        double fd[6] = {hs[0] + c3[0], hs[0] - c3[0], hs[1] + c3[1],
                        hs[1] - c3[1], hs[2] + c3[2], hs[2] - c3[2]};
        int k = 0;
        for (int f = 1; f < 6; ++f)
          if (fd[f] < fd[k]) k = f;
        double dist = -fd[k] - R_SPH;
        double s = (k & 1) ? 1.0 : -1.0;
        double n[2] = {0, 0}, t1[2] = {0, 0}, t2[2] = {0, 0};
        if (k < 2) { n[0] = s; t1[1] = 1; }
        else if (k < 4) { n[1] = s; t1[0] = 1; }
        else { t1[0] = 1; t2[1] = 1; }
        push_contact(E, C, dist, n, t1, t2, vx, vy);
      }
    }
  return walls;
}

static double cost(const orc_consts* C, const edges_t* E, double ax, double ay) {
  double f = 0.5 * C->m * (ax * ax + ay * ay);
  for (int e = 0; e < E->n; ++e) {
    double r = E->jx[e] * ax + E->jy[e] * ay - E->aref[e];
    if (r < 0) f += 0.5 * E->D[e] * r * r;
  }
  return f;
}

/* qacc = argmin cost: semismooth Newton with Armijo backtracking. */
static void solve(const orc_consts* C, const edges_t* E, double* ax_out, double* ay_out) {
  double ax = 0.0, ay = 0.0;
  for (int it = 0; it < 200; ++it) {
    double gx = C->m * ax, gy = C->m * ay, h00 = C->m, h01 = 0.0, h11 = C->m;
    for (int e = 0; e < E->n; ++e) {
      double r = E->jx[e] * ax + E->jy[e] * ay - E->aref[e];
      if (r < 0) {
        gx += E->D[e] * r * E->jx[e];
        gy += E->D[e] * r * E->jy[e];
        h00 += E->D[e] * E->jx[e] * E->jx[e];
        h01 += E->D[e] * E->jx[e] * E->jy[e];
        h11 += E->D[e] * E->jy[e] * E->jy[e];
      }
    }
    double det = h00 * h11 - h01 * h01;
    double px = -(h11 * gx - h01 * gy) / det;
    double py = -(h00 * gy - h01 * gx) / det;
    if (fabs(px) + fabs(py) <= 1e-16 * (1.0 + fabs(ax) + fabs(ay))) break;
    double f0 = cost(C, E, ax, ay), slope = gx * px + gy * py, t = 1.0;
    while (t > 1e-30 && cost(C, E, ax + t * px, ay + t * py) > f0 + 1e-6 * t * slope) t *= 0.5;
    if (t <= 1e-30) break;
    ax += t * px;
    ay += t * py;
  }
  *ax_out = ax;
  *ay_out = ay;
}

static void accel(const orc_maze* mz, const orc_consts* C, double x, double y, double vx,
                  double vy, double* ax, double* ay) {
  edges_t E;
  build_edges(mz, C, x, y, vx, vy, &E);
  solve(C, &E, ax, ay);
}

/* One PointEnv.step physics: q <- mj_step^5(q + delta, v = 0).  Returns 1 if a
 * wall contact existed at the start.  The literal RK4 of mj_RungeKutta is
 * evaluated at every stage (no fast path here). */
static int point_step(const orc_maze* mz, const orc_consts* C, double* px, double* py) {
  edges_t E0;
  int contact = build_edges(mz, C, *px, *py, 0.0, 0.0, &E0) > 0;
  static const double A[3] = {0.5, 0.5, 1.0};
  static const double Bw[4] = {1.0 / 6.0, 1.0 / 3.0, 1.0 / 3.0, 1.0 / 6.0};
  double q[2] = {*px, *py}, v[2] = {0.0, 0.0};
  for (int sub = 0; sub < 5; ++sub) {
    double Xq[4][2], Xv[4][2], F[4][2];
    Xq[0][0] = q[0]; Xq[0][1] = q[1]; Xv[0][0] = v[0]; Xv[0][1] = v[1];
    accel(mz, C, q[0], q[1], v[0], v[1], &F[0][0], &F[0][1]);
    for (int i = 1; i < 4; ++i) {
      for (int d = 0; d < 2; ++d) {
        double dq = A[i - 1] * Xv[i - 1][d];
        double dv = A[i - 1] * F[i - 1][d];
        Xq[i][d] = q[d] + dq * DT;
        Xv[i][d] = v[d] + dv * DT;
      }
      accel(mz, C, Xq[i][0], Xq[i][1], Xv[i][0], Xv[i][1], &F[i][0], &F[i][1]);
    }
    for (int d = 0; d < 2; ++d) {
      double dq = 0.0, dv = 0.0;
      for (int j = 0; j < 4; ++j) {
        dq += Bw[j] * Xv[j][d];
        dv += Bw[j] * F[j][d];
      }
      v[d] = v[d] + dv * DT;
      q[d] = q[d] + dq * DT;
    }
  }
  *px = q[0];
  *py = q[1];
  return contact;
}

int orc_point_physics(const char* maze, const double* qpos, const void* action, int act_f64,
                      int64_t n, double* qpos_out, uint8_t* contact_out, int nthreads) {
  const orc_maze* mz = find_maze(maze);
  if (!mz) return -1;
  orc_consts C = consts();
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 256)
#endif
  for (int64_t i = 0; i < n; ++i) {
    double x = qpos[2 * i], y = qpos[2 * i + 1];
    if (act_f64) {
      const double* a = (const double*)action;
      x = x + 0.2 * a[2 * i];
      y = y + 0.2 * a[2 * i + 1];
    } else {
      const float* a = (const float*)action;
      float sx = 0.2f * a[2 * i], sy = 0.2f * a[2 * i + 1];
      x = x + (double)sx;
      y = y + (double)sy;
    }
    int c = point_step(mz, &C, &x, &y);
    qpos_out[2 * i] = x;
    qpos_out[2 * i + 1] = y;
    if (contact_out) contact_out[i] = (uint8_t)c;
  }
  return 0;
}

/* ------------------------------------------------------------- Philox4x32 */
static void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c[0], p1 = (uint64_t)0xCD9E8D57u * c[2];
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
    uint32_t n1 = (uint32_t)p1;
    uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    uint32_t n3 = (uint32_t)p0;
    c[0] = n0; c[1] = n1; c[2] = n2; c[3] = n3;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

static double u53(uint32_t hi, uint32_t lo) {
  return (double)((((uint64_t)hi << 32) | lo) >> 11) * (1.0 / 9007199254740992.0);
}

void orc_philox4x32(const uint32_t* ctr, uint32_t k0, uint32_t k1, uint32_t* out) {
  uint32_t c[4] = {ctr[0], ctr[1], ctr[2], ctr[3]};
  philox(c, k0, k1);
  memcpy(out, c, sizeof(c));
}

/* reset draws of env i at episode ep (stream key = seed ^ tag) */
static void reset_draws(uint64_t i, uint32_t ep, uint32_t k0, uint32_t k1, double r[4]) {
  uint32_t a[4] = {(uint32_t)i, ep, 0u, (uint32_t)(i >> 32)};
  uint32_t b[4] = {(uint32_t)i, ep, 1u, (uint32_t)(i >> 32)};
  philox(a, k0, k1);
  philox(b, k0, k1);
  r[0] = -1.0 + 2.0 * u53(a[0], a[1]);
  r[1] = -1.0 + 2.0 * u53(a[2], a[3]);
  r[2] = -1.0 + 2.0 * u53(b[0], b[1]);
  r[3] = -1.0 + 2.0 * u53(b[2], b[3]);
}

/* The reset draws [n,4] that libogbx's maze_reset_kernel uses for envs
 * env_base .. env_base+n-1 at episode counter ep (checker of Philox resets). */
void orc_reset_draws(int64_t n, int64_t env_base, uint32_t ep, uint32_t k0, uint32_t k1, double* out) {
  for (int64_t i = 0; i < n; ++i) reset_draws((uint64_t)(env_base + i), ep, k0, k1, out + 4 * i);
}

/* ------------------------------------------------------------- env level */
typedef struct {
  int success_pre, terminate_at_goal, add_noise_to_goal, reward_task_id, max_steps;
  double goal_tol;
} orc_opts;

static void ij_to_xy(int i, int j, double* x, double* y) {
  *x = j * UNIT - OFFX;
  *y = i * UNIT - OFFY;
}

void orc_xy_to_ij(const double* xy, int64_t n, int32_t* ij) {
  for (int64_t t = 0; t < n; ++t) {
    /* Python int() truncates toward zero, as a C cast does */
    ij[2 * t] = (int32_t)((xy[2 * t + 1] + OFFY + 0.5 * UNIT) / UNIT);
    ij[2 * t + 1] = (int32_t)((xy[2 * t] + OFFX + 0.5 * UNIT) / UNIT);
  }
}

static int success_of(double x, double y, double gx, double gy, double tol) {
  double dx = x - gx, dy = y - gy;
  return sqrt(fma(dy, dy, dx * dx)) <= tol; /* 1-D ddot: dx*dx then fma */
}

/* MazeEnv.reset (point): ob = init_xy (+noise), goal = goal_xy (+noise if set) */
static void reset_env(const orc_maze* mz, const orc_opts* o, int task, const double r[4],
                      double* x, double* y, double* gx, double* gy) {
  double ix, iy, bx, by;
  ij_to_xy(mz->tasks[task - 1][0], mz->tasks[task - 1][1], &ix, &iy);
  ij_to_xy(mz->tasks[task - 1][2], mz->tasks[task - 1][3], &bx, &by);
  *x = ix + r[0] * UNIT / 4;
  *y = iy + r[1] * UNIT / 4;
  if (o->add_noise_to_goal) {
    *gx = bx + r[2] * UNIT / 4;
    *gy = by + r[3] * UNIT / 4;
  } else {
    *gx = bx;
    *gy = by;
  }
}

int orc_maze_reset(const char* maze, const int* opts_i, const int32_t* task_id,
                   const double* noise, int64_t n, double* qpos, double* goal, int32_t* elapsed,
                   int32_t* task_out) {
  const orc_maze* mz = find_maze(maze);
  if (!mz) return -1;
  orc_opts o = {opts_i[0], opts_i[1], opts_i[2], opts_i[3], opts_i[4], opts_i[5] ? 0.5 : 1.0};
  for (int64_t i = 0; i < n; ++i) {
    int task = o.reward_task_id > 0 ? o.reward_task_id : task_id[i];
    reset_env(mz, &o, task, noise + 4 * i, &qpos[2 * i], &qpos[2 * i + 1], &goal[2 * i],
              &goal[2 * i + 1]);
    elapsed[i] = 0;
    task_out[i] = task;
  }
  return 0;
}

/* k_steps of TimeLimit(MazeEnv(PointEnv)).step for n envs, host state in/out.
 * opts_i = {success_pre, terminate_at_goal, add_noise_to_goal, reward_task_id,
 *           max_steps, is_not_point}.  Auto-reset draws come from Philox with
 * key (k0, k1), the GLOBAL env index env_base + i and the per-env episode
 * counter, exactly like libogbx (ogbx_maze_opts.env_base). */
int orc_maze_step(const char* maze, const int* opts_i, double* qpos, double* goal,
                  int32_t* elapsed, const int32_t* task, uint32_t* episode, int64_t n,
                  const void* action, int act_f64, int k_steps, double* obs, float* reward,
                  uint8_t* term, uint8_t* trunc, uint8_t* succ, int auto_reset, uint32_t k0,
                  uint32_t k1, int nthreads, int64_t env_base) {
  const orc_maze* mz = find_maze(maze);
  if (!mz) return -1;
  orc_consts C = consts();
  orc_opts o = {opts_i[0], opts_i[1], opts_i[2], opts_i[3], opts_i[4], opts_i[5] ? 0.5 : 1.0};
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 256)
#endif
  for (int64_t i = 0; i < n; ++i) {
    double x = qpos[2 * i], y = qpos[2 * i + 1], gx = goal[2 * i], gy = goal[2 * i + 1];
    int el = elapsed[i];
    uint32_t ep = episode[i];
    for (int k = 0; k < k_steps; ++k) {
      int64_t oi = (int64_t)k * n + i;
      double dx, dy;
      if (act_f64) {
        const double* a = (const double*)action;
        dx = 0.2 * a[2 * oi];
        dy = 0.2 * a[2 * oi + 1];
      } else {
        const float* a = (const float*)action;
        float sx = 0.2f * a[2 * oi], sy = 0.2f * a[2 * oi + 1];
        dx = (double)sx;
        dy = (double)sy;
      }
      int s = 0;
      if (o.success_pre) s = success_of(x, y, gx, gy, o.goal_tol);
      x = x + dx;
      y = y + dy;
      point_step(mz, &C, &x, &y);
      if (!o.success_pre) s = success_of(x, y, gx, gy, o.goal_tol);
      const double ox = x, oy = y; /* ob is taken before a teleport (maze.py:437-451) */
      if (strcmp(maze, "teleport") == 0) {
        /* teleport maze portals (maze.py:149-161): in (4,6), (5,1); out (1,7),
         * (6,1), (6,10); radius 1, triggered within 1.5 (norm as success_of).
         * The out portal is the libogbx Philox draw (key (k0 ^ 0x4D5A0002, k1),
         * counter (i, episode, 0x100 + elapsed, hi32(i))), in place of
         * np.random.randint(3). */
        static const int tin[2][2] = {{4, 6}, {5, 1}}, tout[3][2] = {{1, 7}, {6, 1}, {6, 10}};
        for (int t = 0; t < 2; ++t) {
          double px, py;
          ij_to_xy(tin[t][0], tin[t][1], &px, &py);
          if (success_of(x, y, px, py, 1.0 * 1.5)) {
            const uint64_t gi = (uint64_t)(env_base + i);
            uint32_t c[4] = {(uint32_t)gi, ep, 0x100u + (uint32_t)el, (uint32_t)(gi >> 32)};
            philox(c, k0 ^ 0x4D5A0002u, k1);
            const int oidx = (int)(((uint64_t)c[0] * 3u) >> 32);
            ij_to_xy(tout[oidx][0], tout[oidx][1], &x, &y);
            break;
          }
        }
      }
      float rw = s ? 1.0f : 0.0f;
      if (o.reward_task_id > 0) rw -= 1.0f;
      int te = s && o.terminate_at_goal;
      el += 1;
      int tr = el >= o.max_steps;
      reward[oi] = rw;
      term[oi] = (uint8_t)te;
      trunc[oi] = (uint8_t)tr;
      succ[oi] = (uint8_t)s;
      if (auto_reset && (te || tr)) {
        double r[4];
        ep += 1u;
        reset_draws((uint64_t)(env_base + i), ep, k0, k1, r);
        reset_env(mz, &o, task[i], r, &x, &y, &gx, &gy);
        el = 0;
      }
      double wx = ox, wy = oy;
      if (auto_reset && (te || tr)) {
        wx = x;
        wy = y;
      }
      obs[2 * oi] = wx;
      obs[2 * oi + 1] = wy;
    }
    qpos[2 * i] = x;
    qpos[2 * i + 1] = y;
    goal[2 * i] = gx;
    goal[2 * i + 1] = gy;
    elapsed[i] = el;
    episode[i] = ep;
  }
  return 0;
}

/* get_oracle_subgoal (maze.py:503-550), literal BFS per query. */
int orc_oracle_subgoal(const char* maze, const double* start_xy, const double* goal_xy,
                       int64_t n, double* sub_xy) {
  const orc_maze* mz = find_maze(maze);
  if (!mz) return -1;
  const int H = mz->H, W = mz->W;
  int* bfs = (int*)malloc(sizeof(int) * H * W);
  int* qu = (int*)malloc(sizeof(int) * H * W * 4);
  for (int64_t t = 0; t < n; ++t) {
    int ij[4];
    orc_xy_to_ij(start_xy + 2 * t, 1, ij);
    orc_xy_to_ij(goal_xy + 2 * t, 1, ij + 2);
    for (int k = 0; k < 4; ++k) {
      int hi = (k % 2 == 0) ? H - 1 : W - 1;
      if (ij[k] < 0) ij[k] = 0;
      if (ij[k] > hi) ij[k] = hi;
    }
    for (int c = 0; c < H * W; ++c) bfs[c] = -1;
    bfs[ij[2] * W + ij[3]] = 0;
    int qh = 0, qt = 0;
    qu[qt++] = ij[2] * W + ij[3];
    const int di[4] = {-1, 0, 1, 0}, dj[4] = {0, -1, 0, 1};
    while (qh < qt) {
      int c = qu[qh++], i = c / W, j = c % W;
      for (int k = 0; k < 4; ++k) {
        int ni = i + di[k], nj = j + dj[k];
        if (ni >= 0 && ni < H && nj >= 0 && nj < W && mz->map[ni * W + nj] == '0' &&
            bfs[ni * W + nj] == -1) {
          bfs[ni * W + nj] = bfs[c] + 1;
          qu[qt++] = ni * W + nj;
        }
      }
    }
    int si = ij[0], sj = ij[1];
    for (int k = 0; k < 4; ++k) {
      int ni = ij[0] + di[k], nj = ij[1] + dj[k];
      if (ni >= 0 && ni < H && nj >= 0 && nj < W && mz->map[ni * W + nj] == '0' &&
          bfs[ni * W + nj] < bfs[si * W + sj]) {
        si = ni;
        sj = nj;
      }
    }
    ij_to_xy(si, sj, &sub_xy[2 * t], &sub_xy[2 * t + 1]);
  }
  free(bfs);
  free(qu);
  return 0;
}

/* Point-maze expert action (data_gen_scripts/generate_locomaze.py:147-166, the
 * point actor :44-46) with injected np.random.normal draws `normal` [n,2]:
 * dir = d / (sqrt(fma(dy, dy, dx*dx)) + 1e-6) (np.linalg.norm of a 1-D pair via
 * BLAS ddot), action = clip(dir + normal, -1, 1). */
int orc_expert_action(const char* maze, const double* xy, const double* goal_xy, const double* normal, int64_t n,
                      double* action) {
  double* sub = (double*)malloc(sizeof(double) * 2 * (n > 0 ? n : 1));
  if (orc_oracle_subgoal(maze, xy, goal_xy, n, sub) != 0) {
    free(sub);
    return -1;
  }
  for (int64_t t = 0; t < n; ++t) {
    const double dx = sub[2 * t] - xy[2 * t], dy = sub[2 * t + 1] - xy[2 * t + 1];
    const double den = sqrt(fma(dy, dy, dx * dx)) + 1e-6;
    double a0 = dx / den + normal[2 * t], a1 = dy / den + normal[2 * t + 1];
    action[2 * t] = a0 < -1.0 ? -1.0 : (a0 > 1.0 ? 1.0 : a0);
    action[2 * t + 1] = a1 < -1.0 ? -1.0 : (a1 > 1.0 ? 1.0 : a1);
  }
  free(sub);
  return 0;
}
