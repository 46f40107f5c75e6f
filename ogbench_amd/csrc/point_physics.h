// point_physics.h -- the point-mass contact MODEL shared by the step kernels
// (constants, contact slots, impedance gains, the generic collider and the
// safety net's objective); the solver and the RK4 loop of one PointEnv step
//   qpos <- qpos + 0.2*action ; qvel <- 0 ; mj_step x5 (RK4, dt 0.02)
// are in point_contact.h (point_step_as).  The model is that of the 2-DoF slide-joint sphere of ogbench/locomaze/assets/point.xml inside
// the box walls that MazeEnv.update_tree adds (ogbench/locomaze/maze.py:225-239).
//
// Model (see DESIGN.md "Point-mass contact model" for every assumed MuJoCo
// default; wall-contact parity is pinned to MuJoCo's published
// formulation by tests/mjmodel_np.py, not to MuJoCo's output -- MuJoCo is absent):
//   * M = m*I2, m = density*4/3*pi*r^3 (point.xml:8,28), qacc_smooth = 0
//     (ctrl never written, gravity orthogonal to both slide axes).
//   * Contacts: sphere-floor (always active at dist = 0, J_normal = 0 in the
//     slide space) and sphere-box for wall cells of the 3x3 neighbourhood;
//     condim 3, pyramidal cone, mu = 1 -> edges J = Jn +- mu*Jt_k.
//   * Soft constraint per edge: aref = -B*(J.v) - K*imp*dist, cost 1/2*D*r^2 on
//     r = J.a - aref < 0, D = 1/R, R = max(mjMINVAL, (1-imp)/imp*diagApprox).
//   * qacc = argmin 1/2 m|a|^2 + sum_edges cost, solved exactly (active-set
//     iteration, point_contact.h; damped Newton with Armijo backtracking as the
//     safety net).
//   * RK4 tableau of mj_RungeKutta; mj_advance uses the B-weighted velocity.
//
// Because every edge has aref = -B*J.v - kp with the same B, the residual of an
// edge is r = J.(a + B v) + kp.  The solver therefore works in u = a + B*v:
//   minimise 1/2 m |u - B v|^2 + 1/2 Df |u|^2 + sum_e 1/2 w_e min(0, J_e.u + kp_e)^2
// (the floor's four edges +-e_x, +-e_y at dist 0 sum to the Df term), and
// returns a = u - B*v.  Per wall contact the edges are n+t, n-t (weight D) and
// n (the two edges along the vertical tangent, weight 2D).
//
// Fast path: if the sphere does not touch a wall at qpos+0.2a, every RK stage
// has v = 0, a = 0 and qpos is returned unchanged (+0.0, as mj_integratePos).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cmath>

namespace ogbx {

struct PointModel {
  double mass;        // m
  double h;           // opt.timestep (0.02)
  double B, K;        // solref-derived damping / stiffness
  double diag;        // diagApprox of one pyramid edge
  double D_floor;     // 1/R at imp(dist = 0) = solimp[0]
  double imp_dmin, imp_dmax, imp_width;
  double imp_mid, imp_a, imp_b;  // power-2 sigmoid: y = a x^2 | 1 - b (1-x)^2
  double radius;      // sphere radius 0.7
  double r2_hi;       // radius^2 * (1 + 1e-12): sqrt-free rejection bound
  double sphere_z;    // sphere centre height 0.7
  double box_cz, box_hz;  // wall box centre z / half height
  double box_hxy;     // wall box half size in x and y (maze_unit/2)
  double unit, inv_unit, off_x, off_y;
  // derived solver constants (host-computed, see make_point_model)
  double M;           // m + D_floor
  double m_over_M;    // m / M
  double w_max;       // D of an edge at imp = dmax (|dist| >= width)
  double kp_max;      // K * dmax
  double inv_M2w, inv_M4w, inv_det3;  // closed-form reciprocals at w = w_max
  double inv_width;   // 1 / solimp width
  int32_t nsub;       // frame_skip (5)
  int32_t pad_;
};

constexpr double kMinVal = 1e-15;  // mjMINVAL
// Largest double x with fl(sqrt(x)) <= 0.7 (the point radius, point.xml:28):
// fl(sqrt(x)) - 0.7 > 0  <=>  x > kPointFarD2 (tests/test_utils_cpu.py checks it).
constexpr double kPointFarD2 = 0.49;

// 1/d for d > 0 in the normal range: v_rcp_f64 + one Newton-Raphson
// refinement (3 dependent instructions instead of the 10 of the IEEE division
// sequence).  Measured on gfx950 (scripts/micro/rcp_err.hip, 4M values over
// [2^-20, 2^20)): v_rcp_f64 alone 4.6e-8 relative error, +1 refinement
// 2.2e-15 (10 ulp), +2 refinements equal to 1.0/d.  The second refinement
// cost 0.8 % of the step and changes no parity result at the 1e-9 contact
// tolerance.
__device__ __forceinline__ double fast_recip(double d) {
  double r = __builtin_amdgcn_rcp(d);
  r = fma(r, fma(-d, r, 1.0), r);
  return r;
}

#ifdef OGBX_WAVE_STAMPS
// Diagnostic build only: per-wave path counters of the current step, packed
// [cold-block entries | iteration trips << 20 | band stages << 40], kept in a
// register (no memory traffic on the measured path) and stored with the
// wave's time stamps at the end of maze_step_kernel.
#define OGBX_WPATH(shift) (g_wpath += 1ull << (shift))
#else
#define OGBX_WPATH(shift) ((void)0)
#endif

#ifdef OGBX_PHYS_STATS
// Diagnostic build only (-DOGBX_PHYS_STATS): per-path counters.
__device__ unsigned long long g_phys_stats[32];
#define OGBX_STAT(k) atomicAdd(&g_phys_stats[k], 1ull)
// once per wave when any active lane satisfies cond
#define OGBX_WSTAT(k, cond) do {                                                   \
    const unsigned long long _b = __ballot(1);                                     \
    if (__any(cond) && (int)(threadIdx.x & 63) == __ffsll((long long)_b) - 1)      \
      atomicAdd(&g_phys_stats[k], 1ull); } while (0)
#else
#define OGBX_STAT(k) ((void)0)
#define OGBX_WSTAT(k, cond) ((void)0)
#endif

// A sphere whose centre lies in an empty cell touches at most 3 wall boxes
// (two faces + the corner box between them).  States with the centre deep in
// a wall (contact through a box z face = two pseudo-contacts) are unreachable
// from any reset; there, contacts beyond 3 are dropped.
constexpr int kMaxContacts = 3;

struct ContactSlot {
  double nx, ny;  // Jn: gradient of dist (slide dofs)
  double tx, ty;  // slide projection of the horizontal tangent
  double kp;      // K*imp*dist
  double w;       // D = 1/R of one edge
};

// Three named slots, not an array: LLVM cannot turn a write to a runtime slot
// into a dynamically indexed store, so the contacts never leave VGPRs.
struct Contacts {
  int n;
  bool roles;  // slots hold the role layout of collide_in_frame (s0 x face, s1 y face)
  ContactSlot s0, s1, s2;
};

// Static slot access (k is a compile-time constant in every unrolled loop).
__device__ __forceinline__ const ContactSlot& slot_of(const Contacts& c, int k) {
  return k == 0 ? c.s0 : (k == 1 ? c.s1 : c.s2);
}

// Impedance-dependent (D, K*imp*dist) of a contact at `dist` (MuJoCo
// getimpedance, solimp power 2).  Beyond the transition width these are the
// precomputed constants.  Inside it: x = |dist|/width (as a product with the
// host-rounded reciprocal) and D = 1/R = imp / ((1-imp)*diag) (one division;
// R >= (1-dmax)/dmax*diag never reaches mjMINVAL).  Both differ from MuJoCo's
// literal quotients by at most an ulp (contact path tolerance 1e-9).
__device__ __forceinline__ void contact_gains(const PointModel& pm, double dist, double* D,
                                              double* kp) {
  *D = pm.w_max;
  *kp = pm.kp_max * dist;
  const double x = fabs(dist) * pm.inv_width;
  if (x < 1.0) {
    double imp;
    if (x <= 0.0) {
      imp = pm.imp_dmin;
    } else {
      const double y = x <= pm.imp_mid ? pm.imp_a * (x * x) : 1.0 - pm.imp_b * ((1.0 - x) * (1.0 - x));
      imp = pm.imp_dmin + y * (pm.imp_dmax - pm.imp_dmin);
    }
    *D = imp / ((1.0 - imp) * pm.diag);
    *kp = pm.K * imp * dist;
  }
}

// Clamp of a box-frame coordinate to [-h, h] (the closest point of the box).
// v_max/v_min_f64: two instructions instead of two compares and four selects;
// identical results (signed zeros inside the range pass through unchanged).
__device__ __forceinline__ double clamp_box(double p, double h) {
  return __builtin_fmin(__builtin_fmax(p, -h), h);
}

// Store one contact into slot `slot` (runtime index, per-field selects: a
// branchy store would be merged by SimplifyCFG into one store through a
// selected address -> scratch).
__device__ __forceinline__ void add_contact(const PointModel& pm, Contacts& c, int slot, double dist,
                                            double nx, double ny, double tx, double ty) {
  double D, kp;
  contact_gains(pm, dist, &D, &kp);
  auto put = [&](ContactSlot& d, bool on) {
    d.nx = on ? nx : d.nx;
    d.ny = on ? ny : d.ny;
    d.tx = on ? tx : d.tx;
    d.ty = on ? ty : d.ty;
    d.kp = on ? kp : d.kp;
    d.w = on ? D : d.w;
  };
  put(c.s0, slot == 0);
  put(c.s1, slot == 1);
  put(c.s2, slot == 2);
}

__device__ __forceinline__ void zero_slot(ContactSlot& k) {
  k.nx = 0.0; k.ny = 0.0; k.tx = 0.0; k.ty = 0.0; k.kp = 0.0; k.w = 0.0;
}

// Generic (slow, rare) collision: the sphere centre is in a wall cell, off the
// map, or exactly on a box face.  Exact sphere-box test (MuJoCo sphere-box in
// the box frame; boxes axis aligned, margin 0) of the own cell's box and the
// x-side, y-side and diagonal neighbours, in that order.  One rolled loop with
// one contact-append site keeps this path small (it is inlined).
__device__ __forceinline__ int collide_walls_generic(const PointModel& pm, const uint16_t* nbmask,
                                                     int H, int W, double x, double y, double fi,
                                                     double fj, int sx, int sy, Contacts& c) {
  zero_slot(c.s0);
  zero_slot(c.s1);
  zero_slot(c.s2);
  const double cx = fj * pm.unit - pm.off_x, cy = fi * pm.unit - pm.off_y;
  const double u = pm.unit, hx = pm.box_hxy, hz = pm.box_hz;
  int nc = 0;
#pragma unroll 1
  for (int b = 0; b < 4; ++b) {
    const int dj = (b & 1) ? sx : 0;  // b: 0 own cell, 1 x side, 2 y side, 3 diagonal
    const int di = (b & 2) ? sy : 0;
    if ((b == 1 && sx == 0) || (b == 2 && sy == 0) || (b == 3 && (sx == 0 || sy == 0))) continue;
    const double ii = fi + di, jj = fj + dj;
    if (!(ii >= 0.0 && ii < (double)H && jj >= 0.0 && jj < (double)W)) continue;
    if (!((nbmask[(int)ii * W + (int)jj] >> 4) & 1u)) continue;  // the cell's own wall bit
    const double px = x - (cx + dj * u);
    const double py = y - (cy + di * u);
    const double pz = pm.sphere_z - pm.box_cz;
    const double clx = clamp_box(px, hx);
    const double cly = clamp_box(py, hx);
    const double clz = clamp_box(pz, hz);
    const double tx = clx - px, ty = cly - py, tz = clz - pz;
    const double d2 = tx * tx + ty * ty + tz * tz;
    if (d2 > pm.r2_hi || nc >= kMaxContacts) continue;  // certainly d - r > 0
    double dist, nx, ny, ax, ay;  // ax, ay: tangent of the (first) contact
    int ne = 1;
    bool second = false;          // z face: two pseudo-contacts (tangents e_x, e_y)
    // Face contacts need neither sqrt nor division: sqrt(fl(t*t)) == |t|.
    double d;
    if (ty == 0.0 && tz == 0.0) {
      d = fabs(tx);
      nx = tx > 0.0 ? -1.0 : 1.0;
      ny = -0.0 * ty;
    } else if (tx == 0.0 && tz == 0.0) {
      d = fabs(ty);
      nx = -0.0 * tx;
      ny = ty > 0.0 ? -1.0 : 1.0;
    } else {
      d = sqrt(d2);
      nx = -tx / d;
      ny = -ty / d;
    }
    if (d - pm.radius > 0.0) continue;
    if (d > kMinVal) {
      // centre outside the box: normal along (centre - closest point).
      dist = d - pm.radius;
      ax = -ny;
      ay = nx;
    } else {
      // centre inside the box: push out through the nearest face
      // (faces ordered -x, +x, -y, +y, -z, +z; first strict minimum wins).
      const double f0 = hx + px, f1 = hx - px, f2 = hx + py, f3 = hx - py, f4 = hz + pz,
                   f5 = hz - pz;
      int k = 0;
      double best = f0;
      if (f1 < best) { best = f1; k = 1; }
      if (f2 < best) { best = f2; k = 2; }
      if (f3 < best) { best = f3; k = 3; }
      if (f4 < best) { best = f4; k = 4; }
      if (f5 < best) { best = f5; k = 5; }
      dist = -best - pm.radius;
      const double sgn = (k & 1) ? 1.0 : -1.0;
      if (k < 2) {
        nx = sgn; ny = 0.0; ax = 0.0; ay = 1.0;
      } else if (k < 4) {
        nx = 0.0; ny = sgn; ax = 1.0; ay = 0.0;
      } else {
        nx = 0.0; ny = 0.0; ax = 1.0; ay = 0.0;
        second = true;
        ne = 2;
      }
    }
#pragma unroll 1
    for (int e = 0; e < ne && nc < kMaxContacts; ++e) {
      const bool z2 = second && e == 1;
      add_contact(pm, c, nc, dist, nx, ny, z2 ? 0.0 : ax, z2 ? 1.0 : ay);
      ++nc;
    }
  }
  c.n = nc;
  c.roles = false;
  return nc;
}

// ---------------------------------------------------------------------------
// The objective, in u = a + B v (see the header comment):
//   f(u) = 1/2 M |u - cu|^2 + sum_s sum_e 1/2 w_se min(0, r_se)^2,
//   M = m + Df, cu = m B v / M, and for contact s with a = n.u + kp, b = t.u:
//   e0: r = a + b (weight w), e1: r = a - b (w), e2: r = a (2w).
// Gradient, Hessian and value of f at u for explicit contact rows (the
// damped-Newton safety net of point_contact.h armijo_newton): every slot, an
// empty slot an all-zero row (r = 0, never active, no contribution).
__device__ __forceinline__ void eval_piece(const PointModel& pm, const Contacts& c, double cux, double cuy,
                                           double ux, double uy, double* g, double* h, double* fval) {
#pragma clang fp contract(fast)
  const double M = pm.M;
  g[0] = M * (ux - cux);
  g[1] = M * (uy - cuy);
  h[0] = M; h[1] = 0.0; h[2] = M;
  double f = 0.5 * M * ((ux - cux) * (ux - cux) + (uy - cuy) * (uy - cuy));
#pragma unroll
  for (int s = 0; s < kMaxContacts; ++s) {
    const ContactSlot& k = slot_of(c, s);
    const double a = k.nx * ux + k.ny * uy + k.kp;
    const double b = k.tx * ux + k.ty * uy;
#pragma unroll
    for (int e = 0; e < 3; ++e) {
      const double sg = e == 0 ? 1.0 : (e == 1 ? -1.0 : 0.0);
      const double r = e == 2 ? a : a + sg * b;
      // branch-free: an inactive row contributes with weight 0
      const bool on = r < 0.0;
      const double we = on ? (e == 2 ? 2.0 * k.w : k.w) : 0.0;
      const double jx = e == 2 ? k.nx : k.nx + sg * k.tx;
      const double jy = e == 2 ? k.ny : k.ny + sg * k.ty;
      const double wr = we * r, wjx = we * jx;
      g[0] += wr * jx;
      g[1] += wr * jy;
      h[0] += wjx * jx;
      h[1] += wjx * jy;
      h[2] += (we * jy) * jy;
      f += 0.5 * wr * r;
    }
  }
  *fval = f;
}

// MuJoCo-derived constants of the point model (DESIGN.md lists each source).
// constexpr: every locomaze maze uses maze_unit = 4 and offset 4, so the
// kernels fold kPointModel into immediates instead of reading it per launch.
constexpr PointModel make_point_model(double unit, double off) {
  PointModel pm{};
  const double pi = 3.14159265358979323846;
  const double r = 0.7, density = 100.0;
  pm.mass = density * (4.0 * pi * r * r * r / 3.0);
  pm.h = 0.02;
  pm.nsub = 5;
  // solref (0.02, 1) with refsafe: timeconst = max(0.02, 2*dt) = 0.04
  const double timeconst = 0.02 > 2.0 * pm.h ? 0.02 : 2.0 * pm.h, dampratio = 1.0;
  // solimp (0.9, 0.95, 0.001, 0.5, 2); power 2: a = 1/mid^(p-1), b = 1/(1-mid)^(p-1)
  pm.imp_dmin = 0.9;
  pm.imp_dmax = 0.95;
  pm.imp_width = 0.001;
  pm.imp_mid = 0.5;
  pm.imp_a = 1.0 / pm.imp_mid;
  pm.imp_b = 1.0 / (1.0 - pm.imp_mid);
  const double dmax = pm.imp_dmax;
  pm.K = 1.0 / (dmax * dmax * timeconst * timeconst * dampratio * dampratio);
  pm.B = 2.0 / (dmax * timeconst);
  // body_invweight0 (translation) = mean diag of J M^-1 J' over 3 axes = 2/(3m);
  // pyramid edge diagApprox = tran + mu^2 * tran with mu = 1.
  const double tran = (1.0 / pm.mass + 1.0 / pm.mass + 0.0) / 3.0;
  const double mu = 1.0;
  pm.diag = tran + mu * mu * tran;
  double Rf = (1.0 - pm.imp_dmin) * pm.diag / pm.imp_dmin;
  if (Rf < kMinVal) Rf = kMinVal;
  // Floor: four edges +-e_x, +-e_y, each with D = 1/Rf; exactly one edge of
  // each pair is active, which sums to 1/2 Df |a + B v|^2.
  pm.D_floor = 1.0 / Rf;
  pm.radius = r;
  pm.r2_hi = r * r * (1.0 + 1e-12);
  pm.sphere_z = 0.7;
  pm.box_cz = 0.5 / 2.0 * unit;  // maze_height/2 * maze_unit (maze.py:233)
  pm.box_hz = 0.5 / 2.0 * unit;
  pm.box_hxy = unit / 2.0;
  pm.unit = unit;
  pm.inv_unit = 1.0 / unit;  // exact for unit = 4
  pm.off_x = off;
  pm.off_y = off;
  // solver constants
  pm.M = pm.mass + pm.D_floor;
  pm.m_over_M = pm.mass / pm.M;
  double Rmax = (1.0 - dmax) * pm.diag / dmax;
  if (Rmax < kMinVal) Rmax = kMinVal;
  pm.w_max = 1.0 / Rmax;
  pm.kp_max = pm.K * dmax;
  const double w = pm.w_max, M = pm.M;
  pm.inv_M2w = 1.0 / (M + 2.0 * w);
  pm.inv_M4w = 1.0 / (M + 4.0 * w);
  pm.inv_det3 = 1.0 / ((M + 3.0 * w) * (M + w) - w * w);
  pm.inv_width = 1.0 / pm.imp_width;
  return pm;
}

// The model of every locomaze maze (maze_unit 4, offset 4: maze.py:83-86).
constexpr PointModel kPointModel = make_point_model(4.0, 4.0);

}  // namespace ogbx
