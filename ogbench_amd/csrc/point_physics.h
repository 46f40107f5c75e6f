// point_physics.h -- device restatement of one PointEnv physics step:
//   qpos <- qpos + 0.2*action ; qvel <- 0 ; mj_step x5 (RK4, dt 0.02)
// for the 2-DoF slide-joint sphere of ogbench/locomaze/assets/point.xml inside
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
//   * qacc = argmin 1/2 m|a|^2 + sum_edges cost, solved exactly: closed-form
//     active-set enumeration for one wall contact, full-step semismooth Newton
//     (stops when the active set reproduces itself) for several, and a damped
//     Newton with Armijo backtracking as the safety net.
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
// tolerance (-DOGBX_RCP_NR2 restores it).
__device__ __forceinline__ double fast_recip(double d) {
  double r = __builtin_amdgcn_rcp(d);
  r = fma(r, fma(-d, r, 1.0), r);
#ifdef OGBX_RCP_NR2
  r = fma(r, fma(-d, r, 1.0), r);
#endif
  return r;
}

#ifdef OGBX_PHYS_STAMPS
// Diagnostic build only: per-wave cycle sums of the stage-loop segments
// [collide, solve, update, whole point_step], indexed by global wave id.
__device__ unsigned long long g_phys_stamps[4096 * 4];
__device__ __forceinline__ unsigned long long stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define OGBX_STAMP_DECL unsigned long long _t0 = stamp(), _ta = 0, _tb = 0, _tc = 0, _tl = _t0, _tn;
#define OGBX_STAMP_SEG(acc) do { _tn = stamp(); acc += _tn - _tl; _tl = _tn; } while (0)
#define OGBX_STAMP_END do {                                                          \
    const unsigned w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;               \
    if (w < 4096) {                                                                 \
      atomicMax(&g_phys_stamps[4 * w + 0], _ta); atomicMax(&g_phys_stamps[4 * w + 1], _tb); \
      atomicMax(&g_phys_stamps[4 * w + 2], _tc);                                    \
      atomicMax(&g_phys_stamps[4 * w + 3], stamp() - _t0); } } while (0)
#else
#define OGBX_STAMP_DECL
#define OGBX_STAMP_SEG(acc) ((void)0)
#define OGBX_STAMP_END ((void)0)
#endif

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
#ifdef OGBX_ABL_NO_BAND
  return;
#endif
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
#ifdef OGBX_CLAMP_SELECT
  return p < -h ? -h : (p > h ? h : p);
#else
  return __builtin_fmin(__builtin_fmax(p, -h), h);
#endif
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

// All wall contacts of the sphere at (x, y), branch-light.  Only boxes of the
// 3x3 neighbourhood can be touched (r < maze_unit/2).  With the centre in an
// empty cell the candidates have fixed roles and fixed slots:
//   s0 = the x-side box (a face contact: ty == 0), s1 = the y-side box (face,
//   tx == 0), s2 = the diagonal box (a vertical-edge contact: sqrt + division).
// A neighbour on side s is a candidate only if the centre is within r (+1e-9
// slack) of that side of its cell, so the result equals the full 9-box scan.
// Face contacts use d = |t|, n = -sign(t): bit-identical to MuJoCo's
// d = sqrt(t.t), n = -t/d because sqrt(fl(t*t)) == |t|.  Slots without a
// contact are all-zero (their rows are inactive in every solver).
// Rare geometry (centre in a wall cell / off the map / exactly on a face) is
// routed to collide_walls_generic.
// The cell of the sphere centre and its 3x3 wall mask.  A step moves the
// centre by far less than a cell, so point_step computes this once per step and
// again only when the centre leaves the inner part of the cell (cell_frame_valid).
struct CellFrame {
  double fi, fj, cx, cy;  // cell indices (as doubles) and cell centre
  uint32_t m;             // 3x3 neighbourhood wall mask (0x1FF off the map)
  bool inside;            // cell within the map
};

__device__ __forceinline__ void cell_frame(const PointModel& pm, const uint16_t* nbmask, int H, int W,
                                           double x, double y, CellFrame& f) {
  f.fi = floor((y + pm.off_y + 0.5 * pm.unit) * pm.inv_unit);
  f.fj = floor((x + pm.off_x + 0.5 * pm.unit) * pm.inv_unit);
  f.cx = f.fj * pm.unit - pm.off_x;
  f.cy = f.fi * pm.unit - pm.off_y;
  f.inside = f.fi >= 0.0 && f.fi < (double)H && f.fj >= 0.0 && f.fj < (double)W;
  f.m = f.inside ? nbmask[(int)f.fi * W + (int)f.fj] : 0x1FFu;
}

// True when (x, y) is certainly still in the frame's cell: |offset| < 0.49975
// unit puts (x + off + unit/2) / unit strictly inside (fj, fj + 1), so the
// floor() of cell_frame would return the same cell.
__device__ __forceinline__ bool cell_frame_valid(const PointModel& pm, const CellFrame& f, double x,
                                                 double y) {
  const double lim = 0.49975 * pm.unit;
  return fabs(x - f.cx) < lim && fabs(y - f.cy) < lim;
}

__device__ __forceinline__ int collide_in_frame(const PointModel& pm, const uint16_t* nbmask, int H,
                                                int W, double x, double y, const CellFrame& f,
                                                Contacts& c) {
  const double fi = f.fi, fj = f.fj, cx = f.cx, cy = f.cy;
  const uint32_t m = f.m;
  const double lx = x - cx, ly = y - cy;  // offset from own cell centre
  const double reach = pm.box_hxy - pm.radius - 1e-9;
  const int sx = lx >= reach ? 1 : (lx <= -reach ? -1 : 0);
  const int sy = ly >= reach ? 1 : (ly <= -reach ? -1 : 0);
  bool slow = !f.inside || ((m >> 4) & 1u);
  const double hx = pm.box_hxy, r = pm.radius, u = pm.unit;
  // role validity from the neighbourhood mask
  const bool vX = sx != 0 && ((m >> (4 + sx)) & 1u);
  const bool vY = sy != 0 && ((m >> (4 + 3 * sy)) & 1u);
  const bool vD = sx != 0 && sy != 0 && ((m >> (4 + 3 * sy + sx)) & 1u);
  // x-side box: centre (cx + sx u, cy)
  // (its y offset is ly: the closest point's y is the centre's unless |ly| > hx,
  // when tXy = clamp(ly) - ly != 0 and the face guard below routes to generic;
  // otherwise tXy = ly - ly = +0 exactly, so it is not computed)
  double dX, tXx;
  {
    const double px = x - (cx + sx * u);
    tXx = clamp_box(px, hx) - px;
    dX = fabs(tXx);
  }
  double dY, tYy;
  {
    const double py = y - (cy + sy * u);
    tYy = clamp_box(py, hx) - py;
    dY = fabs(tYy);
  }
  double tDx, tDy, d2D;
  {
    const double px = x - (cx + sx * u), py = y - (cy + sy * u);
    const double clx = clamp_box(px, hx);
    const double cly = clamp_box(py, hx);
    tDx = clx - px;
    tDy = cly - py;
    d2D = tDx * tDx + tDy * tDy;
  }
  const bool cX = vX && dX - r <= 0.0;
  const bool cY = vY && dY - r <= 0.0;
  bool cD = vD && d2D <= pm.r2_hi;
  // exact-geometry guards: face roles must really be faces, d > mjMINVAL
  slow = slow || (cX && (fabs(ly) > hx || dX <= kMinVal)) || (cY && (fabs(lx) > hx || dY <= kMinVal));
  double dD = 0.0, nDx = 0.0, nDy = 0.0;
  OGBX_WSTAT(11, cD);
  OGBX_WSTAT(12, slow);
#ifndef OGBX_DIAG_BRANCHY
  {  // vertical-edge contact of the diagonal box, straight-line (no divergent branch)
#ifdef OGBX_DIAG_SQRT
    const double dd = sqrt(cD ? d2D : 1.0);
    const double inv = fast_recip(dd);
    const bool far = dd - r > 0.0;
    slow = slow || (cD && !far && dd <= kMinVal);
#else
    // The contact test fl(sqrt(d2)) - r > 0 is decided exactly on d2 (far_d2 is
    // the largest double whose correctly rounded root is <= r), so the flag is
    // the oracle's bit for bit; the distance and the normal come from v_rsq_f64
    // + one Newton-Raphson step (~1e-14 relative, the contact tolerance is 1e-9).
    const double d2 = cD ? fmax(d2D, 1e-300) : 1.0;
    const double y0 = __builtin_amdgcn_rsq(d2);
    const double inv = y0 * fma(-0.5 * d2 * y0, y0, 1.5);
    const double dd = d2 * inv;
    const bool far = pm.radius == 0.7 ? d2 > kPointFarD2 : sqrt(d2) - r > 0.0;
    slow = slow || (cD && !far && d2 <= kMinVal * kMinVal);
#endif
    cD = cD && !far;
    dD = cD ? dd : 0.0;
    nDx = cD ? -tDx * inv : 0.0;
    nDy = cD ? -tDy * inv : 0.0;
  }
#else
  if (cD && !slow) {  // vertical-edge contact of the diagonal box
    dD = sqrt(d2D);
    if (dD - r > 0.0) {
      cD = false;
    } else if (dD <= kMinVal) {
      slow = true;
    } else {
      const double inv = fast_recip(dD);
      nDx = -tDx * inv;
      nDy = -tDy * inv;
    }
  }
#endif
  OGBX_WSTAT(10, (cX && fabs(dX - r) * pm.inv_width < 1.0) || (cY && fabs(dY - r) * pm.inv_width < 1.0) ||
                     (cD && fabs(dD - r) * pm.inv_width < 1.0));
  double D, kp;
  // s0: x face, n = (-sign(tx), -ty) with ty = +-0
  contact_gains(pm, dX - r, &D, &kp);
  c.s0.nx = cX ? (tXx > 0.0 ? -1.0 : 1.0) : 0.0;
  c.s0.ny = cX ? -0.0 : 0.0;  // -tXy, tXy = +0
  c.s0.tx = -c.s0.ny;
  c.s0.ty = c.s0.nx;
  c.s0.kp = cX ? kp : 0.0;
  c.s0.w = cX ? D : 0.0;
  // s1: y face
  contact_gains(pm, dY - r, &D, &kp);
  c.s1.nx = cY ? -0.0 : 0.0;  // -tYx, tYx = +0
  c.s1.ny = cY ? (tYy > 0.0 ? -1.0 : 1.0) : 0.0;
  c.s1.tx = -c.s1.ny;
  c.s1.ty = c.s1.nx;
  c.s1.kp = cY ? kp : 0.0;
  c.s1.w = cY ? D : 0.0;
  // s2: diagonal box edge
  contact_gains(pm, dD - r, &D, &kp);
  c.s2.nx = cD ? nDx : 0.0;
  c.s2.ny = cD ? nDy : 0.0;
  c.s2.tx = -c.s2.ny;
  c.s2.ty = c.s2.nx;
  c.s2.kp = cD ? kp : 0.0;
  c.s2.w = cD ? D : 0.0;
  c.n = (int)cX + (int)cY + (int)cD;
  c.roles = true;
#ifndef OGBX_MICRO_NO_GENERIC
  // rare geometry: the generic collider replaces the role slots (placed after
  // the straight-line role path rather than as an early exit: 7 % faster)
  if (__builtin_expect(slow, 0)) collide_walls_generic(pm, nbmask, H, W, x, y, fi, fj, sx, sy, c);
#endif
  return c.n;
}

__device__ __forceinline__ int collide_walls(const PointModel& pm, const uint16_t* nbmask, int H,
                                             int W, double x, double y, Contacts& c) {
  CellFrame f;
  cell_frame(pm, nbmask, H, W, x, y, f);
  return collide_in_frame(pm, nbmask, H, W, x, y, f, c);
}

// ---------------------------------------------------------------------------
// Solvers, all in u = a + B v (see the header comment):
//   f(u) = 1/2 M |u - cu|^2 + sum_s sum_e 1/2 w_se min(0, r_se)^2,
//   M = m + Df, cu = m B v / M, and for contact s with a = n.u + kp, b = t.u:
//   e0: r = a + b (weight w), e1: r = a - b (w), e2: r = a (2w).

// Exact minimiser for exactly ONE wall contact, by active-set enumeration in
// the contact frame (un = n.u, ut = t.u).  The consistent active sets are {},
// {+}, {-}, {0,+}, {0,-}, {0,+,-} ({0} alone and {+,-} without 0 are
// infeasible); each is a closed-form 2x2 solve and exactly one is consistent.
// Returns false if rounding leaves none consistent (caller falls back).
__device__ __forceinline__ bool solve_one_contact(const PointModel& pm, const Contacts& c, double cux,
                                         double cuy, double* ux, double* uy) {
#pragma clang fp contract(fast)
  const double M = pm.M;
  // exactly one slot is non-zero (the others are all-zero): sum them
  const double nx = c.s0.nx + c.s1.nx + c.s2.nx, ny = c.s0.ny + c.s1.ny + c.s2.ny;
  const double tx = c.s0.tx + c.s1.tx + c.s2.tx, ty = c.s0.ty + c.s1.ty + c.s2.ty;
  const double e = c.s0.kp + c.s1.kp + c.s2.kp, w = c.s0.w + c.s1.w + c.s2.w;
  const double cn = nx * cux + ny * cuy, ct = tx * cux + ty * cuy;
  double un = cn, ut = ct;
  bool ok = true;
#ifndef OGBX_ONE_BRANCHY
  const bool empty_ok = cn + e + ct >= 0.0 && cn + e - ct >= 0.0;  // {} is consistent
  {  // straight-line: every candidate is evaluated, the selects pick one
    const double a11 = M + 3.0 * w, a22 = M + w;
    const bool wmax = w == pm.w_max;
    const double i2 = wmax ? pm.inv_M2w : fast_recip(M + 2.0 * w);
    const double i4 = wmax ? pm.inv_M4w : fast_recip(M + 4.0 * w);
    const double idet = wmax ? pm.inv_det3 : fast_recip(a11 * a22 - w * w);
#else
  if (!(cn + e + ct >= 0.0 && cn + e - ct >= 0.0)) {  // {} is not consistent
    double i2, i4, idet;
    const double a11 = M + 3.0 * w, a22 = M + w;
    if (w == pm.w_max) {
      i2 = pm.inv_M2w;
      i4 = pm.inv_M4w;
      idet = pm.inv_det3;
    } else {
      i2 = 1.0 / (M + 2.0 * w);
      i4 = 1.0 / (M + 4.0 * w);
      idet = 1.0 / (a11 * a22 - w * w);
    }
#endif
    // {+}: rank-1 update along J = n + t (|J|^2 = 2)
    const double rp = cn + e + ct;
    const double bpn = cn - w * rp * i2, bpt = ct - w * rp * i2;
    // {-}: J = n - t
    const double rm = cn + e - ct;
    const double bmn = cn - w * rm * i2, bmt = ct + w * rm * i2;
    // {0,+} / {0,-}: [[M+3w, +-w], [+-w, M+w]] u = [M cn - 3 w e, M ct -+ w e]
    const double r1 = M * cn - 3.0 * w * e;
    const double rp2 = M * ct - w * e, rm2 = M * ct + w * e;
    const double dpn = (a22 * r1 - w * rp2) * idet, dpt = (a11 * rp2 - w * r1) * idet;
    const double dmn = (a22 * r1 + w * rm2) * idet, dmt = (a11 * rm2 + w * r1) * idet;
    // {0,+,-}: decoupled
    const double fn = (M * cn - 4.0 * w * e) * i4, ft = M * ct * i2;
    // consistency of each candidate set; the first consistent one wins
    // (selects, not a branch chain: every candidate is already computed)
    const bool kP = bpn + e + bpt < 0.0 && bpn + e - bpt >= 0.0 && bpn + e >= 0.0;
    const bool kM = bmn + e - bmt < 0.0 && bmn + e + bmt >= 0.0 && bmn + e >= 0.0;
    const bool kDP = dpn + e < 0.0 && dpn + e + dpt < 0.0 && dpn + e - dpt >= 0.0;
    const bool kDM = dmn + e < 0.0 && dmn + e - dmt < 0.0 && dmn + e + dmt >= 0.0;
    const bool kF = fn + e + ft < 0.0 && fn + e - ft < 0.0;
    un = kF ? fn : un;
    ut = kF ? ft : ut;
    un = kDM ? dmn : un;
    ut = kDM ? dmt : ut;
    un = kDP ? dpn : un;
    ut = kDP ? dpt : ut;
    un = kM ? bmn : un;
    ut = kM ? bmt : ut;
    un = kP ? bpn : un;
    ut = kP ? bpt : ut;
    ok = kP || kM || kDP || kDM || kF;
#ifndef OGBX_ONE_BRANCHY
    un = empty_ok ? cn : un;
    ut = empty_ok ? ct : ut;
    ok = ok || empty_ok;
#endif
  }
  *ux = un * nx + ut * tx;
  *uy = un * ny + ut * ty;
  return ok;
}

// Residuals, gradient and Hessian (and optionally f) at u.  Returns the
// active-edge mask.  `live` has bit s set when some lane of the wave holds a
// contact in slot s (wave-uniform): empty slots are all-zero rows (r = 0,
// never active), so skipping a slot no lane uses changes nothing.
// Role layout (kRoles): s0 is an x face, n = (s, +-0), t = (+-0, s), and s1 a
// y face, n = (+-0, q), t = (-q, +-0), with s, q in {-1, 0, 1} (0 = no
// contact, w = 0).  Their rows n+t, n-t, n then have entries in {-1, 0, 1}, so
// a, b and the residuals are the generic ones exactly, and the gradient /
// Hessian contributions collapse to sums of the weighted residuals:
//   s0: g += s*(q0+q1+q2, q0-q1),  h += (W0+W1+W2, W0-W1, W0+W1)
//   s1: g += q*(q1-q0, q0+q1+q2),  h += (W0+W1, W1-W0, W0+W1+W2)
// (q_e = W_e r_e, W_e the active weights; only the summation order differs).
template <bool kRoles>
__device__ __forceinline__ void slot_ab(const Contacts& c, int s, double ux, double uy, double* a,
                                        double* b) {
#pragma clang fp contract(fast)
  const ContactSlot& k = slot_of(c, s);
  if (kRoles && s == 0) {
    *a = k.nx * ux + k.kp;
    *b = k.nx * uy;
  } else if (kRoles && s == 1) {
    *a = k.ny * uy + k.kp;
    *b = -(k.ny * ux);
  } else {
    *a = k.nx * ux + k.ny * uy + k.kp;
    *b = k.tx * ux + k.ty * uy;
  }
}

template <bool kWithF, bool kRoles = false>
__device__ __forceinline__ uint32_t eval_piece(const PointModel& pm, const Contacts& c, uint32_t live,
                                               double cux, double cuy, double ux, double uy, double* g,
                                               double* h, double* fval) {
#pragma clang fp contract(fast)
  const double M = pm.M;
  g[0] = M * (ux - cux);
  g[1] = M * (uy - cuy);
  h[0] = M; h[1] = 0.0; h[2] = M;
  double f = 0.0;
  if (kWithF) f = 0.5 * M * ((ux - cux) * (ux - cux) + (uy - cuy) * (uy - cuy));
  uint32_t act = 0;
#pragma unroll
  for (int s = 0; s < kMaxContacts; ++s) {
    if (live & (1u << s)) {
      const ContactSlot& k = slot_of(c, s);
      double a, b;
      slot_ab<kRoles>(c, s, ux, uy, &a, &b);
      if (kRoles && !kWithF && s < 2) {
        const double r0 = a + b, r1 = a - b, r2 = a;
        const bool o0 = r0 < 0.0, o1 = r1 < 0.0, o2 = r2 < 0.0;
        const double W0 = o0 ? k.w : 0.0, W1 = o1 ? k.w : 0.0, W2 = o2 ? 2.0 * k.w : 0.0;
        act |= ((o0 ? 1u : 0u) | (o1 ? 2u : 0u) | (o2 ? 4u : 0u)) << (3 * s);
        const double q0 = W0 * r0, q1 = W1 * r1, q2 = W2 * r2;
        const double qs = q0 + q1 + q2, W01 = W0 + W1;
        if (s == 0) {
          g[0] += k.nx * qs;
          g[1] += k.nx * (q0 - q1);
          h[0] += W01 + W2;
          h[1] += W0 - W1;
          h[2] += W01;
        } else {
          g[0] += k.ny * (q1 - q0);
          g[1] += k.ny * qs;
          h[0] += W01;
          h[1] += W1 - W0;
          h[2] += W01 + W2;
        }
        continue;
      }
#pragma unroll
      for (int e = 0; e < 3; ++e) {
        const double sg = e == 0 ? 1.0 : (e == 1 ? -1.0 : 0.0);
        const double r = e == 2 ? a : a + sg * b;
        // branch-free: an inactive row contributes with weight 0
        const bool on = r < 0.0;
        const double we = on ? (e == 2 ? 2.0 * k.w : k.w) : 0.0;
        const double jx = e == 2 ? k.nx : k.nx + sg * k.tx;
        const double jy = e == 2 ? k.ny : k.ny + sg * k.ty;
        act |= (on ? 1u : 0u) << (3 * s + e);
        const double wr = we * r, wjx = we * jx;
        g[0] += wr * jx;
        g[1] += wr * jy;
        h[0] += wjx * jx;
        h[1] += wjx * jy;
        h[2] += (we * jy) * jy;
        if (kWithF) f += 0.5 * wr * r;
      }
    }
  }
  if (kWithF) *fval = f;
  return act;
}

// Active-edge mask at u only (no derivatives).
template <bool kRoles = false>
__device__ __forceinline__ uint32_t active_set(const Contacts& c, uint32_t live, double ux, double uy) {
#pragma clang fp contract(fast)
  uint32_t act = 0;
#pragma unroll
  for (int s = 0; s < kMaxContacts; ++s) {
    if (live & (1u << s)) {
      double a, b;
      slot_ab<kRoles>(c, s, ux, uy, &a, &b);
      act |= (a + b < 0.0 ? 1u : 0u) << (3 * s);
      act |= (a - b < 0.0 ? 1u : 0u) << (3 * s + 1);
      act |= (a < 0.0 ? 1u : 0u) << (3 * s + 2);
    }
  }
  return act;
}

// Several contacts: full-step semismooth Newton from the warm start *u_io
// (the previous RK stage's solution; the optimum is unique, so the start only
// changes the iteration count).  A full Newton step on the quadratic piece of
// active set A lands on that piece's minimiser; if the active set there is
// still A, the gradient of f vanishes and the point is the optimum (one
// derivative evaluation + one mask evaluation per converged stage).  Safety
// net: damped Newton with Armijo backtracking from cu (monotone, globally
// convergent).
template <bool kRoles>
__device__ __forceinline__ void solve_newton(const PointModel& pm, const Contacts& c, uint32_t live,
                                             double cux, double cuy, double* ux_io, double* uy_io) {
#pragma clang fp contract(fast)
  double ux = *ux_io, uy = *uy_io;
  double g[2], h[3], f;
  bool done = false;
  uint32_t act = eval_piece<false, kRoles>(pm, c, live, cux, cuy, ux, uy, g, h, &f);
#ifndef OGBX_NEWTON_LOOP_ONLY
  {  // OGBX_NEWTON_NFIX unconditional full steps (straight-line, no per-lane
     // exits); converged if the active set after the last step is the piece
     // it minimised
#ifndef OGBX_NEWTON_NFIX
#define OGBX_NEWTON_NFIX 2
#endif
    double idet;
#pragma unroll
    for (int it = 1; it < OGBX_NEWTON_NFIX; ++it) {
      idet = fast_recip(h[0] * h[2] - h[1] * h[1]);
      ux -= (h[2] * g[0] - h[1] * g[1]) * idet;
      uy -= (h[0] * g[1] - h[1] * g[0]) * idet;
      act = eval_piece<false, kRoles>(pm, c, live, cux, cuy, ux, uy, g, h, &f);
    }
    idet = fast_recip(h[0] * h[2] - h[1] * h[1]);
    const double vx = ux - (h[2] * g[0] - h[1] * g[1]) * idet;
    const double vy = uy - (h[0] * g[1] - h[1] * g[0]) * idet;
    const bool conv = (g[0] == 0.0 && g[1] == 0.0) || active_set<kRoles>(c, live, vx, vy) == act;
    ux = (g[0] == 0.0 && g[1] == 0.0) ? ux : vx;
    uy = (g[0] == 0.0 && g[1] == 0.0) ? uy : vy;
    done = conv;
    if (__any(!done)) act = eval_piece<false, kRoles>(pm, c, live, cux, cuy, ux, uy, g, h, &f);
  }
#endif
#pragma unroll 1
  for (int it = 0; it < 8 && !done; ++it) {
    OGBX_STAT(4);
    OGBX_WSTAT(13, true);
    if (g[0] == 0.0 && g[1] == 0.0) {
      done = true;
      break;
    }
    const double idet = fast_recip(h[0] * h[2] - h[1] * h[1]);  // det >= M^2 > 0
    ux -= (h[2] * g[0] - h[1] * g[1]) * idet;
    uy -= (h[0] * g[1] - h[1] * g[0]) * idet;
    if (active_set<kRoles>(c, live, ux, uy) == act) {
      done = true;
      break;
    }
    act = eval_piece<false, kRoles>(pm, c, live, cux, cuy, ux, uy, g, h, &f);
  }
  if (!done) {
    OGBX_STAT(5);
    ux = cux;
    uy = cuy;
#pragma unroll 1
    for (int it = 0; it < 64; ++it) {
      eval_piece<true>(pm, c, live, cux, cuy, ux, uy, g, h, &f);
      const double idet = 1.0 / (h[0] * h[2] - h[1] * h[1]);
      const double px = -(h[2] * g[0] - h[1] * g[1]) * idet;
      const double py = -(h[0] * g[1] - h[1] * g[0]) * idet;
      if (fabs(px) + fabs(py) <= 1e-16 * (1.0 + fabs(ux) + fabs(uy))) break;
      const double slope = g[0] * px + g[1] * py;
      double t = 1.0, g2[2], h2[3], f2;
#pragma unroll 1
      for (int bt = 0; bt < 60; ++bt) {
        eval_piece<true>(pm, c, live, cux, cuy, ux + t * px, uy + t * py, g2, h2, &f2);
        if (f2 <= f + 1e-6 * t * slope) break;
        t *= 0.5;
      }
      ux += t * px;
      uy += t * py;
    }
  }
  *ux_io = ux;
  *uy_io = uy;
}

// qacc of the point mass at velocity (vx, vy) for the given wall contacts.
// (wx, wy): warm start for the multi-contact Newton (previous stage's u);
// on return it holds this stage's u.  The solver path is chosen per WAVE: if
// any lane has >= 2 contacts every contact lane runs Newton (which also solves
// single contacts exactly); otherwise the closed form runs.  One path per wave
// and stage keeps SIMT from executing the union of both.
__device__ __forceinline__ void solve_acc(const PointModel& pm, const Contacts& c, double vx,
                                          double vy, double* ax_out, double* ay_out, double* wx,
                                          double* wy) {
#pragma clang fp contract(fast)
  const double bvx = pm.B * vx, bvy = pm.B * vy;
  const double cux = pm.m_over_M * bvx, cuy = pm.m_over_M * bvy;  // floor-only minimiser
  double ux = cux, uy = cuy;
  OGBX_STAT(c.n);
  bool need_newton;
  OGBX_WSTAT(9, true);
  OGBX_WSTAT(8, c.n >= 2);
#ifndef OGBX_CLOSED_FORM
  // Every lane runs the (warm-started, straight-line) Newton solve, contact or
  // not: the per-wave choice of the closed form for single-contact-only waves
  // (25 % of wave-stages) cost more in branches than it saved (measured 4 %).
  if (true) {
    need_newton = true;
    ux = c.n >= 1 ? *wx : cux;
    uy = c.n >= 1 ? *wy : cuy;
  } else
#endif
  if (__any(c.n >= 2)) {
    need_newton = c.n >= 1;
    ux = c.n >= 1 ? *wx : cux;
    uy = c.n >= 1 ? *wy : cuy;
  } else {
    need_newton = false;
    if (c.n == 1) need_newton = !solve_one_contact(pm, c, cux, cuy, &ux, &uy);
#ifdef OGBX_ABLATE_NEWTON
    need_newton = false;
#endif
  }
  if (need_newton) {
    // Every slot is evaluated: an empty slot is an all-zero row (r = 0, never
    // active, no contribution).  Skipping slots no lane uses (three ballots and
    // a uniform branch per slot and evaluation) measured 17 % slower: the
    // branches break the straight-line schedule of the evaluations.
#ifdef OGBX_LIVE_BALLOTS
    const uint32_t live = (__any(c.s0.w != 0.0) ? 1u : 0u) | (__any(c.s1.w != 0.0) ? 2u : 0u) |
                          (__any(c.s2.w != 0.0) ? 4u : 0u);
#else
    constexpr uint32_t live = 7u;
#endif
#ifdef OGBX_NO_ROLE_EVAL
    solve_newton<false>(pm, c, live, cux, cuy, &ux, &uy);
#else
#ifdef OGBX_ABL_ROLES_ONLY
    solve_newton<true>(pm, c, live, cux, cuy, &ux, &uy);
#else
    if (__any(!c.roles)) solve_newton<false>(pm, c, live, cux, cuy, &ux, &uy);
    else solve_newton<true>(pm, c, live, cux, cuy, &ux, &uy);
#endif
#endif
  }
  *wx = ux;
  *wy = uy;
  *ax_out = ux - bvx;
  *ay_out = uy - bvy;
}

// One PointEnv step starting from qpos + delta with qvel = 0.  Returns 1 if a
// wall contact was present at the start (slow path taken).
// The 5 substeps x 4 RK stages run as one loop of 20 force evaluations so the
// solver is instantiated once (mj_step -> mj_forward + mj_RungeKutta(N=4),
// RK4_A = {1/2 ; 0, 1/2 ; 0, 0, 1}, RK4_B = {1/6, 1/3, 1/3, 1/6}).
__device__ __forceinline__ int point_step(const PointModel& pm, const uint16_t* wall, int H, int W,
                                 double* px, double* py) {
  double x = *px, y = *py;
  Contacts c;
  CellFrame fr;
  OGBX_STAMP_DECL
  cell_frame(pm, wall, H, W, x, y, fr);
  const bool in_contact = collide_in_frame(pm, wall, H, W, x, y, fr, c) != 0;
#ifdef OGBX_MASKED_FREE
  if (!in_contact) {
#else
  // Free lanes of a wave with a contact lane run the contact loop too (their
  // result is discarded below): gfx950 issues a dependent VALU chain about 2x
  // slower when only a few lanes of the wave are active (<= 8 for fp64 ops,
  // <= 16 for 32-bit ops; scripts/micro/lane_count.hip), and the contact loop
  // is exactly such a chain.  The chain length, not the lane count, sets the
  // wave's time, so the extra lanes cost nothing.
  if (!__any(in_contact)) {
#endif
    *px = x + 0.0;
    *py = y + 0.0;
    OGBX_STAMP_END;
    return 0;
  }
  const double x0 = x, y0 = y;
  const double h = pm.h;
  double vx = 0.0, vy = 0.0;                          // X[0] velocity of the substep
  double qsx = x, qsy = y, vsx = 0.0, vsy = 0.0;      // state of the current RK stage
  double sqx = 0.0, sqy = 0.0, svx = 0.0, svy = 0.0;  // B-weighted sums (dX)
  double wux = 0.0, wuy = 0.0;                        // solver warm start (u)
#ifdef OGBX_ABLATE_STAGES
  const int nstage = OGBX_ABLATE_STAGES;
#else
  const int nstage = 4 * pm.nsub;
#endif
  OGBX_STAT(6);
#ifndef OGBX_STAGE_UNROLL
// Unrolled by the RK stage count: the stage index (and its A/B coefficients,
// the e != 0 collide test) become constants (1.71 -> 1.77 G env-steps/s).
#define OGBX_STAGE_UNROLL 4
#endif
#pragma unroll OGBX_STAGE_UNROLL
  for (int e = 0; e < nstage; ++e) {
    const int st = e & 3;
    double fx, fy;
#ifndef OGBX_ABLATE_COLLIDE
    if (e != 0) {
      if (__builtin_expect(!cell_frame_valid(pm, fr, qsx, qsy), 0)) cell_frame(pm, wall, H, W, qsx, qsy, fr);
      collide_in_frame(pm, wall, H, W, qsx, qsy, fr, c);
    }
#endif
    OGBX_STAMP_SEG(_ta);
    solve_acc(pm, c, vsx, vsy, &fx, &fy, &wux, &wuy);
    OGBX_STAMP_SEG(_tb);
    {
#pragma clang fp contract(fast)
    const double b = (st == 0 || st == 3) ? (1.0 / 6.0) : (1.0 / 3.0);
    sqx = sqx + b * vsx;
    sqy = sqy + b * vsy;
    svx = svx + b * fx;
    svy = svy + b * fy;
    if (st < 3) {
      const double cf = (st < 2) ? 0.5 : 1.0;
      qsx = x + h * (cf * vsx);
      qsy = y + h * (cf * vsy);
      vsx = vx + (cf * fx) * h;
      vsy = vy + (cf * fy) * h;
    } else {
      // mj_advance: qvel += h*dX_acc ; qpos += h*dX_vel
      vx = vx + svx * h;
      vy = vy + svy * h;
      x = x + h * sqx;
      y = y + h * sqy;
      qsx = x;
      qsy = y;
      vsx = vx;
      vsy = vy;
      sqx = sqy = svx = svy = 0.0;
    }
    }
    OGBX_STAMP_SEG(_tc);
  }
  OGBX_STAMP_END;
  // lanes that started free keep the exact free step (qpos + 0.0)
  *px = in_contact ? x : x0 + 0.0;
  *py = in_contact ? y : y0 + 0.0;
  return in_contact ? 1 : 0;
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
