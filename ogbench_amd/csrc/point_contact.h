// point_contact.h -- the pointmaze contact step, active-set form (default).
//
// Same model and the same RK4 stage loop as point_physics.h (whose header
// states every assumed MuJoCo default; wall-contact parity is pinned to
// MuJoCo's published formulation by tests/mjmodel_np.py, not to MuJoCo's
// output), with a much shorter per-stage instruction stream.  The step
// kernel runs one wave per SIMD and every wave that holds a contact lane runs
// the whole 20-stage chain, so the launch time is the instruction count (and
// dependency depth) of one stage x 20:
//
//   * Solver.  The optimum u* of
//       f(u) = 1/2 M |u - cu|^2 + sum_s sum_e 1/2 w_s c_e min(0, r_se)^2
//     (c_e = 1, 1, 2 for the edges n+t, n-t, n of contact slot s) is the
//     minimiser of the quadratic piece of its own active-edge set A.  Each
//     iteration BUILDS that piece's normal equations from A,
//       (M I + sum_s w_s [S nn' + T tt' + D (nt' + tn')]) u = M cu - sum_s w_s kp_s (S n + D t),
//       T = a0 + a1, D = a0 - a1, S = T + 2 a2   (a_e = 1 if edge e of s is in A),
//     solves the 2x2 system and evaluates the mask A' at the solution; A' == A
//     certifies the optimum (the piece's gradient vanishes and the activity is
//     consistent), otherwise A := A' (one full semismooth Newton step, as in
//     point_physics.h).  The mask carries over between RK stages and substeps,
//     where it rarely changes, and so do its integer weights (S, T, D), so a
//     stage costs one build + solve + mask (measured: 10 % of wave-stages
//     iterate again).  point_physics.h instead evaluated gradient and Hessian
//     at two iterates and a mask at a third.
//   * Collision.  With the centre inside the inner part of an empty cell
//     (|offset| < 0.49975 unit, checked per stage; otherwise the generic
//     collider of point_physics.h runs), the three candidate boxes have fixed
//     roles: x face, y face, diagonal vertical edge.  The face distance is
//     fl(-s h - p) (the clamp always saturates on the contact side), the
//     diagonal box reuses both face offsets, slot fields are written without
//     selects (an invalid slot is excluded by the validity mask), and the
//     impedance transition band (|dist| < 1e-3) is one wave-uniform branch.
//
// Results agree with point_physics.h and the oracle to rounding (the solve is
// H^-1 rhs instead of u - H^-1 g); contact flags and free-space steps are
// bit-identical (same closest-point arithmetic as the oracle).
#pragma once

#include "point_physics.h"

// Stage-loop unroll (both the lean and the full loop of point_step_as): fully
// unrolled, 20 stages.  Measured per launch at N = 65,536: 17.5 us; unroll 4
// 18.0, 8 18.2, 2 18.9; lean loop 20 with the full loop 4: 18.3.
// Active-set iterations of the lean loop before a lane bails to the full loop.
// Full-loop active-set iterations before the damped-Newton safety net.  The
// lean loop must not iterate longer: a lane it accepts after more iterations
// would be one the full loop hands to armijo_newton, and its result would
// depend on which loop its wave ran.
#define OGBX_FULL_ITERS 7
#ifndef OGBX_LEAN_ITERS
#define OGBX_LEAN_ITERS OGBX_FULL_ITERS
#endif
static_assert(OGBX_LEAN_ITERS <= OGBX_FULL_ITERS, "lean loop may not iterate longer than the full loop");
#ifndef OGBX_AS_UNROLL
#define OGBX_AS_UNROLL 20
#endif

namespace ogbx {

// Edge bits of slot s: 3s (n+t), 3s+1 (n-t), 3s+2 (n, weight 2w).
constexpr uint32_t kSlotBits = 7u;

// The cell of the sphere centre (floor of the reference's xy_to_ij
// arithmetic), with the 3x3 wall mask (own-cell bit cleared).  slow: off the
// map or in a wall cell -- the role collider does not apply.  The frame stays
// valid while the centre is within the cell's half size (|offset| < unit/2):
// every box the sphere can touch is then in its 3x3 neighbourhood and the
// side-box clamps saturate, even where floor() would name the neighbour cell.
struct RoleFrame {
  double cx, cy, fi, fj;
  uint32_t m;
  bool slow;
};

__device__ __forceinline__ void role_frame(const PointModel& pm, const uint16_t* nbmask, int H, int W, double x,
                                           double y, RoleFrame& f) {
  f.fi = floor((y + pm.off_y + 0.5 * pm.unit) * pm.inv_unit);
  f.fj = floor((x + pm.off_x + 0.5 * pm.unit) * pm.inv_unit);
  f.cx = f.fj * pm.unit - pm.off_x;
  f.cy = f.fi * pm.unit - pm.off_y;
  const bool inside = f.fi >= 0.0 && f.fi < (double)H && f.fj >= 0.0 && f.fj < (double)W;
  const uint32_t m = inside ? nbmask[(int)f.fi * W + (int)f.fj] : 0x1FFu;
  f.slow = !inside | ((m >> 4) & 1u);
  f.m = m & ~0x10u;
}

// Slot data of one stage in the role layout (s0 x face n = (nx, 0), s1 y face
// n = (0, ny), s2 diagonal edge; t = perp(n)).  Returns the validity mask.
__device__ __forceinline__ uint32_t collide_roles(const PointModel& pm, const RoleFrame& f, double x, double y,
                                                  Contacts& c, bool* slow) {
  const double lx = x - f.cx, ly = y - f.cy;
  // centre exactly on (or, by rounding, past) the cell's edge: generic collider
  *slow = f.slow | !(fabs(lx) < pm.box_hxy) | !(fabs(ly) < pm.box_hxy);
  const double reach = pm.box_hxy - pm.radius - 1e-9;
  const int sx = lx >= reach ? 1 : (lx <= -reach ? -1 : 0);
  const int sy = ly >= reach ? 1 : (ly <= -reach ? -1 : 0);
  const double sxd = (double)sx, syd = (double)sy;
  const double hx = pm.box_hxy, r = pm.radius;
  // neighbour walls (own-cell bit cleared, so a zero side reads 0)
  const uint32_t vX = (f.m >> (4 + sx)) & 1u;
  const uint32_t vY = (f.m >> (4 + 3 * sy)) & 1u;
  const uint32_t vD = (f.m >> (4 + 3 * sy + sx)) & (uint32_t)(sx & sy) & 1u;
  // closest point of the side box: its face at -s*h (the clamp saturates);
  // the same two roundings as the oracle's cl - (c - b)
  const double px = x - fma(sxd, pm.unit, f.cx), py = y - fma(syd, pm.unit, f.cy);
  const double tx = fma(-sxd, hx, -px), ty = fma(-syd, hx, -py);
  const double dist0 = fabs(tx) - r, dist1 = fabs(ty) - r;
  const double d2 = tx * tx + ty * ty;
  const bool cX = vX & (dist0 <= 0.0);
  const bool cY = vY & (dist1 <= 0.0);
  // fl(sqrt(d2)) - r > 0 decided exactly on d2 (kPointFarD2, point_physics.h)
  const bool cD = vD & !(d2 > kPointFarD2);
  // diagonal box: distance and normal from v_rsq_f64 + one Newton-Raphson step
  const double dq = fmax(d2, 1e-300);
  const double y0 = __builtin_amdgcn_rsq(dq);
  const double inv = y0 * fma(-0.5 * dq * y0, y0, 1.5);
  const double dist2 = dq * inv - r;
  c.s0.nx = __builtin_copysign(1.0, -tx);
  c.s0.ny = 0.0;
  c.s1.nx = 0.0;
  c.s1.ny = __builtin_copysign(1.0, -ty);
  c.s2.nx = -tx * inv;
  c.s2.ny = -ty * inv;
  c.s0.kp = pm.kp_max * dist0;
  c.s1.kp = pm.kp_max * dist1;
  c.s2.kp = pm.kp_max * dist2;
  // an invalid slot has weight 0: its (stale) mask bits and piece weights
  // then contribute nothing, so the weights need no per-stage refresh
  c.s0.w = cX ? pm.w_max : 0.0;
  c.s1.w = cY ? pm.w_max : 0.0;
  c.s2.w = cD ? pm.w_max : 0.0;
  // impedance transition band (point_physics.h contact_gains), wave-uniform
  const double iw = pm.inv_width;
  const bool b0 = cX & (fabs(dist0) * iw < 1.0), b1 = cY & (fabs(dist1) * iw < 1.0),
             b2 = cD & (fabs(dist2) * iw < 1.0);
  OGBX_WSTAT(10, b0 | b1 | b2);
  OGBX_WSTAT(11, cD);
#ifndef OGBX_ABL_NOBAND
  if (__builtin_expect(__any(b0 | b1 | b2), 0)) {
#else
  if (false) {
#endif
    if (b0) contact_gains(pm, dist0, &c.s0.w, &c.s0.kp);
    if (b1) contact_gains(pm, dist1, &c.s1.w, &c.s1.kp);
    if (b2) contact_gains(pm, dist2, &c.s2.w, &c.s2.kp);
  }
  c.n = (int)cX + (int)cY + (int)cD;
  c.roles = true;
  return (cX ? kSlotBits : 0u) | (cY ? kSlotBits << 3 : 0u) | (cD ? kSlotBits << 6 : 0u);
}

// Tangents of the role slots (t = perp(n)), for the generic evaluation when
// some lane of the wave took the generic collider.
__device__ __forceinline__ void role_tangents(Contacts& c) {
  c.s0.tx = -c.s0.ny; c.s0.ty = c.s0.nx;
  c.s1.tx = -c.s1.ny; c.s1.ty = c.s1.nx;
  c.s2.tx = -c.s2.ny; c.s2.ty = c.s2.nx;
}

// Integer weights of a mask, per slot: S = a0 + a1 + 2 a2, T = a0 + a1,
// D = a0 - a1 (as doubles).
struct PieceWeights {
  double S0, T0, D0, S1, T1, D1, S2, T2, D2;
};

__device__ __forceinline__ void piece_weights(uint32_t A, PieceWeights& p) {
  auto one = [&](int s, double& S, double& T, double& D) {
    const int a0 = (A >> (3 * s)) & 1, a1 = (A >> (3 * s + 1)) & 1, a2 = (A >> (3 * s + 2)) & 1;
    T = (double)(a0 + a1);
    D = (double)(a0 - a1);
    S = (double)(a0 + a1 + 2 * a2);
  };
  one(0, p.S0, p.T0, p.D0);
  one(1, p.S1, p.T1, p.D1);
  one(2, p.S2, p.T2, p.D2);
}

// a = n.u + kp and b = t.u of slot s.
template <bool kRoles>
__device__ __forceinline__ void slot_res(const Contacts& c, int s, double ux, double uy, double* a, double* b) {
#pragma clang fp contract(fast)
  const ContactSlot& k = slot_of(c, s);
  if (kRoles && s == 0) {
    *a = k.nx * ux + k.kp;
    *b = k.nx * uy;
  } else if (kRoles && s == 1) {
    *a = k.ny * uy + k.kp;
    *b = -(k.ny * ux);
  } else if (kRoles) {
    *a = k.nx * ux + (k.ny * uy + k.kp);
    *b = k.nx * uy - k.ny * ux;
  } else {
    *a = k.nx * ux + (k.ny * uy + k.kp);
    *b = k.tx * ux + k.ty * uy;
  }
}

// Active-edge mask at u (residual < 0: a + b < 0, a - b < 0, a < 0); the
// bits of invalid slots are meaningless (callers mask them).
template <bool kRoles>
__device__ __forceinline__ uint32_t edge_mask(const Contacts& c, double ux, double uy) {
  uint32_t act = 0;
#pragma unroll
  for (int s = 0; s < kMaxContacts; ++s) {
    double a, b;
    slot_res<kRoles>(c, s, ux, uy, &a, &b);
    act |= (a < -b ? 1u : 0u) << (3 * s);
    act |= (a < b ? 2u : 0u) << (3 * s);
    act |= (a < 0.0 ? 4u : 0u) << (3 * s);
  }
  return act;
}

// Minimiser of the quadratic piece with weights p (see the header).
// mbv = m B v (= M cu).
template <bool kRoles>
__device__ __forceinline__ void piece_min(const PointModel& pm, const Contacts& c, const PieceWeights& p,
                                          double mbvx, double mbvy, double* ux, double* uy) {
#pragma clang fp contract(fast)
  const double M = pm.M;
  double h00, h01, h11, r0, r1;
  if (kRoles) {
    const double w0 = c.s0.w, w1 = c.s1.w, w2 = c.s2.w;
    // faces: x face adds (S, T, D) to (h00, h11, h01), y face (T, S, -D)
    h00 = M + w0 * p.S0 + w1 * p.T1;
    h11 = M + w0 * p.T0 + w1 * p.S1;
    h01 = w0 * p.D0 - w1 * p.D1;
    const double g0 = (w0 * c.s0.kp) * c.s0.nx, g1 = (w1 * c.s1.kp) * c.s1.ny;
    r0 = mbvx - g0 * p.S0 + g1 * p.D1;
    r1 = mbvy - g0 * p.D0 - g1 * p.S1;
    // diagonal edge, t = (-ny, nx)
    const double nx = c.s2.nx, ny = c.s2.ny;
    const double q = nx * nx, s = ny * ny, o = nx * ny;
    const double WS = w2 * p.S2, WT = w2 * p.T2, WD = w2 * p.D2;
    h00 += WS * q + WT * s - 2.0 * (WD * o);
    h11 += WS * s + WT * q + 2.0 * (WD * o);
    h01 += (WS - WT) * o + WD * (q - s);
    const double k2 = c.s2.kp;
    r0 -= k2 * (WS * nx - WD * ny);
    r1 -= k2 * (WS * ny + WD * nx);
  } else {
    h00 = M;
    h11 = M;
    h01 = 0.0;
    r0 = mbvx;
    r1 = mbvy;
#pragma unroll
    for (int s = 0; s < kMaxContacts; ++s) {
      const ContactSlot& k = slot_of(c, s);
      const double S = k.w * (s == 0 ? p.S0 : (s == 1 ? p.S1 : p.S2));
      const double T = k.w * (s == 0 ? p.T0 : (s == 1 ? p.T1 : p.T2));
      const double D = k.w * (s == 0 ? p.D0 : (s == 1 ? p.D1 : p.D2));
      h00 += S * (k.nx * k.nx) + T * (k.tx * k.tx) + 2.0 * D * (k.nx * k.tx);
      h11 += S * (k.ny * k.ny) + T * (k.ty * k.ty) + 2.0 * D * (k.ny * k.ty);
      h01 += S * (k.nx * k.ny) + T * (k.tx * k.ty) + D * (k.nx * k.ty + k.ny * k.tx);
      r0 -= k.kp * (S * k.nx + D * k.tx);
      r1 -= k.kp * (S * k.ny + D * k.ty);
    }
  }
  const double idet = fast_recip(h00 * h11 - h01 * h01);  // det >= M^2 > 0
  *ux = (h11 * r0 - h01 * r1) * idet;
  *uy = (h00 * r1 - h01 * r0) * idet;
}

// Safety net after 8 active-set iterations: damped Newton with Armijo
// backtracking from cu (monotone, globally convergent; point_physics.h).
// Never seen in the bench states.  (Out of line, with the generic collider,
// the kernel is 3.5x smaller but 60 % slower: the call ABI costs registers.)
template <bool kRoles>
__device__ __forceinline__ void armijo_newton(const PointModel& pm, const Contacts& c, uint32_t valid, double cux,
                                              double cuy, double* ux_out, double* uy_out) {
  // explicit rows for eval_piece: tangents of role slots, invalid slots zeroed
  Contacts z = c;
  if (kRoles) role_tangents(z);
  if (!(valid & kSlotBits)) zero_slot(z.s0);
  if (!(valid & (kSlotBits << 3))) zero_slot(z.s1);
  if (!(valid & (kSlotBits << 6))) zero_slot(z.s2);
  double g[2], h[3], f;
  double ux = cux, uy = cuy;
#pragma unroll 1
  for (int it = 0; it < 64; ++it) {
    eval_piece<true>(pm, z, 7u, cux, cuy, ux, uy, g, h, &f);
    const double idet = 1.0 / (h[0] * h[2] - h[1] * h[1]);
    const double px = -(h[2] * g[0] - h[1] * g[1]) * idet;
    const double py = -(h[0] * g[1] - h[1] * g[0]) * idet;
    if (fabs(px) + fabs(py) <= 1e-16 * (1.0 + fabs(ux) + fabs(uy))) break;
    const double slope = g[0] * px + g[1] * py;
    double t = 1.0, g2[2], h2[3], f2;
#pragma unroll 1
    for (int bt = 0; bt < 60; ++bt) {
      eval_piece<true>(pm, z, 7u, cux, cuy, ux + t * px, uy + t * py, g2, h2, &f2);
      if (f2 <= f + 1e-6 * t * slope) break;
      t *= 0.5;
    }
    ux += t * px;
    uy += t * py;
  }
  *ux_out = ux;
  *uy_out = uy;
}

// u* by active-set iteration from the mask *act_io (the previous stage's
// final build mask; pw holds its weights).  Only the valid slots' bits count:
// an invalid slot has w = 0, so whatever its bits and weights, it contributes
// nothing, and its bits are a harmless warm start if the contact reappears.
// On return *act_io is the mask of the converged build (pw its weights).
// One iteration for every lane (straight line), more only while some lane's
// mask still changes; after 8, the damped Newton finishes the lane.
// kBail: a lane still unconverged after the iterations sets *bail instead of
// running the damped Newton (the caller redoes the step with the full loop).
template <bool kRoles, bool kBail = false>
__device__ __forceinline__ void solve_active_set(const PointModel& pm, const Contacts& c, uint32_t valid,
                                                 double vx, double vy, uint32_t* act_io, PieceWeights& pw,
                                                 double* ux_out, double* uy_out, bool* bail = nullptr) {
#pragma clang fp contract(fast)
  const double mB = pm.mass * pm.B;
  const double mbvx = mB * vx, mbvy = mB * vy;
  uint32_t A = *act_io;
  double ux, uy;
  piece_min<kRoles>(pm, c, pw, mbvx, mbvy, &ux, &uy);
  uint32_t A2 = edge_mask<kRoles>(c, ux, uy);
  bool done = ((A2 ^ A) & valid) == 0u;
  OGBX_WSTAT(9, true);
  OGBX_WSTAT(13, !done);
#ifndef OGBX_ABL_NODONE
  if (__builtin_expect(__any(!done), 0)) {
#else
  if (false) {
#endif
#pragma unroll 1
    for (int it = 0; it < (kBail ? OGBX_LEAN_ITERS : OGBX_FULL_ITERS) && !done; ++it) {
      OGBX_STAT(4);
      A = A2 & valid;
      piece_weights(A, pw);
      piece_min<kRoles>(pm, c, pw, mbvx, mbvy, &ux, &uy);
      A2 = edge_mask<kRoles>(c, ux, uy);
      done = ((A2 ^ A) & valid) == 0u;
    }
    if (kBail) {
      *bail |= !done;
    } else if (!done) {
      OGBX_STAT(5);
      armijo_newton<kRoles>(pm, c, valid, mbvx / pm.M, mbvy / pm.M, &ux, &uy);
      A = edge_mask<kRoles>(c, ux, uy) & valid;
      piece_weights(A, pw);
    }
  }
  *act_io = A;
  *ux_out = ux;
  *uy_out = uy;
}

// Contacts at a stage: the role collider, or (rare) the generic collider for
// the lanes whose frame is slow, whose slots then hold contacts 0..n-1 with
// explicit tangents (empty slots zero rows).  Returns the validity mask;
// *generic tells which evaluation THIS LANE uses: the choice is per lane (the
// wave runs both evaluations when it holds both kinds), so a lane's result
// never depends on which envs share its wavefront.
__device__ __forceinline__ uint32_t stage_contacts(const PointModel& pm, const uint16_t* wall, int H, int W,
                                                   double x, double y, const RoleFrame& fr, Contacts& c,
                                                   bool* generic) {
  bool slow;
  uint32_t valid = collide_roles(pm, fr, x, y, c, &slow);
  *generic = slow;
  OGBX_WSTAT(12, slow);
#ifndef OGBX_ABL_NOSLOW
  if (__builtin_expect(__any(slow), 0)) {
#else
  if (false) {
#endif
#ifdef OGBX_WAVE_BAIL  // A/B: the round-2 wave-level choice
    *generic = true;
    role_tangents(c);
#endif
    if (slow) {
      role_tangents(c);
      const double lx = x - fr.cx, ly = y - fr.cy;
      const double reach = pm.box_hxy - pm.radius - 1e-9;
      const int sx = lx >= reach ? 1 : (lx <= -reach ? -1 : 0);
      const int sy = ly >= reach ? 1 : (ly <= -reach ? -1 : 0);
      const int n = collide_walls_generic(pm, wall, H, W, x, y, fr.fi, fr.fj, sx, sy, c);
      valid = n >= 3 ? 0x1FFu : (n == 2 ? 0x3Fu : (n == 1 ? 0x7u : 0u));
    }
  }
  return valid;
}

// The 20-stage RK4 contact loop of one step from (x, y), whose first stage's
// frame, contacts and collider choice the caller has computed.
// kLean: the loop without the frame-refresh and generic-collider branches
// (no lane's centre leaves its cell's inner part during the step: 0 % of the
// bench's wave-stages) and without the damped-Newton safety net (never seen).  Instead of taking them it sets *bail on the lanes
// that would have, and the caller redoes the step with the full loop; when
// no lane bails, both loops execute the same arithmetic.
template <bool kLean>
__device__ __forceinline__ void contact_loop(const PointModel& pm, const uint16_t* wall, int H, int W, double& x,
                                             double& y, RoleFrame fr, Contacts c, uint32_t valid, bool generic,
                                             bool* bail) {
  bool bl = false;
  const double h = pm.h;
  double vx = 0.0, vy = 0.0;
  double qsx = x, qsy = y, vsx = 0.0, vsy = 0.0;
  double sqx = 0.0, sqy = 0.0, svx = 0.0, svy = 0.0;
  // first stage: v = 0, so the mask at u = cu = 0 (every edge of a penetrating
  // contact) starts the iteration one step ahead of the empty set
  uint32_t act = edge_mask<true>(c, 0.0, 0.0) & valid;
  PieceWeights pw;
  piece_weights(act, pw);
  const int nstage = 4 * pm.nsub;
#pragma unroll OGBX_AS_UNROLL
  for (int e = 0; e < nstage; ++e) {
    const int st = e & 3;
    if (e != 0) {
      const double lim = 0.5 * pm.unit;
      const bool stale = !(fabs(qsx - fr.cx) <= lim) | !(fabs(qsy - fr.cy) <= lim);
      if (kLean) {
        bool slow;
        valid = collide_roles(pm, fr, qsx, qsy, c, &slow);
        bl |= stale | slow;
      } else {
#ifndef OGBX_ABL_NOSTALE
        if (__builtin_expect(__any(stale), 0)) {
          if (stale) role_frame(pm, wall, H, W, qsx, qsy, fr);
        }
#endif
        valid = stage_contacts(pm, wall, H, W, qsx, qsy, fr, c, &generic);
      }
    }
    double fx, fy;
    {
#pragma clang fp contract(fast)
      double ux, uy;
      if (kLean) solve_active_set<true, true>(pm, c, valid, vsx, vsy, &act, pw, &ux, &uy, &bl);
      else if (generic) solve_active_set<false>(pm, c, valid, vsx, vsy, &act, pw, &ux, &uy);
      else solve_active_set<true>(pm, c, valid, vsx, vsy, &act, pw, &ux, &uy);
      fx = ux - pm.B * vsx;
      fy = uy - pm.B * vsy;
    }
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
  }
  *bail = bl;
}

// ---------------------------------------------------------------------------
// Pipelined lean loop (default lean form; -DOGBX_LEAN_SERIAL restores
// contact_loop<true>).
//
// In the RK4 stage loop the NEXT stage's position never depends on the current
// stage's solve: qs(e+1) = x + h cf vs(e) inside a substep and x + h sum(b vs)
// at its end, both known before the acceleration of stage e.  So stage e+1's
// collision runs beside stage e's solve, and the two rare per-stage paths --
// an active set that changes (stage e) and an impedance-band contact (stage
// e+1) -- share ONE wave-uniform branch per stage instead of a branch in each
// half.  One basic block per stage gives the scheduler two independent fp64
// chains to interleave; serial, every branch drained the pipeline between
// collision and solve.
//
// The lookahead collider keeps the role layout with the side of every role
// fixed for the step: sx = sign(lx), sy = sign(ly) of the first stage's
// centre (the face normals are then (-sx, 0) and (0, -sy) for the whole step).
// That equals collide_roles' choice at every stage: where collide_roles picks
// side 0 (|l| < h - r) the fixed side's face and corner are out of reach
// (dist > 1e-9), so both see no contact there.  The face distance is
// (h - sx lx) - r, the corner distance sqrt(ex^2 + ey^2) - r with ex = h - sx lx;
// both equal collide_roles' to rounding.  (The first stage -- whose contact
// flag is the reported one -- still comes from the exact stage_contacts.)
// A lane bails to the full loop when its centre leaves the inner part of its
// cell (|l| >= h) or crosses to the far side of its step-start half
// (sx lx <= -1.25, never reachable in a step: contacts move the centre by a
// fraction of their penetration), or when its active set does not settle in
// OGBX_LEAN_ITERS iterations.
struct LeanSides {
  double cx, cy, sxd, syd;
  // per-side radius: r where the side holds a wall, -1e3 where it does not
  // (the distance is then far positive: no contact, no compare against the
  // wall bit); rD likewise and the corner's squared-distance bound
  double rX, rY, rD, farD2;
  double wX, wY, wD;  // w_max on a wall side, 0 elsewhere
  uint32_t bX, bY, bD;  // the slot's edge bits on a wall side
};

__device__ __forceinline__ LeanSides lean_sides(const PointModel& pm, const RoleFrame& fr, double x, double y) {
  LeanSides L;
  L.cx = fr.cx;
  L.cy = fr.cy;
  const bool px = x - fr.cx >= 0.0, py = y - fr.cy >= 0.0;
  L.sxd = px ? 1.0 : -1.0;
  L.syd = py ? 1.0 : -1.0;
  const int sx = px ? 1 : -1, sy = py ? 1 : -1;
  const bool vX = (fr.m >> (4 + sx)) & 1u, vY = (fr.m >> (4 + 3 * sy)) & 1u, vD = (fr.m >> (4 + 3 * sy + sx)) & 1u;
  L.rX = vX ? pm.radius : -1e3;
  L.rY = vY ? pm.radius : -1e3;
  L.rD = vD ? pm.radius : -1e3;
  L.farD2 = vD ? kPointFarD2 : -1.0;
  L.wX = vX ? pm.w_max : 0.0;
  L.wY = vY ? pm.w_max : 0.0;
  L.wD = vD ? pm.w_max : 0.0;
  L.bX = vX ? kSlotBits : 0u;
  L.bY = vY ? kSlotBits << 3 : 0u;
  L.bD = vD ? kSlotBits << 6 : 0u;
  return L;
}

// Distances of the three role slots at (x, y).  emin/emax track the smallest
// and largest face offset e = h - s l over the step (bail test at the end:
// every stage needs 0 < e < h + 1.25).
struct LeanHit {
  double d0, d1, d2, ex, ey, inv;
  bool cX, cY, cD, band;
};

__device__ __forceinline__ void lean_collide(const PointModel& pm, const LeanSides& L, double x, double y,
                                             LeanHit& k, double& emin, double& emax) {
  const double hx = pm.box_hxy;
  const double lx = x - L.cx, ly = y - L.cy;
  k.ex = fma(-L.sxd, lx, hx);  // h - sx lx (sx = +-1: one rounding)
  k.ey = fma(-L.syd, ly, hx);
  emin = fmin(emin, fmin(k.ex, k.ey));
  emax = fmax(emax, fmax(k.ex, k.ey));
  k.d0 = k.ex - L.rX;
  k.d1 = k.ey - L.rY;
  const double d2 = fma(k.ex, k.ex, k.ey * k.ey);
  k.cX = k.d0 <= 0.0;
  k.cY = k.d1 <= 0.0;
  k.cD = !(d2 > L.farD2);
  // e > 0 on both axes at every kept stage, so d2 > 0 (a lane with e <= 0
  // bails and its values here are discarded)
  const double y0 = __builtin_amdgcn_rsq(d2);
  k.inv = y0 * fma(-0.5 * d2 * y0, y0, 1.5);
  k.d2 = d2 * k.inv - L.rD;
#ifdef OGBX_BAND_BRANCH
  // impedance band, conservatively wide (contact_gains decides exactly)
  const double n0 = k.cX ? k.d0 : -1.0, n1 = k.cY ? k.d1 : -1.0, n2 = k.cD ? k.d2 : -1.0;
  k.band = fmax(n0, fmax(n1, n2)) > -1.0001 * pm.imp_width;
#else
  k.band = false;  // the gains of lean_slots cover the band
#endif
}

// Impedance gains of one slot without a branch or a band test
// (-DOGBX_BAND_BRANCH restores the wave-uniform band branch): with
// x = min(|d| / width, 1), the power-2 sigmoid of solimp (mid 0.5) is
// y = 2 x^2 - max(0, 2 x - 1)^2, imp = dmin + (dmax - dmin) y, and with
// u = 1 - imp the gains are D = imp / (u diag) = (1/u - 1) / diag and
// kp = K imp d.  Outside the band (x = 1) they are w_max and kp_max d to an
// ulp.  The per-wave tail of a step is waves with a contact resting inside
// the band (|d| < 1 mm) at every stage, so the band computation is part of
// every stage rather than a branch those waves take 20 times.
static_assert(kPointModel.imp_mid == 0.5 && kPointModel.imp_a == 2.0 && kPointModel.imp_b == 2.0,
              "band_u assumes the default solimp midpoint and power");
__device__ __forceinline__ double band_u(const PointModel& pm, double d) {
  const double x = fmin(fabs(d) * pm.inv_width, 1.0);
  const double m = fmax(fma(2.0, x, -1.0), 0.0);
  const double y = fma(2.0 * x, x, -(m * m));
  return fma(-(pm.imp_dmax - pm.imp_dmin), y, 1.0 - pm.imp_dmin);
}

__device__ __forceinline__ uint32_t lean_slots(const PointModel& pm, const LeanSides& L, const LeanHit& k,
                                               Contacts& c) {
  c.s0.nx = -L.sxd;
  c.s0.ny = 0.0;
  c.s1.nx = 0.0;
  c.s1.ny = -L.syd;
  c.s2.nx = -L.sxd * (k.ex * k.inv);
  c.s2.ny = -L.syd * (k.ey * k.inv);
#ifndef OGBX_BAND_BRANCH
  const double u0 = band_u(pm, k.d0), u1 = band_u(pm, k.d1), u2 = band_u(pm, k.d2);
  // one reciprocal for the three: 1/(u0 u1 u2), two Newton-Raphson steps
  const double p01 = u0 * u1, p = p01 * u2;
  double r = __builtin_amdgcn_rcp(p);
  r = fma(r, fma(-p, r, 1.0), r);
  r = fma(r, fma(-p, r, 1.0), r);
  const double r01 = r * u2;  // 1 / (u0 u1)
  const double idg = 1.0 / pm.diag;
  c.s0.w = k.cX ? fma(r01 * u1, idg, -idg) : 0.0;
  c.s1.w = k.cY ? fma(r01 * u0, idg, -idg) : 0.0;
  c.s2.w = k.cD ? fma(r * p01, idg, -idg) : 0.0;
  c.s0.kp = fma(-u0, pm.K, pm.K) * k.d0;
  c.s1.kp = fma(-u1, pm.K, pm.K) * k.d1;
  c.s2.kp = fma(-u2, pm.K, pm.K) * k.d2;
#else
  c.s0.kp = pm.kp_max * k.d0;
  c.s1.kp = pm.kp_max * k.d1;
  c.s2.kp = pm.kp_max * k.d2;
  c.s0.w = k.cX ? L.wX : 0.0;
  c.s1.w = k.cY ? L.wY : 0.0;
  c.s2.w = k.cD ? L.wD : 0.0;
#endif
  c.n = 0;  // unused by the role evaluation
  c.roles = true;
  return (k.cX ? L.bX : 0u) | (k.cY ? L.bY : 0u) | (k.cD ? L.bD : 0u);
}

// Impedance-band gains of all three slots, branch free (contact_gains without
// its branches; the per-wave tail of the step is waves with a contact resting
// inside the band at every stage, so this path is hot for them).  The three
// quotients imp / ((1 - imp) diag) share one v_rcp_f64 (1/(a b c), two
// Newton-Raphson refinements, then 1/a = (b c)/(a b c) ...): a few ulp from
// the IEEE division (contact tolerance 1e-9).
__device__ __forceinline__ void band_imp(const PointModel& pm, double d, double& imp, double& den, bool& inb) {
  const double x = fabs(d) * pm.inv_width;
  inb = x < 1.0;
  const double xc = fmin(x, 1.0);
  const double lo = pm.imp_a * (xc * xc);
  const double hi = 1.0 - pm.imp_b * ((1.0 - xc) * (1.0 - xc));
  const double yv = xc <= pm.imp_mid ? lo : hi;
  imp = pm.imp_dmin + yv * (pm.imp_dmax - pm.imp_dmin);  // x = 0: y = 0, imp = dmin
  den = (1.0 - imp) * pm.diag;
}

__device__ __forceinline__ void lean_band(const PointModel& pm, const LeanHit& k, Contacts& c) {
  double i0, i1, i2, a0, a1, a2;
  bool b0, b1, b2;
  band_imp(pm, k.d0, i0, a0, b0);
  band_imp(pm, k.d1, i1, a1, b1);
  band_imp(pm, k.d2, i2, a2, b2);
  b0 &= c.s0.w != 0.0;
  b1 &= c.s1.w != 0.0;
  b2 &= c.s2.w != 0.0;
  const double p01 = a0 * a1, p = p01 * a2;
  double r = __builtin_amdgcn_rcp(p);
  r = fma(r, fma(-p, r, 1.0), r);
  r = fma(r, fma(-p, r, 1.0), r);
  const double r01 = r * a2;  // 1 / (a0 a1)
  c.s0.w = b0 ? i0 * (r01 * a1) : c.s0.w;
  c.s1.w = b1 ? i1 * (r01 * a0) : c.s1.w;
  c.s2.w = b2 ? i2 * (r * p01) : c.s2.w;
  c.s0.kp = b0 ? pm.K * i0 * k.d0 : c.s0.kp;
  c.s1.kp = b1 ? pm.K * i1 * k.d1 : c.s1.kp;
  c.s2.kp = b2 ? pm.K * i2 * k.d2 : c.s2.kp;
}


#ifdef OGBX_WAVE_STAMPS
__device__ unsigned long long g_wave_paths[4096];
#endif

__device__ __forceinline__ void contact_loop_pipe(const PointModel& pm, double& x, double& y, const RoleFrame& fr,
                                                  Contacts c, uint32_t valid, bool* bail) {
  bool bl = false;
#ifdef OGBX_WAVE_STAMPS
  unsigned long long g_wpath = 0;
#endif
  const double h = pm.h;
  const LeanSides L = lean_sides(pm, fr, x, y);
  double emin = pm.box_hxy, emax = pm.box_hxy;
  double vx = 0.0, vy = 0.0, vsx = 0.0, vsy = 0.0;
  double sqx = 0.0, sqy = 0.0, svx = 0.0, svy = 0.0;
  uint32_t act = edge_mask<true>(c, 0.0, 0.0) & valid;
  PieceWeights pw;
  piece_weights(act, pw);
  const double mB = pm.mass * pm.B;
  const int nstage = 4 * pm.nsub;
#ifdef OGBX_PHYS_STATS
  uint32_t valid_prev = valid;
#endif
#pragma unroll OGBX_AS_UNROLL
  for (int e = 0; e < nstage; ++e) {
    const int st = e & 3;
    const bool more = e + 1 < nstage;
    // the next stage's position (independent of this stage's solve)
    double nqx, nqy, nsqx, nsqy, nx_ = x, ny_ = y;
    {
#pragma clang fp contract(fast)
      const double b = (st == 0 || st == 3) ? (1.0 / 6.0) : (1.0 / 3.0);
      nsqx = sqx + b * vsx;
      nsqy = sqy + b * vsy;
      if (st < 3) {
        const double cf = (st < 2) ? 0.5 : 1.0;
        nqx = x + h * (cf * vsx);
        nqy = y + h * (cf * vsy);
      } else {
        nx_ = x + h * nsqx;
        ny_ = y + h * nsqy;
        nqx = nx_;
        nqy = ny_;
      }
    }
    // lookahead collision of stage e+1
    LeanHit k;
    bool band_next = false;
#ifndef OGBX_PIPE_CHECK_FIRST
    if (more) {
      lean_collide(pm, L, nqx, nqy, k, emin, emax);
      band_next = k.band;
    }
#endif
    // stage e: one build + solve + mask from the warm-started active set
    double ux, uy;
    const double mbvx = mB * vsx, mbvy = mB * vsy;
    piece_min<true>(pm, c, pw, mbvx, mbvy, &ux, &uy);
    uint32_t A2 = edge_mask<true>(c, ux, uy);
#ifndef OGBX_NO_FIRST_TRIP
    if (e == 0) {
      // The first stage's warm start (every penetrating edge active) is exact
      // for a single contact but wrong for about half of the multi-contact
      // lanes (53 % of all active-set iterations of a step were this stage's):
      // one semismooth Newton step for every lane here, in line.
      act = A2 & valid;
      piece_weights(act, pw);
      piece_min<true>(pm, c, pw, mbvx, mbvy, &ux, &uy);
      A2 = edge_mask<true>(c, ux, uy);
    }
#endif
    bool done = ((A2 ^ act) & valid) == 0u;
    Contacts cn;
    uint32_t valid_n = 0u;
#ifndef OGBX_PIPE_CHECK_FIRST
    if (more) valid_n = lean_slots(pm, L, k, cn);
#endif
    OGBX_WSTAT(9, true);
    OGBX_WSTAT(13, !done);
    OGBX_WSTAT(10, band_next);
#ifdef OGBX_ABL_PIPE_NOITER
    done = true;  // timing-only ablation: no active-set iteration (changes the physics)
#endif
#ifdef OGBX_PHYS_STATS
    if (!done) {
      const uint32_t chg = (A2 ^ act) & valid, fresh = valid & ~valid_prev;
      OGBX_STAT(0);
      if (chg & fresh) OGBX_STAT(1);
      if (chg & ~fresh & 0xDBu) OGBX_STAT(2);
      if (chg & ~fresh & 0x124u) OGBX_STAT(3);
      if (st < 3) OGBX_STAT(6 + st);
      if (e == 0) OGBX_STAT(21);
      if (e == 0 && __builtin_popcount(valid) > 3) OGBX_STAT(22);
      if (e == 4) OGBX_STAT(23);
      if (e >= 1 && e <= 3) OGBX_STAT(23 + e);
      if (e >= 5 && e <= 7) OGBX_STAT(22 + e);
      if (e >= 8) OGBX_STAT(30);
      // the largest |residual| among the edges whose activity flips
      double rmax = 0.0;
      const ContactSlot* sl[3] = {&c.s0, &c.s1, &c.s2};
      for (int q = 0; q < 3; ++q) {
        double a, b;
        slot_res<true>(c, q, ux, uy, &a, &b);
        const double r[3] = {a + b, a - b, a};
        for (int t = 0; t < 3; ++t)
          if ((chg >> (3 * q + t)) & 1u) rmax = fmax(rmax, fabs(r[t]));
      }
      OGBX_STAT(rmax < 1e-12 ? 16 : (rmax < 1e-9 ? 17 : (rmax < 1e-6 ? 18 : (rmax < 1e-3 ? 19 : 20))));
    }
    int trips = 0;
#endif
    if (__builtin_expect(__any(!done | band_next), 0)) {
      OGBX_WPATH(0);
      if (__any(band_next)) OGBX_WPATH(40);
      if (__any(!done)) {
#pragma unroll 1
        for (int it = 0; it < OGBX_LEAN_ITERS && !done; ++it) {
          OGBX_WPATH(20);
#ifdef OGBX_PHYS_STATS
          OGBX_STAT(4);
          ++trips;
#endif
          act = A2 & valid;
          piece_weights(act, pw);
          piece_min<true>(pm, c, pw, mbvx, mbvy, &ux, &uy);
          A2 = edge_mask<true>(c, ux, uy);
          done = ((A2 ^ act) & valid) == 0u;
        }
        bl |= !done;
#ifdef OGBX_PHYS_STATS
        if (trips == 1) OGBX_STAT(5);
#endif
      }
#ifndef OGBX_PIPE_CHECK_FIRST
      if (more && __any(band_next)) lean_band(pm, k, cn);
#endif
    }
#ifdef OGBX_PIPE_CHECK_FIRST
    if (more) {
      lean_collide(pm, L, nqx, nqy, k, emin, emax);
      valid_n = lean_slots(pm, L, k, cn);
    }
#endif
    double fx, fy;
    {
#pragma clang fp contract(fast)
      fx = ux - pm.B * vsx;
      fy = uy - pm.B * vsy;
      const double b = (st == 0 || st == 3) ? (1.0 / 6.0) : (1.0 / 3.0);
      svx = svx + b * fx;
      svy = svy + b * fy;
      if (st < 3) {
        const double cf = (st < 2) ? 0.5 : 1.0;
        sqx = nsqx;
        sqy = nsqy;
        vsx = vx + (cf * fx) * h;
        vsy = vy + (cf * fy) * h;
      } else {
        vx = vx + svx * h;
        vy = vy + svy * h;
        x = nx_;
        y = ny_;
        vsx = vx;
        vsy = vy;
        sqx = sqy = svx = svy = 0.0;
      }
    }
    if (more) {
#ifdef OGBX_PHYS_STATS
      valid_prev = valid;
#endif
      c = cn;
      valid = valid_n;
    }
  }
  *bail = bl | !(emin > 0.0) | !(emax < pm.box_hxy + 1.25);
#ifdef OGBX_WAVE_STAMPS
  {
    const unsigned long long b = __ballot(1);
    const unsigned w = (unsigned)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    if (w < 4096 && (int)(threadIdx.x & 63) == __ffsll((long long)b) - 1) g_wave_paths[w] = g_wpath;
  }
#endif
}

// ---------------------------------------------------------------------------
// The pipelined lean loop in the step's LOCAL frame (default; -DOGBX_LEAN_GLOBAL
// restores contact_loop_pipe).  With the role sides fixed for the step
// (lean_sides), reflect both axes so that they point at the step's walls:
// X = sx (x - cx), Y = sy (y - cy) (exact: |x - cx| <= h and cx a multiple of
// the unit, Sterbenz), velocities and accelerations likewise.  Then the face
// normals are the constants (-1, 0) and (0, -1), the corner normal is
// -(ex, ey) / |e| with ex = h - X, and t = perp(n) in the local frame (the
// edge pair n +- t is symmetric under t -> -t, so the reflection needs no
// relabelling of the mask; the first stage's mask, taken at u = 0, is
// symmetric in the pair anyway).  Every per-stage multiplication by a side
// sign disappears, and the face residuals become differences against
// P = UX + UY, Q = UX - UY.  The position returns to the global frame once,
// x = cx + sx X, at the end of the step.
struct LocalSlots {
  double kp0, kp1, kp2, w0, w1, w2, nx2, ny2;
};

// The 2x2 normal matrix of the last solve and its inverse determinant (for
// the rank-one update of a single flipped edge).
struct PieceSys {
  double h00, h01, h11, idet;
};

// Normal-equation solve of the piece with weights p (local role layout).
__device__ __forceinline__ void local_piece_min(const PointModel& pm, const LocalSlots& c, const PieceWeights& p,
                                                double mbvx, double mbvy, double* ux, double* uy,
                                                PieceSys* sys = nullptr) {
#pragma clang fp contract(fast)
  const double M = pm.M;
  const double w0 = c.w0, w1 = c.w1, w2 = c.w2;
  double h00 = M + w0 * p.S0 + w1 * p.T1;
  double h11 = M + w0 * p.T0 + w1 * p.S1;
  double h01 = w0 * p.D0 - w1 * p.D1;
  const double g0 = w0 * c.kp0, g1 = w1 * c.kp1;
  double r0 = mbvx + g0 * p.S0 - g1 * p.D1;
  double r1 = mbvy + g0 * p.D0 + g1 * p.S1;
  const double nx = c.nx2, ny = c.ny2;
  const double q = nx * nx, s = ny * ny, o = nx * ny;
  const double WS = w2 * p.S2, WT = w2 * p.T2, WD = w2 * p.D2;
  h00 += WS * q + WT * s - 2.0 * (WD * o);
  h11 += WS * s + WT * q + 2.0 * (WD * o);
  h01 += (WS - WT) * o + WD * (q - s);
  const double k2 = c.kp2;
  r0 -= k2 * (WS * nx - WD * ny);
  r1 -= k2 * (WS * ny + WD * nx);
  const double idet = fast_recip(h00 * h11 - h01 * h01);
  *ux = (h11 * r0 - h01 * r1) * idet;
  *uy = (h00 * r1 - h01 * r0) * idet;
  if (sys) *sys = PieceSys{h00, h01, h11, idet};
}

// The solve of the piece that differs from the solved one (system S, solution
// u) by the single edge `e` (bit index): adding (delta = +1) or removing (-1)
// edge e changes the normal equations by the rank-one term delta c w J J' on
// the left and -delta c w kp J on the right, so by Sherman-Morrison
//   u' = u - a rho H^-1 J / (1 + a J' H^-1 J),  a = delta c w,  rho = J.u + kp
// (rho: the edge's residual at u).  ~30 instructions instead of rebuilding the
// piece.  Removing an edge keeps H' = M I + (the other edges) positive
// definite, so the denominator stays positive.
__device__ __forceinline__ void local_rank_one(const LocalSlots& c, const PieceSys& S, uint32_t act, int e,
                                               double* ux, double* uy) {
#pragma clang fp contract(fast)
  const int s = e >= 6 ? 2 : (e >= 3 ? 1 : 0), t = e - 3 * s;
  // slot selection as 0/1 weights, not selects: LLVM turns a select chain over
  // the slot fields into a stack array indexed by s (scratch stores per stage)
  const double f0 = (double)(s == 0), f1 = (double)(s == 1), f2 = (double)(s == 2);
  const double nx = f2 * c.nx2 - f0, ny = f2 * c.ny2 - f1;
  const double sg = (double)(t == 0) - (double)(t == 1);
  const double jx = nx - sg * ny, jy = ny + sg * nx;  // n + sg t, t = (-ny, nx)
  const double w = f0 * c.w0 + f1 * c.w1 + f2 * c.w2;
  const double kp = f0 * c.kp0 + f1 * c.kp1 + f2 * c.kp2;
  const double a = (((act >> e) & 1u) ? -1.0 : 1.0) * (t == 2 ? 2.0 * w : w);
  const double rho = jx * *ux + (jy * *uy + kp);
  const double zx = (S.h11 * jx - S.h01 * jy) * S.idet, zy = (S.h00 * jy - S.h01 * jx) * S.idet;
  const double f = a * rho * fast_recip(1.0 + a * (jx * zx + jy * zy));
  *ux -= f * zx;
  *uy -= f * zy;
}

// Active-edge mask at U (local role layout, bits as edge_mask).
__device__ __forceinline__ uint32_t local_edge_mask(const LocalSlots& c, double ux, double uy) {
#pragma clang fp contract(fast)
  const double P = ux + uy, Q = ux - uy;
  uint32_t m = (c.kp0 < P ? 1u : 0u) | (c.kp0 < Q ? 2u : 0u) | (c.kp0 < ux ? 4u : 0u);
  m |= (c.kp1 < -Q ? 8u : 0u) | (c.kp1 < P ? 16u : 0u) | (c.kp1 < uy ? 32u : 0u);
  const double a = c.nx2 * ux + (c.ny2 * uy + c.kp2);
  const double b = c.nx2 * uy - c.ny2 * ux;
  m |= (a < -b ? 64u : 0u) | (a < b ? 128u : 0u) | (a < 0.0 ? 256u : 0u);
  return m;
}

__device__ __forceinline__ uint32_t local_slots(const PointModel& pm, const LeanSides& L, const LeanHit& k,
                                                LocalSlots& c) {
  c.nx2 = -(k.ex * k.inv);
  c.ny2 = -(k.ey * k.inv);
  const double u0 = band_u(pm, k.d0), u1 = band_u(pm, k.d1), u2 = band_u(pm, k.d2);
  const double p01 = u0 * u1, p = p01 * u2;
  // u in [0.05, 0.1]: 1/(u0 u1 u2) by v_rcp_f64 and one Newton-Raphson step
  // (2e-15 relative, fast_recip; the contact tolerance is 1e-9)
  const double r = fast_recip(p);
  const double r01 = r * u2;
  const double idg = 1.0 / pm.diag;
  c.w0 = k.cX ? fma(r01 * u1, idg, -idg) : 0.0;
  c.w1 = k.cY ? fma(r01 * u0, idg, -idg) : 0.0;
  c.w2 = k.cD ? fma(r * p01, idg, -idg) : 0.0;
  c.kp0 = fma(-u0, pm.K, pm.K) * k.d0;
  c.kp1 = fma(-u1, pm.K, pm.K) * k.d1;
  c.kp2 = fma(-u2, pm.K, pm.K) * k.d2;
  return (k.cX ? L.bX : 0u) | (k.cY ? L.bY : 0u) | (k.cD ? L.bD : 0u);
}

// Slot distances at the local position (X, Y) (lean_collide in the local frame).
__device__ __forceinline__ void local_collide(const PointModel& pm, const LeanSides& L, double X, double Y,
                                              LeanHit& k, double& emin, double& emax) {
  const double hx = pm.box_hxy;
  k.ex = hx - X;
  k.ey = hx - Y;
  emin = fmin(emin, fmin(k.ex, k.ey));
  emax = fmax(emax, fmax(k.ex, k.ey));
  k.d0 = k.ex - L.rX;
  k.d1 = k.ey - L.rY;
  const double d2 = fma(k.ex, k.ex, k.ey * k.ey);
  k.cX = k.d0 <= 0.0;
  k.cY = k.d1 <= 0.0;
  k.cD = !(d2 > L.farD2);
  const double y0 = __builtin_amdgcn_rsq(d2);
  k.inv = y0 * fma(-0.5 * d2 * y0, y0, 1.5);
  k.d2 = d2 * k.inv - L.rD;
  k.band = false;
}

// c0 == nullptr: the first stage's slots come from the local collider too
// (the default; the reported contact flag is computed separately with the
// oracle's exact arithmetic, contact_flags); else from the exact
// stage_contacts (-DOGBX_FIRST_EXACT_SLOTS).
__device__ __forceinline__ void contact_loop_local(const PointModel& pm, double& x, double& y, const RoleFrame& fr,
                                                   const Contacts* c0, uint32_t valid, bool* bail) {
  bool bl = false;
  const double h = pm.h;
  const LeanSides L = lean_sides(pm, fr, x, y);
  double emin = pm.box_hxy, emax = pm.box_hxy;
  // local state: position, substep velocity, stage velocity, RK sums
  double X = L.sxd * (x - L.cx), Y = L.syd * (y - L.cy);
  double vx = 0.0, vy = 0.0, vsx = 0.0, vsy = 0.0;
  double sqx = 0.0, sqy = 0.0, svx = 0.0, svy = 0.0;
  LocalSlots c;
  if (c0 == nullptr) {
    LeanHit k0;
    local_collide(pm, L, X, Y, k0, emin, emax);
    valid = local_slots(pm, L, k0, c);
  } else {
    // the first stage's exact contacts (stage_contacts), in the local frame
    c.kp0 = c0->s0.kp;
    c.kp1 = c0->s1.kp;
    c.kp2 = c0->s2.kp;
    c.w0 = c0->s0.w;
    c.w1 = c0->s1.w;
    c.w2 = c0->s2.w;
    c.nx2 = L.sxd * c0->s2.nx;
    c.ny2 = L.syd * c0->s2.ny;
  }
  uint32_t act = local_edge_mask(c, 0.0, 0.0) & valid;
  PieceWeights pw;
  piece_weights(act, pw);
  const double mB = pm.mass * pm.B;
  const int nstage = 4 * pm.nsub;
#pragma unroll OGBX_AS_UNROLL
  for (int e = 0; e < nstage; ++e) {
    const int st = e & 3;
    const bool more = e + 1 < nstage;
    double nqx, nqy, nsqx, nsqy, nx_ = X, ny_ = Y;
    {
#pragma clang fp contract(fast)
      const double b = (st == 0 || st == 3) ? (1.0 / 6.0) : (1.0 / 3.0);
      nsqx = sqx + b * vsx;
      nsqy = sqy + b * vsy;
      if (st < 3) {
        const double cf = (st < 2) ? 0.5 : 1.0;
        nqx = X + h * (cf * vsx);
        nqy = Y + h * (cf * vsy);
      } else {
        nx_ = X + h * nsqx;
        ny_ = Y + h * nsqy;
        nqx = nx_;
        nqy = ny_;
      }
    }
    LeanHit k;
    if (more) local_collide(pm, L, nqx, nqy, k, emin, emax);
    double ux, uy;
    const double mbvx = mB * vsx, mbvy = mB * vsy;
    PieceSys sys;
    local_piece_min(pm, c, pw, mbvx, mbvy, &ux, &uy, &sys);
    uint32_t A2 = local_edge_mask(c, ux, uy);
#ifndef OGBX_NO_FIRST_TRIP
    if (e == 0) {  // see contact_loop_pipe
      act = A2 & valid;
      piece_weights(act, pw);
      local_piece_min(pm, c, pw, mbvx, mbvy, &ux, &uy, &sys);
      A2 = local_edge_mask(c, ux, uy);
    }
#endif
    bool done = ((A2 ^ act) & valid) == 0u;
    LocalSlots cn;
    uint32_t valid_n = 0u;
    if (more) valid_n = local_slots(pm, L, k, cn);
#ifdef OGBX_PHYS_STATS
    if (!done) {
      const int pc = __builtin_popcount((A2 ^ act) & valid);
      OGBX_STAT(0);
      OGBX_STAT(pc == 1 ? 1 : (pc == 2 ? 2 : 3));
    }
    int trips = 0;
#endif
    if (__builtin_expect(__any(!done), 0)) {
#ifdef OGBX_RANK_ONE
      // 99 % of the lanes that iterate flip exactly one edge (counters,
      // scripts/probe_bail.py): their next piece is a rank-one update.
      // Opt-in (-DOGBX_RANK_ONE): measured slower on gfx950 (13.75 vs 13.2 us
      // at N = 65,536) -- the hot stage keeps the 2x2 system live for it and
      // the cold block grows; the rebuilt piece costs little more.
      const uint32_t chg = (A2 ^ act) & valid;
      if (!done && (chg & (chg - 1u)) == 0u) {
        local_rank_one(c, sys, act, __builtin_ctz(chg), &ux, &uy);
        act ^= chg;
        A2 = local_edge_mask(c, ux, uy);
        done = ((A2 ^ act) & valid) == 0u;
      }
      if (__any(!done)) {
#endif
#pragma unroll 1
      for (int it = 0; it < OGBX_LEAN_ITERS && !done; ++it) {
#ifdef OGBX_PHYS_STATS
        OGBX_STAT(4);
        ++trips;
#endif
        act = A2 & valid;
        piece_weights(act, pw);
        local_piece_min(pm, c, pw, mbvx, mbvy, &ux, &uy);
        A2 = local_edge_mask(c, ux, uy);
        done = ((A2 ^ act) & valid) == 0u;
      }
      bl |= !done;
#ifdef OGBX_PHYS_STATS
      if (trips == 1) OGBX_STAT(5);
#endif
#ifdef OGBX_RANK_ONE
      }
      piece_weights(act, pw);  // the next stage's warm start
#endif
    }
    double fx, fy;
    {
#pragma clang fp contract(fast)
      fx = ux - pm.B * vsx;
      fy = uy - pm.B * vsy;
      const double b = (st == 0 || st == 3) ? (1.0 / 6.0) : (1.0 / 3.0);
      svx = svx + b * fx;
      svy = svy + b * fy;
      if (st < 3) {
        const double cf = (st < 2) ? 0.5 : 1.0;
        sqx = nsqx;
        sqy = nsqy;
        vsx = vx + (cf * fx) * h;
        vsy = vy + (cf * fy) * h;
      } else {
        vx = vx + svx * h;
        vy = vy + svy * h;
        X = nx_;
        Y = ny_;
        vsx = vx;
        vsy = vy;
        sqx = sqy = svx = svy = 0.0;
      }
    }
    if (more) {
      c = cn;
      valid = valid_n;
    }
  }
  *bail = bl | !(emin > 0.0) | !(emax < pm.box_hxy + 1.25);
  x = fma(L.sxd, X, L.cx);
  y = fma(L.syd, Y, L.cy);
}

// The first stage's contact flag with collide_roles' exact arithmetic (the
// reported flag and the free/contact split are bit-exact with the oracle), no
// slot data.  *slow: the lane needs the generic collider.
__device__ __forceinline__ uint32_t contact_flags(const PointModel& pm, const RoleFrame& f, double x, double y,
                                                  bool* slow) {
  const double lx = x - f.cx, ly = y - f.cy;
  *slow = f.slow | !(fabs(lx) < pm.box_hxy) | !(fabs(ly) < pm.box_hxy);
  const double reach = pm.box_hxy - pm.radius - 1e-9;
  const int sx = lx >= reach ? 1 : (lx <= -reach ? -1 : 0);
  const int sy = ly >= reach ? 1 : (ly <= -reach ? -1 : 0);
  const double sxd = (double)sx, syd = (double)sy;
  const double hx = pm.box_hxy, r = pm.radius;
  const uint32_t vX = (f.m >> (4 + sx)) & 1u;
  const uint32_t vY = (f.m >> (4 + 3 * sy)) & 1u;
  const uint32_t vD = (f.m >> (4 + 3 * sy + sx)) & (uint32_t)(sx & sy) & 1u;
  const double px = x - fma(sxd, pm.unit, f.cx), py = y - fma(syd, pm.unit, f.cy);
  const double tx = fma(-sxd, hx, -px), ty = fma(-syd, hx, -py);
  const bool cX = vX & (fabs(tx) - r <= 0.0);
  const bool cY = vY & (fabs(ty) - r <= 0.0);
  const bool cD = vD & !(tx * tx + ty * ty > kPointFarD2);
  return (cX ? kSlotBits : 0u) | (cY ? kSlotBits << 3 : 0u) | (cD ? kSlotBits << 6 : 0u);
}

// One PointEnv physics step (same RK4 loop as point_physics.h point_step).
__device__ __forceinline__ int point_step_as(const PointModel& pm, const uint16_t* wall, int H, int W,
                                             double* px, double* py) {
  double x = *px, y = *py;
  Contacts c;
  RoleFrame fr;
  role_frame(pm, wall, H, W, x, y, fr);
#if !defined(OGBX_LEAN_GLOBAL) && !defined(OGBX_LEAN_SERIAL) && !defined(OGBX_NO_LEAN_SPLIT) && \
    !defined(OGBX_FIRST_EXACT_SLOTS)
  {
    // exact first-stage flags; the lean loop computes its own first-stage
    // slots; the full loop (one call site) takes waves with a generic lane
    // and lanes that bail
    // Every choice is per lane, so a lane's result never depends on which envs
    // share its wavefront (any sharding of the envs reproduces the single
    // run): the lean loop's result is kept unless THIS lane bails or needs the
    // generic collider, in which case the full loop's result is taken.
    bool slow;
    const uint32_t v1 = contact_flags(pm, fr, x, y, &slow);
    bool in_contact = v1 != 0;
#ifdef OGBX_WAVE_BAIL
    {
      bool bail = true;
      const bool any_slow = __any(slow);
      if (any_slow) {
        bool generic;
        in_contact = stage_contacts(pm, wall, H, W, x, y, fr, c, &generic) != 0;
      }
      if (!__any(in_contact)) {
        *px = x + 0.0;
        *py = y + 0.0;
        return 0;
      }
      const double x0 = x, y0 = y;
      if (!any_slow) contact_loop_local(pm, x, y, fr, nullptr, 0u, &bail);
      if (__builtin_expect(__any(bail), 0)) {
        x = x0;
        y = y0;
        role_frame(pm, wall, H, W, x, y, fr);
        bool generic;
        const uint32_t valid = stage_contacts(pm, wall, H, W, x, y, fr, c, &generic);
        contact_loop<false>(pm, wall, H, W, x, y, fr, c, valid, generic, &bail);
      }
      *px = in_contact ? x : x0 + 0.0;
      *py = in_contact ? y : y0 + 0.0;
      return in_contact ? 1 : 0;
    }
#endif
    if (__builtin_expect(__any(slow), 0)) {
      bool generic;
      in_contact = stage_contacts(pm, wall, H, W, x, y, fr, c, &generic) != 0;
    }
    if (!__any(in_contact)) {
      *px = x + 0.0;
      *py = y + 0.0;
      return 0;
    }
    const double x0 = x, y0 = y;
    bool bail;
    contact_loop_local(pm, x, y, fr, nullptr, 0u, &bail);  // a slow lane's values are discarded
    bail |= slow;
    OGBX_WSTAT(14, bail);
    if (__builtin_expect(__any(bail), 0)) {
      double xf = x0, yf = y0;
      role_frame(pm, wall, H, W, xf, yf, fr);
      bool generic, b2;
      const uint32_t valid = stage_contacts(pm, wall, H, W, xf, yf, fr, c, &generic);
      contact_loop<false>(pm, wall, H, W, xf, yf, fr, c, valid, generic, &b2);
      x = bail ? xf : x;
      y = bail ? yf : y;
    }
    *px = in_contact ? x : x0 + 0.0;
    *py = in_contact ? y : y0 + 0.0;
    return in_contact ? 1 : 0;
  }
#else
  bool generic;
  uint32_t valid = stage_contacts(pm, wall, H, W, x, y, fr, c, &generic);
  const bool in_contact = valid != 0;
  // Free lanes of a wave with a contact lane run the loop too (their result
  // is discarded): the chain length, not the lane count, sets the wave's time,
  // and gfx950 issues a dependent chain ~2x slower with <= 8 active lanes.
  if (!__any(in_contact)) {
    *px = x + 0.0;
    *py = y + 0.0;
    return 0;
  }
  const double x0 = x, y0 = y;
#ifndef OGBX_NO_LEAN_SPLIT
  bool bail = true;
#if defined(OGBX_LEAN_GLOBAL)
  if (!__any(generic)) contact_loop_pipe(pm, x, y, fr, c, valid, &bail);
#elif !defined(OGBX_LEAN_SERIAL)
#ifdef OGBX_FIRST_EXACT_SLOTS
  if (!__any(generic)) contact_loop_local(pm, x, y, fr, &c, valid, &bail);
#endif
#else
  if (!__any(generic)) contact_loop<true>(pm, wall, H, W, x, y, fr, c, valid, false, &bail);
#endif
  OGBX_WSTAT(14, bail);
  if (__builtin_expect(__any(bail), 0)) {
    // redo the step with the full loop from the same first stage
    x = x0;
    y = y0;
    role_frame(pm, wall, H, W, x, y, fr);
    valid = stage_contacts(pm, wall, H, W, x, y, fr, c, &generic);
    contact_loop<false>(pm, wall, H, W, x, y, fr, c, valid, generic, &bail);
  }
#else
  bool bail;
  contact_loop<false>(pm, wall, H, W, x, y, fr, c, valid, generic, &bail);
#endif
  *px = in_contact ? x : x0 + 0.0;
  *py = in_contact ? y : y0 + 0.0;
  return in_contact ? 1 : 0;
#endif
}

}  // namespace ogbx
