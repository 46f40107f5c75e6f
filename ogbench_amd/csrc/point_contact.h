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

// Contacts at a stage: the role collider, or (wave-uniform, rare) the generic
// collider for the lanes whose frame is slow, whose slots then hold contacts
// 0..n-1 with explicit tangents (empty slots zero rows).  Returns the
// validity mask; *generic tells which evaluation the wave uses.
__device__ __forceinline__ uint32_t stage_contacts(const PointModel& pm, const uint16_t* wall, int H, int W,
                                                   double x, double y, const RoleFrame& fr, Contacts& c,
                                                   bool* generic) {
  bool slow;
  uint32_t valid = collide_roles(pm, fr, x, y, c, &slow);
  *generic = false;
  OGBX_WSTAT(12, slow);
#ifndef OGBX_ABL_NOSLOW
  if (__builtin_expect(__any(slow), 0)) {
#else
  if (false) {
#endif
    *generic = true;
    role_tangents(c);
    if (slow) {
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

// One PointEnv physics step (same RK4 loop as point_physics.h point_step).
__device__ __forceinline__ int point_step_as(const PointModel& pm, const uint16_t* wall, int H, int W,
                                             double* px, double* py) {
  double x = *px, y = *py;
  Contacts c;
  RoleFrame fr;
  role_frame(pm, wall, H, W, x, y, fr);
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
  if (!__any(generic)) contact_loop<true>(pm, wall, H, W, x, y, fr, c, valid, false, &bail);
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
}

}  // namespace ogbx
