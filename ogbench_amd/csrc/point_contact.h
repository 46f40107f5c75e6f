// point_contact.h -- the pointmaze contact step, active-set form.
//
// Same model and the same RK4 stage loop as the restatement in point_physics.h
// (whose header states every assumed MuJoCo default; wall-contact parity is
// pinned to MuJoCo's published formulation by tests/mjmodel_np.py, not to
// MuJoCo's output), with a short per-stage instruction stream.  The step
// kernel runs one wave per SIMD and every wave that holds a contact lane runs
// the whole 20-stage chain, so the launch time is the instruction count (and
// dependency depth) of one stage x 20.
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
//     consistent), otherwise A := A' (one full semismooth Newton step).  The
//     mask carries over between RK stages and substeps, where it rarely
//     changes, and so do its integer weights (S, T, D).
//   * Two loops.  point_step_as runs the LEAN loop (contact_loop_local) first:
//     the role sides are fixed for the step and both axes reflected so the
//     step's walls lie at +h (constant face normals), the impedance band is
//     part of every stage (branch free), and the next stage's collision runs
//     beside this stage's solve.  A lane that leaves its cell's inner part,
//     needs the generic collider, or whose active set does not settle sets a
//     bail flag; those lanes take the FULL loop's result (contact_loop: frame
//     refresh, generic collider, damped-Newton safety net).  The two loops
//     agree to a few ulp per step (reflected frame, shared reciprocals, band
//     gains in closed form), both well inside the 1e-9 oracle tolerance, and
//     the choice is per lane, so a lane's result never depends on which envs
//     share its wavefront.
//
// Contact flags and free-space steps are bit-identical to the oracle (same
// closest-point arithmetic).
#pragma once

#include "point_physics.h"


namespace ogbx {

// Full-loop active-set iterations before the damped-Newton safety net.  The
// lean loop must not iterate longer: a lane it accepts after more iterations
// would be one the full loop hands to armijo_newton, and its result would
// depend on which loop its wave ran.
constexpr int kFullIters = 7;
constexpr int kLeanIters = kFullIters;
static_assert(kLeanIters <= kFullIters, "lean loop may not iterate longer than the full loop");

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
  if (__builtin_expect(__any(b0 | b1 | b2), 0)) {
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
// A2 = a0 + a1 + a2 and C2 = a2 of slot 2 feed the lean loop's double-angle
// form of the corner terms (local_piece_min).
struct PieceWeights {
  double S0, T0, D0, S1, T1, D1, S2, T2, D2, A2, C2;
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
  const int a2 = (A >> 8) & 1;
  p.A2 = (double)(((A >> 6) & 1) + ((A >> 7) & 1) + a2);
  p.C2 = (double)a2;
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

// Safety net after the active-set iterations: damped Newton with Armijo
// backtracking from cu (monotone, globally convergent).  Never seen in the
// bench states.  (Out of line, with the generic collider, the kernel is 3.5x
// smaller but 60 % slower: the call ABI costs registers.)
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
    eval_piece(pm, z, cux, cuy, ux, uy, g, h, &f);
    const double idet = 1.0 / (h[0] * h[2] - h[1] * h[1]);
    const double px = -(h[2] * g[0] - h[1] * g[1]) * idet;
    const double py = -(h[0] * g[1] - h[1] * g[0]) * idet;
    if (fabs(px) + fabs(py) <= 1e-16 * (1.0 + fabs(ux) + fabs(uy))) break;
    const double slope = g[0] * px + g[1] * py;
    double t = 1.0, g2[2], h2[3], f2;
#pragma unroll 1
    for (int bt = 0; bt < 60; ++bt) {
      eval_piece(pm, z, cux, cuy, ux + t * px, uy + t * py, g2, h2, &f2);
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
// mask still changes; after kFullIters, the damped Newton finishes the lane.
template <bool kRoles>
__device__ __forceinline__ void solve_active_set(const PointModel& pm, const Contacts& c, uint32_t valid,
                                                 double vx, double vy, uint32_t* act_io, PieceWeights& pw,
                                                 double* ux_out, double* uy_out) {
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
  if (__builtin_expect(__any(!done), 0)) {
#pragma unroll 1
    for (int it = 0; it < kFullIters && !done; ++it) {
      OGBX_STAT(4);
      A = A2 & valid;
      piece_weights(A, pw);
      piece_min<kRoles>(pm, c, pw, mbvx, mbvy, &ux, &uy);
      A2 = edge_mask<kRoles>(c, ux, uy);
      done = ((A2 ^ A) & valid) == 0u;
    }
    if (!done) {
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
  if (__builtin_expect(__any(slow), 0)) {
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

// The FULL 20-stage RK4 contact loop of one step from (x, y), whose first
// stage's frame, contacts and collider choice the caller has computed: frame
// refresh when the centre leaves its cell's half size, the generic collider
// per lane, and the damped-Newton safety net.  Takes the lanes the lean loop
// hands over (point_step_as).
__device__ __forceinline__ void contact_loop(const PointModel& pm, const uint16_t* wall, int H, int W, double& x,
                                             double& y, RoleFrame fr, Contacts c, uint32_t valid, bool generic) {
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
  // (by 4, not 20, for the rare full loop: the RK coefficients stay constants
  // and the kernel's code shrinks by 1.3 MB; 11.55 -> 11.48 us per launch at
  // N = 65,536, three A/B rounds.  The lean loop by 4: 12.45 us)
#pragma unroll 4
  for (int e = 0; e < nstage; ++e) {
    const int st = e & 3;
    if (e != 0) {
      const double lim = 0.5 * pm.unit;
      const bool stale = !(fabs(qsx - fr.cx) <= lim) | !(fabs(qsy - fr.cy) <= lim);
      if (__builtin_expect(__any(stale), 0)) {
        if (stale) role_frame(pm, wall, H, W, qsx, qsy, fr);
      }
      valid = stage_contacts(pm, wall, H, W, qsx, qsy, fr, c, &generic);
    }
    double fx, fy;
    {
#pragma clang fp contract(fast)
      double ux, uy;
      if (generic) solve_active_set<false>(pm, c, valid, vsx, vsy, &act, pw, &ux, &uy);
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
}

// ---------------------------------------------------------------------------
// The LEAN loop.
//
// Role sides fixed for the step: sx = sign(lx), sy = sign(ly) of the first
// stage's centre (the face normals are then (-sx, 0) and (0, -sy) for the whole
// step).  That equals collide_roles' choice at every stage: where collide_roles
// picks side 0 (|l| < h - r) the fixed side's face and corner are out of reach
// (dist > 1e-9), so both see no contact there.
//
// Local frame: reflect both axes so that they point at the step's walls,
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
//
// Pipelined stage: the NEXT stage's position never depends on this stage's
// solve (qs(e+1) = x + h cf vs(e) inside a substep, x + h sum(b vs) at its
// end), so its collision runs beside this stage's solve.
//
// A lane bails to the full loop when its centre leaves the inner part of its
// cell (e = h - X < 0) or crosses to the far side of its step-start half
// (e >= h + 1.25, never reachable in a step: contacts move the centre by a
// fraction of their penetration), or when its active set does not settle in
// kLeanIters iterations.
struct LeanSides {
  double cx, cy, sxd, syd;
  // per-side radius: r where the side holds a wall, -1e3 where it does not
  // (the distance is then far positive: no contact, no compare against the
  // wall bit); rD likewise and the corner's squared-distance bound
  double rX, rY, rD, farD2;
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
  return L;
}

// Slot distances of one stage in the local frame.
struct LeanHit {
  double d0, d1, d2, ex, ey, inv;
  bool cX, cY, cD;
};

// Impedance of one slot without a branch or a band test: with
// x = min(|d| / width, 1), the power-2 sigmoid of solimp (mid 0.5) is
// y = 2 x^2 - max(0, 2 x - 1)^2 and imp = dmin + (dmax - dmin) y.  The gains
// are D = imp / ((1 - imp) diag) and kp = K imp d; outside the band (x = 1)
// they are w_max and kp_max d to an ulp.  The per-wave tail of a step is waves
// with a contact resting inside the band (|d| < 1 mm) at every stage, so the
// band computation is part of every stage rather than a branch those waves
// take 20 times.  band_u returns u' = (1 - imp) / (dmax - dmin) = 2 - y
// ((1 - dmin) / (dmax - dmin) = 2 to an ulp), so that every constant of the
// formula is an inline operand; both clamps are the VOP3 clamp bit of the
// producing v_mul / v_fma (x >= 0 and 2x - 1 <= 1, so clamping to [0, 1] is
// exactly the min / max).
static_assert(kPointModel.imp_mid == 0.5 && kPointModel.imp_a == 2.0 && kPointModel.imp_b == 2.0,
              "band_u assumes the default solimp midpoint and power");
static_assert(kPointModel.imp_dmin == 0.9 && kPointModel.imp_dmax == 0.95,
              "band_u assumes (1 - dmin) / (dmax - dmin) = 2");
constexpr double kImpDelta = kPointModel.imp_dmax - kPointModel.imp_dmin;

__device__ __forceinline__ double band_u(const PointModel& pm, double d) {
  const double x = fmin(fmax(fabs(d) * pm.inv_width, 0.0), 1.0);
  const double m = fmin(fmax(fma(2.0, x, -1.0), 0.0), 1.0);
  // (2 - 2x^2 as (1 - x^2) times 2 by the VOP3 output modifier was tried in
  // round 5: gfx950 does not apply omod to this f64 fma -- the contact pin
  // caught a 4.5e-5 error)
  return fma(m, m, fma(-(x + x), x, 2.0));
}

#ifdef OGBX_WAVE_STAMPS
__device__ unsigned long long g_wave_paths[4096];
#endif

#ifdef OGBX_MASK_TRACE
// Diagnostic build only: per global thread (= env at 64 envs per wave) and
// lean stage, the active-edge mask the stage started from and the one it
// settled on (scripts/probe_mask_trace.py).
__device__ uint32_t g_mask_trace[65536 * 40];
#endif

#ifdef OGBX_STAGE_STAMPS
// Diagnostic build only: shader-clock cycles per part of the lean stage,
// summed over the step's 20 stages, per wave (first active lane stores):
// 0 RK offsets + next collision, 1 piece solve, 2 edge mask (+ the first
// stage's Newton step), 3 next slots (band gains, weights), 4 active-set
// iterations, 5 RK update; 6 iteration trips, 7 stages that iterated.  Each
// stamp is an s_memtime between scheduling barriers, so the parts are priced
// in issue order (a part's stall on an earlier part's latency counts to it)
// and the build is slower than the product; the parts' proportions are the
// reading, not their sum.
__device__ unsigned long long g_wave_stages[4096 * 8];
#define OGBX_SS_AT(acc)                              \
  do {                                               \
    __builtin_amdgcn_sched_barrier(0);               \
    const unsigned long long _t = __builtin_amdgcn_s_memtime(); \
    __builtin_amdgcn_sched_barrier(0);               \
    acc += _t - ss_t;                                \
    ss_t = _t;                                       \
  } while (0)
#else
#define OGBX_SS_AT(acc) ((void)0)
#endif

// The slots of one stage, with the stage's normal equations SCALED: with
// u'_s = (1 - imp_s) / (dmax - dmin) of slot s (band_u) and
// P = diag (dmax - dmin) u'_0 u'_1 u'_2, the weight of slot s becomes
// W_s = P w_s = imp_s prod_{t != s} u'_t -- products only, no reciprocal --
// and the mass term mp = M P.  The unknown and the velocities of the lean
// loop are carried divided by K (kp' = kp / K = imp d, mbp = m B P for the
// scaled velocity): the edge tests compare kp with u, so they are
// scale-invariant, and the position update uses h K.  The solution of the
// scaled system is the solution.
// A slot without a contact (no wall on that side, or a wall not touched) has
// kp ~ 1e30: its three edges are then never active, so with its piece weights
// 0 it contributes exactly nothing -- no validity mask and no weight select
// in the stage.  A contact that ends during the step leaves stale active bits
// for one check, which then differs from the new mask: the lane iterates once
// (cold path) and drops them.
struct LocalSlots {
  double kp0, kp1, kp2, w0, w1, w2, nx2, ny2, mp, mbp;
};

__device__ __forceinline__ double kp_or_far(bool on, double kp) {
  // one v_cndmask on the high word: any low word with high word 0x46293E59
  // is a positive double of about 1e30
  return __hiloint2double(on ? __double2hiint(kp) : 0x46293E59, __double2loint(kp));
}

// Normal-equation solve of the piece with weights p (local role layout).
// The corner slot's terms use the double-angle form: with c2 = nx^2 - ny^2,
// s2 = 2 nx ny (nx^2 + ny^2 = 1 to an ulp), S nn' + T tt' + D (nt' + tn') =
// (a0+a1+a2) I + [a2 c2 + (a1-a0) s2] diag(1, -1) + [a2 s2 - (a1-a0) c2] offdiag
// (a_e the edge activities; PieceWeights carries A2 = a0+a1+a2 and C2 = a2).
__device__ __forceinline__ void local_piece_min(const LocalSlots& c, const PieceWeights& p, double vx, double vy,
                                                double* ux, double* uy) {
  // Every fused multiply-add is written out (no contraction pragma here or in
  // local_corner_res): the solve has three call sites -- the stage's solve,
  // the first stage's Newton step and the active-set iterations -- and the
  // iterations' trip count is wave-uniform, so a lane that settled before them
  // reruns the solve at another site.  With contraction left to the compiler
  // the sites fused differently, the rerun differed by 1 ulp, and a lane's
  // result depended on whether another lane of its wave iterated (round 6,
  // scripts/probe_epw_diff.py at 8 envs per wave).  The fusion written here
  // is the compiler's choice at the stage's own site; restoring the settled
  // lanes' values after the loop instead measured 2-7 % slower (register and
  // layout effects on the hot path).
  const double w0 = c.w0, w1 = c.w1, w2 = c.w2;
  const double nx = c.nx2, ny = c.ny2;
  const double c2 = fma(nx, nx, -(ny * ny)), s2 = (nx + nx) * ny;
  const double A = w2 * p.A2, B = w2 * p.D2, C = w2 * p.C2;  // B = -(a1 - a0) w2
  const double X = fma(C, c2, -(B * s2));
  const double mpA = fma(w2, p.A2, c.mp);  // = c.mp + A
  const double h00 = fma(w0, p.S0, fma(w1, p.T1, mpA)) + X;
  const double h11 = fma(w0, p.T0, fma(w1, p.S1, mpA)) - X;
  double h01 = fma(w0, p.D0, -(w1 * p.D1));
  h01 = fma(C, s2, h01);
  h01 = fma(B, c2, h01);
  const double g0 = w0 * c.kp0, g1 = w1 * c.kp1;
  double r0 = fma(-g1, p.D1, fma(g0, p.S0, c.mbp * vx));
  double r1 = fma(g1, p.S1, fma(g0, p.D0, c.mbp * vy));
  const double WS = fma(w2, p.C2, A), k2 = c.kp2;  // = A + C
  r0 = fma(-k2, fma(WS, nx, -(B * ny)), r0);
  r1 = fma(-k2, fma(WS, ny, B * nx), r1);
  const double idet = fast_recip(fma(h00, h11, -(h01 * h01)));
  *ux = fma(h11, r0, -(h01 * r1)) * idet;
  *uy = fma(h00, r1, -(h01 * r0)) * idet;
}

// The corner slot's residual pair (a = n.u + kp, b = t.u) at U: one
// definition for the mask and the settled test, so both see the same values
// (fused explicitly, as local_piece_min).
__device__ __forceinline__ void local_corner_res(const LocalSlots& c, double ux, double uy, double* a, double* b) {
  *a = fma(c.nx2, ux, fma(c.ny2, uy, c.kp2));
  *b = fma(c.nx2, uy, -(c.ny2 * ux));
}

// Active-edge mask at U (local role layout, bits as edge_mask).
__device__ __forceinline__ uint32_t local_edge_mask(const LocalSlots& c, double ux, double uy) {
  const double P = ux + uy, Q = ux - uy;
  uint32_t m = (c.kp0 < P ? 1u : 0u) | (c.kp0 < Q ? 2u : 0u) | (c.kp0 < ux ? 4u : 0u);
  m |= (c.kp1 < -Q ? 8u : 0u) | (c.kp1 < P ? 16u : 0u) | (c.kp1 < uy ? 32u : 0u);
  double a, b;
  local_corner_res(c, ux, uy, &a, &b);
  m |= (a < -b ? 64u : 0u) | (a < b ? 128u : 0u) | (a < 0.0 ? 256u : 0u);
  return m;
}

// M diag (dmax - dmin) and m B diag (dmax - dmin): mp and mbp per u'_0 u'_1 u'_2.
constexpr double kMScale = kPointModel.M * kPointModel.diag * kImpDelta;
constexpr double kMBScale = kPointModel.mass * kPointModel.B * kPointModel.diag * kImpDelta;
// h K: the position increment per unit of scaled velocity.
constexpr double kHK = kPointModel.h * kPointModel.K;

__device__ __forceinline__ void local_slots(const PointModel& pm, const LeanHit& k, LocalSlots& c) {
  c.nx2 = -(k.ex * k.inv);
  c.ny2 = -(k.ey * k.inv);
  const double u0 = band_u(pm, k.d0), u1 = band_u(pm, k.d1), u2 = band_u(pm, k.d2);
  const double i0 = fma(-kImpDelta, u0, 1.0), i1 = fma(-kImpDelta, u1, 1.0), i2 = fma(-kImpDelta, u2, 1.0);
  const double u01 = u0 * u1, u02 = u0 * u2, u12 = u1 * u2;
  c.w0 = i0 * u12;
  c.w1 = i1 * u02;
  c.w2 = i2 * u01;
  const double U = u01 * u2;
  c.mp = kMScale * U;
  c.mbp = kMBScale * U;
  c.kp0 = kp_or_far(k.cX, i0 * k.d0);
  c.kp1 = kp_or_far(k.cY, i1 * k.d1);
  c.kp2 = kp_or_far(k.cD, i2 * k.d2);
}

// Slot distances at the local face offsets (ex, ey) = (h - X, h - Y).  ehi
// tracks the largest high word (as unsigned) of the offsets over the step: it
// stays below that of h + 1.25 = 3.25 exactly while every e is in [+0, 3.25)
// (a negative e sets the sign bit) -- the lean frame's validity, one
// v_max3_u32 per stage.
constexpr uint32_t kLeanEhiLimit = 0x400A0000u;  // high word of 3.25
static_assert(kPointModel.box_hxy + 1.25 == 3.25, "kLeanEhiLimit is the high word of h + 1.25");

__device__ __forceinline__ void local_collide(const LeanSides& L, double ex, double ey, LeanHit& k, uint32_t& ehi) {
  k.ex = ex;
  k.ey = ey;
  // (asm: otherwise LLVM defers the max to the end of the step and keeps
  // every stage's e alive in registers)
  asm("v_max3_u32 %0, %1, %2, %3" : "=v"(ehi) : "v"(ehi), "v"(__double2hiint(ex)), "v"(__double2hiint(ey)));
  k.d0 = ex - L.rX;
  k.d1 = ey - L.rY;
  const double d2 = fma(ex, ex, ey * ey);
  k.cX = k.d0 <= 0.0;
  k.cY = k.d1 <= 0.0;
  k.cD = !(d2 > L.farD2);
  // e >= 0 on both axes at every kept stage, so d2 >= 0 (a lane with e < 0
  // bails and its values here are discarded; d2 = 0 only at the corner point
  // itself, unreachable with a wall there)
  const double y0 = __builtin_amdgcn_rsq(d2);
  k.inv = y0 * fma(-0.5 * d2 * y0, y0, 1.5);
  k.d2 = fma(d2, k.inv, -L.rD);
}

// The lean loop of one step from (x, y) in frame fr; *bail on the lanes whose
// result the caller must take from the full loop instead.
__device__ __forceinline__ void contact_loop_local(const PointModel& pm, double& x, double& y, const RoleFrame& fr,
                                                   bool* bail) {
  bool bl = false;
#ifdef OGBX_WAVE_STAMPS
  unsigned long long g_wpath = 0;
#endif
#ifdef OGBX_STAGE_STAMPS
  unsigned long long ss0 = 0, ss1 = 0, ss2 = 0, ss3 = 0, ss4 = 0, ss5 = 0, ss6 = 0, ss7 = 0;
  unsigned long long ss_t = __builtin_amdgcn_s_memtime();
#endif
  const double h = pm.h;
  const LeanSides L = lean_sides(pm, fr, x, y);
  uint32_t ehi = 0;
  // local state: position, substep velocity, stage velocity, RK sums
  // the face offsets E = h - X of the substep's start position (the loop
  // carries E, not X: a stage's offsets are then one fma from its velocity)
  double Ex = pm.box_hxy - L.sxd * (x - L.cx), Ey = pm.box_hxy - L.syd * (y - L.cy);
  double vx = 0.0, vy = 0.0, vsx = 0.0, vsy = 0.0;
  double sqx = 0.0, sqy = 0.0, svx = 0.0, svy = 0.0;
  LocalSlots c;
  {
    LeanHit k0;
    local_collide(L, Ex, Ey, k0, ehi);
    local_slots(pm, k0, c);
  }
  // first stage: v = 0, so the mask at u = cu = 0 (every edge of a penetrating
  // contact) starts the iteration one step ahead of the empty set
  uint32_t act = local_edge_mask(c, 0.0, 0.0);
  PieceWeights pw;
  piece_weights(act, pw);
  const int nstage = 4 * pm.nsub;
#pragma unroll 20
  for (int e = 0; e < nstage; ++e) {
    const int st = e & 3;
    const bool more = e + 1 < nstage;
    // the next stage's face offsets (velocities are carried divided by K, so
    // the position increment is (h K) cf vs; cf = 1/2 folds into the
    // constant exactly)
    double nex, ney, nsqx, nsqy, nEx = Ex, nEy = Ey;
    {
#pragma clang fp contract(fast)
      const double b = (st == 0 || st == 3) ? (1.0 / 6.0) : (1.0 / 3.0);
      nsqx = sqx + b * vsx;
      nsqy = sqy + b * vsy;
      if (st < 3) {
        const double hcf = (st < 2) ? 0.5 * kHK : kHK;
        nex = fma(-hcf, vsx, Ex);
        ney = fma(-hcf, vsy, Ey);
      } else {
        nEx = fma(-kHK, nsqx, Ex);
        nEy = fma(-kHK, nsqy, Ey);
        nex = nEx;
        ney = nEy;
      }
    }
    LeanHit k;
    if (more) local_collide(L, nex, ney, k, ehi);
    OGBX_SS_AT(ss0);
#ifdef OGBX_MASK_TRACE
    const uint32_t mt_tid = blockIdx.x * blockDim.x + threadIdx.x;
    if (mt_tid < 65536) g_mask_trace[mt_tid * 40 + 2 * e] = act;
#endif
    double ux, uy;
    local_piece_min(c, pw, vsx, vsy, &ux, &uy);
    OGBX_SS_AT(ss1);
    uint32_t A2 = local_edge_mask(c, ux, uy);
    if (e == 0) {
      // The first stage's warm start (every penetrating edge active) is exact
      // for a single contact but wrong for about half of the multi-contact
      // lanes (53 % of all active-set iterations of a step were this stage's):
      // one semismooth Newton step for every lane here, in line.
      act = A2;
      piece_weights(act, pw);
      local_piece_min(c, pw, vsx, vsy, &ux, &uy);
      A2 = local_edge_mask(c, ux, uy);
    }
    // (round 5: the test as signs of the nine residual differences against
    // per-edge expected sign words, v_bitop3-merged -- 5 fewer instructions
    // per stage, no vcc hazards -- measured 11.55 -> 12.2 us per launch)
    bool done = A2 == act;
    OGBX_SS_AT(ss2);
    LocalSlots cn;
    if (more) local_slots(pm, k, cn);
    OGBX_SS_AT(ss3);
#ifdef OGBX_PHYS_STATS
    if (!done) {
      const int pc = __builtin_popcount(A2 ^ act);
      OGBX_STAT(0);
      OGBX_STAT(pc == 1 ? 1 : (pc == 2 ? 2 : 3));
    }
    int trips = 0;
#endif
    if (__builtin_expect(__any(!done), 0)) {
      OGBX_WPATH(0);
      // Every lane runs the iteration (a wave-uniform loop): typically one or
      // two lanes of the wave flip an edge, and gfx950 issues a dependent
      // chain about twice as slowly with <= 8 active lanes, so
      // the divergent per-lane loop ran at half speed (round 5 A/B: 12.10 ->
      // 11.54 us per launch at N = 65,536, 10.79 -> 10.40 at 8,192).  A
      // settled lane is at a fixed point (act == A2, pw = piece_weights(act)):
      // its rerun recomputes the same ux, uy and A2 bit for bit, so every
      // lane's result equals the per-lane loop's.
#pragma unroll 1
      for (int it = 0; it < kLeanIters; ++it) {
        OGBX_WPATH(20);
#ifdef OGBX_STAGE_STAMPS
        ss6 += 1;
        ss7 += it == 0;
#endif
#ifdef OGBX_PHYS_STATS
        if (!done) OGBX_STAT(4);
        trips += !done;
#endif
        act = A2;
        piece_weights(act, pw);
        local_piece_min(c, pw, vsx, vsy, &ux, &uy);
        A2 = local_edge_mask(c, ux, uy);
        done = A2 == act;
        if (!__any(!done)) break;
      }
      bl |= !done;
#ifdef OGBX_PHYS_STATS
      if (trips == 1) OGBX_STAT(5);
#endif
    }
    OGBX_SS_AT(ss4);
#ifdef OGBX_MASK_TRACE
    if (mt_tid < 65536) g_mask_trace[mt_tid * 40 + 2 * e + 1] = act | (done ? 0u : 0x80000000u);
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
        const double hcf = (st < 2) ? 0.5 * h : h;
        sqx = nsqx;
        sqy = nsqy;
        vsx = fma(fx, hcf, vx);
        vsy = fma(fy, hcf, vy);
      } else {
        vx = vx + svx * h;
        vy = vy + svy * h;
        Ex = nEx;
        Ey = nEy;
        vsx = vx;
        vsy = vy;
        sqx = sqy = svx = svy = 0.0;
      }
    }
    if (more) c = cn;
    OGBX_SS_AT(ss5);
  }
#ifdef OGBX_STAGE_STAMPS
  {
    const unsigned long long b = __ballot(1);
    const unsigned w = (unsigned)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    if (w < 4096 && (int)(threadIdx.x & 63) == __ffsll((long long)b) - 1) {
      unsigned long long* o = g_wave_stages + 8 * w;
      o[0] = ss0, o[1] = ss1, o[2] = ss2, o[3] = ss3, o[4] = ss4, o[5] = ss5, o[6] = ss6, o[7] = ss7;
    }
  }
#endif
  *bail = bl | !(ehi < kLeanEhiLimit);
  x = fma(L.sxd, pm.box_hxy - Ex, L.cx);
  y = fma(L.syd, pm.box_hxy - Ey, L.cy);
#ifdef OGBX_WAVE_STAMPS
  {
    const unsigned long long b = __ballot(1);
    const unsigned w = (unsigned)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    if (w < 4096 && (int)(threadIdx.x & 63) == __ffsll((long long)b) - 1) g_wave_paths[w] = g_wpath;
  }
#endif
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

// One PointEnv physics step: qpos (after the action) -> qpos after 5 RK4
// substeps.  Returns 1 if a wall contact was present at the start.
// Free lanes of a wave with a contact lane run the loop too (their result is
// discarded): the chain length, not the lane count, sets the wave's time, and
// gfx950 issues a dependent chain ~2x slower with <= 8 active lanes.
// Every choice is per lane, so a lane's result never depends on which envs
// share its wavefront (any sharding of the envs reproduces the single run):
// the lean loop's result is kept unless THIS lane bails or needs the generic
// collider, in which case the full loop's result is taken.
__device__ __forceinline__ int point_step_as(const PointModel& pm, const uint16_t* wall, int H, int W,
                                             double* px, double* py) {
  double x = *px, y = *py;
  Contacts c;
  RoleFrame fr;
  role_frame(pm, wall, H, W, x, y, fr);
  bool slow;
  const uint32_t v1 = contact_flags(pm, fr, x, y, &slow);
  bool in_contact = v1 != 0;
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
  contact_loop_local(pm, x, y, fr, &bail);  // a slow lane's values are discarded
  bail |= slow;
  OGBX_WSTAT(14, bail);
  if (__builtin_expect(__any(bail), 0)) {
    double xf = x0, yf = y0;
    role_frame(pm, wall, H, W, xf, yf, fr);
    bool generic;
    const uint32_t valid = stage_contacts(pm, wall, H, W, xf, yf, fr, c, &generic);
    contact_loop(pm, wall, H, W, xf, yf, fr, c, valid, generic);
    x = bail ? xf : x;
    y = bail ? yf : y;
  }
  *px = in_contact ? x : x0 + 0.0;
  *py = in_contact ? y : y0 + 0.0;
  return in_contact ? 1 : 0;
}

}  // namespace ogbx
