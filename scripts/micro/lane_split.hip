// Microbenchmark (not shipped; verdict r05 item 2): the lean contact stage of
// pointmaze in its shipped one-lane-per-env form (A: point_contact.h's
// contact_loop_local, included from the product source) against a
// two-lanes-per-env form (B) in which lane 2j carries the x and lane 2j+1 the
// y component of env j.
//
// What B splits and what it cannot: the collision, the band gains and the
// slot weights of a stage are functions of BOTH face offsets (the corner's
// distance and normal, the band product u0 u1 u2 in every weight), and the
// 2x2 normal equations need both diagonals for det -- so those stay computed
// on both lanes (each computing them alone and exchanging would cost more:
// a 64-bit DPP exchange is two 32-bit quad_perm moves on gfx950).  B splits
// what is per component: the RK state and update (offsets, velocities,
// sums), the right-hand side r and the solution u of the 2x2 system.  Three
// exchanges per stage remain on the critical path: the new face offsets
// (both lanes need ex, ey for the collision), the other lane's r (for its
// u), and the solution (both lanes need ux, uy for the edge mask).  Each is
// a pair of quad_perm broadcasts (even lane / odd lane -> both).
//
// The run: n near-wall envs in a walled cell (every neighbour a wall, so
// every stage evaluates face, face and corner slots), the full 20-stage lean
// loop, no free-path early exit.  Prints, per form: the device time per
// launch (1,000 launches behind a spin kernel, one event span) at n = 8,192
// and 65,536 envs, and the max |A - B| of the results.  The ISA instruction
// count per stage (distance between consecutive v_rsq_f64 of the unrolled
// loop) comes from the disassembly: scripts/micro/lane_split_isa.sh.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off \
//          -mllvm -amdgpu-sched-strategy=max-ilp scripts/micro/lane_split.hip -o lane_split
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

#include "../../ogbench_amd/csrc/point_contact.h"

using namespace ogbx;

constexpr PointModel kPm = kPointModel;
constexpr int kH = 8, kW = 8;

__global__ void spin_kernel(long long ticks) {
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

// ------------------------------------------------------------------ form A
__global__ void __launch_bounds__(256) k_one(const uint16_t* __restrict__ nb, const double2* __restrict__ q,
                                             double2* __restrict__ out, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  double x = q[i].x, y = q[i].y;
  RoleFrame fr;
  role_frame(kPm, nb, kH, kW, x, y, fr);
  bool bail;
  contact_loop_local(kPm, x, y, fr, &bail);
  out[i] = make_double2(x, bail ? 1e300 : y);
}

// ------------------------------------------------------------------ form B
template <int C>
__device__ __forceinline__ double dpp64(double v) {
  return __hiloint2double(__builtin_amdgcn_mov_dpp(__double2hiint(v), C, 0xF, 0xF, false),
                          __builtin_amdgcn_mov_dpp(__double2loint(v), C, 0xF, 0xF, false));
}
constexpr int kEven = 0xA0;  // quad_perm [0,0,2,2]: the x lane's value on both lanes
constexpr int kOdd = 0xF5;   // quad_perm [1,1,3,3]: the y lane's value on both lanes

// the stage's right-hand side and solution, own component only (ky: this is
// the y lane); h and det on both lanes as in local_piece_min
__device__ __forceinline__ double pair_piece_u(const LocalSlots& c, const PieceWeights& p, bool ky, double vo,
                                               double* det_inv) {
#pragma clang fp contract(fast)
  const double w0 = c.w0, w1 = c.w1, w2 = c.w2;
  const double nx = c.nx2, ny = c.ny2;
  const double c2 = fma(nx, nx, -(ny * ny)), s2 = (nx + nx) * ny;
  const double A = w2 * p.A2, B = w2 * p.D2, C = w2 * p.C2;
  const double X = fma(C, c2, -(B * s2));
  const double mpA = c.mp + A;
  const double h00 = fma(w0, p.S0, fma(w1, p.T1, mpA)) + X;
  const double h11 = fma(w0, p.T0, fma(w1, p.S1, mpA)) - X;
  double h01 = fma(w0, p.D0, -(w1 * p.D1));
  h01 = fma(C, s2, h01);
  h01 = fma(B, c2, h01);
  const double g0 = w0 * c.kp0, g1 = w1 * c.kp1;
  // own row of r: x lane r0 = mbp vx + g0 S0 - g1 D1 - k2 (WS nx - B ny),
  //               y lane r1 = mbp vy + g0 D0 + g1 S1 - k2 (WS ny + B nx)
  const double ca = ky ? p.D0 : p.S0, cb = ky ? p.S1 : -p.D1;
  const double no = ky ? ny : nx, nt = ky ? nx : ny, sb = ky ? B : -B;
  const double WS = A + C, k2 = c.kp2;
  double r = c.mbp * vo + g0 * ca + g1 * cb;
  r -= k2 * (WS * no + sb * nt);
  const double idet = fast_recip(h00 * h11 - h01 * h01);
  // the other lane's r (a 64-bit swap of the pair)
  const double rx = dpp64<kEven>(r), ry = dpp64<kOdd>(r);
  *det_inv = idet;
  return ky ? (h00 * ry - h01 * rx) * idet : (h11 * rx - h01 * ry) * idet;
}

__device__ __forceinline__ void pair_loop(const PointModel& pm, double& x, double& y, const RoleFrame& fr, bool* bail) {
  const bool ky = threadIdx.x & 1;
  bool bl = false;
  const double h = pm.h;
  const LeanSides L = lean_sides(pm, fr, x, y);
  uint32_t ehi = 0;
  const double so = ky ? L.syd : L.sxd, co = ky ? L.cy : L.cx;
  double Eo = pm.box_hxy - so * ((ky ? y : x) - co);
  double vo = 0.0, vso = 0.0, sqo = 0.0, svo = 0.0;
  LocalSlots c;
  {
    LeanHit k0;
    const double ex = dpp64<kEven>(Eo), ey = dpp64<kOdd>(Eo);
    local_collide(L, ex, ey, k0, ehi);
    local_slots(pm, k0, c);
  }
  uint32_t act = local_edge_mask(c, 0.0, 0.0);
  PieceWeights pw;
  piece_weights(act, pw);
  const int nstage = 4 * pm.nsub;
#pragma unroll 20
  for (int e = 0; e < nstage; ++e) {
    const int st = e & 3;
    const bool more = e + 1 < nstage;
    double neo, nsqo, nEo = Eo;
    {
#pragma clang fp contract(fast)
      const double b = (st == 0 || st == 3) ? (1.0 / 6.0) : (1.0 / 3.0);
      nsqo = sqo + b * vso;
      if (st < 3) {
        const double hcf = (st < 2) ? 0.5 * kHK : kHK;
        neo = fma(-hcf, vso, Eo);
      } else {
        nEo = fma(-kHK, nsqo, Eo);
        neo = nEo;
      }
    }
    LeanHit k;
    if (more) {
      const double nex = dpp64<kEven>(neo), ney = dpp64<kOdd>(neo);
      local_collide(L, nex, ney, k, ehi);
    }
    double idet;
    double uo = pair_piece_u(c, pw, ky, vso, &idet);
    double ux = dpp64<kEven>(uo), uy = dpp64<kOdd>(uo);
    uint32_t A2 = local_edge_mask(c, ux, uy);
    if (e == 0) {
      act = A2;
      piece_weights(act, pw);
      uo = pair_piece_u(c, pw, ky, vso, &idet);
      ux = dpp64<kEven>(uo);
      uy = dpp64<kOdd>(uo);
      A2 = local_edge_mask(c, ux, uy);
    }
    bool done = A2 == act;
    LocalSlots cn;
    if (more) local_slots(pm, k, cn);
    if (__builtin_expect(__any(!done), 0)) {
#pragma unroll 1
      for (int it = 0; it < kLeanIters; ++it) {
        act = A2;
        piece_weights(act, pw);
        uo = pair_piece_u(c, pw, ky, vso, &idet);
        ux = dpp64<kEven>(uo);
        uy = dpp64<kOdd>(uo);
        A2 = local_edge_mask(c, ux, uy);
        done = A2 == act;
        if (!__any(!done)) break;
      }
      bl |= !done;
    }
    {
#pragma clang fp contract(fast)
      const double fo = uo - pm.B * vso;
      const double b = (st == 0 || st == 3) ? (1.0 / 6.0) : (1.0 / 3.0);
      svo = svo + b * fo;
      if (st < 3) {
        const double hcf = (st < 2) ? 0.5 * h : h;
        sqo = nsqo;
        vso = fma(fo, hcf, vo);
      } else {
        vo = vo + svo * h;
        Eo = nEo;
        vso = vo;
        sqo = svo = 0.0;
      }
    }
    if (more) c = cn;
  }
  *bail = bl | !(ehi < kLeanEhiLimit);
  const double Ex = dpp64<kEven>(Eo), Ey = dpp64<kOdd>(Eo);
  x = fma(L.sxd, pm.box_hxy - Ex, L.cx);
  y = fma(L.syd, pm.box_hxy - Ey, L.cy);
}

__global__ void __launch_bounds__(256) k_pair(const uint16_t* __restrict__ nb, const double2* __restrict__ q,
                                              double2* __restrict__ out, int n) {
  const int i = (blockIdx.x * 256 + threadIdx.x) >> 1;
  if (i >= n) return;
  double x = q[i].x, y = q[i].y;
  RoleFrame fr;
  role_frame(kPm, nb, kH, kW, x, y, fr);
  bool bail;
  pair_loop(kPm, x, y, fr, &bail);
  if ((threadIdx.x & 1) == 0) out[i] = make_double2(x, bail ? 1e300 : y);
}

#define CK(x)                                                         \
  do {                                                                \
    hipError_t _e = (x);                                              \
    if (_e != hipSuccess) {                                           \
      std::printf("%s: %s\n", #x, hipGetErrorString(_e));             \
      return 1;                                                       \
    }                                                                 \
  } while (0)

int main() {
  // every cell's 3x3 neighbourhood all walls except the cell itself
  std::vector<uint16_t> nbh(kH * kW, (uint16_t)(0x1FF & ~0x10));
  uint16_t* nb;
  CK(hipMalloc(&nb, nbh.size() * 2));
  CK(hipMemcpy(nb, nbh.data(), nbh.size() * 2, hipMemcpyHostToDevice));
  const int nmax = 65536;
  std::mt19937_64 rng(7);
  std::uniform_real_distribution<double> off(-1.9, 1.9);
  std::vector<double2> qh(nmax);
  const double cx = 3 * 4.0 - 4.0, cy = 3 * 4.0 - 4.0;  // cell (3, 3)
  for (auto& p : qh) p = make_double2(cx + off(rng), cy + off(rng));
  double2 *q, *oa, *ob;
  CK(hipMalloc(&q, nmax * sizeof(double2)));
  CK(hipMalloc(&oa, nmax * sizeof(double2)));
  CK(hipMalloc(&ob, nmax * sizeof(double2)));
  CK(hipMemcpy(q, qh.data(), nmax * sizeof(double2), hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int reps = 1000;
  for (int n : {8192, 16384, 65536}) {
    float ms[2];
    for (int form = 0; form < 2; ++form) {
      CK(hipDeviceSynchronize());
      hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, 0, (long long)(reps * 40e-6 * 1e8));
      CK(hipEventRecord(e0, 0));
      for (int r = 0; r < reps; ++r) {
        if (form == 0)
          hipLaunchKernelGGL(k_one, dim3((n + 255) / 256), dim3(256), 0, 0, nb, q, oa, n);
        else
          hipLaunchKernelGGL(k_pair, dim3((2 * n + 255) / 256), dim3(256), 0, 0, nb, q, ob, n);
      }
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms[form], e0, e1));
    }
    std::vector<double2> ha(n), hb(n);
    CK(hipMemcpy(ha.data(), oa, n * sizeof(double2), hipMemcpyDeviceToHost));
    CK(hipMemcpy(hb.data(), ob, n * sizeof(double2), hipMemcpyDeviceToHost));
    double dmax = 0;
    int bails = 0, same = 0;
    for (int i = 0; i < n; ++i) {
      if (ha[i].y > 1e299 || hb[i].y > 1e299) {
        bails += ha[i].y > 1e299;
        continue;
      }
      dmax = std::fmax(dmax, std::fmax(std::fabs(ha[i].x - hb[i].x), std::fabs(ha[i].y - hb[i].y)));
      same += ha[i].x == hb[i].x && ha[i].y == hb[i].y;
    }
    std::printf("n=%6d  A one-lane %.3f us/launch  B two-lane %.3f us/launch  (B/A %.3f)  max|A-B| %.3g  "
                "bit-equal %d/%d  A bails %d\n",
                n, ms[0] * 1e3 / reps, ms[1] * 1e3 / reps, ms[1] / ms[0], dmax, same, n - bails, bails);
  }
  CK(hipGetLastError());
  return 0;
}
