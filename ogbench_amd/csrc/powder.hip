// powder.hip -- batched powderworld envs on gfx950: the 2-D cellular-automaton
// update, brush paint, render and goal-match success check, plus the C-ABI.
//
// Reference (hliuson/ogbench):
//   element table / PWSim.forward   ogbench/powderworld/sim.py:15-37, 284-308, 363-380
//   BehaviorStone / BehaviorGravity sim.py:574-590, 461-501
//   PWRenderer.render               sim.py:386-453
//   PowderworldEnv reset/step/obs   ogbench/powderworld/powderworld_env.py:284-476
//
// Two kernel families.  The 'easy' element set (empty, wall, plant, stone;
// num_elems == 2): the Sand, FluidFlow, Ice, Water, Fire, Plant and Velocity
// rules are identities there (no sand/dust/water/gas/fire/ice/wood, velocity
// 0), so a forward pass is Stone then Gravity, done SWAR on packed bytes
// below (pw_*_kernel).  Medium/hard (num_elems 5/8) run every rule in LDS
// with float32 velocities (powder_full.h, pwf_*_kernel).
//
// Layout in HBM: world u8[N, H*W], one byte per cell = element id (bits 0-4)
// | GravityInter (bit 5, channel 2) | DidGravity (bit 6, channel 8); every
// other channel of the reference's (9,H,W) float32 world is 0 or a function of
// the id for easy worlds.  ctrl i32[N] = stage | elem<<2 | x<<8 | task<<16 |
// success<<24 (success of the current world, cached: the world only changes
// on the third step of an action and on resets), elapsed i32[N], episode
// u32[N].  Obs u8[N, H, W, 6].
//
// Kernel shape: one 256-thread workgroup per env.  Thread t owns CPT = H*W/256
// consecutive cells of one row (16 at 64x64, 4 at 32x32), held in registers as
// packed bytes ("segment").  Neighbour rows are exchanged through an LDS copy
// of the world; a forward pass (stone rule + gravity, whose row coupling spans
// r-2..r+1) costs two barriers.  Observations are staged in LDS and leave as
// fully coalesced 16-byte stores (the obs write, 24 KB per 64x64 env-step, is
// the HBM floor of the path).
#include <array>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "common.h"

namespace ogbx {

// Observation stores are streaming (123 MB per easy launch, written once and
// far larger than L2): non-temporal 16-byte stores (`nt`), which do not
// allocate in the cache (measured: easy 25.8 -> 23.5 us per launch).
typedef unsigned int pw_u32x4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void pw_nt_store16(uint4* d, const uint4& v) {
  pw_u32x4v x = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(x, reinterpret_cast<pw_u32x4v*>(d));
}

constexpr int kPwMaxSeq = 256;
constexpr int kPwMaxTasks = 8;
constexpr uint32_t kIdMask = 31u, kGrav = 32u, kDidg = 64u;
constexpr int kCtrlSuccess = 1 << 24;

// density (channel 1) and default GravityInter (channel 2) per id: sim.py:15-37
constexpr uint8_t kDensity[21] = {1, 4, 3, 2, 0, 4, 4, 0, 4, 3, 3, 2, 2, 4, 2, 4, 3, 3, 3, 4, 3};
constexpr uint8_t kGravity[21] = {1, 0, 1, 1, 1, 0, 0, 1, 0, 1, 1, 1, 1, 0, 1, 0, 1, 1, 1, 0, 1};
constexpr uint64_t pack_density() {
  uint64_t v = 0;
  for (int i = 0; i < 21; ++i) v |= (uint64_t)kDensity[i] << (3 * i);
  return v;
}
constexpr uint32_t pack_gravity() {
  uint32_t v = 0;
  for (int i = 0; i < 21; ++i) v |= (uint32_t)kGravity[i] << i;
  return v;
}
constexpr uint64_t kDensPacked = pack_density();  // 3 bits per id
constexpr uint32_t kGravPacked = pack_gravity();  // 1 bit per id

__device__ __forceinline__ uint32_t dens_of(uint32_t v) {
  return (uint32_t)(kDensPacked >> (3u * (v & kIdMask))) & 7u;
}
__device__ __forceinline__ uint32_t elem_cell(uint32_t id) {
  return id | (((kGravPacked >> id) & 1u) << 5);
}
// BehaviorGravity's did-gravity reset (sim.py:477): cleared where gravity == 1.
__device__ __forceinline__ uint32_t rd(uint32_t v) { return (v & kGrav) ? (v & ~kDidg) : v; }

struct PowderParams {
  int32_t H, W, grid, brush, xy_size, num_elems, num_tasks, max_steps, tol;
  int32_t tol_task[kPwMaxTasks];  // success tolerance per task
  float vel_q[8];                 // velocity angle-bin thresholds on q (powder_full.h, vel_bin)
  int32_t elem_ids[8];           // _elems: element id per element index
  uint32_t lut[32];              // render colour of each id, R | G<<8 | B<<16
  int32_t seq_len[kPwMaxTasks];  // goal replay sequences (elem idx, x, y)
  int8_t seq[kPwMaxTasks][kPwMaxSeq][3];
  int64_t env_base;              // global index of env 0 of this handle (sharded runs)
};

struct PowderState {
  uint8_t* world;
  int32_t* ctrl;
  int32_t* elapsed;
  uint32_t* episode;
  // medium / hard only
  int8_t* mom;       // [N, H*W] fluid momentum (channel 6)
  float2* vel;       // [N, H*W] velocity (channels 3, 4)
  uint8_t* goal_env; // [N, H*W] goal ids (the goal replay is stochastic)
  // render cache: colour of every cell as of the last state write (R | G << 8,
  // B), so a render-only step reads 3 bytes per cell instead of id + velocity
  uint16_t* crg;     // [N, H*W]
  uint8_t* cb;       // [N, H*W]
};

// Next-episode reset states prepared ahead (medium / hard, ogbx_powder_step):
// an auto-reset's goal replay and initial state depend only on the env's
// task, its next episode number and the seed (Philox), not on the episode
// being played, so pwf_prepare_kernel computes them on a low-priority side
// stream during the episode, a few replay ops per launch, into these shadow
// buffers.  The synchronized auto-reset step then loads them instead of
// replaying.  tag / ep / q: the host epoch the shadow belongs to (bumped by
// every reset or seed change), the episode and task it is for, and the next
// replay op (q > len: complete).  use != 0 only on a step the host
// joined the side stream before; any mismatch replays in line, so results
// never depend on the schedule.
struct PwPrep {
  uint8_t* world;
  int8_t* mom;
  float2* vel;
  uint8_t* goal;
  uint32_t* tag;
  uint32_t* ep;
  int32_t* q;
  int32_t* task;
  uint32_t epoch;
  int32_t use;
};

template <int WS>
struct Geo {
  static constexpr int H = WS, W = WS, CELLS = WS * WS, CPT = CELLS / 256, NW = CPT / 4;
  static constexpr int TPR = W / CPT, OBS = CELLS * 6;
  static_assert(CPT % 4 == 0 && W % CPT == 0, "segment must be whole words of one row");
};

// A thread's CPT cells as packed bytes (NW 32-bit words).
template <int NW>
struct Seg {
  uint32_t w[NW];
  __device__ __forceinline__ uint32_t get(int k) const { return (w[k >> 2] >> ((k & 3) * 8)) & 0xffu; }
  __device__ __forceinline__ void set(int k, uint32_t v) {
    const int s = (k & 3) * 8;
    w[k >> 2] = (w[k >> 2] & ~(0xffu << s)) | ((v & 0xffu) << s);
  }
};

template <int NW>
__device__ __forceinline__ Seg<NW> load_seg(const uint8_t* p) {
  Seg<NW> s;
  if constexpr (NW == 4) {
    const uint4 v = *reinterpret_cast<const uint4*>(p);
    s.w[0] = v.x, s.w[1] = v.y, s.w[2] = v.z, s.w[3] = v.w;
  } else if constexpr (NW == 2) {
    const uint2 v = *reinterpret_cast<const uint2*>(p);
    s.w[0] = v.x, s.w[1] = v.y;
  } else {
    s.w[0] = *reinterpret_cast<const uint32_t*>(p);
  }
  return s;
}

template <int NW>
__device__ __forceinline__ void store_seg(uint8_t* p, const Seg<NW>& s) {
  if constexpr (NW == 4) {
    *reinterpret_cast<uint4*>(p) = make_uint4(s.w[0], s.w[1], s.w[2], s.w[3]);
  } else if constexpr (NW == 2) {
    *reinterpret_cast<uint2*>(p) = make_uint2(s.w[0], s.w[1]);
  } else {
    *reinterpret_cast<uint32_t*>(p) = s.w[0];
  }
}

template <int WS>
struct alignas(16) PwShared {
  alignas(16) uint8_t a[WS * WS];  // world mirror (neighbour exchange)
  alignas(16) uint8_t f[WS * WS];  // gravity "moves down" flags
  alignas(16) uint32_t ob[WS * WS * 6 / 4];  // observation staging
  uint32_t lut[32];
  int32_t elem_ids[8];
  int32_t red[4];
};

// Per-thread view of the env's workgroup.
template <int WS>
struct Blk {
  using G = Geo<WS>;
  using S = Seg<G::NW>;
  PwShared<WS>& sh;
  int t, r, c0;
  __device__ __forceinline__ explicit Blk(PwShared<WS>& s)
      : sh(s), t((int)threadIdx.x), r((int)threadIdx.x / G::TPR), c0(((int)threadIdx.x % G::TPR) * G::CPT) {}

  __device__ __forceinline__ const uint8_t* row(const uint8_t* base, int R) const { return base + R * G::W + c0; }

  // ---- SWAR helpers: four cells per 32-bit word (byte k = cell 4j+k)
  static constexpr uint32_t kLo7 = 0x7F7F7F7Fu, kHi = 0x80808080u, kOnes = 0x01010101u;
  static constexpr uint32_t kIds = 0x1F1F1F1Fu, kGravB = 0x20202020u, kDidgB = 0x40404040u;
  // 0x80 in every byte that is zero, else 0 (exact per byte: no carries)
  __device__ static __forceinline__ uint32_t zbytes(uint32_t y) { return ~(((y & kLo7) + kLo7) | y | kLo7); }
  // 0x80 flags -> 0xFF byte masks
  __device__ static __forceinline__ uint32_t bmask(uint32_t f) { return (f >> 7) * 0xFFu; }
  // bytes 3..6 of {hi:lo} (hi << 8 | lo >> 24): the left neighbours of hi's cells
  __device__ static __forceinline__ uint32_t left_of(uint32_t hi, uint32_t lo) {
    return __builtin_amdgcn_alignbyte(hi, lo, 3);
  }
  // bytes 1..4 of {hi:lo}: the right neighbours of lo's cells
  __device__ static __forceinline__ uint32_t right_of(uint32_t hi, uint32_t lo) {
    return __builtin_amdgcn_alignbyte(hi, lo, 1);
  }
  // density (channel 1) of every byte's element id, v_perm_b32 byte tables
  __device__ static __forceinline__ uint32_t dens4(uint32_t w) {
    constexpr uint32_t d0 = pack4(0), d1 = pack4(4), d2 = pack4(8), d3 = pack4(12), d4 = pack4(16), d5 = pack4(20);
    const uint32_t id = w & kIds, sel = id & 0x07070707u;
    const uint32_t t0 = __builtin_amdgcn_perm(d1, d0, sel);
    const uint32_t t1 = __builtin_amdgcn_perm(d3, d2, sel);
    const uint32_t t2 = __builtin_amdgcn_perm(d5, d4, sel);
    const uint32_t b3 = ((id >> 3) & kOnes) * 0xFFu, b4 = ((id >> 4) & kOnes) * 0xFFu;
    return (t2 & b4) | (~b4 & ((t1 & b3) | (t0 & ~b3)));
  }
  static constexpr uint32_t pack4(int i) {
    uint32_t v = 0;
    for (int k = 0; k < 4; ++k) v |= (uint32_t)(i + k < 21 ? kDensity[i + k] : 0) << (8 * k);
    return v;
  }

  // BehaviorStone (sim.py:580-590) for one row segment: a stone keeps gravity
  // unless both up-left and up-right neighbours are stone (zero-padded conv).
  // upL / upR: the up row's bytes just left / right of the segment (0 outside).
  __device__ __forceinline__ S stone(S cur, const S& up, uint32_t upL, uint32_t upR, bool has_up) const {
#pragma unroll
    for (int j = 0; j < G::NW; ++j) {
      const uint32_t ul = left_of(up.w[j], j == 0 ? (upL << 24) : up.w[j - 1]);
      const uint32_t ur = right_of(j == G::NW - 1 ? upR : up.w[j + 1], up.w[j]);
      const uint32_t st = zbytes((cur.w[j] & kIds) ^ 0x09090909u);
      uint32_t both = zbytes((ul & kIds) ^ 0x09090909u) & zbytes((ur & kIds) ^ 0x09090909u);
      both = has_up ? both : 0u;
      cur.w[j] = (cur.w[j] & ~(st >> 2)) | ((st & ~both) >> 2);
    }
    return cur;
  }

  __device__ __forceinline__ uint32_t left_byte(const uint8_t* base, int R) const {
    return c0 > 0 ? base[R * G::W + c0 - 1] : 0u;
  }
  __device__ __forceinline__ uint32_t right_byte(const uint8_t* base, int R) const {
    return c0 + G::CPT < G::W ? base[R * G::W + c0 + G::CPT] : 0u;
  }
  // BehaviorGravity's did-gravity reset: clear bit 6 where bit 5 (gravity) is set
  __device__ static __forceinline__ uint32_t rd4(uint32_t x) { return x & ~((x & kGravB) << 1); }

  // One PWSim.forward (stone rule, then gravity with periodic rolls) followed
  // by the brush paint (powderworld_env.py:380-391), own = this thread's
  // segment; LDS `a` must mirror the world on entry and mirrors it on exit.
  // paint_id < 0: no paint.
  __device__ __forceinline__ void forward_paint(S& own, int paint_id, int rx, int ry, int brush) const {
    constexpr int H = G::H;
    const uint8_t* A = sh.a;
    const int rm1 = r == 0 ? H - 1 : r - 1, rm2 = r < 2 ? r + H - 2 : r - 2, rp1 = r + 1 == H ? 0 : r + 1;
    const S a_m2 = load_seg<G::NW>(row(A, rm2));
    const S a_m1 = load_seg<G::NW>(row(A, rm1));
    const S a_p1 = load_seg<G::NW>(row(A, rp1));
    const S b_m1 = stone(a_m1, a_m2, left_byte(A, rm2), right_byte(A, rm2), rm1 > 0);
    const S b_0 = stone(own, a_m1, left_byte(A, rm1), right_byte(A, rm1), r > 0);
    const S b_p1 = stone(a_p1, own, left_byte(A, r), right_byte(A, r), rp1 > 0);
    // BehaviorGravity (sim.py:476-501): a cell moves down when the cell below
    // is lighter and both have gravity (0x80 flags per byte)
    S dbb;
#pragma unroll
    for (int j = 0; j < G::NW; ++j) {
      const uint32_t dv = dens4(b_0.w[j]), dw = dens4(b_p1.w[j]);
      const uint32_t lt = ((dv | kHi) - dw - kOnes) & kHi;  // dw < dv (values <= 7: no borrow)
      const uint32_t g = (b_0.w[j] & b_p1.w[j] & kGravB) << 2;
      dbb.w[j] = lt & g;
    }
    store_seg(sh.f + r * G::W + c0, dbb);
    __syncthreads();
    const S f_m1 = load_seg<G::NW>(row(sh.f, rm1));
    const S f_m2 = load_seg<G::NW>(row(sh.f, rm2));
    const bool in_rows = paint_id >= 0 && r >= ry && r < ry + brush;
    const uint32_t pcell = paint_id >= 0 ? elem_cell((uint32_t)paint_id) * kOnes : 0u;
#pragma unroll
    for (int j = 0; j < G::NW; ++j) {
      // overlap resolution (sim.py:487-489): real moves are dbb & ~dbb(above)
      const uint32_t m0 = bmask(dbb.w[j] & ~f_m1.w[j]);
      const uint32_t m1 = bmask(f_m1.w[j] & ~f_m2.w[j]);
      uint32_t v = (rd4(b_p1.w[j]) & m0) | (~m0 & (((rd4(b_m1.w[j]) | kDidgB) & m1) | (rd4(b_0.w[j]) & ~m1)));
      if (in_rows) {
        uint32_t pm = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int c = c0 + 4 * j + b;
          pm |= (c >= rx && c < rx + brush) ? (0xFFu << (8 * b)) : 0u;
        }
        pm &= ~bmask(zbytes((v & kIds) ^ kOnes));  // not onto walls (id 1)
        v = (pcell & pm) | (v & ~pm);
      }
      own.w[j] = v;
    }
    store_seg(sh.a + r * G::W + c0, own);
    __syncthreads();
  }

  // Goal mismatch count (powderworld_env.py:410-418): a goal cell matches if
  // the world id equals it at the cell or at one of its 4 periodic
  // neighbours.  LDS `a` must mirror the world.  Returns the block total.
  __device__ __forceinline__ int errors(const S& own, const uint8_t* __restrict__ goal) const {
    constexpr int H = G::H, W = G::W;
    const uint8_t* A = sh.a;
    const int rm1 = r == 0 ? H - 1 : r - 1, rp1 = r + 1 == H ? 0 : r + 1;
    const S up = load_seg<G::NW>(row(A, rm1));
    const S dn = load_seg<G::NW>(row(A, rp1));
    const S g = load_seg<G::NW>(goal + r * W + c0);
    const uint32_t lft = A[r * W + (c0 == 0 ? W - 1 : c0 - 1)] & kIdMask;
    const uint32_t rgt = A[r * W + (c0 + G::CPT == W ? 0 : c0 + G::CPT)] & kIdMask;
    int err = 0;
#pragma unroll
    for (int j = 0; j < G::NW; ++j) {
      const uint32_t o = own.w[j] & kIds;
      const uint32_t lo = j == 0 ? (lft << 24) : (own.w[j - 1] & kIds);
      const uint32_t hi = j == G::NW - 1 ? rgt : (own.w[j + 1] & kIds);
      const uint32_t gk = g.w[j];
      const uint32_t m = zbytes(gk ^ o) | zbytes(gk ^ left_of(o, lo)) | zbytes(gk ^ right_of(hi, o)) |
                         zbytes(gk ^ (up.w[j] & kIds)) | zbytes(gk ^ (dn.w[j] & kIds));
      err += __builtin_popcount(~m & kHi);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) err += __shfl_xor(err, off);
    if ((t & 63) == 0) sh.red[t >> 6] = err;
    __syncthreads();
    const int total = sh.red[0] + sh.red[1] + sh.red[2] + sh.red[3];
    return total;
  }

  // Blank world (border walls, sim.py np_to_pw of zeros) + one brush paint.
  // The reference runs PWSim.forward on the blank world before the paint; it
  // is an identity there (nothing has a lighter cell below, no stone).
  __device__ __forceinline__ S reset_world(int paint_id, int rx, int ry, int brush) const {
    S own;
#pragma unroll
    for (int k = 0; k < G::CPT; ++k) {
      const int c = c0 + k;
      const bool border = r == 0 || r == G::H - 1 || c == 0 || c == G::W - 1;
      uint32_t v = border ? elem_cell(1) : elem_cell(0);
      if (r >= ry && r < ry + brush && c >= rx && c < rx + brush && !border) v = elem_cell((uint32_t)paint_id);
      own.set(k, v);
    }
    return own;
  }

  // Observation (powderworld_env.py:462-476): RGB of the world + action frame
  // (stage 1: whole frame in the element colour; stage 2: columns of x).
  // Staged in LDS, then written as coalesced 16-byte stores.
  // nt: non-temporal stores (single-step launches; a K-step launch measured
  // faster with plain stores: 205 vs 215 M env-steps/s at K = 48)
  __device__ __forceinline__ void observe(const S& own, uint8_t* __restrict__ dst, int stage, uint32_t acol,
                                          int rx, int brush, bool nt = true) const {
    __syncthreads();  // staging buffer free (previous copy-out done)
    uint32_t words[G::CPT * 6 / 4];
#pragma unroll
    for (int p = 0; p < G::CPT / 2; ++p) {
      const int k0 = 2 * p, k1 = 2 * p + 1;
      const uint32_t C0 = sh.lut[own.get(k0) & kIdMask], C1 = sh.lut[own.get(k1) & kIdMask];
      const bool f0 = stage == 1 || (stage == 2 && c0 + k0 >= rx && c0 + k0 < rx + brush);
      const bool f1 = stage == 1 || (stage == 2 && c0 + k1 >= rx && c0 + k1 < rx + brush);
      const uint32_t A0 = f0 ? acol : 0u, A1 = f1 ? acol : 0u;
      words[3 * p + 0] = C0 | (A0 << 24);
      words[3 * p + 1] = (A0 >> 8) | (C1 << 16);
      words[3 * p + 2] = ((C1 >> 16) & 0xffu) | (A1 << 8);
    }
    uint32_t* st = sh.ob + t * (G::CPT * 6 / 4);
    if constexpr ((G::CPT * 6 / 4) % 4 == 0) {
#pragma unroll
      for (int q = 0; q < G::CPT * 6 / 4; q += 4)
        *reinterpret_cast<uint4*>(st + q) = make_uint4(words[q], words[q + 1], words[q + 2], words[q + 3]);
    } else {
#pragma unroll
      for (int q = 0; q < G::CPT * 6 / 4; q += 2) *reinterpret_cast<uint2*>(st + q) = make_uint2(words[q], words[q + 1]);
    }
    __syncthreads();
    const uint4* src = reinterpret_cast<const uint4*>(sh.ob);
    uint4* d = reinterpret_cast<uint4*>(dst);
    if (nt) {
#pragma unroll
      for (int q = t; q < G::OBS / 16; q += 256) pw_nt_store16(&d[q], src[q]);
    } else {
#pragma unroll
      for (int q = t; q < G::OBS / 16; q += 256) d[q] = src[q];
    }
  }
};

template <int WS>
__device__ __forceinline__ void load_tables(PwShared<WS>& sh, const PowderParams* __restrict__ Pp) {
  const int t = threadIdx.x;
  if (t < 32) sh.lut[t] = Pp->lut[t];
  if (t < 8) sh.elem_ids[t] = Pp->elem_ids[t];
}

__device__ inline uint32_t pw_draw(uint64_t env, uint32_t ep, uint32_t slot, uint32_t k0, uint32_t k1,
                                   uint32_t n) {
  u32x4 w = philox4x32_10({(uint32_t)env, ep, slot, (uint32_t)(env >> 32)}, k0, k1);
  return bounded_u32(w.x, n);
}

}  // namespace ogbx

#include "powder_full.h"

namespace ogbx {

// ---------------------------------------------------------------- kernels

// Goal worlds: replay each task's semantic action sequence (one forward +
// paint per action) from the blank world (powderworld_env.py:322-329).
template <int WS>
__global__ void __launch_bounds__(256) pw_goal_kernel(const PowderParams* __restrict__ Pp, uint8_t* goals) {
  __shared__ PwShared<WS> sh;
  Blk<WS> b(sh);
  using G = Geo<WS>;
  load_tables(sh, Pp);
  const int task = blockIdx.x;
  const int grid = Pp->grid, brush = Pp->brush, len = Pp->seq_len[task];
  typename Blk<WS>::S own = b.reset_world(0, -1000, -1000, brush);
  store_seg(sh.a + b.r * G::W + b.c0, own);
  __syncthreads();
  for (int s = 0; s < len; ++s) {
    const int8_t* q = Pp->seq[task][s];
    b.forward_paint(own, sh.elem_ids[q[0]], q[1] * grid, q[2] * grid, brush);
  }
  typename Blk<WS>::S ids;
#pragma unroll
  for (int k = 0; k < G::CPT; ++k) ids.set(k, own.get(k) & kIdMask);
  store_seg(goals + (size_t)task * G::CELLS + b.r * G::W + b.c0, ids);
}

template <int WS>
__global__ void __launch_bounds__(256) pw_reset_kernel(const PowderParams* __restrict__ Pp, PowderState S,
                                                       const uint8_t* __restrict__ goals,
                                                       const int32_t* __restrict__ task_id,
                                                       const uint8_t* __restrict__ mask,
                                                       const int32_t* __restrict__ reset_action,
                                                       uint8_t* __restrict__ obs, uint8_t* __restrict__ goal_obs,
                                                       uint32_t k0, uint32_t k1) {
  using G = Geo<WS>;
  __shared__ PwShared<WS> sh;
  const int64_t e = blockIdx.x;
  const uint64_t ge = (uint64_t)e + (uint64_t)Pp->env_base;  // global env index (Philox counter)
  if (mask != nullptr && mask[e] == 0) return;
  Blk<WS> b(sh);
  load_tables(sh, Pp);
  const int grid = Pp->grid, brush = Pp->brush, ne = Pp->num_elems, xy = Pp->xy_size, nt = Pp->num_tasks;
  const uint32_t ep = S.episode[e] + 1u;
  int task = task_id ? task_id[e] : 1 + (int)pw_draw(ge, ep, 0, k0, k1, (uint32_t)nt);
  if (task < 1 || task > nt) task = 1;
  int elem, x, y;
  if (reset_action) {
    elem = reset_action[3 * e], x = reset_action[3 * e + 1], y = reset_action[3 * e + 2];
  } else {
    elem = (int)pw_draw(ge, ep, 1, k0, k1, (uint32_t)ne);
    x = (int)pw_draw(ge, ep, 2, k0, k1, (uint32_t)xy);
    y = (int)pw_draw(ge, ep, 3, k0, k1, (uint32_t)xy);
  }
  __syncthreads();  // tables
  typename Blk<WS>::S own = b.reset_world(sh.elem_ids[elem], x * grid, y * grid, brush);
  store_seg(sh.a + b.r * G::W + b.c0, own);
  store_seg(S.world + (size_t)e * G::CELLS + b.r * G::W + b.c0, own);
  __syncthreads();
  const uint8_t* goal = goals + (size_t)(task - 1) * G::CELLS;
  const int errs = b.errors(own, goal);
  b.observe(own, obs + (size_t)e * G::OBS, 0, 0u, 0, brush);
  // goal observation: render of the goal world (stage 0 -> empty action frame)
  const typename Blk<WS>::S g = load_seg<G::NW>(goal + b.r * G::W + b.c0);
  b.observe(g, goal_obs + (size_t)e * G::OBS, 0, 0u, 0, brush);
  if (threadIdx.x == 0) {
    S.ctrl[e] = (task << 16) | (errs < Pp->tol ? kCtrlSuccess : 0);
    S.elapsed[e] = 0;
    S.episode[e] = ep;
  }
}

// k_steps env steps per launch; actions [k, N] int32; draws [k, N] (values of
// np.random.randint for invalid actions) or NULL = Philox.
template <int WS>
__global__ void __launch_bounds__(256) pw_step_kernel(
    const PowderParams* __restrict__ Pp, PowderState S, const uint8_t* __restrict__ goals, int64_t n,
    const int32_t* __restrict__ action, const int32_t* __restrict__ draws, int32_t k_steps,
    uint8_t* __restrict__ obs, float* __restrict__ reward, uint8_t* __restrict__ terminated,
    uint8_t* __restrict__ truncated, uint8_t* __restrict__ success, int32_t auto_reset, uint32_t k0,
    uint32_t k1, uint32_t a0, uint32_t a1) {
  using G = Geo<WS>;
  __shared__ PwShared<WS> sh;
  Blk<WS> b(sh);
  const int64_t e = blockIdx.x;
  const uint64_t ge = (uint64_t)e + (uint64_t)Pp->env_base;  // global env index (Philox counter)
  const int act0 = action[e];  // first step's action, loaded with the world (not after the barrier)
  load_tables(sh, Pp);
  const int grid = Pp->grid, brush = Pp->brush, xy = Pp->xy_size, ne = Pp->num_elems;
  const int max_steps = Pp->max_steps, tol = Pp->tol;
  uint8_t* wdst = S.world + (size_t)e * G::CELLS + b.r * G::W + b.c0;
  typename Blk<WS>::S own = load_seg<G::NW>(wdst);
  store_seg(sh.a + b.r * G::W + b.c0, own);
  int ctrl = S.ctrl[e];
  int el = S.elapsed[e];
  uint32_t ep = S.episode[e];
  const uint8_t* goal = goals + (size_t)(((ctrl >> 16) & 255) - 1) * G::CELLS;
  bool dirty = false;
  __syncthreads();
  for (int k = 0; k < k_steps; ++k) {
    const int64_t o = (int64_t)k * n + e;
    const int act = k == 0 ? act0 : action[o];
    int stage = ctrl & 3, elem = (ctrl >> 2) & 63, x = (ctrl >> 8) & 255;
    bool succ = (ctrl & kCtrlSuccess) != 0;
    auto rnd = [&](int bound) -> int {
      if (draws) return draws[o];
      return (int)pw_draw(ge, ep, (uint32_t)el, a0, a1, (uint32_t)bound);
    };
    if (stage == 0) {
      elem = act >= 0 && act < ne ? act : rnd(ne);
    } else if (stage == 1) {
      x = act >= 0 && act < xy ? act : rnd(xy);
    } else {
      const int y = act >= 0 && act < xy ? act : rnd(xy);
      b.forward_paint(own, sh.elem_ids[elem], x * grid, y * grid, brush);
      succ = b.errors(own, goal) < tol;
      dirty = true;
    }
    stage = stage == 2 ? 0 : stage + 1;
    el += 1;
    const bool trunc = el >= max_steps;
    if (threadIdx.x == 0) {
      reward[o] = succ ? 1.0f : 0.0f;
      terminated[o] = succ;
      truncated[o] = trunc;
      success[o] = succ;
    }
    if (auto_reset && (succ || trunc)) {
      ep += 1u;
      const int re = (int)pw_draw(ge, ep, 1, k0, k1, (uint32_t)ne);
      const int rx = (int)pw_draw(ge, ep, 2, k0, k1, (uint32_t)xy);
      const int ry = (int)pw_draw(ge, ep, 3, k0, k1, (uint32_t)xy);
      own = b.reset_world(sh.elem_ids[re], rx * grid, ry * grid, brush);
      __syncthreads();  // every thread is past its reads of `a`
      store_seg(sh.a + b.r * G::W + b.c0, own);
      __syncthreads();
      succ = b.errors(own, goal) < tol;
      stage = 0;
      el = 0;
      dirty = true;
    }
    ctrl = stage | (elem << 2) | (x << 8) | (ctrl & (255 << 16)) | (succ ? kCtrlSuccess : 0);
    const uint32_t acol = sh.lut[sh.elem_ids[elem & 7] & 31];
    b.observe(own, obs + (size_t)o * G::OBS, stage, acol, x * grid, brush, k_steps == 1);
  }
  if (dirty) store_seg(wdst, own);
  if (threadIdx.x == 0) {
    S.ctrl[e] = ctrl;
    S.elapsed[e] = el;
    S.episode[e] = ep;
  }
}

// Free-standing PWSim.forward on packed worlds [n, H*W] (tests).
template <int WS>
__global__ void __launch_bounds__(256) pw_forward_kernel(const PowderParams* __restrict__ Pp,
                                                         const uint8_t* in, uint8_t* out,
                                                         int32_t steps) {
  using G = Geo<WS>;
  __shared__ PwShared<WS> sh;
  Blk<WS> b(sh);
  const size_t off = (size_t)blockIdx.x * G::CELLS + b.r * G::W + b.c0;
  typename Blk<WS>::S own = load_seg<G::NW>(in + off);
  store_seg(sh.a + b.r * G::W + b.c0, own);
  __syncthreads();
  for (int s = 0; s < steps; ++s) b.forward_paint(own, -1, 0, 0, 0);
  store_seg(out + off, own);
}


// ============================================================ medium / hard
// Full-rule worlds (powder_full.h): the state lives in LDS for the whole
// launch; goal worlds are replayed per env (the forward is stochastic).
// 512 threads per 64x64 world (8 cells per thread), 256 per 32x32 (4 cells
// per thread).  A 64x64 world holds 78 KB of LDS and 8 waves, so two worlds
// share a CU and one world's barrier waits overlap the other's work: 0.280 ->
// 0.220 ms per medium step against 1024 threads (one world per CU).
template <int WS>
constexpr int pwf_nt() { return WS == 64 ? 512 : 256; }  // threads per world
constexpr int kPwfWaves = 4;  // waves per SIMD the register budget is sized for
template <int WS>
using FW = FullWorld<WS, pwf_nt<WS>()>;

template <int WS>
__device__ __forceinline__ void pwf_tables(PwFullShared<WS>& sh, const PowderParams* __restrict__ Pp) {
  const int t = threadIdx.x;
  if (t < 32) sh.lut[t] = Pp->lut[t];
  if (t < 8) sh.elem_ids[t] = Pp->elem_ids[t];
  if (t < 8) sh.vel_q[t] = Pp->vel_q[t];
  if (t < 3) sh.rowm[t][0] = sh.rowm[t][WS + 1] = 0ull;  // zero padding rows
  __syncthreads();
}

// One forward + paint of a reset (powderworld_env.py:284-344): op q < len
// replays goal action q of the task from the blank world; op len keeps the
// goal ids (and renders the goal observation if asked), starts a blank world
// and applies the initial random semantic action (elem, x, y).  rand: [rows,
// 3, H, W] injected fields (row q) or NULL = Philox.  Kernels call this from
// ONE loop so the forward is inlined once per kernel.
template <int WS>
__device__ __forceinline__ void pwf_reset_op(const FW<WS>& fw, const PowderParams* __restrict__ Pp, int task,
                                             int q, int elem, int x, int y, const float* __restrict__ rand,
                                             uint32_t r0, uint32_t r1, uint64_t e, uint32_t ep,
                                             uint8_t* __restrict__ goal_obs) {
  constexpr int C = WS * WS;
  const int grid = Pp->grid, brush = Pp->brush, len = Pp->seq_len[task - 1];
  if (q == 0) fw.blank();
  int pe = elem, px = x, py = y;
  uint32_t slot = kRandStart;
  if (q < len) {
    const int8_t* a = Pp->seq[task - 1][q];
    pe = a[0], px = a[1], py = a[2];
    slot = kRandGoal | (uint32_t)q;
  } else {
    fw.keep_goal();
    if (goal_obs) fw.observe(goal_obs, 0, 0u, 0, brush);
    fw.blank();
  }
  fw.forward_rand(rand ? rand + (size_t)q * 3 * C : nullptr, r0, r1, e, ep, slot);
  fw.paint(fw.s.elem_ids[pe], px * grid, py * grid, brush);
}

template <int WS>
__global__ void __launch_bounds__(pwf_nt<WS>()) __attribute__((amdgpu_waves_per_eu(kPwfWaves))) pwf_reset_kernel(const PowderParams* __restrict__ Pp, PowderState S,
                                                        const int32_t* __restrict__ task_id,
                                                        const uint8_t* __restrict__ mask,
                                                        const int32_t* __restrict__ reset_action,
                                                        const float* __restrict__ rand, int32_t rand_rows,
                                                        uint8_t* __restrict__ obs, uint8_t* __restrict__ goal_obs,
                                                        uint32_t k0, uint32_t k1, uint32_t r0, uint32_t r1) {
  constexpr int C = WS * WS;
  __shared__ PwFullShared<WS> sh;
  const int64_t e = blockIdx.x;
  const uint64_t ge = (uint64_t)e + (uint64_t)Pp->env_base;  // global env index (Philox counter)
  if (mask != nullptr && mask[e] == 0) return;
  FW<WS> fw(sh);
#ifdef OGBX_PWF_RULE_STAMPS
  fw.diag_env = e;
#endif
  pwf_tables(sh, Pp);
  const int ne = Pp->num_elems, xy = Pp->xy_size, nt = Pp->num_tasks;
  const uint32_t ep = S.episode[e] + 1u;
  int task = task_id ? task_id[e] : 1 + (int)pw_draw(ge, ep, 0, k0, k1, (uint32_t)nt);
  if (task < 1 || task > nt) task = 1;
  int elem, x, y;
  if (reset_action) {
    elem = reset_action[3 * e], x = reset_action[3 * e + 1], y = reset_action[3 * e + 2];
  } else {
    elem = (int)pw_draw(ge, ep, 1, k0, k1, (uint32_t)ne);
    x = (int)pw_draw(ge, ep, 2, k0, k1, (uint32_t)xy);
    y = (int)pw_draw(ge, ep, 3, k0, k1, (uint32_t)xy);
  }
  const int len = Pp->seq_len[task - 1];
  for (int q = 0; q <= len; ++q)
    pwf_reset_op(fw, Pp, task, q, elem, x, y, rand ? rand + (size_t)e * rand_rows * 3 * C : nullptr, r0, r1, ge, ep,
                 goal_obs + (size_t)e * C * 6);
#pragma unroll
  for (int k = 0; k < FW<WS>::CPT; ++k) S.goal_env[(size_t)e * C + fw.cell(k)] = sh.g[fw.cell(k)];
  fw.store(S.world + (size_t)e * C, S.mom + (size_t)e * C, S.vel + (size_t)e * C);
  const int errs = fw.errors();
  fw.observe(obs + (size_t)e * C * 6, 0, 0u, 0, Pp->brush, false, S.crg + (size_t)e * C, S.cb + (size_t)e * C);
  if (threadIdx.x == 0) {
    S.ctrl[e] = (task << 16) | (errs < Pp->tol_task[task - 1] ? kCtrlSuccess : 0);
    S.elapsed[e] = 0;
    S.episode[e] = ep;
  }
}

// Up to `ops` replay ops of every env's next-episode reset (PwPrep), from
// its shadow (or the blank world at op 0): the same pwf_reset_op sequence,
// Philox slots and draws as an in-line auto-reset of episode S.episode + 1.
// S.episode / S.ctrl are read while the main stream may be stepping (a
// stale episode gives a shadow for an episode that never comes: not used).
template <int WS>
__global__ void __launch_bounds__(pwf_nt<WS>()) __attribute__((amdgpu_waves_per_eu(kPwfWaves))) pwf_prepare_kernel(
    const PowderParams* __restrict__ Pp, PowderState S, PwPrep prep, int32_t ops, uint32_t k0, uint32_t k1,
    uint32_t r0, uint32_t r1) {
  constexpr int C = WS * WS;
  __shared__ PwFullShared<WS> sh;
  const int64_t e = blockIdx.x;
  const uint64_t ge = (uint64_t)e + (uint64_t)Pp->env_base;
  const uint32_t target = __builtin_amdgcn_readfirstlane(S.episode[e]) + 1u;
  int task = (__builtin_amdgcn_readfirstlane(S.ctrl[e]) >> 16) & 255;
  if (task < 1 || task > Pp->num_tasks) task = 1;
  const int len = Pp->seq_len[task - 1];
  int q = (prep.tag[e] == prep.epoch && prep.ep[e] == target && prep.task[e] == task) ? prep.q[e] : 0;
  q = __builtin_amdgcn_readfirstlane(q);
  if (q > len) return;  // complete (uniform over the workgroup)
  FW<WS> fw(sh);
#ifdef OGBX_PWF_RULE_STAMPS
  fw.diag_env = e;
#endif
  pwf_tables(sh, Pp);
  if (q > 0) {
    fw.load(prep.world + (size_t)e * C, prep.mom + (size_t)e * C, prep.vel + (size_t)e * C);
    __syncthreads();
  }
  const int ne = Pp->num_elems, xy = Pp->xy_size;
  const int re = (int)pw_draw(ge, target, 1, k0, k1, (uint32_t)ne);
  const int rx = (int)pw_draw(ge, target, 2, k0, k1, (uint32_t)xy);
  const int ry = (int)pw_draw(ge, target, 3, k0, k1, (uint32_t)xy);
  for (int j = 0; j < ops && q <= len; ++j, ++q)
    pwf_reset_op(fw, Pp, task, q, re, rx, ry, nullptr, r0, r1, ge, target, nullptr);
  if (q > len) {
#pragma unroll
    for (int k = 0; k < FW<WS>::CPT; ++k) prep.goal[(size_t)e * C + fw.cell(k)] = sh.g[fw.cell(k)];
  }
  fw.store(prep.world + (size_t)e * C, prep.mom + (size_t)e * C, prep.vel + (size_t)e * C);
  if (threadIdx.x == 0) {
    prep.q[e] = q;
    prep.ep[e] = target;
    prep.task[e] = task;
    prep.tag[e] = prep.epoch;
  }
}

// k_steps env steps; rand: [k, N, 3, H, W] injected fields for the forward of
// each third step, or NULL = Philox (auto-resets always use Philox).

// envs per workgroup of an in-phase render-only step (A/B: 4, 8 and 16 equal,
// medium 159.8 -> 158.0 us per step against 4,096 exit-only workgroups)
constexpr int32_t kPwfSparseChunk = 8;
static_assert(kPwfSparseChunk >= 1 && kPwfSparseChunk <= 64, "one ballot per chunk");

template <int WS, bool kSparse>
__global__ void __launch_bounds__(pwf_nt<WS>()) __attribute__((amdgpu_waves_per_eu(kPwfWaves))) pwf_step_kernel(
    const PowderParams* __restrict__ Pp, PowderState S, int64_t n, const int32_t* __restrict__ action,
    const int32_t* __restrict__ draws, const float* __restrict__ rand, int32_t k_steps, uint8_t* __restrict__ obs,
    float* __restrict__ reward, uint8_t* __restrict__ terminated, uint8_t* __restrict__ truncated,
    uint8_t* __restrict__ success, int32_t auto_reset, uint32_t k0, uint32_t k1, uint32_t a0, uint32_t a1,
    uint32_t r0, uint32_t r1, const uint8_t* __restrict__ skip, int32_t refresh, int32_t chunk,
    const int32_t* __restrict__ order, uint32_t* __restrict__ cost, PwPrep prep) {
  constexpr int C = WS * WS, CPT = FW<WS>::CPT;
  __shared__ PwFullShared<WS> sh;
  FW<WS> fw(sh);
  const uint64_t t_start = kSparse ? 0ull : __builtin_amdgcn_s_memtime();
  // kSparse = false: one env per workgroup (e = blockIdx.x).  kSparse: the
  // envs [e0, e0 + chunk) of this workgroup that pwf_light_step_kernel did not
  // step (skip), in turn -- for launches where the light kernel is expected to
  // have stepped nearly every env (in-phase render-only steps): a few envs per
  // workgroup checked by one ballot instead of 4,096 exit-only workgroups of
  // 78 KB LDS, two per CU.  A separate kernel: the env loop around the forward
  // made the one-env kernel 8 % slower (A/B).
  // order (one-env form, in-phase full steps): workgroups in order of the
  // envs' last measured cost, costliest first (pwf_order_kernel), so the
  // launch's last workgroups are short ones; results do not depend on it
  const int64_t e0 = kSparse ? (int64_t)blockIdx.x * chunk : (order ? (int64_t)order[blockIdx.x] : (int64_t)blockIdx.x);
  uint64_t todo;
  if constexpr (!kSparse) {
    todo = (skip != nullptr && skip[e0]) ? 0ull : 1ull;
  } else {
    const int lane = (int)(threadIdx.x & 63u);
    const int64_t ee = e0 + lane;
    todo = __ballot(lane < chunk && ee < n && !(skip != nullptr && skip[ee]));  // the same in every wave
  }
  if (todo == 0) return;
  pwf_tables(sh, Pp);
  const int grid = Pp->grid, brush = Pp->brush, xy = Pp->xy_size, ne = Pp->num_elems;
  const int max_steps = Pp->max_steps;
  for (;;) {
  const int64_t e = kSparse ? e0 + __builtin_ctzll(todo) : e0;
  todo &= todo - 1ull;
  const uint64_t ge = (uint64_t)e + (uint64_t)Pp->env_base;  // global env index (Philox counter)
#ifdef OGBX_PWF_RULE_STAMPS
  fw.diag_env = e;
#endif
  fw.load(S.world + (size_t)e * C, S.mom + (size_t)e * C, S.vel + (size_t)e * C);
#pragma unroll
  for (int k = 0; k < CPT; ++k) sh.g[fw.cell(k)] = S.goal_env[(size_t)e * C + fw.cell(k)];
  int ctrl = S.ctrl[e];
  int el = S.elapsed[e];
  uint32_t ep = S.episode[e];
  const int task = (ctrl >> 16) & 255;
  const int tol = Pp->tol_task[(task >= 1 && task <= Pp->num_tasks ? task : 1) - 1];
  bool dirty = false, goal_dirty = false;
  __syncthreads();
  const int len = Pp->seq_len[task - 1];
  for (int k = 0; k < k_steps; ++k) {
    fw.fence_idx();
    const int64_t o = (int64_t)k * n + e;
    const int act = action[o];
    int stage = ctrl & 3, elem = (ctrl >> 2) & 63, x = (ctrl >> 8) & 255, y = 0;
    bool succ = (ctrl & kCtrlSuccess) != 0;
    auto rnd = [&](int bound) -> int {
      if (draws) return draws[o];
      return (int)pw_draw(ge, ep, (uint32_t)el, a0, a1, (uint32_t)bound);
    };
    if (stage == 0) {
      elem = act >= 0 && act < ne ? act : rnd(ne);
    } else if (stage == 1) {
      x = act >= 0 && act < xy ? act : rnd(xy);
    } else {
      y = act >= 0 && act < xy ? act : rnd(xy);
    }
    const bool fw_step = stage == 2;
    const uint32_t el_step = (uint32_t)el;
    stage = stage == 2 ? 0 : stage + 1;
    el += 1;
    const bool trunc = el >= max_steps;
    // ops: -1 = this step's forward + paint, 0..len = an auto-reset (one loop,
    // one inlined forward)
    int op = fw_step ? -1 : 0, op_end = fw_step ? -1 : -2;
    int re = 0, rx = 0, ry = 0;
    bool reset = false, shadow = false;
    auto finish_step = [&]() {
      if (threadIdx.x == 0) {
        reward[o] = succ ? 1.0f : 0.0f;
        terminated[o] = succ;
        truncated[o] = trunc;
        success[o] = succ;
      }
      if (auto_reset && (succ || trunc)) {
        reset = true;
        ep += 1u;
        // the episode's reset state prepared ahead (PwPrep), else in line
        shadow = prep.use && prep.tag[e] == prep.epoch && prep.ep[e] == ep && prep.task[e] == task &&
                 prep.q[e] > len;
        shadow = __builtin_amdgcn_readfirstlane((int)shadow) != 0;
        if (!shadow) {
          re = (int)pw_draw(ge, ep, 1, k0, k1, (uint32_t)ne);
          rx = (int)pw_draw(ge, ep, 2, k0, k1, (uint32_t)xy);
          ry = (int)pw_draw(ge, ep, 3, k0, k1, (uint32_t)xy);
          op_end = len;
        }
      }
    };
    if (!fw_step) finish_step();
    for (; op <= op_end; ++op) {
      fw.fence_idx();
      if (op < 0) {
        fw.forward_rand(rand ? rand + (size_t)o * 3 * C : nullptr, r0, r1, ge, ep, kRandStep | el_step);
        fw.paint(sh.elem_ids[elem], x * grid, y * grid, brush);
        succ = fw.errors() < tol;
        dirty = true;
        finish_step();
      } else {
        pwf_reset_op(fw, Pp, task, op, re, rx, ry, nullptr, r0, r1, ge, ep, nullptr);
      }
    }
    if (shadow) {
      __syncthreads();  // every lane is past its last read of the stepped world
      fw.load(prep.world + (size_t)e * C, prep.mom + (size_t)e * C, prep.vel + (size_t)e * C);
#pragma unroll
      for (int kk = 0; kk < CPT; ++kk) sh.g[fw.cell(kk)] = prep.goal[(size_t)e * C + fw.cell(kk)];
      __syncthreads();
    }
    if (reset) {
      succ = fw.errors() < tol;
      stage = 0;
      el = 0;
      dirty = goal_dirty = true;
    }
    ctrl = stage | (elem << 2) | (x << 8) | (ctrl & (255 << 16)) | (succ ? kCtrlSuccess : 0);
    const uint32_t acol = sh.lut[sh.elem_ids[elem & 7] & 31];
    // the last step's render also refreshes the cache if the state changed
    const bool cache = k == k_steps - 1 && (dirty || refresh);
    fw.observe(obs + (size_t)o * C * 6, stage, acol, x * grid, brush, false, cache ? S.crg + (size_t)e * C : nullptr,
               cache ? S.cb + (size_t)e * C : nullptr);
  }
  if (dirty) fw.store(S.world + (size_t)e * C, S.mom + (size_t)e * C, S.vel + (size_t)e * C);
  if (goal_dirty) {
#pragma unroll
    for (int k = 0; k < CPT; ++k) S.goal_env[(size_t)e * C + fw.cell(k)] = sh.g[fw.cell(k)];
  }
  if (threadIdx.x == 0) {
    S.ctrl[e] = ctrl;
    S.elapsed[e] = el;
    S.episode[e] = ep;
  }
  if (!kSparse && cost != nullptr && threadIdx.x == 0) cost[e] = (uint32_t)(__builtin_amdgcn_s_memtime() - t_start);
  if (!kSparse || todo == 0) break;
  __syncthreads();  // the next env's load overwrites the LDS state
  }
}

// Longest-first order of an in-phase full step's workgroups (one workgroup):
// a counting sort of the envs by a cost key, costliest bucket first -- the
// last measured shader cycles of the env's workgroup, or (by_task: the
// synchronized goal-replay step) the length of its task's goal sequence.
// The order within a bucket is whatever the LDS atomics give: only the
// schedule depends on it.
// One workgroup of NT threads (hist: 32 words of LDS).
template <int NT>
__device__ __forceinline__ void pwf_order_sort(const PowderParams* __restrict__ Pp, const int32_t* __restrict__ ctrl,
                                               const uint32_t* __restrict__ cost, int32_t n, int32_t by_task,
                                               int32_t* __restrict__ order, uint32_t* hist) {
  const int t = threadIdx.x;
  auto key = [&](int e) -> uint32_t {
    uint32_t c;
    if (by_task) {
      const int task = (ctrl[e] >> 16) & 255;
      c = (uint32_t)Pp->seq_len[(task >= 1 && task <= Pp->num_tasks ? task : 1) - 1] >> 3;
    } else {
      c = cost[e] >> 13;
    }
    return 31u - (c < 31u ? c : 31u);  // bucket 0: costliest
  };
  if (t < 32) hist[t] = 0;
  __syncthreads();
  for (int e = t; e < n; e += NT) atomicAdd(&hist[key(e)], 1u);
  __syncthreads();
  if (t == 0) {
    uint32_t run = 0;
    for (int b = 0; b < 32; ++b) {
      const uint32_t c = hist[b];
      hist[b] = run;
      run += c;
    }
  }
  __syncthreads();
  for (int e = t; e < n; e += NT) order[atomicAdd(&hist[key(e)], 1u)] = e;
}

__global__ void __launch_bounds__(1024) pwf_order_kernel(const PowderParams* __restrict__ Pp,
                                                         const int32_t* __restrict__ ctrl,
                                                         const uint32_t* __restrict__ cost, int32_t n,
                                                         int32_t by_task, int32_t* __restrict__ order) {
  __shared__ uint32_t hist[32];
  pwf_order_sort<1024>(Pp, ctrl, cost, n, by_task, order, hist);
}

// Render-only steps of medium/hard worlds (one step per launch).  An env at
// stage 0 or 1 of the 3-step action machine that does not auto-reset this step
// runs no forward: it draws its sub-action, advances the stage and renders its
// unchanged world (powderworld_env.py:354-427, 462-476).  Its colours come from
// the env's render cache (3 bytes per cell, written by the kernel that last
// changed the state), so the step moves 3 + 6 bytes per cell; inside
// pwf_step_kernel it would hold the full rule set's 78 KB of LDS, i.e. two
// envs per CU with little to overlap their HBM round trips.  This kernel steps
// those envs with a 24 KB staging buffer and marks them in `handled`;
// pwf_step_kernel, launched after it, skips the marked envs.  The predicate is
// evaluated on the pre-step state by this kernel alone.  refresh (the cache
// may be stale, ogbx_powder_env::cache_stale): render from id + velocity as
// the forward kernels do and rewrite the cache.
template <int WS>
__global__ void __launch_bounds__(256) pwf_light_step_kernel(
    const PowderParams* __restrict__ Pp, PowderState S, const int32_t* __restrict__ action,
    const int32_t* __restrict__ draws, uint8_t* __restrict__ obs, float* __restrict__ reward,
    uint8_t* __restrict__ terminated, uint8_t* __restrict__ truncated, uint8_t* __restrict__ success,
    int32_t auto_reset, uint32_t a0, uint32_t a1, uint8_t* __restrict__ handled, int32_t refresh,
    int32_t order_mode, int32_t n, const uint32_t* __restrict__ cost, int32_t* __restrict__ order) {
  constexpr int C = WS * WS, CPT = C / 256;
  static_assert(CPT == 16 || CPT == 4, "64x64 or 32x32 worlds");
  __shared__ alignas(16) uint16_t st[C * 3];  // 6 observation bytes per cell
  __shared__ uint32_t lut[32];
  // order_mode != 0 (the host expects the next step to be an in-phase full
  // step): workgroup 0, dispatched first, sorts the envs for it as
  // pwf_order_kernel would (1: by last cost, 2: by task length) beside this
  // launch's render-only work instead of in a launch of its own before the
  // full one.  It reads cost (written only by full steps) and ctrl's task bits
  // (which no render-only step changes), so the order is the one the full
  // step's own sort would give; env e is then workgroup e + 1.
  if (order_mode != 0 && blockIdx.x == 0) {
    pwf_order_sort<256>(Pp, S.ctrl, cost, n, order_mode == 2 ? 1 : 0, order, reinterpret_cast<uint32_t*>(st));
    return;
  }
  const int64_t e = (int64_t)blockIdx.x - (order_mode != 0 ? 1 : 0);
  const uint64_t ge = (uint64_t)e + (uint64_t)Pp->env_base;  // global env index (Philox counter)
  const int t = threadIdx.x;
  if (t < 32) lut[t] = Pp->lut[t];
  const int ctrl = S.ctrl[e];
  int el = S.elapsed[e];
  const uint32_t ep = S.episode[e];
  int stage = ctrl & 3, elem = (ctrl >> 2) & 63, x = (ctrl >> 8) & 255;
  const bool succ = (ctrl & kCtrlSuccess) != 0;
  const bool full = stage == 2 || (auto_reset && (succ || el + 1 >= Pp->max_steps));
  if (t == 0) handled[e] = full ? 0 : 1;
  if (full) return;  // uniform over the workgroup
  const int act = action[e];
  if (stage == 0) {
    const int ne = Pp->num_elems;
    elem = act >= 0 && act < ne ? act : (draws ? draws[e] : (int)pw_draw(ge, ep, (uint32_t)el, a0, a1, (uint32_t)ne));
  } else {
    const int xy = Pp->xy_size;
    x = act >= 0 && act < xy ? act : (draws ? draws[e] : (int)pw_draw(ge, ep, (uint32_t)el, a0, a1, (uint32_t)xy));
  }
  stage += 1;
  el += 1;
  const bool trunc = el >= Pp->max_steps;
  if (t == 0) {
    reward[e] = succ ? 1.0f : 0.0f;
    terminated[e] = succ;
    truncated[e] = trunc;
    success[e] = succ;
    S.ctrl[e] = stage | (elem << 2) | (x << 8) | (ctrl & (255 << 16)) | (succ ? kCtrlSuccess : 0);
    S.elapsed[e] = el;
  }
  const uint32_t acol = Pp->lut[Pp->elem_ids[elem & 7] & 31];
  const int rx = x * Pp->grid, brush = Pp->brush;
  // thread t: cells [t*CPT, t*CPT + CPT) of one row
  const int c0 = t * CPT;
  uint32_t col[CPT];  // R | G << 8 | B << 16 per cell
  uint16_t* crg = S.crg + (size_t)e * C + c0;
  uint8_t* cb = S.cb + (size_t)e * C + c0;
  if (!refresh) {
    // CPT x (2 + 1) bytes: 16 cells = two 16-byte + one 16-byte load, 4 cells = 8 + 4
    uint32_t g[CPT / 2], b[CPT / 4];
    if constexpr (CPT == 16) {
      const uint4 g0 = reinterpret_cast<const uint4*>(crg)[0], g1 = reinterpret_cast<const uint4*>(crg)[1];
      const uint4 b0 = *reinterpret_cast<const uint4*>(cb);
      g[0] = g0.x, g[1] = g0.y, g[2] = g0.z, g[3] = g0.w, g[4] = g1.x, g[5] = g1.y, g[6] = g1.z, g[7] = g1.w;
      b[0] = b0.x, b[1] = b0.y, b[2] = b0.z, b[3] = b0.w;
    } else {
      const uint2 g0 = *reinterpret_cast<const uint2*>(crg);
      g[0] = g0.x, g[1] = g0.y;
      b[0] = *reinterpret_cast<const uint32_t*>(cb);
    }
#pragma unroll
    for (int k = 0; k < CPT; ++k)
      col[k] = ((g[k >> 1] >> (16 * (k & 1))) & 0xffffu) | (((b[k >> 2] >> (8 * (k & 3))) & 0xffu) << 16);
  } else {
    const uint8_t* wa = S.world + (size_t)e * C + c0;
    const float4* wv = reinterpret_cast<const float4*>(S.vel + (size_t)e * C + c0);
    uint8_t ids[CPT];
    if constexpr (CPT == 16) {
      const uint4 q = *reinterpret_cast<const uint4*>(wa);
      const uint32_t w4[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int k = 0; k < 16; ++k) ids[k] = (uint8_t)(w4[k >> 2] >> (8 * (k & 3)));
    } else {
      const uint32_t q = *reinterpret_cast<const uint32_t*>(wa);
#pragma unroll
      for (int k = 0; k < CPT; ++k) ids[k] = (uint8_t)(q >> (8 * k));
    }
    float4 vv[CPT / 2];
#pragma unroll
    for (int k = 0; k < CPT / 2; ++k) vv[k] = wv[k];
    __syncthreads();  // lut
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const float2 v = (k & 1) ? make_float2(vv[k >> 1].z, vv[k >> 1].w) : make_float2(vv[k >> 1].x, vv[k >> 1].y);
      col[k] = pw_rgb(lut, fid(ids[k]), v);
      crg[k] = (uint16_t)(col[k] & 0xffffu);
      cb[k] = (uint8_t)(col[k] >> 16);
    }
  }
  // the thread's CPT cells are 6 * CPT contiguous observation bytes: packed
  // in registers (cell k at byte 6k: word 3k/2, at bit 0 or 16) and staged
  // with 16- / 8-byte LDS writes
  uint32_t ow[CPT * 6 / 4];
#pragma unroll
  for (int j = 0; j < CPT * 6 / 4; ++j) ow[j] = 0u;
#pragma unroll
  for (int k = 0; k < CPT; ++k) {
    const int cc = (c0 + k) % WS;
    const bool fr = stage == 1 || (stage == 2 && cc >= rx && cc < rx + brush);
    const uint64_t six = (uint64_t)(col[k] & 0xFFFFFFu) | ((uint64_t)((fr ? acol : 0u) & 0xFFFFFFu) << 24);
    const int wi = (6 * k) >> 2, sh = ((6 * k) & 3) * 8;  // sh in {0, 16}
    const uint64_t v = six << sh;
    ow[wi] |= (uint32_t)v;
    ow[wi + 1] |= (uint32_t)(v >> 32);
  }
  if constexpr (CPT == 16) {
    uint4* dst = reinterpret_cast<uint4*>(st) + t * 6;
#pragma unroll
    for (int j = 0; j < 6; ++j) dst[j] = make_uint4(ow[4 * j], ow[4 * j + 1], ow[4 * j + 2], ow[4 * j + 3]);
  } else {
    uint2* dst = reinterpret_cast<uint2*>(st) + t * 3;
#pragma unroll
    for (int j = 0; j < 3; ++j) dst[j] = make_uint2(ow[2 * j], ow[2 * j + 1]);
  }
  __syncthreads();
  const uint4* src = reinterpret_cast<const uint4*>(st);
  uint4* d = reinterpret_cast<uint4*>(obs + (size_t)e * C * 6);
#pragma unroll
  for (int q = t; q < C * 6 / 16; q += 256) pw_nt_store16(&d[q], src[q]);
}

// Free-standing PWSim.forward on worlds in the reference's (n, 9, H, W)
// float32 layout (tests / drop-in): rand [steps, n, 3, H, W] or NULL (Philox
// keyed by the env seed); optional render of the result (n, H, W, 3).
template <int WS>
__global__ void __launch_bounds__(pwf_nt<WS>()) __attribute__((amdgpu_waves_per_eu(kPwfWaves))) pwf_forward_kernel(const PowderParams* __restrict__ Pp,
                                                          const float* __restrict__ in, int64_t n, int32_t steps,
                                                          const float* __restrict__ rand, float* __restrict__ out,
                                                          uint8_t* __restrict__ rgb, uint32_t r0, uint32_t r1) {
  constexpr int C = WS * WS, CPT = FW<WS>::CPT;
  __shared__ PwFullShared<WS> sh;
  FW<WS> fw(sh);
  const int64_t e = blockIdx.x;
#ifdef OGBX_PWF_RULE_STAMPS
  fw.diag_env = e;
#endif
  pwf_tables(sh, Pp);
  const float* w = in + (size_t)e * 9 * C;
#pragma unroll
  for (int k = 0; k < CPT; ++k) {
    const int i = fw.cell(k);
    const uint32_t id = (uint32_t)(int)w[i] & 31u;
    sh.a[i] = (uint8_t)(id | (w[2 * C + i] != 0.0f ? kGrav : 0u) | (w[8 * C + i] > 0.0f ? kDidg : 0u));
    sh.m[i] = (int8_t)(int)w[6 * C + i];
    sh.v[i] = make_float2(w[3 * C + i], w[4 * C + i]);
  }
  __syncthreads();
  for (int q = 0; q < steps; ++q)
    fw.forward_rand(rand ? rand + ((size_t)q * n + e) * 3 * C : nullptr, r0, r1, e, 0u, kRandStep | (uint32_t)q);
  float* d = out + (size_t)e * 9 * C;
#pragma unroll
  for (int k = 0; k < CPT; ++k) {
    const int i = fw.cell(k);
    const uint32_t a = sh.a[i];
    d[i] = (float)fid(a);
    d[C + i] = fdens(a);
    d[2 * C + i] = (float)fgrav(a);
    d[3 * C + i] = sh.v[i].x;
    d[4 * C + i] = sh.v[i].y;
    d[5 * C + i] = 0.0f;
    d[6 * C + i] = (float)sh.m[i];
    d[7 * C + i] = 0.0f;
    d[8 * C + i] = (float)fdidg(a);
  }
  if (rgb) fw.observe(rgb + (size_t)e * C * 3, 0, 0u, 0, 0, true);
}

// Host-side task tables (powderworld_env.py:88-149), elem indices into
// _elem_names = ['plant', 'stone'].
static void easy_tasks(std::vector<std::vector<std::array<int, 3>>>& tasks) {
  auto fill = [](std::vector<std::array<int, 3>>& s, int elem, int parity) {
    for (int y = 7; y >= 0; --y)
      for (int x = 0; x < 8; ++x)
        if (parity < 0 || (x + y) % 2 == parity) s.push_back({elem, x, y});
  };
  auto square = [](std::vector<std::array<int, 3>>& s, int elem, int x, int y, int size) {
    for (int i = 0; i < size; ++i) s.push_back({elem, x + i, y + size - 1});
    for (int i = size - 2; i >= 0; --i) s.push_back({elem, x, y + i});
    for (int i = size - 2; i >= 0; --i) s.push_back({elem, x + size - 1, y + i});
    for (int i = 1; i < size - 1; ++i) s.push_back({elem, x + i, y});
  };
  const int PLANT = 0, STONE = 1;
  tasks.assign(5, {});
  fill(tasks[0], PLANT, -1);
  fill(tasks[1], PLANT, -1);
  fill(tasks[1], STONE, -1);
  fill(tasks[2], PLANT, -1);
  square(tasks[2], STONE, 1, 1, 6);
  fill(tasks[3], PLANT, -1);
  fill(tasks[3], STONE, -1);
  const int sq[4][2] = {{0, 0}, {0, 5}, {5, 0}, {5, 5}};
  for (auto& p : sq) square(tasks[3], PLANT, p[0], p[1], 3);
  fill(tasks[4], PLANT, -1);
  fill(tasks[4], STONE, 0);
}


// medium / hard tables (powderworld_env.py:150-280); element indices into
// _elem_names = [sand, water, fire, plant, stone(, gas, wood, ice)].
using PwSeq = std::vector<std::array<int, 3>>;
static void pw_square(PwSeq& s, int elem, int x, int y, int size) {
  for (int i = 0; i < size; ++i) s.push_back({elem, x + i, y + size - 1});
  for (int i = size - 2; i >= 0; --i) s.push_back({elem, x, y + i});
  for (int i = size - 2; i >= 0; --i) s.push_back({elem, x + size - 1, y + i});
  for (int i = 1; i < size - 1; ++i) s.push_back({elem, x + i, y});
}
static void pw_fill(PwSeq& s, int elem) {
  for (int y = 7; y >= 0; --y)
    for (int x = 0; x < 8; ++x) s.push_back({elem, x, y});
}
static void full_tasks(int ne, std::vector<PwSeq>& t, std::vector<int>& tol) {
  enum { SAND, WATER, FIRE, PLANT, STONE, GAS, WOOD, ICE };
  t.assign(5, {});
  if (ne == 5) {
    pw_square(t[0], PLANT, 1, 1, 6);
    pw_square(t[0], SAND, 0, 0, 8);
    pw_square(t[0], STONE, 2, 2, 4);
    pw_square(t[0], WATER, 3, 3, 2);
    pw_fill(t[1], WATER);
    pw_square(t[1], PLANT, 0, 0, 8);
    pw_square(t[2], STONE, 0, 0, 8);
    for (int i = 0; i < 32; ++i) t[2].push_back({SAND, 3, 1}), t[2].push_back({SAND, 4, 1});
    for (int x = 0; x < 8; ++x) t[3].push_back({PLANT, x, 6});
    for (int x = 0; x < 8; ++x) t[3].push_back({PLANT, x, 7});
    for (int y = 7; y >= 0; --y) t[3].push_back({STONE, 0, y});
    for (int y = 7; y >= 0; --y) t[3].push_back({STONE, 7, y});
    for (int x = 1; x < 7; ++x) t[3].push_back({STONE, x, 4});
    for (int x = 1; x < 7; ++x) t[3].push_back({STONE, x, 3});
    pw_square(t[3], WATER, 2, 0, 3);
    pw_square(t[3], WATER, 3, 0, 3);
    for (int i = 0; i < 4; ++i) t[3].push_back({FIRE, 3, 7}), t[3].push_back({FIRE, 4, 7});
    pw_fill(t[4], PLANT);
    for (int y : {4, 7})
      for (int x = 0; x < 8; ++x) t[4].push_back({WATER, x, y});
    for (int i = 0; i < 2; ++i)
      for (int x = 0; x < 8; ++x) t[4].push_back({FIRE, x, 0});
    tol = {32, 64, 64, 64, 96};
  } else {
    pw_fill(t[0], SAND);
    for (int x = 0; x < 8; ++x) t[0].push_back({SAND, x, 0});
    for (int x = 0; x < 8; ++x) t[0].push_back({WATER, x, 7});
    for (int x = 0; x < 8; ++x) t[0].push_back({GAS, x, 7});
    for (int x = 0; x < 8; ++x) t[0].push_back({WATER, x, 7});
    pw_square(t[1], WOOD, 0, 0, 8);
    pw_square(t[1], PLANT, 1, 1, 6);
    pw_square(t[1], GAS, 2, 2, 4);
    for (int i = 0; i < 3; ++i)
      for (int x = 0; x < 8; ++x) t[1].push_back({FIRE, x, 0});
    for (int x = 0; x < 8; ++x) t[2].push_back({ICE, x, 0});
    for (int y = 7; y >= 0; --y) t[2].push_back({STONE, 2, y});
    for (int y = 7; y >= 0; --y) t[2].push_back({STONE, 5, y});
    for (int y = 7; y > 0; --y) t[2].push_back({WATER, 3, y}), t[2].push_back({WATER, 4, y});
    t[2].push_back({PLANT, 3, 3});
    t[2].push_back({PLANT, 4, 3});
    t[2].push_back({PLANT, 3, 4});
    t[2].push_back({PLANT, 4, 4});
    for (int y = 7; y > 0; --y)
      for (int x : {0, 1, 6, 7}) t[2].push_back({GAS, x, y});
    pw_square(t[3], PLANT, 1, 4, 3);
    pw_square(t[3], WOOD, 4, 4, 3);
    pw_square(t[3], ICE, 1, 1, 3);
    pw_square(t[3], PLANT, 4, 1, 3);
    for (int i = 0; i < 10; ++i) pw_square(t[3], PLANT, 4, 1, 3);
    pw_fill(t[4], WATER);
    pw_square(t[4], PLANT, 3, 3, 2);
    for (int i = 0; i < 4; ++i) pw_square(t[4], STONE, 0, 0, 8);
    pw_square(t[4], ICE, 3, 3, 2);
    tol = {96, 96, 96, 64, 96};
  }
}


// BehaviorVelocity's angle bin (sim.py:938-946) as a function of q = vy / (|v|
// + 0.001): raw = float32(1/2pi) * float32(arccos(q)); ang = vx < 0 ? 1 - raw
// : raw; bin = floor(ang * 8 + 0.5) mod 8, every step rounded to float32.
// bin is a monotone step function of q on each vx branch, so it equals a
// count of exact float32 thresholds, found here by bisection over the
// ordered float32 values in [-1, 1]; the kernel then needs no arccos.
static float pw_vel_raw(float q) {
  const float inv2pi = (float)(1.0 / (2.0 * 3.141592653589793));
  return inv2pi * (float)std::acos((double)q);
}
static int pw_vel_braw(float q, bool neg) {
  const float r = pw_vel_raw(q);
  const float ang = neg ? 1.0f - r : r;
  return (int)std::floor(ang * 8.0f + 0.5f);
}
static int64_t pw_fkey(float f) {
  uint32_t b;
  std::memcpy(&b, &f, 4);
  return f >= 0.0f ? (int64_t)b : -(int64_t)(b & 0x7fffffffu);
}
static float pw_funkey(int64_t k) {
  const uint32_t b = (uint32_t)(k >= 0 ? k : -k);
  float f;
  std::memcpy(&f, &b, 4);
  return k >= 0 ? f : -f;
}
// q[0..3]: vx >= 0, bin = #{k : q <= q[k-1]} (largest q with braw >= k, k = 1..4);
// q[4..7]: vx < 0, braw = 4 + #{k : q >= q[k-1]} (smallest q with braw >= k, k = 5..8).
static void vel_bin_thresholds(float* out) {
  const int64_t lo0 = pw_fkey(-1.0f), hi0 = pw_fkey(1.0f);
  for (int k = 1; k <= 4; ++k) {  // braw(q) >= k holds on [-1, T]
    int64_t lo = lo0, hi = hi0;
    if (pw_vel_braw(-1.0f, false) < k) { out[k - 1] = -2.0f; continue; }
    while (lo < hi) {  // largest key with braw >= k
      const int64_t mid = lo + (hi - lo + 1) / 2;
      if (pw_vel_braw(pw_funkey(mid), false) >= k) lo = mid; else hi = mid - 1;
    }
    out[k - 1] = pw_funkey(lo);
  }
  for (int k = 5; k <= 8; ++k) {  // braw(q) >= k holds on [U, 1]
    int64_t lo = lo0, hi = hi0;
    if (pw_vel_braw(1.0f, true) < k) { out[k - 1] = 2.0f; continue; }
    while (lo < hi) {  // smallest key with braw >= k
      const int64_t mid = lo + (hi - lo) / 2;
      if (pw_vel_braw(pw_funkey(mid), true) >= k) hi = mid; else lo = mid + 1;
    }
    out[k - 1] = pw_funkey(lo);
  }
}

static void task_tables(int ne, std::vector<PwSeq>& t, std::vector<int>& tol) {
  if (ne == 2) {
    easy_tasks(t);
    tol.assign(t.size(), 32);
  } else {
    full_tasks(ne, t, tol);
  }
}
}  // namespace ogbx

struct ogbx_powder_env {
  int32_t device = 0;
  int64_t n = 0;
  bool full = false;  // medium / hard element sets (full rule set)
  int32_t max_seq = 0;
  ogbx::PowderParams P;
  ogbx::PowderParams* Pd = nullptr;
  ogbx::PowderState S{};
  uint8_t* goals = nullptr;  // easy: [num_tasks, H*W] goal ids
  uint8_t* handled = nullptr;  // medium/hard: [N] env stepped by pwf_light_step_kernel this launch
  uint32_t* cost = nullptr;    // medium/hard: [N] shader cycles of the env's last one-env full-kernel workgroup
  int32_t* order = nullptr;    // medium/hard: [N] workgroup -> env of an in-phase full step, costliest first
  // the last light launch sorted `order` for the step after it (by task
  // length if order_by_task); consumed by that step when it is the in-phase
  // full step the host expected.  A stale order is still a permutation of the
  // envs: only the schedule would differ.
  bool order_ready = false, order_by_task = false;
  bool light = true;           // split render-only steps into pwf_light_step_kernel
  // the render cache (S.crg / S.cb) may disagree with the state: set at create
  // and whenever a world or velocity pointer is handed out (the caller may
  // write through it); the next step then renders from the state and rewrites
  // the cache of every env
  bool cache_stale = true;
  // steps since the last reset of every env (-1: unknown, e.g. after a masked
  // reset).  Envs reset together step in phase, so the host can tell the
  // steps on which every in-phase env needs the full kernel (its forward
  // step, or the synchronized truncation + auto-reset) and not launch
  // pwf_light_step_kernel, whose every workgroup would exit.  A wrong guess
  // is harmless: pwf_step_kernel without the skip list steps render-only
  // envs itself, bit-identically (only slower), so out-of-phase envs (an
  // earlier success + auto-reset, a restored state) stay correct.
  int64_t phase = -1;
  uint64_t seed = 0;
  bool was_reset = false;
  // next-episode reset states prepared ahead on a low-priority side stream
  // (PwPrep; medium / hard, in-phase envs with auto-reset)
  int32_t prep_ops = 0;           // replay ops per prepare launch (0: off, the default; OGBX_PWF_PREP_OPS)
  ogbx::PwPrep prep{};            // device buffers + the current epoch
  hipStream_t side = nullptr;     // created on first use, lowest priority
  hipEvent_t ev_fork = nullptr, ev_side = nullptr;
  int64_t prep_launched = 0;      // replay ops launched for the coming synchronized reset
  bool side_pending = false;      // a prepare launch not yet joined
};

using namespace ogbx;

namespace {
// dispatch a kernel template on the world size
template <int WS>
constexpr auto pwf_step_kernel_dense = pwf_step_kernel<WS, false>;
template <int WS>
constexpr auto pwf_step_kernel_sparse = pwf_step_kernel<WS, true>;
#define PWF_LAUNCH(kern, e, grid, stream, ...)                                                 \
  do {                                                                                         \
    if ((e)->P.W == 64)                                                                        \
      hipLaunchKernelGGL(kern<64>, dim3(grid), dim3(pwf_nt<64>()), 0, (hipStream_t)(stream), __VA_ARGS__); \
    else                                                                                       \
      hipLaunchKernelGGL(kern<32>, dim3(grid), dim3(pwf_nt<32>()), 0, (hipStream_t)(stream), __VA_ARGS__); \
  } while (0)
// Every prepared reset state so far is void (a reset or a new seed: the
// Philox keys change): new epoch; in-flight prepare launches finish under the
// old one, whose shadows are never used.  A caller's writes through the state
// pointers need no epoch: a shadow is used only for the episode number and
// task the env holds at its reset.
inline void prep_invalidate(ogbx_powder_env* e) {
  e->prep.epoch += 1u;
  e->prep_launched = 0;
}
#define PW_LAUNCH(kern, e, grid, stream, ...)                                                  \
  do {                                                                                         \
    if ((e)->P.W == 64)                                                                        \
      hipLaunchKernelGGL(kern<64>, dim3(grid), dim3(256), 0, (hipStream_t)(stream), __VA_ARGS__); \
    else                                                                                       \
      hipLaunchKernelGGL(kern<32>, dim3(grid), dim3(256), 0, (hipStream_t)(stream), __VA_ARGS__); \
  } while (0)
}  // namespace

extern "C" {

ogbx_status ogbx_powder_task_table(int32_t num_elems, int32_t task_id, int32_t* seq, int32_t cap,
                                   int32_t* len, int32_t* tol) {
  OGBX_CHECK(num_elems == 2 || num_elems == 5 || num_elems == 8, OGBX_EINVAL, "num_elems must be 2, 5 or 8");
  std::vector<PwSeq> tasks;
  std::vector<int> tols;
  task_tables(num_elems, tasks, tols);
  OGBX_CHECK(task_id >= 1 && task_id <= (int)tasks.size(), OGBX_EINVAL, "task_id out of range");
  const PwSeq& t = tasks[task_id - 1];
  if (len) *len = (int32_t)t.size();
  if (tol) *tol = tols[task_id - 1];
  if (seq)
    for (int q = 0; q < (int)t.size() && q < cap; ++q)
      for (int k = 0; k < 3; ++k) seq[3 * q + k] = t[q][k];
  return OGBX_OK;
}


#ifdef OGBX_PWF_RULE_STAMPS
extern "C" ogbx_status ogbx_diag_pwf_rules(unsigned long long* out) {
  OGBX_HIP(hipDeviceSynchronize());
  OGBX_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(ogbx::g_pwf_rule), 4096 * 16 * sizeof(unsigned long long)));
  return OGBX_OK;
}
#endif

ogbx_status ogbx_powder_create(const ogbx_powder_opts* opts, int64_t n_envs, int32_t device,
                               ogbx_powder_t* out) {
  OGBX_CHECK(opts && out, OGBX_EINVAL, "ogbx_powder_create: null argument");
  *out = nullptr;
  OGBX_CHECK(n_envs > 0 && n_envs <= (1ll << 31), OGBX_EINVAL, "n_envs out of range");
  const int ws = opts->world_size;
  OGBX_CHECK(ws == 32 || ws == 64, OGBX_EINVAL, "world_size must be 32 or 64");
  const int ne = opts->num_elems;
  OGBX_CHECK(ne == 2 || ne == 5 || ne == 8, OGBX_EINVAL, "num_elems must be 2, 5 or 8");
  OGBX_CHECK(opts->grid_size == 4 && opts->brush_size == 4, OGBX_EINVAL,
             "only the registered grid_size=4 / brush_size=4 are supported");
  OGBX_CHECK(opts->max_episode_steps > 0, OGBX_EINVAL, "max_episode_steps must be positive");
  OGBX_CHECK(opts->env_base >= 0, OGBX_EINVAL, "env_base must be >= 0");
  ogbx_status st = use_device(device);
  if (st != OGBX_OK) return st;
  auto* e = new ogbx_powder_env();
  e->device = device;
  e->n = n_envs;
  e->full = ne != 2;
  PowderParams& P = e->P;
  std::memset(&P, 0, sizeof(P));
  P.H = P.W = ws;
  P.grid = opts->grid_size;
  P.brush = opts->brush_size;
  P.xy_size = (ws - P.brush) / P.grid + 1;
  P.num_elems = ne;
  // _elems (powderworld_env.py:57-62): element id per element index
  static const int ids2[2] = {8, 9}, ids8[8] = {2, 3, 7, 8, 9, 4, 5, 6};
  for (int k = 0; k < ne; ++k) P.elem_ids[k] = ne == 2 ? ids2[k] : ids8[k];
  P.max_steps = opts->max_episode_steps;
  P.env_base = opts->env_base;
  // render LUT: uint8(clip(float32(c)/255 * 1 + 0) * 255) (sim.py:402-453)
  static const int colors[21][3] = {
      {236, 240, 241}, {108, 122, 137}, {243, 194, 58}, {75, 119, 190}, {179, 157, 219},
      {202, 105, 36},  {137, 196, 244}, {249, 104, 14}, {38, 194, 129}, {38, 67, 72},
      {157, 41, 51},   {176, 207, 120}, {255, 179, 167}, {191, 85, 236}, {0, 229, 255},
      {61, 90, 254},   {121, 85, 72},   {56, 142, 60},  {158, 157, 36}, {198, 40, 40},
      {224, 64, 251}};
  for (int i = 0; i < 21; ++i)
    for (int c = 0; c < 3; ++c) {
      float v = (float)colors[i][c] / 255.0f;
      v = (1.0f - 0.0f) * v + 0.0f * v;
      v = v < 0.0f ? 0.0f : (v > 1.0f ? 1.0f : v);
      P.lut[i] |= (uint32_t)(uint8_t)(v * 255.0f) << (8 * c);
    }
  vel_bin_thresholds(P.vel_q);
  std::vector<PwSeq> tasks;
  std::vector<int> tols;
  task_tables(ne, tasks, tols);
  P.num_tasks = (int)tasks.size();
  P.tol = tols[0];
  for (int t = 0; t < P.num_tasks; ++t) {
    P.tol_task[t] = tols[t];
    P.seq_len[t] = (int)tasks[t].size();
    e->max_seq = std::max(e->max_seq, P.seq_len[t]);
    for (size_t q = 0; q < tasks[t].size(); ++q)
      for (int k = 0; k < 3; ++k) P.seq[t][q][k] = (int8_t)tasks[t][q][k];
  }
  const size_t n = (size_t)n_envs, HW = (size_t)ws * ws;
  hipError_t h = hipMalloc(&e->Pd, sizeof(PowderParams));
  if (h == hipSuccess) h = hipMemcpy(e->Pd, &P, sizeof(PowderParams), hipMemcpyHostToDevice);
  if (h == hipSuccess) h = hipMalloc(&e->S.world, n * HW);
  if (h == hipSuccess) h = hipMalloc(&e->S.ctrl, n * sizeof(int32_t));
  if (h == hipSuccess) h = hipMalloc(&e->S.elapsed, n * sizeof(int32_t));
  if (h == hipSuccess) h = hipMalloc(&e->S.episode, n * sizeof(uint32_t));
  if (h == hipSuccess) h = hipMemset(e->S.world, 0, n * HW);
  if (h == hipSuccess) h = hipMemset(e->S.ctrl, 0, n * sizeof(int32_t));
  if (h == hipSuccess) h = hipMemset(e->S.elapsed, 0, n * sizeof(int32_t));
  if (h == hipSuccess) h = hipMemset(e->S.episode, 0, n * sizeof(uint32_t));
  if (e->full) {
    if (h == hipSuccess) h = hipMalloc(&e->S.mom, n * HW);
    if (h == hipSuccess) h = hipMalloc(&e->S.vel, n * HW * sizeof(float2));
    if (h == hipSuccess) h = hipMalloc(&e->S.goal_env, n * HW);
    if (h == hipSuccess) h = hipMalloc(&e->S.crg, n * HW * sizeof(uint16_t));
    if (h == hipSuccess) h = hipMalloc(&e->S.cb, n * HW);
    if (h == hipSuccess) h = hipMalloc(&e->handled, n);
    if (h == hipSuccess) h = hipMalloc(&e->cost, n * sizeof(uint32_t));
    if (h == hipSuccess) h = hipMalloc(&e->order, n * sizeof(int32_t));
    if (h == hipSuccess) h = hipMemset(e->cost, 0, n * sizeof(uint32_t));
    if (const char* v = std::getenv("OGBX_PWF_LIGHT")) e->light = std::atoi(v) != 0;  // A/B knob
    if (const char* v = std::getenv("OGBX_PWF_PREP_OPS")) e->prep_ops = std::max(0, std::atoi(v));  // A/B knob
    if (e->prep_ops > 0) {
      if (h == hipSuccess) h = hipMalloc(&e->prep.world, n * HW);
      if (h == hipSuccess) h = hipMalloc(&e->prep.mom, n * HW);
      if (h == hipSuccess) h = hipMalloc(&e->prep.vel, n * HW * sizeof(float2));
      if (h == hipSuccess) h = hipMalloc(&e->prep.goal, n * HW);
      if (h == hipSuccess) h = hipMalloc(&e->prep.tag, n * sizeof(uint32_t));
      if (h == hipSuccess) h = hipMalloc(&e->prep.ep, n * sizeof(uint32_t));
      if (h == hipSuccess) h = hipMalloc(&e->prep.q, n * sizeof(int32_t));
      if (h == hipSuccess) h = hipMalloc(&e->prep.task, n * sizeof(int32_t));
      if (h == hipSuccess) h = hipMemset(e->prep.tag, 0, n * sizeof(uint32_t));
      e->prep.epoch = 1;  // tag 0: never prepared
      int least = 0, greatest = 0;
      if (h == hipSuccess) h = hipDeviceGetStreamPriorityRange(&least, &greatest);
      if (h == hipSuccess) h = hipStreamCreateWithPriority(&e->side, hipStreamNonBlocking, least);
      if (h == hipSuccess) h = hipEventCreateWithFlags(&e->ev_fork, hipEventDisableTiming);
      if (h == hipSuccess) h = hipEventCreateWithFlags(&e->ev_side, hipEventDisableTiming);
    }
    if (h == hipSuccess) h = hipMemset(e->S.mom, 0, n * HW);
    if (h == hipSuccess) h = hipMemset(e->S.vel, 0, n * HW * sizeof(float2));
    if (h == hipSuccess) h = hipMemset(e->S.goal_env, 0, n * HW);
  } else {
    if (h == hipSuccess) h = hipMalloc(&e->goals, (size_t)P.num_tasks * HW);
    if (h == hipSuccess) {
      PW_LAUNCH(pw_goal_kernel, e, P.num_tasks, 0, e->Pd, e->goals);
      h = hipGetLastError();
    }
  }
  if (h == hipSuccess) h = hipDeviceSynchronize();
  if (h != hipSuccess) {
    ogbx_powder_destroy(e);
    return hip_fail(h, "ogbx_powder_create");
  }
  *out = e;
  return OGBX_OK;
}

ogbx_status ogbx_powder_destroy(ogbx_powder_t e) {
  if (!e) return OGBX_OK;
  (void)hipSetDevice(e->device);
  (void)hipFree(e->Pd);
  (void)hipFree(e->S.world);
  (void)hipFree(e->S.ctrl);
  (void)hipFree(e->S.elapsed);
  (void)hipFree(e->S.episode);
  (void)hipFree(e->S.mom);
  (void)hipFree(e->S.vel);
  (void)hipFree(e->S.goal_env);
  (void)hipFree(e->S.crg);
  (void)hipFree(e->S.cb);
  (void)hipFree(e->goals);
  (void)hipFree(e->handled);
  (void)hipFree(e->cost);
  (void)hipFree(e->order);
  if (e->side) (void)hipStreamSynchronize(e->side);
  (void)hipFree(e->prep.world);
  (void)hipFree(e->prep.mom);
  (void)hipFree(e->prep.vel);
  (void)hipFree(e->prep.goal);
  (void)hipFree(e->prep.tag);
  (void)hipFree(e->prep.ep);
  (void)hipFree(e->prep.q);
  (void)hipFree(e->prep.task);
  if (e->ev_fork) (void)hipEventDestroy(e->ev_fork);
  if (e->ev_side) (void)hipEventDestroy(e->ev_side);
  if (e->side) (void)hipStreamDestroy(e->side);
  delete e;
  return OGBX_OK;
}

ogbx_status ogbx_powder_describe(ogbx_powder_t e, int32_t* world_size, int32_t* xy_action_size,
                                 int32_t* num_elems, int32_t* num_tasks, int32_t* tol) {
  OGBX_CHECK(e, OGBX_EINVAL, "null handle");
  if (world_size) *world_size = e->P.W;
  if (xy_action_size) *xy_action_size = e->P.xy_size;
  if (num_elems) *num_elems = e->P.num_elems;
  if (num_tasks) *num_tasks = e->P.num_tasks;
  if (tol) *tol = e->P.tol;
  return OGBX_OK;
}

ogbx_status ogbx_powder_goal_worlds(ogbx_powder_t e, uint8_t* out) {
  OGBX_CHECK(e && out, OGBX_EINVAL, "null argument");
  OGBX_CHECK(!e->full, OGBX_EINVAL,
             "medium/hard goal worlds are stochastic and per env (ogbx_powder_full_state goal_ids)");
  OGBX_HIP(hipSetDevice(e->device));
  OGBX_HIP(hipMemcpy(out, e->goals, (size_t)e->P.num_tasks * e->P.H * e->P.W,
                     hipMemcpyDeviceToHost));
  return OGBX_OK;
}

ogbx_status ogbx_powder_reset(ogbx_powder_t e, const int32_t* task_id, const uint8_t* mask,
                              const int32_t* reset_action, const float* rand, int32_t rand_rows,
                              uint8_t* obs, uint8_t* goal_obs, uint64_t seed, void* stream) {
  OGBX_CHECK(e && obs && goal_obs, OGBX_EINVAL, "ogbx_powder_reset: null argument");
  OGBX_CHECK(rand == nullptr || e->full, OGBX_EINVAL, "rand fields apply to medium/hard worlds only");
  OGBX_CHECK(rand == nullptr || (task_id != nullptr && reset_action != nullptr && rand_rows >= e->max_seq + 1),
             OGBX_EINVAL, "injected rand needs task_id, reset_action and rand_rows >= longest task + 1");
  OGBX_HIP(hipSetDevice(e->device));
  e->seed = seed;
  prep_invalidate(e);
  e->order_ready = false;
  uint32_t k0, k1, r0, r1;
  seed_key(seed, kTagPowderReset, &k0, &k1);
  seed_key(seed, kTagPowderRand, &r0, &r1);
  if (e->full) {
    PWF_LAUNCH(pwf_reset_kernel, e, (uint32_t)e->n, stream, e->Pd, e->S, task_id, mask, reset_action, rand,
              rand_rows, obs, goal_obs, k0, k1, r0, r1);
    OGBX_LAUNCHED("pwf_reset_kernel");
  } else {
    PW_LAUNCH(pw_reset_kernel, e, (uint32_t)e->n, stream, e->Pd, e->S, e->goals, task_id, mask, reset_action,
              obs, goal_obs, k0, k1);
    OGBX_LAUNCHED("pw_reset_kernel");
  }
  e->was_reset = true;
  e->phase = mask == nullptr ? 0 : -1;
  return OGBX_OK;
}

ogbx_status ogbx_powder_step(ogbx_powder_t e, const int32_t* action, int32_t k_steps,
                             const int32_t* draws, const float* rand, uint8_t* obs, float* reward,
                             uint8_t* terminated, uint8_t* truncated, uint8_t* success,
                             int32_t auto_reset, void* stream) {
  OGBX_CHECK(e && action && obs && reward && terminated && truncated && success, OGBX_EINVAL,
             "ogbx_powder_step: null argument");
  OGBX_CHECK(e->was_reset, OGBX_ESTATE, "Cannot call env.step() before calling env.reset()");
  OGBX_CHECK(k_steps >= 1, OGBX_EINVAL, "k_steps must be >= 1");
  OGBX_CHECK(rand == nullptr || e->full, OGBX_EINVAL, "rand fields apply to medium/hard worlds only");
  OGBX_HIP(hipSetDevice(e->device));
  uint32_t k0, k1, a0, a1, r0, r1;
  seed_key(e->seed, kTagPowderReset, &k0, &k1);
  seed_key(e->seed, kTagPowderAction, &a0, &a1);
  seed_key(e->seed, kTagPowderRand, &r0, &r1);
  if (e->full) {
    bool all_full = false;  // every in-phase env runs the full kernel this step
    if (e->phase >= 0 && k_steps == 1) {
      const int64_t T = e->P.max_steps > 0 ? e->P.max_steps : 0;
      const int64_t j = (auto_reset && T > 0) ? e->phase % T : e->phase;  // the env's elapsed steps
      all_full = j % 3 == 2 || (auto_reset && T > 0 && j + 1 >= T);
    }
    const bool light = e->light && k_steps == 1 && !all_full;
    // prepared next-episode resets (PwPrep): in phase with auto-reset, one
    // prepare launch of prep_ops replay ops on the side stream per render-only
    // step until every env's reset is launched (the longest task: max_seq + 1
    // ops); the synchronized reset step joins the side stream and loads them
    const int64_t T = e->P.max_steps > 0 ? e->P.max_steps : 0;
    const bool prep_on = e->prep_ops > 0 && e->side != nullptr && e->phase >= 0 && auto_reset && T > 0 &&
                         k_steps == 1 && rand == nullptr && draws == nullptr;
    ogbx::PwPrep prep = e->prep;
    prep.use = 0;
    bool sync_reset = false;
    if (prep_on) {
      const int64_t j = e->phase % T;
      sync_reset = j + 1 >= T;
      if (sync_reset && e->prep_launched >= e->max_seq + 1 && e->side_pending) {
        OGBX_HIP(hipStreamWaitEvent((hipStream_t)stream, e->ev_side, 0));
        e->side_pending = false;
        prep.use = 1;
      }
    }
    // fork before this render-only step's launches, so that the prepare may
    // run beside them (it reads no state they write but ctrl's stage bits)
    const bool prep_launch = prep_on && light && !sync_reset && e->prep_launched < e->max_seq + 1;
    if (prep_launch) {
      OGBX_HIP(hipEventRecord(e->ev_fork, (hipStream_t)stream));
      OGBX_HIP(hipStreamWaitEvent(e->side, e->ev_fork, 0));
    }
    // the order of the next step's full launch, if the next step is an
    // in-phase full step: sorted by a workgroup of this light launch
    const bool had_order = e->order_ready;
    const bool had_by_task = e->order_by_task;
    e->order_ready = false;
    int32_t order_mode = 0;
    if (light && e->phase >= 0 && e->n <= INT32_MAX) {
      const int64_t jn = (auto_reset && T > 0) ? (e->phase + 1) % T : e->phase + 1;
      const bool sync_next = auto_reset && T > 0 && jn + 1 >= T;
      if (jn % 3 == 2 || sync_next) order_mode = sync_next ? 2 : 1;
    }
    if (light) {
      PW_LAUNCH(pwf_light_step_kernel, e, (uint32_t)e->n + (order_mode ? 1u : 0u), stream, e->Pd, e->S, action, draws,
                obs, reward, terminated, truncated, success, auto_reset, a0, a1, e->handled, (int32_t)e->cache_stale,
                order_mode, (int32_t)e->n, e->cost, e->order);
      OGBX_LAUNCHED("pwf_light_step_kernel");
      e->order_ready = order_mode != 0;
      e->order_by_task = order_mode == 2;
    }
    // in phase, a render-only step leaves (nearly) no env to the full kernel
    if (light && e->phase >= 0) {
      const int32_t chunk = kPwfSparseChunk;
      PWF_LAUNCH(pwf_step_kernel_sparse, e, (uint32_t)((e->n + chunk - 1) / chunk), stream, e->Pd, e->S, e->n,
                 action, draws, rand, k_steps, obs, reward, terminated, truncated, success, auto_reset, k0, k1, a0,
                 a1, r0, r1, e->handled, (int32_t)e->cache_stale, chunk, (const int32_t*)nullptr, (uint32_t*)nullptr,
                 prep);
    } else {
      // in-phase full step: workgroups longest first (the synchronized goal
      // replays by task length, forward steps by last measured cost)
      const int32_t* order = nullptr;
      if (all_full && e->n <= INT32_MAX) {
        const int64_t T = e->P.max_steps > 0 ? e->P.max_steps : 0;
        const int64_t j = (auto_reset && T > 0) ? e->phase % T : e->phase;
        // a synchronized reset step replays by task length, unless it loads
        // prepared states (then the forward-cost order)
        const int32_t by_task = (auto_reset && T > 0 && j + 1 >= T && !prep.use) ? 1 : 0;
        if (!(had_order && had_by_task == (by_task != 0))) {
          hipLaunchKernelGGL(pwf_order_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, e->Pd, e->S.ctrl, e->cost,
                             (int32_t)e->n, by_task, e->order);
          OGBX_LAUNCHED("pwf_order_kernel");
        }
        order = e->order;
      }
      PWF_LAUNCH(pwf_step_kernel_dense, e, (uint32_t)e->n, stream, e->Pd, e->S, e->n, action, draws, rand, k_steps,
                 obs, reward, terminated, truncated, success, auto_reset, k0, k1, a0, a1, r0, r1,
                 light ? e->handled : (const uint8_t*)nullptr, (int32_t)e->cache_stale, 1, order, e->cost, prep);
    }
    OGBX_LAUNCHED("pwf_step_kernel");
    if (sync_reset) e->prep_launched = 0;  // the next episode's round starts
    if (prep_launch) {
      uint32_t pk0, pk1, pr0, pr1;
      seed_key(e->seed, kTagPowderReset, &pk0, &pk1);
      seed_key(e->seed, kTagPowderRand, &pr0, &pr1);
      PWF_LAUNCH(pwf_prepare_kernel, e, (uint32_t)e->n, e->side, e->Pd, e->S, e->prep, e->prep_ops, pk0, pk1, pr0,
                 pr1);
      OGBX_LAUNCHED("pwf_prepare_kernel");
      OGBX_HIP(hipEventRecord(e->ev_side, e->side));
      e->side_pending = true;
      e->prep_launched += e->prep_ops;
    }
    e->cache_stale = false;  // every env's cache was written by one of the two kernels
    if (e->phase >= 0) e->phase += k_steps;
  } else {
    PW_LAUNCH(pw_step_kernel, e, (uint32_t)e->n, stream, e->Pd, e->S, e->goals, e->n, action, draws, k_steps, obs,
              reward, terminated, truncated, success, auto_reset, k0, k1, a0, a1);
    OGBX_LAUNCHED("pw_step_kernel");
  }
  return OGBX_OK;
}

ogbx_status ogbx_powder_state(ogbx_powder_t e, uint8_t** world, int32_t** ctrl, int32_t** elapsed,
                              uint32_t** episode) {
  OGBX_CHECK(e, OGBX_EINVAL, "null handle");
  if (world) *world = e->S.world;
  if (world) e->cache_stale = true;
  if (ctrl) *ctrl = e->S.ctrl;
  if (elapsed) *elapsed = e->S.elapsed;
  if (episode) *episode = e->S.episode;
  e->was_reset = true;
  return OGBX_OK;
}

ogbx_status ogbx_powder_state_view(ogbx_powder_t e, const uint8_t** world, const int8_t** momentum,
                                   const float** velocity, const uint8_t** goal_ids) {
  OGBX_CHECK(e, OGBX_EINVAL, "null handle");
  OGBX_CHECK(e->full || (!momentum && !velocity && !goal_ids), OGBX_EINVAL,
             "easy worlds carry no momentum / velocity / per-env goals");
  if (world) *world = e->S.world;
  if (momentum) *momentum = e->S.mom;
  if (velocity) *velocity = reinterpret_cast<const float*>(e->S.vel);
  if (goal_ids) *goal_ids = e->S.goal_env;
  return OGBX_OK;
}

ogbx_status ogbx_powder_state_written(ogbx_powder_t e) {
  OGBX_CHECK(e, OGBX_EINVAL, "null handle");
  e->cache_stale = true;
  e->phase = -1;  // a restored state need not step in phase with the last reset
  e->was_reset = true;
  return OGBX_OK;
}

ogbx_status ogbx_powder_set_phase(ogbx_powder_t e, int64_t phase) {
  OGBX_CHECK(e, OGBX_EINVAL, "null handle");
  OGBX_CHECK(phase >= -1, OGBX_EINVAL, "phase must be >= -1");
  e->phase = phase;
  return OGBX_OK;
}

ogbx_status ogbx_powder_set_seed(ogbx_powder_t e, uint64_t seed) {
  OGBX_CHECK(e, OGBX_EINVAL, "null handle");
  prep_invalidate(e);
  e->seed = seed;
  return OGBX_OK;
}

ogbx_status ogbx_powder_full_state(ogbx_powder_t e, int8_t** momentum, float** velocity, uint8_t** goal_ids) {
  OGBX_CHECK(e, OGBX_EINVAL, "null handle");
  OGBX_CHECK(e->full, OGBX_EINVAL, "easy worlds carry no momentum / velocity / per-env goals");
  if (momentum) *momentum = e->S.mom;
  if (velocity) *velocity = reinterpret_cast<float*>(e->S.vel);
  if (velocity) e->cache_stale = true;
  if (goal_ids) *goal_ids = e->S.goal_env;
  return OGBX_OK;
}

ogbx_status ogbx_powder_forward(ogbx_powder_t e, const uint8_t* world_in, int64_t n_worlds,
                                int32_t steps, uint8_t* world_out, void* stream) {
  OGBX_CHECK(e && world_in && world_out && n_worlds >= 0 && steps >= 0, OGBX_EINVAL,
             "ogbx_powder_forward: bad argument");
  OGBX_CHECK(!e->full, OGBX_EINVAL, "packed-byte forward is the easy element set; use ogbx_powder_forward_full");
  if (n_worlds == 0) return OGBX_OK;
  OGBX_HIP(hipSetDevice(e->device));
  PW_LAUNCH(pw_forward_kernel, e, (uint32_t)n_worlds, stream, e->Pd, world_in, world_out, steps);
  OGBX_LAUNCHED("pw_forward_kernel");
  return OGBX_OK;
}

ogbx_status ogbx_powder_forward_full(ogbx_powder_t e, const float* world_in, int64_t n_worlds, int32_t steps,
                                     const float* rand, float* world_out, uint8_t* rgb_out, void* stream) {
  OGBX_CHECK(e && world_in && world_out && n_worlds >= 0 && steps >= 0, OGBX_EINVAL,
             "ogbx_powder_forward_full: bad argument");
  if (n_worlds == 0) return OGBX_OK;
  OGBX_HIP(hipSetDevice(e->device));
  uint32_t r0, r1;
  seed_key(e->seed, kTagPowderRand, &r0, &r1);
  PWF_LAUNCH(pwf_forward_kernel, e, (uint32_t)n_worlds, stream, e->Pd, world_in, n_worlds, steps, rand, world_out,
            rgb_out, r0, r1);
  OGBX_LAUNCHED("pwf_forward_kernel");
  return OGBX_OK;
}

}  // extern "C"
