// powder_full.h -- the full powderworld forward (medium / hard element sets)
// as a workgroup-level device routine; included by powder.hip.
//
// Reference: ogbench/powderworld/sim.py -- PWSim.forward (:363-380) running
// Stone, Gravity, Sand, FluidFlow, Ice, Water, Fire, Plant and Velocity
// (:284-308, 461-982) on the (9, H, W) float32 world with three float32 rand
// fields per forward (rand_movement, rand_interact, rand_element).
//
// State per cell (exact for every state the envs reach: densities are a
// function of the id, gravity is the element default except for stone,
// channels 5 and 7 stay 0):
//   a: id (bits 0-4) | GravityInter (bit 5, ch 2) | DidGravity (bit 6, ch 8)
//   m: fluid momentum (ch 6), int8 in {-2, 0, 2}
//   v: velocity (ch 3, ch 4) float32
// Float32 arithmetic follows the reference op by op with no contraction
// (-ffp-contract=off); the 3x3 velocity blur is summed in NumPy's einsum
// order ((t4+t0)+t8 + (t5+t1)) + ((t6+t2) + (t7+t3)) (oracle/powder_full_np.py).
#pragma once

#include <stdint.h>

#include <type_traits>

namespace ogbx {

enum PwElem : int {
  kEmpty = 0, kWall = 1, kSand = 2, kWater = 3, kGas = 4, kWood = 5, kIce = 6, kFire = 7, kPlant = 8,
  kStone = 9, kLava = 10, kAcid = 11, kDust = 12, kFish = 14, kBird = 15, kKangaroo = 16, kMole = 17,
  kLemming = 18
};

// LDS of one env: the state (id|flags, momentum, velocity), the goal ids, the
// rand decision bits and the rule scratch.  A rule's moves are decided by each
// cell's owner from the old state and held in registers across one barrier
// (Moves / commit_moved); conversions go through the scratch flags.
template <int WS>
struct alignas(16) PwFullShared {
  static constexpr int C = WS * WS;
  alignas(16) uint8_t a[C];
  alignas(16) int8_t m[C];
  alignas(16) float2 v[C];
  alignas(16) uint8_t g[C];    // this env's goal ids
  alignas(16) uint16_t rb[C];  // rand decision bits of the current forward (rand_bits)
  union {
    struct {  // rule scratch
      alignas(16) uint8_t f1[C];
      alignas(16) uint8_t f2[C];
      alignas(16) int8_t sw[C];
    };
    alignas(16) uint32_t ob[C * 6 / 4];  // observation staging (between forwards)
  };
  uint32_t lut[32];
  int32_t elem_ids[8];
  float vel_q[8];  // angle-bin thresholds on q (PowderParams::vel_q)
  alignas(8) int32_t red[16];  // presence(); fire() reads it as 8 x uint64 (hot rows per wave)
  int32_t red_e[16];  // errors()
  int32_t red_v[16];  // block_or()
  // per-row cell bitmasks (bit c = column c) of rule predicates, rows -1..H:
  // rows -1 and H are zero padding (pwf_tables), so 3x3 queries read three
  // rows with no bounds branch
  uint64_t rowm[3][WS + 2];
};

// render colours as float32 c / 255 (sim.py:402-453), velocity colour
__constant__ float kPwColDev[21][3] = {
    {236 / 255.f, 240 / 255.f, 241 / 255.f}, {108 / 255.f, 122 / 255.f, 137 / 255.f},
    {243 / 255.f, 194 / 255.f, 58 / 255.f},  {75 / 255.f, 119 / 255.f, 190 / 255.f},
    {179 / 255.f, 157 / 255.f, 219 / 255.f}, {202 / 255.f, 105 / 255.f, 36 / 255.f},
    {137 / 255.f, 196 / 255.f, 244 / 255.f}, {249 / 255.f, 104 / 255.f, 14 / 255.f},
    {38 / 255.f, 194 / 255.f, 129 / 255.f},  {38 / 255.f, 67 / 255.f, 72 / 255.f},
    {157 / 255.f, 41 / 255.f, 51 / 255.f},   {176 / 255.f, 207 / 255.f, 120 / 255.f},
    {255 / 255.f, 179 / 255.f, 167 / 255.f}, {191 / 255.f, 85 / 255.f, 236 / 255.f},
    {0 / 255.f, 229 / 255.f, 255 / 255.f},   {61 / 255.f, 90 / 255.f, 254 / 255.f},
    {121 / 255.f, 85 / 255.f, 72 / 255.f},   {56 / 255.f, 142 / 255.f, 60 / 255.f},
    {158 / 255.f, 157 / 255.f, 36 / 255.f},  {198 / 255.f, 40 / 255.f, 40 / 255.f},
    {224 / 255.f, 64 / 255.f, 251 / 255.f}};

// Render colour of one cell (PWRenderer.render, sim.py:425-453): the exact
// LUT colour at zero velocity, else the float32 blend toward the velocity
// colour with d = clip(|v|/5, 0, 0.5), truncated to uint8.
__device__ __forceinline__ uint32_t pw_rgb(const uint32_t* lut, uint32_t id, float2 v) {
  if (v.x == 0.0f && v.y == 0.0f) return lut[id];
  const float mag = sqrtf(v.x * v.x + v.y * v.y);
  const float d = fminf(fmaxf(mag / 5.0f, 0.0f), 0.5f);
  const float vc[3] = {200 / 255.f, 100 / 255.f, 100 / 255.f};
  uint32_t out = 0;
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) {
    float x = (1.0f - d) * kPwColDev[id][ch] + d * vc[ch];
    x = fminf(fmaxf(x, 0.0f), 1.0f);
    out |= (uint32_t)(x * 255.0f) << (8 * ch);
  }
  return out;
}

// Rand-field purposes (Philox counter word w): goal replay forward s, the
// reset's forward, the forward of elapsed step el.
constexpr uint32_t kRandGoal = 1u << 24, kRandStart = 2u << 24, kRandStep = 3u << 24;

__device__ __forceinline__ uint32_t fid(uint32_t a) { return a & 31u; }
__device__ __forceinline__ uint32_t fgrav(uint32_t a) { return (a >> 5) & 1u; }
__device__ __forceinline__ uint32_t fdidg(uint32_t a) { return (a >> 6) & 1u; }
__device__ __forceinline__ float fdens(uint32_t a) { return (float)((kDensPacked >> (3u * (a & 31u))) & 7u); }
// density as an integer: float32 differences of these small integers compare
// exactly like the integers, so the rules compare dens_i directly
__device__ __forceinline__ uint32_t dens_i(uint32_t a) { return (uint32_t)(kDensPacked >> (3u * (a & 31u))) & 7u; }

constexpr uint32_t bit(int id) { return 1u << id; }
// id in a set of ids: one shift of the set's mask (a compare chain costs a
// v_cmp + v_cndmask per member)
__device__ __forceinline__ bool in_set(uint32_t mask, uint32_t id) { return (mask >> (id & 31u)) & 1u; }

#ifdef OGBX_PWF_RULE_STAMPS
// Diagnostic build only: shader-clock cycles per rule, accumulated per env
// over every forward: slots 0 presence + rands, 1 stone, 2 gravity, 3 sand,
// 4 fluid, 5 ice, 6 water, 7 fire, 8 plant, 9 velocity, 15 forwards.  Keyed
// by the env the kernel set in FullWorld::diag_env (not blockIdx.x: with the
// longest-first order a workgroup is a slot of that step's sort, and a sparse
// workgroup steps several envs).
__device__ unsigned long long g_pwf_rule[4096 * 16];
#define OGBX_RS_ENV (diag_env >= 0 && diag_env < 4096)
#define OGBX_RS_BEGIN() unsigned long long _rs_prev = __builtin_amdgcn_s_memtime()
#define OGBX_RS(slot)                                                                         \
  do {                                                                                        \
    const unsigned long long _t = __builtin_amdgcn_s_memtime();                               \
    if (threadIdx.x == 0 && OGBX_RS_ENV) g_pwf_rule[diag_env * 16 + (slot)] += _t - _rs_prev; \
    _rs_prev = _t;                                                                            \
  } while (0)
// sub-stamps inside one rule (slots 10..14; the velocity rule's parts)
#define OGBX_VS_BEGIN() unsigned long long _vs_prev = __builtin_amdgcn_s_memtime()
#define OGBX_VS(slot) OGBX_RS_AT(_vs_prev, slot)
#define OGBX_RS_AT(prev, slot)                                                                \
  do {                                                                                        \
    const unsigned long long _t = __builtin_amdgcn_s_memtime();                               \
    if (threadIdx.x == 0 && OGBX_RS_ENV) g_pwf_rule[diag_env * 16 + (slot)] += _t - (prev); \
    (prev) = _t;                                                                              \
  } while (0)
#else
#define OGBX_VS_BEGIN() \
  do {                  \
  } while (0)
#define OGBX_VS(slot) \
  do {                \
  } while (0)
#define OGBX_RS_BEGIN() \
  do {                  \
  } while (0)
#define OGBX_RS(slot) \
  do {                \
  } while (0)
#endif
constexpr uint32_t kVelBit = 1u << 31;  // presence mask: some velocity is nonzero

// Workgroup-level full forward on the LDS state of one world, NT threads.
// Thread t owns the CPT cells of column t % W in rows t / W + k * (NT / W):
// for every k the workgroup touches NT consecutive cells, so byte arrays are
// conflict-free and float2 velocities take the natural two LDS passes.
template <int WS, int NT>
struct FullWorld {
  static constexpr int H = WS, W = WS, C = WS * WS, CPT = C / NT, RPK = NT / W;
  static_assert(NT % W == 0 && CPT * RPK == H, "whole rows per slab");
  static_assert(64 % W == 0, "a wave holds whole rows (fluid row skipping)");
  static_assert(CPT <= 8, "per-cell codes are packed 8 bits per cell in Codes");
  // 8 bits per cell of the thread (conversion codes, angle bins)
  using Codes = typename std::conditional<(CPT <= 4), uint32_t, uint64_t>::type;
  PwFullShared<WS>& s;
  mutable int r0, col;
#ifdef OGBX_PWF_RULE_STAMPS
  int64_t diag_env = -1;  // the env the rule stamps are keyed by (set by the kernel)
#endif
  __device__ __forceinline__ explicit FullWorld(PwFullShared<WS>& sh)
      : s(sh),
        r0(W == 64 ? __builtin_amdgcn_readfirstlane((int)threadIdx.x / W) : (int)threadIdx.x / W),
        col((int)threadIdx.x % W) {}

  // Opaque redefinition of the thread's coordinates: cell/neighbour indices are
  // recomputed after it instead of being hoisted (as VGPRs) across the whole
  // forward by loop-invariant code motion.  At W = 64 a wave is one row, so the
  // row is wave-uniform and kept in an SGPR: every row term of a cell or
  // neighbour index is scalar arithmetic, and only the column is per lane.
  __device__ __forceinline__ void fence_idx() const {
    if constexpr (W == 64) {
      int t = __builtin_amdgcn_readfirstlane(r0);
      asm volatile("" : "+s"(t), "+v"(col));
      r0 = t;
    } else {
      asm volatile("" : "+v"(r0), "+v"(col));
    }
  }
  __device__ __forceinline__ int row(int k) const { return r0 + k * RPK; }
  __device__ __forceinline__ int cell(int k) const { return row(k) * W + col; }
  // periodic neighbour (np.roll semantics)
  __device__ __forceinline__ int nb(int k, int dr, int dc) const {
    static_assert((H & (H - 1)) == 0 && (W & (W - 1)) == 0, "power-of-two worlds: wrap by masking");
    return ((row(k) + dr) & (H - 1)) * W + ((col + dc) & (W - 1));
  }
  // zero-padded neighbour (conv2d padding=1): -1 outside
  __device__ __forceinline__ int zp(int k, int dr, int dc) const {
    const int rr = row(k) + dr, cc = col + dc;
    return ((unsigned)rr < (unsigned)H && (unsigned)cc < (unsigned)W) ? rr * W + cc : -1;
  }
  __device__ __forceinline__ void sync() const { __syncthreads(); }

  struct Cell {
    uint8_t a;
    int8_t m;
    float2 v;
  };
  __device__ __forceinline__ Cell get(int i) const { return Cell{s.a[i], s.m[i], s.v[i]}; }
  __device__ __forceinline__ void put(int i, const Cell& x) const {
    s.a[i] = x.a;
    s.m[i] = x.m;
    s.v[i] = x.v;
  }
  __device__ static __forceinline__ Cell elem(uint32_t id) { return Cell{(uint8_t)elem_cell(id), 0, make_float2(0.f, 0.f)}; }

  // 3x3 zero-padded count of cells whose id satisfies pred (integer-valued)
  template <typename P>
  __device__ __forceinline__ int box(int k, P pred) const {
    int n = 0;
#pragma unroll 1
    for (int q = 0; q < 9; ++q) {  // rolled: keeps the register footprint small
      const int j = zp(k, q / 3 - 1, q % 3 - 1);
      const uint32_t x = s.a[j >= 0 ? j : 0];  // branch-free: load, then mask
      n += ((j >= 0) & pred(fid(x))) ? 1 : 0;
    }
    return n;
  }

  // Per-row bitmasks of a cell predicate: a wave holds whole rows, so one
  // ballot per row and slab gives the row's mask; the row masks go to LDS and
  // every cell answers "how many / any X in my zero-padded 3x3" from the three
  // rows' masks with shifts and popcounts -- uniform across the wave, where
  // the per-cell box() loops and the scatter dilations ran divergent
  // few-lane loops.  Call with every thread; a sync() must separate the
  // writes from the reads.
  template <typename P>
  __device__ __forceinline__ void row_masks(uint64_t* rm, P pred) const {
    const int lane = (int)(threadIdx.x & 63u);
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const uint64_t b = __ballot(pred(k));
      if (W == 64) {
        if (lane == 0) rm[row(k)] = b;
      } else {  // W = 32: lanes 0-31 hold one row, lanes 32-63 the next
        if ((lane & 31) == 0) rm[row(k)] = lane == 0 ? (b & 0xFFFFFFFFull) : (b >> 32);
      }
    }
  }
  // row masks of buffer b, indexable by rows -1..H
  __device__ __forceinline__ uint64_t* rmask(int b) const { return s.rowm[b] + 1; }
  // bits (c-1, c, c+1) of row r's mask (zero outside the world: padding rows)
  __device__ __forceinline__ uint32_t win3(const uint64_t* rm, int r) const {
    const uint64_t x = rm[r];
    return (uint32_t)((col == 0 ? x << 1 : x >> (col - 1)) & 7u);
  }
  __device__ __forceinline__ int count3x3(const uint64_t* rm, int k) const {
    const int r = row(k);
    return __popc(win3(rm, r - 1)) + __popc(win3(rm, r)) + __popc(win3(rm, r + 1));
  }
  __device__ __forceinline__ bool any3x3(const uint64_t* rm, int k) const {
    if constexpr (W == 64) {
      // the wave holds exactly row(k): dilate the three row masks once, in
      // scalar registers, and test the lane's column bit
      const int r = __builtin_amdgcn_readfirstlane(row(k));
      uint64_t x = rm[r - 1] | rm[r] | rm[r + 1];
      x = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(x >> 32)) << 32) |
          (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)x);
      const uint64_t d = x | (x << 1) | (x >> 1);
      return (d >> col) & 1u;
    } else {
      const int r = row(k);
      return (win3(rm, r - 1) | win3(rm, r) | win3(rm, r + 1)) != 0u;
    }
  }

  // ------------------------------------------------------------- rules
  // Moves: the owner of each cell decides its new value from the old state
  // and holds it in registers across the barrier that separates the rule's
  // reads from its writes (no LDS staging copy of the world).
  struct Moves {
    uint32_t am[CPT];  // id|flags byte | momentum byte << 8
    float2 v[CPT];
    uint32_t moved = 0;
  };
  __device__ static __forceinline__ void take(Moves& mv, int k, uint32_t a, int m, float2 v) {
    mv.am[k] = (a & 0xFFu) | (((uint32_t)m & 0xFFu) << 8);
    mv.v[k] = v;
    mv.moved |= 1u << k;
  }
  __device__ __forceinline__ void take_from(Moves& mv, int k, int j) const { take(mv, k, s.a[j], s.m[j], s.v[j]); }
  // Write the moved cells (bit k of mv.moved); the others get own(i), an
  // in-place update of the cell itself (or nothing).
  template <typename Own>
  __device__ __forceinline__ void commit_moved(const Moves& mv, Own own) const {
    fence_idx();
    sync();
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const int i = cell(k);
      if ((mv.moved >> k) & 1u) {
        s.a[i] = (uint8_t)mv.am[k];
        s.m[i] = (int8_t)(mv.am[k] >> 8);
        s.v[i] = mv.v[k];
      } else {
        own(i);
      }
    }
    sync();
  }
  // Written in place with no barrier between the reads and the writes: a
  // stone cell's support reads only the id bits (0-4) of its upper diagonal
  // neighbours, and the rule writes only the GravityInter bit (5) of its own
  // cell, so a neighbour's byte read before or after that neighbour's own
  // update gives the same id (LDS byte stores do not tear).
  __device__ __forceinline__ void stone() const {
    fence_idx();
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const int i = cell(k);
      const uint32_t a = s.a[i];
      if (fid(a) == kStone) {
        const int jl = zp(k, -1, -1), jr = zp(k, -1, 1);
        const uint32_t al = s.a[jl >= 0 ? jl : 0], ar = s.a[jr >= 0 ? jr : 0];
        const int sup = ((jl >= 0) & (fid(al) == kStone)) + ((jr >= 0) & (fid(ar) == kStone));
        s.a[i] = (uint8_t)((a & ~kGrav) | (sup < 2 ? kGrav : 0u));
      }
    }
    sync();
  }

  // BehaviorGravity (sim.py:461-501).  The did-gravity reset (rd) is applied
  // to every staged value; moves are decided locally from rows r-2..r+1
  // (real = dbb & ~dbb(above), real_up = real(above)), no flag pass.
  __device__ static __forceinline__ uint32_t rd(uint32_t a) { return fgrav(a) ? (a & ~kDidg) : a; }
  __device__ __forceinline__ bool dbb(int i, int ib) const {
    const uint32_t a = s.a[i], b = s.a[ib];
    return (dens_i(b) < dens_i(a)) & (bool)fgrav(a) & (bool)fgrav(b);
  }
  __device__ __forceinline__ void gravity() const {
    fence_idx();
    Moves mv;
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const int i = cell(k), up = nb(k, -1, 0), up2 = nb(k, -2, 0), dn = nb(k, 1, 0);
      const bool d0 = dbb(i, dn), d1 = dbb(up, i), d2 = dbb(up2, up);
      const bool down = d0 & !d1, raised = d1 & !d2;
      if (down | raised) {
        const int j = down ? dn : up;
        take(mv, k, rd(s.a[j]) | (raised ? kDidg : 0u), s.m[j], s.v[j]);
      }
    }
    commit_moved(mv, [&](int i) { s.a[i] = (uint8_t)rd(s.a[i]); });
  }

  // rows (bit r) holding a cell of the id set `ids`: W = 64 (a wave is a row),
  // one 64-bit word per wave through s.red; ~0 at W = 32.  Contains a barrier.
  __device__ __forceinline__ uint64_t rows_with(uint32_t ids) const {
    if constexpr (W == 64) {
      uint64_t mine = 0;
#pragma unroll
      for (int k = 0; k < CPT; ++k)
        mine |= (__ballot(in_set(ids, fid(s.a[cell(k)]))) != 0ull ? 1ull : 0ull) << row(k);
      if ((threadIdx.x & 63) == 0) reinterpret_cast<uint64_t*>(s.red)[threadIdx.x >> 6] = mine;
      sync();
      uint64_t all = 0;
#pragma unroll
      for (int w = 0; w < NT / 64; ++w) all |= reinterpret_cast<const uint64_t*>(s.red)[w];
      return all;
    } else {
      return ~0ull;
    }
  }
  __device__ static __forceinline__ uint64_t rotl1(uint64_t x) { return (x << 1) | (x >> 63); }

  __device__ __forceinline__ void sand() const {
    fence_idx();
    // A cell changes only if it holds sand / dust or the cell above-diagonal
    // (periodic) does, so rows with neither in rows r, r-1 skip their cells;
    // pass 0 moves sand / dust at most one row down, which widens the set
    // for pass 1.
    const uint64_t S0 = rows_with(bit(kSand) | bit(kDust)), S1 = S0 | rotl1(S0);
#pragma unroll 1
    for (int pass = 0; pass < 2; ++pass) {
      const int go = pass == 0 ? -1 : 1;        // fall toward -1 (left) then +1 (right)
      const uint32_t fl = pass == 0 ? 1u : 0u;  // fall_dir: rm > 0.5, then rm <= 0.5
      const uint64_t act = pass == 0 ? S0 | rotl1(S0) : S1 | rotl1(S1);
      Moves mvs;
#pragma unroll
      for (int k = 0; k < CPT; ++k) {
        if (!((act >> row(k)) & 1ull)) continue;  // wave-uniform at W = 64
        const int i = cell(k), ibl = nb(k, 1, go), iar = nb(k, -1, -go);
        const uint32_t a = s.a[i], bl = s.a[ibl], ar = s.a[iar];
        const bool elem = in_set(bit(kSand) | bit(kDust), fid(a));
        const bool elem_ar = in_set(bit(kSand) | bit(kDust), fid(ar));
        const bool ndg = !fdidg(a);
        const bool f_own = (s.rb[i] & 1u) == fl, f_ar = (s.rb[iar] & 1u) == fl;
        const bool mv = elem & !fdidg(bl) & f_own & (dens_i(a) > dens_i(bl)) & (bool)fgrav(bl) & ndg;
        const bool in = elem_ar & !fdidg(ar) & f_ar & (dens_i(ar) > dens_i(a)) & (bool)fgrav(ar) & ndg;
        if (mv | in) take_from(mvs, k, mv ? ibl : iar);
      }
      commit_moved(mvs, [](int) {});
    }
  }

  static constexpr uint32_t kFluidIds = bit(kEmpty) | bit(kWater) | bit(kGas) | bit(kLava) | bit(kAcid);
  __device__ static __forceinline__ bool is_fluid(uint32_t id) { return (kFluidIds >> id) & 1u; }

  // FluidFlow (sim.py:593-667), two passes (left, then right).  A cell's move
  // decision mv needs only its own state and its side neighbour's, so real
  // (mv & ~mv(back)) and real_in (real(back)) are evaluated locally from three
  // cells of the row.  New momentum per position: sw after pass 1 (0 / +2),
  // f1 (as int8) after pass 2.
  __device__ __forceinline__ bool fluid_mv(int j, int side, int pass, int mom) const {
    const uint32_t a = s.a[j], sd = s.a[side];
    const int m6 = s.m[j] < 0 ? 0 : (s.m[j] > 0 ? 2 : 1);
    // (rm + ch6) + mom > 0.5 for ch6 in {-2, 0, 2}, mom in {0, 2}: rand_bits
    const bool fall = (s.rb[j] >> (1 + m6 + (mom != 0 ? 3 : 0))) & 1u;
    const bool match = pass == 0 ? fall : !fall;
    const uint32_t id = fid(a);
    const bool air = (bit(kKangaroo) | bit(kLemming)) >> id & 1u;
    const bool elem = (kFluidIds >> id) & 1u;
    return match & elem & (!fdidg(a) | air) & (dens_i(a) > dens_i(sd)) & (bool)fgrav(sd) & (bool)fgrav(a);
  }
  // Lane holding the cell (same row, column col + dc): a wave holds whole rows.
  __device__ __forceinline__ int row_lane(int dc) const {
    const int lane = (int)(threadIdx.x & 63u);
    return (lane & (63 & ~(W - 1))) | ((lane + dc) & (W - 1));
  }
  // One lane rotation of the wave (gfx9 DPP wave_rol / wave_ror): the value of
  // lane (lane + 1) mod 64 / (lane - 1) mod 64.  At W = 64 a wave is exactly
  // one row, so this is the periodic row neighbour with no LDS round trip.
  __device__ static __forceinline__ int wave_rot(int x, bool next) {
    return next ? __builtin_amdgcn_update_dpp(0, x, 0x134, 0xF, 0xF, false)
                : __builtin_amdgcn_update_dpp(0, x, 0x13C, 0xF, 0xF, false);
  }
  template <typename T>
  __device__ __forceinline__ T rowx(T x, int dc) const {
    static_assert(sizeof(T) == 4, "32-bit lanes");
    if constexpr (W == 64) {
      // dc in {-2, -1, 1, 2}, a constant after unrolling; every lane active
      int y = __builtin_bit_cast(int, x);
      const bool next = dc > 0;
      y = wave_rot(y, next);
      if (dc == 2 || dc == -2) y = wave_rot(y, next);
      return __builtin_bit_cast(T, y);
    } else {
      return __shfl(x, row_lane(dc), 64);
    }
  }

  // FluidFlow (sim.py:593-667) in registers: fluid moves never leave a row and
  // a wave holds whole rows, so each wave runs both passes on its rows with
  // lane shuffles for the row neighbours -- no LDS staging and no barriers
  // until the rows are written back.  real = mv & ~mv(back), real_in =
  // real(back); the new momentum is per position.  Rows without an element
  // that can start a move are skipped wave-uniformly.
  __device__ __forceinline__ void fluid() const {
    fence_idx();
#pragma unroll 1
    for (int k = 0; k < CPT; ++k) {  // rows are independent: rolled, few live registers
      const int i = cell(k);
      uint32_t a = s.a[i];
      int m = s.m[i];
      float2 v = s.v[i];
      const uint32_t rb = s.rb[i];
      int mom = 0;
      if (__any((kFluidTrig >> fid(a)) & 1u)) {
#pragma unroll
        for (int pass = 0; pass < 2; ++pass) {
          const int go = pass == 0 ? -1 : 1;
          const uint32_t sd = rowx(a, go);
          const uint32_t id = fid(a);
          const int m6 = m < 0 ? 0 : (m > 0 ? 2 : 1);
          // (rm + ch6) + mom > 0.5 for ch6 in {-2, 0, 2}, mom in {0, 2}: rand_bits
          const bool fall = (rb >> (1 + m6 + (mom != 0 ? 3 : 0))) & 1u;
          const bool match = pass == 0 ? fall : !fall;
          const bool air = ((bit(kKangaroo) | bit(kLemming)) >> id) & 1u;
          const bool elem = (kFluidIds >> id) & 1u;
          const int mv = (int)(match & elem & (!fdidg(a) | air) & (dens_i(a) > dens_i(sd)) & (bool)fgrav(sd) &
                               (bool)fgrav(a));
          const int mv1 = rowx(mv, -go), mv2 = rowx(mv, -2 * go);
          const bool real = mv & !mv1, real_in = mv1 & !mv2;
          mom += real_in ? (pass == 0 ? 2 : -2) : 0;
          const uint32_t ab = rowx(a, -go);
          const int ms = rowx(m, go), mb = rowx(m, -go);
          const float vsx = rowx(v.x, go), vsy = rowx(v.y, go), vbx = rowx(v.x, -go), vby = rowx(v.y, -go);
          a = real ? sd : (real_in ? ab : a);
          m = real ? ms : (real_in ? mb : m);
          v = real ? make_float2(vsx, vsy) : (real_in ? make_float2(vbx, vby) : v);
        }
      }
      const uint32_t id = fid(a);
      if (is_fluid(id) || id == kKangaroo || id == kLemming) m = mom;
      s.a[i] = (uint8_t)a;
      s.m[i] = (int8_t)m;
      s.v[i] = v;
    }
    sync();
  }

  __device__ __forceinline__ void ice() const {
    fence_idx();
    uint64_t* melt = rmask(0);  // empty | fire | lava | water
    row_masks(melt, [&](int k) {
      const uint32_t x = fid(s.a[cell(k)]);
      return in_set(bit(kEmpty) | bit(kFire) | bit(kLava) | bit(kWater), x);
    });
    sync();
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const uint32_t id = fid(s.a[cell(k)]);
      const bool to = (id == kIce) & ri_lt(k, kRi002) & (count3x3(melt, k) > 1);
      if (to) put(cell(k), elem(kWater));  // decided from masks only: in place
    }
    sync();
  }

  __device__ __forceinline__ void water() const {
    fence_idx();
    uint64_t* ice = rmask(0);
    row_masks(ice, [&](int k) { return fid(s.a[cell(k)]) == kIce; });
    sync();
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const uint32_t id = fid(s.a[cell(k)]);
      const bool to = (id == kWater) & re_lt(k, kRe005) & (count3x3(ice, k) >= 3);
      if (to) put(cell(k), elem(kIce));  // decided from masks only: in place
    }
    sync();
  }

  static constexpr uint32_t kBurnable = bit(kWood) | bit(kPlant) | bit(kGas) | bit(kDust) | bit(kFish) | bit(kBird) |
                                        bit(kKangaroo) | bit(kMole) | bit(kLemming);
  __device__ static __forceinline__ bool burnable(uint32_t x) { return in_set(kBurnable, x); }

  // BehaviorFire (sim.py:700-790).  The "is there X in my 3x3" and "how
  // many burnable cells in my 3x3" questions are answered from per-row
  // bitmasks (row_masks): fire|lava before the burn, the burnable cells after
  // it, and the spread sources.
  __device__ __forceinline__ void fire() const {
    static_assert(CPT <= 8, "conversion codes packed 8 bits per cell");
    fence_idx();
    uint64_t* hotm = rmask(0);   // fire | lava before the burn
    uint64_t* burnm = rmask(1);  // burnable cells after the burn
    uint64_t* srcm = rmask(2);   // fire spread sources
    uint32_t flb = 0;             // bit k: this cell was fire or lava before the burn
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const uint32_t id = fid(s.a[cell(k)]);
      flb |= in_set(bit(kFire) | bit(kLava), id) ? 1u << k : 0u;
    }
    row_masks(hotm, [&](int k) { return ((flb >> k) & 1u) != 0u; });
    // rows holding fire or lava (W = 64: a wave is a row; one 64-bit word per
    // wave, OR-ed after the barrier).  Every effect of the rule needs fire or
    // lava in the cell's zero-padded 3x3 (burns, ignition, fading), or a
    // burning 4-neighbour (impulses, periodic), so a row with no hot cell in
    // rows r-1..r+1 (A3) changes nothing and one with none in A3 of r-1..r+1
    // (A5, periodic) reads no non-zero burn flag: such rows skip their cells.
    uint64_t A3 = ~0ull, A5 = ~0ull;
    if constexpr (W == 64) {
      uint64_t mine = 0;
#pragma unroll
      for (int k = 0; k < CPT; ++k) mine |= (__ballot((flb >> k) & 1u) != 0ull ? 1ull : 0ull) << row(k);
      if ((threadIdx.x & 63) == 0) reinterpret_cast<uint64_t*>(s.red)[threadIdx.x >> 6] = mine;
    }
    sync();
    if constexpr (W == 64) {
      uint64_t hot = 0;
#pragma unroll
      for (int w = 0; w < NT / 64; ++w) hot |= reinterpret_cast<const uint64_t*>(s.red)[w];
      A3 = hot | (hot << 1) | (hot >> 1);
      A5 = A3 | (A3 << 1) | (A3 >> 63) | (A3 >> 1) | (A3 << 63);
    }
    // burn decisions; f2 bit 0: burns (pushes its 4 neighbours with 8), bit 1:
    // dust near fire (pushes with 30)
    Codes conv = 0;  // 8 bits per cell: new id + 1, 0 = unchanged
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const int i = cell(k);
      if (!((A3 >> row(k)) & 1ull)) {  // wave-uniform at W = 64
        s.f2[i] = 0;
        continue;
      }
      const uint32_t id = fid(s.a[i]);
      const bool nr = any3x3(hotm, k);
      const bool p005 = ri_lt(k, kRi005), p02 = ri_lt(k, kRi02);
      // burn candidates: wood, bird at ri < 0.05; plant, gas and the animals at
      // ri < 0.2; dust always
      constexpr uint32_t k005 = bit(kWood) | bit(kBird);
      constexpr uint32_t k02 = bit(kPlant) | bit(kGas) | bit(kFish) | bit(kLemming) | bit(kKangaroo) | bit(kMole);
      const bool cand = (in_set(k005, id) & p005) | (in_set(k02, id) & p02) | (id == kDust);
      const bool burn = cand & nr, burn_ice = (id == kIce) & p02 & nr;
      s.f2[i] = (uint8_t)((burn ? 1 : 0) | (((id == kDust) & nr) ? 2 : 0));
      conv |= (Codes)(burn ? kFire + 1u : (burn_ice ? kWater + 1u : 0u)) << (8 * k);
    }
    // burnable cells of the post-burn world (the owner knows its cell's
    // conversion already), published with the burn flags
    row_masks(burnm, [&](int k) {
      const uint32_t to = (uint32_t)(conv >> (8 * k)) & 0xFFu;
      return burnable(to ? to - 1 : fid(s.a[cell(k)]));
    });
    sync();
    // impulses away from a burning neighbour (sim.py:744-752): left, above,
    // below, right; then the conversions (own cells, in place)
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      if (!((A5 >> row(k)) & 1ull)) continue;
      const int i = cell(k);
      const uint32_t L = s.f2[nb(k, 0, -1)], U = s.f2[nb(k, -1, 0)], D = s.f2[nb(k, 1, 0)], R = s.f2[nb(k, 0, 1)];
      const uint32_t to = (uint32_t)(conv >> (8 * k)) & 0xFFu;
      if (to) {
        put(i, elem(to - 1));
      } else if ((L | U | D | R) & 3u) {
        float2 v = s.v[i];
        v.y = v.y + 8.0f * (float)(L & 1);
        v.x = v.x + 8.0f * (float)(U & 1);
        v.x = v.x - 8.0f * (float)(D & 1);
        v.y = v.y - 8.0f * (float)(R & 1);
        v.y = v.y + 30.0f * (float)((L >> 1) & 1);
        v.x = v.x + 30.0f * (float)((U >> 1) & 1);
        v.x = v.x - 30.0f * (float)((D >> 1) & 1);
        v.y = v.y - 30.0f * (float)((R >> 1) & 1);
        s.v[i] = v;
      }
    }
    // (no barrier: the steps below read only own cells and the row masks)
    // fire spread sources: (fire or lava before the burn) with a burnable
    // neighbour, and lava; fading fire (no burnable neighbour)
    uint32_t fade = 0, nbr = 0;  // bit k: some burnable cell in the 3x3
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      if (!((A3 >> row(k)) & 1ull)) continue;  // no fire / lava cell, no source
      const uint32_t id = fid(s.a[cell(k)]);
      const bool b = any3x3(burnm, k);
      nbr |= b ? 1u << k : 0u;
      fade |= ((id == kFire) & re_lt(k, kRe04) & !b) ? 1u << k : 0u;
    }
    row_masks(srcm, [&](int k) {
      const bool fl = (flb >> k) & 1u;
      return (fl & ((nbr >> k) & 1u)) | (fid(s.a[cell(k)]) == kLava);
    });
    sync();
    // empty cells next to a source ignite (ri < 0.3); fire with re < 0.4 and
    // no burnable neighbour fades to empty (sim.py:778-790)
    Codes conv2 = 0;
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      if (!((A3 >> row(k)) & 1ull)) continue;  // no source in the 3x3, no fading fire
      const uint32_t id = fid(s.a[cell(k)]);
      const bool burn_empty = (id == kEmpty) & ri_lt(k, kRi03) & any3x3(srcm, k);
      bool fd = (fade >> k) & 1u;
      if (burn_empty & re_lt(k, kRe04)) fd = !((nbr >> k) & 1u);
      conv2 |= (Codes)(fd ? kEmpty + 1u : (burn_empty ? kFire + 1u : 0u)) << (8 * k);
    }
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const uint32_t to = (uint32_t)(conv2 >> (8 * k)) & 0xFFu;
      if (to) put(cell(k), elem(to - 1));
    }
    sync();
  }

  __device__ __forceinline__ void plant() const {
    fence_idx();
    uint64_t* plm = rmask(0);  // plant
    uint64_t* iwm = rmask(1);  // ice | wood
    row_masks(plm, [&](int k) { return fid(s.a[cell(k)]) == kPlant; });
    row_masks(iwm, [&](int k) {
      const uint32_t x = fid(s.a[cell(k)]);
      return in_set(bit(kIce) | bit(kWood), x);
    });
    // every conversion needs a plant in the zero-padded 3x3 (count >= 1), so
    // rows with no plant in rows r-1..r+1 skip their cells (W = 64)
    uint64_t act = ~0ull;
    if constexpr (W == 64) {
      uint64_t mine = 0;
#pragma unroll
      for (int k = 0; k < CPT; ++k)
        mine |= (__ballot(fid(s.a[cell(k)]) == kPlant) != 0ull ? 1ull : 0ull) << row(k);
      if ((threadIdx.x & 63) == 0) reinterpret_cast<uint64_t*>(s.red)[threadIdx.x >> 6] = mine;
    }
    sync();
    if constexpr (W == 64) {
      uint64_t pr = 0;
#pragma unroll
      for (int w = 0; w < NT / 64; ++w) pr |= reinterpret_cast<const uint64_t*>(s.red)[w];
      act = pr | (pr << 1) | (pr >> 1);
    }
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      if (!((act >> row(k)) & 1ull)) continue;
      const uint32_t id = fid(s.a[cell(k)]);
      const bool grow = id == kWater && ri_lt(k, kRi005);
      const bool seed = id == kEmpty && ri_lt(k, kRi02);
      const int cnt = count3x3(plm, k);
      bool to_plant = grow && cnt <= 3 && cnt >= 1;
      const bool to_empty = grow && cnt > 3;
      if (seed && cnt > 0) to_plant = any3x3(iwm, k);
      // decided from the own cell and the row masks only: converted in place
      if (to_plant | to_empty) put(cell(k), elem(to_plant ? (uint32_t)kPlant : (uint32_t)kEmpty));
    }
    sync();
  }

  // direction d (sim.py direction_func) as (dr, dc): 0 right, 1 below-right,
  // 2 below, 3 below-left, 4 left, 5 above-left, 6 above, 7 above-right
  __device__ static __forceinline__ void dir_of(int d, int& dr, int& dc) {
    dr = (int)((0x01A9u >> (2 * d)) & 3u) - 1;  // 2 bits (value + 1) per direction
    dc = (int)((0x901Au >> (2 * d)) & 3u) - 1;
  }

  // Cells a velocity pass may move, listed when at most kSwapList (two
  // chunks of a wave).
  // (A/B, medium / hard per step: 128 161.3 / 186.0 us, 64 163.2 / 188.9,
  // 256 162.4 / 187.3, 512 169.0 / 194.9, the block rounds alone 166.0 /
  // 191.3: a longer list costs registers in the whole inlined forward)
  static constexpr uint32_t kSwapList = 128;

  // block_or of the bins plus the world's candidate count (cells with a bin)
  // and this wave's first list slot, through one barrier.
  __device__ __forceinline__ uint32_t bins_reduce(uint32_t dirs, Codes binr, uint32_t* total, uint32_t* base) const {
    uint32_t cnt = 0;
#pragma unroll
    for (int k = 0; k < CPT; ++k)
      cnt += (uint32_t)__popcll(__ballot(((uint32_t)(binr >> (8 * k)) & 0xFFu) != 0xFFu));
    dirs = wave_or(dirs);
    const int w = (int)(threadIdx.x >> 6);
    if ((threadIdx.x & 63) == 0) {
      s.red_v[w] = (int32_t)dirs;
      s.red_e[w] = (int32_t)cnt;  // red_e: errors() reads it only across its own barriers
    }
    sync();
    uint32_t all = 0, tot = 0, b = 0;
#pragma unroll
    for (int q = 0; q < NT / 64; ++q) {
      all |= (uint32_t)s.red_v[q];
      const uint32_t c = (uint32_t)s.red_e[q];
      b += q < w ? c : 0u;
      tot += c;
    }
    *total = tot;
    *base = b;
    return all;
  }

  // The swap rounds of one velocity pass run by the first wave over the list
  // of cells that may move (same decisions and writes as the block rounds;
  // the list is in cell order within each wave's slice, and no two matches
  // of a round write the same sw entry, so the order does not matter).
  __device__ __forceinline__ void swap_rounds_listed(Codes binr, uint32_t dirs, uint32_t total, uint32_t base) const {
    static_assert(kSwapList <= C / 2, "list of uint16 entries in f2");
    uint16_t* list = reinterpret_cast<uint16_t*>(s.f2);
    const int lane = (int)(threadIdx.x & 63u);
    const uint64_t lt = (1ull << lane) - 1ull;
    uint32_t off = base;
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const uint32_t b = (uint32_t)(binr >> (8 * k)) & 0xFFu;
      const uint64_t m = __ballot(b != 0xFFu);
      if (b != 0xFFu) list[off + (uint32_t)__popcll(m & lt)] = (uint16_t)(cell(k) | (int)(b << 12));
      off += (uint32_t)__popcll(m);
    }
    sync();
    if (threadIdx.x < 64) {
      constexpr int kChunks = kSwapList / 64;
#pragma unroll 1
      for (int d = 0; d < 8; ++d) {
        if (!((dirs >> d) & 1u)) continue;
        int dr, dc;
        dir_of(d, dr, dc);
        int ii[kChunks], jj[kChunks];
        uint32_t mk = 0;
#pragma unroll
        for (int q = 0; q < kChunks; ++q) {  // phase 1: f1 = d + 1 on matches
          const uint32_t e = (uint32_t)(lane + 64 * q);
          ii[q] = 0;
          jj[q] = 0;
          if (e < total) {
            const uint32_t ent = list[e];
            if ((ent >> 12) == (uint32_t)d) {
              const int i = (int)(ent & 0xFFFu), r = i / W, c = i % W;
              const int j = ((r + dr) & (H - 1)) * W + ((c + dc) & (W - 1));
              ii[q] = i;
              jj[q] = j;
              if ((s.sw[i] == -1) & (s.sw[j] == -1) & (fid(s.a[j]) == kEmpty)) {
                s.f1[i] = (uint8_t)(d + 1);
                mk |= 1u << q;
              }
            }
          }
        }
#pragma unroll
        for (int q = 0; q < kChunks; ++q) {  // phase 2: the choices
          if ((mk >> q) & 1u) {
            const int i = ii[q], r = i / W, c = i % W;
            const int back = ((r - dr) & (H - 1)) * W + ((c - dc) & (W - 1));
            s.sw[jj[q]] = (int8_t)((d + 4) & 7);
            if (s.f1[back] != (uint8_t)(d + 1)) s.sw[i] = (int8_t)d;
          }
        }
      }
    }
    sync();
  }

  __device__ __forceinline__ void velocity() const {
    fence_idx();
    OGBX_VS_BEGIN();
#pragma unroll 1
    for (int pass = 0; pass < 2; ++pass) {
      fence_idx();
      // f2 = angle bin of cells that may move (mag above the pass threshold, not
      // wall), 0xFF otherwise; sw = chosen swap direction (-1 none)
      uint32_t dirs = 0;  // angle bins present among the cells that may move
      Codes binr = 0;  // 8 bits per cell: bin, 0xFF = cannot move
#pragma unroll
      for (int k = 0; k < CPT; ++k) {
        const int i = cell(k);
        const float2 v = s.v[i];
        const float ss = v.x * v.x + v.y * v.y, thr = pass == 0 ? 1.0f : 2.0f;
        uint8_t b8 = 0xFF;
        // sqrt is monotone and exact at the squares 1 and 4, so mag > thr
        // needs ss > thr * thr: only those cells take the root and the quotient
        const float mag = ss > thr * thr ? sqrtf(ss) : 0.0f;
        if (mag > thr && fid(s.a[i]) != kWall) {
          // floor(8 * ang + 0.5) mod 8 with ang from float32 arccos(q): a count
          // of exact float32 thresholds on q (host: vel_bin_thresholds)
          const float q = v.y / (mag + 0.001f);
          int b;
          if (v.x < 0.0f) {
            b = (4 + (q >= s.vel_q[4]) + (q >= s.vel_q[5]) + (q >= s.vel_q[6]) + (q >= s.vel_q[7])) & 7;
          } else {
            b = (q <= s.vel_q[0]) + (q <= s.vel_q[1]) + (q <= s.vel_q[2]) + (q <= s.vel_q[3]);
          }
          b8 = (uint8_t)b;
          dirs |= 1u << b8;
        }
        binr |= (Codes)b8 << (8 * k);
        s.sw[i] = -1;
        s.f1[i] = 0;
      }
      // the world's bins and its count of cells that may move (one barrier)
      uint32_t ncand = 0, wbase = 0;
      dirs = bins_reduce(dirs, binr, &ncand, &wbase);
      OGBX_VS(10);
      if (dirs == 0) {
        // no swap anywhere: v = v * 0.5 + v * 0.5 in place.  With no cell
        // above pass 0's threshold (|v| > 1) none is above pass 1's (|v| > 2)
        // either -- the in-place update changes no normal float, and a
        // subnormal component stays far below both -- so pass 1 is the same
        // update again, applied here without its bins and barrier.
        const int reps = pass == 0 ? 2 : 1;
#pragma unroll
        for (int k = 0; k < CPT; ++k) {
          float2 v = s.v[cell(k)];
          for (int r = 0; r < reps; ++r) {
            v.x = v.x * 0.5f + v.x * 0.5f;
            v.y = v.y * 0.5f + v.y * 0.5f;
          }
          s.v[cell(k)] = v;
        }
        sync();
        OGBX_VS(12);
        if (pass == 0) break;
        continue;
      }
      // Swap rounds in direction order (sim.py:950-962), sparse: only the
      // cells whose bin is the round's direction test for a match (their bins
      // live in registers); a match stamps f1 = d + 1 and, after a barrier,
      // writes its own choice d and its target's (d + 4) mod 8 -- the
      // target's choice wins when a matched cell is itself a target, as in
      // the reference's where(m, a, .) then where(opp, a + 4, .).  Rounds whose
      // bin no cell occupies are identities and skipped.
      if (ncand <= kSwapList) {
        // few cells may move: list them (cell | bin << 12 in f2, free during
        // this rule) and let ONE wave run every round -- its LDS operations
        // are ordered, so the rounds need no barriers (two per round below)
        swap_rounds_listed(binr, dirs, ncand, wbase);
      } else
#pragma unroll 1
      for (int d = 0; d < 8; ++d) {
        if (!((dirs >> d) & 1u)) continue;
        fence_idx();
        int dr, dc;
        dir_of(d, dr, dc);
        uint32_t mk = 0;
#pragma unroll
        for (int k = 0; k < CPT; ++k) {
          if (((uint32_t)(binr >> (8 * k)) & 0xFFu) == (uint32_t)d) {
            const int i = cell(k), j = nb(k, dr, dc);
            if ((s.sw[i] == -1) & (s.sw[j] == -1) & (fid(s.a[j]) == kEmpty)) {
              s.f1[i] = (uint8_t)(d + 1);
              mk |= 1u << k;
            }
          }
        }
        sync();
#pragma unroll
        for (int k = 0; k < CPT; ++k) {
          if ((mk >> k) & 1u) {
            const int i = cell(k);
            s.sw[nb(k, dr, dc)] = (int8_t)((d + 4) & 7);
            if (s.f1[nb(k, -dr, -dc)] != (uint8_t)(d + 1)) s.sw[i] = (int8_t)d;
          }
        }
        sync();
      }
      OGBX_VS(11);
      Moves mvs;
#pragma unroll
      for (int k = 0; k < CPT; ++k) {
        const int i = cell(k);
        const int w = s.sw[i];
        if (w >= 0) {
          int dr, dc;
          dir_of(w, dr, dc);
          const int j = nb(k, dr, dc);
          const float2 old = s.v[i], nv = s.v[j];
          take(mvs, k, s.a[j], s.m[j], make_float2(nv.x * 0.5f + old.x * 0.5f, nv.y * 0.5f + old.y * 0.5f));
        }
      }
      // unswapped cells: v = v * 0.5 + v * 0.5 in place
      commit_moved(mvs, [&](int i) {
        float2 v = s.v[i];
        v.x = v.x * 0.5f + v.x * 0.5f;
        v.y = v.y * 0.5f + v.y * 0.5f;
        s.v[i] = v;
      });
      OGBX_VS(12);
    }
    // decay (x0.95) fused into the 3x3 blur (zero padded) of the decayed
    // field, NumPy's einsum summation order.  A wave holds whole rows: each
    // cell loads its own column of rows r-1, r, r+1 (3 LDS reads instead of
    // 9) and takes the column neighbours' taps from the adjacent lanes with
    // DPP wave shifts (zero outside the row); the results stay in registers
    // until every thread has read the field.
    const float w18 = 1.0f / 18.0f;
    fence_idx();
    float2 res[CPT];
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const int r = row(k);
      const float2 z = make_float2(0.f, 0.f);
      const float2 vu0 = s.v[((r - 1) & (H - 1)) * W + col], vm = s.v[r * W + col],
                   vd0 = s.v[((r + 1) & (H - 1)) * W + col];
      const float2 vu = r > 0 ? vu0 : z, vd = r < H - 1 ? vd0 : z;
      float tx[9], ty[9];
      tx[1] = (vu.x * 0.95f) * w18, ty[1] = (vu.y * 0.95f) * w18;
      tx[4] = (vm.x * 0.95f) * w18, ty[4] = (vm.y * 0.95f) * w18;
      tx[7] = (vd.x * 0.95f) * w18, ty[7] = (vd.y * 0.95f) * w18;
#pragma unroll
      for (int q = 1; q < 9; q += 3) {
        tx[q - 1] = col_prev(tx[q]), ty[q - 1] = col_prev(ty[q]);
        tx[q + 1] = col_next(tx[q]), ty[q + 1] = col_next(ty[q]);
      }
      float2 own = vm;
      own.x = own.x * 0.95f;
      own.y = own.y * 0.95f;
      const float bx = (((tx[4] + tx[0]) + tx[8]) + (tx[5] + tx[1])) + ((tx[6] + tx[2]) + (tx[7] + tx[3]));
      const float by = (((ty[4] + ty[0]) + ty[8]) + (ty[5] + ty[1])) + ((ty[6] + ty[2]) + (ty[7] + ty[3]));
      res[k] = make_float2(bx + own.x * 0.5f, by + own.y * 0.5f);
    }
    sync();
#pragma unroll
    for (int k = 0; k < CPT; ++k) s.v[cell(k)] = res[k];
    sync();
    OGBX_VS(13);
  }

  // The value at column col - 1 / col + 1 of the same row (a wave holds whole
  // rows: DPP wave_shr / wave_shl by one lane), +0 outside the world.
  // At W = 64 the wave is the row: the shift's out-of-range lane (column 0 /
  // 63) already reads +0 (bound_ctrl), so no select is needed.
  __device__ __forceinline__ float col_prev(float x) const {
    const float y = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x138, 0xF, 0xF, true));
    if constexpr (W == 64) return y;
    return col == 0 ? 0.0f : y;
  }
  __device__ __forceinline__ float col_next(float x) const {
    const float y = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x130, 0xF, 0xF, true));
    if constexpr (W == 64) return y;
    return col == W - 1 ? 0.0f : y;
  }

  // ------------------------------------------------------------- env helpers
  // Blank world: walls on the border, empty inside (powderworld_env.py:309-313).
  __device__ __forceinline__ void blank() const {
    fence_idx();
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const int r = row(k), c = col;
      const bool border = r == 0 || r == H - 1 || c == 0 || c == W - 1;
      put(cell(k), elem(border ? (uint32_t)kWall : (uint32_t)kEmpty));
    }
    sync();
  }

  // Every use of a rand field in the rules is a float32 comparison with a
  // constant after adding a few possible integers (sim.py: sand rm > 0.5;
  // fluid (rm + ch6) + mom > 0.5 with ch6 in {-2,0,2}, mom in {0,2}; ri below
  // 0.02/0.05/0.2/0.3; re below 0.05/0.4), so a cell's three floats reduce
  // exactly to 12 decision bits:
  //   bit 0 rm > 0.5 | bits 1-3 (rm + {-2,0,2}) + 0 > 0.5 | bits 4-6 ... + 2 > 0.5
  //   | bits 7-9 ri category (0: < 0.02, 1: < 0.05, 2: < 0.2, 3: < 0.3, 4)
  //   | bits 10-11 re category (0: < 0.05, 1: < 0.4, 2)
  __device__ static __forceinline__ uint32_t rand_bits(float rm, float ri, float re) {
    uint32_t b = rm > 0.5f ? 1u : 0u;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const float x = rm + (float)(2 * j - 2);
      b |= (x + 0.0f > 0.5f ? 1u : 0u) << (1 + j);
      b |= (x + 2.0f > 0.5f ? 1u : 0u) << (4 + j);
    }
    const uint32_t ic = ri < 0.02f ? 0u : (ri < 0.05f ? 1u : (ri < 0.2f ? 2u : (ri < 0.3f ? 3u : 4u)));
    const uint32_t ec = re < 0.05f ? 0u : (re < 0.4f ? 1u : 2u);
    return b | (ic << 7) | (ec << 10);
  }
  // The same 12 bits straight from the three Philox words (u01f_from(w) =
  // (w >> 8) 2^-24, so each decision is a threshold on the word): with rm in
  // [0, 1), bits 1-6 are the constants 0 | rm>.5 | 1 | fl(fl(rm - 2) + 2) > .5
  // | 1 | 1, and every threshold below is where the float32 decision of
  // rand_bits switches (tests/test_powder_rand_bits.py checks all 2^24
  // words of each field against rand_bits).  Eight integer compares per cell
  // instead of three conversions and twenty float operations.
  static constexpr uint32_t kRmHalf = 8388609u << 8, kRmHalfR = 8388610u << 8;
  static constexpr uint32_t kRiT0 = 335545u << 8, kRiT1 = 838861u << 8, kRiT2 = 3355444u << 8, kRiT3 = 5033165u << 8;
  static constexpr uint32_t kReT0 = 838861u << 8, kReT1 = 6710887u << 8;
  __device__ static __forceinline__ uint32_t rand_bits_w(uint32_t wm, uint32_t wi, uint32_t we) {
    const uint32_t b = 0x68u | (wm >= kRmHalf ? 0x5u : 0u) | (wm >= kRmHalfR ? 0x10u : 0u);
    const uint32_t ic = (uint32_t)(wi >= kRiT0) + (uint32_t)(wi >= kRiT1) + (uint32_t)(wi >= kRiT2) +
                        (uint32_t)(wi >= kRiT3);
    const uint32_t ec = (uint32_t)(we >= kReT0) + (uint32_t)(we >= kReT1);
    return b | (ic << 7) | (ec << 10);
  }
  static constexpr uint32_t kRi002 = 1, kRi005 = 2, kRi02 = 3, kRi03 = 4, kRe005 = 1, kRe04 = 2;
  __device__ __forceinline__ bool ri_lt(int k, uint32_t cat) const { return ((s.rb[cell(k)] >> 7) & 7u) < cat; }
  __device__ __forceinline__ bool re_lt(int k, uint32_t cat) const { return ((s.rb[cell(k)] >> 10) & 3u) < cat; }

  // Rand decision bits of one forward for this thread's cells: from injected
  // fields (src = [3, H, W] float32) or Philox (three 4x32 draws per four cells).
  // Philox: the cells of a column whose rows are congruent mod H/4 form a
  // group of four (a thread owns whole groups for CPT = 4 or 8, whatever the
  // thread count), and the group's 12 floats are the 12 words of three calls
  // with counter (4 g + c, env, episode, slot), g = the group's first cell:
  // cell j of the group takes words 3j, 3j + 1, 3j + 2 of the calls' 12.
  __device__ __forceinline__ void fill_rands(const float* __restrict__ src, uint32_t k0, uint32_t k1, uint64_t env, uint32_t ep,
                             uint32_t slot) const {
    fence_idx();
    if (src) {
#pragma unroll 2
      for (int k = 0; k < CPT; ++k) {
        const int i = cell(k);
        s.rb[i] = (uint16_t)rand_bits(src[i], src[C + i], src[2 * C + i]);
      }
      return;
    }
    static_assert(CPT % 4 == 0, "whole groups of four cells per thread");
    constexpr int G = CPT / 4;  // groups per thread; member j of group q is cell q + j G
#pragma unroll 1
    for (int q = 0; q < G; ++q) {
      const uint32_t g = (uint32_t)cell(q);  // row(q) < H / 4: the group's first cell
      uint32_t w[12];
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const u32x4 x = philox4x32_10_wide({4u * g + (uint32_t)c, (uint32_t)env, ep, slot}, k0 ^ (uint32_t)(env >> 32), k1);
        w[4 * c] = x.x, w[4 * c + 1] = x.y, w[4 * c + 2] = x.z, w[4 * c + 3] = x.w;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
        s.rb[cell(q + j * G)] = (uint16_t)rand_bits_w(w[3 * j], w[3 * j + 1], w[3 * j + 2]);
    }
  }

  __device__ __forceinline__ void forward_rand(const float* __restrict__ src, uint32_t k0, uint32_t k1, uint64_t env, uint32_t ep,
                               uint32_t slot) const {
    OGBX_RS_BEGIN();
    const uint32_t P = presence();
    if (P & kRandUsers) fill_rands(src, k0, k1, env, ep, slot);  // own cells; presence() synced already
    sync();
    OGBX_RS(0);
#ifdef OGBX_PWF_RULE_STAMPS
    if (threadIdx.x == 0 && OGBX_RS_ENV) g_pwf_rule[diag_env * 16 + 15] += 1;
    forward_masked(P, _rs_prev);
#else
    forward_masked(P);
#endif
  }

  // HBM <-> LDS for one env's state (bytes, momentum, velocity)
  __device__ __forceinline__ void load(const uint8_t* __restrict__ a, const int8_t* __restrict__ m,
                       const float2* __restrict__ v) const {
    fence_idx();
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const int i = cell(k);
      s.a[i] = a[i];
      s.m[i] = m[i];
      s.v[i] = v[i];
    }
  }
  __device__ __forceinline__ void store(uint8_t* __restrict__ a, int8_t* __restrict__ m, float2* __restrict__ v) const {
    fence_idx();
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const int i = cell(k);
      a[i] = s.a[i];
      m[i] = s.m[i];
      v[i] = s.v[i];
    }
  }
  // goal ids <- current ids
  __device__ __forceinline__ void keep_goal() const {
    fence_idx();
#pragma unroll
    for (int k = 0; k < CPT; ++k) s.g[cell(k)] = (uint8_t)fid(s.a[cell(k)]);
  }

  // Goal mismatch count against s.g (powderworld_env.py:410-418); block total.
  __device__ __forceinline__ int errors() const {
    fence_idx();
    int err = 0;
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const uint32_t gk = s.g[cell(k)];
      const bool m = gk == fid(s.a[cell(k)]) || gk == fid(s.a[nb(k, 0, -1)]) || gk == fid(s.a[nb(k, 0, 1)]) ||
                     gk == fid(s.a[nb(k, -1, 0)]) || gk == fid(s.a[nb(k, 1, 0)]);
      err += __popcll(__ballot(!m));  // wave-uniform count, no lane shuffles
    }
    if ((threadIdx.x & 63) == 0) s.red_e[threadIdx.x >> 6] = err;
    sync();
    int total = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) total += s.red_e[w];
    sync();
    return total;
  }

  // PWRenderer colour of a cell, blended toward the velocity colour by
  // clip(|v| / 5, 0, 0.5) (sim.py:402-453), as R | G << 8 | B << 16.
  __device__ __forceinline__ uint32_t rgb(uint32_t id, float2 v) const { return pw_rgb(s.lut, id, v); }

  // Observation: RGB of the world + action frame (powderworld_env.py:462-476),
  // staged in LDS (6 bytes per cell as three 16-bit stores) and written as
  // 16-byte stores.  rgb_only: 3 channels.  crg / cb: also write every cell's
  // colour to the env's render cache (R | G << 8, B).
  __device__ __forceinline__ void observe(uint8_t* __restrict__ dst, int stage, uint32_t acol, int rx, int brush,
                                          bool rgb_only = false, uint16_t* __restrict__ crg = nullptr,
                                          uint8_t* __restrict__ cb = nullptr) const {
    fence_idx();
    const bool fr = stage == 1 || (stage == 2 && col >= rx && col < rx + brush);
    const uint32_t px = fr ? acol : 0u;
    sync();  // staging shares LDS with the rule scratch
    uint16_t* st = reinterpret_cast<uint16_t*>(s.ob);
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const int i = cell(k);
      const uint32_t c = rgb(fid(s.a[i]), s.v[i]);
      if (crg != nullptr) {
        crg[i] = (uint16_t)(c & 0xffffu);
        cb[i] = (uint8_t)(c >> 16);
      }
      st[3 * i] = (uint16_t)(c & 0xffffu);
      st[3 * i + 1] = (uint16_t)(((c >> 16) & 0xffu) | ((px & 0xffu) << 8));
      st[3 * i + 2] = (uint16_t)((px >> 8) & 0xffffu);
    }
    sync();
    if (!rgb_only) {
      const uint4* src = reinterpret_cast<const uint4*>(s.ob);
      uint4* d = reinterpret_cast<uint4*>(dst);
      for (int q = threadIdx.x; q < C * 6 / 16; q += NT) pw_nt_store16(&d[q], src[q]);
    } else {
      const uint8_t* src = reinterpret_cast<const uint8_t*>(s.ob);
      for (int q = threadIdx.x; q < C * 3; q += NT) dst[q] = src[(q / 3) * 6 + q % 3];
    }
    sync();  // staging shares LDS with the rule scratch
  }

  // OR over the wave with DPP (every lane active): quad butterflies, then the
  // 8- and 16-lane mirrors leave each 16-lane row's OR in all of its lanes;
  // the four rows are combined from lanes 0, 16, 32, 48.  No LDS round trip
  // (__shfl_xor is a ds_bpermute per step).
  __device__ static __forceinline__ uint32_t wave_or(uint32_t x) {
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x141, 0xF, 0xF, false);  // row_half_mirror
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x140, 0xF, 0xF, false);  // row_mirror
    return (uint32_t)(__builtin_amdgcn_readlane((int)x, 0) | __builtin_amdgcn_readlane((int)x, 16) |
                      __builtin_amdgcn_readlane((int)x, 32) | __builtin_amdgcn_readlane((int)x, 48));
  }

  // Bitmask of the ids present in the world (+ kVelBit if some velocity is
  // nonzero).  A rule whose trigger elements are absent is an identity and is
  // skipped; the mask is then widened by what each executed rule can create.
  __device__ __forceinline__ uint32_t presence() const {
    fence_idx();
    uint32_t m = 0;
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const int i = cell(k);
      const float2 v = s.v[i];
      m |= bit((int)fid(s.a[i])) | ((v.x != 0.0f || v.y != 0.0f) ? kVelBit : 0u);
    }
    m = wave_or(m);
    // red is free: its last readers (the previous forward) are past many barriers
    if ((threadIdx.x & 63) == 0) s.red[threadIdx.x >> 6] = (int32_t)m;
    sync();
    uint32_t all = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) all |= (uint32_t)s.red[w];
    return all;
  }

  // OR of a per-thread mask over the workgroup (own slots red_v; a barrier
  // must separate two calls -- velocity's passes have several between them)
  __device__ __forceinline__ uint32_t block_or(uint32_t m) const {
    m = wave_or(m);
    if ((threadIdx.x & 63) == 0) s.red_v[threadIdx.x >> 6] = (int32_t)m;
    sync();
    uint32_t all = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) all |= (uint32_t)s.red_v[w];
    return all;
  }

  // fluid flow can only move cells if one of these is present (own fluid
  // heavier than a gravity side: water/gas/lava/acid, empty beside gas or
  // fire, the air animals)
  static constexpr uint32_t kFluidTrig =
      bit(kWater) | bit(kGas) | bit(kFire) | bit(kLava) | bit(kAcid) | bit(kKangaroo) | bit(kLemming);
  static constexpr uint32_t kRandUsers = bit(kSand) | bit(kDust) | kFluidTrig | bit(kIce) | bit(kFire) |
                                         bit(kLava) | bit(kPlant) | bit(kWater);

#ifdef OGBX_PWF_RULE_STAMPS
  __device__ __forceinline__ void forward_masked(uint32_t P, unsigned long long _rs_prev) const {
#else
  __device__ __forceinline__ void forward_masked(uint32_t P) const {
#endif
    constexpr uint32_t R = ~0u;  // every rule (bits: 1 stone, 4 sand, 8 fluid, 16 ice, 32 water, 64 fire, 128 plant, 256 velocity)
    if ((R & 1) && (P & bit(kStone))) stone();
    OGBX_RS(1);
    gravity();
    OGBX_RS(2);
    if ((R & 4) && (P & (bit(kSand) | bit(kDust)))) sand();
    OGBX_RS(3);
    if ((R & 8) && (P & kFluidTrig)) {
      fluid();
    } else {
      // no move possible: the new momentum of every fluid cell is 0
#pragma unroll
      for (int k = 0; k < CPT; ++k) {
        const uint32_t id = fid(s.a[cell(k)]);
        if (is_fluid(id) || id == kKangaroo || id == kLemming) s.m[cell(k)] = 0;
      }
      sync();
    }
    OGBX_RS(4);
    if (P & bit(kIce)) {
      if (R & 16) ice();
      P |= bit(kWater);
    }
    OGBX_RS(5);
    if ((R & 32) && (P & bit(kWater)) && (P & bit(kIce))) water();
    OGBX_RS(6);
    if (P & (bit(kFire) | bit(kLava))) {
      if (R & 64) fire();
      P |= bit(kFire) | bit(kWater) | bit(kEmpty) | kVelBit;
    }
    OGBX_RS(7);
    if ((R & 128) && (P & bit(kPlant))) plant();
    OGBX_RS(8);
    if ((R & 256) && (P & kVelBit)) velocity();
    OGBX_RS(9);
  }


  // brush paint of own cells (powderworld_env.py:380-391)
  __device__ __forceinline__ void paint(int elem_id, int rx, int ry, int brush) const {
    fence_idx();
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const int r = row(k), c = col;
      if (r >= ry && r < ry + brush && c >= rx && c < rx + brush && fid(s.a[cell(k)]) != kWall)
        put(cell(k), elem((uint32_t)elem_id));
    }
    sync();
  }
};

}  // namespace ogbx
