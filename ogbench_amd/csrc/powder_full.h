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

namespace ogbx {

enum PwElem : int {
  kEmpty = 0, kWall = 1, kSand = 2, kWater = 3, kGas = 4, kWood = 5, kIce = 6, kFire = 7, kPlant = 8,
  kStone = 9, kLava = 10, kAcid = 11, kDust = 12, kFish = 14, kBird = 15, kKangaroo = 16, kMole = 17,
  kLemming = 18
};

template <int WS>
struct alignas(16) PwFullShared {
  static constexpr int C = WS * WS;
  alignas(16) uint8_t a[C];
  alignas(16) int8_t m[C];
  alignas(16) float2 v[C];
  alignas(16) uint8_t f1[C];
  alignas(16) uint8_t f2[C];
  alignas(16) int16_t cnt[C];
  alignas(16) int8_t sw[C];
  alignas(16) uint8_t g[C];              // this env's goal ids
  alignas(16) uint32_t ob[C * 6 / 4];    // observation staging
  uint32_t lut[32];
  int32_t elem_ids[8];
  int32_t red[4];
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

// Rand-field purposes (Philox counter word w): goal replay forward s, the
// reset's forward, the forward of elapsed step el.
constexpr uint32_t kRandGoal = 1u << 24, kRandStart = 2u << 24, kRandStep = 3u << 24;

__device__ __forceinline__ uint32_t fid(uint32_t a) { return a & 31u; }
__device__ __forceinline__ uint32_t fgrav(uint32_t a) { return (a >> 5) & 1u; }
__device__ __forceinline__ uint32_t fdidg(uint32_t a) { return (a >> 6) & 1u; }
__device__ __forceinline__ float fdens(uint32_t a) { return (float)((kDensPacked >> (3u * (a & 31u))) & 7u); }

// Workgroup-level full forward on the LDS state of one world.  Thread t owns
// CPT consecutive cells of one row.  rm/ri/re: this thread's rand values.
template <int WS>
struct FullWorld {
  static constexpr int H = WS, W = WS, C = WS * WS, CPT = C / 256, TPR = W / CPT;
  PwFullShared<WS>& s;
  int r, c0;
  __device__ __forceinline__ explicit FullWorld(PwFullShared<WS>& sh)
      : s(sh), r((int)threadIdx.x / TPR), c0(((int)threadIdx.x % TPR) * CPT) {}

  __device__ __forceinline__ int cell(int k) const { return r * W + c0 + k; }
  // periodic neighbour (np.roll semantics)
  __device__ __forceinline__ int nb(int k, int dr, int dc) const {
    int rr = r + dr, cc = c0 + k + dc;
    rr = rr < 0 ? rr + H : (rr >= H ? rr - H : rr);
    cc = cc < 0 ? cc + W : (cc >= W ? cc - W : cc);
    return rr * W + cc;
  }
  // zero-padded neighbour (conv2d padding=1): -1 outside
  __device__ __forceinline__ int zp(int k, int dr, int dc) const {
    const int rr = r + dr, cc = c0 + k + dc;
    return (rr < 0 || rr >= H || cc < 0 || cc >= W) ? -1 : rr * W + cc;
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
#pragma unroll
    for (int dr = -1; dr <= 1; ++dr)
#pragma unroll
      for (int dc = -1; dc <= 1; ++dc) {
        const int j = zp(k, dr, dc);
        n += (j >= 0 && pred(fid(s.a[j]))) ? 1 : 0;
      }
    return n;
  }

  // ------------------------------------------------------------- rules
  __device__ void stone() const {
    uint8_t na[CPT];
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const int i = cell(k);
      uint32_t a = s.a[i];
      if (fid(a) == kStone) {
        const int jl = zp(k, -1, -1), jr = zp(k, -1, 1);
        const int sup = (jl >= 0 && fid(s.a[jl]) == kStone) + (jr >= 0 && fid(s.a[jr]) == kStone);
        a = (a & ~kGrav) | (sup < 2 ? kGrav : 0u);
      }
      na[k] = (uint8_t)a;
    }
    sync();
#pragma unroll
    for (int k = 0; k < CPT; ++k) s.a[cell(k)] = na[k];
    sync();
  }

  __device__ void gravity() const {
    // did-gravity reset where gravity == 1 (own cells), then the move flags
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const int i = cell(k);
      const uint32_t a = s.a[i];
      if (fgrav(a)) s.a[i] = (uint8_t)(a & ~kDidg);
    }
    sync();
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const uint32_t a = s.a[cell(k)], b = s.a[nb(k, 1, 0)];
      s.f1[cell(k)] = (fdens(b) - fdens(a) < 0.0f) && fgrav(a) && fgrav(b);
    }
    sync();
    Cell nc[CPT];
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const int i = cell(k);
      const bool real = s.f1[i] && !s.f1[nb(k, -1, 0)];
      const bool real_up = s.f1[nb(k, -1, 0)] && !s.f1[nb(k, -2, 0)];
      if (real) {
        nc[k] = get(nb(k, 1, 0));
      } else if (real_up) {
        nc[k] = get(nb(k, -1, 0));
        nc[k].a |= (uint8_t)kDidg;
      } else {
        nc[k] = get(i);
      }
    }
    sync();
#pragma unroll
    for (int k = 0; k < CPT; ++k) put(cell(k), nc[k]);
    sync();
  }

  __device__ void sand(const float* rm) const {
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      const int go = pass == 0 ? -1 : 1;  // fall toward -1 (left) then +1 (right)
#pragma unroll
      for (int k = 0; k < CPT; ++k) s.f2[cell(k)] = pass == 0 ? (rm[k] > 0.5f) : (rm[k] <= 0.5f);
      sync();
      Cell nc[CPT];
#pragma unroll
      for (int k = 0; k < CPT; ++k) {
        const int i = cell(k), ibl = nb(k, 1, go), iar = nb(k, -1, -go);
        const uint32_t a = s.a[i], bl = s.a[ibl], ar = s.a[iar];
        const bool elem = fid(a) == kSand || fid(a) == kDust;
        const bool elem_ar = fid(ar) == kSand || fid(ar) == kDust;
        const bool ndg = !fdidg(a);
        const bool mv = elem && !fdidg(bl) && s.f2[i] && (fdens(a) - fdens(bl) > 0.0f) && fgrav(bl) && ndg;
        const bool in = elem_ar && !fdidg(ar) && s.f2[iar] && (fdens(ar) - fdens(a) > 0.0f) && fgrav(ar) && ndg;
        nc[k] = mv ? get(ibl) : (in ? get(iar) : get(i));
      }
      sync();
#pragma unroll
      for (int k = 0; k < CPT; ++k) put(cell(k), nc[k]);
      sync();
    }
  }

  __device__ static __forceinline__ bool is_fluid(uint32_t id) {
    return id == kEmpty || id == kWater || id == kGas || id == kLava || id == kAcid;
  }

  __device__ void fluid(const float* rm) const {
    float mom[CPT];
#pragma unroll
    for (int k = 0; k < CPT; ++k) mom[k] = 0.0f;
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      const int go = pass == 0 ? -1 : 1;
#pragma unroll
      for (int k = 0; k < CPT; ++k) {
        const int i = cell(k);
        const uint32_t a = s.a[i], sd = s.a[nb(k, 0, go)];
        const bool fall = (rm[k] + (float)s.m[i]) + mom[k] > 0.5f;
        const bool match = pass == 0 ? fall : !fall;
        const bool air = fid(a) == kKangaroo || fid(a) == kLemming;
        const bool elem = is_fluid(fid(a)) || air;
        s.f1[i] = match && elem && (!fdidg(a) || air) && (fdens(a) - fdens(sd) > 0.0f) && fgrav(sd) && fgrav(a);
      }
      sync();
#pragma unroll
      for (int k = 0; k < CPT; ++k) s.f2[cell(k)] = s.f1[cell(k)] && !s.f1[nb(k, 0, -go)];
      sync();
      Cell nc[CPT];
#pragma unroll
      for (int k = 0; k < CPT; ++k) {
        const int i = cell(k);
        const bool real = s.f2[i], real_in = s.f2[nb(k, 0, -go)];
        if (real_in) mom[k] = mom[k] + (pass == 0 ? 2.0f : -2.0f);
        nc[k] = real ? get(nb(k, 0, go)) : (real_in ? get(nb(k, 0, -go)) : get(i));
      }
      sync();
#pragma unroll
      for (int k = 0; k < CPT; ++k) put(cell(k), nc[k]);
      sync();
    }
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const int i = cell(k);
      const uint32_t id = fid(s.a[i]);
      if (is_fluid(id) || id == kKangaroo || id == kLemming) s.m[i] = (int8_t)mom[k];
    }
    sync();
  }

  // element conversions of own cells decided from the current ids
  template <typename Rule>
  __device__ __forceinline__ void convert(Rule rule) const {
    int to[CPT];
#pragma unroll
    for (int k = 0; k < CPT; ++k) to[k] = rule(k);
    sync();
#pragma unroll
    for (int k = 0; k < CPT; ++k)
      if (to[k] >= 0) put(cell(k), elem((uint32_t)to[k]));
    sync();
  }

  __device__ void ice(const float* ri) const {
    convert([&](int k) {
      const uint32_t id = fid(s.a[cell(k)]);
      if (id != kIce || !(ri[k] < 0.02f)) return -1;
      const int n = box(k, [](uint32_t x) { return x == kEmpty || x == kFire || x == kLava || x == kWater; });
      return n > 1 ? (int)kWater : -1;
    });
  }

  __device__ void water(const float* re) const {
    convert([&](int k) {
      const uint32_t id = fid(s.a[cell(k)]);
      if (id != kWater || !(re[k] < 0.05f)) return -1;
      return box(k, [](uint32_t x) { return x == kIce; }) >= 3 ? (int)kIce : -1;
    });
  }

  __device__ static __forceinline__ bool burnable(uint32_t x) {
    return x == kWood || x == kPlant || x == kGas || x == kDust || x == kFish || x == kBird || x == kKangaroo ||
           x == kMole || x == kLemming;
  }

  __device__ void fire(const float* ri, const float* re) const {
    bool fl[CPT];
    int conv_to[CPT];
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const int i = cell(k);
      const uint32_t id = fid(s.a[i]);
      fl[k] = id == kFire || id == kLava;
      const bool near = box(k, [](uint32_t x) { return x == kFire || x == kLava; }) > 0;
      const float p = ri[k];
      const bool burn = ((id == kWood && p < 0.05f) || (id == kPlant && p < 0.2f) || (id == kGas && p < 0.2f) ||
                         id == kDust || (id == kBird && p < 0.05f) ||
                         ((id == kFish || id == kLemming || id == kKangaroo || id == kMole) && p < 0.2f)) &&
                        near;
      const bool burn_ice = id == kIce && p < 0.2f && near;
      s.f1[i] = burn;                   // pushes its 4 neighbours with 8
      s.f2[i] = id == kDust && near;    // and dust with 30
      conv_to[k] = burn ? (int)kFire : (burn_ice ? (int)kWater : -1);
    }
    sync();
    float2 nv[CPT];
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      float2 v = s.v[cell(k)];
      // impulses away from a burning neighbour (sim.py:744-752): left, above, below, right
      v.y = v.y + 8.0f * (float)s.f1[nb(k, 0, -1)];
      v.x = v.x + 8.0f * (float)s.f1[nb(k, -1, 0)];
      v.x = v.x - 8.0f * (float)s.f1[nb(k, 1, 0)];
      v.y = v.y - 8.0f * (float)s.f1[nb(k, 0, 1)];
      v.y = v.y + 30.0f * (float)s.f2[nb(k, 0, -1)];
      v.x = v.x + 30.0f * (float)s.f2[nb(k, -1, 0)];
      v.x = v.x - 30.0f * (float)s.f2[nb(k, 1, 0)];
      v.y = v.y - 30.0f * (float)s.f2[nb(k, 0, 1)];
      nv[k] = v;
    }
    sync();
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      s.v[cell(k)] = nv[k];
      if (conv_to[k] >= 0) put(cell(k), elem((uint32_t)conv_to[k]));
    }
    sync();
    // fire spread from (fire or lava before the burn) x burnable neighbours, and lava
    int nbr[CPT];
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      nbr[k] = box(k, [](uint32_t x) { return burnable(x); });
      s.cnt[cell(k)] = (int16_t)(nbr[k] * (fl[k] ? 1 : 0) + (fid(s.a[cell(k)]) == kLava ? 1 : 0));
    }
    sync();
    int to[CPT];
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      int in_range = 0;
#pragma unroll
      for (int dr = -1; dr <= 1; ++dr)
#pragma unroll
        for (int dc = -1; dc <= 1; ++dc) {
          const int j = zp(k, dr, dc);
          in_range += j >= 0 ? s.cnt[j] : 0;
        }
      const uint32_t id = fid(s.a[cell(k)]);
      const bool burn_empty = id == kEmpty && in_range > 0 && ri[k] < 0.3f;
      const uint32_t id2 = burn_empty ? (uint32_t)kFire : id;
      const bool fade = id2 == kFire && re[k] < 0.4f && nbr[k] == 0;
      to[k] = fade ? (int)kEmpty : (burn_empty ? (int)kFire : -1);
    }
    sync();
#pragma unroll
    for (int k = 0; k < CPT; ++k)
      if (to[k] >= 0) put(cell(k), elem((uint32_t)to[k]));
    sync();
  }

  __device__ void plant(const float* ri) const {
    convert([&](int k) {
      const uint32_t id = fid(s.a[cell(k)]);
      if (id != kWater && id != kEmpty) return -1;
      const int cnt = box(k, [](uint32_t x) { return x == kPlant; });
      const bool grow = id == kWater && ri[k] < 0.05f;
      bool to_plant = grow && cnt <= 3 && cnt >= 1;
      const bool to_empty = grow && cnt > 3;
      if (!to_plant && id == kEmpty && ri[k] < 0.2f && cnt > 0)
        to_plant = box(k, [](uint32_t x) { return x == kIce || x == kWood; }) > 0;
      return to_plant ? (int)kPlant : (to_empty ? (int)kEmpty : -1);
    });
  }

  // direction d (sim.py direction_func) as (dr, dc): 0 right, 1 below-right,
  // 2 below, 3 below-left, 4 left, 5 above-left, 6 above, 7 above-right
  __device__ static __forceinline__ void dir_of(int d, int& dr, int& dc) {
    dr = (int)((0x01A9u >> (2 * d)) & 3u) - 1;  // 2 bits (value + 1) per direction
    dc = (int)((0x901Au >> (2 * d)) & 3u) - 1;
  }

  __device__ void velocity() const {
    const float inv2pi = (float)(1.0 / (2.0 * 3.141592653589793));
#pragma unroll 1
    for (int pass = 0; pass < 2; ++pass) {
      int bin[CPT];
      bool enough[CPT];
#pragma unroll
      for (int k = 0; k < CPT; ++k) {
        const int i = cell(k);
        const float2 v = s.v[i];
        const float mag = sqrtf(v.x * v.x + v.y * v.y);
        const float q = v.y / (mag + 0.001f);
        const float raw = inv2pi * (float)acos((double)q);
        const float ang = v.x < 0.0f ? 1.0f - raw : raw;
        float b = floorf(ang * 8.0f + 0.5f);
        b = b - 8.0f * floorf(b / 8.0f);  // np.remainder(., 8) for b >= 0
        bin[k] = (int)b;
        enough[k] = mag > (pass == 0 ? 1.0f : 2.0f) && fid(s.a[i]) != kWall;
        s.sw[i] = -1;
      }
      sync();
#pragma unroll 1
      for (int d = 0; d < 8; ++d) {
        int dr, dc;
        dir_of(d, dr, dc);
#pragma unroll
        for (int k = 0; k < CPT; ++k) {
          const int i = cell(k), j = nb(k, dr, dc);
          s.f1[i] = bin[k] == d && enough[k] && s.sw[i] == -1 && s.sw[j] == -1 && fid(s.a[j]) == kEmpty;
        }
        sync();
        int8_t nsw[CPT];
#pragma unroll
        for (int k = 0; k < CPT; ++k) {
          const int i = cell(k);
          int8_t w = s.sw[i];
          if (s.f1[i]) w = (int8_t)d;
          if (s.f1[nb(k, -dr, -dc)]) w = (int8_t)((d + 4) & 7);
          nsw[k] = w;
        }
        sync();
#pragma unroll
        for (int k = 0; k < CPT; ++k) s.sw[cell(k)] = nsw[k];
        sync();
      }
      Cell nc[CPT];
#pragma unroll
      for (int k = 0; k < CPT; ++k) {
        const int i = cell(k);
        const int w = s.sw[i];
        int j = i;
        if (w >= 0) {
          int dr, dc;
          dir_of(w, dr, dc);
          j = nb(k, dr, dc);
        }
        nc[k] = get(j);
        const float2 old = s.v[i];
        nc[k].v.x = nc[k].v.x * 0.5f + old.x * 0.5f;
        nc[k].v.y = nc[k].v.y * 0.5f + old.y * 0.5f;
      }
      sync();
#pragma unroll
      for (int k = 0; k < CPT; ++k) put(cell(k), nc[k]);
      sync();
    }
    // decay and 3x3 blur (zero padded), NumPy's einsum summation order
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const int i = cell(k);
      float2 v = s.v[i];
      v.x = v.x * 0.95f;
      v.y = v.y * 0.95f;
      s.v[i] = v;
    }
    sync();
    const float w18 = 1.0f / 18.0f;
    float2 nv[CPT];
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      float tx[9], ty[9];
#pragma unroll
      for (int q = 0; q < 9; ++q) {
        const int j = zp(k, q / 3 - 1, q % 3 - 1);
        const float2 v = j >= 0 ? s.v[j] : make_float2(0.f, 0.f);
        tx[q] = v.x * w18;
        ty[q] = v.y * w18;
      }
      const float2 own = s.v[cell(k)];
      const float bx = (((tx[4] + tx[0]) + tx[8]) + (tx[5] + tx[1])) + ((tx[6] + tx[2]) + (tx[7] + tx[3]));
      const float by = (((ty[4] + ty[0]) + ty[8]) + (ty[5] + ty[1])) + ((ty[6] + ty[2]) + (ty[7] + ty[3]));
      nv[k] = make_float2(bx + own.x * 0.5f, by + own.y * 0.5f);
    }
    sync();
#pragma unroll
    for (int k = 0; k < CPT; ++k) s.v[cell(k)] = nv[k];
    sync();
  }

  // ------------------------------------------------------------- env helpers
  // Blank world: walls on the border, empty inside (powderworld_env.py:309-313).
  __device__ void blank() const {
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const int c = c0 + k;
      const bool border = r == 0 || r == H - 1 || c == 0 || c == W - 1;
      put(cell(k), elem(border ? (uint32_t)kWall : (uint32_t)kEmpty));
    }
    sync();
  }

  // The three rand fields of one forward for this thread's cells: injected
  // (src = [3, H, W] float32) or Philox (one 4x32 draw per cell).
  __device__ void rands(const float* __restrict__ src, uint32_t k0, uint32_t k1, uint64_t env, uint32_t ep,
                        uint32_t slot, float* rm, float* ri, float* re) const {
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const int i = cell(k);
      if (src) {
        rm[k] = src[i];
        ri[k] = src[C + i];
        re[k] = src[2 * C + i];
      } else {
        const u32x4 w = philox4x32_10({(uint32_t)i, (uint32_t)env, ep, slot}, k0 ^ (uint32_t)(env >> 32), k1);
        rm[k] = u01f_from(w.x);
        ri[k] = u01f_from(w.y);
        re[k] = u01f_from(w.z);
      }
    }
  }

  __device__ void forward_rand(const float* __restrict__ src, uint32_t k0, uint32_t k1, uint64_t env, uint32_t ep,
                               uint32_t slot) const {
    float rm[CPT], ri[CPT], re[CPT];
    rands(src, k0, k1, env, ep, slot, rm, ri, re);
    forward(rm, ri, re);
  }

  // HBM <-> LDS for one env's state (bytes, momentum, velocity)
  __device__ void load(const uint8_t* __restrict__ a, const int8_t* __restrict__ m,
                       const float2* __restrict__ v) const {
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const int i = cell(k);
      s.a[i] = a[i];
      s.m[i] = m[i];
      s.v[i] = v[i];
    }
  }
  __device__ void store(uint8_t* __restrict__ a, int8_t* __restrict__ m, float2* __restrict__ v) const {
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const int i = cell(k);
      a[i] = s.a[i];
      m[i] = s.m[i];
      v[i] = s.v[i];
    }
  }
  // goal ids <- current ids
  __device__ void keep_goal() const {
#pragma unroll
    for (int k = 0; k < CPT; ++k) s.g[cell(k)] = (uint8_t)fid(s.a[cell(k)]);
  }

  // Goal mismatch count against s.g (powderworld_env.py:410-418); block total.
  __device__ int errors() const {
    int err = 0;
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const uint32_t gk = s.g[cell(k)];
      const bool m = gk == fid(s.a[cell(k)]) || gk == fid(s.a[nb(k, 0, -1)]) || gk == fid(s.a[nb(k, 0, 1)]) ||
                     gk == fid(s.a[nb(k, -1, 0)]) || gk == fid(s.a[nb(k, 1, 0)]);
      err += m ? 0 : 1;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) err += __shfl_xor(err, off);
    if ((threadIdx.x & 63) == 0) s.red[threadIdx.x >> 6] = err;
    sync();
    const int total = s.red[0] + s.red[1] + s.red[2] + s.red[3];
    sync();
    return total;
  }

  // PWRenderer colour of a cell, blended toward the velocity colour by
  // clip(|v| / 5, 0, 0.5) (sim.py:402-453), as R | G << 8 | B << 16.
  __device__ __forceinline__ uint32_t rgb(uint32_t id, float2 v) const {
    if (v.x == 0.0f && v.y == 0.0f) return s.lut[id];
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

  // Observation: RGB of the world + action frame (powderworld_env.py:462-476),
  // staged in LDS and written as 16-byte stores.  rgb_only: 3 channels.
  __device__ void observe(uint8_t* __restrict__ dst, int stage, uint32_t acol, int rx, int brush,
                          bool rgb_only = false) const {
    constexpr int NWD = CPT * 6 / 4;
    uint32_t words[NWD];
#pragma unroll
    for (int q = 0; q < NWD; ++q) words[q] = 0;
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const int i = cell(k), c = c0 + k;
      const uint32_t col = rgb(fid(s.a[i]), s.v[i]);
      const bool fr = stage == 1 || (stage == 2 && c >= rx && c < rx + brush);
      const uint32_t px = fr ? acol : 0u;
#pragma unroll
      for (int ch = 0; ch < 6; ++ch) {
        const int p = 6 * k + ch;
        const uint32_t b = ch < 3 ? (col >> (8 * ch)) & 0xffu : (px >> (8 * (ch - 3))) & 0xffu;
        words[p >> 2] |= b << (8 * (p & 3));
      }
    }
    sync();  // staging buffer free
    uint32_t* st = s.ob + threadIdx.x * NWD;
#pragma unroll
    for (int q = 0; q < NWD; ++q) st[q] = words[q];
    sync();
    if (!rgb_only) {
      const uint4* src = reinterpret_cast<const uint4*>(s.ob);
      uint4* d = reinterpret_cast<uint4*>(dst);
      for (int q = threadIdx.x; q < C * 6 / 16; q += 256) d[q] = src[q];
    } else {
      const uint8_t* src = reinterpret_cast<const uint8_t*>(s.ob);
      for (int q = threadIdx.x; q < C * 3; q += 256) dst[q] = src[(q / 3) * 6 + q % 3];
    }
  }

  __device__ void forward(const float* rm, const float* ri, const float* re) const {
    stone();
    gravity();
    sand(rm);
    fluid(rm);
    ice(ri);
    water(re);
    fire(ri, re);
    plant(ri);
    velocity();
  }

  // brush paint of own cells (powderworld_env.py:380-391)
  __device__ void paint(int elem_id, int rx, int ry, int brush) const {
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const int c = c0 + k;
      if (r >= ry && r < ry + brush && c >= rx && c < rx + brush && fid(s.a[cell(k)]) != kWall)
        put(cell(k), elem((uint32_t)elem_id));
    }
    sync();
  }
};

}  // namespace ogbx
