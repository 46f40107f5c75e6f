// powder.hip -- batched powderworld envs on gfx950: the 2-D cellular-automaton
// update, brush paint, render and goal-match success check, plus the C-ABI.
//
// Reference (hliuson/ogbench):
//   element table / PWSim.forward   ogbench/powderworld/sim.py:15-37, 284-308, 363-380
//   BehaviorStone / BehaviorGravity sim.py:574-590, 461-501
//   PWRenderer.render               sim.py:386-453
//   PowderworldEnv reset/step/obs   ogbench/powderworld/powderworld_env.py:284-476
//
// Scope: the 'easy' element set (empty, wall, plant, stone; num_elems == 2).
// For those elements the Sand, FluidFlow, Ice, Water, Fire, Plant and Velocity
// rules are identities (no sand/dust/water/gas/fire/ice/wood, velocity 0), so
// a forward pass is Stone then Gravity.  medium/hard are rejected at create.
//
// Layout in HBM: world u8[N, H*W], one byte per cell = element id (bits 0-4)
// | GravityInter (bit 5, channel 2) | DidGravity (bit 6, channel 8); every
// other channel of the reference's (9,H,W) float32 world is 0 or a function of
// the id for easy worlds.  ctrl i32[N] = stage | elem<<2 | x<<8 | task<<16,
// elapsed i32[N], episode u32[N].  Obs u8[N, H, W, 6].
//
// One 256-thread workgroup per env; the world lives in LDS for the whole
// launch (k_steps steps); each thread owns a contiguous run of CPT cells of
// one row (CPT = H*W/256: 16 at 64x64, 4 at 32x32).
#include <array>
#include <cstring>
#include <string>
#include <vector>

#include "common.h"

namespace ogbx {

constexpr int kPwMaxCells = 64 * 64;
constexpr int kPwMaxSeq = 256;
constexpr int kPwMaxTasks = 8;
constexpr uint8_t kIdMask = 31, kGrav = 32, kDidg = 64;

// density (channel 1) and default GravityInter (channel 2) per id: sim.py:15-37
__constant__ uint8_t c_density[21] = {1, 4, 3, 2, 0, 4, 4, 0, 4, 3, 3, 2, 2, 4, 2, 4, 3, 3, 3, 4, 3};
__constant__ uint8_t c_gravity[21] = {1, 0, 1, 1, 1, 0, 0, 1, 0, 1, 1, 1, 1, 0, 1, 0, 1, 1, 1, 0, 1};

struct PowderParams {
  int32_t H, W, grid, brush, xy_size, num_elems, num_tasks, max_steps, tol;
  int32_t elem_ids[8];           // _elems: element id per element index
  uint8_t lut[21][4];            // render colour of each id (uint8(color*255))
  int32_t seq_len[kPwMaxTasks];  // goal replay sequences (elem idx, x, y)
  int8_t seq[kPwMaxTasks][kPwMaxSeq][3];
};

struct PowderState {
  uint8_t* world;
  int32_t* ctrl;
  int32_t* elapsed;
  uint32_t* episode;
};

__device__ inline uint8_t elem_cell(int id) {
  return (uint8_t)(id | (c_gravity[id] ? kGrav : 0));
}

// ---- block-level pieces (all 256 threads of the env's workgroup call them)

// One PWSim.forward for an easy world in LDS (a -> a, scratch b/f).
__device__ void pw_forward(uint8_t* a, uint8_t* b, uint8_t* f, int H, int W, int cpt) {
  const int t = threadIdx.x;
  const int r = (t * cpt) / W, c0 = (t * cpt) % W;
  // BehaviorStone (sim.py:580-590): stone.grav = stone(r-1,c-1)+stone(r-1,c+1) < 2
  for (int k = 0; k < cpt; ++k) {
    const int c = c0 + k;
    uint8_t v = a[r * W + c];
    if ((v & kIdMask) == 9) {
      int sup = 0;
      if (r > 0) {
        if (c > 0 && (a[(r - 1) * W + c - 1] & kIdMask) == 9) ++sup;
        if (c < W - 1 && (a[(r - 1) * W + c + 1] & kIdMask) == 9) ++sup;
      }
      v = (uint8_t)((v & ~kGrav) | (sup < 2 ? kGrav : 0));
    }
    b[r * W + c] = v;
  }
  __syncthreads();
  // BehaviorGravity (sim.py:476-501): did-gravity reset where gravity == 1, then
  // swap with the cell below (periodic roll) when it is lighter and both have
  // gravity; a cell that both sinks and receives keeps its content.
  for (int k = 0; k < cpt; ++k) {
    const int c = c0 + k;
    uint8_t v = b[r * W + c];
    if (v & kGrav) v &= (uint8_t)~kDidg;
    const int rb = r + 1 == H ? 0 : r + 1;
    const uint8_t w = b[rb * W + c];
    const bool dbb = (int)c_density[w & kIdMask] - (int)c_density[v & kIdMask] < 0 && (v & kGrav) &&
                     (w & kGrav);
    b[r * W + c] = v;  // did-gravity reset applied in place (own cell only)
    f[r * W + c] = dbb;
  }
  __syncthreads();
  uint8_t real[64];
  for (int k = 0; k < cpt; ++k) {
    const int c = c0 + k;
    const int ra = r == 0 ? H - 1 : r - 1;
    real[k] = f[r * W + c] && !f[ra * W + c];
  }
  __syncthreads();
  for (int k = 0; k < cpt; ++k) f[r * W + c0 + k] = real[k];
  __syncthreads();
  for (int k = 0; k < cpt; ++k) {
    const int c = c0 + k;
    const int ra = r == 0 ? H - 1 : r - 1, rb = r + 1 == H ? 0 : r + 1;
    auto reset_didg = [](uint8_t v) { return (v & kGrav) ? (uint8_t)(v & ~kDidg) : v; };
    uint8_t v;
    if (f[r * W + c]) {
      v = reset_didg(b[rb * W + c]);
    } else if (f[ra * W + c]) {
      v = (uint8_t)(reset_didg(b[ra * W + c]) | kDidg);
    } else {
      v = b[r * W + c];
    }
    a[r * W + c] = v;
  }
  __syncthreads();
}

// Brush paint (powderworld_env.py:380-391): elem over the brush square unless wall.
__device__ void pw_paint(uint8_t* a, int W, int cpt, int elem_id, int rx, int ry, int brush) {
  const int t = threadIdx.x;
  const int r = (t * cpt) / W, c0 = (t * cpt) % W;
  if (r >= ry && r < ry + brush) {
    for (int k = 0; k < cpt; ++k) {
      const int c = c0 + k;
      if (c >= rx && c < rx + brush && (a[r * W + c] & kIdMask) != 1) a[r * W + c] = elem_cell(elem_id);
    }
  }
  __syncthreads();
}

// Observation (powderworld_env.py:462-476): RGB of the world + action frame.
__device__ void pw_observe(const PowderParams& P, const uint8_t* a, uint8_t* obs, int stage,
                           int elem_id, int x) {
  const int W = P.W, cpt = (P.H * P.W) >> 8;
  const int t = threadIdx.x;
  const int r = (t * cpt) / W, c0 = (t * cpt) % W;
  const int rx = x * P.grid;
  uint8_t buf[16 * 6];
  const int nout = cpt * 6;
  for (int k = 0; k < cpt; ++k) {
    const int c = c0 + k;
    const int id = a[r * W + c] & kIdMask;
    buf[6 * k + 0] = P.lut[id][0];
    buf[6 * k + 1] = P.lut[id][1];
    buf[6 * k + 2] = P.lut[id][2];
    const bool act = stage == 1 || (stage == 2 && c >= rx && c < rx + P.brush);
    buf[6 * k + 3] = act ? P.lut[elem_id][0] : 0;
    buf[6 * k + 4] = act ? P.lut[elem_id][1] : 0;
    buf[6 * k + 5] = act ? P.lut[elem_id][2] : 0;
  }
  uint8_t* dst = obs + (size_t)(t * cpt) * 6;
  if ((nout & 15) == 0) {
    for (int q = 0; q < nout; q += 16) {
      uint4 v;
      memcpy(&v, buf + q, 16);
      *reinterpret_cast<uint4*>(dst + q) = v;
    }
  } else {
    for (int q = 0; q < nout; q += 8) {
      uint2 v;
      memcpy(&v, buf + q, 8);
      *reinterpret_cast<uint2*>(dst + q) = v;
    }
  }
}

// Goal mismatch count (powderworld_env.py:410-418): a goal cell matches if the
// world id equals it at the cell or one of the 4 periodic neighbours.
__device__ int pw_errors(const PowderParams& P, const uint8_t* a, const uint8_t* goal, int* red) {
  const int H = P.H, W = P.W, cpt = (H * W) >> 8;
  const int t = threadIdx.x;
  const int r = (t * cpt) / W, c0 = (t * cpt) % W;
  int err = 0;
  for (int k = 0; k < cpt; ++k) {
    const int c = c0 + k;
    const int g = goal[r * W + c];
    const int cl = c == 0 ? W - 1 : c - 1, cr = c + 1 == W ? 0 : c + 1;
    const int ra = r == 0 ? H - 1 : r - 1, rb = r + 1 == H ? 0 : r + 1;
    const bool m = (a[r * W + c] & kIdMask) == g || (a[r * W + cl] & kIdMask) == g ||
                   (a[r * W + cr] & kIdMask) == g || (a[ra * W + c] & kIdMask) == g ||
                   (a[rb * W + c] & kIdMask) == g;
    err += !m;
  }
  // wave reduction, then one LDS add per wave
  for (int off = 32; off > 0; off >>= 1) err += __shfl_xor(err, off);
  if (threadIdx.x == 0) *red = 0;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) atomicAdd(red, err);
  __syncthreads();
  const int total = *red;
  __syncthreads();
  return total;
}

// Blank world (border walls) + one random semantic action x3 steps
// (powderworld_env.py:307-341): forward is an identity on the blank world.
__device__ void pw_reset_world(const PowderParams& P, uint8_t* a, uint8_t* b, uint8_t* f, int elem,
                               int x, int y) {
  const int H = P.H, W = P.W, cpt = (H * W) >> 8;
  const int t = threadIdx.x;
  const int r = (t * cpt) / W, c0 = (t * cpt) % W;
  for (int k = 0; k < cpt; ++k) {
    const int c = c0 + k;
    const bool border = r == 0 || r == H - 1 || c == 0 || c == W - 1;
    a[r * W + c] = border ? elem_cell(1) : elem_cell(0);
  }
  __syncthreads();
  pw_forward(a, b, f, H, W, cpt);
  pw_paint(a, W, cpt, P.elem_ids[elem], x * P.grid, y * P.grid, P.brush);
}

__device__ inline void load_world(uint8_t* a, const uint8_t* src, int n) {
  for (int q = threadIdx.x * 16; q < n; q += blockDim.x * 16)
    *reinterpret_cast<uint4*>(a + q) = *reinterpret_cast<const uint4*>(src + q);
  __syncthreads();
}

__device__ inline void store_world(uint8_t* dst, const uint8_t* a, int n) {
  for (int q = threadIdx.x * 16; q < n; q += blockDim.x * 16)
    *reinterpret_cast<uint4*>(dst + q) = *reinterpret_cast<const uint4*>(a + q);
}

__device__ inline uint32_t pw_draw(uint64_t env, uint32_t ep, uint32_t slot, uint32_t k0, uint32_t k1,
                                   uint32_t n) {
  u32x4 w = philox4x32_10({(uint32_t)env, ep, slot, (uint32_t)(env >> 32)}, k0, k1);
  return bounded_u32(w.x, n);
}

// ---------------------------------------------------------------- kernels

__global__ void __launch_bounds__(256) pw_goal_kernel(const PowderParams* __restrict__ Pp,
                                                      uint8_t* goals) {
  const PowderParams& P = *Pp;
  __shared__ uint8_t a[kPwMaxCells], b[kPwMaxCells], f[kPwMaxCells];
  const int task = blockIdx.x;
  const int H = P.H, W = P.W, cpt = (H * W) >> 8;
  const int t = threadIdx.x;
  const int r = (t * cpt) / W, c0 = (t * cpt) % W;
  for (int k = 0; k < cpt; ++k) {
    const int c = c0 + k;
    const bool border = r == 0 || r == H - 1 || c == 0 || c == W - 1;
    a[r * W + c] = border ? elem_cell(1) : elem_cell(0);
  }
  __syncthreads();
  for (int s = 0; s < P.seq_len[task]; ++s) {
    pw_forward(a, b, f, H, W, cpt);
    pw_paint(a, W, cpt, P.elem_ids[P.seq[task][s][0]], P.seq[task][s][1] * P.grid,
             P.seq[task][s][2] * P.grid, P.brush);
  }
  for (int k = 0; k < cpt; ++k) goals[(size_t)task * H * W + r * W + c0 + k] = a[r * W + c0 + k] & kIdMask;
}

__global__ void __launch_bounds__(256) pw_reset_kernel(const PowderParams* __restrict__ Pp,
                                                       PowderState S, const uint8_t* goals,
                                                       const int32_t* task_id, const uint8_t* mask,
                                                       const int32_t* reset_action, uint8_t* obs,
                                                       uint8_t* goal_obs, uint32_t k0, uint32_t k1) {
  const PowderParams& P = *Pp;
  __shared__ uint8_t a[kPwMaxCells], b[kPwMaxCells], f[kPwMaxCells];
  const int64_t e = blockIdx.x;
  if (mask != nullptr && mask[e] == 0) return;
  const int HW = P.H * P.W;
  const uint32_t ep = S.episode[e] + 1u;
  int task = task_id ? task_id[e] : 1 + (int)pw_draw(e, ep, 0, k0, k1, (uint32_t)P.num_tasks);
  if (task < 1 || task > P.num_tasks) task = 1;
  int elem, x, y;
  if (reset_action) {
    elem = reset_action[3 * e];
    x = reset_action[3 * e + 1];
    y = reset_action[3 * e + 2];
  } else {
    elem = (int)pw_draw(e, ep, 1, k0, k1, (uint32_t)P.num_elems);
    x = (int)pw_draw(e, ep, 2, k0, k1, (uint32_t)P.xy_size);
    y = (int)pw_draw(e, ep, 3, k0, k1, (uint32_t)P.xy_size);
  }
  pw_reset_world(P, a, b, f, elem, x, y);
  store_world(S.world + (size_t)e * HW, a, HW);
  pw_observe(P, a, obs + (size_t)e * HW * 6, 0, 0, 0);
  // goal observation: render of the goal world (stage 0 -> empty action frame)
  const uint8_t* g = goals + (size_t)(task - 1) * HW;
  for (int q = threadIdx.x; q < HW; q += blockDim.x) b[q] = g[q];
  __syncthreads();
  pw_observe(P, b, goal_obs + (size_t)e * HW * 6, 0, 0, 0);
  if (threadIdx.x == 0) {
    S.ctrl[e] = task << 16;
    S.elapsed[e] = 0;
    S.episode[e] = ep;
  }
}

// k_steps env steps per launch; actions [k, N] int32; draws [k, N] (values of
// np.random.randint for invalid actions) or NULL = Philox.
__global__ void __launch_bounds__(256) pw_step_kernel(
    const PowderParams* __restrict__ Pp, PowderState S, const uint8_t* __restrict__ goals,
    int64_t n, const int32_t* __restrict__ action, const int32_t* __restrict__ draws, int32_t k_steps,
    uint8_t* __restrict__ obs, float* __restrict__ reward, uint8_t* __restrict__ terminated,
    uint8_t* __restrict__ truncated, uint8_t* __restrict__ success, int32_t auto_reset, uint32_t k0,
    uint32_t k1, uint32_t a0, uint32_t a1) {
  const PowderParams& P = *Pp;
  __shared__ uint8_t a[kPwMaxCells], b[kPwMaxCells], f[kPwMaxCells];
  __shared__ int red;
  const int64_t e = blockIdx.x;
  const int HW = P.H * P.W;
  load_world(a, S.world + (size_t)e * HW, HW);
  int ctrl = S.ctrl[e];
  int el = S.elapsed[e];
  uint32_t ep = S.episode[e];
  bool dirty = false;
  for (int k = 0; k < k_steps; ++k) {
    const int64_t o = (int64_t)k * n + e;
    const int act = action[o];
    int stage = ctrl & 3, elem = (ctrl >> 2) & 63, x = (ctrl >> 8) & 255;
    const int task = (ctrl >> 16) & 255;
    auto rnd = [&](uint32_t bound) -> int {
      if (draws) return draws[o];
      return (int)pw_draw(e, ep, (uint32_t)el, a0, a1, bound);
    };
    if (stage == 0) {
      elem = act >= 0 && act < P.num_elems ? act : rnd((uint32_t)P.num_elems);
    } else if (stage == 1) {
      x = act >= 0 && act < P.xy_size ? act : rnd((uint32_t)P.xy_size);
    } else {
      const int y = act >= 0 && act < P.xy_size ? act : rnd((uint32_t)P.xy_size);
      pw_forward(a, b, f, P.H, P.W, HW >> 8);
      pw_paint(a, P.W, HW >> 8, P.elem_ids[elem], x * P.grid, y * P.grid, P.brush);
      dirty = true;
    }
    stage = stage == 2 ? 0 : stage + 1;
    const int errs = pw_errors(P, a, goals + (size_t)(task - 1) * HW, &red);
    const bool succ = errs < P.tol;
    el += 1;
    const bool trunc = el >= P.max_steps;
    uint8_t* ob = obs + (size_t)o * HW * 6;
    if (auto_reset && (succ || trunc)) {
      ep += 1u;
      const int re = (int)pw_draw(e, ep, 1, k0, k1, (uint32_t)P.num_elems);
      const int rx = (int)pw_draw(e, ep, 2, k0, k1, (uint32_t)P.xy_size);
      const int ry = (int)pw_draw(e, ep, 3, k0, k1, (uint32_t)P.xy_size);
      pw_reset_world(P, a, b, f, re, rx, ry);
      stage = 0;
      el = 0;
      dirty = true;
    }
    ctrl = stage | (elem << 2) | (x << 8) | (task << 16);
    pw_observe(P, a, ob, stage, P.elem_ids[elem & 7], x);
    if (threadIdx.x == 0) {
      reward[o] = succ ? 1.0f : 0.0f;
      terminated[o] = succ;
      truncated[o] = trunc;
      success[o] = succ;
    }
  }
  if (dirty) store_world(S.world + (size_t)e * HW, a, HW);
  if (threadIdx.x == 0) {
    S.ctrl[e] = ctrl;
    S.elapsed[e] = el;
    S.episode[e] = ep;
  }
}

// Free-standing PWSim.forward on packed worlds [n, H*W] (tests).
__global__ void __launch_bounds__(256) pw_forward_kernel(const PowderParams* __restrict__ Pp,
                                                         const uint8_t* in, uint8_t* out,
                                                         int32_t steps) {
  const PowderParams& P = *Pp;
  __shared__ uint8_t a[kPwMaxCells], b[kPwMaxCells], f[kPwMaxCells];
  const int HW = P.H * P.W;
  load_world(a, in + (size_t)blockIdx.x * HW, HW);
  for (int s = 0; s < steps; ++s) pw_forward(a, b, f, P.H, P.W, HW >> 8);
  store_world(out + (size_t)blockIdx.x * HW, a, HW);
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

}  // namespace ogbx

struct ogbx_powder_env {
  int32_t device = 0;
  int64_t n = 0;
  ogbx::PowderParams P;
  ogbx::PowderParams* Pd = nullptr;
  ogbx::PowderState S{};
  uint8_t* goals = nullptr;  // [num_tasks, H*W] goal ids
  uint64_t seed = 0;
  bool was_reset = false;
};

using namespace ogbx;

extern "C" {

ogbx_status ogbx_powder_create(const ogbx_powder_opts* opts, int64_t n_envs, int32_t device,
                               ogbx_powder_t* out) {
  OGBX_CHECK(opts && out, OGBX_EINVAL, "ogbx_powder_create: null argument");
  *out = nullptr;
  OGBX_CHECK(n_envs > 0 && n_envs <= (1ll << 31), OGBX_EINVAL, "n_envs out of range");
  const int ws = opts->world_size;
  OGBX_CHECK(ws == 32 || ws == 64, OGBX_EINVAL, "world_size must be 32 or 64");
  OGBX_CHECK(opts->num_elems == 2 || opts->num_elems == 5 || opts->num_elems == 8, OGBX_EINVAL,
             "num_elems must be 2, 5 or 8");
  OGBX_CHECK(opts->num_elems == 2, OGBX_EINVAL,
             "only powderworld-easy (num_elems=2) dynamics are implemented");
  OGBX_CHECK(opts->grid_size == 4 && opts->brush_size == 4, OGBX_EINVAL,
             "only the registered grid_size=4 / brush_size=4 are supported");
  OGBX_CHECK(opts->max_episode_steps > 0, OGBX_EINVAL, "max_episode_steps must be positive");
  ogbx_status st = use_device(device);
  if (st != OGBX_OK) return st;
  auto* e = new ogbx_powder_env();
  e->device = device;
  e->n = n_envs;
  PowderParams& P = e->P;
  std::memset(&P, 0, sizeof(P));
  P.H = P.W = ws;
  P.grid = opts->grid_size;
  P.brush = opts->brush_size;
  P.xy_size = (ws - P.brush) / P.grid + 1;
  P.num_elems = 2;
  P.elem_ids[0] = 8;  // plant
  P.elem_ids[1] = 9;  // stone
  P.max_steps = opts->max_episode_steps;
  P.tol = 32;
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
      P.lut[i][c] = (uint8_t)(v * 255.0f);
    }
  std::vector<std::vector<std::array<int, 3>>> tasks;
  easy_tasks(tasks);
  P.num_tasks = (int)tasks.size();
  for (int t = 0; t < P.num_tasks; ++t) {
    P.seq_len[t] = (int)tasks[t].size();
    for (size_t s = 0; s < tasks[t].size(); ++s)
      for (int k = 0; k < 3; ++k) P.seq[t][s][k] = (int8_t)tasks[t][s][k];
  }
  const size_t n = (size_t)n_envs, HW = (size_t)ws * ws;
  hipError_t h = hipMalloc(&e->Pd, sizeof(PowderParams));
  if (h == hipSuccess) h = hipMemcpy(e->Pd, &P, sizeof(PowderParams), hipMemcpyHostToDevice);
  if (h == hipSuccess) h = hipMalloc(&e->S.world, n * HW);
  if (h == hipSuccess) h = hipMalloc(&e->S.ctrl, n * sizeof(int32_t));
  if (h == hipSuccess) h = hipMalloc(&e->S.elapsed, n * sizeof(int32_t));
  if (h == hipSuccess) h = hipMalloc(&e->S.episode, n * sizeof(uint32_t));
  if (h == hipSuccess) h = hipMalloc(&e->goals, (size_t)P.num_tasks * HW);
  if (h == hipSuccess) h = hipMemset(e->S.world, 0, n * HW);
  if (h == hipSuccess) h = hipMemset(e->S.ctrl, 0, n * sizeof(int32_t));
  if (h == hipSuccess) h = hipMemset(e->S.elapsed, 0, n * sizeof(int32_t));
  if (h == hipSuccess) h = hipMemset(e->S.episode, 0, n * sizeof(uint32_t));
  if (h == hipSuccess) {
    hipLaunchKernelGGL(pw_goal_kernel, dim3(P.num_tasks), dim3(256), 0, 0, e->Pd, e->goals);
    h = hipGetLastError();
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
  (void)hipFree(e->goals);
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
  OGBX_HIP(hipSetDevice(e->device));
  OGBX_HIP(hipMemcpy(out, e->goals, (size_t)e->P.num_tasks * e->P.H * e->P.W,
                     hipMemcpyDeviceToHost));
  return OGBX_OK;
}

ogbx_status ogbx_powder_reset(ogbx_powder_t e, const int32_t* task_id, const uint8_t* mask,
                              const int32_t* reset_action, uint8_t* obs, uint8_t* goal_obs,
                              uint64_t seed, void* stream) {
  OGBX_CHECK(e && obs && goal_obs, OGBX_EINVAL, "ogbx_powder_reset: null argument");
  OGBX_HIP(hipSetDevice(e->device));
  e->seed = seed;
  uint32_t k0, k1;
  seed_key(seed, kTagPowderReset, &k0, &k1);
  hipLaunchKernelGGL(pw_reset_kernel, dim3((uint32_t)e->n), dim3(256), 0, (hipStream_t)stream,
                     e->Pd, e->S, e->goals, task_id, mask, reset_action, obs, goal_obs, k0, k1);
  OGBX_LAUNCHED("pw_reset_kernel");
  e->was_reset = true;
  return OGBX_OK;
}

ogbx_status ogbx_powder_step(ogbx_powder_t e, const int32_t* action, int32_t k_steps,
                             const int32_t* draws, uint8_t* obs, float* reward,
                             uint8_t* terminated, uint8_t* truncated, uint8_t* success,
                             int32_t auto_reset, void* stream) {
  OGBX_CHECK(e && action && obs && reward && terminated && truncated && success, OGBX_EINVAL,
             "ogbx_powder_step: null argument");
  OGBX_CHECK(e->was_reset, OGBX_ESTATE, "Cannot call env.step() before calling env.reset()");
  OGBX_CHECK(k_steps >= 1, OGBX_EINVAL, "k_steps must be >= 1");
  OGBX_HIP(hipSetDevice(e->device));
  uint32_t k0, k1, a0, a1;
  seed_key(e->seed, kTagPowderReset, &k0, &k1);
  seed_key(e->seed, kTagPowderAction, &a0, &a1);
  hipLaunchKernelGGL(pw_step_kernel, dim3((uint32_t)e->n), dim3(256), 0, (hipStream_t)stream,
                     e->Pd, e->S, e->goals, e->n, action, draws, k_steps, obs, reward, terminated,
                     truncated, success, auto_reset, k0, k1, a0, a1);
  OGBX_LAUNCHED("pw_step_kernel");
  return OGBX_OK;
}

ogbx_status ogbx_powder_state(ogbx_powder_t e, uint8_t** world, int32_t** ctrl, int32_t** elapsed) {
  OGBX_CHECK(e, OGBX_EINVAL, "null handle");
  if (world) *world = e->S.world;
  if (ctrl) *ctrl = e->S.ctrl;
  if (elapsed) *elapsed = e->S.elapsed;
  e->was_reset = true;
  return OGBX_OK;
}

ogbx_status ogbx_powder_forward(ogbx_powder_t e, const uint8_t* world_in, int64_t n_worlds,
                                int32_t steps, uint8_t* world_out, void* stream) {
  OGBX_CHECK(e && world_in && world_out && n_worlds >= 0 && steps >= 0, OGBX_EINVAL,
             "ogbx_powder_forward: bad argument");
  if (n_worlds == 0) return OGBX_OK;
  OGBX_HIP(hipSetDevice(e->device));
  hipLaunchKernelGGL(pw_forward_kernel, dim3((uint32_t)n_worlds), dim3(256), 0,
                     (hipStream_t)stream, e->Pd, world_in, world_out, steps);
  OGBX_LAUNCHED("pw_forward_kernel");
  return OGBX_OK;
}

}  // extern "C"
