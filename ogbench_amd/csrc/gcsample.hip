// gcsample.hip -- offline replay on gfx950: one fused launch draws the sample
// indices, relabels value/actor goals in hindsight and gathers every dataset
// column of the batch from the HBM-resident trajectory buffer.
//
// Reference (hliuson/ogbench):
//   Dataset.get_random_idxs / get_subset   impls/utils/datasets.py:65-83
//   GCDataset.sample                       impls/utils/datasets.py:213-294
//   GCDataset.sample_goals                 impls/utils/datasets.py:296-327
//
// Layout: every column is a dense [R, row_bytes] device array (torch tensor).
// One workgroup handles a tile of TB samples: lanes 0..TB-1 compute the four
// row selectors of their sample into LDS, then all 256 lanes stream the rows
// of every column (widest aligned unit: 16, 8 or 4 bytes) into the batch.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <mutex>
#include <type_traits>

#include "common.h"

namespace ogbx {

constexpr int kGcMaxTile = 64;
constexpr int kGcMaxCols = 32;

template <int N>
struct GcColumnsN {
  ogbx_gc_column c[N];
};
using GcColumns = GcColumnsN<kGcMaxCols>;
// A sampler plan's batches of at most 16 columns (GC 9, HGC 15) launch with
// this half-size table: the host's launch cost grows with the kernel
// arguments (a 1,376-byte argument 2.5 -> 3.4 us per launch on ROCm 7,
// profiles/r06_launch_host.txt), and a steady sample(1024) call is host-bound.
constexpr int kGcSmallCols = 16;
using GcColumnsSmall = GcColumnsN<kGcSmallCols>;

__device__ inline uint64_t bounded64(uint32_t hi, uint32_t lo, uint64_t n) {
  const uint64_t u = ((uint64_t)hi << 32) | lo;
  return __umul64hi(u, n);
}

struct GoalDraws {
  int64_t pick;
  int64_t geom;
  double dist, u_traj, u_cur;
};

// GCDataset.sample_goals for one sample (datasets.py:296-327).
// rand_goal = valid_idxs[d.pick] (or d.pick), loaded by the caller together
// with the sample's other index loads.
__device__ inline int64_t sample_goal(int64_t idx, int64_t final_idx, const GoalDraws& d,
                                      int64_t rand_goal, double p_cur, double thresh, int geom,
                                      int cur_is_one) {
  if (cur_is_one) return idx;
  int64_t traj;
  if (geom) {
    const int64_t s = idx + d.geom;
    traj = s < final_idx ? s : final_idx;
  } else {
    const int64_t lo = idx + 1 < final_idx ? idx + 1 : final_idx;
    traj = (int64_t)rint((double)lo * d.dist + (double)final_idx * (1.0 - d.dist));
  }
  int64_t goal = d.u_traj < thresh ? traj : rand_goal;
  goal = d.u_cur < p_cur ? idx : goal;
  return goal;
}

// The sample's dependent index loads, issued back to back so that they share
// one HBM round trip: idx = valid_idxs[pick], its trajectory end, and the
// random goals valid_idxs[goal pick] (datasets.py:65-70, 307-309).  Every
// condition is wave-uniform (pointer presence), so no load address waits on
// another load; for explicit idxs (pick < 0) the end needs idx first.
// Periodic buffer (ogbx_gc_buffer.period > 0): pick p lies in period
// q = p / period_picks at offset r, so idx = q period + r and its trajectory
// end is q period + period_end -- no index load at all.  The IEEE quotient is
// off by at most one near an integer; the remainder test corrects it.
__device__ inline int64_t periodic_row(const ogbx_gc_buffer& buf, int64_t pick, int64_t* q_out) {
  // the quotient estimate by the reciprocal (a function of the kernel
  // arguments alone, so it is computed off the sample's chain): within one of
  // floor(pick / period_picks) like the IEEE quotient, and the remainder test
  // below makes q exact either way
  const double inv_pp = 1.0 / (double)buf.period_picks;
  int64_t q = (int64_t)((double)pick * inv_pp);
  int64_t r = pick - q * buf.period_picks;
  if (r < 0) {
    --q;
    r += buf.period_picks;
  } else if (r >= buf.period_picks) {
    ++q;
    r -= buf.period_picks;
  }
  *q_out = q;
  return q * buf.period + r;
}

__device__ inline void index_loads(const ogbx_gc_buffer& buf, bool explicit_idxs, int64_t pick,
                                   int64_t* idx, int64_t* fin) {
  const int64_t* __restrict__ vi = buf.valid_idxs;
  if (!explicit_idxs && buf.period > 0) {
    int64_t q;
    *idx = periodic_row(buf, pick, &q);
    *fin = q * buf.period + buf.period_end;
  } else if (explicit_idxs) {
    *fin = buf.traj_end[*idx];
  } else if (buf.valid_pairs) {
    const longlong2 p = reinterpret_cast<const longlong2*>(buf.valid_pairs)[pick];
    *idx = p.x;
    *fin = p.y;
  } else if (vi && buf.valid_traj_end) {
    *idx = vi[pick];
    *fin = buf.valid_traj_end[pick];
  } else if (vi) {
    *idx = vi[pick];
    *fin = buf.traj_end[*idx];
  } else {
    *idx = pick;
    *fin = buf.traj_end[pick];
  }
}

__device__ inline int64_t rand_goal_of(const ogbx_gc_buffer& buf, int64_t pick) {
  if (buf.period > 0) {
    int64_t q;
    return periodic_row(buf, pick, &q);
  }
  if (buf.valid_pairs) return buf.valid_pairs[2 * pick];
  return buf.valid_idxs ? buf.valid_idxs[pick] : pick;
}

// Source row pitch of a column in units of T (src_stride 0 = dense rows).
template <typename T>
__device__ __forceinline__ int64_t src_pitch(const ogbx_gc_column& col) {
  return (col.src_stride ? (int64_t)col.src_stride : col.row_bytes) / (int64_t)sizeof(T);
}

__device__ inline int64_t geometric_from(double u, double log_q) {
  // legacy RandomState.geometric inversion: ceil(log(1-u) / log(1-p))
  double g = ceil(log(1.0 - u) / log_q);
  return g < 1.0 ? 1 : (int64_t)g;
}

// Threads [t0, blockDim.x) copy (t0 = 64: the first wave is busy elsewhere).
template <typename T>
__device__ inline void copy_rows(const ogbx_gc_column& col, const int64_t* sel, int64_t base,
                                 int tile, int t0) {
  const int64_t units = col.row_bytes / (int64_t)sizeof(T);
  const int64_t pitch = src_pitch<T>(col);
  const T* __restrict__ src = (const T*)col.src;
  T* __restrict__ dst = (T*)col.dst;
  const int64_t total = units * tile;
  const int step = blockDim.x - t0, tid = threadIdx.x - t0;
  int64_t b = tid / units, k = tid % units;
  const int64_t sb = step / units, sk = step % units;
  for (int64_t f = tid; f < total; f += step) {
    dst[(base + b) * units + k] = src[sel[b] * pitch + k];
    k += sk;
    b += sb;
    if (k >= units) {
      k -= units;
      b += 1;
    }
  }
}

// Copy every column row of a tile.  For small tiles (latency-bound launches)
// whose columns are all 4-byte granular with rows of <= 128 words, each
// (column, sample) row is one job for one wave: the job's column descriptor
// and row index are wave-uniform (scalar loads, one LDS broadcast), lanes
// cover the row's words, and each wave issues the loads of up to kJ jobs
// before any store, so all column rows of the tile share one HBM round trip.
// Otherwise each column is copied with its widest aligned unit.
// Waves [wave0, blockDim.x / 64) copy (wave0 = 1: the first wave computes the
// next call's selectors meanwhile, gc_ahead_kernel).
// kNt: non-temporal stores on the small-tile path (the HGC hit kernel: its 3.6
// MB of rows per launch leave less to the end-of-kernel write-back, 6.44 ->
// 6.34 us; GC's 1.3 MB measured 4.34 -> 4.38 us and keeps plain stores)
template <int kSel, bool kNt = false, class Cols = GcColumns>
__device__ inline void copy_tile(const Cols& cols, int num_cols, const int64_t (*sel)[kGcMaxTile], int64_t base,
                                 int n_here, bool flat4, int wave0 = 0) {
  if ((int)(threadIdx.x >> 6) < wave0) return;
  if (flat4) {
    constexpr int kJ = 8, kSlots = 2;
    const int nw = (int)(blockDim.x >> 6) - wave0;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) - wave0;
    const int lane = (int)(threadIdx.x & 63);
    const int jobs = num_cols * n_here;
    for (int j0 = wave; j0 < jobs; j0 += nw * kJ) {
      uint32_t v[kJ][kSlots];
      uint32_t* d[kJ][kSlots];
#pragma unroll
      for (int u = 0; u < kJ; ++u) {
        const int j = j0 + u * nw;
#pragma unroll
        for (int q = 0; q < kSlots; ++q) d[u][q] = nullptr;
        if (j < jobs) {
          const int c = j / n_here, b = j - c * n_here;
          const ogbx_gc_column& col = cols.c[c];
          const int units = (int)(col.row_bytes >> 2);
          const uint32_t* src = (const uint32_t*)col.src + sel[col.select][b] * src_pitch<uint32_t>(col);
          uint32_t* dst = (uint32_t*)col.dst + (base + b) * units;
#pragma unroll
          for (int q = 0; q < kSlots; ++q) {
            const int k = lane + 64 * q;
            if (k < units) {
              v[u][q] = src[k];
              d[u][q] = dst + k;
            }
          }
        }
      }
#pragma unroll
      for (int u = 0; u < kJ; ++u)
#pragma unroll
        for (int q = 0; q < kSlots; ++q)
          if (d[u][q]) {
            if constexpr (kNt)
              __builtin_nontemporal_store(v[u][q], d[u][q]);
            else
              *d[u][q] = v[u][q];
          }
    }
    return;
  }
  for (int c = 0; c < num_cols; ++c) {
    const ogbx_gc_column& col = cols.c[c];
    const int64_t* srow = sel[col.select];
    const uintptr_t align = (uintptr_t)col.src | (uintptr_t)col.dst | (uintptr_t)col.src_stride;
    const int t0 = 64 * wave0;
    if (col.row_bytes % 16 == 0 && align % 16 == 0)
      copy_rows<uint4>(col, srow, base, n_here, t0);
    else if (col.row_bytes % 8 == 0 && align % 8 == 0)
      copy_rows<uint2>(col, srow, base, n_here, t0);
    else if (col.row_bytes % 4 == 0 && align % 4 == 0)
      copy_rows<uint32_t>(col, srow, base, n_here, t0);
    else
      copy_rows<uint8_t>(col, srow, base, n_here, t0);
  }
}

// The tile's Philox words, one call per lane: sample b of the tile, call q
// (q < calls) -> wb[q][b].  A B = 1024 launch has two samples per workgroup,
// so in-lane calls would run kCalls dependent-free chains on two lanes; spread
// over 2 * kCalls lanes each lane runs one.  Same counters and keys as the
// in-lane form, so the words are identical.
constexpr bool kGcSpread = true;
// Every lane of a wave that has a call computes one (lanes past the last call
// repeat one and store nothing): gfx950 issues a dependent integer chain about
// twice as slowly with <= 16 active lanes, and a B = 1,024 tile
// has 5-7 calls.
__device__ inline void tile_philox(uint4 (*wb)[kGcMaxTile], int calls, int n_here, int64_t base,
                                   uint32_t call_lo, uint32_t call_hi, uint32_t k0, uint32_t k1) {
  const int tot = calls * n_here, span = (tot + 63) & ~63;
  for (int t = threadIdx.x; t < span; t += blockDim.x) {
    const int tt = t < tot ? t : t % tot;
    const int b = tt / calls, q = tt - b * calls;
    const uint64_t su = (uint64_t)(base + b);
    const u32x4 w = philox4x32_10({(uint32_t)su, call_lo, (uint32_t)q, (uint32_t)(su >> 32) ^ call_hi}, k0, k1);
    if (t < tot) wb[q][b] = make_uint4(w.x, w.y, w.z, w.w);
  }
}
// Tile of this workgroup: consecutive workgroup ids go round-robin to the 8
// XCDs, each with its own L2, so tiles are numbered XCD-major -- the
// workgroups of one XCD own a contiguous run of samples and the partial
// 128-B lines where one sample's output rows meet the next are merged in
// that XCD's L2 instead of being written back twice.
__device__ inline int64_t xcd_tile() {
  const int64_t b = blockIdx.x, nb = gridDim.x;
  const int64_t per = nb >> 3, rem = nb & 7, x = b & 7;
  return x * per + (x < rem ? x : rem) + (b >> 3);
}

__device__ inline u32x4 tile_word(const uint4 (*wb)[kGcMaxTile], int q, int b) {
  const uint4 v = wb[q][b];
  return u32x4{v.x, v.y, v.z, v.w};
}

template <bool kInj>
__global__ void __launch_bounds__(256) gc_sample_kernel(
    ogbx_gc_buffer buf, ogbx_gc_config cfg, GcColumns cols, int32_t num_cols, int64_t total,
    int tile, ogbx_gc_draws dr, uint32_t k0, uint32_t k1, uint32_t call_lo, uint32_t call_hi,
    double v_log_q, double a_log_q, int64_t* idxs_out, int64_t* vgoal_out, int64_t* agoal_out,
    double* masks, double* rewards, ogbx_gc_draw_record rec, bool flat4) {
  __shared__ int64_t sel[4][kGcMaxTile];
  __shared__ uint4 wb[(!kInj && kGcSpread) ? 5 : 1][kGcMaxTile];
  const int64_t base = xcd_tile() * tile;
  int n_here = (int)((total - base) < tile ? (total - base) : tile);
  if (!kInj && kGcSpread) {
    tile_philox(wb, 5, n_here, base, call_lo, call_hi, k0, k1);
    __syncthreads();
  }
  // The whole first wave runs the sample chains (lane b % n_here; only lanes
  // b < n_here store): a chain on a few active lanes issues about twice as
  // slowly on gfx950, and a B = 1,024 tile has one sample.
  if (threadIdx.x < 64 && n_here > 0) {
    const int b = (int)threadIdx.x % n_here;
    const bool own = (int)threadIdx.x < n_here;
    const int64_t s = base + b;
    const uint64_t su = (uint64_t)s;
    const uint32_t c0 = (uint32_t)su, c3 = (uint32_t)(su >> 32) ^ call_hi;
    u32x4 w0, w1, w2, w3, w4;
    if (!kInj && kGcSpread) {
      w0 = tile_word(wb, 0, b), w1 = tile_word(wb, 1, b), w2 = tile_word(wb, 2, b), w3 = tile_word(wb, 3, b),
      w4 = tile_word(wb, 4, b);
    } else {
      w0 = philox4x32_10({c0, call_lo, 0u, c3}, k0, k1);
      w1 = philox4x32_10({c0, call_lo, 1u, c3}, k0, k1);
      w2 = philox4x32_10({c0, call_lo, 2u, c3}, k0, k1);
      w3 = philox4x32_10({c0, call_lo, 3u, c3}, k0, k1);
      w4 = philox4x32_10({c0, call_lo, 4u, c3}, k0, k1);
    }
    const int64_t npick = buf.valid_idxs ? buf.num_valid : buf.num_rows;
    // sample index (datasets.py:65-70)
    int64_t idx = 0, pick = -1, final_idx;
    if (kInj && dr.idxs) idx = dr.idxs[s];
    else pick = (kInj && dr.pick) ? dr.pick[s] : (int64_t)bounded64(w0.x, w0.y, (uint64_t)npick);
    GoalDraws v, a;
    v.pick = (kInj && dr.v_pick) ? dr.v_pick[s] : (int64_t)bounded64(w0.z, w0.w, (uint64_t)npick);
    a.pick = (kInj && dr.a_pick) ? dr.a_pick[s] : (int64_t)bounded64(w1.x, w1.y, (uint64_t)npick);
    index_loads(buf, kInj && dr.idxs != nullptr, pick, &idx, &final_idx);
    const int64_t v_rand = cfg.value_cur_is_one ? 0 : rand_goal_of(buf, v.pick);
    const int64_t a_rand = cfg.actor_cur_is_one ? 0 : rand_goal_of(buf, a.pick);
    const int64_t next = idx + 1 < buf.num_rows ? idx + 1 : buf.num_rows - 1;
    const double uvg = u01_from(w1.z, w1.w), uag = u01_from(w2.x, w2.y);
    v.geom = (kInj && dr.v_geom) ? dr.v_geom[s] : (cfg.value_geom_sample ? geometric_from(uvg, v_log_q) : 0);
    a.geom = (kInj && dr.a_geom) ? dr.a_geom[s] : (cfg.actor_geom_sample ? geometric_from(uag, a_log_q) : 0);
    v.dist = (kInj && dr.v_dist) ? dr.v_dist[s] : uvg;
    a.dist = (kInj && dr.a_dist) ? dr.a_dist[s] : uag;
    v.u_traj = (kInj && dr.v_u_traj) ? dr.v_u_traj[s] : u01_from(w2.z, w2.w);
    v.u_cur = (kInj && dr.v_u_cur) ? dr.v_u_cur[s] : u01_from(w3.x, w3.y);
    a.u_traj = (kInj && dr.a_u_traj) ? dr.a_u_traj[s] : u01_from(w3.z, w3.w);
    a.u_cur = (kInj && dr.a_u_cur) ? dr.a_u_cur[s] : u01_from(w4.x, w4.y);
    const int64_t vg = sample_goal(idx, final_idx, v, v_rand, cfg.value_p_curgoal,
                                   cfg.value_traj_thresh, cfg.value_geom_sample, cfg.value_cur_is_one);
    const int64_t ag = sample_goal(idx, final_idx, a, a_rand, cfg.actor_p_curgoal,
                                   cfg.actor_traj_thresh, cfg.actor_geom_sample, cfg.actor_cur_is_one);
    if (own) {
    sel[0][b] = idx;
    sel[1][b] = next;
    sel[2][b] = vg;
    sel[3][b] = ag;
    if (idxs_out) idxs_out[s] = idx;
    if (vgoal_out) vgoal_out[s] = vg;
    if (agoal_out) agoal_out[s] = ag;
    const double succ = idx == vg ? 1.0 : 0.0;
    masks[s] = 1.0 - succ;
    rewards[s] = succ - (cfg.gc_negative ? 1.0 : 0.0);
    if (rec.pick) {
      rec.pick[s] = pick;
      rec.v_pick[s] = v.pick;
      rec.v_geom[s] = v.geom;
      rec.v_dist[s] = v.dist;
      rec.v_u_traj[s] = v.u_traj;
      rec.v_u_cur[s] = v.u_cur;
      rec.a_pick[s] = a.pick;
      rec.a_geom[s] = a.geom;
      rec.a_dist[s] = a.dist;
      rec.a_u_traj[s] = a.u_traj;
      rec.a_u_cur[s] = a.u_cur;
    }
    }  // own
  }
  __syncthreads();
  copy_tile<0>(cols, num_cols, sel, base, n_here, flat4);
}

// ---------------------------------------------------------------- look-ahead
// One sample's selectors and scalars, as GCDataset.sample draws them with the
// Philox words w0..w4 (the same arithmetic as gc_sample_kernel's Philox path).
struct GcPick {
  int64_t idx, next, vg, ag;
  double mask, reward;
};

__device__ inline GcPick gc_chain(const ogbx_gc_buffer& buf, const ogbx_gc_config& cfg, const u32x4& w0,
                                  const u32x4& w1, const u32x4& w2, const u32x4& w3, const u32x4& w4,
                                  double v_log_q, double a_log_q) {
  const int64_t npick = buf.valid_idxs ? buf.num_valid : buf.num_rows;
  const int64_t pick = (int64_t)bounded64(w0.x, w0.y, (uint64_t)npick);
  GoalDraws v, a;
  v.pick = (int64_t)bounded64(w0.z, w0.w, (uint64_t)npick);
  a.pick = (int64_t)bounded64(w1.x, w1.y, (uint64_t)npick);
  int64_t idx = 0, final_idx;
  index_loads(buf, false, pick, &idx, &final_idx);
  const int64_t v_rand = cfg.value_cur_is_one ? 0 : rand_goal_of(buf, v.pick);
  const int64_t a_rand = cfg.actor_cur_is_one ? 0 : rand_goal_of(buf, a.pick);
  const double uvg = u01_from(w1.z, w1.w), uag = u01_from(w2.x, w2.y);
  v.geom = cfg.value_geom_sample ? geometric_from(uvg, v_log_q) : 0;
  a.geom = cfg.actor_geom_sample ? geometric_from(uag, a_log_q) : 0;
  v.dist = uvg;
  a.dist = uag;
  v.u_traj = u01_from(w2.z, w2.w);
  v.u_cur = u01_from(w3.x, w3.y);
  a.u_traj = u01_from(w3.z, w3.w);
  a.u_cur = u01_from(w4.x, w4.y);
  GcPick p;
  p.idx = idx;
  p.next = idx + 1 < buf.num_rows ? idx + 1 : buf.num_rows - 1;
  p.vg = sample_goal(idx, final_idx, v, v_rand, cfg.value_p_curgoal, cfg.value_traj_thresh, cfg.value_geom_sample,
                     cfg.value_cur_is_one);
  p.ag = sample_goal(idx, final_idx, a, a_rand, cfg.actor_p_curgoal, cfg.actor_traj_thresh, cfg.actor_geom_sample,
                     cfg.actor_cur_is_one);
  const double succ = idx == p.vg ? 1.0 : 0.0;
  p.mask = 1.0 - succ;
  p.reward = succ - (cfg.gc_negative ? 1.0 : 0.0);
  return p;
}

// The first wave's chain of sample s under call (lo, hi): lanes 0..4 each run
// one Philox call, every lane then runs the chain on the broadcast words (a
// chain on one active lane issues about twice as slowly).
__device__ inline GcPick gc_wave_chain(const ogbx_gc_buffer& buf, const ogbx_gc_config& cfg, int64_t s, uint32_t lo,
                                       uint32_t hi, uint32_t k0, uint32_t k1, double v_log_q, double a_log_q) {
  const uint64_t su = (uint64_t)s;
  const uint32_t q = (uint32_t)(threadIdx.x & 63) % 5u;
  const u32x4 w = philox4x32_10({(uint32_t)su, lo, q, (uint32_t)(su >> 32) ^ hi}, k0, k1);
  u32x4 ws[5];
#pragma unroll
  for (int c = 0; c < 5; ++c)
    ws[c] = u32x4{(uint32_t)__builtin_amdgcn_readlane((int)w.x, c), (uint32_t)__builtin_amdgcn_readlane((int)w.y, c),
                  (uint32_t)__builtin_amdgcn_readlane((int)w.z, c), (uint32_t)__builtin_amdgcn_readlane((int)w.w, c)};
  return gc_chain(buf, cfg, ws[0], ws[1], ws[2], ws[3], ws[4], v_log_q, a_log_q);
}

// GCDataset.sample with look-ahead (one sample per workgroup, Philox draws):
// the selectors of this call come from ahead_in (stored by the previous
// call's launch; NULL: computed here first), and while waves 1..3 gather the
// rows, the first wave computes the NEXT call's selectors (call next_lo/hi)
// into ahead_out.  The draw chain of a call is thereby off its own critical
// path.  Words per sample (kGcAheadWords): idx, next, value goal, actor goal,
// mask, reward.  kHit (ahead_in valid) and the miss form (ahead_in ignored)
// are separate kernels: one kernel holding both paths spilled kernel
// arguments to VGPR lanes in a preamble every wave ran (HGC: 60 SGPR
// spills), and the hit path then measured 8.3 us against 6.4 us alone.
constexpr int kGcAheadWords = OGBX_GC_AHEAD_WORDS;
constexpr int64_t kGcAheadMaxSamples = 1024;

template <bool kHit, class Cols = GcColumns>
__global__ void __launch_bounds__(256) gc_ahead_kernel(
    ogbx_gc_buffer buf, ogbx_gc_config cfg, Cols cols, int32_t num_cols, uint32_t k0, uint32_t k1,
    uint32_t call_lo, uint32_t call_hi, uint32_t next_lo, uint32_t next_hi, double v_log_q, double a_log_q,
    const int64_t* __restrict__ ahead_in, int64_t* __restrict__ ahead_out, int64_t* idxs_out, int64_t* vgoal_out,
    int64_t* agoal_out, double* masks, double* rewards, bool flat4) {
  __shared__ int64_t sel[4][kGcMaxTile];
  const int64_t s = xcd_tile();
  const int t = (int)threadIdx.x;
  auto publish = [&](const GcPick& p) {
    sel[0][0] = p.idx;
    sel[1][0] = p.next;
    sel[2][0] = p.vg;
    sel[3][0] = p.ag;
    if (idxs_out) idxs_out[s] = p.idx;
    if (vgoal_out) vgoal_out[s] = p.vg;
    if (agoal_out) agoal_out[s] = p.ag;
    masks[s] = p.mask;
    rewards[s] = p.reward;
  };
  if constexpr (kHit) {
    // Hit: no block barrier.  The first wave runs the next call's chain from
    // the kernel's first instruction and writes this call's scalar outputs
    // from the record after it (a gathering wave that stored them would wait
    // for their write acknowledgements at its first row use: vmcnt counts
    // stores); each gathering wave reads the record's selectors into its own
    // LDS column (sel[.][wave]: written and read by the same wave, whose LDS
    // operations complete in order), so the gather waits for one record load
    // and never for the chain.
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6), lane = t & 63;
    if (wave == 0) {
      const int64_t v = lane < 6 ? ahead_in[s * kGcAheadWords + lane] : 0;
      if (ahead_out) {
        const GcPick p = gc_wave_chain(buf, cfg, s, next_lo, next_hi, k0, k1, v_log_q, a_log_q);
        if (t == 0) {
          longlong2* o = reinterpret_cast<longlong2*>(ahead_out + s * kGcAheadWords);
          o[0] = make_longlong2(p.idx, p.next);
          o[1] = make_longlong2(p.vg, p.ag);
          o[2] = make_longlong2(__double_as_longlong(p.mask), __double_as_longlong(p.reward));
        }
      }
      if (lane == 0 && idxs_out) idxs_out[s] = v;
      if (lane == 2 && vgoal_out) vgoal_out[s] = v;
      if (lane == 3 && agoal_out) agoal_out[s] = v;
      if (lane == 4) masks[s] = __longlong_as_double(v);
      if (lane == 5) rewards[s] = __longlong_as_double(v);
      return;
    }
    if (lane < 4) sel[lane][wave] = ahead_in[s * kGcAheadWords + lane];
    __builtin_amdgcn_wave_barrier();
    copy_tile<0>(cols, num_cols, reinterpret_cast<const int64_t(*)[kGcMaxTile]>(&sel[0][wave]), s, 1, flat4, 1);
    return;
  }
  if (t < 64) {
    const GcPick p = gc_wave_chain(buf, cfg, s, call_lo, call_hi, k0, k1, v_log_q, a_log_q);
    if (t == 0) publish(p);
  }
  __syncthreads();
  if (ahead_out && t < 64) {
    const GcPick p = gc_wave_chain(buf, cfg, s, next_lo, next_hi, k0, k1, v_log_q, a_log_q);
    if (t == 0) {
      longlong2* o = reinterpret_cast<longlong2*>(ahead_out + s * kGcAheadWords);
      o[0] = make_longlong2(p.idx, p.next);
      o[1] = make_longlong2(p.vg, p.ag);
      o[2] = make_longlong2(__double_as_longlong(p.mask), __double_as_longlong(p.reward));
    }
  } else {
    copy_tile<0>(cols, num_cols, sel, s, 1, flat4, ahead_out ? 1 : 0);
  }
}

// HGCDataset.compute_high_next_idxs (datasets.py:478-491) for one sample.
__device__ inline void high_next(int64_t idx, int64_t fin, int64_t goal, int64_t K, int64_t* next,
                                 int64_t* steps) {
  int64_t st = K < fin - idx ? K : fin - idx;
  const int64_t diff = goal - idx;
  if (0 <= diff && diff < st) st = diff;
  *steps = st;
  *next = idx + st;
}

constexpr int kHgcSel = 10;

// HGCDataset.sample (datasets.py:496-643): same tile structure as
// gc_sample_kernel with ten row selectors and the hierarchical scalars.
template <bool kInj>
__global__ void __launch_bounds__(256) hgc_sample_kernel(
    ogbx_gc_buffer buf, ogbx_gc_config cfg, ogbx_hgc_config hc, GcColumns cols, int32_t num_cols,
    int64_t total, int tile, ogbx_hgc_draws dr, uint32_t k0, uint32_t k1, uint32_t call_lo,
    uint32_t call_hi, double v_log_q, double a_log_q, double l_log_q, ogbx_hgc_outputs o,
    ogbx_hgc_draw_record rec, bool flat4) {
  __shared__ int64_t sel[kHgcSel][kGcMaxTile];
  __shared__ uint4 wb[(!kInj && kGcSpread) ? 7 : 1][kGcMaxTile];
  const int64_t base = xcd_tile() * tile;
  const int n_here = (int)((total - base) < tile ? (total - base) : tile);
  if (!kInj && kGcSpread) {
    tile_philox(wb, hc.has_low_value_goals ? 7 : 5, n_here, base, call_lo, call_hi, k0, k1);
    __syncthreads();
  }
  if (threadIdx.x < 64 && n_here > 0) {  // the whole first wave: see gc_sample_kernel
    const int b = (int)threadIdx.x % n_here;
    const bool own = (int)threadIdx.x < n_here;
    const int64_t s = base + b;
    const uint64_t su = (uint64_t)s;
    const uint32_t c0 = (uint32_t)su, c3 = (uint32_t)(su >> 32) ^ call_hi;
    u32x4 w0, w1, w2, w3, w4;
    if (!kInj && kGcSpread) {
      w0 = tile_word(wb, 0, b), w1 = tile_word(wb, 1, b), w2 = tile_word(wb, 2, b), w3 = tile_word(wb, 3, b),
      w4 = tile_word(wb, 4, b);
    } else {
      w0 = philox4x32_10({c0, call_lo, 0u, c3}, k0, k1);
      w1 = philox4x32_10({c0, call_lo, 1u, c3}, k0, k1);
      w2 = philox4x32_10({c0, call_lo, 2u, c3}, k0, k1);
      w3 = philox4x32_10({c0, call_lo, 3u, c3}, k0, k1);
      w4 = philox4x32_10({c0, call_lo, 4u, c3}, k0, k1);
    }
    const int64_t npick = buf.valid_idxs ? buf.num_valid : buf.num_rows;
    const ogbx_gc_draws& g = dr.gc;
    int64_t idx = 0, pick = -1, fin;
    if (kInj && g.idxs) idx = g.idxs[s];
    else pick = (kInj && g.pick) ? g.pick[s] : (int64_t)bounded64(w0.x, w0.y, (uint64_t)npick);
    GoalDraws v, a, l;
    v.pick = (kInj && g.v_pick) ? g.v_pick[s] : (int64_t)bounded64(w0.z, w0.w, (uint64_t)npick);
    a.pick = (kInj && g.a_pick) ? g.a_pick[s] : (int64_t)bounded64(w1.x, w1.y, (uint64_t)npick);
    u32x4 w5{}, w6{};
    int64_t l_rand = 0;
    if (hc.has_low_value_goals) {
      if (!kInj && kGcSpread) {
        w5 = tile_word(wb, 5, b);
        w6 = tile_word(wb, 6, b);
      } else {
        w5 = philox4x32_10({c0, call_lo, 5u, c3}, k0, k1);
        w6 = philox4x32_10({c0, call_lo, 6u, c3}, k0, k1);
      }
      l.pick = (kInj && dr.l_pick) ? dr.l_pick[s] : (int64_t)bounded64(w5.x, w5.y, (uint64_t)npick);
    }
    index_loads(buf, kInj && g.idxs != nullptr, pick, &idx, &fin);
    const int64_t v_rand = cfg.value_cur_is_one ? 0 : rand_goal_of(buf, v.pick);
    const int64_t a_rand = cfg.actor_cur_is_one ? 0 : rand_goal_of(buf, a.pick);
    if (hc.has_low_value_goals && !cfg.value_cur_is_one) l_rand = rand_goal_of(buf, l.pick);
    const int64_t next = idx + 1 < buf.num_rows ? idx + 1 : buf.num_rows - 1;
    const double uvg = u01_from(w1.z, w1.w), uag = u01_from(w2.x, w2.y);
    v.geom = (kInj && g.v_geom) ? g.v_geom[s] : (cfg.value_geom_sample ? geometric_from(uvg, v_log_q) : 0);
    a.geom = (kInj && g.a_geom) ? g.a_geom[s] : (cfg.actor_geom_sample ? geometric_from(uag, a_log_q) : 0);
    v.dist = (kInj && g.v_dist) ? g.v_dist[s] : uvg;
    a.dist = (kInj && g.a_dist) ? g.a_dist[s] : uag;
    v.u_traj = (kInj && g.v_u_traj) ? g.v_u_traj[s] : u01_from(w2.z, w2.w);
    v.u_cur = (kInj && g.v_u_cur) ? g.v_u_cur[s] : u01_from(w3.x, w3.y);
    a.u_traj = (kInj && g.a_u_traj) ? g.a_u_traj[s] : u01_from(w3.z, w3.w);
    a.u_cur = (kInj && g.a_u_cur) ? g.a_u_cur[s] : u01_from(w4.x, w4.y);
    const int64_t hvg = sample_goal(idx, fin, v, v_rand, cfg.value_p_curgoal, cfg.value_traj_thresh,
                                    cfg.value_geom_sample, cfg.value_cur_is_one);
    const int64_t hag = sample_goal(idx, fin, a, a_rand, cfg.actor_p_curgoal, cfg.actor_traj_thresh,
                                    cfg.actor_geom_sample, cfg.actor_cur_is_one);
    int64_t lvg = idx;
    if (hc.has_low_value_goals) {
      l.geom = (kInj && dr.l_geom) ? dr.l_geom[s] : geometric_from(u01_from(w5.z, w5.w), l_log_q);
      l.dist = 0.0;
      l.u_traj = (kInj && dr.l_u_traj) ? dr.l_u_traj[s] : u01_from(w6.x, w6.y);
      l.u_cur = (kInj && dr.l_u_cur) ? dr.l_u_cur[s] : u01_from(w6.z, w6.w);
      lvg = sample_goal(idx, fin, l, l_rand, cfg.value_p_curgoal, cfg.value_traj_thresh, 1,
                        cfg.value_cur_is_one);
      if (rec.l_pick && own) {
        rec.l_pick[s] = l.pick;
        rec.l_geom[s] = l.geom;
        rec.l_u_traj[s] = l.u_traj;
        rec.l_u_cur[s] = l.u_cur;
      }
    }
    int64_t hv_next, hv_steps, lv_next, lv_steps, ha_next, ha_steps, la_next, la_steps;
    high_next(idx, fin, hvg, hc.value_subgoal_steps, &hv_next, &hv_steps);
    high_next(idx, fin, hvg, hc.low_subgoal_steps, &lv_next, &lv_steps);
    high_next(idx, fin, hag, hc.actor_subgoal_steps, &ha_next, &ha_steps);
    const int64_t la_goal = idx + hc.actor_subgoal_steps < fin ? idx + hc.actor_subgoal_steps : fin;
    high_next(idx, fin, hag, hc.low_subgoal_steps, &la_next, &la_steps);
    if (own) {
    const int t = b;
    sel[0][t] = idx;
    sel[1][t] = next;
    sel[2][t] = hvg;
    sel[3][t] = hag;
    sel[4][t] = hv_next;
    sel[5][t] = lv_next;
    sel[6][t] = lvg;
    sel[7][t] = ha_next;
    sel[8][t] = la_goal;
    sel[9][t] = la_next;
    if (o.idxs) o.idxs[s] = idx;
    if (o.high_value_goal_idxs) o.high_value_goal_idxs[s] = hvg;
    if (o.high_actor_goal_idxs) o.high_actor_goal_idxs[s] = hag;
    if (o.low_value_goal_idxs) o.low_value_goal_idxs[s] = lvg;
    const double neg = cfg.gc_negative ? 1.0 : 0.0;
    o.high_value_offsets[s] = hvg - idx;
    o.high_value_subgoal_steps[s] = hv_steps;
    o.high_value_masks[s] = hc.hv_mask_table[hv_steps];
    o.high_value_rewards[s] = hc.hv_reward_table[hv_steps];
    o.low_value_subgoal_steps[s] = lv_steps;
    if (hc.has_low_value_goals) {
      const double ls = idx == lvg ? 1.0 : 0.0;
      o.low_value_masks[s] = 1.0 - ls;
      o.low_value_rewards[s] = ls - neg;
    } else {
      o.low_value_masks[s] = hc.lv_mask_table[lv_steps];
      o.low_value_rewards[s] = hc.lv_reward_table[lv_steps];
    }
    const double succ = idx == hvg ? 1.0 : 0.0;
    o.masks[s] = 1.0 - succ;
    o.rewards[s] = succ - neg;
    if (rec.gc.pick) {
      rec.gc.pick[s] = pick;
      rec.gc.v_pick[s] = v.pick;
      rec.gc.v_geom[s] = v.geom;
      rec.gc.v_dist[s] = v.dist;
      rec.gc.v_u_traj[s] = v.u_traj;
      rec.gc.v_u_cur[s] = v.u_cur;
      rec.gc.a_pick[s] = a.pick;
      rec.gc.a_geom[s] = a.geom;
      rec.gc.a_dist[s] = a.dist;
      rec.gc.a_u_traj[s] = a.u_traj;
      rec.gc.a_u_cur[s] = a.u_cur;
    }
    }  // own
  }
  __syncthreads();
  copy_tile<0>(cols, num_cols, sel, base, n_here, flat4);
}

// HGC look-ahead: one sample's ten selectors and nine scalar outputs (the
// order of ogbx_hgc_outputs from high_value_offsets on), as hgc_sample_kernel's
// Philox path computes them.
struct HgcPick {
  int64_t sel[kHgcSel];
  int64_t w[9];  // offsets, hv steps, hv mask, hv reward, lv steps, lv mask, lv reward, mask, reward (f64 as bits)
};

// The HGC reward tables held in the first wave's registers: lane t holds
// entries t and t + 64 of the value / low tables (loaded when the chain
// starts, so they arrive while it runs), and the chain's lookups are lane
// reads instead of global loads that wait for the subgoal step counts.  Valid when both tables have at most 128 entries (subgoal
// steps <= 127).  The mask tables are held the same way (the caller's tables,
// not 1 - (s < K) recomputed, so a C-ABI host's own tables give the same
// result as the direct ogbx_hgc_sample).
struct HgcTables {
  double hv0, hv1, lv0, lv1, hm0, hm1, lm0, lm1;
  bool regs;
};

__device__ __forceinline__ HgcTables hgc_tables_load(const ogbx_hgc_config& hc) {
  HgcTables tb{0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, hc.value_subgoal_steps < 128 && hc.low_subgoal_steps < 128};
  const int t = (int)(threadIdx.x & 63);
  // clamped indices, every lane, no branch (a region around the loads made
  // the compiler wait for them at its end); entries past K are never looked
  // up, and with K >= 128 the lookups read the tables in memory instead
  const int64_t kv = hc.value_subgoal_steps, kl = hc.low_subgoal_steps;
  tb.hv0 = hc.hv_reward_table[min((int64_t)t, kv)];
  tb.hv1 = hc.hv_reward_table[min((int64_t)t + 64, kv)];
  tb.lv0 = hc.lv_reward_table[min((int64_t)t, kl)];
  tb.lv1 = hc.lv_reward_table[min((int64_t)t + 64, kl)];
  tb.hm0 = hc.hv_mask_table[min((int64_t)t, kv)];
  tb.hm1 = hc.hv_mask_table[min((int64_t)t + 64, kv)];
  tb.lm0 = hc.lv_mask_table[min((int64_t)t, kl)];
  tb.lm1 = hc.lv_mask_table[min((int64_t)t + 64, kl)];
  return tb;
}

// entry s (wave-uniform) of a register-held table
__device__ __forceinline__ double table_lane(double v0, double v1, int64_t s) {
  const int i = __builtin_amdgcn_readfirstlane((int)s);
  const double v = i < 64 ? v0 : v1;
  const int l = i & 63;
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l),
                          __builtin_amdgcn_readlane(__double2loint(v), l));
}

__device__ inline HgcPick hgc_chain(const ogbx_gc_buffer& buf, const ogbx_gc_config& cfg, const ogbx_hgc_config& hc,
                                    const u32x4* wv, double v_log_q, double a_log_q, double l_log_q,
                                    const HgcTables& tb) {
  const u32x4 w0 = wv[0], w1 = wv[1], w2 = wv[2], w3 = wv[3], w4 = wv[4];
  const int64_t npick = buf.valid_idxs ? buf.num_valid : buf.num_rows;
  const int64_t pick = (int64_t)bounded64(w0.x, w0.y, (uint64_t)npick);
  GoalDraws v, a, l;
  v.pick = (int64_t)bounded64(w0.z, w0.w, (uint64_t)npick);
  a.pick = (int64_t)bounded64(w1.x, w1.y, (uint64_t)npick);
  u32x4 w5{}, w6{};
  int64_t l_rand = 0;
  if (hc.has_low_value_goals) {
    w5 = wv[5];
    w6 = wv[6];
    l.pick = (int64_t)bounded64(w5.x, w5.y, (uint64_t)npick);
  }
  int64_t idx = 0, fin;
  index_loads(buf, false, pick, &idx, &fin);
  const int64_t v_rand = cfg.value_cur_is_one ? 0 : rand_goal_of(buf, v.pick);
  const int64_t a_rand = cfg.actor_cur_is_one ? 0 : rand_goal_of(buf, a.pick);
  if (hc.has_low_value_goals && !cfg.value_cur_is_one) l_rand = rand_goal_of(buf, l.pick);
  const int64_t next = idx + 1 < buf.num_rows ? idx + 1 : buf.num_rows - 1;
  const double uvg = u01_from(w1.z, w1.w), uag = u01_from(w2.x, w2.y);
  v.geom = cfg.value_geom_sample ? geometric_from(uvg, v_log_q) : 0;
  a.geom = cfg.actor_geom_sample ? geometric_from(uag, a_log_q) : 0;
  v.dist = uvg;
  a.dist = uag;
  v.u_traj = u01_from(w2.z, w2.w);
  v.u_cur = u01_from(w3.x, w3.y);
  a.u_traj = u01_from(w3.z, w3.w);
  a.u_cur = u01_from(w4.x, w4.y);
  const int64_t hvg = sample_goal(idx, fin, v, v_rand, cfg.value_p_curgoal, cfg.value_traj_thresh,
                                  cfg.value_geom_sample, cfg.value_cur_is_one);
  const int64_t hag = sample_goal(idx, fin, a, a_rand, cfg.actor_p_curgoal, cfg.actor_traj_thresh,
                                  cfg.actor_geom_sample, cfg.actor_cur_is_one);
  int64_t lvg = idx;
  if (hc.has_low_value_goals) {
    l.geom = geometric_from(u01_from(w5.z, w5.w), l_log_q);
    l.dist = 0.0;
    l.u_traj = u01_from(w6.x, w6.y);
    l.u_cur = u01_from(w6.z, w6.w);
    lvg = sample_goal(idx, fin, l, l_rand, cfg.value_p_curgoal, cfg.value_traj_thresh, 1, cfg.value_cur_is_one);
  }
  int64_t hv_next, hv_steps, lv_next, lv_steps, ha_next, ha_steps, la_next, la_steps;
  high_next(idx, fin, hvg, hc.value_subgoal_steps, &hv_next, &hv_steps);
  high_next(idx, fin, hvg, hc.low_subgoal_steps, &lv_next, &lv_steps);
  high_next(idx, fin, hag, hc.actor_subgoal_steps, &ha_next, &ha_steps);
  const int64_t la_goal = idx + hc.actor_subgoal_steps < fin ? idx + hc.actor_subgoal_steps : fin;
  high_next(idx, fin, hag, hc.low_subgoal_steps, &la_next, &la_steps);
  HgcPick p;
  p.sel[0] = idx;
  p.sel[1] = next;
  p.sel[2] = hvg;
  p.sel[3] = hag;
  p.sel[4] = hv_next;
  p.sel[5] = lv_next;
  p.sel[6] = lvg;
  p.sel[7] = ha_next;
  p.sel[8] = la_goal;
  p.sel[9] = la_next;
  const double neg = cfg.gc_negative ? 1.0 : 0.0;
  p.w[0] = hvg - idx;
  p.w[1] = hv_steps;
  if (tb.regs) {
    p.w[2] = __double_as_longlong(table_lane(tb.hm0, tb.hm1, hv_steps));
    p.w[3] = __double_as_longlong(table_lane(tb.hv0, tb.hv1, hv_steps));
  } else {
    p.w[2] = __double_as_longlong(hc.hv_mask_table[hv_steps]);
    p.w[3] = __double_as_longlong(hc.hv_reward_table[hv_steps]);
  }
  p.w[4] = lv_steps;
  if (hc.has_low_value_goals) {
    const double ls = idx == lvg ? 1.0 : 0.0;
    p.w[5] = __double_as_longlong(1.0 - ls);
    p.w[6] = __double_as_longlong(ls - neg);
  } else if (tb.regs) {
    p.w[5] = __double_as_longlong(table_lane(tb.lm0, tb.lm1, lv_steps));
    p.w[6] = __double_as_longlong(table_lane(tb.lv0, tb.lv1, lv_steps));
  } else {
    p.w[5] = __double_as_longlong(hc.lv_mask_table[lv_steps]);
    p.w[6] = __double_as_longlong(hc.lv_reward_table[lv_steps]);
  }
  const double succ = idx == hvg ? 1.0 : 0.0;
  p.w[7] = __double_as_longlong(1.0 - succ);
  p.w[8] = __double_as_longlong(succ - neg);
  return p;
}

__device__ inline HgcPick hgc_wave_chain(const ogbx_gc_buffer& buf, const ogbx_gc_config& cfg,
                                         const ogbx_hgc_config& hc, int64_t s, uint32_t lo, uint32_t hi, uint32_t k0,
                                         uint32_t k1, double v_log_q, double a_log_q, double l_log_q) {
  // the reward tables: issued first, they arrive while the Philox calls and
  // the goal chain run (their lookups come last)
  const HgcTables tb = hgc_tables_load(hc);
  const uint64_t su = (uint64_t)s;
  const uint32_t calls = hc.has_low_value_goals ? 7u : 5u;
  const uint32_t q = (uint32_t)(threadIdx.x & 63) % calls;
  const u32x4 w = philox4x32_10({(uint32_t)su, lo, q, (uint32_t)(su >> 32) ^ hi}, k0, k1);
  u32x4 ws[7];
#pragma unroll
  for (int c = 0; c < 7; ++c)
    ws[c] = u32x4{(uint32_t)__builtin_amdgcn_readlane((int)w.x, c), (uint32_t)__builtin_amdgcn_readlane((int)w.y, c),
                  (uint32_t)__builtin_amdgcn_readlane((int)w.z, c), (uint32_t)__builtin_amdgcn_readlane((int)w.w, c)};
  return hgc_chain(buf, cfg, hc, ws, v_log_q, a_log_q, l_log_q, tb);
}

constexpr int kHgcAheadWords = OGBX_HGC_AHEAD_WORDS;
static_assert(kHgcAheadWords >= kHgcSel + 9, "HGC look-ahead record: 10 selectors + 9 scalars");

// HGCDataset.sample with look-ahead (gc_ahead_kernel's scheme).
template <bool kHit, class Cols = GcColumns>
__global__ void __launch_bounds__(256) hgc_ahead_kernel(
    ogbx_gc_buffer buf, ogbx_gc_config cfg, ogbx_hgc_config hc, Cols cols, int32_t num_cols, uint32_t k0,
    uint32_t k1, uint32_t call_lo, uint32_t call_hi, uint32_t next_lo, uint32_t next_hi, double v_log_q,
    double a_log_q, double l_log_q, const int64_t* __restrict__ ahead_in, int64_t* __restrict__ ahead_out,
    ogbx_hgc_outputs o, bool flat4) {
  __shared__ int64_t sel[kHgcSel][kGcMaxTile];
  const int64_t s = xcd_tile();
  const int t = (int)threadIdx.x;
  // scalar word j (0..8) of a record -> its output (static j: no pointer array)
  auto put_scalar = [&](int j, int64_t v) {
    switch (j) {
      case 0: o.high_value_offsets[s] = v; break;
      case 1: o.high_value_subgoal_steps[s] = v; break;
      case 2: o.high_value_masks[s] = __longlong_as_double(v); break;
      case 3: o.high_value_rewards[s] = __longlong_as_double(v); break;
      case 4: o.low_value_subgoal_steps[s] = v; break;
      case 5: o.low_value_masks[s] = __longlong_as_double(v); break;
      case 6: o.low_value_rewards[s] = __longlong_as_double(v); break;
      case 7: o.masks[s] = __longlong_as_double(v); break;
      default: o.rewards[s] = __longlong_as_double(v); break;
    }
  };
  auto put_index = [&](int k, int64_t v) {
    if (k == 0 && o.idxs) o.idxs[s] = v;
    if (k == 2 && o.high_value_goal_idxs) o.high_value_goal_idxs[s] = v;
    if (k == 3 && o.high_actor_goal_idxs) o.high_actor_goal_idxs[s] = v;
    if (k == 6 && o.low_value_goal_idxs) o.low_value_goal_idxs[s] = v;
  };
  if constexpr (kHit) {
    // Hit: no block barrier (gc_ahead_kernel's scheme)
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6), lane = t & 63;
    if (wave == 0) {
      const int64_t v = lane < kHgcSel + 9 ? ahead_in[s * kHgcAheadWords + lane] : 0;
      if (ahead_out) {
        const HgcPick p = hgc_wave_chain(buf, cfg, hc, s, next_lo, next_hi, k0, k1, v_log_q, a_log_q, l_log_q);
        if (t == 0) {
          int64_t* r = ahead_out + s * kHgcAheadWords;
#pragma unroll
          for (int k = 0; k < kHgcSel; ++k) r[k] = p.sel[k];
#pragma unroll
          for (int j = 0; j < 9; ++j) r[kHgcSel + j] = p.w[j];
        }
      }
      if (lane < kHgcSel)
        put_index(lane, v);
      else if (lane < kHgcSel + 9)
        put_scalar(lane - kHgcSel, v);
      return;
    }
    if (lane < kHgcSel) sel[lane][wave] = ahead_in[s * kHgcAheadWords + lane];
    __builtin_amdgcn_wave_barrier();
    copy_tile<0, true>(cols, num_cols, reinterpret_cast<const int64_t(*)[kGcMaxTile]>(&sel[0][wave]), s, 1, flat4, 1);
    return;
  }
  if (t < 64) {
    const HgcPick p = hgc_wave_chain(buf, cfg, hc, s, call_lo, call_hi, k0, k1, v_log_q, a_log_q, l_log_q);
    if (t == 0) {
#pragma unroll
      for (int k = 0; k < kHgcSel; ++k) {
        sel[k][0] = p.sel[k];
        put_index(k, p.sel[k]);
      }
#pragma unroll
      for (int j = 0; j < 9; ++j) put_scalar(j, p.w[j]);
    }
  }
  __syncthreads();
  if (ahead_out && t < 64) {
    const HgcPick p = hgc_wave_chain(buf, cfg, hc, s, next_lo, next_hi, k0, k1, v_log_q, a_log_q, l_log_q);
    if (t == 0) {
      int64_t* r = ahead_out + s * kHgcAheadWords;
#pragma unroll
      for (int k = 0; k < kHgcSel; ++k) r[k] = p.sel[k];
#pragma unroll
      for (int j = 0; j < 9; ++j) r[kHgcSel + j] = p.w[j];
    }
  } else {
    copy_tile<0>(cols, num_cols, sel, s, 1, flat4, ahead_out ? 1 : 0);
  }
}

__global__ void traj_end_kernel(const int64_t* __restrict__ term, int64_t nterm, int64_t nrows,
                                int64_t* __restrict__ out) {
  int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nrows) return;
  // searchsorted(term, r, side='left'): first position with term[pos] >= r
  int64_t lo = 0, hi = nterm;
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    if (term[mid] < r) lo = mid + 1;
    else hi = mid;
  }
  out[r] = lo < nterm ? term[lo] : term[nterm - 1];
}

struct PositiveF32 {
  const float* x;
  __device__ bool operator()(const int64_t& i) const { return x[i] > 0.0f; }
};

}  // namespace ogbx

using namespace ogbx;

// Every column 4-byte granular and aligned with rows of <= 128 words (the
// per-wave job copy of copy_tile).
static bool flat4_columns(const GcColumns& cc, int num_cols) {
  for (int i = 0; i < num_cols; ++i) {
    const ogbx_gc_column& c = cc.c[i];
    if (c.row_bytes % 4 != 0 || c.row_bytes > 512 ||
        ((uintptr_t)c.src | (uintptr_t)c.dst | (uintptr_t)c.src_stride) % 4 != 0)
      return false;
  }
  return true;
}

// True when any draw is injected (parity replays); the Philox-only kernels
// carry no per-draw pointer tests, so their index loads issue back to back.
static bool any_draw(const ogbx_gc_draws& d) {
  return d.idxs || d.pick || d.v_pick || d.v_geom || d.v_dist || d.v_u_traj || d.v_u_cur ||
         d.a_pick || d.a_geom || d.a_dist || d.a_u_traj || d.a_u_cur;
}

// period == 0, or a whole number of periods covering the buffer with the
// picks and the trajectory end inside one period.
static bool periodic_ok(const ogbx_gc_buffer& b) {
  if (b.period == 0) return true;
  const int64_t npick = b.valid_idxs ? b.num_valid : b.num_rows;
  return b.period > 0 && b.period_picks > 0 && b.period_picks <= b.period && b.period_end >= 0 &&
         b.period_end < b.period && b.num_rows % b.period == 0 &&
         npick == (b.num_rows / b.period) * b.period_picks;
}

extern "C" {

ogbx_status ogbx_gc_sample(const ogbx_gc_buffer* buf, const ogbx_gc_config* cfg,
                           const ogbx_gc_column* cols, int32_t num_cols, int64_t batch,
                           int64_t num_batches, const ogbx_gc_draws* draws, uint64_t seed,
                           uint64_t call_index, int64_t* idxs_out, int64_t* value_goal_out,
                           int64_t* actor_goal_out, double* masks, double* rewards,
                           const ogbx_gc_draw_record* record, void* stream) {
  OGBX_CHECK(buf && cfg && masks && rewards, OGBX_EINVAL, "ogbx_gc_sample: null argument");
  OGBX_CHECK(num_cols >= 0 && num_cols <= kGcMaxCols, OGBX_EINVAL,
             "ogbx_gc_sample: at most 32 columns");
  OGBX_CHECK(batch > 0 && num_batches > 0, OGBX_EINVAL, "batch and num_batches must be > 0");
  OGBX_CHECK(buf->num_rows > 0 && buf->traj_end, OGBX_EINVAL, "empty trajectory buffer");
  OGBX_CHECK(buf->valid_idxs == nullptr || buf->num_valid > 0, OGBX_EINVAL,
             "no valid transitions in the dataset");
  OGBX_CHECK(periodic_ok(*buf), OGBX_EINVAL, "ogbx_gc_buffer: inconsistent period fields");
  GcColumns cc{};
  for (int i = 0; i < num_cols; ++i) {
    OGBX_CHECK(cols[i].src_stride == 0 || cols[i].src_stride >= cols[i].row_bytes, OGBX_EINVAL,
               "ogbx_gc_sample: src_stride below row_bytes");
    OGBX_CHECK(cols[i].src && cols[i].dst && cols[i].row_bytes > 0 && cols[i].select >= 0 &&
                   cols[i].select <= 3,
               OGBX_EINVAL, "ogbx_gc_sample: bad column descriptor");
    cc.c[i] = cols[i];
  }
  ogbx_gc_draws dr{};
  if (draws) dr = *draws;
  ogbx_gc_draw_record rec{};
  if (record) rec = *record;
  const int64_t total = batch * num_batches;
  // tile: one sample per workgroup up to 1024 samples (B = 1024: 1,024
  // workgroups of 256 threads; measured against 2 and 4 samples per workgroup
  // and 64- to 1024-thread workgroups), then up to 64 per workgroup
  int64_t tile = total / 1024;
  if (tile < 1) tile = 1;
  if (tile > kGcMaxTile) tile = kGcMaxTile;
  const int64_t blocks = (total + tile - 1) / tile;
  uint32_t k0, k1;
  seed_key(seed, kTagGcSample, &k0, &k1);
  const double v_log_q = std::log(1.0 - (1.0 - cfg->value_discount));
  const double a_log_q = std::log(1.0 - (1.0 - cfg->actor_discount));
  auto kern = any_draw(dr) ? gc_sample_kernel<true> : gc_sample_kernel<false>;
  hipLaunchKernelGGL(kern, dim3((uint32_t)blocks), dim3(256), 0, (hipStream_t)stream,
                     *buf, *cfg, cc, num_cols, total, (int)tile, dr, k0, k1,
                     (uint32_t)call_index, (uint32_t)(call_index >> 32), v_log_q, a_log_q,
                     idxs_out, value_goal_out, actor_goal_out, masks, rewards, rec,
                     tile <= 4 && flat4_columns(cc, num_cols));
  OGBX_LAUNCHED("gc_sample_kernel");
  return OGBX_OK;
}

ogbx_status ogbx_gc_sample_ahead(const ogbx_gc_buffer* buf, const ogbx_gc_config* cfg,
                                 const ogbx_gc_column* cols, int32_t num_cols, int64_t batch,
                                 int64_t num_batches, uint64_t seed, uint64_t call_index,
                                 const int64_t* ahead_in, int64_t* ahead_out, int64_t* idxs_out,
                                 int64_t* value_goal_out, int64_t* actor_goal_out, double* masks,
                                 double* rewards, void* stream) {
  OGBX_CHECK(buf && cfg && masks && rewards, OGBX_EINVAL, "ogbx_gc_sample_ahead: null argument");
  OGBX_CHECK(num_cols >= 0 && num_cols <= kGcMaxCols, OGBX_EINVAL, "ogbx_gc_sample_ahead: at most 32 columns");
  OGBX_CHECK(batch > 0 && num_batches > 0, OGBX_EINVAL, "batch and num_batches must be > 0");
  const int64_t total = batch * num_batches;
  OGBX_CHECK(total <= kGcAheadMaxSamples, OGBX_EINVAL,
             "ogbx_gc_sample_ahead: at most 1024 samples per call (one per workgroup)");
  OGBX_CHECK(buf->num_rows > 0 && buf->traj_end, OGBX_EINVAL, "empty trajectory buffer");
  OGBX_CHECK(buf->valid_idxs == nullptr || buf->num_valid > 0, OGBX_EINVAL, "no valid transitions in the dataset");
  OGBX_CHECK(periodic_ok(*buf), OGBX_EINVAL, "ogbx_gc_buffer: inconsistent period fields");
  OGBX_CHECK(ahead_in != ahead_out || ahead_in == nullptr, OGBX_EINVAL,
             "ogbx_gc_sample_ahead: ahead_in and ahead_out must differ");
  GcColumns cc{};
  for (int i = 0; i < num_cols; ++i) {
    OGBX_CHECK(cols[i].src_stride == 0 || cols[i].src_stride >= cols[i].row_bytes, OGBX_EINVAL,
               "ogbx_gc_sample_ahead: src_stride below row_bytes");
    OGBX_CHECK(cols[i].src && cols[i].dst && cols[i].row_bytes > 0 && cols[i].select >= 0 && cols[i].select <= 3,
               OGBX_EINVAL, "ogbx_gc_sample_ahead: bad column descriptor");
    cc.c[i] = cols[i];
  }
  uint32_t k0, k1;
  seed_key(seed, kTagGcSample, &k0, &k1);
  const double v_log_q = std::log(1.0 - (1.0 - cfg->value_discount));
  const double a_log_q = std::log(1.0 - (1.0 - cfg->actor_discount));
  const uint64_t next = call_index + 1;
  const auto kern = ahead_in ? gc_ahead_kernel<true> : gc_ahead_kernel<false>;
  hipLaunchKernelGGL(kern, dim3((uint32_t)total), dim3(256), 0, (hipStream_t)stream, *buf, *cfg, cc,
                     num_cols, k0, k1, (uint32_t)call_index, (uint32_t)(call_index >> 32), (uint32_t)next,
                     (uint32_t)(next >> 32), v_log_q, a_log_q, ahead_in, ahead_out, idxs_out, value_goal_out,
                     actor_goal_out, masks, rewards, flat4_columns(cc, num_cols));
  OGBX_LAUNCHED("gc_ahead_kernel");
  return OGBX_OK;
}

ogbx_status ogbx_hgc_sample(const ogbx_gc_buffer* buf, const ogbx_gc_config* cfg,
                            const ogbx_hgc_config* hcfg, const ogbx_gc_column* cols,
                            int32_t num_cols, int64_t batch, int64_t num_batches,
                            const ogbx_hgc_draws* draws, uint64_t seed, uint64_t call_index,
                            const ogbx_hgc_outputs* out, const ogbx_hgc_draw_record* record,
                            void* stream) {
  OGBX_CHECK(buf && cfg && hcfg && out, OGBX_EINVAL, "ogbx_hgc_sample: null argument");
  OGBX_CHECK(out->high_value_offsets && out->high_value_subgoal_steps && out->high_value_masks &&
                 out->high_value_rewards && out->low_value_subgoal_steps && out->low_value_masks &&
                 out->low_value_rewards && out->masks && out->rewards,
             OGBX_EINVAL, "ogbx_hgc_sample: missing scalar output");
  OGBX_CHECK(hcfg->hv_mask_table && hcfg->hv_reward_table && hcfg->lv_mask_table && hcfg->lv_reward_table,
             OGBX_EINVAL, "ogbx_hgc_sample: missing reward/mask tables");
  OGBX_CHECK(hcfg->value_subgoal_steps >= 0 && hcfg->low_subgoal_steps >= 0 && hcfg->actor_subgoal_steps >= 0,
             OGBX_EINVAL, "ogbx_hgc_sample: negative subgoal steps");
  OGBX_CHECK(!hcfg->has_low_value_goals || (hcfg->low_discount > 0.0 && hcfg->low_discount < 1.0),
             OGBX_EINVAL, "ogbx_hgc_sample: low_discount must be in (0, 1)");
  OGBX_CHECK(num_cols >= 0 && num_cols <= kGcMaxCols, OGBX_EINVAL, "ogbx_hgc_sample: at most 32 columns");
  OGBX_CHECK(batch > 0 && num_batches > 0, OGBX_EINVAL, "batch and num_batches must be > 0");
  OGBX_CHECK(buf->num_rows > 0 && buf->traj_end, OGBX_EINVAL, "empty trajectory buffer");
  OGBX_CHECK(buf->valid_idxs == nullptr || buf->num_valid > 0, OGBX_EINVAL,
             "no valid transitions in the dataset");
  OGBX_CHECK(periodic_ok(*buf), OGBX_EINVAL, "ogbx_gc_buffer: inconsistent period fields");
  GcColumns cc{};
  for (int i = 0; i < num_cols; ++i) {
    OGBX_CHECK(cols[i].src_stride == 0 || cols[i].src_stride >= cols[i].row_bytes, OGBX_EINVAL,
               "ogbx_gc_sample: src_stride below row_bytes");
    OGBX_CHECK(cols[i].src && cols[i].dst && cols[i].row_bytes > 0 && cols[i].select >= 0 &&
                   cols[i].select < kHgcSel,
               OGBX_EINVAL, "ogbx_hgc_sample: bad column descriptor");
    cc.c[i] = cols[i];
  }
  ogbx_hgc_draws dr{};
  if (draws) dr = *draws;
  ogbx_hgc_draw_record rec{};
  if (record) rec = *record;
  const int64_t total = batch * num_batches;
  int64_t tile = total / 1024;  // as ogbx_gc_sample
  if (tile < 1) tile = 1;
  if (tile > kGcMaxTile) tile = kGcMaxTile;
  const int64_t blocks = (total + tile - 1) / tile;
  uint32_t k0, k1;
  seed_key(seed, kTagHgcSample, &k0, &k1);
  const double v_log_q = std::log(1.0 - (1.0 - cfg->value_discount));
  const double a_log_q = std::log(1.0 - (1.0 - cfg->actor_discount));
  const double l_log_q = hcfg->has_low_value_goals ? std::log(1.0 - (1.0 - hcfg->low_discount)) : 0.0;
  const bool inj = any_draw(dr.gc) || dr.l_pick || dr.l_geom || dr.l_u_traj || dr.l_u_cur;
  auto kern = inj ? hgc_sample_kernel<true> : hgc_sample_kernel<false>;
  hipLaunchKernelGGL(kern, dim3((uint32_t)blocks), dim3(256), 0, (hipStream_t)stream, *buf,
                     *cfg, *hcfg, cc, num_cols, total, (int)tile, dr, k0, k1, (uint32_t)call_index,
                     (uint32_t)(call_index >> 32), v_log_q, a_log_q, l_log_q, *out, rec,
                     tile <= 4 && flat4_columns(cc, num_cols));
  OGBX_LAUNCHED("hgc_sample_kernel");
  return OGBX_OK;
}

ogbx_status ogbx_hgc_sample_ahead(const ogbx_gc_buffer* buf, const ogbx_gc_config* cfg,
                                  const ogbx_hgc_config* hcfg, const ogbx_gc_column* cols, int32_t num_cols,
                                  int64_t batch, int64_t num_batches, uint64_t seed, uint64_t call_index,
                                  const int64_t* ahead_in, int64_t* ahead_out, const ogbx_hgc_outputs* out,
                                  void* stream) {
  OGBX_CHECK(buf && cfg && hcfg && out, OGBX_EINVAL, "ogbx_hgc_sample_ahead: null argument");
  OGBX_CHECK(out->high_value_offsets && out->high_value_subgoal_steps && out->high_value_masks &&
                 out->high_value_rewards && out->low_value_subgoal_steps && out->low_value_masks &&
                 out->low_value_rewards && out->masks && out->rewards,
             OGBX_EINVAL, "ogbx_hgc_sample_ahead: missing scalar output");
  OGBX_CHECK(hcfg->hv_mask_table && hcfg->hv_reward_table && hcfg->lv_mask_table && hcfg->lv_reward_table,
             OGBX_EINVAL, "ogbx_hgc_sample_ahead: missing reward/mask tables");
  OGBX_CHECK(hcfg->value_subgoal_steps >= 0 && hcfg->low_subgoal_steps >= 0 && hcfg->actor_subgoal_steps >= 0,
             OGBX_EINVAL, "ogbx_hgc_sample_ahead: negative subgoal steps");
  OGBX_CHECK(!hcfg->has_low_value_goals || (hcfg->low_discount > 0.0 && hcfg->low_discount < 1.0), OGBX_EINVAL,
             "ogbx_hgc_sample_ahead: low_discount must be in (0, 1)");
  OGBX_CHECK(num_cols >= 0 && num_cols <= kGcMaxCols, OGBX_EINVAL, "ogbx_hgc_sample_ahead: at most 32 columns");
  OGBX_CHECK(batch > 0 && num_batches > 0, OGBX_EINVAL, "batch and num_batches must be > 0");
  const int64_t total = batch * num_batches;
  OGBX_CHECK(total <= kGcAheadMaxSamples, OGBX_EINVAL,
             "ogbx_hgc_sample_ahead: at most 1024 samples per call (one per workgroup)");
  OGBX_CHECK(buf->num_rows > 0 && buf->traj_end, OGBX_EINVAL, "empty trajectory buffer");
  OGBX_CHECK(buf->valid_idxs == nullptr || buf->num_valid > 0, OGBX_EINVAL, "no valid transitions in the dataset");
  OGBX_CHECK(periodic_ok(*buf), OGBX_EINVAL, "ogbx_gc_buffer: inconsistent period fields");
  OGBX_CHECK(ahead_in != ahead_out || ahead_in == nullptr, OGBX_EINVAL,
             "ogbx_hgc_sample_ahead: ahead_in and ahead_out must differ");
  GcColumns cc{};
  for (int i = 0; i < num_cols; ++i) {
    OGBX_CHECK(cols[i].src_stride == 0 || cols[i].src_stride >= cols[i].row_bytes, OGBX_EINVAL,
               "ogbx_hgc_sample_ahead: src_stride below row_bytes");
    OGBX_CHECK(cols[i].src && cols[i].dst && cols[i].row_bytes > 0 && cols[i].select >= 0 &&
                   cols[i].select < kHgcSel,
               OGBX_EINVAL, "ogbx_hgc_sample_ahead: bad column descriptor");
    cc.c[i] = cols[i];
  }
  uint32_t k0, k1;
  seed_key(seed, kTagHgcSample, &k0, &k1);
  const double v_log_q = std::log(1.0 - (1.0 - cfg->value_discount));
  const double a_log_q = std::log(1.0 - (1.0 - cfg->actor_discount));
  const double l_log_q = hcfg->has_low_value_goals ? std::log(1.0 - (1.0 - hcfg->low_discount)) : 0.0;
  const uint64_t next = call_index + 1;
  const auto kern = ahead_in ? hgc_ahead_kernel<true> : hgc_ahead_kernel<false>;
  hipLaunchKernelGGL(kern, dim3((uint32_t)total), dim3(256), 0, (hipStream_t)stream, *buf, *cfg, *hcfg,
                     cc, num_cols, k0, k1, (uint32_t)call_index, (uint32_t)(call_index >> 32), (uint32_t)next,
                     (uint32_t)(next >> 32), v_log_q, a_log_q, l_log_q, ahead_in, ahead_out, *out,
                     flat4_columns(cc, num_cols));
  OGBX_LAUNCHED("hgc_ahead_kernel");
  return OGBX_OK;
}

}  // extern "C"

// ---------------------------------------------------------------- sampler plans
// A plan owns everything a steady stream of GCDataset / HGCDataset.sample
// calls repeats: the validated buffer and config, the Philox key, the
// geometric log terms, up to OGBX_GC_PLAN_SLOTS prepared output batches (the
// column descriptors as one kernel-argument image), and the look-ahead state:
// one pair of selector buffers per stream (allocated on the stream's first
// call, never shared across streams) and the (stream, samples, call) the
// last launch stored selectors for.  A call is then one lookup and one launch.
namespace {
constexpr int kPlanStreams = 8;

struct PlanBatch {
  bool set = false;
  GcColumns cc{};
  int32_t ncols = 0;
  int64_t batch = 0, nb = 0;
  int64_t *idxs = nullptr, *vg = nullptr, *ag = nullptr;
  double *masks = nullptr, *rewards = nullptr;
  ogbx_hgc_outputs hout{};
  bool flat4 = false;
  bool small = false;  // ncols <= kGcSmallCols: launch with cs
  GcColumnsSmall cs{};
};

struct PlanPair {
  void* stream = nullptr;
  int64_t* buf[2] = {nullptr, nullptr};
};
}  // namespace

struct ogbx_gc_plan_s {
  ogbx_gc_buffer buf;
  ogbx_gc_config cfg;
  ogbx_hgc_config hcfg;
  bool hgc = false, lookahead = true;
  int device = 0;
  uint32_t k0 = 0, k1 = 0;
  double v_log_q = 0, a_log_q = 0, l_log_q = 0;
  PlanBatch slots[OGBX_GC_PLAN_SLOTS];
  PlanPair pairs[kPlanStreams];
  int npairs = 0;
  // the selectors in pairs[key_pair].buf[key_which] belong to (key_total, key_call)
  bool key_valid = false;
  int key_pair = 0, key_which = 0;
  int64_t key_total = 0;
  uint64_t key_call = 0;
  int64_t hits = 0;
  // guards pairs / npairs / key_* / hits: ctypes releases the GIL, so two
  // host threads may call ogbx_gc_plan_sample on one plan (uncontended: ~20 ns)
  std::mutex mu;
};

extern "C" {

ogbx_status ogbx_gc_plan_create(const ogbx_gc_buffer* buf, const ogbx_gc_config* cfg,
                                const ogbx_hgc_config* hcfg, uint64_t seed, int32_t lookahead,
                                ogbx_gc_plan_t* plan) {
  OGBX_CHECK(buf && cfg && plan, OGBX_EINVAL, "ogbx_gc_plan_create: null argument");
  OGBX_CHECK(buf->num_rows > 0 && buf->traj_end, OGBX_EINVAL, "empty trajectory buffer");
  OGBX_CHECK(buf->valid_idxs == nullptr || buf->num_valid > 0, OGBX_EINVAL, "no valid transitions in the dataset");
  OGBX_CHECK(periodic_ok(*buf), OGBX_EINVAL, "ogbx_gc_buffer: inconsistent period fields");
  if (hcfg) {
    OGBX_CHECK(hcfg->hv_mask_table && hcfg->hv_reward_table && hcfg->lv_mask_table && hcfg->lv_reward_table,
               OGBX_EINVAL, "ogbx_gc_plan_create: missing reward/mask tables");
    OGBX_CHECK(hcfg->value_subgoal_steps >= 0 && hcfg->low_subgoal_steps >= 0 && hcfg->actor_subgoal_steps >= 0,
               OGBX_EINVAL, "ogbx_gc_plan_create: negative subgoal steps");
    OGBX_CHECK(!hcfg->has_low_value_goals || (hcfg->low_discount > 0.0 && hcfg->low_discount < 1.0), OGBX_EINVAL,
               "ogbx_gc_plan_create: low_discount must be in (0, 1)");
  }
  auto* p = new (std::nothrow) ogbx_gc_plan_s();
  OGBX_CHECK(p, OGBX_ENOMEM, "ogbx_gc_plan_create: out of host memory");
  p->buf = *buf;
  p->cfg = *cfg;
  p->hgc = hcfg != nullptr;
  if (hcfg) p->hcfg = *hcfg;
  p->lookahead = lookahead != 0;
  // the plan's device is the buffer's, not whichever device is current: the
  // look-ahead selector pairs are allocated there on a stream's first call
  hipPointerAttribute_t attr{};
  if (hipPointerGetAttributes(&attr, buf->traj_end) == hipSuccess && attr.type == hipMemoryTypeDevice)
    p->device = attr.device;
  else if (hipGetDevice(&p->device) != hipSuccess)
    p->device = 0;
  seed_key(seed, p->hgc ? kTagHgcSample : kTagGcSample, &p->k0, &p->k1);
  p->v_log_q = std::log(1.0 - (1.0 - cfg->value_discount));
  p->a_log_q = std::log(1.0 - (1.0 - cfg->actor_discount));
  p->l_log_q = (hcfg && hcfg->has_low_value_goals) ? std::log(1.0 - (1.0 - hcfg->low_discount)) : 0.0;
  *plan = p;
  return OGBX_OK;
}

ogbx_status ogbx_gc_plan_set_batch(ogbx_gc_plan_t p, int32_t slot, const ogbx_gc_column* cols, int32_t num_cols,
                                   int64_t batch, int64_t num_batches, int64_t* idxs_out, int64_t* value_goal_out,
                                   int64_t* actor_goal_out, double* masks, double* rewards,
                                   const ogbx_hgc_outputs* hgc_out) {
  OGBX_CHECK(p, OGBX_EINVAL, "null plan");
  OGBX_CHECK(slot >= 0 && slot < OGBX_GC_PLAN_SLOTS, OGBX_EINVAL, "ogbx_gc_plan_set_batch: slot out of range");
  OGBX_CHECK(num_cols >= 0 && num_cols <= kGcMaxCols, OGBX_EINVAL, "ogbx_gc_plan_set_batch: at most 32 columns");
  OGBX_CHECK(batch > 0 && num_batches > 0, OGBX_EINVAL, "batch and num_batches must be > 0");
  if (p->hgc) {
    OGBX_CHECK(hgc_out && hgc_out->high_value_offsets && hgc_out->high_value_subgoal_steps &&
                   hgc_out->high_value_masks && hgc_out->high_value_rewards && hgc_out->low_value_subgoal_steps &&
                   hgc_out->low_value_masks && hgc_out->low_value_rewards && hgc_out->masks && hgc_out->rewards,
               OGBX_EINVAL, "ogbx_gc_plan_set_batch: missing HGC scalar output");
  } else {
    OGBX_CHECK(masks && rewards, OGBX_EINVAL, "ogbx_gc_plan_set_batch: null masks / rewards");
  }
  PlanBatch b;
  const int max_sel = p->hgc ? kHgcSel - 1 : 3;
  for (int i = 0; i < num_cols; ++i) {
    OGBX_CHECK(cols[i].src_stride == 0 || cols[i].src_stride >= cols[i].row_bytes, OGBX_EINVAL,
               "ogbx_gc_plan_set_batch: src_stride below row_bytes");
    OGBX_CHECK(cols[i].src && cols[i].dst && cols[i].row_bytes > 0 && cols[i].select >= 0 &&
                   cols[i].select <= max_sel,
               OGBX_EINVAL, "ogbx_gc_plan_set_batch: bad column descriptor");
    b.cc.c[i] = cols[i];
  }
  b.ncols = num_cols;
  b.batch = batch;
  b.nb = num_batches;
  b.idxs = idxs_out;
  b.vg = value_goal_out;
  b.ag = actor_goal_out;
  b.masks = masks;
  b.rewards = rewards;
  if (hgc_out) b.hout = *hgc_out;
  b.flat4 = flat4_columns(b.cc, num_cols);
  b.small = num_cols <= kGcSmallCols;
  for (int i = 0; i < kGcSmallCols && i < num_cols; ++i) b.cs.c[i] = b.cc.c[i];
  b.set = true;
  std::lock_guard<std::mutex> guard(p->mu);
  p->slots[slot] = b;
  return OGBX_OK;
}

ogbx_status ogbx_gc_plan_sample(ogbx_gc_plan_t p, int32_t slot, uint64_t call_index, void* stream) {
  OGBX_CHECK(p, OGBX_EINVAL, "null plan");
  std::lock_guard<std::mutex> guard(p->mu);
  OGBX_CHECK(slot >= 0 && slot < OGBX_GC_PLAN_SLOTS && p->slots[slot].set, OGBX_EINVAL,
             "ogbx_gc_plan_sample: no batch in this slot");
  const PlanBatch& b = p->slots[slot];
  const int64_t total = b.batch * b.nb;
  hipStream_t s = (hipStream_t)stream;
  const uint32_t clo = (uint32_t)call_index, chi = (uint32_t)(call_index >> 32);
  if (!p->lookahead || total > kGcAheadMaxSamples) {
    p->key_valid = false;
    int64_t tile = total / 1024;  // as ogbx_gc_sample
    if (tile < 1) tile = 1;
    if (tile > kGcMaxTile) tile = kGcMaxTile;
    const int64_t blocks = (total + tile - 1) / tile;
    const bool f4 = tile <= 4 && b.flat4;
    if (p->hgc) {
      hipLaunchKernelGGL(hgc_sample_kernel<false>, dim3((uint32_t)blocks), dim3(256), 0, s, p->buf, p->cfg, p->hcfg,
                         b.cc, b.ncols, total, (int)tile, ogbx_hgc_draws{}, p->k0, p->k1, clo, chi, p->v_log_q,
                         p->a_log_q, p->l_log_q, b.hout, ogbx_hgc_draw_record{}, f4);
      OGBX_LAUNCHED("hgc_sample_kernel");
    } else {
      hipLaunchKernelGGL(gc_sample_kernel<false>, dim3((uint32_t)blocks), dim3(256), 0, s, p->buf, p->cfg, b.cc,
                         b.ncols, total, (int)tile, ogbx_gc_draws{}, p->k0, p->k1, clo, chi, p->v_log_q, p->a_log_q,
                         b.idxs, b.vg, b.ag, b.masks, b.rewards, ogbx_gc_draw_record{}, f4);
      OGBX_LAUNCHED("gc_sample_kernel");
    }
    return OGBX_OK;
  }
  // this stream's buffer pair (allocated on its first call; with every pair
  // taken, the call runs without look-ahead: nothing stored, nothing read)
  int pi = -1;
  for (int i = 0; i < p->npairs; ++i)
    if (p->pairs[i].stream == stream) pi = i;
  if (pi < 0 && p->npairs < kPlanStreams) {
    const size_t words = (size_t)kGcAheadMaxSamples * (p->hgc ? kHgcAheadWords : kGcAheadWords);
    int cur = 0;
    OGBX_HIP(hipGetDevice(&cur));
    if (cur != p->device) OGBX_HIP(hipSetDevice(p->device));
    PlanPair pr;
    pr.stream = stream;
    hipError_t e0 = hipMalloc(&pr.buf[0], words * sizeof(int64_t));
    hipError_t e1 = e0 == hipSuccess ? hipMalloc(&pr.buf[1], words * sizeof(int64_t)) : e0;
    if (cur != p->device) (void)hipSetDevice(cur);
    if (e0 != hipSuccess || e1 != hipSuccess) {
      if (pr.buf[0]) (void)hipFree(pr.buf[0]);
      return hip_fail(e0 != hipSuccess ? e0 : e1, "hipMalloc (look-ahead buffers)");
    }
    pi = p->npairs++;
    p->pairs[pi] = pr;
  }
  const int64_t* in = nullptr;
  int64_t* out = nullptr;
  int which = 0;
  if (pi >= 0) {
    const bool hit = p->key_valid && p->key_pair == pi && p->key_total == total && p->key_call == call_index;
    if (hit) {
      in = p->pairs[pi].buf[p->key_which];
      which = 1 - p->key_which;
      ++p->hits;
    }
    out = p->pairs[pi].buf[which];
  }
  const uint64_t next = call_index + 1;
  auto launch = [&](const auto& cols) {
    using C = std::decay_t<decltype(cols)>;
    if (p->hgc) {
      const auto kern = in ? hgc_ahead_kernel<true, C> : hgc_ahead_kernel<false, C>;
      hipLaunchKernelGGL(kern, dim3((uint32_t)total), dim3(256), 0, s, p->buf, p->cfg, p->hcfg, cols, b.ncols, p->k0,
                         p->k1, clo, chi, (uint32_t)next, (uint32_t)(next >> 32), p->v_log_q, p->a_log_q, p->l_log_q,
                         in, out, b.hout, b.flat4);
    } else {
      const auto kern = in ? gc_ahead_kernel<true, C> : gc_ahead_kernel<false, C>;
      hipLaunchKernelGGL(kern, dim3((uint32_t)total), dim3(256), 0, s, p->buf, p->cfg, cols, b.ncols, p->k0, p->k1,
                         clo, chi, (uint32_t)next, (uint32_t)(next >> 32), p->v_log_q, p->a_log_q, in, out, b.idxs,
                         b.vg, b.ag, b.masks, b.rewards, b.flat4);
    }
  };
  if (b.small)
    launch(b.cs);
  else
    launch(b.cc);
  OGBX_LAUNCHED(p->hgc ? "hgc_ahead_kernel" : "gc_ahead_kernel");
  p->key_valid = pi >= 0;
  p->key_pair = pi;
  p->key_which = which;
  p->key_total = total;
  p->key_call = next;
  return OGBX_OK;
}

int64_t ogbx_gc_plan_hits(ogbx_gc_plan_t p) {
  if (!p) return -1;
  std::lock_guard<std::mutex> guard(p->mu);
  return p->hits;
}

ogbx_status ogbx_gc_plan_destroy(ogbx_gc_plan_t p) {
  if (!p) return OGBX_OK;
  hipError_t err = hipSuccess;
  for (int i = 0; i < p->npairs; ++i)
    for (int k = 0; k < 2; ++k)
      if (p->pairs[i].buf[k]) {
        const hipError_t e = hipFree(p->pairs[i].buf[k]);  // waits for in-flight launches
        if (err == hipSuccess) err = e;
      }
  delete p;
  if (err != hipSuccess) return hip_fail(err, "hipFree (look-ahead buffers)");
  return OGBX_OK;
}

}  // extern "C"

extern "C" {

ogbx_status ogbx_gc_traj_end(const int64_t* terminal_locs, int64_t num_terminals,
                             int64_t num_rows, int64_t* traj_end, void* stream) {
  OGBX_CHECK(terminal_locs && traj_end && num_terminals > 0 && num_rows > 0, OGBX_EINVAL,
             "ogbx_gc_traj_end: bad argument");
  hipLaunchKernelGGL(traj_end_kernel, dim3((uint32_t)((num_rows + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, terminal_locs, num_terminals, num_rows, traj_end);
  OGBX_LAUNCHED("traj_end_kernel");
  return OGBX_OK;
}

ogbx_status ogbx_nonzero_f32(const float* x, int64_t n, int64_t* out, int64_t* count,
                             void* stream) {
  OGBX_CHECK(x && out && count && n >= 0, OGBX_EINVAL, "ogbx_nonzero_f32: bad argument");
  hipStream_t s = (hipStream_t)stream;
  hipcub::CountingInputIterator<int64_t> it(0);
  PositiveF32 pred{x};
  size_t tmp_bytes = 0;
  OGBX_HIP(hipcub::DeviceSelect::If(nullptr, tmp_bytes, it, out, count, n, pred, s));
  void* tmp = nullptr;
  OGBX_HIP(hipMallocAsync(&tmp, tmp_bytes > 0 ? tmp_bytes : 1, s));
  hipError_t e = hipcub::DeviceSelect::If(tmp, tmp_bytes, it, out, count, n, pred, s);
  hipError_t e2 = hipFreeAsync(tmp, s);
  if (e != hipSuccess) return hip_fail(e, "hipcub::DeviceSelect::If");
  if (e2 != hipSuccess) return hip_fail(e2, "hipFreeAsync");
  return OGBX_OK;
}

}  // extern "C"
