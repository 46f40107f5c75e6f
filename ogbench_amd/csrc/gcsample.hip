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

#include "common.h"

namespace ogbx {

constexpr int kGcMaxTile = 64;
constexpr int kGcMaxCols = 32;

struct GcColumns {
  ogbx_gc_column c[kGcMaxCols];
};

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
  int64_t q = (int64_t)((double)pick / (double)buf.period_picks);
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

template <typename T>
__device__ inline void copy_rows(const ogbx_gc_column& col, const int64_t* sel, int64_t base,
                                 int tile) {
  const int64_t units = col.row_bytes / (int64_t)sizeof(T);
  const int64_t pitch = src_pitch<T>(col);
  const T* __restrict__ src = (const T*)col.src;
  T* __restrict__ dst = (T*)col.dst;
  const int64_t total = units * tile;
  const int step = blockDim.x;
  int64_t b = threadIdx.x / units, k = threadIdx.x % units;
  const int64_t sb = step / units, sk = step % units;
  for (int64_t f = threadIdx.x; f < total; f += step) {
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
template <int kSel>
__device__ inline void copy_tile(const GcColumns& cols, int num_cols, const int64_t (*sel)[kGcMaxTile], int64_t base,
                                 int n_here, bool flat4) {
  if (flat4) {
    constexpr int kJ = 8, kSlots = 2;
    const int nw = (int)(blockDim.x >> 6);
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
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
          if (d[u][q]) *d[u][q] = v[u][q];
    }
    return;
  }
  for (int c = 0; c < num_cols; ++c) {
    const ogbx_gc_column& col = cols.c[c];
    const int64_t* srow = sel[col.select];
    const uintptr_t align = (uintptr_t)col.src | (uintptr_t)col.dst | (uintptr_t)col.src_stride;
    if (col.row_bytes % 16 == 0 && align % 16 == 0)
      copy_rows<uint4>(col, srow, base, n_here);
    else if (col.row_bytes % 8 == 0 && align % 8 == 0)
      copy_rows<uint2>(col, srow, base, n_here);
    else if (col.row_bytes % 4 == 0 && align % 4 == 0)
      copy_rows<uint32_t>(col, srow, base, n_here);
    else
      copy_rows<uint8_t>(col, srow, base, n_here);
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
