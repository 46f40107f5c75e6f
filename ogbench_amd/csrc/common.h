// common.h -- shared internals of libogbx: status/error plumbing and the
// Philox4x32-10 counter-based generator used for every on-device draw.
//
// Written for gfx950 only (wave64, CDNA4).  No CUDA spellings, no dual paths.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/ogbx.h"

namespace ogbx {

// ---------------------------------------------------------------- errors
void set_error(const std::string& msg);
ogbx_status fail(ogbx_status code, const std::string& msg);
ogbx_status hip_fail(hipError_t e, const char* what);
// Verify that `device` exists and is a gfx950 part; make it current.
ogbx_status use_device(int32_t device);

#define OGBX_HIP(call)                                       \
  do {                                                       \
    hipError_t _e = (call);                                  \
    if (_e != hipSuccess) return ::ogbx::hip_fail(_e, #call); \
  } while (0)

#define OGBX_CHECK(cond, code, msg)              \
  do {                                           \
    if (!(cond)) return ::ogbx::fail(code, msg); \
  } while (0)

// Launch-error check after a kernel launch (hipGetLastError is cheap and
// capture-safe).
#define OGBX_LAUNCHED(what)                                   \
  do {                                                        \
    hipError_t _e = hipGetLastError();                        \
    if (_e != hipSuccess) return ::ogbx::hip_fail(_e, what);  \
  } while (0)

// ---------------------------------------------------------------- Philox
// Philox4x32-10 (Salmon et al., SC'11).  Counter = (c0,c1,c2,c3), key = (k0,k1).
// Streams used by libogbx (documented in DESIGN.md):
//   key  = (lo32(seed), hi32(seed) ^ stream_tag)
//   ctr  = (object index, episode/call counter, draw slot, 0)
struct u32x4 {
  uint32_t x, y, z, w;
};

__host__ __device__ inline uint32_t mulhi32(uint32_t a, uint32_t b) {
  return (uint32_t)(((uint64_t)a * (uint64_t)b) >> 32);
}

__host__ __device__ inline u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0 = mulhi32(M0, c.x), lo0 = M0 * c.x;
    uint32_t hi1 = mulhi32(M1, c.z), lo1 = M1 * c.z;
    u32x4 n;
    n.x = hi1 ^ c.y ^ k0;
    n.y = lo1;
    n.z = hi0 ^ c.w ^ k1;
    n.w = lo0;
    c = n;
    k0 += W0;
    k1 += W1;
  }
  return c;
}

// The same Philox4x32-10 with both halves of a round's 32x32 -> 64 product
// from one v_mad_u64_u32 (LLVM emits a v_mul_hi_u32 + v_mul_lo_u32 pair):
// +6 % throughput with identical words (scripts/micro/philox_mul.hip).  For
// throughput-bound callers (every lane drawing, e.g. powder rand fields) with
// wave-uniform keys (k0, k1 go in scalar operands);
// latency-bound chains keep the pair, whose halves issue independently.
__device__ __forceinline__ u32x4 philox4x32_10_wide(u32x4 c, uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint64_t p0, p1, c0, c1;
    asm("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(p0), "=s"(c0) : "v"(M0), "v"(c.x));
    asm("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(p1), "=s"(c1) : "v"(M1), "v"(c.z));
    u32x4 n;
    // hi ^ c ^ key as one v_bitop3_b32 (truth table 0x96: S0 ^ S1 ^ S2; gfx950
    // has no v_xor3_b32) with the key as its scalar operand (LLVM
    // keeps two v_xor_b32 here): callers pass wave-uniform keys
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(n.x) : "v"((uint32_t)(p1 >> 32)), "v"(c.y), "s"(k0));
    n.y = (uint32_t)p1;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(n.z) : "v"((uint32_t)(p0 >> 32)), "v"(c.w), "s"(k1));
    n.w = (uint32_t)p0;
    c = n;
    k0 += W0;
    k1 += W1;
  }
  return c;
}

// 53-bit uniform double in [0, 1) from two 32-bit words.
__host__ __device__ inline double u01_from(uint32_t hi, uint32_t lo) {
  uint64_t v = ((uint64_t)hi << 32) | (uint64_t)lo;
  return (double)(v >> 11) * 0x1.0p-53;
}

// 24-bit uniform float in [0, 1).
__host__ __device__ inline float u01f_from(uint32_t w) { return (float)(w >> 8) * 0x1.0p-24f; }

// Unbiased-enough integer in [0, n) via 64-bit multiply-shift (n < 2^32).
__host__ __device__ inline uint32_t bounded_u32(uint32_t w, uint32_t n) {
  return (uint32_t)(((uint64_t)w * (uint64_t)n) >> 32);
}

enum StreamTag : uint32_t {
  kTagMazeReset = 0x4D5A0001u,
  kTagMazeTeleport = 0x4D5A0002u,
  kTagMazeExpert = 0x4D5A0003u,
  kTagMazeGoal = 0x4D5A0004u,
  kTagPowderReset = 0x50570001u,
  kTagPowderAction = 0x50570002u,
  kTagPowderRand = 0x50570003u,
  kTagGcSample = 0x47430001u,
  kTagHgcSample = 0x47430002u,
};

inline void seed_key(uint64_t seed, uint32_t tag, uint32_t* k0, uint32_t* k1) {
  *k0 = (uint32_t)(seed & 0xffffffffu);
  *k1 = (uint32_t)(seed >> 32) ^ tag;
}

}  // namespace ogbx
