// Shared device/host helpers for the grace_amd HIP codec library (gfx950 / CDNA4 only).
//
// Conventions used by every kernel in this library:
//   * wave64: ballots are 64-bit, lane prefix counts use v_mbcnt_{lo,hi};
//   * streaming kernels move 16 B per lane (float4) and grid-stride over the bucket;
//   * the library is compiled with -ffp-contract=off so every f32 add/mul rounds exactly like
//     the reference's separate torch ops (no silent FMA contraction);
//   * every launch is stream-ordered on the caller's stream; nothing allocates or syncs.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/grace_hip.h"

namespace grace {

constexpr int kWave = 64;

// aux operand of the raw buffer load / store builtins for the sc1 cache policy: 16-B write-through
// stores (one fabric write per 16 B instead of one per dword) and loads that bypass the
// (non-coherent) local L2 -- the agent-scope hand-offs of DESIGN.md §4
constexpr int kSc1 = 16;

// ------------------------------------------------------------------------------------------------
// host-side error plumbing
void set_error(const char* where, hipError_t e);
void set_error_msg(const char* msg);

#define GRACE_CHECK_LAUNCH(name)                              \
  do {                                                        \
    hipError_t _e = hipGetLastError();                        \
    if (_e != hipSuccess) {                                   \
      ::grace::set_error(name, _e);                           \
      return GRACE_ERR_HIP;                                   \
    }                                                         \
  } while (0)

#define GRACE_REQUIRE(cond, msg)                              \
  do {                                                        \
    if (!(cond)) {                                            \
      ::grace::set_error_msg(msg);                            \
      return GRACE_ERR_ARG;                                   \
    }                                                         \
  } while (0)

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Grid size for a streaming kernel: enough blocks to fill 256 CUs several times over, capped so
// each thread grid-strides over a few 16-B vectors (cdna_hip_programming.md Guideline 11).
inline unsigned stream_grid(int64_t n_vec, int block, int64_t cap = 2048) {
  int64_t g = (n_vec + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

// ------------------------------------------------------------------------------------------------
// device helpers
__device__ __forceinline__ uint32_t f2u(float x) { return __float_as_uint(x); }
__device__ __forceinline__ float u2f(uint32_t x) { return __uint_as_float(x); }

// Ordering key of |x|: monotone in |x|; NaN above +inf; -0 == +0.
__device__ __forceinline__ uint32_t abs_key(float x) { return f2u(x) & 0x7FFFFFFFu; }

// Lane's position among the set lanes of a 64-bit ballot mask (v_mbcnt_lo/hi).
__device__ __forceinline__ uint32_t lane_rank(uint64_t mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

__device__ __forceinline__ int lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

// Counter-based generator for the "device" randomness mode: a 64-bit mix of (seed, stream, i).
// Not bit-compatible with torch's generators; parity tests inject the reference's streams.
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}
// 32 random bits for element i of the stream keyed by seed.  mix64(seed) is loop-invariant, so a
// grid-stride loop pays three 32-bit multiplies per element (64-bit multiplies are 4x dearer on
// CDNA and would make the streaming codecs ALU-bound).
__device__ __forceinline__ uint32_t rand32(uint64_t seed, uint64_t i) {
  const uint64_t k = mix64(seed);
  const uint32_t h = ((uint32_t)i * 0x9E3779B1u) ^ (uint32_t)k ^ ((uint32_t)(i >> 32) * 0x7FEB352Du);
  return fmix32(h + (uint32_t)(k >> 32));
}
__device__ __forceinline__ float uniform01(uint64_t seed, uint64_t i) {
  // 24 random bits -> [0, 1)
  return (float)(rand32(seed, i) >> 8) * (1.0f / 16777216.0f);
}
// Four uniforms for the quad starting at element i: one rand32 hash (its 32-bit multiplies are
// quarter-rate on CDNA) seeds three xorshift32 steps (shifts and xors only).  A pure function of
// (seed, i) like uniform01, at about a third of its VALU cost per element.
__device__ __forceinline__ void uniform01x4(uint64_t seed, uint64_t i, float (&u)[4]) {
  uint32_t h = rand32(seed, i);
  u[0] = (float)(h >> 8) * (1.0f / 16777216.0f);
  h = h ? h : 0x9E3779B9u;   // xorshift32 has no zero state
#pragma unroll
  for (int j = 1; j < 4; ++j) {
    h ^= h << 13;
    h ^= h >> 17;
    h ^= h << 5;
    u[j] = (float)(h >> 8) * (1.0f / 16777216.0f);
  }
}

// 64-bit value moved across lanes by one DPP pattern (two 32-bit DPP movs)
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const uint64_t b = (uint64_t)__double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)b, CTRL, 0xF, 0xF, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(b >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
// Sum over each 16-lane DPP row by symmetric butterflies (quad xor 1, quad xor 2, half-mirror,
// mirror): every step adds the same two operands in every lane, so all 16 lanes hold the
// bit-identical total -- no LDS traffic, no lgkm waits.
__device__ __forceinline__ double row16_sum(double v) {
  v += dpp_f64<0xB1>(v);    // quad_perm [1,0,3,2]
  v += dpp_f64<0x4E>(v);    // quad_perm [2,3,0,1]
  v += dpp_f64<0x141>(v);   // row_half_mirror
  v += dpp_f64<0x140>(v);   // row_mirror
  return v;
}

// Wave-level reductions (64 lanes) via cross-lane shuffles.
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// Reduction over the 32 lanes of each half-wave (xor offsets < 32 never cross halves).
template <typename T>
__device__ __forceinline__ T half_sum(T v) {
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

}  // namespace grace
