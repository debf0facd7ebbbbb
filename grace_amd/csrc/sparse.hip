// Random-k and threshold sparsifiers for CDNA4.
//
// Random-k (grace_dl/dist/compressor/randomk.py:6-41): k indices drawn WITH replacement from
// [0, numel) from a generator seeded by sum(bytes(name)) + global_step (identical on every rank),
// payload = values at those indices.  Device mode: a counter-based hash of (seed, j); torch_cpu
// mode (exact parity) passes the reference generator's indices in.
//
// Threshold (grace_dl/dist/compressor/threshold.py:6-27): idx = where(|x| >= min(thr, max(x)))
// in ascending index order (bit-exact with torch.where).  Three short launches: per-chunk
// (signed max, count at thr) -> one workgroup derives the bound and the chunk offsets (and flags
// a recount if max(x) < thr) -> ordered compaction per chunk with a block scan.
#include <math.h>

#include "common.h"

namespace grace {

constexpr int kSBlock = 256;
constexpr int kThrChunk = 16384;

__global__ __launch_bounds__(kSBlock) void randomk_idx_kernel(uint64_t seed, int64_t numel, int64_t k,
                                                             int64_t* __restrict__ idx) {
  for (int64_t j = (int64_t)blockIdx.x * kSBlock + threadIdx.x; j < k; j += (int64_t)gridDim.x * kSBlock) {
    const uint64_t h = mix64(seed * 0x9E3779B97F4A7C15ull ^ mix64((uint64_t)j + 0x632BE59BD9B4E019ull));
    // unbiased enough for numel < 2^31: 64-bit product high word
    idx[j] = (int64_t)__umul64hi(h, (uint64_t)numel);
  }
}

__global__ __launch_bounds__(kSBlock) void gather_kernel(const float* __restrict__ x, const int64_t* __restrict__ idx,
                                                        int64_t k, float* __restrict__ vals) {
  for (int64_t j = (int64_t)blockIdx.x * kSBlock + threadIdx.x; j < k; j += (int64_t)gridDim.x * kSBlock)
    vals[j] = x[idx[j]];
}

// World-1 Allgather(RandomK, ResidualMemory).step (randomk.py:24-41, residual.py:10-20,
// allgather.py:40-45) in three launches instead of compensate + gather + two decodes + subtract +
// sum: (1) one streaming pass t = beta r + gamma g -> r' = t, out = 0 (16 B per element); (2) the
// payload gather vals = t[idx]; (3) the scatter out[idx] = 0 + vals, r'[idx] = vals - vals.  The
// gather completes before the scatter (kernel boundary), so duplicate indices (drawn with
// replacement) read t, never a zeroed entry -- as zeros.scatter_ / t - decompress do.
constexpr int kRQ = 4;   // quads per lane per round, all loads in flight first
template <bool HAS_RES>
__global__ __launch_bounds__(kSBlock) void randomk_pass_kernel(const float* __restrict__ g, float* __restrict__ r,
                                                              float beta, float gamma, int64_t n,
                                                              float* __restrict__ out) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  const int64_t stride = (int64_t)gridDim.x * kSBlock;
  // out may be null (the sharded step's replicated mode decodes the gathered payload instead)
  const bool vec = ((reinterpret_cast<uintptr_t>(g) | reinterpret_cast<uintptr_t>(r) |
                     reinterpret_cast<uintptr_t>(out)) & 15u) == 0;
  const int64_t nq = vec ? n >> 2 : 0;
  const f4 z = {0.f, 0.f, 0.f, 0.f};
  for (int64_t q0 = (int64_t)blockIdx.x * kSBlock + threadIdx.x; q0 < nq; q0 += stride * kRQ) {
    f4 gv[kRQ], rv[kRQ];
#pragma unroll
    for (int u = 0; u < kRQ; ++u) {
      const int64_t q = q0 + u * stride < nq ? q0 + u * stride : q0;
      gv[u] = __builtin_nontemporal_load(reinterpret_cast<const f4*>(g) + q);
      if (HAS_RES) rv[u] = __builtin_nontemporal_load(reinterpret_cast<const f4*>(r) + q);
    }
#pragma unroll
    for (int u = 0; u < kRQ; ++u) {
      if (q0 + u * stride >= nq) break;
      f4 t = gv[u];
      if (HAS_RES) t = f4{beta * rv[u].x + gamma * gv[u].x, beta * rv[u].y + gamma * gv[u].y,
                          beta * rv[u].z + gamma * gv[u].z, beta * rv[u].w + gamma * gv[u].w};
      __builtin_nontemporal_store(t, reinterpret_cast<f4*>(r) + q0 + u * stride);
      if (out) __builtin_nontemporal_store(z, reinterpret_cast<f4*>(out) + q0 + u * stride);
    }
  }
  for (int64_t i = nq * 4 + (int64_t)blockIdx.x * kSBlock + threadIdx.x; i < n; i += stride) {
    r[i] = HAS_RES ? beta * r[i] + gamma * g[i] : g[i];
    if (out) out[i] = 0.f;
  }
}

// Sharded random-k (grace_amd/dist/sharded_randomk.py): this rank holds the bucket's elements
// [lo, lo + m); idx are the k GLOBAL indices every rank draws alike.  The gather takes t for the
// drawn indices this rank holds and +0 for the others (every index has exactly one owner, so the
// ranks' payloads sum to the whole bucket's payload, -0 excepted, which the step's 0 + d makes +0
// anyway); the scatter zeroes r' at this rank's drawn positions and writes 0 + t to its dense slice.
__global__ __launch_bounds__(kSBlock) void randomk_shard_gather_kernel(const float* __restrict__ t,
                                                                      const int64_t* __restrict__ idx, int64_t k,
                                                                      int64_t lo, int64_t m, float* __restrict__ vals) {
  for (int64_t j = (int64_t)blockIdx.x * kSBlock + threadIdx.x; j < k; j += (int64_t)gridDim.x * kSBlock) {
    const int64_t i = idx[j] - lo;
    vals[j] = (i >= 0 && i < m) ? t[i] : 0.f;
  }
}
__global__ __launch_bounds__(kSBlock) void randomk_shard_scatter_kernel(const int64_t* __restrict__ idx,
                                                                       const float* __restrict__ vals, int64_t k,
                                                                       int64_t lo, int64_t m, float* __restrict__ r,
                                                                       float* __restrict__ out) {
  for (int64_t j = (int64_t)blockIdx.x * kSBlock + threadIdx.x; j < k; j += (int64_t)gridDim.x * kSBlock) {
    const int64_t i = idx[j] - lo;
    if (i < 0 || i >= m) continue;
    const float v = vals[j];
    if (out) out[i] = 0.f + v;
    if (r) r[i] = v - v;
  }
}

// World-1 Allgather(RandomK, ResidualMemory).step in ONE streaming pass (the dense variant; no
// payload is materialised: at world 1 the step's result is out alone).  The drawn indices are
// grouped by 8192-element chunk first (payload.hip's counting sort: u16 offsets + chunk ends);
// workgroup c marks its chunk's selected offsets in an LDS bitmap (duplicates set the same bit,
// as zeros.scatter_ writes the same value twice), then streams the chunk once:
// selected -> out = 0 + t, r' = t - t; else out = 0, r' = t.  16 B per element and no random
// gathers / scatters (which move whole lines for 4-B values).
template <typename IdxT>
hipError_t group_by_chunk(const float* vals, const IdxT* idx, int64_t k, int64_t nchunks, float* vals_out,
                          uint16_t* off_out, uint32_t* ends_out, uint32_t* ticket, hipStream_t s);
size_t group_scratch_bytes(int64_t nchunks);
constexpr int kRkChunkLog = 13;                  // = payload.hip kPChunkLog
constexpr int kRkChunk = 1 << kRkChunkLog;
constexpr int kRkQ = kRkChunk / (4 * kSBlock);   // quads per thread per array
// SPARSE (recycled output): `out` holds the previous step's result of this name, non-zero only at
// the previous grouping (poffs / pends): those positions not drawn again are cleared, and only the
// drawn ones are written (out is not streamed; r' still is)
template <bool HAS_RES, bool SPARSE>
__global__ __launch_bounds__(kSBlock) void randomk_dense_pass_kernel(const float* __restrict__ g, float* __restrict__ r,
                                                                    float beta, float gamma, int64_t n,
                                                                    const uint16_t* __restrict__ offs,
                                                                    const uint32_t* __restrict__ ends,
                                                                    float* __restrict__ out,
                                                                    const uint16_t* __restrict__ poffs,
                                                                    const uint32_t* __restrict__ pends) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  __shared__ uint32_t bm[kRkChunk / 32];
  const int64_t c = blockIdx.x;
  const int64_t c0 = c << kRkChunkLog, c1 = min(c0 + (int64_t)kRkChunk, n);
  const int t = threadIdx.x;
  const bool vec = ((reinterpret_cast<uintptr_t>(g) | reinterpret_cast<uintptr_t>(r) |
                     reinterpret_cast<uintptr_t>(out)) & 15u) == 0 && c1 - c0 == kRkChunk;
  f4 gv[kRkQ], rv[kRkQ];
  if (vec) {
#pragma unroll
    for (int u = 0; u < kRkQ; ++u) {
      const int64_t e = c0 + 4 * ((int64_t)u * kSBlock + t);
      gv[u] = __builtin_nontemporal_load(reinterpret_cast<const f4*>(g + e));
      if (HAS_RES) rv[u] = __builtin_nontemporal_load(reinterpret_cast<const f4*>(r + e));
    }
  }
  for (int w = t; w < kRkChunk / 32; w += kSBlock) bm[w] = 0u;
  __syncthreads();
  const uint32_t e0 = c > 0 ? ends[c - 1] : 0u, e1 = ends[c];
  for (uint32_t j = e0 + t; j < e1; j += kSBlock) {
    const uint32_t o = offs[j];
    atomicOr(&bm[o >> 5], 1u << (o & 31));
  }
  __syncthreads();
  if constexpr (SPARSE) {   // the previous result's non-zeros in this chunk, unless drawn again
    const uint32_t p0 = c > 0 ? pends[c - 1] : 0u, p1 = pends[c];
    for (uint32_t j = p0 + t; j < p1; j += kSBlock) {
      const uint32_t o = poffs[j];
      if (!((bm[o >> 5] >> (o & 31)) & 1u)) out[c0 + o] = 0.f;
    }
  }
  auto one = [&](float tv, int64_t i, float& o, float& rr) {
    const int64_t l = i - c0;
    const bool sel = (bm[l >> 5] >> (l & 31)) & 1u;
    o = sel ? 0.f + tv : 0.f;
    rr = sel ? tv - tv : tv;
  };
  if (vec) {
#pragma unroll
    for (int u = 0; u < kRkQ; ++u) {
      const int64_t e = c0 + 4 * ((int64_t)u * kSBlock + t);
      f4 tt = gv[u];
      if (HAS_RES) tt = f4{beta * rv[u].x + gamma * gv[u].x, beta * rv[u].y + gamma * gv[u].y,
                           beta * rv[u].z + gamma * gv[u].z, beta * rv[u].w + gamma * gv[u].w};
      f4 o, rr;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float a, b;
        one(tt[j], e + j, a, b);
        o[j] = a;
        rr[j] = b;
        if constexpr (SPARSE) {
          const int64_t l = e + j - c0;
          if ((bm[l >> 5] >> (l & 31)) & 1u) out[e + j] = a;
        }
      }
      if constexpr (!SPARSE) __builtin_nontemporal_store(o, reinterpret_cast<f4*>(out + e));
      __builtin_nontemporal_store(rr, reinterpret_cast<f4*>(r + e));
    }
  } else {
    for (int64_t i = c0 + t; i < c1; i += kSBlock) {
      const float tv = HAS_RES ? beta * r[i] + gamma * g[i] : g[i];
      float a, b;
      one(tv, i, a, b);
      const int64_t l = i - c0;
      if (!SPARSE || ((bm[l >> 5] >> (l & 31)) & 1u)) out[i] = a;
      r[i] = b;
    }
  }
}

__global__ __launch_bounds__(kSBlock) void randomk_scatter_kernel(const int64_t* __restrict__ idx,
                                                                 const float* __restrict__ vals, int64_t k,
                                                                 float* __restrict__ r, float* __restrict__ out) {
  for (int64_t j = (int64_t)blockIdx.x * kSBlock + threadIdx.x; j < k; j += (int64_t)gridDim.x * kSBlock) {
    const int64_t i = idx[j];
    const float v = vals[j];
    out[i] = 0.f + v;
    r[i] = v - v;
  }
}

// Random-k without replacement (grace_dl/torch/compressor/randomk.py:10, randperm(numel)[:k]):
// j -> pi(j) for j < k, pi a keyed pseudorandom permutation of [0, numel): a balanced 4-round
// Feistel network on 2h bits (2^(2h) >= numel, so at most 4x numel) restricted to [0, numel) by
// cycle walking, which keeps it a bijection.  Distinct j give distinct indices with no sort and no
// shared state; every rank derives the same indices from the same seed.
__device__ __forceinline__ uint64_t feistel(uint64_t x, int h, uint64_t key) {
  const uint64_t mask = (1ull << h) - 1ull;
  uint64_t l = x >> h, r = x & mask;
#pragma unroll
  for (int round = 0; round < 4; ++round) {
    const uint64_t f = mix64(r ^ mix64(key + 0x9E3779B97F4A7C15ull * (uint64_t)(round + 1))) & mask;
    const uint64_t t = l ^ f;
    l = r;
    r = t;
  }
  return (l << h) | r;
}

__global__ __launch_bounds__(kSBlock) void randperm_idx_kernel(uint64_t seed, int64_t numel, int64_t k, int h,
                                                              int64_t* __restrict__ idx) {
  const uint64_t key = mix64(seed ^ 0xD1B54A32D192ED03ull);
  for (int64_t j = (int64_t)blockIdx.x * kSBlock + threadIdx.x; j < k; j += (int64_t)gridDim.x * kSBlock) {
    uint64_t y = feistel((uint64_t)j, h, key);
    while (y >= (uint64_t)numel) y = feistel(y, h, key);   // cycle walk: terminates (finite cycle through j)
    idx[j] = (int64_t)y;
  }
}

__global__ __launch_bounds__(kSBlock) void widen_i32_kernel(const int32_t* __restrict__ src, int64_t n,
                                                           int64_t* __restrict__ dst) {
  for (int64_t j = (int64_t)blockIdx.x * kSBlock + threadIdx.x; j < n; j += (int64_t)gridDim.x * kSBlock)
    dst[j] = (int64_t)src[j];
}

// ------------------------------------------------------------------------------------------------
// threshold
struct ThrPart { float mx; uint32_t nan; uint32_t cnt; uint32_t pad; };

template <int BLOCK>
__device__ __forceinline__ uint32_t blk_excl_scan(uint32_t v, uint32_t* s_w, uint32_t* total) {
  constexpr int NW = BLOCK / kWave;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(inc, o, 64);
    if (lane >= o) inc += t;
  }
  if (lane == 63) s_w[w] = inc;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t acc = 0;
    for (int i = 0; i < NW; ++i) { const uint32_t t = s_w[i]; s_w[i] = acc; acc += t; }
    s_w[NW] = acc;
  }
  __syncthreads();
  const uint32_t r = s_w[w] + inc - v;
  if (total) *total = s_w[NW];
  __syncthreads();
  return r;
}

// pass 1: per chunk signed max (NaN flagged) and count(|x| >= bound)
__global__ __launch_bounds__(kSBlock) void thr_stats_kernel(const float* __restrict__ x, int64_t n, float bound,
                                                           ThrPart* __restrict__ part) {
  const int64_t base = (int64_t)blockIdx.x * kThrChunk;
  const int64_t end = min(base + (int64_t)kThrChunk, n);
  float mx = -INFINITY;
  uint32_t nan = 0, cnt = 0;
  for (int64_t i = base + threadIdx.x; i < end; i += kSBlock) {
    const float v = x[i];
    if (v != v) nan = 1; else mx = fmaxf(mx, v);
    cnt += fabsf(v) >= bound;
  }
  __shared__ float sm[kSBlock / kWave];
  __shared__ uint32_t sn[kSBlock / kWave], sc[kSBlock / kWave];
  mx = wave_max(mx);
  cnt = wave_sum(cnt);
  nan = __ballot(nan != 0) != 0;
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { sm[w] = mx; sn[w] = nan; sc[w] = cnt; }
  __syncthreads();
  if (threadIdx.x == 0) {
    ThrPart p{-INFINITY, 0u, 0u, 0u};
    for (int j = 0; j < kSBlock / kWave; ++j) { p.mx = fmaxf(p.mx, sm[j]); p.nan |= sn[j]; p.cnt += sc[j]; }
    part[blockIdx.x] = p;
  }
}

// World-1 Allgather(Threshold, Residual|None).step without a payload (threshold.py:12-27,
// residual.py:10-20, allgather.py:40-45): out = (0 + decompress) / 1 and, with memory,
// r' = t - decompress, where the selection bound is min(thr, max t) (signed max; a NaN max keeps
// thr).  Any tensor with an element >= thr has bound = thr, so ONE streaming pass selects at thr
// speculatively (16 B per element with memory, 8 without) while it reduces max t; the workgroup
// that arrives last at the per-chunk partials decides whether the speculation held.  If it did not
// (max t < thr), a fix-up pass recomputes every element at bound = max t: t is recovered exactly
// from what the first pass wrote (|out| >= thr ? out : r'; without memory g is only read), and the
// fix-up kernel returns at once when nothing needs fixing.  Two launches and one read of the
// inputs in the common case, against three launches and t written then re-read before.
// MODE 0: no memory (t = g, read-only); 1: residual memory, first step (t = g); 2: residual memory.
typedef float f4s __attribute__((ext_vector_type(4)));
constexpr int kThrU = 4;   // quads per lane per round (all loads first)

__device__ __forceinline__ void thr_sel(float t, float bound, float& o, float& rr) {
  const bool sel = fabsf(t) >= bound;
  o = sel ? 0.f + t : 0.f;
  rr = sel ? t - t : t;
}

template <int MODE>
__global__ __launch_bounds__(kSBlock) void thr_spec_kernel(const float* __restrict__ g, float* __restrict__ r,
                                                          float beta, float gamma, int64_t n, float thr,
                                                          float* __restrict__ out, ThrPart* __restrict__ part,
                                                          uint32_t* __restrict__ meta) {
  __shared__ float sm[kSBlock / kWave];
  __shared__ uint32_t sn[kSBlock / kWave];
  __shared__ uint32_t s_last;
  const int64_t base = (int64_t)blockIdx.x * kThrChunk;
  const int64_t end = min(base + (int64_t)kThrChunk, n);
  const bool vec = ((reinterpret_cast<uintptr_t>(g) | reinterpret_cast<uintptr_t>(r) |
                     reinterpret_cast<uintptr_t>(out)) & 15u) == 0;
  const int64_t qe = vec ? base + ((end - base) & ~(int64_t)3) : base;   // [base, qe) in quads
  float mx = -INFINITY;
  uint32_t nan = 0;
  auto acc = [&](float v) { if (v != v) nan = 1; else mx = fmaxf(mx, v); };
  auto process = [&](int64_t e, const f4s& gq, const f4s& rq) {
    f4s t = gq;
    if (MODE == 2) t = f4s{beta * rq.x + gamma * gq.x, beta * rq.y + gamma * gq.y, beta * rq.z + gamma * gq.z,
                           beta * rq.w + gamma * gq.w};
    f4s o, rr;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc(t[j]);
      float oj, rj;
      thr_sel(t[j], thr, oj, rj);
      o[j] = oj;
      rr[j] = rj;
    }
    __builtin_nontemporal_store(o, reinterpret_cast<f4s*>(out + e));
    if (MODE != 0) __builtin_nontemporal_store(rr, reinterpret_cast<f4s*>(r + e));
  };
  if (qe - base == kThrChunk) {
    // a whole chunk: a compile-time number of rounds, the next round's loads issued before the
    // current round is processed (8 or 16 x 16 B in flight per lane, no guarded loads)
    constexpr int NR = kThrChunk / (4 * kSBlock * kThrU);
    const int64_t b0 = base + 4 * (int64_t)threadIdx.x;
    f4s gv[kThrU], rv[kThrU];
#pragma unroll
    for (int u = 0; u < kThrU; ++u) {
      gv[u] = __builtin_nontemporal_load(reinterpret_cast<const f4s*>(g + b0 + 4 * (int64_t)u * kSBlock));
      if (MODE == 2) rv[u] = __builtin_nontemporal_load(reinterpret_cast<const f4s*>(r + b0 + 4 * (int64_t)u * kSBlock));
    }
#pragma unroll
    for (int q = 0; q < NR; ++q) {
      const int64_t e0 = b0 + (int64_t)q * 4 * kSBlock * kThrU;
      f4s gn[kThrU], rn[kThrU];
      if (q + 1 < NR) {
#pragma unroll
        for (int u = 0; u < kThrU; ++u) {
          const int64_t e = e0 + 4 * (int64_t)kSBlock * kThrU + 4 * (int64_t)u * kSBlock;
          gn[u] = __builtin_nontemporal_load(reinterpret_cast<const f4s*>(g + e));
          if (MODE == 2) rn[u] = __builtin_nontemporal_load(reinterpret_cast<const f4s*>(r + e));
        }
      }
#pragma unroll
      for (int u = 0; u < kThrU; ++u) process(e0 + 4 * (int64_t)u * kSBlock, gv[u], rv[u]);
      if (q + 1 < NR) {
#pragma unroll
        for (int u = 0; u < kThrU; ++u) { gv[u] = gn[u]; rv[u] = rn[u]; }
      }
    }
  } else {
    for (int64_t e0 = base + 4 * (int64_t)threadIdx.x; e0 < qe; e0 += 4 * (int64_t)kSBlock * kThrU) {
      f4s gv[kThrU], rv[kThrU];
#pragma unroll
      for (int u = 0; u < kThrU; ++u) {
        const int64_t e = e0 + 4 * (int64_t)u * kSBlock < qe ? e0 + 4 * (int64_t)u * kSBlock : e0;
        gv[u] = __builtin_nontemporal_load(reinterpret_cast<const f4s*>(g + e));
        if (MODE == 2) rv[u] = __builtin_nontemporal_load(reinterpret_cast<const f4s*>(r + e));
      }
#pragma unroll
      for (int u = 0; u < kThrU; ++u) {
        const int64_t e = e0 + 4 * (int64_t)u * kSBlock;
        if (e >= qe) break;
        process(e, gv[u], rv[u]);
      }
    }
  }
  for (int64_t i = qe + threadIdx.x; i < end; i += kSBlock) {
    const float t = MODE == 2 ? beta * r[i] + gamma * g[i] : g[i];
    acc(t);
    float o, rr;
    thr_sel(t, thr, o, rr);
    out[i] = o;
    if (MODE != 0) r[i] = rr;
  }
  // the chunk's (max, NaN) partial, write-through; the last workgroup to arrive decides the bound
  mx = wave_max(mx);
  nan = __ballot(nan != 0) != 0;
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { sm[w] = mx; sn[w] = nan; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float pm = -INFINITY;
    uint32_t pn = 0;
    for (int j = 0; j < kSBlock / kWave; ++j) { pm = fmaxf(pm, sm[j]); pn |= sn[j]; }
    uint32_t* pw = reinterpret_cast<uint32_t*>(&part[blockIdx.x]);
    __hip_atomic_store(pw, __float_as_uint(pm), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(pw + 1, pn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    s_last = atomicAdd(&meta[4], 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (!s_last) return;
  // the grid runs several workgroups per CU, outside the guide's measured fence-free row (one per
  // CU): the last arriver keeps the agent-scope acquire before it reads the others' partials
  // (MI355X_MICROARCH.md, Consumer condition (4); one invalidate in one workgroup per launch)
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  mx = -INFINITY;
  nan = 0;
  for (int64_t j = threadIdx.x; j < (int64_t)gridDim.x; j += kSBlock) {
    const uint32_t* pj = reinterpret_cast<const uint32_t*>(&part[j]);
    const float m = __uint_as_float(__hip_atomic_load(pj, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    nan |= __hip_atomic_load(pj + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    mx = fmaxf(mx, m);
  }
  mx = wave_max(mx);
  nan = __ballot(nan != 0) != 0;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) { sm[w] = mx; sn[w] = nan; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float gm = -INFINITY;
    uint32_t gn = 0;
    for (int j = 0; j < kSBlock / kWave; ++j) { gm = fmaxf(gm, sm[j]); gn |= sn[j]; }
    // torch.max propagates NaN; Python min(thr, NaN) returns thr (NaN < thr is False)
    const bool use_max = !gn && gm < thr;
    meta[0] = __float_as_uint(use_max ? gm : thr);
    meta[2] = use_max ? 1u : 0u;   // the speculative pass selected at thr: fix up at max t
    meta[4] = 0u;                  // ticket left zeroed for the next call
  }
}

// fix-up pass: only when the speculative pass was wrong (max t < thr); returns at once otherwise
template <int MODE>
__global__ __launch_bounds__(kSBlock) void thr_fix_kernel(const float* __restrict__ g, float* __restrict__ r,
                                                         int64_t n, float thr, const uint32_t* __restrict__ meta,
                                                         float* __restrict__ out) {
  if (meta[2] == 0u) return;
  const float bound = __uint_as_float(meta[0]);
  for (int64_t i = (int64_t)blockIdx.x * kSBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kSBlock) {
    float t;
    if (MODE == 0) {
      t = g[i];
    } else {   // what the speculative pass wrote: out = 0 + t where it selected, r' = t elsewhere
      const float o = out[i], rv = r[i];
      t = fabsf(o) >= thr ? o : rv;
    }
    float o, rr;
    thr_sel(t, bound, o, rr);
    out[i] = o;
    if (MODE != 0) r[i] = rr;
  }
}

// pass 2 (one workgroup): global max -> bound = min(thr, max) with Python's min (NaN max -> thr);
// exclusive offsets of the chunk counts; meta = {bound bits, total, recount flag}
__global__ __launch_bounds__(1024) void thr_bound_kernel(ThrPart* __restrict__ part, int64_t nchunks, float thr,
                                                        uint32_t* __restrict__ offs, uint32_t* __restrict__ meta,
                                                        int final_pass, int fixed_bound) {
  __shared__ uint32_t s_w[1024 / kWave + 1];
  __shared__ float s_mx;
  __shared__ uint32_t s_nan;
  if (threadIdx.x == 0) { s_mx = -INFINITY; s_nan = 0; }
  __syncthreads();
  float mx = -INFINITY;
  uint32_t nan = 0;
  for (int64_t j = threadIdx.x; j < nchunks; j += 1024) { mx = fmaxf(mx, part[j].mx); nan |= part[j].nan; }
  mx = wave_max(mx);
  nan = __ballot(nan != 0) != 0;
  // reduce per-wave maxima through LDS
  __shared__ float s_wm[1024 / kWave];
  __shared__ uint32_t s_wn[1024 / kWave];
  if ((threadIdx.x & 63) == 0) { s_wm[threadIdx.x >> 6] = mx; s_wn[threadIdx.x >> 6] = nan; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float m = -INFINITY;
    uint32_t nn = 0;
    for (int w = 0; w < 1024 / kWave; ++w) { m = fmaxf(m, s_wm[w]); nn |= s_wn[w]; }
    s_mx = m;
    s_nan = nn;
  }
  __syncthreads();
  // torch.max propagates NaN; Python min(thr, NaN) returns thr (NaN < thr is False)
  const float gmax = s_nan ? __int_as_float(0x7FC00000) : s_mx;
  const bool use_max = !fixed_bound && !s_nan && gmax < thr;
  const float bound = use_max ? gmax : thr;
  // chunk offsets (valid when the counts were taken at `bound`)
  uint32_t run = 0;
  for (int64_t j0 = 0; j0 < nchunks; j0 += 1024) {
    const int64_t j = j0 + threadIdx.x;
    const uint32_t c = j < nchunks ? part[j].cnt : 0u;
    uint32_t tot;
    const uint32_t ex = blk_excl_scan<1024>(c, s_w, &tot);
    if (j < nchunks) offs[j] = run + ex;
    run += tot;
  }
  if (threadIdx.x == 0) {
    meta[0] = __float_as_uint(bound);
    meta[1] = run;
    meta[2] = (!final_pass && use_max) ? 1u : 0u;   // counts were taken at thr: recount at max
  }
}

// device-side recount (the host-free variant): only when pass 2 flagged max(x) < thr, count again at
// the bound it chose; the bound kernel then runs as the final pass and clears the flag
__global__ __launch_bounds__(kSBlock) void thr_restats_kernel(const float* __restrict__ x, int64_t n,
                                                             const uint32_t* __restrict__ meta,
                                                             ThrPart* __restrict__ part) {
  if (meta[2] == 0u) return;
  const float bound = __uint_as_float(meta[0]);
  const int64_t base = (int64_t)blockIdx.x * kThrChunk;
  const int64_t end = min(base + (int64_t)kThrChunk, n);
  uint32_t cnt = 0;
  for (int64_t i = base + threadIdx.x; i < end; i += kSBlock) cnt += fabsf(x[i]) >= bound;
  __shared__ uint32_t sc[kSBlock / kWave];
  cnt = wave_sum(cnt);
  if ((threadIdx.x & 63) == 0) sc[threadIdx.x >> 6] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t c = 0;
    for (int j = 0; j < kSBlock / kWave; ++j) c += sc[j];
    part[blockIdx.x].cnt = c;
  }
}
__global__ __launch_bounds__(1024) void thr_reoffset_kernel(ThrPart* __restrict__ part, int64_t nchunks,
                                                           uint32_t* __restrict__ offs, uint32_t* __restrict__ meta) {
  __shared__ uint32_t s_w[1024 / kWave + 1];
  if (meta[2] == 0u) return;
  uint32_t run = 0;
  for (int64_t j0 = 0; j0 < nchunks; j0 += 1024) {
    const int64_t j = j0 + threadIdx.x;
    const uint32_t c = j < nchunks ? part[j].cnt : 0u;
    uint32_t tot;
    const uint32_t ex = blk_excl_scan<1024>(c, s_w, &tot);
    if (j < nchunks) offs[j] = run + ex;
    run += tot;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    meta[1] = run;
    meta[2] = 0u;
  }
}

// r[idx[j]] -= vals[j]: ResidualMemory.update's r = t - decompress(payload) (residual.py:16-20)
// when r already holds t; the decompressed tensor is the scattered values and zeros elsewhere
__global__ __launch_bounds__(kSBlock) void sparse_sub_kernel(const float* __restrict__ vals,
                                                            const int32_t* __restrict__ idx, int64_t count,
                                                            float* __restrict__ r) {
  for (int64_t j = (int64_t)blockIdx.x * kSBlock + threadIdx.x; j < count; j += (int64_t)gridDim.x * kSBlock)
    r[idx[j]] = r[idx[j]] - vals[j];
}

// pass 3: ordered compaction of |x| >= bound.  Entries at positions >= cap are dropped (the
// capacity-bounded exchange record); hdr, when given, receives {count, cap}.
template <typename IdxT>
__global__ __launch_bounds__(kSBlock) void thr_write_kernel(const float* __restrict__ x, int64_t n,
                                                           const uint32_t* __restrict__ offs,
                                                           const uint32_t* __restrict__ meta,
                                                           float* __restrict__ vals, IdxT* __restrict__ idx,
                                                           int64_t cap, uint32_t* __restrict__ hdr) {
  __shared__ uint32_t s_w[kSBlock / kWave + 1];
  const float bound = __uint_as_float(meta[0]);
  if (hdr && blockIdx.x == 0 && threadIdx.x == 0) {
    hdr[0] = meta[1];
    hdr[1] = (uint32_t)cap;
    hdr[2] = 0u;
    hdr[3] = 0u;
  }
  const int64_t base = (int64_t)blockIdx.x * kThrChunk;
  const int64_t end = min(base + (int64_t)kThrChunk, n);
  uint32_t run = offs[blockIdx.x];
  for (int64_t j0 = base; j0 < end; j0 += kSBlock) {
    const int64_t i = j0 + threadIdx.x;
    float v = 0.f;
    bool sel = false;
    if (i < end) { v = x[i]; sel = fabsf(v) >= bound; }
    uint32_t tot;
    const uint32_t ex = blk_excl_scan<kSBlock>(sel ? 1u : 0u, s_w, &tot);
    if (sel && (int64_t)(run + ex) < cap) { vals[run + ex] = v; idx[run + ex] = (IdxT)i; }
    run += tot;
  }
}

// ---- capacity-bounded variable-size exchange -------------------------------------------------
// One record per rank, `stride` = 4 + 2 cap words: {count, cap, 0, 0 | vals f32[cap] | idx i32[cap]}.
// count may exceed cap (overflow): only the first cap entries (ascending index order) travel.
constexpr int kRecHdr = 4;

__device__ __forceinline__ int64_t rec_count(const uint32_t* rec, int64_t cap) {
  return min((int64_t)rec[0], cap);
}

// rank w's entries, added in rank order (one launch per rank on one stream = the reference's
// ((0 + d0) + d1) + ... order, allgather.py:40-45), tagging the last rank that touched each element
__global__ __launch_bounds__(kSBlock) void rec_scatter_kernel(const uint32_t* __restrict__ rec, int64_t cap,
                                                             int32_t w, float* __restrict__ out,
                                                             int32_t* __restrict__ tags) {
  const int64_t c = rec_count(rec, cap);
  const float* vals = reinterpret_cast<const float*>(rec + kRecHdr);
  const int32_t* idx = reinterpret_cast<const int32_t*>(rec + kRecHdr + cap);
  for (int64_t j = (int64_t)blockIdx.x * kSBlock + threadIdx.x; j < c; j += (int64_t)gridDim.x * kSBlock) {
    const int32_t i = idx[j];
    out[i] = out[i] + vals[j];
    tags[i] = w;
  }
}

// divide each aggregated element once (by the entry of the last rank that touched it), and
// stat = {max count over ranks, overflow flag} -- identical on every rank, so every rank takes the
// same capacity decision without exchanging anything else
__global__ __launch_bounds__(kSBlock) void rec_divide_kernel(const uint32_t* __restrict__ rec, int64_t stride,
                                                            int64_t cap, int32_t world, float divisor,
                                                            int32_t do_divide, float* __restrict__ out,
                                                            const int32_t* __restrict__ tags,
                                                            uint32_t* __restrict__ stat) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    uint32_t mx = 0u;
    for (int w = 0; w < world; ++w) mx = max(mx, rec[(int64_t)w * stride]);
    stat[0] = mx;
    stat[1] = (int64_t)mx > cap ? 1u : 0u;
  }
  if (!do_divide) return;
  const int64_t total = (int64_t)world * cap;
  for (int64_t j = (int64_t)blockIdx.x * kSBlock + threadIdx.x; j < total; j += (int64_t)gridDim.x * kSBlock) {
    const int64_t w = j / cap, e = j - w * cap;
    const uint32_t* r = rec + w * stride;
    if (e >= rec_count(r, cap)) continue;
    const int32_t i = reinterpret_cast<const int32_t*>(r + kRecHdr + cap)[e];
    if (tags[i] == (int32_t)w) out[i] = out[i] / divisor;
  }
}

// r[idx] -= vals over the entries that travelled (ResidualMemory.update, residual.py:16-20)
__global__ __launch_bounds__(kSBlock) void rec_sub_kernel(const uint32_t* __restrict__ rec, int64_t cap,
                                                         float* __restrict__ r) {
  const int64_t c = rec_count(rec, cap);
  const float* vals = reinterpret_cast<const float*>(rec + kRecHdr);
  const int32_t* idx = reinterpret_cast<const int32_t*>(rec + kRecHdr + cap);
  for (int64_t j = (int64_t)blockIdx.x * kSBlock + threadIdx.x; j < c; j += (int64_t)gridDim.x * kSBlock)
    r[idx[j]] = r[idx[j]] - vals[j];
}

}  // namespace grace

using namespace grace;

extern "C" {

grace_status_t grace_randomk_indices(uint64_t seed, int64_t numel, int64_t k, int64_t* idx, void* stream) {
  GRACE_REQUIRE(idx && numel >= 1 && k >= 0, "grace_randomk_indices: bad arguments");
  if (k == 0) return GRACE_OK;
  randomk_idx_kernel<<<stream_grid(k, kSBlock, 2048), kSBlock, 0, as_stream(stream)>>>(seed, numel, k, idx);
  GRACE_CHECK_LAUNCH("grace_randomk_indices");
  return GRACE_OK;
}

grace_status_t grace_randomk_step_w1(const float* g, float* residual, int32_t has_residual, float beta, float gamma,
                                     int64_t n, const int64_t* idx, int64_t k, float* vals, float* out,
                                     void* stream) {
  GRACE_REQUIRE(g && residual && idx && vals && out && n >= 1 && k >= 0, "grace_randomk_step_w1: bad arguments");
  hipStream_t s = as_stream(stream);
  const unsigned grid = stream_grid((n + 3) / 4, kSBlock * kRQ, 4096);
  if (has_residual) randomk_pass_kernel<true><<<grid, kSBlock, 0, s>>>(g, residual, beta, gamma, n, out);
  else randomk_pass_kernel<false><<<grid, kSBlock, 0, s>>>(g, residual, beta, gamma, n, out);
  GRACE_CHECK_LAUNCH("grace_randomk_step_w1");
  if (k == 0) return GRACE_OK;
  gather_kernel<<<stream_grid(k, kSBlock, 2048), kSBlock, 0, s>>>(residual, idx, k, vals);
  GRACE_CHECK_LAUNCH("grace_randomk_step_w1");
  randomk_scatter_kernel<<<stream_grid(k, kSBlock, 2048), kSBlock, 0, s>>>(idx, vals, k, residual, out);
  GRACE_CHECK_LAUNCH("grace_randomk_step_w1");
  return GRACE_OK;
}

grace_status_t grace_randomk_shard_step(const float* g, float* residual, int32_t has_residual, float beta, float gamma,
                                       int64_t lo, int64_t m, const int64_t* idx, int64_t k, float* vals, float* out,
                                       void* stream) {
  GRACE_REQUIRE(g && residual && vals && lo >= 0 && m >= 1 && k >= 0 && (k == 0 || idx),
                "grace_randomk_shard_step: bad arguments");
  hipStream_t s = as_stream(stream);
  const unsigned grid = stream_grid((m + 3) / 4, kSBlock * kRQ, 4096);
  if (has_residual) randomk_pass_kernel<true><<<grid, kSBlock, 0, s>>>(g, residual, beta, gamma, m, out);
  else randomk_pass_kernel<false><<<grid, kSBlock, 0, s>>>(g, residual, beta, gamma, m, out);
  GRACE_CHECK_LAUNCH("grace_randomk_shard_step");
  if (k == 0) return GRACE_OK;
  randomk_shard_gather_kernel<<<stream_grid(k, kSBlock, 2048), kSBlock, 0, s>>>(residual, idx, k, lo, m, vals);
  GRACE_CHECK_LAUNCH("grace_randomk_shard_step");
  randomk_shard_scatter_kernel<<<stream_grid(k, kSBlock, 2048), kSBlock, 0, s>>>(idx, vals, k, lo, m, residual, out);
  GRACE_CHECK_LAUNCH("grace_randomk_shard_step");
  return GRACE_OK;
}

grace_status_t grace_randomk_decode(const float* vals, const int64_t* idx, int64_t k, float* out, int64_t n,
                                    void* stream) {
  GRACE_REQUIRE(out && n >= 1 && k >= 0 && (k == 0 || (vals && idx)), "grace_randomk_decode: bad arguments");
  grace_status_t st = grace_fill(out, 0.f, n, stream);
  if (st != GRACE_OK || k == 0) return st;
  randomk_shard_scatter_kernel<<<stream_grid(k, kSBlock, 2048), kSBlock, 0, as_stream(stream)>>>(idx, vals, k, 0, n,
                                                                                                  nullptr, out);
  GRACE_CHECK_LAUNCH("grace_randomk_decode");
  return GRACE_OK;
}

size_t grace_randomk_step_w1_dense_workspace_bytes(int64_t n, int64_t k) {
  const int64_t nch = (n + kRkChunk - 1) / kRkChunk;
  return group_scratch_bytes(nch) + ((sizeof(uint32_t) * (size_t)nch + 255) & ~(size_t)255) +
         sizeof(uint16_t) * (size_t)(k < 1 ? 1 : k);
}

size_t grace_randomk_group_bytes(int64_t n, int64_t k) {
  const int64_t nch = (n + kRkChunk - 1) / kRkChunk;
  return ((sizeof(uint32_t) * (size_t)nch + 255) & ~(size_t)255) + sizeof(uint16_t) * (size_t)(k < 1 ? 1 : k);
}

grace_status_t grace_randomk_step_w1_dense(const float* g, float* residual, int32_t has_residual, float beta,
                                           float gamma, int64_t n, const int64_t* idx, int64_t k, float* out,
                                           void* grp, const void* prev_grp, void* ws, size_t ws_bytes,
                                           void* stream) {
  GRACE_REQUIRE(g && residual && out && ws && n >= 1 && n < ((int64_t)1 << 31) && k >= 0 && (k == 0 || idx) &&
                    ws_bytes >= grace_randomk_step_w1_dense_workspace_bytes(n, k),
                "grace_randomk_step_w1_dense: bad arguments (n < 2^31, workspace)");
  const int64_t nch = (n + kRkChunk - 1) / kRkChunk;
  GRACE_REQUIRE(nch <= 32768, "grace_randomk_step_w1_dense: n <= 2^28");
  GRACE_REQUIRE(!prev_grp || grp, "grace_randomk_step_w1_dense: a recycled output needs this step's grouping buffer");
  hipStream_t s = as_stream(stream);
  char* p = reinterpret_cast<char*>(ws);
  uint32_t* scratch = reinterpret_cast<uint32_t*>(p);   // the grouping's tickets and counts (left zeroed)
  // this step's grouping: into the caller's per-name buffer `grp` (it becomes the next step's
  // prev_grp), or into the workspace
  char* q = grp ? reinterpret_cast<char*>(grp) : p + group_scratch_bytes(nch);
  const size_t eb = (sizeof(uint32_t) * (size_t)nch + 255) & ~(size_t)255;
  uint32_t* ends = reinterpret_cast<uint32_t*>(q);
  uint16_t* offs = reinterpret_cast<uint16_t*>(q + eb);
  const uint32_t* pends = prev_grp ? reinterpret_cast<const uint32_t*>(prev_grp) : nullptr;
  const uint16_t* poffs = prev_grp ? reinterpret_cast<const uint16_t*>(reinterpret_cast<const char*>(prev_grp) + eb) : nullptr;
  const hipError_t e = group_by_chunk<int64_t>(nullptr, idx, k, nch, nullptr, offs, ends, scratch, s);
  if (e != hipSuccess) { set_error("grace_randomk_step_w1_dense", e); return GRACE_ERR_HIP; }
  if (prev_grp) {
    if (has_residual)
      randomk_dense_pass_kernel<true, true><<<(unsigned)nch, kSBlock, 0, s>>>(g, residual, beta, gamma, n, offs, ends, out,
                                                                            poffs, pends);
    else
      randomk_dense_pass_kernel<false, true><<<(unsigned)nch, kSBlock, 0, s>>>(g, residual, beta, gamma, n, offs, ends,
                                                                             out, poffs, pends);
  } else if (has_residual) {
    randomk_dense_pass_kernel<true, false><<<(unsigned)nch, kSBlock, 0, s>>>(g, residual, beta, gamma, n, offs, ends, out,
                                                                           nullptr, nullptr);
  } else {
    randomk_dense_pass_kernel<false, false><<<(unsigned)nch, kSBlock, 0, s>>>(g, residual, beta, gamma, n, offs, ends, out,
                                                                            nullptr, nullptr);
  }
  GRACE_CHECK_LAUNCH("grace_randomk_step_w1_dense");
  return GRACE_OK;
}

grace_status_t grace_gather(const float* x, const int64_t* idx, int64_t k, float* vals, void* stream) {
  GRACE_REQUIRE(x && idx && vals && k >= 0, "grace_gather: bad arguments");
  if (k == 0) return GRACE_OK;
  gather_kernel<<<stream_grid(k, kSBlock, 2048), kSBlock, 0, as_stream(stream)>>>(x, idx, k, vals);
  GRACE_CHECK_LAUNCH("grace_gather");
  return GRACE_OK;
}

size_t grace_threshold_workspace_bytes(int64_t n) {
  const int64_t nch = (n + kThrChunk - 1) / kThrChunk;
  return 64 + sizeof(ThrPart) * (size_t)nch + sizeof(uint32_t) * (size_t)nch + 256;
}

// Stage 1: statistics and offsets.  The caller reads meta (bound bits, count, recount flag) from
// the workspace (first 16 bytes) to size the outputs, then calls grace_threshold_write.
grace_status_t grace_threshold_count(const float* x, int64_t n, float thr, void* ws, void* stream) {
  GRACE_REQUIRE(x && ws && n >= 1, "grace_threshold_count: bad arguments");
  const int64_t nch = (n + kThrChunk - 1) / kThrChunk;
  char* p = reinterpret_cast<char*>(ws);
  uint32_t* meta = reinterpret_cast<uint32_t*>(p);
  ThrPart* part = reinterpret_cast<ThrPart*>(p + 64);
  uint32_t* offs = reinterpret_cast<uint32_t*>(p + 64 + sizeof(ThrPart) * nch);
  hipStream_t s = as_stream(stream);
  thr_stats_kernel<<<(unsigned)nch, kSBlock, 0, s>>>(x, n, thr, part);
  GRACE_CHECK_LAUNCH("grace_threshold_count");
  thr_bound_kernel<<<1, 1024, 0, s>>>(part, nch, thr, offs, meta, 0, 0);
  GRACE_CHECK_LAUNCH("grace_threshold_count");
  return GRACE_OK;
}

grace_status_t grace_threshold_step_w1(const float* g, float* residual, int32_t mode, float beta, float gamma,
                                       int64_t n, float thr, void* ws, float* out, void* stream) {
  GRACE_REQUIRE(g && out && ws && n >= 1 && mode >= 0 && mode <= 2 && (mode == 0 || residual),
                "grace_threshold_step_w1: bad arguments");
  const int64_t nch = (n + kThrChunk - 1) / kThrChunk;
  char* p = reinterpret_cast<char*>(ws);
  uint32_t* meta = reinterpret_cast<uint32_t*>(p);
  ThrPart* part = reinterpret_cast<ThrPart*>(p + 64);
  uint32_t* offs = reinterpret_cast<uint32_t*>(p + 64 + sizeof(ThrPart) * nch);
  (void)offs;
  hipStream_t s = as_stream(stream);
  GRACE_REQUIRE(nch < (int64_t)1 << 31, "grace_threshold_step_w1: too many chunks");
  const unsigned fgrid = stream_grid(n, kSBlock, 1024);
  if (mode == 0) {
    thr_spec_kernel<0><<<(unsigned)nch, kSBlock, 0, s>>>(g, nullptr, beta, gamma, n, thr, out, part, meta);
    GRACE_CHECK_LAUNCH("grace_threshold_step_w1");
    thr_fix_kernel<0><<<fgrid, kSBlock, 0, s>>>(g, nullptr, n, thr, meta, out);
  } else if (mode == 1) {
    thr_spec_kernel<1><<<(unsigned)nch, kSBlock, 0, s>>>(g, residual, beta, gamma, n, thr, out, part, meta);
    GRACE_CHECK_LAUNCH("grace_threshold_step_w1");
    thr_fix_kernel<1><<<fgrid, kSBlock, 0, s>>>(g, residual, n, thr, meta, out);
  } else {
    thr_spec_kernel<2><<<(unsigned)nch, kSBlock, 0, s>>>(g, residual, beta, gamma, n, thr, out, part, meta);
    GRACE_CHECK_LAUNCH("grace_threshold_step_w1");
    thr_fix_kernel<2><<<fgrid, kSBlock, 0, s>>>(g, residual, n, thr, meta, out);
  }
  GRACE_CHECK_LAUNCH("grace_threshold_step_w1");
  return GRACE_OK;
}

// Recount at max(x) (only when max(x) < thr, flagged by stage 1).
grace_status_t grace_threshold_recount(const float* x, int64_t n, float bound, void* ws, void* stream) {
  GRACE_REQUIRE(x && ws && n >= 1, "grace_threshold_recount: bad arguments");
  const int64_t nch = (n + kThrChunk - 1) / kThrChunk;
  char* p = reinterpret_cast<char*>(ws);
  uint32_t* meta = reinterpret_cast<uint32_t*>(p);
  ThrPart* part = reinterpret_cast<ThrPart*>(p + 64);
  uint32_t* offs = reinterpret_cast<uint32_t*>(p + 64 + sizeof(ThrPart) * nch);
  hipStream_t s = as_stream(stream);
  thr_stats_kernel<<<(unsigned)nch, kSBlock, 0, s>>>(x, n, bound, part);
  GRACE_CHECK_LAUNCH("grace_threshold_recount");
  thr_bound_kernel<<<1, 1024, 0, s>>>(part, nch, bound, offs, meta, 1, 0);
  GRACE_CHECK_LAUNCH("grace_threshold_recount");
  return GRACE_OK;
}

// Stage 1 without any host decision: the recount (max(x) < thr) is decided on the device, so the
// count (ws[4..8]) can be exchanged between ranks before anything is read on the host.
grace_status_t grace_threshold_count_dev(const float* x, int64_t n, float thr, void* ws, void* stream) {
  GRACE_REQUIRE(x && ws && n >= 1, "grace_threshold_count_dev: bad arguments");
  grace_status_t st = grace_threshold_count(x, n, thr, ws, stream);
  if (st != GRACE_OK) return st;
  const int64_t nch = (n + kThrChunk - 1) / kThrChunk;
  char* p = reinterpret_cast<char*>(ws);
  uint32_t* meta = reinterpret_cast<uint32_t*>(p);
  ThrPart* part = reinterpret_cast<ThrPart*>(p + 64);
  uint32_t* offs = reinterpret_cast<uint32_t*>(p + 64 + sizeof(ThrPart) * nch);
  hipStream_t s = as_stream(stream);
  thr_restats_kernel<<<(unsigned)nch, kSBlock, 0, s>>>(x, n, meta, part);
  GRACE_CHECK_LAUNCH("grace_threshold_count_dev");
  thr_reoffset_kernel<<<1, 1024, 0, s>>>(part, nch, offs, meta);
  GRACE_CHECK_LAUNCH("grace_threshold_count_dev");
  return GRACE_OK;
}

grace_status_t grace_sparse_sub(const float* vals, const int32_t* idx, int64_t count, float* r, void* stream) {
  GRACE_REQUIRE(count >= 0 && (count == 0 || (vals && idx && r)), "grace_sparse_sub: bad arguments");
  if (count == 0) return GRACE_OK;
  sparse_sub_kernel<<<stream_grid(count, kSBlock, 2048), kSBlock, 0, as_stream(stream)>>>(vals, idx, count, r);
  GRACE_CHECK_LAUNCH("grace_sparse_sub");
  return GRACE_OK;
}

grace_status_t grace_threshold_write(const float* x, int64_t n, const void* ws, float* vals, int32_t* idx,
                                     void* stream) {
  GRACE_REQUIRE(x && ws && n >= 1, "grace_threshold_write: bad arguments");
  const int64_t nch = (n + kThrChunk - 1) / kThrChunk;
  const char* p = reinterpret_cast<const char*>(ws);
  const uint32_t* meta = reinterpret_cast<const uint32_t*>(p);
  const uint32_t* offs = reinterpret_cast<const uint32_t*>(p + 64 + sizeof(ThrPart) * nch);
  thr_write_kernel<int32_t><<<(unsigned)nch, kSBlock, 0, as_stream(stream)>>>(x, n, offs, meta, vals, idx, n,
                                                                           nullptr);
  GRACE_CHECK_LAUNCH("grace_threshold_write");
  return GRACE_OK;
}

grace_status_t grace_randomk_perm_indices(uint64_t seed, int64_t numel, int64_t k, int64_t* idx, void* stream) {
  GRACE_REQUIRE(idx && numel >= 1 && k >= 0 && k <= numel && numel < ((int64_t)1 << 62),
                "grace_randomk_perm_indices: bad arguments (0 <= k <= numel)");
  if (k == 0) return GRACE_OK;
  int h = 1;
  while ((int64_t)1 << (2 * h) < numel) ++h;
  randperm_idx_kernel<<<stream_grid(k, kSBlock, 2048), kSBlock, 0, as_stream(stream)>>>(seed, numel, k, h, idx);
  GRACE_CHECK_LAUNCH("grace_randomk_perm_indices");
  return GRACE_OK;
}

grace_status_t grace_widen_i32(const int32_t* src, int64_t n, int64_t* dst, void* stream) {
  GRACE_REQUIRE(n >= 0 && (n == 0 || (src && dst)), "grace_widen_i32: bad arguments");
  if (n == 0) return GRACE_OK;
  widen_i32_kernel<<<stream_grid(n, kSBlock, 2048), kSBlock, 0, as_stream(stream)>>>(src, n, dst);
  GRACE_CHECK_LAUNCH("grace_widen_i32");
  return GRACE_OK;
}

// Horovod-flavour threshold (grace_dl/torch/compressor/threshold.py:17): |x| > thr, no max rule.
// The caller passes bound = the smallest f32 above thr (|x| > thr <=> |x| >= bound for every
// f32, NaN never selected), or NaN when thr is +inf (nothing selected).
grace_status_t grace_threshold_count_fixed(const float* x, int64_t n, float bound, void* ws, void* stream) {
  GRACE_REQUIRE(x && ws && n >= 1, "grace_threshold_count_fixed: bad arguments");
  const int64_t nch = (n + kThrChunk - 1) / kThrChunk;
  char* p = reinterpret_cast<char*>(ws);
  uint32_t* meta = reinterpret_cast<uint32_t*>(p);
  ThrPart* part = reinterpret_cast<ThrPart*>(p + 64);
  uint32_t* offs = reinterpret_cast<uint32_t*>(p + 64 + sizeof(ThrPart) * nch);
  hipStream_t s = as_stream(stream);
  thr_stats_kernel<<<(unsigned)nch, kSBlock, 0, s>>>(x, n, bound, part);
  GRACE_CHECK_LAUNCH("grace_threshold_count_fixed");
  thr_bound_kernel<<<1, 1024, 0, s>>>(part, nch, bound, offs, meta, 1, 1);
  GRACE_CHECK_LAUNCH("grace_threshold_count_fixed");
  return GRACE_OK;
}

grace_status_t grace_threshold_write_i64(const float* x, int64_t n, const void* ws, float* vals, int64_t* idx,
                                         void* stream) {
  GRACE_REQUIRE(x && ws && n >= 1, "grace_threshold_write_i64: bad arguments");
  const int64_t nch = (n + kThrChunk - 1) / kThrChunk;
  const char* p = reinterpret_cast<const char*>(ws);
  const uint32_t* meta = reinterpret_cast<const uint32_t*>(p);
  const uint32_t* offs = reinterpret_cast<const uint32_t*>(p + 64 + sizeof(ThrPart) * nch);
  thr_write_kernel<int64_t><<<(unsigned)nch, kSBlock, 0, as_stream(stream)>>>(x, n, offs, meta, vals, idx, n,
                                                                           nullptr);
  GRACE_CHECK_LAUNCH("grace_threshold_write_i64");
  return GRACE_OK;
}

size_t grace_exchange_record_words(int64_t cap) { return (size_t)(kRecHdr + 2 * cap); }

// Writes this rank's capacity-bounded exchange record (after grace_threshold_count_dev).
grace_status_t grace_threshold_write_capped(const float* x, int64_t n, const void* ws, uint32_t* rec, int64_t cap,
                                            void* stream) {
  GRACE_REQUIRE(x && ws && rec && n >= 1 && cap >= 1 && cap <= n && n < ((int64_t)1 << 31),
                "grace_threshold_write_capped: bad arguments (1 <= cap <= n)");
  const int64_t nch = (n + kThrChunk - 1) / kThrChunk;
  const char* p = reinterpret_cast<const char*>(ws);
  const uint32_t* meta = reinterpret_cast<const uint32_t*>(p);
  const uint32_t* offs = reinterpret_cast<const uint32_t*>(p + 64 + sizeof(ThrPart) * nch);
  float* vals = reinterpret_cast<float*>(rec + kRecHdr);
  int32_t* idx = reinterpret_cast<int32_t*>(rec + kRecHdr + cap);
  thr_write_kernel<int32_t><<<(unsigned)nch, kSBlock, 0, as_stream(stream)>>>(x, n, offs, meta, vals, idx, cap, rec);
  GRACE_CHECK_LAUNCH("grace_threshold_write_capped");
  return GRACE_OK;
}

// Rank-ordered decode + aggregate of W gathered records (stride = grace_exchange_record_words(cap)
// words apart) into out[n] (zero-filled here), each element divided once by `divisor`; stat
// (device, u32[2]) = {max count over ranks, overflow = max count > cap}.
grace_status_t grace_sparse_aggregate_capped(const uint32_t* recs, int64_t stride, int64_t cap, int32_t world,
                                             float divisor, float* out, int32_t* tags, int64_t n, uint32_t* stat,
                                             void* stream) {
  GRACE_REQUIRE(recs && out && tags && stat && world >= 1 && cap >= 1 && stride == kRecHdr + 2 * cap && n >= 1,
                "grace_sparse_aggregate_capped: bad arguments");
  grace_status_t st = grace_fill(out, 0.f, n, stream);
  if (st != GRACE_OK) return st;
  hipStream_t s = as_stream(stream);
  const unsigned g = stream_grid(cap, kSBlock, 1024);
  for (int w = 0; w < world; ++w) {
    rec_scatter_kernel<<<g, kSBlock, 0, s>>>(recs + (int64_t)w * stride, cap, w, out, tags);
    GRACE_CHECK_LAUNCH("grace_sparse_aggregate_capped");
  }
  const int do_div = divisor != 1.0f;
  rec_divide_kernel<<<do_div ? stream_grid((int64_t)world * cap, kSBlock, 2048) : 1u, kSBlock, 0, s>>>(
      recs, stride, cap, world, divisor, do_div, out, tags, stat);
  GRACE_CHECK_LAUNCH("grace_sparse_aggregate_capped");
  return GRACE_OK;
}

grace_status_t grace_sparse_sub_capped(const uint32_t* rec, int64_t cap, float* r, void* stream) {
  GRACE_REQUIRE(rec && r && cap >= 1, "grace_sparse_sub_capped: bad arguments");
  rec_sub_kernel<<<stream_grid(cap, kSBlock, 2048), kSBlock, 0, as_stream(stream)>>>(rec, cap, r);
  GRACE_CHECK_LAUNCH("grace_sparse_sub_capped");
  return GRACE_OK;
}

}  // extern "C"
