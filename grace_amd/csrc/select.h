// Shared selection building blocks of the top-k engines (topk.hip: single bucket and per-tensor
// segments; shard.hip: the sharded global cut): block scans, descending histogram bin search, the unique
// composite selection key and an exact single-workgroup radix select over composite keys.
#pragma once

#include "common.h"

namespace grace {

// block-wide exclusive scan of one uint32 per thread (BLOCK threads, wave64)
template <int BLOCK>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* s_w, uint32_t* total) {
  constexpr int NW = BLOCK / kWave;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t t = __shfl_up(inc, o, 64);
    if (lane >= o) inc += t;
  }
  if (lane == 63) s_w[w] = inc;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t acc = 0;
    for (int i = 0; i < NW; ++i) {
      uint32_t t = s_w[i];
      s_w[i] = acc;
      acc += t;
    }
    s_w[NW] = acc;
  }
  __syncthreads();
  const uint32_t r = s_w[w] + inc - v;
  if (total) *total = s_w[NW];
  __syncthreads();
  return r;
}

// Padded LDS histogram layout: bin b at word b + b / 32.  find_bins_desc's thread t reads bins
// 32 t .. 32 t + 31 of a 32768-bin histogram; unpadded, the 64 lanes of a wave hit the same two
// banks (a 32-way conflict on every read: ~7 us of a segment bracket); padded, their stride is 33
// words and every lane has a bank of its own.  NBINS + NBINS / 32 words.
__device__ __forceinline__ int hist_pad(int b) { return b + (b >> 5); }

// Given a histogram hist[NBINS] (in LDS or global; PAD: the hist_pad layout) find, scanning from
// the top, the bin d where the running count reaches `rank` (1-based): sum_{b>d} < rank <=
// sum_{b>=d}, for NR ranks at once (one block scan).  Returns d[q] and above[q] = sum_{b>d[q]}.
// All BLOCK threads must call; NBINS % BLOCK == 0; s_res needs 2*NR words.
template <int BLOCK, int NBINS, int NR, bool PAD = false>
__device__ void find_bins_desc(const uint32_t* hist, const uint32_t (&rank)[NR], uint32_t* s_w,
                               uint32_t* s_res, int (&d)[NR], uint32_t (&above)[NR]) {
  constexpr int PER = NBINS / BLOCK;
  const int t = threadIdx.x;
  const int top = NBINS - 1 - t * PER;  // this thread covers bins top, top-1, ..., top-PER+1
  // the thread's bins stay in registers: with a global histogram, re-reading them in the search
  // below was a chain of dependent global loads (the segmented find kernel's 22 us)
  uint32_t h[PER], s = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j) h[j] = hist[PAD ? hist_pad(top - j) : top - j];
#pragma unroll
  for (int j = 0; j < PER; ++j) s += h[j];
  if (t < 2 * NR) s_res[t] = 0;
  const uint32_t ex = block_excl_scan<BLOCK>(s, s_w, nullptr);
#pragma unroll
  for (int q = 0; q < NR; ++q) {
    if (ex < rank[q] && rank[q] <= ex + s) {
      uint32_t acc = ex;
      bool found = false;
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        if (!found && acc + h[j] >= rank[q]) {
          s_res[2 * q] = (uint32_t)(top - j);
          s_res[2 * q + 1] = acc;
          found = true;
        }
        acc += h[j];
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < NR; ++q) {
    d[q] = (int)s_res[2 * q];
    above[q] = s_res[2 * q + 1];
  }
  __syncthreads();
}

template <int BLOCK, int NBINS>
__device__ int find_bin_desc(const uint32_t* hist, uint32_t rank, uint32_t* s_w, uint32_t* s_res,
                             uint32_t* above_out) {
  const uint32_t r[1] = {rank};
  int d[1];
  uint32_t ab[1];
  find_bins_desc<BLOCK, NBINS, 1>(hist, r, s_w, s_res, d, ab);
  if (above_out) *above_out = ab[0];
  return d[0];
}

// composite selection key: larger |t| first, then lower index first; unique per element
__device__ __forceinline__ uint64_t comp_key(uint32_t key, uint32_t idx) {
  return ((uint64_t)key << 32) | (uint64_t)(0xFFFFFFFFu - idx);
}

// Boundary-list entries cross workgroups (and XCDs, whose L2s are not coherent with each other):
// they are written with agent-scope (sc1, write-through) stores and read back with agent-scope
// loads, so the arrival protocol needs no L2 writeback / invalidate fences.
__device__ __forceinline__ void st_agent_i2(int2* p, int2 v) {
  const uint64_t u = (uint64_t)(uint32_t)v.x | ((uint64_t)(uint32_t)v.y << 32);
  __hip_atomic_store(reinterpret_cast<uint64_t*>(p), u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int2 ld_agent_i2(const int2* p) {
  const uint64_t u = __hip_atomic_load(reinterpret_cast<const uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return make_int2((int)(uint32_t)u, (int)(uint32_t)(u >> 32));
}

// Exact single-workgroup radix select: returns T such that exactly `need` items of src have
// composite >= T (composites are unique).  Passes of 11/11/11/11/11/9 bits from the top; a caller
// that knows the top digit every item shares starts at pass 1 with that prefix.  Stops as soon as
// the chosen bin holds exactly the items still needed (every one of them is taken: T = the prefix
// with zero low bits) -- for untied keys that is after the key bits, so the index passes are skipped.
template <int BLOCK = 1024, typename Src>
__device__ uint64_t block_select_comp(const Src& src, int64_t N, uint32_t need, uint32_t* hist,
                                      uint32_t* s_w, uint32_t* s_res, int first_pass = 0,
                                      uint64_t prefix0 = 0, uint64_t pmask0 = 0) {
#ifdef GRACE_SELECT_U1   // A/B build only
  constexpr int kU = 1;
#else
  constexpr int kU = 4;   // items per thread per round, all loaded before any is counted
#endif
  uint64_t prefix = prefix0, pmask = pmask0;
  uint32_t rem = need;
  for (int p = first_pass; p < 6; ++p) {
    const int shift = p < 5 ? 53 - 11 * p : 0;
    const uint32_t dmask = p < 5 ? 2047u : 511u;
    for (int b = threadIdx.x; b < 2048; b += BLOCK) hist[b] = 0;
    __syncthreads();
    for (int64_t j0 = threadIdx.x; j0 < N; j0 += (int64_t)BLOCK * kU) {
      uint64_t c[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int64_t j = j0 + (int64_t)u * BLOCK;
        c[u] = src(j < N ? j : j0);
      }
#pragma unroll
      for (int u = 0; u < kU; ++u)
        if (j0 + (int64_t)u * BLOCK < N && (c[u] & pmask) == prefix) atomicAdd(&hist[(c[u] >> shift) & dmask], 1u);
    }
    __syncthreads();
    uint32_t above;
    const int d = find_bin_desc<BLOCK, 2048>(hist, rem, s_w, s_res, &above);
    rem -= above;
    prefix |= (uint64_t)d << shift;
    pmask |= (uint64_t)dmask << shift;
#ifdef GRACE_SELECT_NOEARLY   // A/B build only
    const bool whole = false;
#else
    const bool whole = hist[d] == rem;   // LDS, identical for every thread
#endif
    __syncthreads();
    if (whole) break;
  }
  return prefix;
}

}  // namespace grace
