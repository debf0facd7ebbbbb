// Index-sorted sparse payloads and their rank-ordered aggregate (the world > 1 decode of
// Allgather(TopK), grace_dl/dist/communicator/allgather.py:40-45).
//
// The W payloads of a step land on every rank; decoding them with one random scatter per rank
// read-modify-writes the 256 MiB output W times (~55 us per rank on MI355X).  Instead each rank
// groups its own payload by 8192-element output chunk before the exchange (a counting sort by
// chunk: LDS histograms, a scan of the counts, LDS-ranked scatter -- a full radix sort of the indices is not
// needed and costs ~10x more), and the decode is one pass over the OUTPUT: a workgroup per chunk
// finds every rank's sub-range of that chunk from a boundary table, accumulates the ranks in
// order in LDS -- ((0 + d0) + d1) + ... exactly as Python's sum -- divides, and writes the chunk
// densely, which also replaces the zero-fill.  Each rank's chunk end offsets (a by-product of the
// grouping) travel with its payload, so the receiver needs no pass to find the sub-ranges.  The
// grouped payload carries each entry's offset inside its chunk as a u16 (13 bits) instead of the
// int32 index: 6 B per entry on the wire instead of 8.

#include "common.h"

namespace grace {

constexpr int kPChunkLog = 13;
constexpr int kPChunk = 1 << kPChunkLog;
#ifndef GRACE_P_BLOCK
#define GRACE_P_BLOCK 256
#endif
// decode workgroup (A/B knob; 8 x 671 K entries into 256 MiB, tools/exp_wn_local.py: 256 threads
// 58 us, 512 68 us, 1024 146 us)
constexpr int kPBlock = GRACE_P_BLOCK;

#ifndef GRACE_GROUP_BLOCK
#define GRACE_GROUP_BLOCK 1024
#endif
#ifndef GRACE_GROUP_PER
#define GRACE_GROUP_PER 4
#endif
// 4096 entries per workgroup over 1024 threads: the per-workgroup clear and scan of the 8192-bin
// LDS histogram (one bin per output chunk) dominate a pass, so they are spread over as many threads
// as possible (A/B, 671,088 entries: 256 x 16 -> 37.4 us, 512 x 8 -> 29.7, 1024 x 4 -> 27.6,
// 1024 x 8 -> 35.3, 256 x 64 -> 64.1)
constexpr int kGroupBlock = GRACE_GROUP_BLOCK;
constexpr int kGroupPer = GRACE_GROUP_PER;             // entries per thread
constexpr int kMaxGroupChunks = 32768;                 // LDS histogram bins (128 KB): n <= 2^28

// pass 1: per-workgroup LDS histogram of chunk ids, flushed with one device atomic per non-zero bin
// into the chunk counts (the caller's zeroed workspace) -- and nothing after it: no ticket, no scan.
// pass 2 finds every chunk's start itself (each workgroup scans the counts, a kernel boundary
// later), so the histogram pass ends as soon as its adds are issued.  (r05: the last arriver's scan
// here was a ~4 us tail of vmcnt(0), ticket and one workgroup's scan on the grouping's chain.)
template <typename IdxT>
__global__ __launch_bounds__(kGroupBlock) void group_hist_kernel(const IdxT* __restrict__ idx, int64_t k,
                                                                int64_t nchunks, uint32_t* __restrict__ counts) {
  extern __shared__ uint32_t h[];
  for (int64_t c = threadIdx.x; c < nchunks; c += kGroupBlock) h[c] = 0u;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kGroupBlock * kGroupPer;
#pragma unroll 4
  for (int e = 0; e < kGroupPer; ++e) {
    const int64_t j = base + (int64_t)e * kGroupBlock + threadIdx.x;
    if (j < k) atomicAdd(&h[(int64_t)idx[j] >> kPChunkLog], 1u);
  }
  __syncthreads();
  for (int64_t c = threadIdx.x; c < nchunks; c += kGroupBlock)
    if (h[c]) atomicAdd(&counts[c], h[c]);
}

// exclusive scan of the chunk counts by one workgroup, kScanPer counts per thread per round: f(c,
// exclusive start of chunk c, count of c) for every chunk; the counts come from device atomics of an
// earlier launch, read with agent loads
constexpr int kScanPer = 8;
template <typename F>
__device__ __forceinline__ void scan_counts(const uint32_t* counts, int64_t nchunks, uint32_t* s_w, F f) {
  constexpr int NT = kGroupBlock;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t run = 0;
  for (int64_t c0 = 0; c0 < nchunks; c0 += NT * kScanPer) {
    const int64_t cb = c0 + (int64_t)threadIdx.x * kScanPer;
    uint32_t v[kScanPer], sum = 0;
#pragma unroll
    for (int e = 0; e < kScanPer; ++e) {
      v[e] = cb + e < nchunks ? __hip_atomic_load(counts + cb + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
      sum += v[e];
    }
    uint32_t inc = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = __shfl_up(inc, o, 64);
      if (lane >= o) inc += t;
    }
    if (lane == 63) s_w[w] = inc;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t acc = 0;
      for (int i = 0; i < NT / kWave; ++i) { const uint32_t t = s_w[i]; s_w[i] = acc; acc += t; }
      s_w[NT / kWave] = acc;
    }
    __syncthreads();
    uint32_t ex = run + s_w[w] + inc - sum;
#pragma unroll
    for (int e = 0; e < kScanPer; ++e) {
      if (cb + e < nchunks) f(cb + e, ex, v[e]);
      ex += v[e];
    }
    run += s_w[NT / kWave];
    __syncthreads();
  }
}

// pass 2: each workgroup reserves its range of every chunk it touches (one returning atomic per
// non-zero bin on the chunk's cursor), adds the chunk starts from its own scan of the counts, ranks
// its entries within a bin with LDS atomics, and writes them grouped by chunk.  Workgroup 0 writes
// the chunk end offsets (the inclusive scan); the last workgroup to finish re-zeroes the counts and
// cursors for the next grouping (the scratch lives in the caller's workspace, so no memset launch
// precedes the histogram pass).
template <typename IdxT>
__global__ __launch_bounds__(kGroupBlock) void group_scatter_kernel(const float* __restrict__ vals,
                                                                   const IdxT* __restrict__ idx, int64_t k,
                                                                   int64_t nchunks, uint32_t* __restrict__ counts,
                                                                   uint32_t* __restrict__ cursor,
                                                                   float* __restrict__ vals_out,
                                                                   uint16_t* __restrict__ off_out,
                                                                   uint32_t* __restrict__ ends_out,
                                                                   uint32_t* __restrict__ ticket) {
  extern __shared__ uint32_t h[];
  __shared__ uint32_t s_w[kGroupBlock / kWave + 1];
  __shared__ uint32_t s_last;
  const int64_t base = (int64_t)blockIdx.x * kGroupBlock * kGroupPer;
  int32_t ii[kGroupPer];
  float vv[kGroupPer];
#pragma unroll
  for (int e = 0; e < kGroupPer; ++e) {   // the entries' loads first: their latency overlaps the scan's
    const int64_t j = base + (int64_t)e * kGroupBlock + threadIdx.x;
    ii[e] = j < k ? (int32_t)idx[j] : -1;
    vv[e] = j < k && vals ? vals[j] : 0.f;
  }
  for (int64_t c = threadIdx.x; c < nchunks; c += kGroupBlock) h[c] = 0u;
  __syncthreads();
#pragma unroll
  for (int e = 0; e < kGroupPer; ++e)
    if (ii[e] >= 0) atomicAdd(&h[ii[e] >> kPChunkLog], 1u);
  __syncthreads();
  for (int64_t c = threadIdx.x; c < nchunks; c += kGroupBlock)
    if (h[c]) h[c] = atomicAdd(&cursor[c], h[c]);     // this workgroup's first slot inside chunk c
  __syncthreads();
  // + the chunk's start: every bin a thread owns in the scan is its own to update
  const bool w0 = blockIdx.x == 0;
  scan_counts(counts, nchunks, s_w, [&](int64_t c, uint32_t start, uint32_t cnt) {
    h[c] += start;
    if (w0) ends_out[c] = start + cnt;
  });
  __syncthreads();
#pragma unroll
  for (int e = 0; e < kGroupPer; ++e) {
    if (ii[e] < 0) continue;
    const uint32_t pos = atomicAdd(&h[ii[e] >> kPChunkLog], 1u);
    if (vals_out) vals_out[pos] = vv[e];
    off_out[pos] = (uint16_t)(ii[e] & (kPChunk - 1));   // the offset inside its chunk (13 bits)
  }
  // every workgroup's cursor atomics and count reads are done once it arrives: the last one re-zeroes
  // them for the next grouping
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    s_last = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
    if (s_last) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!s_last) return;
  for (int64_t c = threadIdx.x; c < nchunks; c += kGroupBlock) {
    __hip_atomic_store(counts + c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(cursor + c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// One workgroup per 8192-element output chunk.  Rank w's entries of chunk c are [ends_w[c - 1],
// ends_w[c]) of its grouped payload (the chunk end offsets travel with the payload, so no receiver
// pass rebuilds them).  The bounds of every rank go to LDS in one round trip; then, kRankBatch ranks
// at a time, every thread loads its entry of each rank of the batch (all loads in flight together)
// and the entries are added into the LDS tile rank by rank -- ((0 + d0) + d1) + ... exactly as
// Python's sum, since indices are unique within a rank and a barrier separates the ranks.  Ranks
// with more than kPBlock entries in the chunk finish their remaining rounds in order before the
// next rank.  The tile is divided and written densely (the zero-fill included).
// SMALLW (world <= 64): every wave keeps the ranks' bounds in registers (lane w holds rank w's,
// read with readlane), so the tile is the workgroup's only LDS -- 32 KB, five workgroups per CU
// instead of four with the 8 KB bounds table beside it.
constexpr int kRankBatch = 8;
constexpr int kMaxRanks = 1024;
template <bool SMALLW>
__global__ __launch_bounds__(kPBlock) void chunk_accumulate_kernel(const float* __restrict__ vals,
                                                                  const uint16_t* __restrict__ off,
                                                                  const int32_t* __restrict__ ends, int64_t stride,
                                                                  int world, float divisor,
                                                                  float* __restrict__ out, int64_t n) {
  __shared__ float tile[kPChunk];
  __shared__ int32_t s_b[SMALLW ? 1 : 2 * kMaxRanks];
  const int t = threadIdx.x;
  const int64_t ch = blockIdx.x;
  const int64_t c0 = ch << kPChunkLog;
  int32_t bl = 0, el = 0;   // SMALLW: lane w's rank-w bounds
  if constexpr (SMALLW) {
    const int lane = t & 63;
    if (lane < world) {
      const int32_t* ew = ends + (int64_t)lane * stride;
      bl = ch > 0 ? ew[ch - 1] : 0;
      el = ew[ch];
    }
  } else {
    for (int w = t; w < world; w += kPBlock) {
      const int32_t* ew = ends + (int64_t)w * stride;
      s_b[2 * w] = ch > 0 ? ew[ch - 1] : 0;
      s_b[2 * w + 1] = ew[ch];
    }
  }
  auto bnd = [&](int w, int32_t& b, int32_t& e) {   // w wave-uniform
    if constexpr (SMALLW) {
      b = __builtin_amdgcn_readlane(bl, w);
      e = __builtin_amdgcn_readlane(el, w);
    } else {
      b = s_b[2 * w];
      e = s_b[2 * w + 1];
    }
  };
  for (int e = t; e < kPChunk; e += kPBlock) tile[e] = 0.f;
  __syncthreads();
  for (int w0 = 0; w0 < world; w0 += kRankBatch) {
    int32_t l[kRankBatch];
    float v[kRankBatch];
#pragma unroll
    for (int q = 0; q < kRankBatch; ++q) {   // unconditional (clamped) loads: all in flight at once
      const int w = w0 + q < world ? w0 + q : w0;
      int32_t b, e;
      bnd(w, b, e);
      const int32_t p = b + t;
      const bool ok = w0 + q < world && p < e;
      const int64_t pc = (int64_t)w * stride + (ok ? p : 0);
      const int32_t li = off[2 * (int64_t)w * stride + (ok ? p : 0)];   // rank w's u16 offsets: 2 w stride on
      v[q] = vals[pc];
      l[q] = ok ? li : -1;
    }
#pragma unroll
    for (int q = 0; q < kRankBatch; ++q) {
      const int w = w0 + q;
      if (w >= world) break;
      if (l[q] >= 0) tile[l[q]] = tile[l[q]] + v[q];
      int32_t s0, s1;
      bnd(w, s0, s1);
      for (int32_t p = s0 + kPBlock + t; p < s1; p += kPBlock) {   // rare: > 256 entries
        const int32_t lp = off[2 * (int64_t)w * stride + p];
        tile[lp] = tile[lp] + vals[(int64_t)w * stride + p];
      }
      __syncthreads();
    }
  }
  typedef float f4 __attribute__((ext_vector_type(4)));
  if (c0 + kPChunk <= n && (reinterpret_cast<uintptr_t>(out) & 15u) == 0) {
    for (int e = t * 4; e < kPChunk; e += kPBlock * 4) {
      f4 q = {tile[e], tile[e + 1], tile[e + 2], tile[e + 3]};
      if (divisor != 1.0f) { q.x = q.x / divisor; q.y = q.y / divisor; q.z = q.z / divisor; q.w = q.w / divisor; }
      __builtin_nontemporal_store(q, reinterpret_cast<f4*>(out + c0 + e));
    }
  } else {
    for (int e = t; e < kPChunk && c0 + e < n; e += kPBlock)
      out[c0 + e] = divisor != 1.0f ? tile[e] / divisor : tile[e];
  }
}

// group entries by 8192-element chunk (u16 offsets, chunk end offsets); vals optional.  Shared by
// grace_sort_payload and the world-1 random-k step (sparse.hip).
// scratch: [ticket | 252 B | counts u32[kMaxGroupChunks] | cursors u32[kMaxGroupChunks]]
// (group_scratch_bytes), zeroed once and left zeroed by every call
template <typename IdxT>
hipError_t group_by_chunk(const float* vals, const IdxT* idx, int64_t k, int64_t nchunks, float* vals_out,
                          uint16_t* off_out, uint32_t* ends_out, uint32_t* scratch, hipStream_t s) {
  if (k == 0) return hipMemsetAsync(ends_out, 0, sizeof(uint32_t) * nchunks, s);
  uint32_t* counts = scratch + 64;
  uint32_t* cursor = counts + kMaxGroupChunks;
  const unsigned nb = (unsigned)((k + (int64_t)kGroupBlock * kGroupPer - 1) / ((int64_t)kGroupBlock * kGroupPer));
  const size_t lds = sizeof(uint32_t) * (size_t)nchunks;
  group_hist_kernel<IdxT><<<nb, kGroupBlock, lds, s>>>(idx, k, nchunks, counts);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  group_scatter_kernel<IdxT><<<nb, kGroupBlock, lds, s>>>(vals, idx, k, nchunks, counts, cursor, vals_out, off_out,
                                                          ends_out, scratch);
  return hipGetLastError();
}
template hipError_t group_by_chunk<int64_t>(const float*, const int64_t*, int64_t, int64_t, float*, uint16_t*,
                                            uint32_t*, uint32_t*, hipStream_t);
// fixed size whatever nchunks is: a caller that places other data after the scratch must never let
// a larger call's counts land on a smaller call's data (the counts must stay zeroed)
size_t group_scratch_bytes(int64_t nchunks) {
  (void)nchunks;
  return 256 + 2 * sizeof(uint32_t) * (size_t)kMaxGroupChunks;
}

}  // namespace grace

using namespace grace;

extern "C" {

size_t grace_sort_payload_workspace_bytes(int64_t k, int64_t n) {
  (void)k;
  return group_scratch_bytes((n + kPChunk - 1) / kPChunk);   // ticket, chunk counts and cursors, left zeroed
}

// groups the payload by 8192-element output chunk (chunk-ascending; order within a chunk is
// unspecified -- the aggregate does not depend on it); ends_out[c] = end of chunk c's entries
grace_status_t grace_sort_payload(const float* vals, const int32_t* idx, int64_t k, int64_t n, float* vals_out,
                                  uint16_t* off_out, uint32_t* ends_out, void* ws, size_t ws_bytes, void* stream) {
  const int64_t nchunks = (n + kPChunk - 1) / kPChunk;
  GRACE_REQUIRE(vals && idx && vals_out && off_out && ends_out && ws && k >= 0 && k < ((int64_t)1 << 31) &&
                    n >= 1 && nchunks <= kMaxGroupChunks && ws_bytes >= grace_sort_payload_workspace_bytes(k, n),
                "grace_sort_payload: bad arguments (n <= 2^28)");
  const hipError_t e = group_by_chunk<int32_t>(vals, idx, k, nchunks, vals_out, off_out, ends_out,
                                               reinterpret_cast<uint32_t*>(ws), as_stream(stream));
  if (e != hipSuccess) { set_error("grace_sort_payload", e); return GRACE_ERR_HIP; }
  return GRACE_OK;
}

grace_status_t grace_sparse_aggregate_sorted(const float* vals, const uint16_t* off, const uint32_t* ends,
                                             int64_t stride, int32_t world, float divisor, float* out, int64_t n,
                                             void* stream) {
  GRACE_REQUIRE(vals && off && ends && out && world >= 1 && world <= kMaxRanks && n >= 1 &&
                    (n + kPChunk - 1) / kPChunk <= kMaxGroupChunks,
                "grace_sparse_aggregate_sorted: bad arguments (1 <= world <= 1024, n <= 2^28)");
  const int64_t nchunks = (n + kPChunk - 1) / kPChunk;
#ifndef GRACE_DEC_SMALLW
#define GRACE_DEC_SMALLW 1
#endif
  if (GRACE_DEC_SMALLW && world <= kWave)
    chunk_accumulate_kernel<true><<<(unsigned)nchunks, kPBlock, 0, as_stream(stream)>>>(
        vals, off, reinterpret_cast<const int32_t*>(ends), stride, world, divisor, out, n);
  else
    chunk_accumulate_kernel<false><<<(unsigned)nchunks, kPBlock, 0, as_stream(stream)>>>(
        vals, off, reinterpret_cast<const int32_t*>(ends), stride, world, divisor, out, n);
  GRACE_CHECK_LAUNCH("grace_sparse_aggregate_sorted");
  return GRACE_OK;
}

}  // extern "C"
