// Sharded top-k with residual error feedback (BASELINE configs[4]): ONE gradient
// bucket of n elements split into contiguous shards, one per rank; the ranks together select
// exactly the single-GPU top-k of the whole bucket (TopKCompressor, grace_dl/dist/compressor/
// topk.py:32-42, with the single-GPU engine's tie rule: larger |t| first, lower global index
// first), keep the residual of their own shard (ResidualMemory, memory/residual.py:10-20) and
// decode the dense result (replicated, or only their own slice).
//
// One exchange per step, no host synchronisation, exact by construction.  The global top-k is
// contained in the union of the ranks' LOCAL top-k (a rank contributes at most k entries, and
// those are its own best k by the same composite order), so:
//   1. local: the single-GPU engine (grace_topk_residual_step, 12 B/element) selects this
//      shard's top-k_loc, k_loc = min(k, m), straight into this rank's record
//      [header | vals f32[cap] | local idx i32[cap]] (cap = k; idx -1 pads a short shard); it
//      leaves r' = t - t at its picks and r' = t elsewhere;
//   2. ONE all_gather_into_tensor of the fixed-size records (8 k bytes per rank);
//   3. shard_hist (every rank, identically): a 32768-bin histogram of key >> 16 over the W * cap
//      gathered entries; the last workgroup to arrive finds the bin B holding the k-th key;
//   4. shard_apply: entries above B are selected, below B rejected; the bin-B entries go to a
//      boundary list and a histogram of their next 11 key bits (sub-bins);
//   5. shard_bnd: the boundary list decided in parallel by that sub-bin; the last workgroup ranks
//      the few entries in the cut's sub-bin exactly by (key, global index).
//      A selected entry is written to the dense output (0 + v); an own entry the global cut rejects
//      gets its t back in the residual (r' = v: the engine had zeroed it), and pay_idx marks this
//      rank's record entries with their global index (selected) or -1.
// No sample exchange, no capacity guess and no bracket-miss protocol: the record capacity is k
// (a rank can hold at most k of the global top-k), and a degenerate local bucket is handled inside
// the local engine's own exact fallback.  The partition (shard lengths) is agreed on a name's first
// step; each record header carries its shard length and shard_hist checks it against the agreed
// table, setting bit 1 of the caller's pinned status word on a mismatch (sharded.py raises at the
// next step, or redoes the step exactly with check_sizes=True).
#include "common.h"
#include "select.h"

namespace grace {

constexpr int kShHdr = 8;            // record header words: [0] = this rank's shard length
constexpr int kShBlock = 1024;
constexpr int kShPer = 4;            // entries per thread per round (all loads before any use)
constexpr int kShBins = 32768;       // key >> 16: 1/128-octave bins
constexpr int kShMaxWorld = 1024;
constexpr int kShMaxGrid = 512;
constexpr unsigned kShHistGrid = 32;
constexpr int kShSub = 2048;         // boundary sub-bins: key bits 15..5 of the bin-B entries
constexpr int kShTakePer = 8;        // last arriver: boundary entries per thread per round
constexpr int kShPairCap = 1024;     // sub-bin entries ranked pairwise
constexpr int64_t kShBndGrid = 64;   // shard_bnd workgroups at most

// Diagnostic build only (-DGRACE_STAMPS): s_memrealtime stamps (100 MHz) in the free tail of the
// 256-byte ctl block (slots 0..23).  Never in shipped builds.
#ifdef GRACE_STAMPS
#define SH_STAMP(cond, ctlp, slot)                                                                         \
  do {                                                                                                     \
    if (threadIdx.x == 0 && (cond))                                                                        \
      reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(ctlp) + 64)[slot] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define SH_STAMP(cond, ctlp, slot) do { } while (0)
#endif

struct ShCtl {
  int32_t b1;        // boundary bin; -1 = every valid entry is selected
  uint32_t above;    // valid entries in bins above b1
  uint32_t need;     // entries still to take from bin b1
  uint32_t ticket1;  // shard_hist arrivals (reset by the last)
  uint32_t ticket2;  // shard_apply arrivals (reset by the last)
  uint32_t nb;       // boundary-list fill counter (reset by the last shard_bnd)
  uint32_t ticket3;  // shard_bnd / shard_fused arrivals (reset by the last)
  uint32_t n2;       // cut-sub-bin list fill counter (reset by the last shard_bnd / shard_fused)
  uint32_t bar_count, bar_gen;   // shard_fused grid barrier
  uint32_t pad[6];
};
static_assert(sizeof(ShCtl) == 64, "ShCtl layout");

struct ShArgs {
  const int32_t* recs;  // W gathered records, `stride` words each
  int64_t stride, cap;
  int32_t world, rank;
  const int64_t* tab;   // device [m_0 .. m_{W-1}, base_0 .. base_{W-1}]: the agreed partition
  int64_t k;
  float* r;             // this rank's residual shard
  float* out;           // dense output, zero-filled, global range [out_base, out_base + out_len)
  int64_t out_base, out_len;
  int32_t* pay_idx;     // this rank's record entries: global index if selected, -1 otherwise
  int32_t* sel_gi;      // optional [world * cap]: every entry's global index if selected, else -1
                        // (the positions the next step clears in a recycled output)
  ShCtl* ctl;
  uint32_t* hist;       // [kShBins], left zeroed
  uint32_t* hist2;      // [kShSub] sub-bin histogram of the boundary entries, left zeroed
  uint32_t* bnd;        // boundary list of entry numbers [world * cap]
  uint32_t* bnd2;       // entries of the cut's sub-bin [world * cap]
  int32_t* status;      // pinned host word (system-scope fetch_or), may be null
};

__device__ __forceinline__ const float* rec_vals(const ShArgs& a, uint32_t w) {
  return reinterpret_cast<const float*>(a.recs + (int64_t)w * a.stride + kShHdr);
}
__device__ __forceinline__ const int32_t* rec_idx(const ShArgs& a, uint32_t w) {
  return a.recs + (int64_t)w * a.stride + kShHdr + a.cap;
}

// entry number e -> (rank w, slot j); N = world * cap < 2^31 (checked on the host)
__device__ __forceinline__ void split_entry(uint32_t e, uint32_t cap, uint32_t& w, uint32_t& j) {
  w = e / cap;
  j = e - w * cap;
}

// 3. the histogram of key >> 16 over the gathered entries; the last arriver finds bin B
__global__ __launch_bounds__(kShBlock) void shard_hist_kernel(ShArgs a) {
  __shared__ uint32_t h[kShBins + kShBins / 32];   // hist_pad layout (select.h)
  __shared__ uint32_t s_w[kShBlock / kWave + 1];
  __shared__ uint32_t s_res[2];
  __shared__ uint32_t s_last;
  const int t = threadIdx.x;
  SH_STAMP(blockIdx.x == 0, a.ctl, 0);
  for (int b = t; b < kShBins + kShBins / 32; b += kShBlock) h[b] = 0u;
  __syncthreads();
  const uint32_t cap = (uint32_t)a.cap, N = (uint32_t)a.world * cap;
  const uint32_t step = gridDim.x * kShBlock * kShPer;
  for (uint32_t e0 = blockIdx.x * kShBlock * kShPer + t; e0 < N; e0 += step) {
    int32_t li[kShPer];
    float v[kShPer];
#pragma unroll
    for (int u = 0; u < kShPer; ++u) {
      const uint32_t e = e0 + u * kShBlock;
      uint32_t w, j;
      split_entry(e < N ? e : e0, cap, w, j);
      li[u] = rec_idx(a, w)[j];
      v[u] = rec_vals(a, w)[j];
    }
#pragma unroll
    for (int u = 0; u < kShPer; ++u)
      if (e0 + u * kShBlock < N && li[u] >= 0) atomicAdd(&h[hist_pad(abs_key(v[u]) >> 16)], 1u);
  }
  __syncthreads();
  SH_STAMP(blockIdx.x == 0, a.ctl, 1);
  for (int b = t; b < kShBins; b += kShBlock) {
    const uint32_t c = h[hist_pad(b)];
    if (c) atomicAdd(&a.hist[b], c);
  }
  // arrival (DESIGN §4 memory-model table, row 1: device atomics, vmcnt(0), barrier, one ticket)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  SH_STAMP(blockIdx.x == 0, a.ctl, 2);
  if (t == 0) s_last = atomicAdd(&a.ctl->ticket1, 1u) == gridDim.x - 1 ? 1u : 0u;
  __syncthreads();
  if (!s_last) return;
  SH_STAMP(true, a.ctl, 3);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // several workgroups per CU possible: keep the acquire
  // last workgroup (after the acquire): the merged histogram into LDS with every 16-B load in
  // flight at once (one agent-scope atomic load per bin was a chain of 32 round trips per thread),
  // the global one re-zeroed
  constexpr int kV = kShBins / 4 / kShBlock;
  uint4* hg = reinterpret_cast<uint4*>(a.hist);
  uint4 hv[kV];
#pragma unroll
  for (int u = 0; u < kV; ++u) hv[u] = hg[t + u * kShBlock];
  uint32_t tot = 0;
#pragma unroll
  for (int u = 0; u < kV; ++u) {
    const int b0 = hist_pad(4 * (t + u * kShBlock));   // 4 bins never straddle a pad word
    h[b0] = hv[u].x;
    h[b0 + 1] = hv[u].y;
    h[b0 + 2] = hv[u].z;
    h[b0 + 3] = hv[u].w;
    tot += hv[u].x + hv[u].y + hv[u].z + hv[u].w;
    hg[t + u * kShBlock] = make_uint4(0u, 0u, 0u, 0u);
  }
  uint32_t total;
  block_excl_scan<kShBlock>(tot, s_w, &total);   // also a barrier: h complete
  const uint32_t k = (uint32_t)a.k;
  int b1 = -1;
  uint32_t above = total;
  if (total > k) {
    const uint32_t rank[1] = {k};
    int d[1];
    uint32_t ab[1];
    find_bins_desc<kShBlock, kShBins, 1, true>(h, rank, s_w, s_res, d, ab);
    b1 = d[0];
    above = ab[0];
  }
  if (t == 0) {
    a.ctl->b1 = b1;
    a.ctl->above = above;
    a.ctl->need = b1 < 0 ? 0u : k - above;
    a.ctl->ticket1 = 0u;
  }
  // the partition every rank planned with vs the shard lengths the records carry
  uint32_t bad = 0;
  for (int w = t; w < a.world; w += kShBlock)
    if ((int64_t)(uint32_t)a.recs[(int64_t)w * a.stride] != a.tab[w]) bad = 1u;
  if (total < k) bad |= 2u;   // fewer valid entries than k (only after a repartition)
  bad = __ballot(bad & 1u) ? 1u : 0u;
  if (a.status && (t & 63) == 0 && bad) __hip_atomic_fetch_or(a.status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (a.status && t == 0 && total < k) __hip_atomic_fetch_or(a.status, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  SH_STAMP(true, a.ctl, 4);
}

// the decision for one entry: dense output, and for this rank's entries pay_idx and the residual
__device__ __forceinline__ void shard_take(const ShArgs& a, bool sel, uint32_t w, uint32_t j, int32_t li, float v,
                                           int64_t gbase) {
  const int64_t gi = gbase + li;
  if (sel) {
    const int64_t o = gi - a.out_base;
    if (o >= 0 && o < a.out_len) a.out[o] = 0.f + v;
  }
  if ((int32_t)w == a.rank) {
    a.pay_idx[j] = sel ? (int32_t)gi : -1;
    if (!sel) a.r[li] = v;   // the local engine zeroed it (r' = t - t); the global cut rejects it: r' = t
  }
  if (a.sel_gi) a.sel_gi[(int64_t)w * a.cap + j] = sel ? (int32_t)gi : -1;
}
// a padding entry (idx -1: a shard shorter than cap)
__device__ __forceinline__ void shard_pad(const ShArgs& a, uint32_t w, uint32_t j) {
  shard_pad(a, w, j);
  if (a.sel_gi) a.sel_gi[(int64_t)w * a.cap + j] = -1;
}

struct BndComp {   // composite key of boundary entry j (plain loads: read after the last arriver's acquire)
  const ShArgs* a;
  const int64_t* base;
  __device__ uint64_t operator()(int64_t jj) const {
    const uint32_t e = a->bnd[jj];
    uint32_t w, j;
    split_entry(e, (uint32_t)a->cap, w, j);
    const int64_t gi = base[w] + rec_idx(*a, w)[j];
    return comp_key(abs_key(rec_vals(*a, w)[j]), (uint32_t)gi);
  }
};

// boundary sub-bin of an entry of bin B: key bits 15..5 (composite bits 47..37)
__device__ __forceinline__ int sub_bin(uint32_t key) { return (int)((key >> 5) & (kShSub - 1)); }

// 4. apply the cut: above B selected, below rejected; the bin-B entries go to the boundary list and
// into a 2048-bin histogram of their next 11 key bits (sub-bins) for shard_bnd.  One level of bins
// (key >> 16, 1/128 octave) leaves thousands of entries in bin B at W = 8 -- the eight local top-k
// lists pile up around the global cut, more so as the residual feedback accumulates -- and ranking
// them in one workgroup by a radix select over indirect loads took 30-120 us.
__global__ __launch_bounds__(kShBlock) void shard_apply_kernel(ShArgs a) {
  __shared__ int64_t s_base[kShMaxWorld];
  __shared__ uint32_t s_h2[kShSub];
  __shared__ uint32_t s_bnd[kShBlock * kShPer];   // this round's boundary entries, staged
  __shared__ uint32_t s_cnt, s_gbase;
  const int t = threadIdx.x;
  for (int w = t; w < a.world; w += kShBlock) s_base[w] = a.tab[a.world + w];
  for (int b = t; b < kShSub; b += kShBlock) s_h2[b] = 0u;
  SH_STAMP(blockIdx.x == 0, a.ctl, 5);
  const int32_t b1 = a.ctl->b1;         // written by shard_hist (kernel boundary)
  const uint32_t need = a.ctl->need;
  if (t == 0) s_cnt = 0u;
  __syncthreads();
  const uint32_t cap = (uint32_t)a.cap, N = (uint32_t)a.world * cap;
  const uint32_t step = gridDim.x * kShBlock * kShPer;
  // uniform rounds (the workgroup barriers below): every thread runs every round
  for (uint32_t r0 = blockIdx.x * kShBlock * kShPer; r0 < N; r0 += step) {
    const uint32_t e0 = r0 + t;
    int32_t li[kShPer];
    float v[kShPer];
#pragma unroll
    for (int u = 0; u < kShPer; ++u) {
      const uint32_t e = e0 + u * kShBlock;
      uint32_t w, j;
      split_entry(e < N ? e : N - 1, cap, w, j);
      li[u] = rec_idx(a, w)[j];
      v[u] = rec_vals(a, w)[j];
    }
#pragma unroll
    for (int u = 0; u < kShPer; ++u) {
      const uint32_t e = e0 + u * kShBlock;
      bool inb = false;
      if (e < N) {
        uint32_t w, j;
        split_entry(e, cap, w, j);
        if (li[u] < 0) {
          shard_pad(a, w, j);
        } else {
          const uint32_t key = abs_key(v[u]);
          const int kb = (int)(key >> 16);
          inb = kb == b1;
          if (inb) atomicAdd(&s_h2[sub_bin(key)], 1u);
          else shard_take(a, kb > b1, w, j, li[u], v[u], s_base[w]);
        }
      }
      // boundary entries staged in LDS (one LDS atomic per wave); the round's list leaves with ONE
      // global reservation per workgroup (a device atomic per wave on the one counter serialised
      // thousands of round trips)
      const uint64_t m = __ballot(inb);
      if (m) {
        uint32_t base0 = 0;
        if (lane_rank(m) == 0 && inb) base0 = atomicAdd(&s_cnt, (uint32_t)__popcll(m));
        base0 = __shfl(base0, __builtin_ctzll(m), 64);
        if (inb) s_bnd[base0 + lane_rank(m)] = e;
      }
    }
    __syncthreads();
    const uint32_t cnt = s_cnt;
    if (t == 0 && cnt) s_gbase = atomicAdd(&a.ctl->nb, cnt);
    __syncthreads();
    // write-through (sc1) stores for the last arriver
    for (uint32_t q = t; q < cnt; q += kShBlock)
      __hip_atomic_store(&a.bnd[s_gbase + q], s_bnd[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (t == 0) s_cnt = 0u;
    __syncthreads();
  }
  for (int b = t; b < kShSub; b += kShBlock) {   // the sub-bin counts (device atomics)
    const uint32_t c = s_h2[b];
    if (c) atomicAdd(&a.hist2[b], c);
  }
  SH_STAMP(blockIdx.x == 0, a.ctl, 6);
}

// 5. the boundary list in parallel: every workgroup finds the sub-bin B2 holding the cut from the
// (kernel-boundary complete) sub-bin histogram -- identically -- and decides its slice of the list:
// above / below B2 at once, B2's entries to a second list (one reservation per workgroup and round);
// the last workgroup to arrive ranks those pairwise by the composite (key, global index).  One
// workgroup walking a list of tens of thousands of entries (the local top-k lists pile up around
// the global cut as the residual feedback accumulates) took 30-70 us.
__global__ __launch_bounds__(kShBlock) void shard_bnd_kernel(ShArgs a) {
  __shared__ int64_t s_base[kShMaxWorld];
  __shared__ uint32_t hsel[2048];
  __shared__ uint32_t s_h2[kShSub];
  __shared__ uint32_t s_stage[kShBlock * kShTakePer];
  __shared__ uint64_t s_comp[kShPairCap];
  __shared__ uint32_t s_ent[kShPairCap];
  __shared__ uint32_t s_cnt, s_gbase;
  __shared__ uint32_t s_w[kShBlock / kWave + 1];
  __shared__ uint32_t s_res[2];
  __shared__ uint32_t s_last;
  const int t = threadIdx.x;
  for (int w = t; w < a.world; w += kShBlock) s_base[w] = a.tab[a.world + w];
  SH_STAMP(blockIdx.x == 0, a.ctl, 7);
  for (int b = t; b < kShSub; b += kShBlock) s_h2[b] = a.hist2[b];
  const uint32_t nb = a.ctl->nb, need = a.ctl->need;   // kernel boundary: plain loads
  const int32_t b1 = a.ctl->b1;
  if (t == 0) s_cnt = 0u;
  __syncthreads();
  int b2 = kShSub;        // need == 0: every boundary entry is rejected
  uint32_t need2 = 0;
  if (need >= nb) {
    b2 = -1;              // every boundary entry is selected
  } else if (need > 0) {
    const uint32_t rank[1] = {need};
    int d[1];
    uint32_t ab[1];
    find_bins_desc<kShBlock, kShSub, 1>(s_h2, rank, s_w, s_res, d, ab);
    b2 = d[0];
    need2 = need - ab[0];
  }
  SH_STAMP(blockIdx.x == 0, a.ctl, 8);
  const uint32_t cap = (uint32_t)a.cap;
  const uint32_t step = gridDim.x * kShBlock * kShTakePer;
  for (uint32_t r0 = blockIdx.x * kShBlock * kShTakePer; r0 < nb; r0 += step) {   // uniform rounds
    const uint32_t j0 = r0 + t;
    uint32_t e[kShTakePer];
#pragma unroll
    for (int u = 0; u < kShTakePer; ++u) {
      const uint32_t jj = j0 + u * kShBlock;
      e[u] = a.bnd[jj < nb ? jj : nb - 1];
    }
    int32_t li[kShTakePer];
    float v[kShTakePer];
#pragma unroll
    for (int u = 0; u < kShTakePer; ++u) {
      uint32_t w, j;
      split_entry(e[u], cap, w, j);
      li[u] = rec_idx(a, w)[j];
      v[u] = rec_vals(a, w)[j];
    }
#pragma unroll
    for (int u = 0; u < kShTakePer; ++u) {
      bool in2 = false;
      if (j0 + u * kShBlock < nb) {
        uint32_t w, j;
        split_entry(e[u], cap, w, j);
        const int sb = sub_bin(abs_key(v[u]));
        in2 = sb == b2;
        if (!in2) shard_take(a, sb > b2, w, j, li[u], v[u], s_base[w]);
      }
      const uint64_t m = __ballot(in2);
      if (m) {
        uint32_t base0 = 0;
        if (lane_rank(m) == 0 && in2) base0 = atomicAdd(&s_cnt, (uint32_t)__popcll(m));
        base0 = __shfl(base0, __builtin_ctzll(m), 64);
        if (in2) s_stage[base0 + lane_rank(m)] = e[u];
      }
    }
    __syncthreads();
    const uint32_t cnt = s_cnt;
    if (t == 0 && cnt) s_gbase = atomicAdd(&a.ctl->n2, cnt);
    __syncthreads();
    for (uint32_t q = t; q < cnt; q += kShBlock)   // write-through (sc1) for the last arriver
      __hip_atomic_store(&a.bnd2[s_gbase + q], s_stage[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (t == 0) s_cnt = 0u;
    __syncthreads();
  }
  // arrival (DESIGN §4 memory-model table, row 1: write-through stores, vmcnt(0), barrier, ticket)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  SH_STAMP(blockIdx.x == 0, a.ctl, 9);
  if (t == 0) s_last = atomicAdd(&a.ctl->ticket3, 1u) == gridDim.x - 1 ? 1u : 0u;
  __syncthreads();
  if (!s_last) return;
  SH_STAMP(true, a.ctl, 10);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // several workgroups per CU possible: keep the acquire
  const uint32_t n2 = __hip_atomic_load(&a.ctl->n2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (n2 <= (uint32_t)kShPairCap) {
    // rank the cut sub-bin's entries pairwise (unique composites): the need2 highest are selected
    for (uint32_t q = t; q < n2; q += kShBlock) {
      const uint32_t e = a.bnd2[q];
      uint32_t w, j;
      split_entry(e, cap, w, j);
      s_ent[q] = e;
      s_comp[q] = comp_key(abs_key(rec_vals(a, w)[j]), (uint32_t)(s_base[w] + rec_idx(a, w)[j]));
    }
    __syncthreads();
    for (uint32_t q = t; q < n2; q += kShBlock) {
      const uint64_t me = s_comp[q];
      uint32_t rk = 0;
      for (uint32_t o = 0; o < n2; ++o) rk += s_comp[o] > me;
      uint32_t w, j;
      split_entry(s_ent[q], cap, w, j);
      shard_take(a, rk < need2, w, j, rec_idx(a, w)[j], rec_vals(a, w)[j], s_base[w]);
    }
  } else {
    // massive ties (more than kShPairCap entries share key bits 31..5): exact radix select over
    // the whole boundary list, then every boundary entry decided again by T (the decisions above
    // stand: T agrees with them, so those writes repeat)
    const BndComp src{&a, s_base};
    const uint64_t p0 = ((uint64_t)(uint32_t)b1 << 48) & (0x7FFull << 53);
    const uint64_t T = block_select_comp<kShBlock>(src, (int64_t)nb, need, hsel, s_w, s_res, 1, p0, 0x7FFull << 53);
    for (uint32_t jj = t; jj < nb; jj += kShBlock) {
      const uint32_t e = a.bnd[jj];
      uint32_t w, j;
      split_entry(e, cap, w, j);
      const int32_t li = rec_idx(a, w)[j];
      const float v = rec_vals(a, w)[j];
      const int64_t gi = s_base[w] + li;
      shard_take(a, comp_key(abs_key(v), (uint32_t)gi) >= T, w, j, li, v, s_base[w]);
    }
  }
  // every workgroup has read the sub-bin histogram (they all arrived): re-zero it for the next call
  for (int b = t; b < kShSub; b += kShBlock) a.hist2[b] = 0u;
  if (t == 0) {
#ifdef GRACE_STAMPS
    reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(a.ctl) + 64)[2 * 12] = nb;   // slot 12: nb, n2
    reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(a.ctl) + 64)[2 * 12 + 1] = n2;
#endif
    a.ctl->nb = 0u;
    a.ctl->n2 = 0u;
    a.ctl->ticket3 = 0u;
  }
  SH_STAMP(true, a.ctl, 11);
}

// ---- the whole select in ONE launch for a co-resident grid (every workgroup resident at once,
// checked on the host): each thread keeps its PER entries in registers through three phases
// separated by grid barriers, so no list is written or re-read except the cut's last few entries.
//   1. a 2048-bin histogram of key >> 20 (1/8 octave) -> device atomics -> barrier;
//   2. every workgroup reads the merged histogram (agent-scope loads) and finds the bin C1 holding
//      the k-th key (identically); its entries above C1 are selected, below rejected; the C1 ones are
//      counted by key bits 19..9 (2048 sub-bins) -> device atomics -> barrier;
//   3. every workgroup finds the sub-bin B2 of the cut the same way and decides its C1 entries; the
//      entries of B2 itself (sharing key bits 31..9: a handful) go to a write-through list, and the
//      last workgroup to arrive ranks them by the composite (key, global index).
// Three launches with a 32768-bin first level (its zeroing, flush and single-workgroup scan) and a
// boundary list walked after a kernel boundary cost 55 us per rank at W = 8; the waits here are
// bounded (a run-out sets status bit 3 and the host raises).
constexpr uint32_t kShSpinMax = 1u << 24;
#ifndef GRACE_SHARD_PER
#define GRACE_SHARD_PER 4   // entries per thread of the one-launch select (A/B knob; 16 is the fallback)
#endif

// Same-address device atomics serialise: one barrier counter (or one histogram copy) that every
// one of 132 workgroups adds to cost ~6 us per barrier.  So the workgroups arrive in 8 groups
// (blockIdx % 8: one XCD each under round-robin dispatch), the last of each group arrives at the
// top counter, and the histograms are kept as 8 copies that every reader sums.
constexpr int kShGroups = 8;
static_assert(2 * kShGroups * 2048 <= kShBins, "the histogram copies fit the first-level histogram's space");

__device__ __forceinline__ void sh_grid_barrier(const ShArgs& a, uint32_t nblocks) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t* grp = a.hist2;                 // group counters [0, 8) and the top counter [8]
    const uint32_t g = blockIdx.x % kShGroups;
    const uint32_t in_g = (nblocks - g + kShGroups - 1) / kShGroups;
    const uint32_t ngroups = nblocks < (uint32_t)kShGroups ? nblocks : (uint32_t)kShGroups;
    const uint32_t gen = __hip_atomic_load(&a.ctl->bar_gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (atomicAdd(grp + g, 1u) == in_g - 1) {
      __hip_atomic_store(grp + g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (atomicAdd(grp + kShGroups, 1u) == ngroups - 1) {
        __hip_atomic_store(grp + kShGroups, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(&a.ctl->bar_gen, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    uint32_t spins = 0;
    while (__hip_atomic_load(&a.ctl->bar_gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gen) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > kShSpinMax) {   // never expected (co-resident grid): flag, do not hang
        if (a.status) __hip_atomic_fetch_or(a.status, 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
  }
  __syncthreads();
}

// the 8 copies of a merged 2048-bin histogram summed into LDS (agent-scope loads: other XCDs'
// atomics) and the bin holding the rank-th largest (descending); returns the bin (-1 if fewer than
// `rank` entries) and the count above it
__device__ __forceinline__ int sh_find(const uint32_t* gh, uint32_t* hl, uint32_t rank, uint32_t* s_w,
                                       uint32_t* s_res, uint32_t& above, uint32_t& total) {
  for (int b = threadIdx.x; b < 2048; b += kShBlock) {
    uint32_t c[kShGroups];
#pragma unroll
    for (int q = 0; q < kShGroups; ++q) c[q] = __hip_atomic_load(gh + q * 2048 + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t sum = 0;
#pragma unroll
    for (int q = 0; q < kShGroups; ++q) sum += c[q];
    hl[b] = sum;
  }
  __syncthreads();
  uint32_t c = 0;
  for (int b = threadIdx.x; b < 2048; b += kShBlock) c += hl[b];
  block_excl_scan<kShBlock>(c, s_w, &total);
  if (rank == 0 || total < rank) { above = total; return rank == 0 ? 2048 : -1; }
  const uint32_t r1[1] = {rank};
  int d[1];
  uint32_t ab[1];
  find_bins_desc<kShBlock, 2048, 1>(hl, r1, s_w, s_res, d, ab);
  above = ab[0];
  return d[0];
}

template <int PER>
__global__ __launch_bounds__(kShBlock) void shard_fused_kernel(ShArgs a) {
  __shared__ int64_t s_base[kShMaxWorld];
  __shared__ uint32_t hl[2048];
  __shared__ uint32_t hsel[2048];
  __shared__ uint32_t s_stage[kShBlock * PER];
  __shared__ uint64_t s_comp[kShPairCap];
  __shared__ uint32_t s_ent[kShPairCap];
  __shared__ uint32_t s_w[kShBlock / kWave + 1];
  __shared__ uint32_t s_res[2];
  __shared__ uint32_t s_cnt, s_gbase, s_last;
  const int t = threadIdx.x;
  const uint32_t nblk = gridDim.x;
  SH_STAMP(blockIdx.x == 0, a.ctl, 0);
  for (int w = t; w < a.world; w += kShBlock) s_base[w] = a.tab[a.world + w];
  for (int b = t; b < 2048; b += kShBlock) hl[b] = 0u;
  if (t == 0) s_cnt = 0u;
  const uint32_t cap = (uint32_t)a.cap, N = (uint32_t)a.world * cap;
  const uint32_t e0 = blockIdx.x * kShBlock * PER + t;
  int32_t li[PER];
  float v[PER];
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const uint32_t e = e0 + u * kShBlock;
    uint32_t w, j;
    split_entry(e < N ? e : N - 1, cap, w, j);
    li[u] = rec_idx(a, w)[j];
    v[u] = rec_vals(a, w)[j];
  }
  __syncthreads();
  uint32_t valid = 0;
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const uint32_t e = e0 + u * kShBlock;
    if (e < N) {
      if (li[u] >= 0) {
        valid |= 1u << u;
        atomicAdd(&hl[abs_key(v[u]) >> 20], 1u);
      } else {
        uint32_t w, j;
        split_entry(e, cap, w, j);
        shard_pad(a, w, j);
      }
    }
  }
  __syncthreads();
  uint32_t* hcopy = a.hist + (blockIdx.x % kShGroups) * 2048;        // coarse copies: hist[0, 16384)
  uint32_t* scopy = a.hist + (kShGroups + blockIdx.x % kShGroups) * 2048;   // sub-bin copies: hist[16384, 32768)
  for (int b = t; b < 2048; b += kShBlock)
    if (hl[b]) atomicAdd(&hcopy[b], hl[b]);
  SH_STAMP(blockIdx.x == 0, a.ctl, 1);
  sh_grid_barrier(a, nblk);
  SH_STAMP(blockIdx.x == 0, a.ctl, 2);
  // ---- phase 2: the coarse cut
  const uint32_t k = (uint32_t)a.k;
  uint32_t above1, total;
  const int c1 = sh_find(a.hist, hl, k, s_w, s_res, above1, total);   // -1: every valid entry selected
  if (blockIdx.x == 0) {   // the partition every rank planned with vs the shard lengths the records carry
    uint32_t bad = 0;
    for (int w = t; w < a.world; w += kShBlock)
      if ((int64_t)(uint32_t)a.recs[(int64_t)w * a.stride] != a.tab[w]) bad = 1u;
    if (a.status && bad) __hip_atomic_fetch_or(a.status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (a.status && t == 0 && total < k) __hip_atomic_fetch_or(a.status, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __syncthreads();   // every thread has read hl
  for (int b = t; b < 2048; b += kShBlock) hl[b] = 0u;
  __syncthreads();
  // decisions only: the writes wait until after the next barrier, whose vmcnt(0) would otherwise
  // wait for thousands of scattered partial-line stores to complete
  uint32_t inb = 0, sel = 0;
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    if (!((valid >> u) & 1u)) continue;
    const uint32_t key = abs_key(v[u]);
    const int cb = (int)(key >> 20);
    if (cb == c1) {
      inb |= 1u << u;
      atomicAdd(&hl[(key >> 9) & 2047u], 1u);
    } else {
      sel |= (uint32_t)(cb > c1) << u;
    }
  }
  __syncthreads();
  for (int b = t; b < 2048; b += kShBlock)
    if (hl[b]) atomicAdd(&scopy[b], hl[b]);
  SH_STAMP(blockIdx.x == 0, a.ctl, 3);
  sh_grid_barrier(a, nblk);
  SH_STAMP(blockIdx.x == 0, a.ctl, 4);
  // ---- phase 3: the sub-bin cut inside C1
  const uint32_t need = c1 < 0 ? 0u : k - above1;
  uint32_t above2, total2;
  const int b2 = c1 < 0 ? -1 : sh_find(a.hist + kShGroups * 2048, hl, need, s_w, s_res, above2, total2);
  const uint32_t need2 = c1 < 0 ? 0u : need - above2;
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    bool in2 = false;
    if ((valid >> u) & 1u) {
      bool take_sel = (sel >> u) & 1u;
      if ((inb >> u) & 1u) {
        const int sb = (int)((abs_key(v[u]) >> 9) & 2047u);
        in2 = sb == b2;
        take_sel = sb > b2;
      }
      if (!in2) {
        uint32_t w, j;
        split_entry(e0 + u * kShBlock, cap, w, j);
        shard_take(a, take_sel, w, j, li[u], v[u], s_base[w]);
      }
    }
    const uint64_t m = __ballot(in2);
    if (m) {
      uint32_t base0 = 0;
      if (lane_rank(m) == 0 && in2) base0 = atomicAdd(&s_cnt, (uint32_t)__popcll(m));
      base0 = __shfl(base0, __builtin_ctzll(m), 64);
      if (in2) s_stage[base0 + lane_rank(m)] = e0 + u * kShBlock;
    }
  }
  __syncthreads();
  const uint32_t cnt = s_cnt;
  if (t == 0 && cnt) s_gbase = atomicAdd(&a.ctl->n2, cnt);
  __syncthreads();
  for (uint32_t q = t; q < cnt; q += kShBlock)   // write-through (sc1) for the last arriver
    __hip_atomic_store(&a.bnd2[s_gbase + q], s_stage[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // arrival (DESIGN §4 memory-model table, row 1: write-through stores, vmcnt(0), barrier, ticket)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  SH_STAMP(blockIdx.x == 0, a.ctl, 5);
  if (t == 0) s_last = atomicAdd(&a.ctl->ticket3, 1u) == nblk - 1 ? 1u : 0u;
  __syncthreads();
  if (!s_last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // several workgroups per CU possible: keep the acquire
  SH_STAMP(true, a.ctl, 6);
  const uint32_t n2 = __hip_atomic_load(&a.ctl->n2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (n2 <= (uint32_t)kShPairCap) {
    for (uint32_t q = t; q < n2; q += kShBlock) {
      const uint32_t e = a.bnd2[q];
      uint32_t w, j;
      split_entry(e, cap, w, j);
      s_ent[q] = e;
      s_comp[q] = comp_key(abs_key(rec_vals(a, w)[j]), (uint32_t)(s_base[w] + rec_idx(a, w)[j]));
    }
    __syncthreads();
    for (uint32_t q = t; q < n2; q += kShBlock) {
      const uint64_t me = s_comp[q];
      uint32_t rk = 0;
      for (uint32_t o = 0; o < n2; ++o) rk += s_comp[o] > me;
      uint32_t w, j;
      split_entry(s_ent[q], cap, w, j);
      shard_take(a, rk < need2, w, j, rec_idx(a, w)[j], rec_vals(a, w)[j], s_base[w]);
    }
  } else {
    // massive ties (more than kShPairCap entries share key bits 31..9): exact radix select over
    // the cut sub-bin's list
    const uint32_t* lst = a.bnd2;
    const ShArgs* ap = &a;
    const int64_t* bp = s_base;
    auto src = [lst, ap, bp](int64_t jj) {
      const uint32_t e = lst[jj];
      uint32_t w, j;
      split_entry(e, (uint32_t)ap->cap, w, j);
      return comp_key(abs_key(rec_vals(*ap, w)[j]), (uint32_t)(bp[w] + rec_idx(*ap, w)[j]));
    };
    const uint64_t T = block_select_comp<kShBlock>(src, (int64_t)n2, need2, hsel, s_w, s_res);
    for (uint32_t jj = t; jj < n2; jj += kShBlock) {
      const uint32_t e = a.bnd2[jj];
      uint32_t w, j;
      split_entry(e, cap, w, j);
      const int32_t l = rec_idx(a, w)[j];
      const float x = rec_vals(a, w)[j];
      shard_take(a, comp_key(abs_key(x), (uint32_t)(s_base[w] + l)) >= T, w, j, l, x, s_base[w]);
    }
  }
  // every workgroup has read both histograms (they all arrived): re-zero their copies
  for (int b = t; b < 2 * kShGroups * 2048; b += kShBlock) a.hist[b] = 0u;
  if (t == 0) {
    a.ctl->n2 = 0u;
    a.ctl->ticket3 = 0u;
  }
  SH_STAMP(true, a.ctl, 7);
}

// whether `grid` workgroups of shard_fused_kernel<PER> are resident at once: at most one per CU
// (the occupancy API can be one block per CU high, the guide's caveat), cached per device
template <int PER>
static bool sh_fused_fits(int64_t grid) {
  static int cached[64];
  static bool init[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return false;
  if (!init[dev]) {
    int per_cu = 0, cus = 0;
    const bool ok = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, shard_fused_kernel<PER>, kShBlock, 0) == hipSuccess &&
                    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess;
    cached[dev] = ok && per_cu >= 1 ? cus : 0;
    init[dev] = true;
  }
  return grid >= 1 && grid <= cached[dev];
}

// recycled output: zero the previous step's selected positions (its sel_gi list), 8 index loads in
// flight per thread
__global__ __launch_bounds__(256) void shard_clear_kernel(float* __restrict__ out, int64_t out_base, int64_t out_len,
                                                         const int32_t* __restrict__ sel_gi, int64_t count) {
  constexpr int kU = 8;
  for (int64_t j0 = (int64_t)blockIdx.x * 256 * kU + threadIdx.x; j0 < count; j0 += (int64_t)gridDim.x * 256 * kU) {
    int32_t gi[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t j = j0 + (int64_t)u * 256;
      gi[u] = sel_gi[j < count ? j : j0];   // clamped, unconditional
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t o = (int64_t)gi[u] - out_base;
      if (j0 + (int64_t)u * 256 < count && gi[u] >= 0 && o >= 0 && o < out_len) out[o] = 0.f;
    }
  }
}

static size_t sh_ws_bytes(int64_t world, int64_t cap) {
  return 256 + sizeof(uint32_t) * (kShBins + kShSub) + 2 * ((sizeof(uint32_t) * world * cap + 255) & ~(size_t)255);
}

}  // namespace grace

using namespace grace;

extern "C" {

size_t grace_shard_record_words(int64_t cap) { return (size_t)(kShHdr + 2 * cap); }

size_t grace_shard_select_workspace_bytes(int32_t world, int64_t cap) { return sh_ws_bytes(world, cap); }

grace_status_t grace_shard_clear(float* out, int64_t out_base, int64_t out_len, const int32_t* sel_gi, int64_t count,
                                 void* stream) {
  GRACE_REQUIRE(out && sel_gi && out_base >= 0 && out_len >= 0 && count >= 0, "grace_shard_clear: bad arguments");
  if (count == 0) return GRACE_OK;
  int64_t g = (count + 256 * 8 - 1) / (256 * 8);
  g = g > 1024 ? 1024 : g;
  shard_clear_kernel<<<(unsigned)g, 256, 0, as_stream(stream)>>>(out, out_base, out_len, sel_gi, count);
  GRACE_CHECK_LAUNCH("grace_shard_clear");
  return GRACE_OK;
}

grace_status_t grace_shard_select(const int32_t* recs, int32_t world, int32_t rank, int64_t cap, const int64_t* tab,
                                  int64_t k, float* residual, float* out, int64_t out_base, int64_t out_len,
                                  int32_t* pay_idx, int32_t* sel_gi, void* ws, size_t ws_bytes, int32_t* status_host,
                                  void* stream) {
  GRACE_REQUIRE(recs && tab && residual && out && pay_idx && ws && world >= 1 && world <= kShMaxWorld &&
                    rank >= 0 && rank < world && cap >= 1 && k >= 1 && out_base >= 0 && out_len >= 0 &&
                    (int64_t)world * cap < ((int64_t)1 << 31),
                "grace_shard_select: bad arguments");
  GRACE_REQUIRE(ws_bytes >= sh_ws_bytes(world, cap), "grace_shard_select: workspace too small");
  char* p = reinterpret_cast<char*>(ws);
  ShArgs a;
  a.recs = recs;
  a.stride = kShHdr + 2 * cap;
  a.cap = cap;
  a.world = world;
  a.rank = rank;
  a.tab = tab;
  a.k = k;
  a.r = residual;
  a.out = out;
  a.out_base = out_base;
  a.out_len = out_len;
  a.pay_idx = pay_idx;
  a.sel_gi = sel_gi;
  a.ctl = reinterpret_cast<ShCtl*>(p);
  a.hist = reinterpret_cast<uint32_t*>(p + 256);
  a.hist2 = reinterpret_cast<uint32_t*>(p + 256 + sizeof(uint32_t) * kShBins);
  a.bnd = reinterpret_cast<uint32_t*>(p + 256 + sizeof(uint32_t) * (kShBins + kShSub));
  a.bnd2 = a.bnd + (((sizeof(uint32_t) * world * cap + 255) & ~(size_t)255) / sizeof(uint32_t));
  a.status = status_host;
  const int64_t N = (int64_t)world * cap;
  hipStream_t s = as_stream(stream);
#ifndef GRACE_SHARD_3K   // A/B: the three-launch select
  {  // one launch when the grid that holds every entry in registers is co-resident
    constexpr int P0 = GRACE_SHARD_PER;
    const int64_t g4 = (N + kShBlock * P0 - 1) / (kShBlock * P0), g16 = (N + kShBlock * 16 - 1) / (kShBlock * 16);
    if (sh_fused_fits<P0>(g4)) {
      shard_fused_kernel<P0><<<(unsigned)g4, kShBlock, 0, s>>>(a);
      GRACE_CHECK_LAUNCH("grace_shard_select");
      return GRACE_OK;
    }
    if (sh_fused_fits<16>(g16)) {
      shard_fused_kernel<16><<<(unsigned)g16, kShBlock, 0, s>>>(a);
      GRACE_CHECK_LAUNCH("grace_shard_select");
      return GRACE_OK;
    }
  }
#endif
  int64_t g = (N + kShBlock * kShPer - 1) / (kShBlock * kShPer);
  const unsigned grid = (unsigned)(g < 1 ? 1 : (g > kShMaxGrid ? kShMaxGrid : g));
  // the histogram flush's device atomics all land on the few bins around the k-th key: fewer
  // workgroups, each looping over more entries, means fewer atomics per bin
  const unsigned hgrid = grid < kShHistGrid ? grid : kShHistGrid;
  shard_hist_kernel<<<hgrid, kShBlock, 0, s>>>(a);
  GRACE_CHECK_LAUNCH("grace_shard_select");
  shard_apply_kernel<<<grid, kShBlock, 0, s>>>(a);
  GRACE_CHECK_LAUNCH("grace_shard_select");
  // the boundary list's length is on the device: a fixed grid, each workgroup looping
  const int64_t gb = (N + kShBlock * kShTakePer - 1) / (kShBlock * kShTakePer);
  shard_bnd_kernel<<<(unsigned)(gb < 1 ? 1 : (gb > kShBndGrid ? kShBndGrid : gb)), kShBlock, 0, s>>>(a);
  GRACE_CHECK_LAUNCH("grace_shard_select");
  return GRACE_OK;
}

}  // extern "C"
