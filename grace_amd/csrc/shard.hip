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
//   3. grace_shard_select, three launches, identical on every rank, no workgroup ever waits for
//      another (each phase's reduction is read after a kernel boundary, or by a last arriver):
//        shard_coarse  a 2048-bin histogram of key >> 20 (1/8 octave) over the W * cap entries;
//        shard_apply   every workgroup finds the coarse bin C1 of the k-th key from it; entries
//                      above C1 are selected, below rejected; the C1 entries go to a list and a
//                      2048-bin histogram of key bits 19..9 (sub-bins).  The list is kept in blocks:
//                      a round's 4096 entries put their C1 entries, compacted, in the same block of
//                      the list with the count beside it, so no workgroup reserves list space
//                      through a global atomic (r06);
//        shard_bnd     every workgroup finds the sub-bin B2 of the cut; the C1 list is decided in
//                      parallel, one list block per workgroup; the few B2 entries (sharing key bits
//                      31..9) are ranked exactly by the composite (key, global index) by the last
//                      arriver, from whole entries carried in the cut list (no record reads).
//      Each kernel issues its first round's loads before it sums the histogram copies, so the two
//      round trips overlap (r06: 41.5 -> 34.0 us at configs[4], profiles/r06_shard_select_ab.txt).
//      A selected entry is written to the dense output (0 + v); an own entry the global cut rejects
//      gets its t back in the residual (r' = v: the engine had zeroed it), and pay_idx marks this
//      rank's record entries with their global index (selected) or -1.
// Same-address device atomics serialise (~40 ns each): every histogram is kept as 8 copies (one
// per group of workgroups, blockIdx % 8) that its readers sum.  A one-launch variant with two
// software grid barriers measured 30 us against 55 us for an earlier three-launch form, but a
// barrier needs the whole grid resident, and two processes sharing one GPU (or any concurrent
// kernel that fills the CUs) left it waiting on workgroups that could not be scheduled.  A one-launch
// form WITHOUT that hazard (r06: each phase's blocks claimed through a counter by running
// workgroups, a workgroup waiting only on a phase's done count) was bit-exact but slower, 48-49 us
// against 33-34 us: its per-phase claims and done counts are same-address atomics from every
// workgroup (profiles/r06_shard_select_ab.txt), more than the two kernel boundaries it removes.
// No sample exchange, no capacity guess and no bracket-miss protocol: the record capacity is k
// (a rank can hold at most k of the global top-k), and a degenerate local bucket is handled inside
// the local engine's own exact fallback.  The partition (shard lengths) is agreed on a name's first
// step; each record header carries its shard length and shard_apply checks it against the agreed
// table, setting bit 1 of the caller's pinned status word on a mismatch (sharded.py raises at the
// next step, or redoes the step exactly with check_sizes=True).
#include "common.h"
#include "select.h"

namespace grace {

constexpr int kShHdr = 8;            // record header words: [0] = this rank's shard length
constexpr int kShBlock = 1024;
constexpr int kShPer = 4;            // entries per thread per round (all loads before any use)
constexpr int kShBins = 2048;        // coarse bins (key >> 20) and sub-bins (key bits 19..9)
constexpr int kShGroups = 8;         // histogram copies (arrival groups: blockIdx % 8)
constexpr int kShMaxWorld = 1024;
constexpr int kShMaxGrid = 512;
constexpr uint32_t kShListBlock = kShBlock * kShPer;   // one apply round = one block of the C1 list
constexpr int kShPairCap = 1024;     // cut sub-bin entries ranked pairwise

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
  int32_t c1;        // coarse bin of the k-th key; -1 = every valid entry is selected
  uint32_t need;     // entries still to take from bin C1
  uint32_t nb;       // diagnostic builds: the C1 list's length (reset by the last shard_bnd)
  uint32_t n2;       // cut sub-bin list fill counter (reset by the last shard_bnd)
  uint32_t ticket;   // shard_bnd arrivals (reset by the last)
  uint32_t pad[11];
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
  uint32_t* hist;       // [kShGroups][kShBins] coarse copies, left zeroed
  uint32_t* hist2;      // [kShGroups][kShBins] sub-bin copies, left zeroed
  uint4* bnd;           // C1 entries {entry number, global index, value bits, 0} [world * cap], in blocks
                        // of kShListBlock: block b holds bcnt[b] entries from its start
  uint32_t* bcnt;       // [ceil(world * cap / kShListBlock)]
  uint4* bnd2;          // entries of the cut's sub-bin, the same form [world * cap]
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

__device__ __forceinline__ int coarse_bin(uint32_t key) { return (int)(key >> 20); }
__device__ __forceinline__ int sub_bin(uint32_t key) { return (int)((key >> 9) & (kShBins - 1)); }

// the decision for one entry: dense output, for this rank's entries pay_idx and the residual, and
// the entry's selection record
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
  if ((int32_t)w == a.rank) a.pay_idx[j] = -1;
  if (a.sel_gi) a.sel_gi[(int64_t)w * a.cap + j] = -1;
}

// one round of kShPer entries per thread, every load issued before any is used (clamped index)
__device__ __forceinline__ void load_entries(const ShArgs& a, uint32_t e0, uint32_t N, int32_t (&li)[kShPer],
                                             float (&v)[kShPer]) {
#pragma unroll
  for (int u = 0; u < kShPer; ++u) {
    const uint32_t e = e0 + u * kShBlock;
    uint32_t w, j;
    split_entry(e < N ? e : N - 1, (uint32_t)a.cap, w, j);
    li[u] = rec_idx(a, w)[j];
    v[u] = rec_vals(a, w)[j];
  }
}

// this workgroup's LDS counts into its group's copy of a global histogram (device atomics)
__device__ __forceinline__ void flush_copy(uint32_t* gh, const uint32_t* hl) {
  uint32_t* copy = gh + (blockIdx.x % kShGroups) * kShBins;
  for (int b = threadIdx.x; b < kShBins; b += kShBlock)
    if (hl[b]) atomicAdd(&copy[b], hl[b]);
}

// the kShGroups copies of a histogram written by an EARLIER launch, summed into LDS, and the bin
// holding the rank-th largest (descending); -1 if fewer than `rank` counts, kShBins if rank == 0
__device__ __forceinline__ int find_from_copies(const uint32_t* gh, uint32_t* hl, uint32_t rank, uint32_t* s_w,
                                                uint32_t* s_res, uint32_t& above, uint32_t& total) {
  // every copy of both of this thread's bins loaded before any is summed: ONE round trip
  constexpr int PER = kShBins / kShBlock;
  static_assert(kShBins % kShBlock == 0, "whole bins per thread");
  uint32_t c[PER][kShGroups];
#pragma unroll
  for (int p = 0; p < PER; ++p)
#pragma unroll
    for (int q = 0; q < kShGroups; ++q) c[p][q] = gh[q * kShBins + p * kShBlock + threadIdx.x];
  uint32_t mine = 0;
#pragma unroll
  for (int p = 0; p < PER; ++p) {
    uint32_t sum = 0;
#pragma unroll
    for (int q = 0; q < kShGroups; ++q) sum += c[p][q];
    hl[p * kShBlock + threadIdx.x] = sum;
    mine += sum;
  }
  block_excl_scan<kShBlock>(mine, s_w, &total);   // (its barriers also publish hl)
  if (rank == 0 || total < rank) { above = total; return rank == 0 ? kShBins : -1; }
  const uint32_t r1[1] = {rank};
  int d[1];
  uint32_t ab[1];
  find_bins_desc<kShBlock, kShBins, 1>(hl, r1, s_w, s_res, d, ab);
  above = ab[0];
  return d[0];
}

// list entries: plain accesses across a kernel boundary; WT: the cut list, read by the last
// arriver of the SAME launch -- agent-scope atomics (written through, read past the non-coherent
// caches)
template <bool WT>
__device__ __forceinline__ void put_entry(uint4* d, const uint4& q) {
  if constexpr (WT) {
    uint64_t* p = reinterpret_cast<uint64_t*>(d);
    __hip_atomic_store(p, (uint64_t)q.x | ((uint64_t)q.y << 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(p + 1, (uint64_t)q.z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    *d = q;
  }
}
template <bool WT>
__device__ __forceinline__ uint4 get_entry(const uint4* s) {
  if constexpr (WT) {
    const uint64_t* p = reinterpret_cast<const uint64_t*>(s);
    const uint64_t q01 = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t q23 = __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return make_uint4((uint32_t)q01, (uint32_t)(q01 >> 32), (uint32_t)q23, 0u);
  } else {
    return *s;
  }
}

// the coarse histogram of one round of entries (loaded by the caller)
__device__ __forceinline__ void coarse_round(uint32_t e0, uint32_t N, const int32_t (&li)[kShPer],
                                             const float (&v)[kShPer], uint32_t* hl) {
#pragma unroll
  for (int u = 0; u < kShPer; ++u)
    if (e0 + u * kShBlock < N && li[u] >= 0) atomicAdd(&hl[coarse_bin(abs_key(v[u]))], 1u);
}

// the coarse cut over one round = one list block (its entries loaded by the caller): above C1
// selected, below rejected; the C1 entries counted into the LDS sub-bin histogram hl and compacted
// into the same block of the C1 list, their count in bcnt -- no global reservation
__device__ __forceinline__ void apply_round(const ShArgs& a, uint32_t r0, uint32_t N, int c1,
                                            const int32_t (&li)[kShPer], const float (&v)[kShPer],
                                            uint32_t* hl, const int64_t* s_base, uint32_t* s_cnt) {
  const int t = threadIdx.x;
  const uint32_t cap = (uint32_t)a.cap;
  const uint32_t e0 = r0 + t;
  uint32_t off[kShPer];   // this thread's C1 entries: their place in the block
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
        const int cb = coarse_bin(key);
        inb = cb == c1;
        if (inb) atomicAdd(&hl[sub_bin(key)], 1u);
        else shard_take(a, cb > c1, w, j, li[u], v[u], s_base[w]);
      }
    }
    // C1 entries placed by one LDS atomic per wave
    const uint64_t m = __ballot(inb);
    off[u] = ~0u;
    if (m) {
      uint32_t base0 = 0;
      if (lane_rank(m) == 0 && inb) base0 = atomicAdd(s_cnt, (uint32_t)__popcll(m));
      base0 = __shfl(base0, __builtin_ctzll(m), 64);
      if (inb) off[u] = base0 + lane_rank(m);
    }
  }
#pragma unroll
  for (int u = 0; u < kShPer; ++u) {
    if (off[u] != ~0u) {
      // the entry with its global index and value: the sub-bin pass decides it without going back
      // to the records (a dependent load chain per entry)
      const uint32_t e = e0 + u * kShBlock;
      const uint32_t w = e / cap;
      put_entry<false>(&a.bnd[r0 + off[u]], make_uint4(e, (uint32_t)(s_base[w] + li[u]), f2u(v[u]), 0u));
    }
  }
  __syncthreads();
  if (t == 0) {
    a.bcnt[r0 / kShListBlock] = *s_cnt;
#ifdef GRACE_STAMPS
    atomicAdd(&a.ctl->nb, *s_cnt);   // diagnostic: the C1 list's length (ctl slot 12)
#endif
    *s_cnt = 0u;
  }
  __syncthreads();
}

// the sub-bin cut over one block of the C1 list (its count and entries loaded by the caller): the
// entries outside the cut sub-bin b2 decided; the b2 entries appended, whole, to the cut list
// (write-through for the last arriver)
__device__ __forceinline__ void bnd_round(const ShArgs& a, uint32_t cnt_b, const uint4 (&q4)[kShPer], int b2,
                                          const int64_t* s_base, uint32_t* s_cnt, uint32_t* s_gbase) {
  const int t = threadIdx.x;
  const uint32_t cap = (uint32_t)a.cap;
  uint32_t off[kShPer];   // this thread's cut entries: their place in the workgroup's share
#pragma unroll
  for (int u = 0; u < kShPer; ++u) {
    bool in2 = false;
    if (t + u * kShBlock < cnt_b) {
      uint32_t w, j;
      split_entry(q4[u].x, cap, w, j);
      const float v = u2f(q4[u].z);
      const int sb = sub_bin(abs_key(v));
      in2 = sb == b2;
      if (!in2) shard_take(a, sb > b2, w, j, (int32_t)((int64_t)q4[u].y - s_base[w]), v, s_base[w]);
    }
    const uint64_t m = __ballot(in2);
    off[u] = ~0u;
    if (m) {
      uint32_t base0 = 0;
      if (lane_rank(m) == 0 && in2) base0 = atomicAdd(s_cnt, (uint32_t)__popcll(m));
      base0 = __shfl(base0, __builtin_ctzll(m), 64);
      if (in2) off[u] = base0 + lane_rank(m);
    }
  }
  __syncthreads();
  const uint32_t cnt = *s_cnt;
  if (t == 0 && cnt) *s_gbase = atomicAdd(&a.ctl->n2, cnt);
  __syncthreads();
#pragma unroll
  for (int u = 0; u < kShPer; ++u)
    if (off[u] != ~0u) put_entry<true>(&a.bnd2[*s_gbase + off[u]], q4[u]);
  __syncthreads();
  if (t == 0) *s_cnt = 0u;
  __syncthreads();
}

// the last arriver: the cut sub-bin's entries ranked exactly by the composite (key, global index),
// the need2 highest selected; then the sub-bin histogram copies re-zeroed
__device__ __forceinline__ void rank_cut(const ShArgs& a, uint32_t need2, const int64_t* s_base, uint64_t* s_comp,
                                         uint32_t* hl, uint32_t* s_w, uint32_t* s_res) {
  const int t = threadIdx.x;
  const uint32_t cap = (uint32_t)a.cap;
  // the counter and, below, the cut list are read with agent-scope atomic loads (as they were
  // written): no acquire fence on the common path
  const uint32_t n2 = __hip_atomic_load(&a.ctl->n2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // a cut-list entry: its record slot (w, j), local index and value
  auto entry = [&](const uint4& q, uint32_t& w, uint32_t& j, int32_t& l, float& x) {
    split_entry(q.x, cap, w, j);
    l = (int32_t)((int64_t)q.y - s_base[w]);
    x = u2f(q.z);
  };
  if (n2 <= (uint32_t)kShPairCap) {
    // rank pairwise (unique composites); one entry per thread, kept in registers, loaded
    // unconditionally (the list is whole blocks long): in flight with n2
    const uint4 q = get_entry<true>(&a.bnd2[t]);
    if ((uint32_t)t < n2) s_comp[t] = comp_key(abs_key(u2f(q.z)), q.y);
    __syncthreads();
    if ((uint32_t)t < n2) {
      const uint64_t me = s_comp[t];
      uint32_t rk = 0;
      uint32_t o = 0;
      // 8 LDS reads in flight per step (one at a time, the loop waited an LDS latency per entry)
      for (; o + 8 <= n2; o += 8) {
        uint64_t c[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) c[u] = s_comp[o + u];
#pragma unroll
        for (int u = 0; u < 8; ++u) rk += c[u] > me;
      }
      for (; o < n2; ++o) rk += s_comp[o] > me;
      SH_STAMP(true, a.ctl, 13);
      uint32_t w, j;
      int32_t l;
      float x;
      entry(q, w, j, l, x);
      shard_take(a, rk < need2, w, j, l, x, s_base[w]);
    }
  } else {
    // massive ties (more than kShPairCap entries share key bits 31..9): exact radix select over
    // the cut sub-bin's list (plain loads, after the acquire)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    const uint4* lst = a.bnd2;
    auto src = [lst](int64_t jj) {
      const uint4 q = lst[jj];
      return comp_key(abs_key(u2f(q.z)), q.y);
    };
    const uint64_t T = block_select_comp<kShBlock>(src, (int64_t)n2, need2, hl, s_w, s_res);
    for (uint32_t jj = t; jj < n2; jj += kShBlock) {
      const uint4 q = a.bnd2[jj];
      uint32_t w, j;
      int32_t l;
      float x;
      entry(q, w, j, l, x);
      shard_take(a, comp_key(abs_key(x), q.y) >= T, w, j, l, x, s_base[w]);
    }
  }
  SH_STAMP(true, a.ctl, 14);
  for (int b = t; b < kShGroups * kShBins; b += kShBlock) a.hist2[b] = 0u;
  if (t == 0) {
#ifdef GRACE_STAMPS
    reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(a.ctl) + 64)[2 * 12] = a.ctl->nb;   // slot 12: nb, n2
    reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(a.ctl) + 64)[2 * 12 + 1] = n2;
#endif
    a.ctl->nb = 0u;
    a.ctl->n2 = 0u;
  }
}

// the partition every rank planned with vs the shard lengths the records carry (status bit 1),
// and fewer valid entries than k (bit 2)
__device__ __forceinline__ void check_records(const ShArgs& a, uint32_t total) {
  const int t = threadIdx.x;
  uint32_t bad = 0;
  for (int w = t; w < a.world; w += kShBlock)
    if ((int64_t)(uint32_t)a.recs[(int64_t)w * a.stride] != a.tab[w]) bad = 1u;
  if (a.status && bad) __hip_atomic_fetch_or(a.status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (a.status && t == 0 && total < (uint32_t)a.k) __hip_atomic_fetch_or(a.status, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// 3a. the coarse histogram (key >> 20) of the valid gathered entries
__global__ __launch_bounds__(kShBlock) void shard_coarse_kernel(ShArgs a) {
  __shared__ uint32_t hl[kShBins];
  const int t = threadIdx.x;
  SH_STAMP(blockIdx.x == 0, a.ctl, 0);
  for (int b = t; b < kShBins; b += kShBlock) hl[b] = 0u;
  __syncthreads();
  const uint32_t N = (uint32_t)a.world * (uint32_t)a.cap;
  for (uint32_t e0 = blockIdx.x * kShBlock * kShPer + t; e0 < N; e0 += gridDim.x * kShBlock * kShPer) {
    int32_t li[kShPer];
    float v[kShPer];
    load_entries(a, e0, N, li, v);
    coarse_round(e0, N, li, v, hl);
  }
  __syncthreads();
  flush_copy(a.hist, hl);
  SH_STAMP(blockIdx.x == 0, a.ctl, 1);
}

// 3b. the coarse cut: above C1 selected, below rejected; the C1 entries listed and sub-binned
__global__ __launch_bounds__(kShBlock) void shard_apply_kernel(ShArgs a) {
  __shared__ int64_t s_base[kShMaxWorld];
  __shared__ uint32_t hl[kShBins];
  __shared__ uint32_t s_w[kShBlock / kWave + 1];
  __shared__ uint32_t s_res[2];
  __shared__ uint32_t s_cnt;
  const int t = threadIdx.x;
  SH_STAMP(blockIdx.x == 0, a.ctl, 2);
  for (int w = t; w < a.world; w += kShBlock) s_base[w] = a.tab[a.world + w];
  const uint32_t k = (uint32_t)a.k;
  uint32_t above, total;
  const uint32_t N = (uint32_t)a.world * (uint32_t)a.cap;
  // the first round's entries are loaded before the histogram copies: both in flight together
  int32_t li[kShPer];
  float v[kShPer];
  if (blockIdx.x * kShListBlock < N) load_entries(a, blockIdx.x * kShListBlock + t, N, li, v);
  const int c1 = find_from_copies(a.hist, hl, k, s_w, s_res, above, total);   // -1: every valid entry selected
  SH_STAMP(blockIdx.x == 0, a.ctl, 8);
  if (blockIdx.x == 0) {
    check_records(a, total);
    if (t == 0) a.ctl->need = c1 < 0 ? 0u : k - above;   // for shard_bnd (kernel boundary)
  }
  __syncthreads();   // every thread has read hl
  for (int b = t; b < kShBins; b += kShBlock) hl[b] = 0u;
  if (t == 0) s_cnt = 0u;
  __syncthreads();
  // uniform rounds (the workgroup barriers inside): every thread runs every round
  for (uint32_t r0 = blockIdx.x * kShListBlock; r0 < N; r0 += gridDim.x * kShListBlock) {
    if (r0 != blockIdx.x * kShListBlock) load_entries(a, r0 + t, N, li, v);
    apply_round(a, r0, N, c1, li, v, hl, s_base, &s_cnt);
  }
  SH_STAMP(blockIdx.x == 0, a.ctl, 9);
  flush_copy(a.hist2, hl);
  SH_STAMP(blockIdx.x == 0, a.ctl, 3);
}

// 3c. the sub-bin cut over the C1 list in parallel; the last arriver ranks the cut sub-bin
__global__ __launch_bounds__(kShBlock) void shard_bnd_kernel(ShArgs a) {
  static_assert(kShPairCap <= kShBlock, "the pairwise ranking holds one cut entry per thread");
  __shared__ int64_t s_base[kShMaxWorld];
  __shared__ uint32_t hl[kShBins];
  __shared__ uint64_t s_comp[kShPairCap];
  __shared__ uint32_t s_w[kShBlock / kWave + 1];
  __shared__ uint32_t s_res[2];
  __shared__ uint32_t s_cnt, s_gbase, s_last;
  const int t = threadIdx.x;
  SH_STAMP(blockIdx.x == 0, a.ctl, 4);
  for (int w = t; w < a.world; w += kShBlock) s_base[w] = a.tab[a.world + w];
  const uint32_t need = a.ctl->need;   // kernel boundary: plain loads
  if (t == 0) s_cnt = 0u;
  const uint32_t N = (uint32_t)a.world * (uint32_t)a.cap;
  const uint32_t nblk = (N + kShListBlock - 1) / kShListBlock;
  // the first list block is loaded before the histogram copies: both in flight together
  uint32_t cnt_b = 0;
  uint4 q4[kShPer];
  if (blockIdx.x < nblk) {
    cnt_b = a.bcnt[blockIdx.x];
#pragma unroll
    for (int u = 0; u < kShPer; ++u)   // unconditional (the list is whole blocks long)
      q4[u] = a.bnd[blockIdx.x * kShListBlock + t + u * kShBlock];
  }
  // b2: the sub-bin of the cut within C1; kShBins (need == 0): every C1 entry is rejected, -1 (need
  // above the C1 count): every C1 entry is selected
  uint32_t above2, total2;
  const int b2 = find_from_copies(a.hist2, hl, need, s_w, s_res, above2, total2);
  const uint32_t need2 = b2 >= 0 && b2 < kShBins ? need - above2 : 0u;
  SH_STAMP(blockIdx.x == 0, a.ctl, 10);
  for (uint32_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {   // uniform rounds: one list block each
    if (blk != blockIdx.x) {
      cnt_b = a.bcnt[blk];
#pragma unroll
      for (int u = 0; u < kShPer; ++u) q4[u] = a.bnd[blk * kShListBlock + t + u * kShBlock];   // in flight with cnt_b
    }
    bnd_round(a, cnt_b, q4, b2, s_base, &s_cnt, &s_gbase);
  }
  // the coarse histogram's copies were last read by shard_apply: re-zeroed here by every workgroup
  // (the sub-bin copies, read above, by the last arriver)
  for (int b = blockIdx.x * kShBlock + t; b < kShGroups * kShBins; b += gridDim.x * kShBlock) a.hist[b] = 0u;
  // arrival (DESIGN §4 memory-model table, row 1: write-through stores, vmcnt(0), barrier, ticket)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  SH_STAMP(blockIdx.x == 0, a.ctl, 5);
  if (t == 0) s_last = atomicAdd(&a.ctl->ticket, 1u) == gridDim.x - 1 ? 1u : 0u;
  __syncthreads();
  if (!s_last) return;
  SH_STAMP(true, a.ctl, 6);
  rank_cut(a, need2, s_base, s_comp, hl, s_w, s_res);
  if (t == 0) a.ctl->ticket = 0u;
  SH_STAMP(true, a.ctl, 7);
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

// one list (bnd or bnd2, uint4 entries): whole blocks of kShListBlock entries
static size_t sh_list_bytes(int64_t world, int64_t cap) {
  return sizeof(uint4) * kShListBlock * ((world * cap + kShListBlock - 1) / kShListBlock);
}
static size_t sh_bcnt_bytes(int64_t world, int64_t cap) {
  return (sizeof(uint32_t) * ((world * cap + kShListBlock - 1) / kShListBlock) + 255) & ~(size_t)255;
}
static size_t sh_ws_bytes(int64_t world, int64_t cap) {
  return 256 + 2 * sizeof(uint32_t) * kShGroups * kShBins + 2 * sh_list_bytes(world, cap) + sh_bcnt_bytes(world, cap);
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
  a.hist2 = a.hist + kShGroups * kShBins;
  a.bnd = reinterpret_cast<uint4*>(a.hist2 + kShGroups * kShBins);
  a.bnd2 = a.bnd + sh_list_bytes(world, cap) / sizeof(uint4);
  a.bcnt = reinterpret_cast<uint32_t*>(a.bnd2 + sh_list_bytes(world, cap) / sizeof(uint4));
  a.status = status_host;
  const int64_t N = (int64_t)world * cap;
  int64_t g = (N + kShBlock * kShPer - 1) / (kShBlock * kShPer);
  const unsigned grid = (unsigned)(g < 1 ? 1 : (g > kShMaxGrid ? kShMaxGrid : g));
  hipStream_t s = as_stream(stream);
  shard_coarse_kernel<<<grid, kShBlock, 0, s>>>(a);
  GRACE_CHECK_LAUNCH("grace_shard_select");
  shard_apply_kernel<<<grid, kShBlock, 0, s>>>(a);
  GRACE_CHECK_LAUNCH("grace_shard_select");
  // one workgroup per block of the C1 list (the apply's grid)
  shard_bnd_kernel<<<grid, kShBlock, 0, s>>>(a);
  GRACE_CHECK_LAUNCH("grace_shard_select");
  return GRACE_OK;
}

}  // extern "C"
