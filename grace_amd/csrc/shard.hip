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
//                      2048-bin histogram of key bits 19..9 (sub-bins);
//        shard_bnd     every workgroup finds the sub-bin B2 of the cut; the C1 list is decided in
//                      parallel by sub-bin; the few B2 entries (sharing key bits 31..9) are ranked
//                      exactly by the composite (key, global index) by the last arriver.
//      A selected entry is written to the dense output (0 + v); an own entry the global cut rejects
//      gets its t back in the residual (r' = v: the engine had zeroed it), and pay_idx marks this
//      rank's record entries with their global index (selected) or -1.
// Same-address device atomics serialise (~40 ns each): every histogram is kept as 8 copies (one
// per group of workgroups, blockIdx % 8) that its readers sum.  A one-launch variant with two
// software grid barriers measured 30 us against 55 us for an earlier three-launch form, but a
// barrier needs the whole grid resident, and two processes sharing one GPU (or any concurrent
// kernel that fills the CUs) left it waiting on workgroups that could not be scheduled.
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
constexpr int kShTakePer = 8;        // shard_bnd: list entries per thread per round
constexpr int kShPairCap = 1024;     // cut sub-bin entries ranked pairwise
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
  int32_t c1;        // coarse bin of the k-th key; -1 = every valid entry is selected
  uint32_t need;     // entries still to take from bin C1
  uint32_t nb;       // C1 list fill counter (reset by the last shard_bnd)
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
  uint4* bnd;           // C1 entries {entry number, global index, value bits, 0} [world * cap]
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
  for (int b = threadIdx.x; b < kShBins; b += kShBlock) {
    uint32_t c[kShGroups];
#pragma unroll
    for (int q = 0; q < kShGroups; ++q) c[q] = gh[q * kShBins + b];
    uint32_t sum = 0;
#pragma unroll
    for (int q = 0; q < kShGroups; ++q) sum += c[q];
    hl[b] = sum;
  }
  __syncthreads();
  uint32_t c = 0;
  for (int b = threadIdx.x; b < kShBins; b += kShBlock) c += hl[b];
  block_excl_scan<kShBlock>(c, s_w, &total);
  if (rank == 0 || total < rank) { above = total; return rank == 0 ? kShBins : -1; }
  const uint32_t r1[1] = {rank};
  int d[1];
  uint32_t ab[1];
  find_bins_desc<kShBlock, kShBins, 1>(hl, r1, s_w, s_res, d, ab);
  above = ab[0];
  return d[0];
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
#pragma unroll
    for (int u = 0; u < kShPer; ++u)
      if (e0 + u * kShBlock < N && li[u] >= 0) atomicAdd(&hl[coarse_bin(abs_key(v[u]))], 1u);
  }
  __syncthreads();
  flush_copy(a.hist, hl);
  SH_STAMP(blockIdx.x == 0, a.ctl, 1);
}

// 3b. the coarse cut: above C1 selected, below rejected; the C1 entries listed and sub-binned
__global__ __launch_bounds__(kShBlock) void shard_apply_kernel(ShArgs a) {
  __shared__ int64_t s_base[kShMaxWorld];
  __shared__ uint32_t hl[kShBins];
  __shared__ uint4 s_stage[kShBlock * kShPer];      // this round's C1 entries, staged
  __shared__ uint32_t s_w[kShBlock / kWave + 1];
  __shared__ uint32_t s_res[2];
  __shared__ uint32_t s_cnt, s_gbase;
  const int t = threadIdx.x;
  SH_STAMP(blockIdx.x == 0, a.ctl, 2);
  for (int w = t; w < a.world; w += kShBlock) s_base[w] = a.tab[a.world + w];
  const uint32_t k = (uint32_t)a.k;
  uint32_t above, total;
  const int c1 = find_from_copies(a.hist, hl, k, s_w, s_res, above, total);   // -1: every valid entry selected
  if (blockIdx.x == 0) {
    // the partition every rank planned with vs the shard lengths the records carry
    uint32_t bad = 0;
    for (int w = t; w < a.world; w += kShBlock)
      if ((int64_t)(uint32_t)a.recs[(int64_t)w * a.stride] != a.tab[w]) bad = 1u;
    if (a.status && bad) __hip_atomic_fetch_or(a.status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (a.status && t == 0 && total < k) __hip_atomic_fetch_or(a.status, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (t == 0) {   // for shard_bnd (kernel boundary)
      a.ctl->c1 = c1;
      a.ctl->need = c1 < 0 ? 0u : k - above;
    }
  }
  __syncthreads();   // every thread has read hl
  for (int b = t; b < kShBins; b += kShBlock) hl[b] = 0u;
  if (t == 0) s_cnt = 0u;
  __syncthreads();
  const uint32_t cap = (uint32_t)a.cap, N = (uint32_t)a.world * cap;
  // uniform rounds (the workgroup barriers below): every thread runs every round
  for (uint32_t r0 = blockIdx.x * kShBlock * kShPer; r0 < N; r0 += gridDim.x * kShBlock * kShPer) {
    const uint32_t e0 = r0 + t;
    int32_t li[kShPer];
    float v[kShPer];
    load_entries(a, e0, N, li, v);
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
      // C1 entries staged in LDS (one LDS atomic per wave); the round's list leaves with ONE
      // global reservation per workgroup
      const uint64_t m = __ballot(inb);
      if (m) {
        uint32_t base0 = 0;
        if (lane_rank(m) == 0 && inb) base0 = atomicAdd(&s_cnt, (uint32_t)__popcll(m));
        base0 = __shfl(base0, __builtin_ctzll(m), 64);
        if (inb) {
          // the entry with its global index and value: shard_bnd decides it without going back
          // to the records (a dependent load chain per entry)
          const uint32_t w = e / cap;
          s_stage[base0 + lane_rank(m)] = make_uint4(e, (uint32_t)(s_base[w] + li[u]), f2u(v[u]), 0u);
        }
      }
    }
    __syncthreads();
    const uint32_t cnt = s_cnt;
    if (t == 0 && cnt) s_gbase = atomicAdd(&a.ctl->nb, cnt);
    __syncthreads();
    for (uint32_t q = t; q < cnt; q += kShBlock) a.bnd[s_gbase + q] = s_stage[q];   // read after the boundary
    __syncthreads();
    if (t == 0) s_cnt = 0u;
    __syncthreads();
  }
  flush_copy(a.hist2, hl);
  SH_STAMP(blockIdx.x == 0, a.ctl, 3);
}

// 3c. the sub-bin cut over the C1 list in parallel; the last arriver ranks the cut sub-bin
__global__ __launch_bounds__(kShBlock) void shard_bnd_kernel(ShArgs a) {
  __shared__ int64_t s_base[kShMaxWorld];
  __shared__ uint32_t hl[kShBins];
  __shared__ uint32_t s_stage[kShBlock * kShTakePer];
  __shared__ uint64_t s_comp[kShPairCap];
  __shared__ uint32_t s_ent[kShPairCap];
  __shared__ uint32_t s_w[kShBlock / kWave + 1];
  __shared__ uint32_t s_res[2];
  __shared__ uint32_t s_cnt, s_gbase, s_last;
  const int t = threadIdx.x;
  SH_STAMP(blockIdx.x == 0, a.ctl, 4);
  for (int w = t; w < a.world; w += kShBlock) s_base[w] = a.tab[a.world + w];
  const uint32_t nb = a.ctl->nb, need = a.ctl->need;   // kernel boundary: plain loads
  if (t == 0) s_cnt = 0u;
  int b2 = kShBins;       // need == 0: every C1 entry is rejected
  uint32_t need2 = 0;
  if (need >= nb) {
    b2 = -1;              // every C1 entry is selected
    __syncthreads();
  } else if (need > 0) {
    uint32_t above2, total2;
    b2 = find_from_copies(a.hist2, hl, need, s_w, s_res, above2, total2);
    need2 = need - above2;
  } else {
    __syncthreads();
  }
  const uint32_t cap = (uint32_t)a.cap;
  const uint32_t step = gridDim.x * kShBlock * kShTakePer;
  for (uint32_t r0 = blockIdx.x * kShBlock * kShTakePer; r0 < nb; r0 += step) {   // uniform rounds
    const uint32_t j0 = r0 + t;
    uint4 q4[kShTakePer];
#pragma unroll
    for (int u = 0; u < kShTakePer; ++u) {
      const uint32_t jj = j0 + u * kShBlock;
      q4[u] = a.bnd[jj < nb ? jj : nb - 1];
    }
#pragma unroll
    for (int u = 0; u < kShTakePer; ++u) {
      bool in2 = false;
      if (j0 + u * kShBlock < nb) {
        uint32_t w, j;
        split_entry(q4[u].x, cap, w, j);
        const float v = u2f(q4[u].z);
        const int sb = sub_bin(abs_key(v));
        in2 = sb == b2;
        if (!in2) shard_take(a, sb > b2, w, j, (int32_t)((int64_t)q4[u].y - s_base[w]), v, s_base[w]);
      }
      const uint64_t m = __ballot(in2);
      if (m) {
        uint32_t base0 = 0;
        if (lane_rank(m) == 0 && in2) base0 = atomicAdd(&s_cnt, (uint32_t)__popcll(m));
        base0 = __shfl(base0, __builtin_ctzll(m), 64);
        if (in2) s_stage[base0 + lane_rank(m)] = q4[u].x;
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
  SH_STAMP(blockIdx.x == 0, a.ctl, 5);
  if (t == 0) s_last = atomicAdd(&a.ctl->ticket, 1u) == gridDim.x - 1 ? 1u : 0u;
  __syncthreads();
  if (!s_last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // several workgroups per CU possible: keep the acquire
  SH_STAMP(true, a.ctl, 6);
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
    const uint64_t T = block_select_comp<kShBlock>(src, (int64_t)n2, need2, hl, s_w, s_res);
    for (uint32_t jj = t; jj < n2; jj += kShBlock) {
      const uint32_t e = a.bnd2[jj];
      uint32_t w, j;
      split_entry(e, cap, w, j);
      const int32_t l = rec_idx(a, w)[j];
      const float x = rec_vals(a, w)[j];
      shard_take(a, comp_key(abs_key(x), (uint32_t)(s_base[w] + l)) >= T, w, j, l, x, s_base[w]);
    }
  }
  // every launch before has finished and every workgroup of this one has arrived: re-zero the
  // histogram copies and counters for the next call
  for (int b = t; b < kShGroups * kShBins; b += kShBlock) {
    a.hist[b] = 0u;
    a.hist2[b] = 0u;
  }
  if (t == 0) {
#ifdef GRACE_STAMPS
    reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(a.ctl) + 64)[2 * 12] = nb;   // slot 12: nb, n2
    reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(a.ctl) + 64)[2 * 12 + 1] = n2;
#endif
    a.ctl->nb = 0u;
    a.ctl->n2 = 0u;
    a.ctl->ticket = 0u;
  }
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

static size_t sh_list_bytes(int64_t world, int64_t cap) { return (sizeof(uint32_t) * world * cap + 255) & ~(size_t)255; }
static size_t sh_ws_bytes(int64_t world, int64_t cap) {
  return 256 + 2 * sizeof(uint32_t) * kShGroups * kShBins + 5 * sh_list_bytes(world, cap);
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
  a.bnd2 = reinterpret_cast<uint32_t*>(a.bnd) + 4 * (sh_list_bytes(world, cap) / sizeof(uint32_t));
  a.status = status_host;
  const int64_t N = (int64_t)world * cap;
  int64_t g = (N + kShBlock * kShPer - 1) / (kShBlock * kShPer);
  const unsigned grid = (unsigned)(g < 1 ? 1 : (g > kShMaxGrid ? kShMaxGrid : g));
  hipStream_t s = as_stream(stream);
  shard_coarse_kernel<<<grid, kShBlock, 0, s>>>(a);
  GRACE_CHECK_LAUNCH("grace_shard_select");
  shard_apply_kernel<<<grid, kShBlock, 0, s>>>(a);
  GRACE_CHECK_LAUNCH("grace_shard_select");
  // the C1 list's length is on the device: a fixed grid, each workgroup looping
  const int64_t gb = (N + kShBlock * kShTakePer - 1) / (kShBlock * kShTakePer);
  shard_bnd_kernel<<<(unsigned)(gb < 1 ? 1 : (gb > kShBndGrid ? kShBndGrid : gb)), kShBlock, 0, s>>>(a);
  GRACE_CHECK_LAUNCH("grace_shard_select");
  return GRACE_OK;
}

}  // extern "C"
