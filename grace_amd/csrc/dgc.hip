// Deep Gradient Compression (DGC) for CDNA4: sampled threshold + error-feedback memory with
// momentum correction.
//
// Reference semantics (sands-lab/grace):
//   DgcCompressor.compress  grace_dl/dist/compressor/dgc.py:12-43
//     sample 1 % of the elements (uniform indices, with replacement), thr = the k_s-th largest
//     |sample| (k_s = max(1, int(numel * ratio * 0.01))); mask = |t| >= thr; then up to 10 times:
//     selected > 1.3 numel ratio -> thr *= 1.3, selected < 0.7 numel ratio -> thr *= 0.7, else stop;
//     payload = (t[where(mask)], where(mask)) in ascending index order, int64 indices.
//   DgcMemory.compensate / update  grace_dl/dist/memory/dgc.py:15-39
//     r = momentum r + g (first step r = g);  a = a + r (first step a = g);  t = a;
//     after compress: r = r * ~mask, a = a * ~mask (a multiply: masked entries become +-0 / NaN).
//
// The reference re-scans the whole tensor once per threshold adjustment (up to 11 times).  Here
// every threshold the loop could ever visit is known up front -- thr0 * 1.3^a * 0.7^b along the
// 2^10 paths of the loop, computed with the same f32 multiplications in the same order -- so ONE
// pass histograms |t| against that sorted table (binary search in LDS, only for the few elements
// above its smallest entry), a single thread replays the loop on exact counts, and two more
// passes produce the ordered payload (per-chunk counts, then the compaction).
#include <math.h>

#include "common.h"

namespace grace {

constexpr int kDBlock = 256;
constexpr int kDChunk = 4096;          // elements per compaction chunk
constexpr int kDChunkW1 = 16384;       // elements per workgroup of the world-1 speculative pass
constexpr int kDepth = 10;              // dgc.py:26 range(10)
constexpr int kNodes = (1 << (kDepth + 1)) - 1;   // 2047 thresholds the loop can visit
constexpr int kTab = 2048;              // sorted table (padded with +inf)
constexpr int kDQ = 4;                  // quads per thread per round in the streaming passes
typedef float f4d __attribute__((ext_vector_type(4)));

struct DgcMeta {
  uint32_t thr0;      // bits of the sampled threshold
  uint32_t thr;       // bits of the final threshold
  uint32_t total;     // selected count at the final threshold
  uint32_t nan0;      // thr0 is NaN
  uint32_t fix;       // world-1 fused step: the speculative pass at thr0 was wrong, the gated fix-up runs
  uint32_t ticket;    // world-1 fused step: arrivals of the speculative pass (left zeroed)
  uint32_t pad[10];
};
static_assert(sizeof(DgcMeta) == 64, "DgcMeta layout");

constexpr int kLutShift = 18;                         // coarse key bins: 1/32 octave
constexpr int kLut = (0x7F800000 >> kLutShift) + 2;   // every finite / inf key's bin, plus its end

struct DgcWs {
  DgcMeta* meta;
  float* tab;         // [kTab] ascending
  uint32_t* hist;     // [kTab + 1]
  uint16_t* lut;      // [kLut]: table entries with key < (b << kLutShift)
  uint32_t* part;     // [nchunks] counts
  uint32_t* offs;     // [nchunks] exclusive offsets
};

static inline size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

static DgcWs dgc_carve(void* ws, int64_t n) {
  const int64_t nch = (n + kDChunk - 1) / kDChunk;
  char* p = reinterpret_cast<char*>(ws);
  DgcWs w;
  w.meta = reinterpret_cast<DgcMeta*>(p);
  p += 256;
  w.tab = reinterpret_cast<float*>(p);
  p += al256(sizeof(float) * kTab);
  w.hist = reinterpret_cast<uint32_t*>(p);
  p += al256(sizeof(uint32_t) * (kTab + 1));
  w.lut = reinterpret_cast<uint16_t*>(p);
  p += al256(sizeof(uint16_t) * kLut);
  w.part = reinterpret_cast<uint32_t*>(p);
  p += al256(sizeof(uint32_t) * nch);
  w.offs = reinterpret_cast<uint32_t*>(p);
  return w;
}

static size_t dgc_ws_bytes(int64_t n) {
  const int64_t nch = (n + kDChunk - 1) / kDChunk;
  return 256 + al256(sizeof(float) * kTab) + al256(sizeof(uint32_t) * (kTab + 1)) +
         al256(sizeof(uint16_t) * kLut) + 2 * al256(sizeof(uint32_t) * nch);
}

// compensate: r = m r + g (r = g first), a = a + r (a = g first); returns a in `acc`
__device__ __forceinline__ void dgc_comp1(float gv, float& rv, float& av, int has_state, float m) {
  if (has_state) { rv = m * rv + gv; av = av + rv; } else { rv = gv; av = gv; }
}
__device__ __forceinline__ bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// The device generator's sample index j: iid uniform over [0, n) (dgc.py:17-19 draws numel-range
// uniforms).  (A stratified draw, one uniform index per stratum of n / ns elements, made the gather
// SLOWER -- 54.9 vs 42.8 us for 671 K samples of g, r, a: the chip's in-flight gathers then crowd a
// few MB of addresses instead of spreading over every bank; profiles/r05_dgc_ab.txt.)
__device__ __forceinline__ int64_t dgc_sample_index(uint64_t seed, int64_t j, int64_t n) {
  const uint64_t h = ((uint64_t)rand32(seed, (uint64_t)j) << 32) | rand32(seed ^ 0xD6E8FEB86659FD93ull, (uint64_t)j);
  return (int64_t)(((unsigned __int128)h * (uint64_t)n) >> 64);
}

// ------------------------------------------------------------------------------------------------
// sample: |t[idx_j]|, idx from the caller (parity: torch's CPU uniform_(0, numel).long()) or the
// counter-based generator (uniform integer in [0, numel))
__global__ __launch_bounds__(kDBlock) void dgc_sample_kernel(const float* __restrict__ t, int64_t n,
                                                            const int64_t* __restrict__ sidx, uint64_t seed,
                                                            int64_t ns, float* __restrict__ out) {
  for (int64_t j = (int64_t)blockIdx.x * kDBlock + threadIdx.x; j < ns; j += (int64_t)gridDim.x * kDBlock) {
    int64_t i;
    if (sidx) {
      i = sidx[j];
    } else {
      i = dgc_sample_index(seed, j, n);
    }
    out[j] = fabsf(t[i]);
  }
}

// the same sample of the compensated tensor t = a + (m r + g) (t = g on a name's first step), read
// from the memory state BEFORE compensation: the world-1 fused step samples without materialising t
__global__ __launch_bounds__(kDBlock) void dgc_sample_comp_kernel(const float* __restrict__ g,
                                                                 const float* __restrict__ r,
                                                                 const float* __restrict__ a, int has_state,
                                                                 float momentum, int64_t n,
                                                                 const int64_t* __restrict__ sidx, uint64_t seed,
                                                                 int64_t ns, float* __restrict__ out) {
  for (int64_t j = (int64_t)blockIdx.x * kDBlock + threadIdx.x; j < ns; j += (int64_t)gridDim.x * kDBlock) {
    int64_t i;
    if (sidx) {
      i = sidx[j];
    } else {
      i = dgc_sample_index(seed, j, n);
    }
    const float gv = g[i];
    float rv = has_state ? r[i] : 0.f, av = has_state ? a[i] : 0.f;
    dgc_comp1(gv, rv, av, has_state, momentum);
    out[j] = fabsf(av);
  }
}

// ------------------------------------------------------------------------------------------------
// thr0 without the sample's full top-k: torch.topk(samples, k_s)[0].min() (dgc.py:20-21) is the
// k_s-th largest sampled magnitude, or NaN when the sample holds a NaN (topk ranks NaN above
// everything and torch.min propagates it).  Radix select on the magnitude bits (order-preserving for
// sign-clear floats) in three digits, one launch each: 11 bits (30..20), 11 bits (19..9), 9 bits
// (8..0).  Every workgroup loads all of its elements first (one memory latency), histograms those
// that share the digits chosen so far in LDS and adds its non-zero bins to a global histogram with
// agent-scope atomics; after vmcnt(0) it takes a ticket, and the last to arrive reads the histogram
// back (agent-scope loads: the other XCDs' adds are not in its L2), picks the digit holding the
// remaining rank counting down from the top, and re-zeroes what it consumed (the state is left
// zeroed).  No cache-wide fences.  (8 copies of the global histogram, blockIdx % 8, summed by the
// last arriver: no faster -- profiles/r05_dgc_ab.txt.)
constexpr int kKthBlock = 256;
constexpr int kKthBins = 2048;
constexpr int kKthPer = 16;      // elements per thread per round, all loads in flight together
struct KthState {
  uint32_t hist[kKthBins];
  uint32_t prefix;   // the digits chosen so far, in place
  uint32_t kleft;    // the rank still to find among the elements sharing them (1-based)
  uint32_t nan;
  uint32_t ticket;
};

template <int L>
__global__ __launch_bounds__(kKthBlock) void dgc_kth_kernel(const float* __restrict__ x, int64_t ns, uint32_t ks,
                                                            KthState* __restrict__ st, float* __restrict__ out) {
  constexpr int kShift = L == 0 ? 20 : (L == 1 ? 9 : 0);
  constexpr int kBins = L == 2 ? 512 : 2048;
  constexpr int kHi = L == 0 ? 31 : (L == 1 ? 20 : 9);   // bits at and above this must match the prefix
  __shared__ uint32_t h[kKthBins];
  __shared__ uint32_t s_last, s_nan;
  const int t = threadIdx.x;
  for (int b = t; b < kBins; b += kKthBlock) h[b] = 0u;
  if (t == 0) s_nan = 0u;
  const uint32_t pre = L == 0 ? 0u : st->prefix;   // written by the previous launch's last arriver
  __syncthreads();
  uint32_t nan = 0;
  for (int64_t base = (int64_t)blockIdx.x * (kKthBlock * kKthPer); base < ns;
       base += (int64_t)gridDim.x * (kKthBlock * kKthPer)) {
    uint32_t key[kKthPer];
#pragma unroll
    for (int u = 0; u < kKthPer; ++u) {
      const int64_t j = base + u * kKthBlock + t;
      key[u] = j < ns ? abs_key(x[j]) : 0xFFFFFFFFu;   // no magnitude has the sign bit
    }
#pragma unroll
    for (int u = 0; u < kKthPer; ++u) {
      if (key[u] == 0xFFFFFFFFu) continue;
      if constexpr (L == 0) nan |= key[u] > 0x7F800000u;
      if (L == 0 || (key[u] >> kHi) == (pre >> kHi)) atomicAdd(&h[(key[u] >> kShift) & (kBins - 1)], 1u);
    }
  }
  if constexpr (L == 0) { if (nan) s_nan = 1u; }
  __syncthreads();
  for (int b = t; b < kBins; b += kKthBlock)
    if (h[b]) __hip_atomic_fetch_add(&st->hist[b], h[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (L == 0 && t == 0 && s_nan) __hip_atomic_fetch_or(&st->nan, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this workgroup's adds have completed
  __syncthreads();
  if (t == 0) s_last = __hip_atomic_fetch_add(&st->ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                       gridDim.x - 1;
  __syncthreads();
  if (!s_last) return;
  for (int b = t; b < kBins; b += kKthBlock) {
    h[b] = __hip_atomic_load(&st->hist[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (h[b]) __hip_atomic_store(&st->hist[b], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (t >= kWave) return;
  // wave 0: lane l owns bins [l per, (l + 1) per); suffix sums over the lanes find the lane holding
  // the remaining rank, which then walks its bins from the top
  constexpr int per = kBins / kWave;
  const uint32_t kl = L == 0 ? ks : st->kleft;
  uint32_t s = 0;
  for (int b = 0; b < per; ++b) s += h[t * per + b];
  uint32_t suf = s;
  for (int o = 1; o < kWave; o <<= 1) {
    const uint32_t v = __shfl_down(suf, o, kWave);
    if (t + o < kWave) suf += v;
  }
  const uint64_t reach = __ballot(suf >= kl);
  const int owner = 63 - __builtin_clzll(reach);   // lanes 0..owner reach the rank (suffix sums fall with l)
  if (t != owner) return;
  uint32_t rem = kl - (suf - s);
  int bin = per - 1;
  for (; bin > 0; --bin) {
    const uint32_t c = h[t * per + bin];
    if (rem <= c) break;
    rem -= c;
  }
  const uint32_t key = pre | ((uint32_t)(t * per + bin) << kShift);
  if constexpr (L == 2) {
    const uint32_t nn = __hip_atomic_load(&st->nan, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    out[0] = nn ? u2f(0x7FC00000u) : u2f(key);
    __hip_atomic_store(&st->nan, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    st->prefix = 0u;
    st->kleft = 0u;
  } else {
    st->prefix = key;
    st->kleft = rem;
  }
  __hip_atomic_store(&st->ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------------------------------------------
// table: thr0 = min of the top-k_s sampled magnitudes (torch.min propagates NaN), then every
// threshold of the adjustment tree (node = path bits from the root, 1 -> *1.3, 0 -> *0.7, the
// multiplications in loop order), bitonic-sorted ascending; the counts are zeroed.
template <bool GATED = false>
__global__ __launch_bounds__(1024) void dgc_table_kernel(const float* __restrict__ topv, int64_t ks, DgcWs w) {
  if constexpr (GATED) { if (w.meta->fix == 0u) return; }
  __shared__ float s[kTab];
  __shared__ float s_min;
  __shared__ uint32_t s_nan;
  const int t = threadIdx.x;
  float mn = INFINITY;
  uint32_t nan = 0;
  for (int64_t j = t; j < ks; j += 1024) {
    const float v = topv[j];
    if (v != v) nan = 1; else mn = fminf(mn, v);
  }
  // block reduce
  __shared__ float sm[1024 / kWave];
  __shared__ uint32_t sn[1024 / kWave];
  for (int o = 32; o > 0; o >>= 1) mn = fminf(mn, __shfl_xor(mn, o, 64));
  nan = __ballot(nan != 0) != 0;
  if ((t & 63) == 0) { sm[t >> 6] = mn; sn[t >> 6] = nan; }
  __syncthreads();
  if (t == 0) {
    float m = INFINITY;
    uint32_t nn = 0;
    for (int j = 0; j < 1024 / kWave; ++j) { m = fminf(m, sm[j]); nn |= sn[j]; }
    s_min = m;
    s_nan = nn;
    w.meta->thr0 = nn ? 0x7FC00000u : __float_as_uint(m);
    w.meta->nan0 = nn;
  }
  __syncthreads();
  const float thr0 = s_min;
  const float up = 1.3f, down = 0.7f;   // the Python floats as the f32 operands torch multiplies by
  for (int node = t; node < kTab; node += 1024) {
    float x = INFINITY;
    if (node < kNodes) {
      // node in heap order: depth d = floor(log2(node + 1)), path = the d bits below the leading 1
      const uint32_t id = (uint32_t)node + 1u;
      const int d = 31 - __clz(id);
      x = thr0;
      for (int b = d - 1; b >= 0; --b) x = ((id >> b) & 1u) ? x * up : x * down;
    }
    s[node] = x;
  }
  __syncthreads();
  // bitonic sort ascending (kTab = 2048 = 2 x 1024 threads)
  for (int size = 2; size <= kTab; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int e = t; e < kTab / 2; e += 1024) {
        const int lo = 2 * e - (e & (stride - 1));
        const int hi = lo + stride;
        const bool asc = (lo & size) == 0;
        const float a = s[lo], b = s[hi];
        if ((a > b) == asc) { s[lo] = b; s[hi] = a; }
      }
      __syncthreads();
    }
  }
  for (int e = t; e < kTab; e += 1024) w.tab[e] = s[e];
  for (int e = t; e <= kTab; e += 1024) w.hist[e] = 0u;
  // coarse-bin index: lut[b] = number of entries whose key is below b << kLutShift, so an element
  // of coarse bin b has its upper bound in [lut[b], lut[b + 1]] (entries are >= 0 or +inf, or all
  // NaN, which nothing passes)
  for (int b = t; b < kLut; b += 1024) {
    const uint32_t kb = (uint32_t)b << kLutShift;
    int lo = 0, hi = kTab;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (__float_as_uint(s[mid]) < kb) lo = mid + 1; else hi = mid;
    }
    w.lut[b] = (uint16_t)lo;
  }
}

// thr0 alone (the world-1 fused step needs the table only on its fix-up path): min of the top-k_s
// sampled magnitudes, NaN if any is NaN -- dgc_table_kernel's reduction
__global__ __launch_bounds__(1024) void dgc_thr0_kernel(const float* __restrict__ topv, int64_t ks, DgcWs w) {
  __shared__ float sm[1024 / kWave];
  __shared__ uint32_t sn[1024 / kWave];
  const int t = threadIdx.x;
  float mn = INFINITY;
  uint32_t nan = 0;
  for (int64_t j = t; j < ks; j += 1024) {
    const float v = topv[j];
    if (v != v) nan = 1; else mn = fminf(mn, v);
  }
  for (int o = 32; o > 0; o >>= 1) mn = fminf(mn, __shfl_xor(mn, o, 64));
  nan = __ballot(nan != 0) != 0;
  if ((t & 63) == 0) { sm[t >> 6] = mn; sn[t >> 6] = nan; }
  __syncthreads();
  if (t == 0) {
    float m = INFINITY;
    uint32_t nn = 0;
    for (int j = 0; j < 1024 / kWave; ++j) { m = fminf(m, sm[j]); nn |= sn[j]; }
    w.meta->thr0 = nn ? 0x7FC00000u : __float_as_uint(m);
    w.meta->nan0 = nn;
  }
}

// number of table entries <= key (upper bound); NaN compares false -> 0
__device__ __forceinline__ int tab_bin(const float* tab, float key) {
  if (!(key >= tab[0])) return 0;
  int lo = 1, hi = kTab;            // answer in [1, kTab]
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;   // is tab[mid] <= key ?
    if (key >= tab[mid]) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// tab_bin through the coarse-bin index: a binary search over the few entries of the key's 1/32
// octave instead of all 2048 (11 dependent LDS reads per element made the pass 0.94 TB/s)
__device__ __forceinline__ int tab_bin_lut(const float* tab, const uint16_t* lut, float key) {
  const uint32_t b = __float_as_uint(key) >> kLutShift;   // key >= tab[0] >= 0 here
  int lo = lut[b], hi = lut[b + 1];
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (key >= tab[mid]) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// one pass: histogram of |t| over the table (elements below the smallest entry skip the search)
template <bool GATED>
__global__ __launch_bounds__(kDBlock) void dgc_count_kernel(const float* __restrict__ t, int64_t n, DgcWs w) {
  if constexpr (GATED) { if (w.meta->fix == 0u) return; }
  __shared__ float tab[kTab];
  __shared__ uint32_t h[kTab + 1];
  __shared__ uint16_t lut[kLut];
  for (int e = threadIdx.x; e < kTab; e += kDBlock) tab[e] = w.tab[e];
  for (int e = threadIdx.x; e <= kTab; e += kDBlock) h[e] = 0u;
  for (int e = threadIdx.x; e < kLut; e += kDBlock) lut[e] = w.lut[e];
  __syncthreads();
  const float t0 = tab[0];
  const int64_t n4 = n >> 2;
  const bool vec = (reinterpret_cast<uintptr_t>(t) & 15u) == 0;
  const int64_t stride = (int64_t)gridDim.x * kDBlock;
  if (vec) {
    for (int64_t q0 = (int64_t)blockIdx.x * kDBlock + threadIdx.x; q0 < n4; q0 += stride * kDQ) {
      f4d v[kDQ];
#pragma unroll
      for (int u = 0; u < kDQ; ++u) {   // every quad of the round in flight before any is searched
        const int64_t q = q0 + u * stride < n4 ? q0 + u * stride : q0;
        v[u] = __builtin_nontemporal_load(reinterpret_cast<const f4d*>(t) + q);
      }
#pragma unroll
      for (int u = 0; u < kDQ; ++u) {
        if (q0 + u * stride >= n4) break;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float a = fabsf(v[u][j]);
          if (a >= t0) atomicAdd(&h[tab_bin_lut(tab, lut, a)], 1u);
        }
      }
    }
  }
  for (int64_t i = (vec ? n4 * 4 : 0) + (int64_t)blockIdx.x * kDBlock + threadIdx.x; i < n; i += stride) {
    const float a = fabsf(t[i]);
    if (a >= t0) atomicAdd(&h[tab_bin_lut(tab, lut, a)], 1u);
  }
  __syncthreads();
  for (int e = threadIdx.x; e <= kTab; e += kDBlock)
    if (h[e]) atomicAdd(&w.hist[e], h[e]);
}

// replay dgc.py:23-36 on the exact counts (one thread): count(|t| >= x) for a table value x at
// lower-bound position p is the number of elements whose bin is > p
template <bool GATED>
__global__ void dgc_replay_kernel(int64_t n, double ratio, DgcWs w) {
  if constexpr (GATED) { if (w.meta->fix == 0u) return; }
  __shared__ uint32_t suf[kTab + 2];
  __shared__ float tab[kTab];
  // the histogram and the table into LDS by every lane (the single-thread replay below then reads
  // no global memory in its dependent chains: 62 -> a few us)
  for (int e = threadIdx.x; e < kTab; e += blockDim.x) tab[e] = w.tab[e];
  {  // suffix sums of the kTab + 1 bins: lane l owns a contiguous run, one wave scan of the run totals
    constexpr int kRun = (kTab + 1 + 63) / 64;
    const int l = threadIdx.x;            // launched with exactly one wave
    uint32_t v[kRun], tot = 0;
#pragma unroll
    for (int i = 0; i < kRun; ++i) {
      const int b = l * kRun + i;
      v[i] = b <= kTab ? w.hist[b] : 0u;
      tot += v[i];
    }
    uint32_t above = tot;                 // inclusive scan from the top lane down
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t x = __shfl_down(above, o, 64);
      if (l + o < 64) above += x;
    }
    uint32_t acc = above - tot;           // bins of the lanes above this one
#pragma unroll
    for (int i = kRun - 1; i >= 0; --i) {
      const int b = l * kRun + i;
      acc += v[i];
      if (b <= kTab) suf[b] = acc;
    }
    if (l == 0) suf[kTab + 1] = 0;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  // torch compares the int64 count tensor with the Python float (1.3 * numel * ratio, a double)
  // in the default dtype, f32
  const float hi = (float)(1.3 * (double)n * ratio);
  const float lo = (float)(0.7 * (double)n * ratio);
  auto count_ge = [&](float x) -> uint32_t {
    if (x != x) return 0u;
    int a = 0, b = kTab;            // first index with tab >= x
    while (a < b) {
      const int mid = (a + b) >> 1;
      if (tab[mid] < x) a = mid + 1; else b = mid;
    }
    return suf[a + 1];
  };
  float thr = __uint_as_float(w.meta->thr0);
  uint32_t sel = count_ge(thr);
  for (int it = 0; it < kDepth; ++it) {
    if ((float)sel > hi) thr = 1.3f * thr;
    else if ((float)sel < lo) thr = 0.7f * thr;
    else break;
    sel = count_ge(thr);
  }
  w.meta->thr = __float_as_uint(thr);
  w.meta->total = sel;
}

// per-chunk counts at the final threshold, then exclusive offsets (one workgroup)
__global__ __launch_bounds__(kDBlock) void dgc_chunk_kernel(const float* __restrict__ t, int64_t n, DgcWs w) {
  const float thr = __uint_as_float(w.meta->thr);
  const int64_t base = (int64_t)blockIdx.x * kDChunk;
  const int64_t end = min(base + (int64_t)kDChunk, n);
  uint32_t c = 0;
  for (int64_t i = base + threadIdx.x; i < end; i += kDBlock) c += fabsf(t[i]) >= thr;
  c = wave_sum(c);
  __shared__ uint32_t sc[kDBlock / kWave];
  if ((threadIdx.x & 63) == 0) sc[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t s = 0;
    for (int j = 0; j < kDBlock / kWave; ++j) s += sc[j];
    w.part[blockIdx.x] = s;
  }
}

template <int BLOCK>
__device__ __forceinline__ uint32_t dgc_excl_scan(uint32_t v, uint32_t* s_w, uint32_t* total) {
  constexpr int NW = BLOCK / kWave;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t x = __shfl_up(inc, o, 64);
    if (lane >= o) inc += x;
  }
  if (lane == 63) s_w[wv] = inc;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t acc = 0;
    for (int i = 0; i < NW; ++i) { const uint32_t x = s_w[i]; s_w[i] = acc; acc += x; }
    s_w[NW] = acc;
  }
  __syncthreads();
  const uint32_t r = s_w[wv] + inc - v;
  if (total) *total = s_w[NW];
  __syncthreads();
  return r;
}

__global__ __launch_bounds__(1024) void dgc_offsets_kernel(int64_t nch, DgcWs w) {
  __shared__ uint32_t s_w[1024 / kWave + 1];
  uint32_t run = 0;
  for (int64_t j0 = 0; j0 < nch; j0 += 1024) {
    const int64_t j = j0 + threadIdx.x;
    const uint32_t c = j < nch ? w.part[j] : 0u;
    uint32_t tot;
    const uint32_t ex = dgc_excl_scan<1024>(c, s_w, &tot);
    if (j < nch) w.offs[j] = run + ex;
    run += tot;
  }
  if (threadIdx.x == 0) w.meta->total = run;
}

// ordered compaction of |t| >= thr: values f32, indices int64 (torch.where order).  With a header
// pointer it writes the capacity-bounded exchange record of sparse.hip instead -- {count, cap, 0,
// 0 | vals f32[cap] | idx i32[cap]}, entries past cap (ascending index order) dropped.
constexpr int kDgcRecHdr = 4;          // = sparse.hip kRecHdr (grace_exchange_record_words)
template <typename IdxT>
__global__ __launch_bounds__(kDBlock) void dgc_write_kernel(const float* __restrict__ t, int64_t n, DgcWs w,
                                                           float* __restrict__ vals, IdxT* __restrict__ idx,
                                                           int64_t cap, uint32_t* __restrict__ hdr) {
  __shared__ uint32_t s_w[kDBlock / kWave + 1];
  const float thr = __uint_as_float(w.meta->thr);
  if (hdr && blockIdx.x == 0 && threadIdx.x == 0) {
    hdr[0] = w.meta->total;
    hdr[1] = (uint32_t)cap;
    hdr[2] = 0u;
    hdr[3] = 0u;
  }
  const int64_t base = (int64_t)blockIdx.x * kDChunk;
  const int64_t end = min(base + (int64_t)kDChunk, n);
  uint32_t run = w.offs[blockIdx.x];
  for (int64_t j0 = base; j0 < end; j0 += kDBlock) {
    const int64_t i = j0 + threadIdx.x;
    float v = 0.f;
    bool sel = false;
    if (i < end) { v = t[i]; sel = fabsf(v) >= thr; }
    uint32_t tot;
    const uint32_t ex = dgc_excl_scan<kDBlock>(sel ? 1u : 0u, s_w, &tot);
    if (sel && (int64_t)(run + ex) < cap) { vals[run + ex] = v; idx[run + ex] = (IdxT)i; }
    run += tot;
  }
}

// DgcMemory.update (memory/dgc.py:21-28) over the entries that travelled in this rank's record:
// r = r * 0, a = a * 0 at those indices (the mask multiply, so a negative entry becomes -0 exactly
// as r * ~mask does).  Without overflow the record holds every selected index, so this equals
// grace_dgc_mask_update; on overflow the unsent entries keep r and a (error feedback).
__global__ __launch_bounds__(kDBlock) void dgc_rec_mask_kernel(const uint32_t* __restrict__ rec, int64_t cap,
                                                              float* __restrict__ r, float* __restrict__ a) {
  const int64_t c = min((int64_t)rec[0], cap);
  const int32_t* idx = reinterpret_cast<const int32_t*>(rec + kDgcRecHdr + cap);
  for (int64_t j = (int64_t)blockIdx.x * kDBlock + threadIdx.x; j < c; j += (int64_t)gridDim.x * kDBlock) {
    const int32_t i = idx[j];
    r[i] = r[i] * 0.f;
    a[i] = a[i] * 0.f;
  }
}

// ------------------------------------------------------------------------------------------------
// memory
// Elementwise memory kernels: a thread owns kDQ quads per round (16-B loads, all issued before use)
// when every buffer is 16-B aligned; the scalar loop covers the rest.  (One 4-B access per thread
// per element made the 256 MiB DGC step 1.36 ms.)
// compensate in place (r, a) or, for the world-1 fused step's fix-up, from (r, a) into (ro, ao)
// (GATED: only when that step's speculative pass flagged meta->fix)
template <bool GATED>
__global__ __launch_bounds__(kDBlock) void dgc_compensate_kernel(const float* __restrict__ g, const float* r,
                                                                const float* a, int has_state,
                                                                float momentum, int64_t n, float* ro, float* ao,
                                                                const DgcMeta* __restrict__ gate) {
  if constexpr (GATED) { if (gate->fix == 0u) return; }
  const int64_t stride = (int64_t)gridDim.x * kDBlock;
  const int64_t nq = (al16(g) && al16(r) && al16(a) && al16(ro) && al16(ao)) ? n >> 2 : 0;
  for (int64_t q0 = (int64_t)blockIdx.x * kDBlock + threadIdx.x; q0 < nq; q0 += stride * kDQ) {
    f4d gv[kDQ], rv[kDQ], av[kDQ];
#pragma unroll
    for (int u = 0; u < kDQ; ++u) {
      const int64_t q = q0 + u * stride < nq ? q0 + u * stride : q0;
      gv[u] = __builtin_nontemporal_load(reinterpret_cast<const f4d*>(g) + q);
      if (has_state) {
        rv[u] = __builtin_nontemporal_load(reinterpret_cast<const f4d*>(r) + q);
        av[u] = __builtin_nontemporal_load(reinterpret_cast<const f4d*>(a) + q);
      }
    }
#pragma unroll
    for (int u = 0; u < kDQ; ++u) {
      if (q0 + u * stride >= nq) break;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float rj = has_state ? rv[u][j] : 0.f, aj = has_state ? av[u][j] : 0.f;
        dgc_comp1(gv[u][j], rj, aj, has_state, momentum);
        rv[u][j] = rj;
        av[u][j] = aj;
      }
      __builtin_nontemporal_store(rv[u], reinterpret_cast<f4d*>(ro) + q0 + u * stride);
      __builtin_nontemporal_store(av[u], reinterpret_cast<f4d*>(ao) + q0 + u * stride);
    }
  }
  for (int64_t i = nq * 4 + (int64_t)blockIdx.x * kDBlock + threadIdx.x; i < n; i += stride) {
    float rv = has_state ? r[i] : 0.f, av = has_state ? a[i] : 0.f;
    dgc_comp1(g[i], rv, av, has_state, momentum);
    ro[i] = rv;
    ao[i] = av;
  }
}

// World-1 Allgather(DgcCompressor, DgcMemory).step in ONE streaming pass (memory/dgc.py:15-39 with
// compressor/dgc.py:12-50, allgather.py:40-45): compensate, select at the sampled threshold thr0,
// mask the memory and write (0 + decompress) / 1, from the old state (g, r, a) into NEW buffers
// (ro, ao) -- 24 B per element against compensate 20 + threshold count 4 + mask / output 20.  The
// reference's adjustment loop keeps thr0 whenever count(|t| >= thr0) is within [0.7, 1.3] k (the
// sampled estimate: almost always), so the pass selects at thr0 speculatively while it counts;
// the workgroup that arrives last checks the loop's first test on the exact count.  If thr0 does
// not stand, meta->fix is set and the gated fix-up launches (compensate from the untouched old
// state, count, replay, mask) redo the step exactly; otherwise they return at once.
template <bool HAS>
__global__ __launch_bounds__(kDBlock) void dgc_w1_spec_kernel(const float* __restrict__ g, const float* __restrict__ r,
                                                             const float* __restrict__ a, float momentum, int64_t n,
                                                             double ratio, DgcMeta* __restrict__ meta,
                                                             uint32_t* __restrict__ part, float* __restrict__ ro,
                                                             float* __restrict__ ao, float* __restrict__ out) {
  __shared__ uint32_t sc[kDBlock / kWave];
  __shared__ uint32_t s_last;
  const float thr = __uint_as_float(meta->thr0);
  const int64_t base = (int64_t)blockIdx.x * kDChunkW1;
  const int64_t end = min(base + (int64_t)kDChunkW1, n);
  const bool vec = al16(g) && al16(r) && al16(a) && al16(ro) && al16(ao) && al16(out);
  const int64_t qe = vec ? base + ((end - base) & ~(int64_t)3) : base;
  uint32_t cnt = 0;
  auto one = [&](float gv, float rv, float av, float& rn, float& an, float& o) {
    dgc_comp1(gv, rv, av, HAS ? 1 : 0, momentum);   // av = t
    const bool sel = fabsf(av) >= thr;
    const float keep = sel ? 0.f : 1.f;
    cnt += sel;
    o = sel ? 0.f + av : 0.f;
    rn = rv * keep;
    an = av * keep;
  };
  for (int64_t e0 = base + 4 * (int64_t)threadIdx.x; e0 < qe; e0 += 4 * (int64_t)kDBlock * kDQ) {
    f4d gv[kDQ], rv[kDQ], av[kDQ];
#pragma unroll
    for (int u = 0; u < kDQ; ++u) {
      const int64_t e = e0 + 4 * (int64_t)u * kDBlock < qe ? e0 + 4 * (int64_t)u * kDBlock : e0;
      gv[u] = __builtin_nontemporal_load(reinterpret_cast<const f4d*>(g + e));
      if (HAS) {
        rv[u] = __builtin_nontemporal_load(reinterpret_cast<const f4d*>(r + e));
        av[u] = __builtin_nontemporal_load(reinterpret_cast<const f4d*>(a + e));
      }
    }
#pragma unroll
    for (int u = 0; u < kDQ; ++u) {
      const int64_t e = e0 + 4 * (int64_t)u * kDBlock;
      if (e >= qe) break;
      f4d rn, an, o;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float x, y, z;
        one(gv[u][j], HAS ? rv[u][j] : 0.f, HAS ? av[u][j] : 0.f, x, y, z);
        rn[j] = x;
        an[j] = y;
        o[j] = z;
      }
      __builtin_nontemporal_store(rn, reinterpret_cast<f4d*>(ro + e));
      __builtin_nontemporal_store(an, reinterpret_cast<f4d*>(ao + e));
      __builtin_nontemporal_store(o, reinterpret_cast<f4d*>(out + e));
    }
  }
  for (int64_t i = qe + threadIdx.x; i < end; i += kDBlock) {
    float x, y, z;
    one(g[i], HAS ? r[i] : 0.f, HAS ? a[i] : 0.f, x, y, z);
    ro[i] = x;
    ao[i] = y;
    out[i] = z;
  }
  // the chunk's count, write-through; the last workgroup to arrive decides whether thr0 stands
  cnt = wave_sum(cnt);
  if ((threadIdx.x & 63) == 0) sc[threadIdx.x >> 6] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t c = 0;
    for (int j = 0; j < kDBlock / kWave; ++j) c += sc[j];
    __hip_atomic_store(&part[blockIdx.x], c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    s_last = atomicAdd(&meta->ticket, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (!s_last) return;
  // the grid runs several workgroups per CU, outside the guide's measured fence-free row (one per
  // CU): the last arriver keeps the agent-scope acquire before it reads the others' partials
  // (MI355X_MICROARCH.md, Consumer condition (4); one invalidate in one workgroup per launch)
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  uint32_t tot = 0;
  for (int64_t j = threadIdx.x; j < (int64_t)gridDim.x; j += kDBlock)
    tot += __hip_atomic_load(&part[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  tot = wave_sum(tot);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sc[threadIdx.x >> 6] = tot;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t sel = 0;
    for (int j = 0; j < kDBlock / kWave; ++j) sel += sc[j];
    // dgc_replay_kernel's first test: the loop breaks at once iff the count is within the bounds
    const float hi = (float)(1.3 * (double)n * ratio);
    const float lo = (float)(0.7 * (double)n * ratio);
    const bool stands = !((float)sel > hi) && !((float)sel < lo);
    meta->fix = stands ? 0u : 1u;
    if (stands) {
      meta->thr = meta->thr0;
      meta->total = sel;
    }
    meta->ticket = 0u;
  }
}

// update: keep = !(|t| >= thr) as in mask = tensor.abs() >= thr; r = r * keep, a = a * keep
// (t is the compensated tensor the mask came from; it may alias a).  OUT: the world-1 Allgather
// result in the same pass, out = 0 + t where selected and 0 elsewhere -- (0 + decompress) / 1
// of the payload grace_dgc_write would have produced (dgc.py:45-50, allgather.py:40-45).
template <bool OUT, bool GATED = false>
__global__ __launch_bounds__(kDBlock) void dgc_mask_kernel(const float* t, float* r, float* a, int64_t n,
                                                          const DgcMeta* __restrict__ meta, float* out) {
  if constexpr (GATED) { if (meta->fix == 0u) return; }
  const float thr = __uint_as_float(meta->thr);
  const bool alias = t == a;
  const int64_t stride = (int64_t)gridDim.x * kDBlock;
  const int64_t nq = (al16(t) && al16(r) && al16(a) && (!OUT || al16(out))) ? n >> 2 : 0;
  for (int64_t q0 = (int64_t)blockIdx.x * kDBlock + threadIdx.x; q0 < nq; q0 += stride * kDQ) {
    f4d tv[kDQ], rv[kDQ], av[kDQ];
#pragma unroll
    for (int u = 0; u < kDQ; ++u) {
      const int64_t q = q0 + u * stride < nq ? q0 + u * stride : q0;
      tv[u] = __builtin_nontemporal_load(reinterpret_cast<const f4d*>(t) + q);
      rv[u] = __builtin_nontemporal_load(reinterpret_cast<const f4d*>(r) + q);
      if (!alias) av[u] = __builtin_nontemporal_load(reinterpret_cast<const f4d*>(a) + q);
    }
#pragma unroll
    for (int u = 0; u < kDQ; ++u) {
      if (q0 + u * stride >= nq) break;
      f4d o;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool sel = fabsf(tv[u][j]) >= thr;
        const float keep = sel ? 0.f : 1.f;
        const float avj = alias ? tv[u][j] : av[u][j];
        o[j] = sel ? 0.f + tv[u][j] : 0.f;
        rv[u][j] = rv[u][j] * keep;
        av[u][j] = avj * keep;
      }
      __builtin_nontemporal_store(rv[u], reinterpret_cast<f4d*>(r) + q0 + u * stride);
      __builtin_nontemporal_store(av[u], reinterpret_cast<f4d*>(a) + q0 + u * stride);
      if constexpr (OUT) __builtin_nontemporal_store(o, reinterpret_cast<f4d*>(out) + q0 + u * stride);
    }
  }
  for (int64_t i = nq * 4 + (int64_t)blockIdx.x * kDBlock + threadIdx.x; i < n; i += stride) {
    const float tv = t[i];
    const bool sel = fabsf(tv) >= thr;
    const float keep = sel ? 0.f : 1.f;
    const float av = alias ? tv : a[i];
    r[i] = r[i] * keep;
    a[i] = av * keep;
    if constexpr (OUT) out[i] = sel ? 0.f + tv : 0.f;
  }
}

// gradient clipping (memory/dgc.py:16-19): sum of squares (f64 accumulate) of one tensor
__global__ __launch_bounds__(kDBlock) void sumsq_kernel(const float* __restrict__ x, int64_t n,
                                                       double* __restrict__ part) {
  double s = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * kDBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kDBlock) {
    const double v = x[i];
    s += v * v;
  }
  s = wave_sum(s);
  __shared__ double sw[kDBlock / kWave];
  if ((threadIdx.x & 63) == 0) sw[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0.0;
    for (int j = 0; j < kDBlock / kWave; ++j) a += sw[j];
    part[blockIdx.x] = a;
  }
}

__global__ void sumsq_finish_kernel(const double* __restrict__ part, int nb, float* __restrict__ out) {
  if (threadIdx.x == 0) {
    double a = 0.0;
    for (int j = 0; j < nb; ++j) a += part[j];
    *out = (float)a;
  }
}

// clamp(x, -c, c) with c = sqrt(s / world) read from the device (after the caller's all_reduce)
__global__ __launch_bounds__(kDBlock) void clip_kernel(const float* __restrict__ x, const float* __restrict__ s,
                                                      float world, float* __restrict__ out, int64_t n) {
  const float c = sqrtf(*s / world);
  for (int64_t i = (int64_t)blockIdx.x * kDBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kDBlock)
    out[i] = fminf(fmaxf(x[i], -c), c);
}

}  // namespace grace

using namespace grace;

extern "C" {

size_t grace_dgc_workspace_bytes(int64_t n) { return dgc_ws_bytes(n < 1 ? 1 : n); }

grace_status_t grace_dgc_sample(const float* t, int64_t n, const int64_t* sample_idx, uint64_t seed, int64_t ns,
                                float* sample_abs, void* stream) {
  GRACE_REQUIRE(t && sample_abs && n >= 1 && ns >= 1, "grace_dgc_sample: bad arguments");
  dgc_sample_kernel<<<stream_grid(ns, kDBlock, 1024), kDBlock, 0, as_stream(stream)>>>(t, n, sample_idx, seed, ns,
                                                                                      sample_abs);
  GRACE_CHECK_LAUNCH("grace_dgc_sample");
  return GRACE_OK;
}

grace_status_t grace_dgc_threshold(const float* t, int64_t n, const float* top_vals, int64_t ks, double ratio,
                                   void* ws, void* stream) {
  GRACE_REQUIRE(t && top_vals && ws && n >= 1 && ks >= 1, "grace_dgc_threshold: bad arguments");
  hipStream_t s = as_stream(stream);
  DgcWs w = dgc_carve(ws, n);
  const int64_t nch = (n + kDChunk - 1) / kDChunk;
  dgc_table_kernel<<<1, 1024, 0, s>>>(top_vals, ks, w);
  GRACE_CHECK_LAUNCH("grace_dgc_threshold");
  dgc_count_kernel<false><<<stream_grid((n + 3) / 4, kDBlock, 2048), kDBlock, 0, s>>>(t, n, w);
  GRACE_CHECK_LAUNCH("grace_dgc_threshold");
  dgc_replay_kernel<false><<<1, 64, 0, s>>>(n, ratio, w);
  GRACE_CHECK_LAUNCH("grace_dgc_threshold");
  dgc_chunk_kernel<<<(unsigned)nch, kDBlock, 0, s>>>(t, n, w);
  GRACE_CHECK_LAUNCH("grace_dgc_threshold");
  dgc_offsets_kernel<<<1, 1024, 0, s>>>(nch, w);
  GRACE_CHECK_LAUNCH("grace_dgc_threshold");
  return GRACE_OK;
}

grace_status_t grace_dgc_write(const float* t, int64_t n, const void* ws, float* vals, int64_t* idx, void* stream) {
  GRACE_REQUIRE(t && ws && n >= 1, "grace_dgc_write: bad arguments");
  DgcWs w = dgc_carve(const_cast<void*>(ws), n);
  const int64_t nch = (n + kDChunk - 1) / kDChunk;
  dgc_write_kernel<int64_t><<<(unsigned)nch, kDBlock, 0, as_stream(stream)>>>(t, n, w, vals, idx, n, nullptr);
  GRACE_CHECK_LAUNCH("grace_dgc_write");
  return GRACE_OK;
}

grace_status_t grace_dgc_write_capped(const float* t, int64_t n, const void* ws, uint32_t* rec, int64_t cap,
                                      void* stream) {
  GRACE_REQUIRE(t && ws && rec && n >= 1 && cap >= 1 && cap <= n && n < ((int64_t)1 << 31),
                "grace_dgc_write_capped: bad arguments (1 <= cap <= n < 2^31)");
  DgcWs w = dgc_carve(const_cast<void*>(ws), n);
  const int64_t nch = (n + kDChunk - 1) / kDChunk;
  float* vals = reinterpret_cast<float*>(rec + kDgcRecHdr);
  int32_t* idx = reinterpret_cast<int32_t*>(rec + kDgcRecHdr + cap);
  dgc_write_kernel<int32_t><<<(unsigned)nch, kDBlock, 0, as_stream(stream)>>>(t, n, w, vals, idx, cap, rec);
  GRACE_CHECK_LAUNCH("grace_dgc_write_capped");
  return GRACE_OK;
}

grace_status_t grace_dgc_mask_update_capped(const uint32_t* rec, int64_t cap, float* residual, float* accum,
                                            void* stream) {
  GRACE_REQUIRE(rec && residual && accum && cap >= 1, "grace_dgc_mask_update_capped: bad arguments");
  dgc_rec_mask_kernel<<<stream_grid(cap, kDBlock, 2048), kDBlock, 0, as_stream(stream)>>>(rec, cap, residual, accum);
  GRACE_CHECK_LAUNCH("grace_dgc_mask_update_capped");
  return GRACE_OK;
}

grace_status_t grace_dgc_compensate(const float* g, float* residual, float* accum, int32_t has_state,
                                    float momentum, int64_t n, void* stream) {
  GRACE_REQUIRE(g && residual && accum && n >= 0, "grace_dgc_compensate: bad arguments");
  if (n == 0) return GRACE_OK;
  dgc_compensate_kernel<false><<<stream_grid((n + 3) / 4, kDBlock * kDQ, 4096), kDBlock, 0, as_stream(stream)>>>(
      g, residual, accum, has_state, momentum, n, residual, accum, nullptr);
  GRACE_CHECK_LAUNCH("grace_dgc_compensate");
  return GRACE_OK;
}

grace_status_t grace_dgc_mask_update(const float* t, float* residual, float* accum, int64_t n, const void* ws,
                                     void* stream) {
  GRACE_REQUIRE(t && residual && accum && ws && n >= 0, "grace_dgc_mask_update: bad arguments");
  if (n == 0) return GRACE_OK;
  dgc_mask_kernel<false><<<stream_grid((n + 3) / 4, kDBlock * kDQ, 4096), kDBlock, 0, as_stream(stream)>>>(
      t, residual, accum, n, reinterpret_cast<const DgcMeta*>(ws), nullptr);
  GRACE_CHECK_LAUNCH("grace_dgc_mask_update");
  return GRACE_OK;
}

grace_status_t grace_dgc_select(const float* t, int64_t n, const float* top_vals, int64_t ks, double ratio, void* ws,
                                void* stream) {
  GRACE_REQUIRE(t && top_vals && ws && n >= 1 && ks >= 1, "grace_dgc_select: bad arguments");
  hipStream_t s = as_stream(stream);
  DgcWs w = dgc_carve(ws, n);
  dgc_table_kernel<<<1, 1024, 0, s>>>(top_vals, ks, w);
  GRACE_CHECK_LAUNCH("grace_dgc_select");
  dgc_count_kernel<false><<<stream_grid((n + 3) / 4, kDBlock, 2048), kDBlock, 0, s>>>(t, n, w);
  GRACE_CHECK_LAUNCH("grace_dgc_select");
  dgc_replay_kernel<false><<<1, 64, 0, s>>>(n, ratio, w);
  GRACE_CHECK_LAUNCH("grace_dgc_select");
  return GRACE_OK;
}

grace_status_t grace_dgc_step_w1(const float* t, float* residual, float* accum, int64_t n, const void* ws, float* out,
                                 void* stream) {
  GRACE_REQUIRE(t && residual && accum && ws && out && n >= 0, "grace_dgc_step_w1: bad arguments");
  if (n == 0) return GRACE_OK;
  dgc_mask_kernel<true><<<stream_grid((n + 3) / 4, kDBlock * kDQ, 4096), kDBlock, 0, as_stream(stream)>>>(
      t, residual, accum, n, reinterpret_cast<const DgcMeta*>(ws), out);
  GRACE_CHECK_LAUNCH("grace_dgc_step_w1");
  return GRACE_OK;
}

grace_status_t grace_dgc_sample_comp(const float* g, const float* residual, const float* accum, int32_t has_state,
                                     float momentum, int64_t n, const int64_t* sample_idx, uint64_t seed, int64_t ns,
                                     float* sample_abs, void* stream) {
  GRACE_REQUIRE(g && sample_abs && n >= 1 && ns >= 1 && (!has_state || (residual && accum)),
                "grace_dgc_sample_comp: bad arguments");
  dgc_sample_comp_kernel<<<stream_grid(ns, kDBlock, 1024), kDBlock, 0, as_stream(stream)>>>(
      g, residual, accum, has_state, momentum, n, sample_idx, seed, ns, sample_abs);
  GRACE_CHECK_LAUNCH("grace_dgc_sample_comp");
  return GRACE_OK;
}

size_t grace_dgc_sample_kth_workspace_bytes(void) { return al256(sizeof(KthState)); }

grace_status_t grace_dgc_sample_kth(const float* sample_abs, int64_t ns, int64_t ks, void* ws, float* out,
                                    void* stream) {
  GRACE_REQUIRE(sample_abs && ws && out && ns >= 1 && ks >= 1 && ks <= ns && ns < ((int64_t)1 << 32),
                "grace_dgc_sample_kth: bad arguments");
  hipStream_t s = as_stream(stream);
  KthState* st = reinterpret_cast<KthState*>(ws);
  const int64_t nb = (ns + kKthPer * kKthBlock - 1) / (kKthPer * kKthBlock);
  const unsigned grid = (unsigned)(nb < 1024 ? nb : 1024);
  dgc_kth_kernel<0><<<grid, kKthBlock, 0, s>>>(sample_abs, ns, (uint32_t)ks, st, out);
  GRACE_CHECK_LAUNCH("grace_dgc_sample_kth");
  dgc_kth_kernel<1><<<grid, kKthBlock, 0, s>>>(sample_abs, ns, (uint32_t)ks, st, out);
  GRACE_CHECK_LAUNCH("grace_dgc_sample_kth");
  dgc_kth_kernel<2><<<grid, kKthBlock, 0, s>>>(sample_abs, ns, (uint32_t)ks, st, out);
  GRACE_CHECK_LAUNCH("grace_dgc_sample_kth");
  return GRACE_OK;
}

size_t grace_dgc_step_w1_fused_workspace_bytes(int64_t n) {
  return dgc_ws_bytes(n < 1 ? 1 : n) + 256 + sizeof(uint32_t) * (size_t)((n + kDChunkW1 - 1) / kDChunkW1);
}

grace_status_t grace_dgc_step_w1_fused(const float* g, const float* residual, const float* accum, int32_t has_state,
                                       float momentum, int64_t n, const float* top_vals, int64_t ks, double ratio,
                                       void* ws, float* residual_out, float* accum_out, float* out, void* stream) {
  GRACE_REQUIRE(g && top_vals && ws && residual_out && accum_out && out && n >= 1 && ks >= 1 &&
                    (!has_state || (residual && accum)) && n < ((int64_t)1 << 40),
                "grace_dgc_step_w1_fused: bad arguments");
  GRACE_REQUIRE(residual_out != residual && accum_out != accum && residual_out != accum_out,
                "grace_dgc_step_w1_fused: the new state must not alias the old");
  hipStream_t s = as_stream(stream);
  DgcWs w = dgc_carve(ws, n);
  uint32_t* part = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(ws) + dgc_ws_bytes(n) + 256);
  const int64_t nch = (n + kDChunkW1 - 1) / kDChunkW1;
  GRACE_REQUIRE(nch < ((int64_t)1 << 31), "grace_dgc_step_w1_fused: too many chunks");
  dgc_thr0_kernel<<<1, 1024, 0, s>>>(top_vals, ks, w);
  GRACE_CHECK_LAUNCH("grace_dgc_step_w1_fused");
  if (has_state)
    dgc_w1_spec_kernel<true><<<(unsigned)nch, kDBlock, 0, s>>>(g, residual, accum, momentum, n, ratio, w.meta, part,
                                                             residual_out, accum_out, out);
  else
    dgc_w1_spec_kernel<false><<<(unsigned)nch, kDBlock, 0, s>>>(g, residual, accum, momentum, n, ratio, w.meta, part,
                                                              residual_out, accum_out, out);
  GRACE_CHECK_LAUNCH("grace_dgc_step_w1_fused");
  // gated fix-up (returns at once unless thr0 did not stand): the reference's full adjustment loop,
  // on grids small enough that the no-op launches cost little
#ifdef GRACE_DGC_NO_FIXUP   // diagnostic A/B build only: what the five no-op launches cost (wrong when a fix is due)
  return GRACE_OK;
#endif
  dgc_table_kernel<true><<<1, 1024, 0, s>>>(top_vals, ks, w);   // the adjustment table, zeroed counts
  GRACE_CHECK_LAUNCH("grace_dgc_step_w1_fused");
  const unsigned sg = stream_grid((n + 3) / 4, kDBlock * kDQ, 1024);
  dgc_compensate_kernel<true><<<sg, kDBlock, 0, s>>>(g, residual, accum, has_state, momentum, n, residual_out,
                                                     accum_out, w.meta);
  GRACE_CHECK_LAUNCH("grace_dgc_step_w1_fused");
  dgc_count_kernel<true><<<stream_grid((n + 3) / 4, kDBlock, 1024), kDBlock, 0, s>>>(accum_out, n, w);
  GRACE_CHECK_LAUNCH("grace_dgc_step_w1_fused");
  dgc_replay_kernel<true><<<1, 64, 0, s>>>(n, ratio, w);
  GRACE_CHECK_LAUNCH("grace_dgc_step_w1_fused");
  dgc_mask_kernel<true, true><<<sg, kDBlock, 0, s>>>(accum_out, residual_out, accum_out, n, w.meta, out);
  GRACE_CHECK_LAUNCH("grace_dgc_step_w1_fused");
  return GRACE_OK;
}

size_t grace_sumsq_workspace_bytes(void) { return sizeof(double) * 1024; }

grace_status_t grace_sumsq(const float* x, int64_t n, void* ws, float* out, void* stream) {
  GRACE_REQUIRE(x && ws && out && n >= 0, "grace_sumsq: bad arguments");
  const unsigned nb = n ? stream_grid(n, kDBlock, 1024) : 1;
  hipStream_t s = as_stream(stream);
  sumsq_kernel<<<nb, kDBlock, 0, s>>>(x, n, reinterpret_cast<double*>(ws));
  GRACE_CHECK_LAUNCH("grace_sumsq");
  sumsq_finish_kernel<<<1, 64, 0, s>>>(reinterpret_cast<const double*>(ws), (int)nb, out);
  GRACE_CHECK_LAUNCH("grace_sumsq");
  return GRACE_OK;
}

grace_status_t grace_clip_by_sumsq(const float* x, const float* sumsq_dev, float world, float* out, int64_t n,
                                   void* stream) {
  GRACE_REQUIRE(x && sumsq_dev && out && n >= 0 && world > 0.f, "grace_clip_by_sumsq: bad arguments");
  if (n == 0) return GRACE_OK;
  clip_kernel<<<stream_grid(n, kDBlock, 2048), kDBlock, 0, as_stream(stream)>>>(x, sumsq_dev, world, out, n);
  GRACE_CHECK_LAUNCH("grace_clip_by_sumsq");
  return GRACE_OK;
}

}  // extern "C"
