// Exact top-k sparsification with fused residual error feedback, for CDNA4 (gfx950).
//
// Reference semantics (sands-lab/grace):
//   ResidualMemory.compensate  t = beta*r + gamma*g         grace_dl/dist/memory/residual.py:10-14
//   TopKCompressor.compress    idx = topk(|t|, k), vals = t[idx]  grace_dl/dist/compressor/topk.py:32-42
//   ResidualMemory.update      r' = t - zeros.scatter_(idx, vals) residual.py:16-20
//   Allgather.send_receive     out = (0 + decode(payload)) / 1    communicator/allgather.py:40-45
// Tie rule (ours, deterministic): larger |t| first (NaN largest), lower index first among equal |t|.
// torch.topk(sorted=False) returns the same set modulo ties at the k-th value.
//
// The reference's native selector (radixtopk_cuda/rdxtopk_cuda.cu:410-534) makes 4 histogram
// passes over the keys with a device->host sync per digit.  Here the whole selection stays on the
// device, the bucket is streamed ONCE, and no step ever syncs the host:
//
//   1. sample   (<=128 WGs)     stratified sample of up to 131072 |t| keys (hash-offset strata)
//                               into a 32768-bin LDS histogram of key>>16, flushed with atomics.
//   2. select   (1 WG)          ranks of the k-th key in the sample +-6 sigma (binomial) ->
//                               thr_hi >= thr_lo bracketing the k-th largest key; zeroes this
//                               step's counters, cursors and histograms.
//   3. main     (n/12288 WGs)   one streaming pass: t = beta r + gamma g, write r' (and the dense
//                               world-1 output), key > thr_hi  -> "sure": appended to the payload;
//                               thr_lo <= key <= thr_hi -> candidate list + 2048-bin histogram
//                               of the candidate key range.  Appends use wave64 ballot + mbcnt
//                               into LDS staging, one global atomic per workgroup and list.
//   4. finalize (128 WGs)       every WG finds the boundary bin B from the global histogram;
//                               candidates above B go to the payload and those in B to a short
//                               boundary list (block scan + one atomic per round); the last WG
//                               to arrive selects the final `need` entries of B by (key, -idx).
//                               If the bracket missed (or a list overflowed) that WG runs the
//                               exact single-workgroup radix select instead (rare, same result).
// Small buckets (n <= 32768) run a single-workgroup kernel with the bucket held in LDS.
#include <math.h>
#include <string.h>

#include <hip/hip_ext.h>

#include "common.h"
#include "select.h"

namespace grace {

// dense outputs written by a top-k launch
// kDenseOut: no memory (Allgather(TopK, NoneMemory) at world 1): t = g, only the dense output is
// written next to the payload, the input stays read-only
// kResSwap: the W > 1 residual step into a SECOND residual buffer (read g and r_in, write r; no dense
// output): like kDenseFused the main pass writes every provisional pick (key > thr_mid) as selected
// (r = t - t) and the finalize fixes up the candidates it decides otherwise, because t stays
// recoverable from g and the untouched r_in; kDenseRes (in place) must keep t in r and zero the k
// selected positions in the finalize instead (537 K scattered stores at 2^26, 1 %)
enum DenseMode : int { kDenseNone = 0, kDenseRes = 1, kDenseFused = 2, kDenseOut = 3, kResSwap = 4 };
template <int MODE> constexpr bool kWritesR = MODE == kDenseRes || MODE == kDenseFused || MODE == kResSwap;
template <int MODE> constexpr bool kWritesOut = MODE == kDenseFused || MODE == kDenseOut;
// the main pass writes provisional picks as selected; the finalize fixes up its candidates
template <int MODE> constexpr bool kProv = kWritesOut<MODE> || MODE == kResSwap;

#ifndef GRACE_MAIN_BLOCK
#define GRACE_MAIN_BLOCK 256
#endif
#ifndef GRACE_MAIN_VEC
#define GRACE_MAIN_VEC 12
#endif
constexpr int kMainBlock = GRACE_MAIN_BLOCK;
constexpr int kMainVec = GRACE_MAIN_VEC;                   // float4 per thread
constexpr int kMainChunk = kMainBlock * 4 * kMainVec;      // 12288 elements per workgroup (A/B, 256 MiB
                                                           // top-k 1 % + residual: 8192 / 12288 / 16384 /
                                                           // 20480 / 24576 -> 240 / 195 / 196.5 / 204 / 205 us)
#ifndef GRACE_MAIN_VEC_12B
#define GRACE_MAIN_VEC_12B 20
#endif
#ifndef GRACE_MAIN_VEC_NORES
#define GRACE_MAIN_VEC_NORES 32
#endif
// Chunk length by the bytes the pass moves per element: each workgroup has fixed costs (histogram
// clear and flush, list flushes), so the fewer bytes per element, the longer its chunk.  A/B at
// 256 MiB (main pass):
//   16 B (g, r read; r', out written; the world-1 headline): 8192 / 12288 / 16384 / 20480 / 24576 /
//        32768 elements -> 240 / 194-198 / 196-206 / 204 / 205 / 209 us;
//   12 B (g, r read; r' written; world > 1): 12288 / 16384 / 20480 -> 217-221 / 208-212 / 206 us;
//    8 B (no residual stream; no memory or a first step): 16384 -> 132, 32768 -> 107 us;
//        24576 / 28672 / 40960 -> 116 / 114 / 112 us.
template <bool HAS_RES, int MODE>
constexpr int kBytesOf = 4 + (HAS_RES ? 4 : 0) + (kWritesR<MODE> ? 4 : 0) + (kWritesOut<MODE> ? 4 : 0);
template <bool HAS_RES, int MODE>
constexpr int kVecOf = kBytesOf<HAS_RES, MODE> >= 16 ? kMainVec
                       : (kBytesOf<HAS_RES, MODE> >= 12 ? GRACE_MAIN_VEC_12B : GRACE_MAIN_VEC_NORES);
template <bool HAS_RES, int MODE> constexpr int kChunkOf = kMainBlock * 4 * kVecOf<HAS_RES, MODE>;
// (r05 A/B at BASELINE configs[4]'s 8.4 M-element shard, 12 B per element: 410 chunks of 20480
// leave CUs with 1-2 workgroups, yet chunks of 16384 (512, two per CU) or 12288 (683) ran the local
// step in 57.5-58.4 / 59.2-60.3 us against 57.3-57.4 -- the small bucket's main pass is bound by
// its per-workgroup latency, not by the balance; 8192 spills 176-200 B with the residual stream)
constexpr int kHistBins = 2048;                            // candidate histogram
constexpr int kStage = 1024;                               // LDS staging entries per list (all waves)
constexpr int kSelBlock = 1024;                            // single-workgroup selectors
constexpr int kSmallN = 32768;                             // single-workgroup path
constexpr int kSampleRunLen = 16;
constexpr int kSampleRuns = 2048;
constexpr int kSample = kSampleRuns * kSampleRunLen;       // 32768 keys, 32 per thread
#ifndef GRACE_FIN_BLOCKS
#define GRACE_FIN_BLOCKS 128
#endif
constexpr int kFinBlocks = GRACE_FIN_BLOCKS;
constexpr int kFinPer = 8;                                 // candidates per thread per round


struct TopkCtl {
  uint32_t thr_lo;
  uint32_t thr_hi;
  uint32_t shift;
  int32_t status;      // 0 fast path, 1 exact fallback, 2 a parallel-fallback wait ran out (aborted)
  uint32_t n_sure;
  uint32_t n_cand;
  uint32_t n_sel;
  uint32_t n_bnd;
  int32_t boundary_bin;
  uint32_t need;
  uint32_t ticket;     // finalize kernel arrival counter
  uint32_t n_bacc;     // boundary-list fill counter
  uint32_t bticket;    // bracket kernel arrival counter (reset by its last workgroup)
  uint32_t pad0;       // (unused; the parallel fallback's counters live in TopkWs::fb)
  uint32_t pad1;
  uint32_t thr_mid;    // provisional selection threshold of the fused main pass (key > thr_mid)
};
static_assert(sizeof(TopkCtl) == 64, "ctl layout");

// Diagnostic build only (-DGRACE_STAMPS): s_memrealtime stamps (100 MHz) at phase boundaries,
// stored in the free tail of the 256-byte ctl block of the workspace.  Never in shipped builds.
#ifdef GRACE_STAMPS
#define STAMP_IF(cond, ctlp, slot)                                                                 \
  do {                                                                                             \
    if (threadIdx.x == 0 && (cond))                                                                \
      reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(ctlp) + 64)[slot] =                     \
          __builtin_amdgcn_s_memrealtime();                                                        \
  } while (0)
#else
#define STAMP_IF(cond, ctlp, slot) do { } while (0)
#endif
#define STAMP(ctlp, slot) STAMP_IF(blockIdx.x == 0, ctlp, slot)

#ifndef GRACE_SAMPLE_MAX
#define GRACE_SAMPLE_MAX 131072
#endif
constexpr int kSampleMax = GRACE_SAMPLE_MAX;               // stratified sample size
// The sample a bucket's bracket draws: every element up to kSampleMax, else kSampleMax.  (r05
// A/B at BASELINE configs[4]'s 8.4 M-element shard: one sample per 256 elements, 32 K instead of
// 131 K, took the bracket from 16.6 to 14.1 us but doubled the candidates, finalize 11.8 -> 17.0
// us: local step 59.5 -> 58.7 us, within the spread -- the bracket's cost is its fixed LDS zeroing,
// flush and fan-in, not its random reads.)  r06, same shard, one box, two runs each: 64 K samples
// 54.0 / 54.4 us, 32 K 54.6 / 54.8, 131 K 55.6 / 56.6 (profiles/r06_sample_ab.txt) -- while at the
// 2^26-element headline 64 K costs +3 us: half the sample up to 2^24 elements.
constexpr int64_t kHalfSampleMaxN = (int64_t)1 << 24;
__host__ __device__ inline int64_t bracket_sample_n(int64_t n) {
  const int64_t cap = n <= kHalfSampleMaxN ? kSampleMax / 2 : kSampleMax;
  return n < cap ? n : cap;
}
constexpr int kSampleBlock = 1024;
#ifndef GRACE_BRACKET_BLOCK
#define GRACE_BRACKET_BLOCK 1024
#endif
// single-GPU bracket: one sample per thread.  A/B (step, one process): 1024 -> 232 us, 512 -> 236-240
// (twice the workgroups, each still one per CU for the 136 KB of LDS histograms), 256 -> 256
constexpr int kBracketBlock = GRACE_BRACKET_BLOCK;
constexpr int kBracketBins = 32768;                        // key >> 16: 1/64-octave bins
#ifndef GRACE_SAMPLE_RUN
#define GRACE_SAMPLE_RUN 1
#endif
constexpr int kBracketRun = GRACE_SAMPLE_RUN;              // adjacent elements per sampling thread
constexpr int kCoarseBins = 2048;                          // key >> 20: 1/8-octave bins
// A/B knob: the bracket's search in every main-pass workgroup instead of the bracket's last sampler.
// Measured slower (r05, tools/ab_main_search.sh, profiles/r05_main_search_ab.txt): headline step
// 0.2330-0.2373 vs 0.2294-0.2314 ms, topk_main 204-209 vs 198-200 us -- 5462 workgroups x 2096
// agent-scope histogram loads (46 MB at the memory side) and a search latency at every
// workgroup's start cost more than the bracket's tail they remove.
#ifndef GRACE_MAIN_SEARCH
#define GRACE_MAIN_SEARCH 0
#endif
constexpr bool kMainSearch = GRACE_MAIN_SEARCH != 0;       // the bracket's search in the main pass
constexpr int kHistStride = 1;
// copies of the bracket's sample histograms (workgroup b flushes into copy b % kSampleCopies; the
// search sums them): same-address device atomics serialise, and every sampling workgroup adds to
// the same popular bins
#ifndef GRACE_SAMPLE_COPIES
#define GRACE_SAMPLE_COPIES 1
#endif
constexpr int kSampleCopies = GRACE_SAMPLE_COPIES;

// Workspace layout.  Every counter / histogram region is left zeroed by the step that used it
// (the select kernel re-zeroes what the next step accumulates into), so the caller only has to
// zero the workspace once, at allocation.
struct TopkWs {
  TopkCtl* ctl;
  uint32_t* hist;      // candidate histogram [kHistBins]
  uint32_t* chist;     // coarse sample histogram [kCoarseBins] (single-GPU bracket)
  uint32_t* shist;     // fine sample histogram [kBracketBins]
  int2* cand;
  int2* bnd;
  int64_t cap;
  uint32_t* fb;        // parallel exact fallback scratch [kFbWords] (zero between uses)
  int32_t* hstatus;    // registered pinned host status word (grace_topk_status_word) or null
  uint32_t spin_max;   // bound of every parallel-fallback wait, in microseconds of wall time
                       // (grace_topk_fallback_spin_limit; s_memrealtime runs at 100 MHz)
};

static inline int64_t topk_cap(int64_t n, int64_t k) {
  int64_t c = 2 * k + 65536;
  return c < n ? c : n;
}

static inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// parallel exact fallback scratch (see parallel_exact): tickets, counters, histograms, slice counts
constexpr int kFbWordsHost = 64 + 3 * 2048 + 2 * 1024;
// the host word every top-k launch reports a run-out to, and the bound of the fallback's waits
static int32_t* g_topk_hstatus = nullptr;
// 2 s: the claimed-slice fallback always progresses, so only a true hang (a device so oversubscribed
// that a claimed slice's workgroup makes no progress for seconds) may trip it
static uint32_t g_fb_spin_max = 2000000u;

static TopkWs carve(void* ws, int64_t n, int64_t k) {
  char* p = reinterpret_cast<char*>(ws);
  TopkWs w;
  w.cap = topk_cap(n, k);
  w.ctl = reinterpret_cast<TopkCtl*>(p);
  p += 256;
  // right after ctl, at the same address for every (n, k): the workspace is shared by calls of
  // every shape, and the fallback's tickets and histograms must be zero wherever a call finds them
  w.fb = reinterpret_cast<uint32_t*>(p);
  p += align256(sizeof(uint32_t) * kFbWordsHost);
  w.hist = reinterpret_cast<uint32_t*>(p);
  p += align256(sizeof(uint32_t) * kHistBins * kHistStride);
  w.chist = reinterpret_cast<uint32_t*>(p);
  p += align256(sizeof(uint32_t) * kCoarseBins * kSampleCopies);
  w.shist = reinterpret_cast<uint32_t*>(p);
  p += align256(sizeof(uint32_t) * kBracketBins * kSampleCopies);
  w.cand = reinterpret_cast<int2*>(p);
  p += align256(sizeof(int2) * w.cap);
  w.bnd = reinterpret_cast<int2*>(p);
  w.hstatus = g_topk_hstatus;
  w.spin_max = g_fb_spin_max;
  return w;
}

static size_t ws_bytes(int64_t n, int64_t k) {
  const int64_t cap = topk_cap(n, k);
  return 256 + align256(sizeof(uint32_t) * kHistBins * kHistStride) +
         align256(sizeof(uint32_t) * kCoarseBins * kSampleCopies) +
         align256(sizeof(uint32_t) * kBracketBins * kSampleCopies) +
         2 * align256(sizeof(int2) * cap) + align256(sizeof(uint32_t) * kFbWordsHost);
}

// ------------------------------------------------------------------------------------------------
// event timer for the dominant kernel (bench.py reads it; off by default)
static int g_timer_on = 0;
static constexpr int kMaxEv = 8192;
static hipEvent_t g_ev[2 * kMaxEv];
static int g_ev_created = 0;
static int g_ev_used = 0;

// With the timer on, the dominant kernel is launched with hipExtLaunchKernelGGL, whose start / stop
// events ride on the kernel's own dispatch packet: no separate marker packets, so no extra
// system-scope release (an L2 writeback of every XCD, ~6 us per hipEventRecord on gfx950) is
// inserted between the step's kernels and the timed step is the untimed one.
// armed by grace_topk_arm_main_event: completes with the next main pass launched from this thread
static thread_local hipEvent_t t_main_ev = nullptr;

template <typename... KArgs, typename... Args>
static void launch_timed(void (*kern)(KArgs...), dim3 grid, dim3 block, hipStream_t s, Args... args) {
  if (t_main_ev) {
    hipEvent_t ev = t_main_ev;
    t_main_ev = nullptr;
    const bool timed = g_timer_on && g_ev_used < kMaxEv;
    const int slot = timed ? g_ev_used++ : 0;
    hipExtLaunchKernelGGL(kern, grid, block, 0, s, timed ? g_ev[2 * slot] : nullptr, ev, 0, args...);
    if (timed) (void)hipEventRecord(g_ev[2 * slot + 1], s);
  } else if (g_timer_on && g_ev_used < kMaxEv) {
    const int slot = g_ev_used++;
    hipExtLaunchKernelGGL(kern, grid, block, 0, s, g_ev[2 * slot], g_ev[2 * slot + 1], 0, args...);
  } else {
    kern<<<grid, block, 0, s>>>(args...);
  }
}

// ------------------------------------------------------------------------------------------------
// ------------------------------------------------------------------------------------------------
// Streaming accesses of the bucket are non-temporal (touched once per step): on gfx950 the
// nt 16-B loads+stores lift the 2-read/2-write stream from ~5.1 to ~6.4 TB/s (tools/hbm_probe).
typedef float f32x4 __attribute__((ext_vector_type(4)));
template <bool VEC>
__device__ __forceinline__ float4 load4(const float* p, int64_t i, int64_t n) {
  if (VEC && i + 3 < n) {
    const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p + i));
    return make_float4(v.x, v.y, v.z, v.w);
  }
  float4 v;
  v.x = i < n ? p[i] : 0.f;
  v.y = i + 1 < n ? p[i + 1] : 0.f;
  v.z = i + 2 < n ? p[i + 2] : 0.f;
  v.w = i + 3 < n ? p[i + 3] : 0.f;
  return v;
}
template <bool VEC>
__device__ __forceinline__ void store4(float* p, int64_t i, int64_t n, float4 v) {
  if (VEC && i + 3 < n) {
    const f32x4 x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<f32x4*>(p + i));
    return;
  }
  if (i < n) p[i] = v.x;
  if (i + 1 < n) p[i + 1] = v.y;
  if (i + 2 < n) p[i + 2] = v.z;
  if (i + 3 < n) p[i + 3] = v.w;
}
__device__ __forceinline__ float comp4(const float4& v, int j) {
  return j == 0 ? v.x : (j == 1 ? v.y : (j == 2 ? v.z : v.w));
}
__device__ __forceinline__ void set4(float4& v, int j, float x) {
  if (j == 0) v.x = x; else if (j == 1) v.y = x; else if (j == 2) v.z = x; else v.w = x;
}

struct StepArgs {
  const float* g;      // gradient (or x for compress-only)
  float* r;            // residual in/out (may be null for kDenseNone)
  float beta, gamma;
  int64_t n, k;
  float* vals;
  int32_t* idx;
  float* out;          // dense output (kDenseFused, kDenseOut)
  int64_t sample_n;    // stratified sample size (<= kSampleMax)
  int64_t stratum;     // n / sample_n
  // residual-sample carry (grace_topk_residual_step_carry), f32[carry_thr_off(sample_n) + 2]: the bracket writes
  // the step's t[pos(s)] to rs_out[s] (it computes them anyway), the finalize writes the step's
  // composite selection threshold (selected <=> comp_key >= T) as a u64 at rs_out + sample_n;
  // rs_in = the previous step's rs_out for this residual: the next bracket derives r'[pos(s)] from
  // it instead of reading r (half the sample's random DRAM reads).  Either may be null; both are
  // only used when kCarryMinStratum <= stratum.
  const float* rs_in;
  float* rs_out;
  // payload index of element 0 (segmented top-k: the segment's offset in the flat buffer); the
  // single-bucket engine leaves it 0.  Only payload indices carry it; r / out stay local.
  int64_t idx_base;
  // recycled dense output (grace_topk_residual_step_carry with prev_idx): `out` holds exactly the
  // previous step's result, whose non-zeros are among prev_idx[0 .. prev_count); the bracket launch
  // zeroes those and the main pass writes only the elements it selects (sparse), not 4 B each
  const int32_t* prev_idx;
  int64_t prev_count;
  // the residual the step READS (kResSwap: a second buffer; every other mode: r itself, set by
  // run_topk / seg_step_args)
  const float* r_in;
};

// the carry is for large buckets, where the bracket's random reads cost (stratum >= 256)
constexpr int64_t kCarryMinStratum = 256;
// word offset of the carry's u64 threshold after S sample words: 8-B aligned for any S (a segment's
// sample count n / 256 can be odd)
__host__ __device__ __forceinline__ int64_t carry_thr_off(int64_t S) { return (S + 1) & ~(int64_t)1; }

template <bool HAS_RES>
__device__ __forceinline__ float compensate(const StepArgs& a, int64_t i) {
  if constexpr (HAS_RES) return a.beta * a.r_in[i] + a.gamma * a.g[i];
  return a.g[i];
}

// ------------------------------------------------------------------------------------------------
// 1. bracket = sample (sample_n/1024 workgroups) + select (one workgroup).
//
// sample: every thread takes one element from its stratum of n / sample_n at a hashed offset
// (single elements, so spatially correlated gradients do not inflate the sample variance) and
// counts its key's top 16 bits (key >> 16: 1/64-octave bins) in an LDS histogram; non-zero bins
// are flushed with one global atomic each.
// select: reads the 32768-bin histogram with coalesced loads, finds both bracketing sample ranks
// with one block scan, rounds the thresholds OUTWARD to bin edges (the rounding only widens the
// candidate band) and re-zeroes the histogram and every counter the next kernels accumulate into.
__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7FEB352Du; x ^= x >> 15; x *= 0x846CA68Bu; x ^= x >> 16;
  return x;
}

// element index of sample sidx: a hashed offset inside its stratum [sidx * st, sidx * st + st)
__device__ __forceinline__ int64_t sample_pos(int64_t sidx, uint32_t st) {
  const uint32_t off = (uint32_t)(((uint64_t)hash32((uint32_t)sidx * 0x9E3779B9u + 0x5EEDu) * st) >> 32);
  return sidx * (int64_t)st + off;
}

#ifndef GRACE_SAMPLE_PER
#define GRACE_SAMPLE_PER 1
#endif
#ifndef GRACE_SAMPLE_DEFF
#define GRACE_SAMPLE_DEFF 1.0
#endif
// variance inflation allowed for in the bracket's margin (design effect of clustered samples)
constexpr double kSampleDeff = GRACE_SAMPLE_DEFF;
#ifndef GRACE_SAMPLE_SIGMA
#define GRACE_SAMPLE_SIGMA 6.0
#endif
constexpr double kSampleSigma = GRACE_SAMPLE_SIGMA;        // bracket half-width in binomial sigmas
constexpr double kSurePoisson = 1e-6;                      // small-sample "sure" rank: miss probability
constexpr int kSamplePer = GRACE_SAMPLE_PER;               // samples per thread: 1 is fastest --
                                                           // the strided samples are latency-bound
                                                           // random loads that want many waves

// The sample ranks (descending, 0-based) that bracket the k-th largest of n with ~kSampleSigma
// binomial sigmas, and the sample's own estimate of the k-th rank (the provisional threshold);
// r1 = the 1-based ranks clamped into the sample.
struct BracketRanks {
  int64_t rank_hi, rank_lo;
  uint32_t r1[3];
};
__device__ __forceinline__ BracketRanks bracket_ranks(int64_t S, int64_t k, int64_t n) {
  BracketRanks b;
  const double p = (double)k / (double)n;
  const double mu = p * (double)S;
  const double sd = sqrt(kSampleDeff * mu * (1.0 - p) + 1.0);
  b.rank_hi = (int64_t)floor(mu - kSampleSigma * sd - 2.0);   // < 0: nothing is "sure"
  b.rank_lo = (int64_t)ceil(mu + kSampleSigma * sd + 2.0);    // >= S: everything a candidate
  if (b.rank_hi < 0) {
    // Few samples above the k-th (a segment's 512..2048 samples at 1 %: mu ~ 5..20): the normal
    // margin leaves nothing sure, the candidate histogram then spans every key above lo and its
    // 1/16-octave bins put thousands of candidates in the boundary bin.  "Sure" fails (n_sure > k)
    // only when fewer than rank_hi + 1 samples fall among the k largest, an event of probability
    // P(Poisson(mu) <= rank_hi): take the largest rank_hi with that below kSurePoisson.  A miss is
    // still exact (the finalize's fallback), only slower.
    double term = exp(-mu), cdf = term;
    for (int64_t j = 0; j < 64 && cdf <= kSurePoisson; ++j) {
      b.rank_hi = j;
      term *= mu / (double)(j + 1);
      cdf += term;
    }
  }
  const int64_t rank_mid = (int64_t)floor(mu);
  b.r1[0] = (uint32_t)((b.rank_hi < 0 ? 0 : (b.rank_hi >= S ? S - 1 : b.rank_hi)) + 1);
  b.r1[1] = (uint32_t)((b.rank_lo < 0 ? 0 : (b.rank_lo >= S ? S - 1 : b.rank_lo)) + 1);
  b.r1[2] = (uint32_t)((rank_mid < 0 ? 0 : (rank_mid >= S ? S - 1 : rank_mid)) + 1);
  return b;
}
// candidate histogram bin of key (lo <= key <= hi): keys above the binned range share the top bin
__device__ __forceinline__ uint32_t cand_bin(uint32_t key, uint32_t lo, uint32_t sh) {
  return min((key - lo) >> sh, (uint32_t)kHistBins - 1u);
}
// the bracket from the fine bins (key >> 16) holding the three ranks: sure = key > hi (rounded up
// to the top of its bin: fewer sure), candidates from the bottom of the low bin (more candidates),
// the provisional threshold in the middle of its bin, clamped into the band
struct BracketThr { uint32_t lo, hi, sh, mid; };
__device__ __forceinline__ BracketThr bracket_thresholds(const BracketRanks& b, int64_t S, uint32_t d_hi,
                                                        uint32_t d_lo, uint32_t d_mid) {
  uint32_t hi = (d_hi << 16) | 0xFFFFu;
  // top of the binned key range: hi, or with nothing sure the top of the sample maximum's bin
  // (r1[0] = 1 then); the keys above it share the top bin (binning clamps), so the 2048 bins
  // resolve the band the k-th key lies in instead of every key up to +inf
  uint32_t top = hi;
  uint32_t lo = d_lo << 16;
  if (b.rank_hi < 0) hi = 0x7FFFFFFFu;
  if (b.rank_lo >= S) lo = 0u;
  if (lo > hi) lo = hi;
  if (top < lo) top = lo;
  uint32_t sh = 0;
  const uint64_t span = (uint64_t)top - (uint64_t)lo;   // keys lo..top -> bins 0..span>>sh
  while ((span >> sh) >= (uint64_t)kHistBins) ++sh;
  uint32_t mid = (d_mid << 16) | 0x8000u;
  mid = mid < lo ? lo : (mid > hi ? hi : mid);
  return BracketThr{lo, hi, sh, mid};
}
__device__ __forceinline__ void bracket_publish(TopkCtl* ctl, const BracketThr& t) {
  ctl->thr_lo = t.lo;
  ctl->thr_hi = t.hi;
  ctl->shift = t.sh;
  ctl->thr_mid = t.mid;
}

// The bracket's search, by one workgroup of NT threads once the sample histograms are complete:
// thread t owns kCPT consecutive coarse bins from the top down, one block scan finds the coarse bins
// of the three bracketing ranks, then one 16-lane group per rank scans that coarse bin's 16 fine
// bins (descending) for the first lane whose running count reaches the rank.  Every thread returns
// the same thresholds.  The histograms were filled by device atomics: agent-scope loads.
template <int NT>
__device__ __forceinline__ BracketThr bracket_search(const StepArgs& a, const TopkWs& w, uint32_t* s_w,
                                                     uint32_t* s_fc, uint32_t* s_res) {
  const int tid = threadIdx.x;
  const int64_t S = a.sample_n;
  const BracketRanks br = bracket_ranks(S, a.k, a.n);
  const uint32_t(&r1)[3] = br.r1;
  const uint32_t rk0 = br.r1[0], rk1 = br.r1[1], rk2 = br.r1[2];
  constexpr int kCPT = kCoarseBins / NT;
  static_assert(kCPT * NT == kCoarseBins && kCPT >= 1 && NT >= 64, "coarse bins tile the block");
  const int top = kCoarseBins - 1 - kCPT * tid;
  uint32_t hc[kCPT], hs = 0;
#pragma unroll
  for (int c = 0; c < kCPT; ++c) {
    uint32_t x[kSampleCopies];
#pragma unroll
    for (int q = 0; q < kSampleCopies; ++q)
      x[q] = __hip_atomic_load(w.chist + q * kCoarseBins + top - c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    hc[c] = 0;
#pragma unroll
    for (int q = 0; q < kSampleCopies; ++q) hc[c] += x[q];
    hs += hc[c];
  }
  if (tid < 6) s_fc[tid] = 0;
  const uint32_t ex = block_excl_scan<NT>(hs, s_w, nullptr);
#pragma unroll
  for (int q = 0; q < 3; ++q)
    if (ex < r1[q] && r1[q] <= ex + hs) {
      uint32_t acc = ex;
#pragma unroll
      for (int c = 0; c < kCPT; ++c) {
        if (r1[q] <= acc + hc[c]) {
          s_fc[2 * q] = (uint32_t)(top - c);
          s_fc[2 * q + 1] = acc;
          break;
        }
        acc += hc[c];
      }
    }
  __syncthreads();
  if (tid < 64) {
    const int q = tid >> 4, j = tid & 15;
    const bool act = q < 3;
    const uint32_t bin = act ? s_fc[2 * q] * 16 + (15 - j) : 0u;
    uint32_t v = 0u;
    if (act) {
      uint32_t x[kSampleCopies];
#pragma unroll
      for (int c = 0; c < kSampleCopies; ++c)
        x[c] = __hip_atomic_load(w.shist + c * kBracketBins + bin, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
      for (int c = 0; c < kSampleCopies; ++c) v += x[c];
    }
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      const uint32_t u = __shfl_up(v, o, 16);
      if (j >= o) v += u;
    }
    const int qc = act ? q : 0;
    // (selects of SSA values: a dynamic index, or selects of r1's elements that the compiler folds
    // back into one, keep r1 in scratch memory)
    const uint32_t rq = qc == 0 ? rk0 : (qc == 1 ? rk1 : rk2);
    const uint64_t bal = __ballot(act && s_fc[2 * qc + 1] + v >= rq);
    const uint32_t hm = (uint32_t)(bal >> (16 * q)) & 0xFFFFu;
    if (act && j == __ffs(hm) - 1) s_res[q] = bin;
  }
  __syncthreads();
  return bracket_thresholds(br, S, s_res[0], s_res[1], s_res[2]);
}

// Single-GPU bracket: sample + select in ONE launch.  The sample workgroups count their keys into
// a fine (key >> 16, 32768 bins) and a coarse (key >> 20, 2048 bins) LDS histogram and flush both
// with global atomics, wait for them (vmcnt(0)) and take a ticket; the last to arrive reads the
// merged COARSE histogram back with agent-scope loads (the other XCDs' atomics are not in its L2),
// finds the coarse bin of each bracketing rank, then reads only those bins' 16 fine counts.
// Nothing on this path waits on re-zeroing: the sample workgroups zero the counters the main pass
// accumulates into (the previous step's finalize has completed, stream order), and the finalize
// kernel zeroes both sample histograms once the main pass no longer needs them.
// recycled output: zero the previous result's non-zeros (its payload positions), kU index loads in
// flight per thread; the clear workgroups run beside the sample workgroups, whose random loads
// leave HBM mostly idle
__device__ __forceinline__ void clear_prev(const StepArgs& a, unsigned b, unsigned nb) {
  constexpr int kU = 8;
  const int64_t cnt = a.prev_count;
  for (int64_t j0 = (int64_t)b * kBracketBlock * kU + threadIdx.x; j0 < cnt; j0 += (int64_t)nb * kBracketBlock * kU) {
    int32_t ix[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t j = j0 + (int64_t)u * kBracketBlock;
      ix[u] = a.prev_idx[j < cnt ? j : j0];   // clamped, unconditional
    }
#pragma unroll
    for (int u = 0; u < kU; ++u)
      if (j0 + (int64_t)u * kBracketBlock < cnt && ix[u] >= 0 && ix[u] < a.n) a.out[ix[u]] = 0.f;
  }
}
constexpr int kClearPer = kBracketBlock * 8;   // previous-payload entries per clear workgroup and round
constexpr int kClearMax = 96;                   // clear workgroups at most

template <bool HAS_RES>
__global__ __launch_bounds__(kBracketBlock) void topk_bracket(StepArgs a, TopkWs w) {
  // workgroups past the sample grid clear the recycled output (no ticket: not part of the sample)
  const unsigned nsamp = (unsigned)((a.sample_n / kBracketRun + kBracketBlock - 1) / kBracketBlock);
  if (blockIdx.x >= nsamp) {
    clear_prev(a, blockIdx.x - nsamp, gridDim.x - nsamp);
    return;
  }
  __shared__ uint32_t lh[kBracketBins];
  __shared__ uint32_t lc[kCoarseBins];
  __shared__ uint32_t s_w[kSelBlock / kWave + 1];
  __shared__ uint32_t s_fc[6];
  __shared__ uint32_t s_res[3];
  __shared__ uint32_t s_last;
  const int tid = threadIdx.x;
  STAMP(w.ctl, 0);
  const uint32_t st = (uint32_t)a.stratum;
  const int64_t sidx = (int64_t)blockIdx.x * kBracketBlock + tid;
  // kBracketRun > 1 (A/B builds): every thread takes a run of adjacent elements at a hashed,
  // run-aligned offset in a stratum of kBracketRun * stratum elements -- fewer DRAM rows opened
  // per sample, at the price of samples that are no longer independent on correlated buckets
  const bool valid = sidx * kBracketRun < a.sample_n;
  float t[kBracketRun];
#pragma unroll
  for (int q = 0; q < kBracketRun; ++q) t[q] = 0.f;
  if (valid) {
    if constexpr (kBracketRun == 1) {
#ifdef GRACE_SAMPLE_SEQ   // diagnostic A/B build only: contiguous sample positions
      t[0] = compensate<HAS_RES>(a, sidx);
#else
      const int64_t pos = sample_pos(sidx, st);
      if (HAS_RES && a.rs_in) {
        // carried t'(pos) of this residual's previous step and that step's selection threshold:
        // r'(pos) exactly as its main pass + finalize left it, from one random DRAM read (g) per
        // sample instead of two
        const float tp = a.rs_in[sidx];
        const uint64_t Tp = *reinterpret_cast<const uint64_t*>(a.rs_in + carry_thr_off(a.sample_n));
        const float gv = a.g[pos];
        const float rp = comp_key(abs_key(tp), (uint32_t)pos) >= Tp ? tp - tp : tp;
        t[0] = a.beta * rp + a.gamma * gv;
      } else {
        t[0] = compensate<HAS_RES>(a, pos);
      }
      if (a.rs_out) a.rs_out[sidx] = t[0];   // this step's t(pos), for the next step's bracket
#endif
    } else {
      const uint32_t off = (uint32_t)(((uint64_t)hash32((uint32_t)sidx * 0x9E3779B9u + 0x5EEDu) * st) >> 32) *
                           kBracketRun;
      const int64_t i0 = sidx * (int64_t)st * kBracketRun + off;
#pragma unroll
      for (int q = 0; q < kBracketRun; ++q) t[q] = compensate<HAS_RES>(a, i0 + q);
    }
  }
  // counters of this step's main / finalize passes (their previous users have completed)
  if (blockIdx.x == 0 && tid >= 3 && tid < 12) reinterpret_cast<uint32_t*>(w.ctl)[tid] = 0u;
  if (blockIdx.x < (unsigned)(kHistBins / kBracketBlock))
    w.hist[(blockIdx.x * kBracketBlock + tid) * kHistStride] = 0u;
  for (int b = tid; b < kBracketBins; b += kBracketBlock) lh[b] = 0;
  for (int b = tid; b < kCoarseBins; b += kBracketBlock) lc[b] = 0;
  __syncthreads();
  STAMP(w.ctl, 1);
  if (valid) {
#pragma unroll
    for (int q = 0; q < kBracketRun; ++q) {
      const uint32_t key = abs_key(t[q]);
      atomicAdd(&lh[key >> 16], 1u);
      atomicAdd(&lc[key >> 20], 1u);
    }
  }
  __syncthreads();
  const int cp = (int)(blockIdx.x % kSampleCopies);
  for (int b = tid; b < kBracketBins; b += kBracketBlock)
    if (lh[b]) atomicAdd(&w.shist[cp * kBracketBins + b], lh[b]);
  for (int b = tid; b < kCoarseBins; b += kBracketBlock)
    if (lc[b]) atomicAdd(&w.chist[cp * kCoarseBins + b], lc[b]);
  STAMP(w.ctl, 2);
  // kMainSearch: no last arriver here -- every main-pass workgroup runs the search itself, a kernel
  // boundary later (the tail of waiting for the last sampler and one workgroup's search leaves the
  // chain, as the payload grouping's histogram pass did)
  if constexpr (kMainSearch) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) s_last = atomicAdd(&w.ctl->bticket, 1u) == nsamp - 1;
  __syncthreads();
  if (!s_last) return;
  STAMP_IF(true, w.ctl, 3);
  // sample ranks bracketing the k-th largest with ~6 sigma, and the sample's k-th estimate
  const BracketThr thr = bracket_search<kBracketBlock>(a, w, s_w, s_fc, s_res);
  STAMP_IF(true, w.ctl, 4);
  if (tid == 0) {
    // the fused main pass writes candidates above the provisional threshold as selected
    bracket_publish(w.ctl, thr);
    w.ctl->bticket = 0u;
  }
  STAMP_IF(true, w.ctl, 5);
}

// ------------------------------------------------------------------------------------------------
// 2. main streaming pass
//
// Each workgroup streams one 12288-element chunk: 3 groups of 4 float4 per lane per array, with
// the next group's loads issued before the current group is classified (16-B loads, 8 in flight
// per lane).  Per group every lane flags its elements with key >= lo, a DPP wave scan of the
// counts places them in the wave's own LDS region (no atomic), and the staged entries leave with
// one global atomic per list and workgroup at the end, sorted into sure / candidate there.
#ifndef GRACE_MAIN_GROUP
#define GRACE_MAIN_GROUP 4
#endif
constexpr int kGroup = GRACE_MAIN_GROUP;
#ifndef GRACE_MAIN_RING
#define GRACE_MAIN_RING 0
#endif
constexpr bool kMainRing = GRACE_MAIN_RING != 0;   // main_chunk_v2's copy-free load ring (A/B knob)


__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  return v;
}

// FAST = aligned buffers and a chunk entirely inside the bucket: unconditional nt 16-B loads and
// stores (a guarded load makes hipcc wait vmcnt(0) at the merge, serialising every load).
template <bool FAST>
__device__ __forceinline__ float4 ld4(const float* p, int64_t i, int64_t n) {
  if constexpr (FAST) {
    const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p + i));
    return make_float4(v.x, v.y, v.z, v.w);
  } else {
    return load4<false>(p, i, n);
  }
}
template <bool FAST>
__device__ __forceinline__ void st4(float* p, int64_t i, int64_t n, float4 v) {
  if constexpr (FAST) {
    const f32x4 x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<f32x4*>(p + i));
  } else {
    store4<false>(p, i, n, v);
  }
}

template <bool HAS_RES, bool FAST>
__device__ __forceinline__ void load_group(const StepArgs& a, int64_t gbase, float4 (&rv)[kGroup],
                                           float4 (&gv)[kGroup]) {
#pragma unroll
  for (int u = 0; u < kGroup; ++u) {
    const int64_t i0 = gbase + (int64_t)u * (kMainBlock * 4);
    if constexpr (HAS_RES) rv[u] = ld4<FAST>(a.r_in, i0, a.n);
    gv[u] = ld4<FAST>(a.g, i0, a.n);
  }
}

constexpr int kMainWaves = kMainBlock / 64;
constexpr int kStageWave = kStage / kMainWaves;            // each wave's own region of each list

struct MainShared {
  uint32_t hist[kHistBins];
  // v3: ONE staged list of flagged elements, kListWave entries per wave (sure / candidate decided at
  // the flush); v2 (A/B build): sure = list[0 .. kStage), candidates = list[kStage .. 2 kStage)
  int2 list[2 * kStage];
  uint32_t wcnt[kMainWaves];   // each wave's staged count (v2: packed sure | cand << 16), for the flush
  uint32_t gbase[2];           // the chunk's reservations in the global sure / candidate lists
  uint32_t cnt[2];             // v3 flush: the chunk's sure / candidate counts, then their positions
};
constexpr int kListWave = 2 * kStage / kMainWaves;         // v3: each wave's region of the one list

// wave-wide inclusive scan of one uint32 per lane: DPP row shifts within each 16-lane row, then
// the row broadcasts (gfx9 row_bcast:15 / row_bcast:31) -- 6 VALU, no LDS, no loop
__device__ __forceinline__ uint32_t wave_incl_scan_dpp(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);   // row_shr:1
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);   // row_shr:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);   // row_shr:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);   // row_shr:8
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);   // row_bcast:15
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);   // row_bcast:31
  return v;
}

// v2 classification of one group (kGroup float4 per lane per array, already loaded): a DPP wave
// scan of the lanes' packed 16|16 counts places the entries in the wave's OWN regions of the two
// LDS lists at its running fill (wfill, wave-uniform) -- no reservation atomic (r05: the per-lane
// ds_add_rtn of r04 became the compiler's atomic-optimizer loop, a readlane / writelane per active
// lane); one branch per flagged element position for both lists; the candidate histogram is built
// from the staged entries at the flush instead of a masked ds_add per element.  Returns the wave's
// new fill.
// UNIT: beta = gamma = 1, t = r + g (1 * x is x bit for bit, so this is the reference's
// beta * r + gamma * g).
template <bool HAS_RES, int MODE, bool FAST, bool SKEL = false, bool SPARSE = false, bool UNIT = false>
__device__ __forceinline__ uint32_t classify_group(const StepArgs& a, const TopkWs& w, MainShared& sm, uint32_t lo,
                                                   uint32_t hi, uint32_t sh, uint32_t mid, int64_t gbase,
                                                   const float4 (&rc)[kGroup], const float4 (&gc)[kGroup],
                                                   uint32_t wfill) {
  const int64_t n = a.n;
  float4 t[kGroup];
  uint32_t msure = 0, mcand = 0;   // bit u*4+j
#pragma unroll
  for (int u = 0; u < kGroup; ++u) {
    if constexpr (HAS_RES && UNIT) {
      t[u].x = rc[u].x + gc[u].x;
      t[u].y = rc[u].y + gc[u].y;
      t[u].z = rc[u].z + gc[u].z;
      t[u].w = rc[u].w + gc[u].w;
    } else if constexpr (HAS_RES) {
      t[u].x = a.beta * rc[u].x + a.gamma * gc[u].x;
      t[u].y = a.beta * rc[u].y + a.gamma * gc[u].y;
      t[u].z = a.beta * rc[u].z + a.gamma * gc[u].z;
      t[u].w = a.beta * rc[u].w + a.gamma * gc[u].w;
    } else {
      t[u] = gc[u];
    }
    const int64_t i0 = gbase + (int64_t)u * (kMainBlock * 4);
    float4 rout = t[u], dout = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float tv = comp4(t[u], j);
      const uint32_t key = abs_key(tv);
#ifdef GRACE_MAIN_STREAM_ONLY   // diagnostic A/B build only: the streaming ceiling of this layout
      constexpr bool kSkel = true;
#else
      constexpr bool kSkel = SKEL;
#endif
      // SKEL (grace_topk_stream_probe): the same loads and stores with no classification -- the
      // streaming ceiling of this exact layout (nothing is listed; the per-chunk flushes still run)
      //
      // The flags are integer arithmetic on the 31-bit keys (sign bits of differences that cannot
      // overflow), not comparisons: 16 comparisons per group became 16 live 64-bit lane masks, and
      // the compiler spilled SGPRs to VGPR lanes (r05: 31 spills, 349 v_readlane in topk_main).
      const uint32_t vbit = (FAST || i0 + j < n) ? 1u : 0u;
      const uint32_t f_sure = kSkel ? 0u : ((hi - key) >> 31) & vbit;              // key > hi
      const uint32_t f_lo = kSkel ? 0u : (((key - lo) >> 31) ^ 1u) & vbit;         // key >= lo
      msure |= f_sure << (u * 4 + j);
      mcand |= (f_lo & (f_sure ^ 1u)) << (u * 4 + j);
      if constexpr (kProv<MODE>) {
        // sure elements, and candidates above the provisional threshold, are written as selected;
        // the finalize fixes up only the candidates whose final decision differs.  lo <= mid <= hi
        // (bracket_publish), so "sure or (candidate and key > mid)" is key > mid: an all-ones
        // mask selects r' = t - t and out = 0 + t bitwise
        const uint32_t m = kSkel ? 0u : (uint32_t)((int32_t)(mid - key) >> 31) & (0u - vbit);
        set4(rout, j, u2f((f2u(tv - tv) & m) | (f2u(tv) & ~m)));
        if constexpr (kWritesOut<MODE>) {
          set4(dout, j, u2f(f2u(0.f + tv) & m));
          // recycled output: only the selected elements are written (the rest is already zero)
          if constexpr (SPARSE) if (m) a.out[i0 + j] = 0.f + tv;
        }
      }
    }
    if constexpr (kWritesR<MODE>) st4<FAST>(a.r, i0, n, rout);
    if constexpr (kWritesOut<MODE> && !SPARSE) st4<FAST>(a.out, i0, n, dout);
  }
  if constexpr (SKEL) return wfill;
  const uint32_t msel = msure | mcand;
  const uint32_t cnt = __popc(msure) | (__popc(mcand) << 16);
  const uint32_t incl = wave_incl_scan_dpp(cnt);
  const uint32_t tot = __builtin_amdgcn_readlane(incl, 63);
  if (msel) {
    const uint32_t cs = cnt & 0xFFFFu, cc = cnt >> 16;
    const uint32_t bse = wfill + incl - cnt;   // this lane's first slots in the wave's regions
    uint32_t ps = bse & 0xFFFFu, pc = bse >> 16;
    const uint32_t wb = (threadIdx.x >> 6) * kStageWave;
    // entries past the wave's region spill to the global lists (rare: one global atomic per lane)
    const uint32_t over_s = ps + cs > (uint32_t)kStageWave ? min(ps + cs - (uint32_t)kStageWave, cs) : 0u;
    const uint32_t over_c = pc + cc > (uint32_t)kStageWave ? min(pc + cc - (uint32_t)kStageWave, cc) : 0u;
    uint32_t gs = 0, gcn = 0;
    if (over_s) gs = atomicAdd(&w.ctl->n_sure, over_s);
    if (over_c) gcn = atomicAdd(&w.ctl->n_cand, over_c);
#pragma unroll
    for (int u = 0; u < kGroup; ++u) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int b = u * 4 + j;
        if ((msel >> b) & 1u) {
          const int64_t i = gbase + (int64_t)u * (kMainBlock * 4) + j;
          const float tv = comp4(t[u], j);
          const int2 e = make_int2((int)i, (int)f2u(tv));
          if ((msure >> b) & 1u) {
            if (ps < (uint32_t)kStageWave) {
              sm.list[wb + ps] = e;
            } else if (gs < (uint32_t)a.k) {
              a.vals[gs] = tv; a.idx[gs] = (int32_t)(e.x + a.idx_base); ++gs;
            }
            ++ps;
          } else {
            if (pc < (uint32_t)kStageWave) {
              sm.list[kStage + wb + pc] = e;
            } else {
              atomicAdd(&sm.hist[cand_bin(abs_key(tv), lo, sh)], 1u);
              if (gcn < (uint32_t)w.cap) w.cand[gcn] = e;
              ++gcn;
            }
            ++pc;
          }
        }
      }
    }
  }
  return wfill + tot;
}

// ------------------------------------------------------------------------------------------------
// v3 classification (r06).  The r05 SQ counters of the no-memory main pass (4 B read per element,
// profiles/r06_nomem_sq_summary.json) showed 2640 VALU instructions per wave for 128 elements per
// lane -- 20 per element, 35 us of the SIMDs' issue time against a 43 us read stream, half of them
// in v2's walk over the 16 element positions of a group (one divergent block per position that any
// lane flagged, ~10 of 16 with ~15 flagged elements per wave and group).  v3 keeps per element only
// what every element needs: its dense outputs, if any, and ONE flag bit (key >= lo) shifted into a
// per-lane 16-bit mask -- a compare and an add-with-carry.  The flagged elements (~1.5 %) are then
// visited by a per-lane set-bit loop whose trip count is the wave's largest popcount (typically 2),
// which classifies them exactly and stages them in the wave's region of ONE LDS list; the flush
// splits sure entries from candidates.
#ifndef GRACE_MAIN_V2
#define GRACE_MAIN_V2 0
#endif
constexpr bool kMainV3 = GRACE_MAIN_V2 == 0;   // A/B knob: 1 builds the r05 classification

// t[e >> 2].(e & 3) of a lane whose element e is known only at run time: a select tree on e's bits
__device__ __forceinline__ float sel16(const float4 (&t)[4], uint32_t e) {
  const float4 p = (e & 4u) ? t[1] : t[0];
  const float4 q = (e & 4u) ? t[3] : t[2];
  const float4 c = (e & 8u) ? q : p;
  const float x = (e & 1u) ? c.y : c.x;
  const float y = (e & 1u) ? c.w : c.z;
  return (e & 2u) ? y : x;
}

// a flagged element past its wave's LDS region (massive ties inside the band): classified here and
// appended with one global atomic (rare; the finalize sees list overflows as usual)
__device__ __forceinline__ void spill_entry(const StepArgs& a, const TopkWs& w, MainShared& sm, int2 e, uint32_t key,
                                            uint32_t lo, uint32_t hi, uint32_t sh) {
  if (key > hi) {
    const uint32_t gp = atomicAdd(&w.ctl->n_sure, 1u);
    if (gp < (uint32_t)a.k) {
      a.vals[gp] = u2f((uint32_t)e.y);
      a.idx[gp] = (int32_t)(e.x + a.idx_base);
    }
  } else {
    atomicAdd(&sm.hist[cand_bin(key, lo, sh)], 1u);
    const uint32_t gp = atomicAdd(&w.ctl->n_cand, 1u);
    if (gp < (uint32_t)w.cap) w.cand[gp] = e;
  }
}

template <bool HAS_RES, int MODE, bool FAST, bool SKEL = false, bool SPARSE = false, bool UNIT = false>
__device__ __forceinline__ uint32_t classify_group_v3(const StepArgs& a, const TopkWs& w, MainShared& sm, uint32_t lo,
                                                      uint32_t hi, uint32_t sh, uint32_t mid, int64_t gbase,
                                                      const float4 (&rc)[kGroup], const float4 (&gc)[kGroup],
                                                      uint32_t wfill) {
  static_assert(kGroup == 4, "sel16 picks from 4 float4 per lane");
#ifdef GRACE_MAIN_STREAM_ONLY   // diagnostic A/B build only: the streaming ceiling of this layout
  constexpr bool kSkel = true;
#else
  constexpr bool kSkel = SKEL;
#endif
  // the exact provisional decision (key > mid) per element, where a dense output depends on it
  constexpr bool kDenseProv = kProv<MODE> && (kWritesR<MODE> || (kWritesOut<MODE> && !SPARSE));
  const int64_t n = a.n;
  const float lo_f = u2f(lo);
  float4 t[kGroup];
  uint32_t m = 0;   // element e = u * 4 + j flagged at bit 15 - e
#pragma unroll
  for (int u = 0; u < kGroup; ++u) {
    if constexpr (HAS_RES && UNIT) {
      t[u].x = rc[u].x + gc[u].x;
      t[u].y = rc[u].y + gc[u].y;
      t[u].z = rc[u].z + gc[u].z;
      t[u].w = rc[u].w + gc[u].w;
    } else if constexpr (HAS_RES) {
      t[u].x = a.beta * rc[u].x + a.gamma * gc[u].x;
      t[u].y = a.beta * rc[u].y + a.gamma * gc[u].y;
      t[u].z = a.beta * rc[u].z + a.gamma * gc[u].z;
      t[u].w = a.beta * rc[u].w + a.gamma * gc[u].w;
    } else {
      t[u] = gc[u];
    }
    const int64_t i0 = gbase + (int64_t)u * (kMainBlock * 4);
    float4 rout = t[u], dout = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float tv = comp4(t[u], j);
      bool f;
      if constexpr (kDenseProv) {
        // sure elements, and candidates above the provisional threshold, are written as selected
        // (r' = t - t, out = 0 + t); the finalize fixes up the candidates it decides otherwise.
        // lo <= mid <= hi (bracket_publish), so that set is key > mid
        const uint32_t key = abs_key(tv);
        const bool sel = !kSkel && key > mid;
        set4(rout, j, sel ? tv - tv : tv);
        if constexpr (kWritesOut<MODE> && !SPARSE) set4(dout, j, sel ? 0.f + tv : 0.f);
        f = key >= lo;
      } else {
        // a superset test, made exact in the loop below: |t| >= lo, or NaN (unordered); a denormal
        // flushed to 0 would compare as 0 on both sides
        f = !(fabsf(tv) < lo_f);
      }
      if (!FAST) f = f && i0 + j < n;
      if (kSkel) f = false;
      m = m + m + (f ? 1u : 0u);
    }
    if constexpr (kWritesR<MODE>) st4<FAST>(a.r, i0, n, rout);
    if constexpr (kWritesOut<MODE> && !SPARSE) st4<FAST>(a.out, i0, n, dout);
  }
  if constexpr (SKEL) return wfill;
  const uint32_t cnt = __popc(m);
  const uint32_t incl = wave_incl_scan_dpp(cnt);
  const uint32_t tot = __builtin_amdgcn_readlane(incl, 63);
  uint32_t slot = wfill + incl - cnt;   // this lane's first slot in the wave's region
  const uint32_t wb = (threadIdx.x >> 6) * kListWave;
  uint32_t ovf = 0;                      // flagged elements past the region (bit 15 - e)
  while (m) {
    const uint32_t b = (uint32_t)__builtin_ctz(m);
    m &= m - 1u;
    const uint32_t e = 15u - b;
    const float tv = sel16(t, e);
    const uint32_t key = abs_key(tv);
    const bool ok = key >= lo;             // exact (the float flag was a superset)
    // (recycled output: the flush writes the provisional picks, so that no global store sits
    // between a group's loads and their waits -- vmcnt counts stores too)
    // a flag the exact test rejects leaves an empty entry
    const int2 ent = ok ? make_int2((int)(gbase + (int64_t)(e >> 2) * (kMainBlock * 4) + (e & 3u)), (int)f2u(tv))
                        : make_int2(-1, 0);
    if (slot < (uint32_t)kListWave) sm.list[wb + slot] = ent;
    else ovf |= (ok ? 1u : 0u) << b;
    ++slot;
  }
  // rare: entries past the wave's region leave through global atomics, outside the loop above so
  // that its memory operations stay store-only
  if (__ballot(ovf != 0)) {
    while (ovf) {
      const uint32_t b = (uint32_t)__builtin_ctz(ovf);
      ovf &= ovf - 1u;
      const uint32_t e = 15u - b;
      const float tv = sel16(t, e);
      const int64_t i = gbase + (int64_t)(e >> 2) * (kMainBlock * 4) + (e & 3u);
      const uint32_t key = abs_key(tv);
      if constexpr (SPARSE && kWritesOut<MODE>) if (key > mid) a.out[i] = 0.f + tv;
      spill_entry(a, w, sm, make_int2((int)i, (int)f2u(tv)), key, lo, hi, sh);
    }
  }
  return wfill + tot;
}

// v3 flush: the waves' regions are concatenated; one pass counts sure / candidate entries with wave
// ballots, one reservation per list and chunk, a second pass writes them (wave ballot ranks, one LDS
// add per wave and list); candidates are counted into the LDS histogram there
template <bool SPARSE_OUT>
__device__ __forceinline__ void flush_staged_v3(const StepArgs& a, const TopkWs& w, MainShared& sm, uint32_t lo,
                                                uint32_t hi, uint32_t sh, uint32_t mid, uint32_t wfill) {
  const int tid = threadIdx.x;
  if ((tid & 63) == 0) sm.wcnt[tid >> 6] = min(wfill, (uint32_t)kListWave);
  if (tid == 0) sm.cnt[0] = 0u;
  __syncthreads();
  uint32_t off[kMainWaves + 1];
  off[0] = 0;
#pragma unroll
  for (int v = 0; v < kMainWaves; ++v) off[v + 1] = off[v] + sm.wcnt[v];
  const uint32_t ne = off[kMainWaves];
  auto entry = [&](uint32_t j) {
    int v = 0;
#pragma unroll
    for (int x = 1; x < kMainWaves; ++x) v += j >= off[x];
    return sm.list[v * kListWave + (j - off[v])];
  };
  uint32_t ns_w = 0, nc_w = 0;   // this wave's counts (wave-uniform)
  for (uint32_t j0 = 0; j0 < ne; j0 += kMainBlock) {
    const uint32_t j = j0 + tid;
    const int2 e = j < ne ? entry(j) : make_int2(-1, 0);
    const bool sure = e.x >= 0 && abs_key(u2f((uint32_t)e.y)) > hi;
    ns_w += (uint32_t)__popcll(__ballot(sure));
    nc_w += (uint32_t)__popcll(__ballot(e.x >= 0 && !sure));
  }
  if ((tid & 63) == 0 && (ns_w | nc_w)) atomicAdd(&sm.cnt[0], ns_w | (nc_w << 16));
  __syncthreads();
  if (tid == 0) {
    const uint32_t c = sm.cnt[0], ns = c & 0xFFFFu, nc = c >> 16;
#ifdef GRACE_DIAG_NORESERVE   // timing-only A/B build (wrong results): no atomic return to wait for
    sm.gbase[0] = (uint32_t)((blockIdx.x * 97u) % (uint32_t)(a.k > 2048 ? a.k - 2048 : 1));
    sm.gbase[1] = (uint32_t)((blockIdx.x * 53u) % (uint32_t)(w.cap > 2048 ? w.cap - 2048 : 1));
    (void)ns; (void)nc;
#else
    sm.gbase[0] = ns ? atomicAdd(&w.ctl->n_sure, ns) : 0u;
    sm.gbase[1] = nc ? atomicAdd(&w.ctl->n_cand, nc) : 0u;
#endif
    sm.cnt[0] = 0u;
    sm.cnt[1] = 0u;
  }
  __syncthreads();
  for (uint32_t j0 = 0; j0 < ne; j0 += kMainBlock) {
    const uint32_t j = j0 + tid;
    const int2 e = j < ne ? entry(j) : make_int2(-1, 0);
    const uint32_t key = abs_key(u2f((uint32_t)e.y));
    const bool sure = e.x >= 0 && key > hi, cand = e.x >= 0 && !sure;
    const uint64_t bs = __ballot(sure), bc = __ballot(cand);
    uint32_t base_s = 0, base_c = 0;
    if ((tid & 63) == 0) {
      if (bs) base_s = atomicAdd(&sm.cnt[0], (uint32_t)__popcll(bs));
      if (bc) base_c = atomicAdd(&sm.cnt[1], (uint32_t)__popcll(bc));
    }
    base_s = __builtin_amdgcn_readfirstlane(base_s);
    base_c = __builtin_amdgcn_readfirstlane(base_c);
    // recycled output: only the provisional picks (key > mid, mid >= lo) are written
    if constexpr (SPARSE_OUT) if (e.x >= 0 && key > mid) a.out[e.x] = 0.f + u2f((uint32_t)e.y);
    if (sure) {
      const uint32_t gp = sm.gbase[0] + base_s + lane_rank(bs);
      if (gp < (uint32_t)a.k) {
        a.vals[gp] = u2f((uint32_t)e.y);
        a.idx[gp] = (int32_t)(e.x + a.idx_base);
      }
    } else if (cand) {
      atomicAdd(&sm.hist[cand_bin(key, lo, sh)], 1u);
      const uint32_t gp = sm.gbase[1] + base_c + lane_rank(bc);
      if (gp < (uint32_t)w.cap) w.cand[gp] = e;
    }
  }
  __syncthreads();   // the list and wcnt are free for the next chunk
}

template <bool HAS_RES, int MODE, bool FAST, bool SKEL = false, bool SPARSE = false, bool UNIT = false>
__device__ __forceinline__ uint32_t classify_group_sel(const StepArgs& a, const TopkWs& w, MainShared& sm, uint32_t lo,
                                                       uint32_t hi, uint32_t sh, uint32_t mid, int64_t gbase,
                                                       const float4 (&rc)[kGroup], const float4 (&gc)[kGroup],
                                                       uint32_t wfill) {
  if constexpr (kMainV3)
    return classify_group_v3<HAS_RES, MODE, FAST, SKEL, SPARSE, UNIT>(a, w, sm, lo, hi, sh, mid, gbase, rc, gc, wfill);
  else
    return classify_group<HAS_RES, MODE, FAST, SKEL, SPARSE, UNIT>(a, w, sm, lo, hi, sh, mid, gbase, rc, gc, wfill);
}

template <bool HAS_RES, int MODE, bool FAST, bool SKEL = false, bool SPARSE = false, bool UNIT = false,
          int NV = kVecOf<HAS_RES, MODE>>
__device__ __forceinline__ uint32_t main_chunk_v2(const StepArgs& a, const TopkWs& w, MainShared& sm,
                                                  uint32_t lo, uint32_t hi, uint32_t sh, uint32_t mid, int64_t chunk) {
  constexpr int NG = NV / kGroup;
  static_assert(NG * kGroup == NV, "groups tile the chunk (group 2 / 3 / 6 lost 0-5 %, A/B)");
  const int64_t cbase = chunk * (kMainBlock * 4 * NV) + (int64_t)threadIdx.x * 4;
  uint32_t wfill = 0;
  if constexpr (kMainV3 && FAST) {
    // v3: the group loop fully unrolled over a static ring of R group buffers (R - 1 groups' loads
    // in flight ahead of the one being classified).  Every load is unconditional at compile time:
    // a load that a run-time condition may skip (the r05 ring's `q + R - 1 < NG`), or a rotating
    // copy of the next group's buffer into the current one (v2), made hipcc wait vmcnt(0) -- for
    // every load in flight -- once per group
    constexpr int R = HAS_RES ? 2 : 3;   // buffers: 2 x (r, g) or 3 x g
    constexpr int64_t S = (int64_t)kGroup * (kMainBlock * 4);
    float4 rb[R][kGroup], gb[R][kGroup];
#pragma unroll
    for (int p = 0; p < R - 1; ++p)
      if (p < NG) load_group<HAS_RES, FAST>(a, cbase + p * S, rb[p], gb[p]);
#pragma unroll
    for (int q = 0; q < NG; ++q) {
      // no instruction crosses a group boundary: the scheduler would otherwise hoist later groups'
      // loads and spill (the unrolled ring at 128 VGPRs with 15-70 spilled)
      __builtin_amdgcn_sched_barrier(0);
      if (q + R - 1 < NG) load_group<HAS_RES, FAST>(a, cbase + (q + R - 1) * S, rb[(q + R - 1) % R], gb[(q + R - 1) % R]);
      wfill = classify_group_v3<HAS_RES, MODE, FAST, SKEL, SPARSE, UNIT>(a, w, sm, lo, hi, sh, mid, cbase + q * S,
                                                                         rb[q % R], gb[q % R], wfill);
    }
    return wfill;
  }
  if constexpr (kMainRing) {
    // A static ring of R group buffers, R - 1 groups' loads in flight ahead of the one being
    // classified: the loop body is unrolled over the R slots, so no buffer is ever copied.  (The
    // rotating copies of the loops below, next -> current after each group, made hipcc wait
    // vmcnt(0) -- for the next group's loads AND the stores just issued -- before every group: each
    // wave's memory pipeline drained once per group.)
    constexpr int R = HAS_RES ? 2 : 3;   // buffers: 2 x (r, g) or 3 x g, 64 / 48 VGPRs
    constexpr int64_t S = (int64_t)kGroup * (kMainBlock * 4);
    float4 rb[R][kGroup], gb[R][kGroup];
#pragma unroll
    for (int p = 0; p < R - 1; ++p)
      if (p < NG) load_group<HAS_RES, FAST>(a, cbase + p * S, rb[p], gb[p]);
#pragma unroll 1
    for (int q0 = 0; q0 < NG; q0 += R) {
#pragma unroll
      for (int j = 0; j < R; ++j) {
        const int q = q0 + j;
        if (q < NG) {   // workgroup-uniform
          if (q + R - 1 < NG) load_group<HAS_RES, FAST>(a, cbase + (q + R - 1) * S, rb[(j + R - 1) % R], gb[(j + R - 1) % R]);
          wfill = classify_group_sel<HAS_RES, MODE, FAST, SKEL, SPARSE, UNIT>(a, w, sm, lo, hi, sh, mid, cbase + q * S,
                                                                          rb[j], gb[j], wfill);
        }
      }
    }
    return wfill;
  }
  float4 rc[kGroup], gc[kGroup];
#ifndef GRACE_MAIN_PREFETCH1   // A/B build only: one group ahead on every stream
  if constexpr (!HAS_RES && NG >= 3) {
    // one input stream (g only): the loads run TWO groups ahead, so a lane keeps as many bytes in
    // flight as with the residual stream (8 x 16 B)
    float4 g1[kGroup], g2[kGroup];
    load_group<false, FAST>(a, cbase, rc, gc);
    load_group<false, FAST>(a, cbase + kGroup * (kMainBlock * 4), rc, g1);
#pragma unroll 1
    for (int q = 0; q < NG; ++q) {
      const int64_t gbase = cbase + (int64_t)q * kGroup * (kMainBlock * 4);
      if (q + 2 < NG) load_group<false, FAST>(a, gbase + 2 * kGroup * (kMainBlock * 4), rc, g2);
      wfill = classify_group_sel<false, MODE, FAST, SKEL, SPARSE, UNIT>(a, w, sm, lo, hi, sh, mid, gbase, rc, gc, wfill);
#pragma unroll
      for (int u = 0; u < kGroup; ++u) { gc[u] = g1[u]; g1[u] = g2[u]; }
    }
    return wfill;
  }
#endif
  load_group<HAS_RES, FAST>(a, cbase, rc, gc);
#pragma unroll 1
  for (int q = 0; q < NG; ++q) {
    const int64_t gbase = cbase + (int64_t)q * kGroup * (kMainBlock * 4);
    float4 rn[kGroup], gn[kGroup];
    if (q + 1 < NG) load_group<HAS_RES, FAST>(a, gbase + kGroup * (kMainBlock * 4), rn, gn);
    wfill = classify_group_sel<HAS_RES, MODE, FAST, SKEL, SPARSE, UNIT>(a, w, sm, lo, hi, sh, mid, gbase, rc, gc, wfill);
#pragma unroll
    for (int u = 0; u < kGroup; ++u) { rc[u] = rn[u]; gc[u] = gn[u]; }
  }
  return wfill;
}

// the staged lists of one chunk leave with one global atomic per list: the waves' regions are
// concatenated in wave order (v2: the staged candidates are counted into the LDS histogram here)
__device__ __forceinline__ void flush_staged_v2(const StepArgs& a, const TopkWs& w, MainShared& sm, uint32_t lo,
                                                uint32_t sh, uint32_t wfill) {
  const int tid = threadIdx.x;
  if ((tid & 63) == 0) sm.wcnt[tid >> 6] = wfill;
  __syncthreads();
  uint32_t os[kMainWaves + 1], oc[kMainWaves + 1];
  os[0] = oc[0] = 0;
#pragma unroll
  for (int v = 0; v < kMainWaves; ++v) {
    const uint32_t f = sm.wcnt[v];
    os[v + 1] = os[v] + min(f & 0xFFFFu, (uint32_t)kStageWave);
    oc[v + 1] = oc[v] + min(f >> 16, (uint32_t)kStageWave);
  }
  const uint32_t ns = os[kMainWaves], nc = oc[kMainWaves];
  if (tid == 0) {
    // one reservation per chunk and list (5461 per step on each counter: as 8 copies, a timing-only
    // build, the main pass was 2 us faster in 196 -- within the spread, so the one counter stays)
#ifdef GRACE_DIAG_NORESERVE   // timing-only A/B build (wrong results): no atomic return to wait for
    sm.gbase[0] = (uint32_t)((blockIdx.x * 97u) % (uint32_t)(a.k > 2048 ? a.k - 2048 : 1));
    sm.gbase[1] = (uint32_t)((blockIdx.x * 53u) % (uint32_t)(w.cap > 2048 ? w.cap - 2048 : 1));
#else
    sm.gbase[0] = ns ? atomicAdd(&w.ctl->n_sure, ns) : 0u;
    sm.gbase[1] = nc ? atomicAdd(&w.ctl->n_cand, nc) : 0u;
#endif
  }
  __syncthreads();
  for (uint32_t j = tid; j < ns; j += kMainBlock) {
    const uint32_t gp = sm.gbase[0] + j;
    if (gp < (uint32_t)a.k) {
      int v = 0;
#pragma unroll
      for (int x = 1; x < kMainWaves; ++x) v += j >= os[x];
      const int2 e = sm.list[v * kStageWave + (j - os[v])];
      a.vals[gp] = u2f((uint32_t)e.y);
      a.idx[gp] = (int32_t)(e.x + a.idx_base);
    }
  }
  for (uint32_t j = tid; j < nc; j += kMainBlock) {
    const uint32_t gp = sm.gbase[1] + j;
    int v = 0;
#pragma unroll
    for (int x = 1; x < kMainWaves; ++x) v += j >= oc[x];
    const int2 e = sm.list[kStage + v * kStageWave + (j - oc[v])];
    atomicAdd(&sm.hist[cand_bin(abs_key(u2f((uint32_t)e.y)), lo, sh)], 1u);
    if (gp < (uint32_t)w.cap) w.cand[gp] = e;
  }
  __syncthreads();   // the lists and wcnt are free for the next chunk
}

template <bool SPARSE_OUT = false>
__device__ __forceinline__ void flush_staged(const StepArgs& a, const TopkWs& w, MainShared& sm, uint32_t lo,
                                             uint32_t hi, uint32_t sh, uint32_t mid, uint32_t wfill) {
  if constexpr (kMainV3) flush_staged_v3<SPARSE_OUT>(a, w, sm, lo, hi, sh, mid, wfill);
  else flush_staged_v2(a, w, sm, lo, sh, wfill);
}

// NV: float4 per lane per chunk
template <bool HAS_RES, int MODE, bool VEC, bool SKEL = false, bool SPARSE = false, int NV = kVecOf<HAS_RES, MODE>>
__global__ __launch_bounds__(kMainBlock, 4) void topk_main(StepArgs a, TopkWs w) {   // <= 128 VGPRs: 4 WGs/CU
  __shared__ MainShared sm;
  const int tid = threadIdx.x;
  // SKEL (the in-bench streaming ceiling): only the loads and stores -- no histogram zeroing, list
  // flushes or barriers, so the ceiling is a strictly lighter kernel than the one it bounds (with
  // the flushes left in, the real pass beat its fastest launch by 0.5 % on one box)
  if constexpr (!SKEL) {
    for (int b = tid; b < kHistBins; b += kMainBlock) sm.hist[b] = 0;
  }
  uint32_t lo, hi, sh, mid;
  if constexpr (kMainSearch && !SKEL) {
    __shared__ uint32_t s_w[kMainBlock / kWave + 1], s_fc[6], s_res[3];
    const BracketThr t = bracket_search<kMainBlock>(a, w, s_w, s_fc, s_res);
    lo = t.lo; hi = t.hi; sh = t.sh; mid = t.mid;
    if (blockIdx.x == 0 && tid == 0) bracket_publish(w.ctl, t);   // for the finalize (next launch)
  } else {
    lo = w.ctl->thr_lo; hi = w.ctl->thr_hi; sh = w.ctl->shift; mid = w.ctl->thr_mid;
  }
  constexpr int64_t kCh = (int64_t)kMainBlock * 4 * NV;
  const int64_t nchunks = (a.n + kCh - 1) / kCh;
  const bool unit = HAS_RES && a.beta == 1.f && a.gamma == 1.f;
  if constexpr (!SKEL) __syncthreads();
  // one chunk per workgroup (grid-stride if the grid is capped); the staged lists leave after
  // every chunk, the histogram once at the end
  for (int64_t chunk = blockIdx.x; chunk < nchunks; chunk += gridDim.x) {
    uint32_t wfill;
    if (VEC && (chunk + 1) * kCh <= a.n && unit)
      wfill = main_chunk_v2<HAS_RES, MODE, VEC, SKEL, SPARSE, true, NV>(a, w, sm, lo, hi, sh, mid, chunk);
    else if (VEC && (chunk + 1) * kCh <= a.n)
      wfill = main_chunk_v2<HAS_RES, MODE, VEC, SKEL, SPARSE, false, NV>(a, w, sm, lo, hi, sh, mid, chunk);
    else
      wfill = main_chunk_v2<HAS_RES, MODE, false, SKEL, SPARSE, false, NV>(a, w, sm, lo, hi, sh, mid, chunk);
    if constexpr (!SKEL) flush_staged<SPARSE && kWritesOut<MODE>>(a, w, sm, lo, hi, sh, mid, wfill);
    (void)wfill;
  }
  if constexpr (SKEL) return;
  __syncthreads();
  for (int b = tid; b < kHistBins; b += kMainBlock) {
    const uint32_t h = sm.hist[b];
    if (h) atomicAdd(&w.hist[b * kHistStride], h);
  }
}

// ------------------------------------------------------------------------------------------------
// ------------------------------------------------------------------------------------------------
// selected element sinks shared by the boundary / fallback / small kernels
template <int MODE>
__device__ __forceinline__ void emit(const StepArgs& a, uint32_t pos, int64_t i, float v) {
  a.vals[pos] = v;
  a.idx[pos] = (int32_t)(i + a.idx_base);
  if constexpr (kWritesR<MODE>) a.r[i] = v - v;
  if constexpr (kWritesOut<MODE>) a.out[i] = 0.f + v;   // (0 + d) of the Python sum
}

// Ordered (ascending index) single-workgroup write of every element with composite >= T over a
// source f(i) of length n: payload from `pos0`, dense outputs rewritten for every element.
template <int MODE, int BLOCK = kSelBlock, typename F>
__device__ void block_write_selected(const StepArgs& a, const F& f, int64_t n, uint64_t T,
                                     uint32_t pos0, uint32_t* s_w) {
  uint32_t run = pos0;
  for (int64_t j0 = 0; j0 < n; j0 += BLOCK) {
    const int64_t i = j0 + threadIdx.x;
    float v = 0.f;
    bool sel = false;
    if (i < n) {
      v = f(i);
      sel = comp_key(abs_key(v), (uint32_t)i) >= T;
    }
    uint32_t tot;
    const uint32_t ex = block_excl_scan<BLOCK>(sel ? 1u : 0u, s_w, &tot);
    if (i < n) {
      if (sel) {
        emit<MODE>(a, run + ex, i, v);
      } else {
        if constexpr (kWritesR<MODE>) a.r[i] = v;
        if constexpr (kWritesOut<MODE>) a.out[i] = 0.f;
      }
    }
    run += tot;
  }
}

// 3. finalize (+ boundary): every finalize workgroup scans the candidate histogram for the
// boundary bin B; candidates above B go to the payload (one block scan + one global atomic per
// round), those in B to the boundary list.  The last workgroup to arrive then ranks the boundary
// list exactly by (key, -index) -- or, if the sampled bracket failed or a list overflowed, runs the
// exact single-workgroup radix select over the whole bucket (slow, rare, same result).
// Generic over the workgroup size and over agent-scope loads (AG: for a caller that reads data other
// workgroups wrote earlier in the same launch).  A main + finalize fusion built on it (write-through
// main stores, the last 64 chunks finalizing) was correct but 30 us slower per step, so the
// finalize stays its own launch.
constexpr int kPairCap = 1024;   // boundary lists up to this size are ranked pairwise

template <int BLOCK>
struct FinShared {
  uint32_t s_w[BLOCK / kWave + 1];
  uint32_t hist[2048];
  uint64_t s_comp[kPairCap];
  int2 s_ent[kPairCap];
  uint32_t s_res[2];
  int s_B;
  uint32_t s_need, s_pos, s_last, s_claim;
};

template <bool AG>
__device__ __forceinline__ uint32_t ld_u32(const uint32_t* p) {
  if constexpr (AG) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return *p;
}
template <bool AG>
__device__ __forceinline__ float ld_f32(const float* p) {
  if constexpr (AG) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return *p;
}
template <bool AG>
__device__ __forceinline__ int2 ld_i2(const int2* p) {
  if constexpr (AG) return ld_agent_i2(p);
  return *p;
}

// t as recorded by the main pass (fallback input); agent-scope loads when AG
template <int MODE, bool AG>
struct MainTs {
  const float* g; const float* r; const float* out;
  const float* rin; float beta, gamma;   // kResSwap: t recomputed from g and the untouched r_in
  __device__ float operator()(int64_t i) const {
    if constexpr (MODE == kDenseNone || MODE == kDenseOut) return g[i];
    if constexpr (MODE == kResSwap) return rin ? beta * rin[i] + gamma * g[i] : g[i];
    if constexpr (MODE == kDenseRes) return ld_f32<AG>(r + i);
    const float o = ld_f32<AG>(out + i), rr = ld_f32<AG>(r + i);   // both issued: no dependent load
    return f2u(o) != 0u ? o : rr;
  }
  // four consecutive elements (i % 4 == 0, 16-B aligned buffers): 16-B loads unless AG
  __device__ float4 quad(int64_t i) const {
    if constexpr (AG) {
      return make_float4((*this)(i), (*this)(i + 1), (*this)(i + 2), (*this)(i + 3));
    } else {
      if constexpr (MODE == kDenseNone || MODE == kDenseOut) return *reinterpret_cast<const float4*>(g + i);
      if constexpr (MODE == kResSwap) {
        const float4 gg = *reinterpret_cast<const float4*>(g + i);
        if (!rin) return gg;
        const float4 rr = *reinterpret_cast<const float4*>(rin + i);
        return make_float4(beta * rr.x + gamma * gg.x, beta * rr.y + gamma * gg.y, beta * rr.z + gamma * gg.z,
                           beta * rr.w + gamma * gg.w);
      }
      if constexpr (MODE == kDenseRes) return *reinterpret_cast<const float4*>(r + i);
      const float4 o = *reinterpret_cast<const float4*>(out + i), rr = *reinterpret_cast<const float4*>(r + i);
      return make_float4(f2u(o.x) != 0u ? o.x : rr.x, f2u(o.y) != 0u ? o.y : rr.y, f2u(o.z) != 0u ? o.z : rr.z,
                         f2u(o.w) != 0u ? o.w : rr.w);
    }
  }
};

// the step's composite selection threshold into the residual-sample carry (selected <=> comp >= T)
__device__ __forceinline__ void carry_threshold(const StepArgs& a, uint64_t T) {
  if (a.rs_out) *reinterpret_cast<uint64_t*>(a.rs_out + carry_thr_off(a.sample_n)) = T;
}

// the boundary list into LDS (pairwise-ranking case); issued by the last workgroup BEFORE its own
// deferred scattered writes, so the in-order vmcnt wait for these loads does not also wait for them
template <int BLOCK>
__device__ __forceinline__ bool boundary_preload(const TopkWs& w, bool ok, uint32_t need, uint32_t nb,
                                                 FinShared<BLOCK>& fs) {
  if (!ok || need == 0 || nb > (uint32_t)kPairCap) return false;
  for (int j = threadIdx.x; j < (int)nb; j += BLOCK) {
    const int2 e = ld_agent_i2(w.bnd + j);
    fs.s_ent[j] = e;
    fs.s_comp[j] = comp_key(abs_key(u2f((uint32_t)e.y)), (uint32_t)e.x);
  }
  return true;
}

// boundary-bin entry not selected: in the fused mode undo a provisional selection (key > mid)
template <int MODE>
__device__ __forceinline__ void unselect(const StepArgs& a, int2 e, uint32_t mid) {
  if constexpr (kProv<MODE>) {
    const float v = u2f((uint32_t)e.y);
    if (abs_key(v) > mid) {
      if constexpr (kWritesR<MODE>) a.r[e.x] = v;
      if constexpr (kWritesOut<MODE>) a.out[e.x] = 0.f;
    }
  }
}

template <int MODE, int BLOCK, bool AG>
__device__ void boundary_work(const StepArgs& a, const TopkWs& w, bool ok, uint32_t need, uint32_t nb,
                              FinShared<BLOCK>& fs, bool preloaded, uint32_t mid) {
  const uint32_t k = (uint32_t)a.k;
  if (ok) {
    if (need == 0) {   // exactly k sure elements: selected <=> key > thr_hi
      if (threadIdx.x == 0) carry_threshold(a, ((uint64_t)w.ctl->thr_hi + 1) << 32);
      return;
    }
    const uint32_t pos0 = k - need;
    if (nb <= (uint32_t)kPairCap) {
      // rank by pairwise comparison of unique composites; G adjacent lanes share one entry's
      // comparisons and combine their counts with xor-shuffles
      const int nbi = (int)nb;
      if (!preloaded) boundary_preload<BLOCK>(w, ok, need, nb, fs);
      int G = 1;
      while (G < 16 && nbi * (G * 2) <= BLOCK) G *= 2;
      __syncthreads();
      const int part = threadIdx.x % G;
      for (int el = threadIdx.x / G; el < nbi; el += BLOCK / G) {
        const uint64_t me = fs.s_comp[el];
        uint32_t rank = 0;
        for (int q = part; q < nbi; q += G) rank += fs.s_comp[q] > me;
        for (int o = 1; o < G; o <<= 1) rank += __shfl_xor(rank, o, 64);
        if (part == 0) {
          const int2 e = fs.s_ent[el];
          if (rank == need - 1) carry_threshold(a, me);
          if (rank < need) emit<MODE>(a, pos0 + rank, e.x, u2f((uint32_t)e.y));
          else unselect<MODE>(a, e, mid);
        }
      }
      return;
    }
    const int2* bnd = w.bnd;
    auto src = [bnd](int64_t j) {
      const int2 e = ld_agent_i2(bnd + j);
      return comp_key(abs_key(u2f((uint32_t)e.y)), (uint32_t)e.x);
    };
    const uint64_t T = block_select_comp<BLOCK>(src, nb, need, fs.hist, fs.s_w, fs.s_res);
    if (threadIdx.x == 0) { fs.s_pos = 0; carry_threshold(a, T); }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < nb; j += BLOCK) {
      const int2 e = ld_agent_i2(bnd + j);
      if (comp_key(abs_key(u2f((uint32_t)e.y)), (uint32_t)e.x) >= T) {
        const uint32_t p = atomicAdd(&fs.s_pos, 1u);
        emit<MODE>(a, pos0 + p, e.x, u2f((uint32_t)e.y));
      } else {
        unselect<MODE>(a, e, mid);
      }
    }
    return;
  }
  // ---- exact fallback over the whole bucket (bracket failed or a list overflowed)
  if (threadIdx.x == 0) w.ctl->status = 1;
  const MainTs<MODE, AG> f{a.g, a.r, a.out, a.r_in != a.r ? a.r_in : nullptr, a.beta, a.gamma};
  auto src = [f](int64_t i) { return comp_key(abs_key(f(i)), (uint32_t)i); };
  const uint64_t T = block_select_comp<BLOCK>(src, a.n, k, fs.hist, fs.s_w, fs.s_res);
  if (threadIdx.x == 0) carry_threshold(a, T);
  block_write_selected<MODE, BLOCK>(a, f, a.n, T, 0u, fs.s_w);
}

// One round of routed candidates: payload writes of the above-boundary ones (bits of fsel) from
// slot ps on, and their residual / dense writes -- in the fused mode only where the main pass's
// provisional decision (key > mid) was wrong, in both directions (fbelow: below the boundary bin).
template <int MODE>
__device__ __forceinline__ void write_round(const StepArgs& a, const int2 (&e)[kFinPer], uint32_t fsel,
                                            uint32_t fbelow, uint32_t ps, uint32_t mid, TopkCtl* dbg_ctl = nullptr) {
#pragma unroll
  for (int u = 0; u < kFinPer; ++u) {
    const float v = u2f((uint32_t)e[u].y);
    const bool above_mid = abs_key(v) > mid;
    if ((fsel >> u) & 1u) {
      a.vals[ps] = v;
      a.idx[ps] = (int32_t)(e[u].x + a.idx_base);
      if constexpr (MODE == kDenseRes) a.r[e[u].x] = v - v;
      if constexpr (kProv<MODE>) {
        if (!above_mid) {
          if constexpr (kWritesR<MODE>) a.r[e[u].x] = v - v;
          if constexpr (kWritesOut<MODE>) a.out[e[u].x] = 0.f + v;
        }
      }
      ++ps;
    } else if (kProv<MODE> && ((fbelow >> u) & 1u) && above_mid) {
      if constexpr (kWritesR<MODE>) a.r[e[u].x] = v;
      if constexpr (kWritesOut<MODE>) a.out[e[u].x] = 0.f;
    }
  }
#ifdef GRACE_STAMPS   // diagnostic: fix-up writes of this round (ctl stamp slot 18: selected below mid, 19: rejected above)
  if (dbg_ctl) {
    uint32_t f1 = 0, f2 = 0;
#pragma unroll
    for (int u = 0; u < kFinPer; ++u) {
      const bool am = abs_key(u2f((uint32_t)e[u].y)) > mid;
      f1 += ((fsel >> u) & 1u) && !am;
      f2 += !((fsel >> u) & 1u) && ((fbelow >> u) & 1u) && am;
    }
    if (f1) atomicAdd(reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(dbg_ctl) + 64) + 18, (unsigned long long)f1);
    if (f2) atomicAdd(reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(dbg_ctl) + 64) + 19, (unsigned long long)f2);
  }
#endif
}

// ---- parallel exact fallback (the sampled bracket missed or a list overflowed: in practice massive
// ties, e.g. a bucket that is mostly exact zeros, or a constant one).  The finalize workgroups
// radix-select the k-th largest KEY over the whole bucket together, one digit per phase (3 phases),
// then take the ties at that key lowest index first from per-slice counts: a count phase and an
// ordered write phase.  The bucket is cut into slices that the workgroups CLAIM one at a time
// (a ticket per phase), and a phase ends when every slice of it is DONE (a second counter per
// phase), not when every workgroup has arrived.  So a workgroup only ever waits for slices that a
// running workgroup has claimed: the fallback needs no co-residency and cannot deadlock when other
// kernels (another process, RCCL) hold CUs -- a workgroup that starts late finds the slices taken
// and only follows the phases.  Every wait is still bounded (TopkWs::spin_max): a wait that runs out
// aborts the fallback in every workgroup (no payload written past k) and reports it in ctl->status
// (2) and in the registered pinned host word (grace_topk_status_word), which the Python layer turns
// into TopKWaitError.  Scratch: the workspace's fallback region (kFbWords), zero on entry; the last
// workgroup to leave re-zeroes what was accumulated.
constexpr int kFbSlicesMax = 1024;
constexpr int kFbSliceMin = 4096;
// fallback scratch, uint32 words: claim tickets [0, 8), done counters [16, 24), the abort flag (32)
// and the exit ticket (48) on 64-B lines of their own, then the three digit histograms and the
// per-slice (key > T, key == T) counts
constexpr int kFbClaim = 0, kFbDone = 16, kFbAbort = 32, kFbExit = 48, kFbHist = 64;
constexpr int kFbCnt = kFbHist + 3 * 2048;
constexpr int kFbWords = kFbCnt + 2 * kFbSlicesMax;
static_assert(kFbWords == kFbWordsHost, "fallback scratch size");

__device__ __forceinline__ uint32_t ld_agent_u32(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// one thread: stop the fallback everywhere and report it (device ctl and the host word)
__device__ __forceinline__ void fb_abort(const TopkWs& w) {
  __hip_atomic_store(w.fb + kFbAbort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_fetch_max(&w.ctl->status, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (w.hstatus) __hip_atomic_fetch_or(w.hstatus, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// every thread of the workgroup: wait until phase p's done counter reaches `nsl` (sc1 polls of a
// counter that only receives device atomics, after which the phase's data is read with sc1 loads).
// false (for every thread) when the fallback was aborted, here or elsewhere.
template <int BLOCK>
__device__ bool fb_wait(const TopkWs& w, int p, uint32_t nsl, FinShared<BLOCK>& fs) {
  if (threadIdx.x == 0) {
    uint32_t ok = 1;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    const uint64_t lim = (uint64_t)w.spin_max * 100u;   // 100 MHz ticks
    for (;;) {
      asm volatile("" ::: "memory");
      if (ld_agent_u32(w.fb + kFbDone + p) >= nsl) break;
      if (ld_agent_u32(w.fb + kFbAbort)) { ok = 0; break; }
      if (__builtin_amdgcn_s_memrealtime() - t0 >= lim) { fb_abort(w); ok = 0; break; }
      __builtin_amdgcn_s_sleep(2);
    }
    fs.s_res[0] = ok;
  }
  __syncthreads();
  const bool ok = fs.s_res[0] != 0;
  __syncthreads();
  return ok;
}

// one wave-aggregated key into the LDS histogram, for the bin of the wave's first active lane:
// degenerate buckets (ties: all zeros, a constant) put every key of a wave in one bin, and a
// workgroup's LDS atomics on one address serialise (loop exits can leave lanes inactive)
__device__ __forceinline__ void hist_add_agg(uint32_t* hist, int bin) {
  const int b0 = __builtin_amdgcn_readfirstlane(bin);
  const uint64_t same = __ballot(bin == b0);
  const int lead = __ffsll((unsigned long long)__ballot(1)) - 1;
  if (bin >= 0 && bin != b0) atomicAdd(&hist[bin], 1u);
  if (b0 >= 0 && (int)(threadIdx.x & 63) == lead) atomicAdd(&hist[b0], (uint32_t)__popcll(same));
}

constexpr int kFbUnroll = 8;   // parallel fallback: elements per thread per ordered-write round
constexpr int kFbQ = 8;        // parallel fallback: quads in flight per thread (histogram / count passes)

template <int MODE, int BLOCK, bool AG>
__device__ void parallel_exact(const StepArgs& a, const TopkWs& w, int fcnt, FinShared<BLOCK>& fs) {
  const int t = threadIdx.x;
  const uint32_t k = (uint32_t)a.k;
  uint32_t* fb = w.fb;
  // slices of whole quads (16-B loads) when the buffers are 16-B aligned; [q1, s1) is a scalar tail
  const bool vq = !AG && ((reinterpret_cast<uintptr_t>(a.g) | reinterpret_cast<uintptr_t>(a.r) |
                           reinterpret_cast<uintptr_t>(a.out)) & 15u) == 0;
  int64_t L = (a.n + kFbSlicesMax - 1) / kFbSlicesMax;
  L = L < kFbSliceMin ? kFbSliceMin : ((L + 3) & ~(int64_t)3);
  const uint32_t nsl = (uint32_t)((a.n + L - 1) / L);
  if (t == 0) __hip_atomic_fetch_max(&w.ctl->status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const MainTs<MODE, AG> f{a.g, a.r, a.out, a.r_in != a.r ? a.r_in : nullptr, a.beta, a.gamma};
  auto bounds = [&](uint32_t s, int64_t& s0, int64_t& q1, int64_t& s1) {
    s0 = (int64_t)s * L;
    s1 = s0 + L < a.n ? s0 + L : a.n;
    q1 = vq ? s0 + ((s1 - s0) & ~(int64_t)3) : s0;
  };
  // fn(key, in) for every element of slice s, in no particular order; every load of a round
  // issued before any key is used
  auto for_keys = [&](uint32_t s, auto&& fn) {
    int64_t s0, q1, s1;
    bounds(s, s0, q1, s1);
    for (int64_t b = s0 + 4 * (int64_t)t; b < q1; b += 4 * (int64_t)BLOCK * kFbQ) {
      float4 v[kFbQ];
#pragma unroll
      for (int u = 0; u < kFbQ; ++u) {
        const int64_t i = b + 4 * (int64_t)u * BLOCK;
        v[u] = f.quad(i < q1 ? i : s0);
      }
#pragma unroll
      for (int u = 0; u < kFbQ; ++u) {
        const bool in = b + 4 * (int64_t)u * BLOCK < q1;
        fn(abs_key(v[u].x), in); fn(abs_key(v[u].y), in); fn(abs_key(v[u].z), in); fn(abs_key(v[u].w), in);
      }
    }
    for (int64_t i = q1 + t; i < s1; i += BLOCK) fn(abs_key(f(i)), true);
  };
  // runs body(s) for every slice of phase p this workgroup claims; the next claim is issued before
  // the current slice's work (its ticket latency hides behind the loads); returns the slice count
  auto claim_loop = [&](int p, auto&& body) -> uint32_t {
    if (t == 0) fs.s_claim = atomicAdd(fb + kFbClaim + p, 1u);
    __syncthreads();
    uint32_t s = fs.s_claim, mine = 0;
    __syncthreads();
    while (s < nsl) {
      uint32_t nxt = 0;
      if (t == 0) nxt = atomicAdd(fb + kFbClaim + p, 1u);
      body(s);
      ++mine;
      if (t == 0) fs.s_claim = nxt;
      __syncthreads();
      s = fs.s_claim;
      __syncthreads();
    }
    return mine;
  };
  // this workgroup's slices of phase p are complete: its stores / atomics performed, then one add
  auto done = [&](int p, uint32_t mine) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0 && mine) atomicAdd(fb + kFbDone + p, mine);
  };
  bool ok = true;
  // 1. the exact k-th largest key T (31-bit keys: digits of 11, 11 and 9 bits)
  uint32_t prefix = 0, pmask = 0, rem = k;
  for (int p = 0; p < 3 && ok; ++p) {
    const int shift = p == 0 ? 20 : (p == 1 ? 9 : 0);
    const uint32_t dmask = p < 2 ? 2047u : 511u;
    for (int b = t; b < 2048; b += BLOCK) fs.hist[b] = 0;
    __syncthreads();
    const uint32_t mine = claim_loop(p, [&](uint32_t s) {
      for_keys(s, [&](uint32_t key, bool in) {
        hist_add_agg(fs.hist, in && (key & pmask) == prefix ? (int)((key >> shift) & dmask) : -1);
      });
    });
    __syncthreads();
    if (mine)
      for (int b = t; b < 2048; b += BLOCK)
        if (fs.hist[b]) atomicAdd(fb + kFbHist + p * 2048 + b, fs.hist[b]);
    done(p, mine);
    ok = fb_wait<BLOCK>(w, p, nsl, fs);
    if (!ok) break;
    for (int b = t; b < 2048; b += BLOCK) fs.hist[b] = ld_agent_u32(fb + kFbHist + p * 2048 + b);
    __syncthreads();
    uint32_t above;
    const int d = find_bin_desc<BLOCK, 2048>(fs.hist, rem, fs.s_w, fs.s_res, &above);
    rem -= above;
    prefix |= (uint32_t)d << shift;
    pmask |= dmask << shift;
  }
  const uint32_t T = prefix, need_eq = rem;    // take every key > T and the need_eq lowest-index == T
  // 2. per-slice counts
  if (ok) {
    const uint32_t mine = claim_loop(3, [&](uint32_t s) {
      uint32_t ngt = 0, neq = 0;
      for_keys(s, [&](uint32_t key, bool in) {
        ngt += in && key > T;
        neq += in && key == T;
      });
      uint32_t tgt, teq;
      block_excl_scan<BLOCK>(ngt, fs.s_w, &tgt);
      block_excl_scan<BLOCK>(neq, fs.s_w, &teq);
      if (t == 0) {
        __hip_atomic_store(fb + kFbCnt + 2 * s, tgt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(fb + kFbCnt + 2 * s + 1, teq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    });
    done(3, mine);
    ok = fb_wait<BLOCK>(w, 3, nsl, fs);
  }
  // 3. each slice in index order: selected-before = (# key > T before) + min(# key == T before,
  //    need_eq); each thread owns kFbUnroll consecutive elements of a round (two quads when whole),
  //    one block scan per round; r' and the dense output leave as 16-B stores for whole quads
  static_assert(kFbUnroll == 8, "two quads per thread per round");
  if (ok) {
    claim_loop(4, [&](uint32_t s) {
      if (s == 0 && t == 0 && need_eq == 0) carry_threshold(a, ((uint64_t)T + 1) << 32);
      uint32_t pg = 0, pe = 0;                 // counts of the slices before s
      for (uint32_t j = t; j < s; j += BLOCK) {
        pg += ld_agent_u32(fb + kFbCnt + 2 * j);
        pe += ld_agent_u32(fb + kFbCnt + 2 * j + 1);
      }
      uint32_t gt_run, eq_run;
      block_excl_scan<BLOCK>(pg, fs.s_w, &gt_run);
      block_excl_scan<BLOCK>(pe, fs.s_w, &eq_run);
      int64_t s0, q1, s1;
      bounds(s, s0, q1, s1);
      for (int64_t j0 = s0; j0 < s1; j0 += (int64_t)BLOCK * kFbUnroll) {
        const int64_t ib = j0 + (int64_t)t * kFbUnroll;
        const bool whole = ib + kFbUnroll <= q1;
        float v[kFbUnroll];
        if (whole) {
          const float4 x0 = f.quad(ib), x1 = f.quad(ib + 4);
          v[0] = x0.x; v[1] = x0.y; v[2] = x0.z; v[3] = x0.w; v[4] = x1.x; v[5] = x1.y; v[6] = x1.z; v[7] = x1.w;
        } else {
#pragma unroll
          for (int u = 0; u < kFbUnroll; ++u) v[u] = f(ib + u < s1 ? ib + u : s0);
        }
        uint32_t cg = 0, ce = 0;
#pragma unroll
        for (int u = 0; u < kFbUnroll; ++u) {
          const uint32_t key = abs_key(v[u]);
          cg += ib + u < s1 && key > T;
          ce += ib + u < s1 && key == T;
        }
        uint32_t tot;
        const uint32_t ex = block_excl_scan<BLOCK>(cg | (ce << 16), fs.s_w, &tot);
        uint32_t g_before = gt_run + (ex & 0xFFFFu), e_before = eq_run + (ex >> 16);
        float rv[kFbUnroll], ov[kFbUnroll];
#pragma unroll
        for (int u = 0; u < kFbUnroll; ++u) {
          const int64_t i = ib + u;
          rv[u] = v[u];
          ov[u] = 0.f;
          if (i < s1) {
            const uint32_t key = abs_key(v[u]);
            const bool gt = key > T, eq = key == T;
            if (gt || (eq && e_before < need_eq)) {
              if (eq && e_before == need_eq - 1) carry_threshold(a, comp_key(T, (uint32_t)i));   // the last tie taken
              const uint32_t pos = g_before + min(e_before, need_eq);
              if (pos < k) {   // always, unless the counts were corrupted
                a.vals[pos] = v[u];
                a.idx[pos] = (int32_t)(i + a.idx_base);
              }
              rv[u] = v[u] - v[u];
              ov[u] = 0.f + v[u];   // (0 + d) of the Python sum
            }
            g_before += gt;
            e_before += eq;
          }
        }
        if constexpr (MODE != kDenseNone) {
          if (whole) {
            if constexpr (kWritesR<MODE>) {
              *reinterpret_cast<float4*>(a.r + ib) = make_float4(rv[0], rv[1], rv[2], rv[3]);
              *reinterpret_cast<float4*>(a.r + ib + 4) = make_float4(rv[4], rv[5], rv[6], rv[7]);
            }
            if constexpr (kWritesOut<MODE>) {
              *reinterpret_cast<float4*>(a.out + ib) = make_float4(ov[0], ov[1], ov[2], ov[3]);
              *reinterpret_cast<float4*>(a.out + ib + 4) = make_float4(ov[4], ov[5], ov[6], ov[7]);
            }
          } else {
#pragma unroll
            for (int u = 0; u < kFbUnroll; ++u) {
              if (ib + u < s1) {
                if constexpr (kWritesR<MODE>) a.r[ib + u] = rv[u];
                if constexpr (kWritesOut<MODE>) a.out[ib + u] = ov[u];
              }
            }
          }
        }
        gt_run += tot & 0xFFFFu;
        eq_run += tot >> 16;
      }
    });
  }
  // leave: the last workgroup out (every other one is past its last access to the scratch) re-zeroes
  // the tickets, counters, flags and histograms (the per-slice counts are rewritten before any read)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) fs.s_last = atomicAdd(fb + kFbExit, 1u) == (uint32_t)fcnt - 1;
  __syncthreads();
  if (fs.s_last)
    for (int z = t; z < kFbCnt; z += BLOCK) __hip_atomic_store(fb + z, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// finalize workgroup `fi` of `fcnt`; returns true in the workgroup that ran the boundary step
template <int MODE, int BLOCK, bool AG>
__device__ bool finalize_run(const StepArgs& a, const TopkWs& w, int fi, int fcnt, FinShared<BLOCK>& fs,
                             bool parallel) {
  constexpr int PER = kHistBins / BLOCK;
  const int t = threadIdx.x;
  const uint32_t n_sure = ld_u32<AG>(&w.ctl->n_sure), n_cand = ld_u32<AG>(&w.ctl->n_cand);
  const uint32_t thr_lo = w.ctl->thr_lo, shift = w.ctl->shift, mid = w.ctl->thr_mid;   // bracket launch
  const uint32_t k = (uint32_t)a.k;
  const bool ok = n_sure <= k && (uint64_t)n_sure + n_cand >= k && n_cand <= (uint64_t)w.cap;
  {  // the bracket's sample histograms are free again: zero them for the next step.  Write-through
     // (agent scope): the parallel fallback below accumulates into this memory with device
     // atomics in the same launch, which a dirty zero line left in some XCD's L2 would overwrite.
     // 16-B sc1 buffer stores: one fabric write per 16 B
    constexpr int kS4 = kBracketBins * kSampleCopies / 4;
    constexpr int kZ4 = kS4 + kCoarseBins * kSampleCopies / 4;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(w.shist, (short)0, kS4 * 16, 0x00020000);
    const auto rc = __builtin_amdgcn_make_buffer_rsrc(w.chist, (short)0, (kZ4 - kS4) * 16, 0x00020000);
    typedef float f4v __attribute__((ext_vector_type(4)));
    const f4v zero = {0.f, 0.f, 0.f, 0.f};
    for (int z = fi * BLOCK + t; w.shist && z < kZ4; z += fcnt * BLOCK) {
      if (z < kS4) __builtin_amdgcn_raw_buffer_store_b128(zero, rs, z * 16, 0, 16);
      else __builtin_amdgcn_raw_buffer_store_b128(zero, rc, (z - kS4) * 16, 0, 16);
    }
  }
  // every finalize workgroup: the parallel fallback (slices claimed, so no co-residency needed);
  // a caller without its scratch (segmented: per-tensor workspaces) lets the last workgroup alone
  // run the single-workgroup exact select below (same result, slower)
  if (!ok && parallel && fcnt > 1) {
    parallel_exact<MODE, BLOCK, AG>(a, w, fcnt, fs);
    return fi == 0;
  }
  int B = -1;
  uint32_t need = 0, nb = 0;
  int2 e[kFinPer];
  uint32_t fsel = 0, fbelow = 0, ps = 0;
  bool defer = false;
  if (ok) {
    const uint32_t target = k - n_sure;
    const int top = kHistBins - 1 - t * PER;
    uint32_t h[PER], sum = 0;
#pragma unroll
    for (int j = 0; j < PER; ++j) { h[j] = ld_u32<AG>(&w.hist[(top - j) * kHistStride]); sum += h[j]; }
    if (t == 0) { fs.s_B = -1; fs.s_need = 0; }
    const uint32_t ex = block_excl_scan<BLOCK>(sum, fs.s_w, nullptr);
    uint32_t acc = ex;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      if (target > 0 && acc < target && target <= acc + h[j]) { fs.s_B = top - j; fs.s_need = target - acc; }
      if (target > 0 && acc < target && target <= acc + h[j]) fs.s_res[0] = h[j];
      acc += h[j];
    }
    __syncthreads();
    B = fs.s_B;
    need = fs.s_need;
    nb = B >= 0 ? fs.s_res[0] : 0u;
    __syncthreads();
    if (fi == 0 && t == 0) {
      w.ctl->boundary_bin = B;
      w.ctl->need = need;
      w.ctl->n_bnd = nb;
    }
    STAMP_IF(fi == 0, w.ctl, 9);
    // fused mode, no candidate needed (k sure elements): every candidate is unselected, but the
    // provisionally selected ones still need their fix-ups -> route with the boundary above all bins
    if (kProv<MODE> && B < 0) B = kHistBins;
    // residual-only mode: sure entries still hold t in r; zero them now
    // (kFinPer entries per thread per round, every load issued before any store: one dependent
    // load -> store chain per entry made this 14 us of the finalize at k = 671 K)
    if constexpr (MODE == kDenseRes) {
      const uint32_t stride = (uint32_t)(fcnt * BLOCK);
      for (uint32_t j0 = fi * BLOCK + t; j0 < n_sure; j0 += stride * kFinPer) {
        float v[kFinPer];
        uint32_t ix[kFinPer];
#pragma unroll
        for (int u = 0; u < kFinPer; ++u) {
          const uint32_t j = j0 + u * stride < n_sure ? j0 + u * stride : j0;   // clamped, unconditional
          v[u] = ld_f32<AG>(a.vals + j);
          ix[u] = ld_u32<AG>(reinterpret_cast<const uint32_t*>(a.idx) + j);
        }
#pragma unroll
        for (int u = 0; u < kFinPer; ++u)
          if (j0 + u * stride < n_sure) a.r[(int64_t)(int32_t)ix[u] - a.idx_base] = v[u] - v[u];
      }
    }
    if (B >= 0) {
      // contiguous slice per workgroup, kFinPer candidates per thread per round held in registers;
      // one block scan places them, one global atomic per list per round reserves the space.  The
      // boundary-list stores go first; a single-round slice (the common case) defers its payload
      // and dense writes past the arrival ticket, so the boundary ranking does not wait for them.
      const uint32_t per = (n_cand + fcnt - 1) / fcnt;
      const uint32_t b0 = fi * per, b1 = min(n_cand, b0 + per);
      defer = b1 > b0 && b1 - b0 <= (uint32_t)(BLOCK * kFinPer);
      for (uint32_t r0 = b0; r0 < b1; r0 += BLOCK * kFinPer) {
        uint32_t fb = 0;
        fsel = 0;
        fbelow = 0;
#pragma unroll
        for (int u = 0; u < kFinPer; ++u) {
          const uint32_t j = r0 + u * BLOCK + t;
          e[u] = ld_i2<AG>(w.cand + (j < b1 ? j : b0));   // clamped, unconditional
          const int bin = j < b1 ? (int)cand_bin(abs_key(u2f((uint32_t)e[u].y)), thr_lo, shift) : -1;
          fsel |= (uint32_t)(bin > B) << u;
          fb |= (uint32_t)(bin == B) << u;
          fbelow |= (uint32_t)(j < b1 && bin < B) << u;
        }
        const uint32_t packed = (uint32_t)__popc(fsel) | ((uint32_t)__popc(fb) << 16);
        uint32_t tot;
        const uint32_t ex = block_excl_scan<BLOCK>(packed, fs.s_w, &tot);
        if (t == 0) {
          // one reservation per workgroup and list (128 on each counter: as 8 copies, a timing-only
          // build, the finalize was 1 us faster in 11.7 -- not worth a two-level position scheme)
          fs.s_res[0] = (tot & 0xFFFFu) ? atomicAdd(&w.ctl->n_sel, tot & 0xFFFFu) : 0u;
          fs.s_res[1] = (tot >> 16) ? atomicAdd(&w.ctl->n_bacc, tot >> 16) : 0u;
        }
        __syncthreads();
        ps = n_sure + fs.s_res[0] + (ex & 0xFFFFu);
        uint32_t pb = fs.s_res[1] + (ex >> 16);
        __syncthreads();
#pragma unroll
        for (int u = 0; u < kFinPer; ++u)
          if ((fb >> u) & 1u) st_agent_i2(w.bnd + pb++, e[u]);
        if (!defer) write_round<MODE>(a, e, fsel, fbelow, ps, mid, w.ctl);
      }
    }
  }
  // arrival: every wave's (write-through) boundary stores complete, then one ticket per
  // workgroup; the last one finishes the boundary bin
  STAMP_IF(fi == 0, w.ctl, 10);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) fs.s_last = atomicAdd(&w.ctl->ticket, 1u) == (uint32_t)fcnt - 1;
  __syncthreads();
  const bool last = fs.s_last;
  const bool preloaded = last && boundary_preload<BLOCK>(w, ok, need, nb, fs);
  if (defer) write_round<MODE>(a, e, fsel, fbelow, ps, mid, w.ctl);
  if (!last) return false;
  STAMP_IF(true, w.ctl, 11);
  boundary_work<MODE, BLOCK, AG>(a, w, ok, need, nb, fs, preloaded, mid);
  __syncthreads();
  STAMP_IF(true, w.ctl, 12);
  return true;
}

template <int MODE>
__global__ __launch_bounds__(kSelBlock) void topk_finalize(StepArgs a, TopkWs w) {
  __shared__ FinShared<kSelBlock> fs;
  STAMP(w.ctl, 8);
  finalize_run<MODE, kSelBlock, false>(a, w, blockIdx.x, gridDim.x, fs, true);
}

// ------------------------------------------------------------------------------------------------
// small buckets: everything in one workgroup, t staged in LDS
template <bool HAS_RES, int MODE>
__device__ void small_body(const StepArgs& a, float* s_t, uint32_t* hist, uint32_t* s_w, uint32_t* s_res) {
  const int64_t n = a.n;
  for (int64_t i = threadIdx.x; i < n; i += kSelBlock) s_t[i] = compensate<HAS_RES>(a, i);
  __syncthreads();
  const float* st = s_t;
  auto src = [st](int64_t i) { return comp_key(abs_key(st[i]), (uint32_t)i); };
  const uint32_t k = (uint32_t)a.k;
  uint64_t T = 0;
  if ((int64_t)k < n) T = block_select_comp(src, n, k, hist, s_w, s_res);
  auto f = [st](int64_t i) { return st[i]; };
  block_write_selected<MODE>(a, f, n, T, 0u, s_w);
}

template <bool HAS_RES, int MODE>
__global__ __launch_bounds__(kSelBlock) void topk_small(StepArgs a) {
  __shared__ float s_t[kSmallN];
  __shared__ uint32_t hist[2048];
  __shared__ uint32_t s_w[kSelBlock / kWave + 1];
  __shared__ uint32_t s_res[2];
  small_body<HAS_RES, MODE>(a, s_t, hist, s_w, s_res);
}

// ------------------------------------------------------------------------------------------------
// k >= n on a large bucket: every element is selected, payload in index order
template <bool HAS_RES, int MODE>
__global__ __launch_bounds__(256) void topk_all(StepArgs a) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n;
       i += (int64_t)gridDim.x * blockDim.x)
    emit<MODE>(a, (uint32_t)i, i, compensate<HAS_RES>(a, i));
}

#ifndef GRACE_MAIN_VEC_NORES_BIG
#define GRACE_MAIN_VEC_NORES_BIG 64
#endif
constexpr int kNoresBigVec = GRACE_MAIN_VEC_NORES_BIG;
constexpr int64_t kNoresBigMinN = (int64_t)1024 * kMainBlock * 4 * kNoresBigVec;   // 2^26 at 64

// the main pass at NV float4 per lane per chunk (one chunk per workgroup)
template <bool HAS_RES, int MODE, int NV>
static void launch_main(const StepArgs& a, const TopkWs& w, bool sparse, bool vec, hipStream_t s) {
  constexpr int64_t kCh = (int64_t)kMainBlock * 4 * NV;
  const unsigned nblk = (unsigned)((a.n + kCh - 1) / kCh);
  if (sparse) {
    if constexpr (kWritesOut<MODE>) {
      if (vec)
        launch_timed(topk_main<HAS_RES, MODE, true, false, true, NV>, dim3(nblk), dim3(kMainBlock), s, a, w);
      else
        launch_timed(topk_main<HAS_RES, MODE, false, false, true, NV>, dim3(nblk), dim3(kMainBlock), s, a, w);
    }
  } else if (vec) {
    launch_timed(topk_main<HAS_RES, MODE, true, false, false, NV>, dim3(nblk), dim3(kMainBlock), s, a, w);
  } else {
    launch_timed(topk_main<HAS_RES, MODE, false, false, false, NV>, dim3(nblk), dim3(kMainBlock), s, a, w);
  }
}

template <bool HAS_RES, int MODE>
static grace_status_t run_topk(StepArgs a, void* ws, size_t bytes, hipStream_t s) {
  if (!a.r_in) a.r_in = a.r;
  if (a.n <= kSmallN) {
    topk_small<HAS_RES, MODE><<<1, kSelBlock, 0, s>>>(a);
    GRACE_CHECK_LAUNCH("topk_small");
    return GRACE_OK;
  }
  if (a.k >= a.n) {
    topk_all<HAS_RES, MODE><<<stream_grid(a.n, 256), 256, 0, s>>>(a);
    GRACE_CHECK_LAUNCH("topk_all");
    return GRACE_OK;
  }
  if (bytes < ws_bytes(a.n, a.k)) {
    set_error_msg("grace_topk: workspace too small");
    return GRACE_ERR_WORKSPACE;
  }
  TopkWs w = carve(ws, a.n, a.k);
  const bool vec = ((reinterpret_cast<uintptr_t>(a.g) | reinterpret_cast<uintptr_t>(a.r) |
                     reinterpret_cast<uintptr_t>(a.out)) & 15u) == 0;
  a.sample_n = bracket_sample_n(a.n);
  a.stratum = a.n / a.sample_n;
  if (a.stratum < kCarryMinStratum) a.rs_in = a.rs_out = nullptr;   // (grace_topk_carry_size says 0)
  // >= 33 sample workgroups (n > kSmallN): the first two zero the candidate histogram
  static_assert(kSmallN >= kHistBins, "bracket grid covers the histogram zeroing");
  // runs of kBracketRun samples only when the sample tiles the bucket into whole runs
  static_assert((kSampleMax / 2) % (kBracketRun * kBracketBlock) == 0, "sample runs tile the grid");
  if (kBracketRun > 1 && a.sample_n < kSampleMax / 2) {
    set_error_msg("grace_topk: sample runs need n >= the sample size (A/B build)");
    return GRACE_ERR_ARG;
  }
  const bool sparse = kWritesOut<MODE> && a.out && a.prev_idx && a.prev_count > 0;
  if (!sparse) a.prev_idx = nullptr;
  const unsigned nclr = sparse ? (unsigned)min((int64_t)kClearMax, (a.prev_count + kClearPer - 1) / kClearPer) : 0u;
  topk_bracket<HAS_RES><<<(unsigned)((a.sample_n / kBracketRun + kBracketBlock - 1) / kBracketBlock) + nclr,
                          kBracketBlock, 0, s>>>(a, w);
  GRACE_CHECK_LAUNCH("topk_bracket");
  bool big = false;
  if constexpr (!HAS_RES && kMainV3 && kVecOf<HAS_RES, MODE> == GRACE_MAIN_VEC_NORES) {
    // 4 / 8 B per element (no residual stream): large buckets take chunks of kNoresBigVec float4 per
    // lane, so that the grid is ONE balanced generation (2^26 elements: 1024 workgroups, 4 per CU;
    // 32 float4 gave 2048 for 1536 resident slots).  r06 A/B (tools/ab_v3.py, 256 MiB, 1 %): main
    // pass with the recycled output, 32 / 40 / 48 / 64 / 80 / 96 / 128 float4 -> 72.2 / 67.4 / 67.3 /
    // 59.2-60.6 / 69.2 / 72.7 / 58.5 us (820 and 683 workgroups leave CUs unevenly loaded).  Only for
    // k <= n / 50: a wave's LDS region holds 512 flagged elements, ~1.45 % of 16384 at k = 1 %.
    // (only the 4 / 8 B classes: the first residual step's 12 B pass keeps its 20-float4 chunks)
    big = a.n >= kNoresBigMinN && a.k <= a.n / 50;
    if (big) launch_main<HAS_RES, MODE, kNoresBigVec>(a, w, sparse, vec, s);
  }
  if (!big) launch_main<HAS_RES, MODE, kVecOf<HAS_RES, MODE>>(a, w, sparse, vec, s);
  GRACE_CHECK_LAUNCH("topk_main");
  // finalize workgroups by the candidate capacity -- one routing round (kSelBlock * kFinPer
  // candidates) each for the band the bracket can produce -- and by the bucket (at most 2^19
  // elements each for the exact fallback's slices), so a small bucket's last arrival waits for
  // 16-25 workgroups instead of 128 (the 2^26 headline keeps 128).  r05 A/B at configs[4]'s 8.4 M
  // shard: local step 57.7 / 57.8 -> 56.7 / 57.0 us.
  int fblocks = kFinBlocks;
  {
    const int64_t c = std::max(w.cap / ((int64_t)kSelBlock * kFinPer) + 1, a.n >> 19);
    fblocks = (int)(c < 16 ? 16 : (c > kFinBlocks ? kFinBlocks : c));
  }
  topk_finalize<MODE><<<fblocks, kSelBlock, 0, s>>>(a, w);
  GRACE_CHECK_LAUNCH("topk_finalize");
  return GRACE_OK;
}

// ------------------------------------------------------------------------------------------------
// ------------------------------------------------------------------------------------------------
// sparse decode / aggregate
__global__ void scatter_kernel(const float* vals, const int32_t* idx, int64_t count, float* out) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < count;
       j += (int64_t)gridDim.x * blockDim.x)
    out[idx[j]] = vals[j];
}
__global__ void scatter_kernel_i64(const float* vals, const int64_t* idx, int64_t count, float* out) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < count;
       j += (int64_t)gridDim.x * blockDim.x)
    out[idx[j]] = vals[j];
}
__global__ void scatter_add_tag_kernel(const float* vals, const int32_t* idx, int64_t count, int32_t w,
                                       float* out, int32_t* tags) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < count;
       j += (int64_t)gridDim.x * blockDim.x) {
    const int32_t i = idx[j];
    out[i] = out[i] + vals[j];
    tags[i] = w;
  }
}
// every aggregated element is divided exactly once: by the entry of the last rank that touched it
// (tags[i] holds that rank after the ordered scatters).  One launch over all W payloads; the
// per-rank prefix counts travel in the kernel arguments.
constexpr int kMaxAggWorld = 64;
struct AggCum { int64_t v[kMaxAggWorld + 1]; };

__global__ void tag_divide_kernel(const int32_t* idx, int64_t stride, AggCum cum, int32_t world, float divisor,
                                  float* out, const int32_t* tags) {
  const int64_t total = cum.v[world];
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < total;
       j += (int64_t)gridDim.x * blockDim.x) {
    int w = 0;
    while (w + 1 < world && cum.v[w + 1] <= j) ++w;
    const int32_t i = idx[w * stride + (j - cum.v[w])];
    if (tags[i] == w) out[i] = out[i] / divisor;
  }
}

// ------------------------------------------------------------------------------------------------
// Segmented top-k: the reference's DDP loop calls Communicator.step once per
// parameter tensor (examples/dist/CIFAR10-dawndist/core.py:203-206), each a TopKCompressor(ratio)
// with its own k_i = max(1, int(n_i * ratio)) (grace_dl/dist/compressor/topk.py:34) and its own
// residual (grace_dl/dist/memory/residual.py:10-20).  All tensors sit back to back in one flat
// buffer (the segments) and the single-bucket engine above runs on every segment at once, in
// THREE launches, streaming every element once (16 B per element at world 1):
//   prep     one workgroup per segment: a small segment (n <= kSegSmallMax) is selected exactly in LDS
//            and written out completely (small_body); a large one gets its sampled bracket
//            (n/256 samples, 512..2048, into a 32768-bin LDS histogram; the engine's ranks and
//            thresholds) and its counters / candidate histogram zeroed;
//   main     one chunk of one large segment per workgroup: the engine's main pass (main_chunk_v2)
//            with that segment's bracket, lists and histogram;
//   finalize one workgroup per large segment: the engine's finalize (finalize_run) as its own
//            last arriver -- boundary bin, exact ranking by (|t| desc, index asc), or the
//            segment's exact fallback when its bracket missed.
// Payload indices are global (flat-buffer) indices (StepArgs::idx_base = the segment's offset).
// sample sizes: every sample is two random DRAM reads (g, r), and the bracket launch is bound by
// their row activations: 8192 per large segment (45 ResNet-50 tensors, 737 K reads) took 47 us
#ifndef GRACE_SEG_SAMPLE_MAX
#define GRACE_SEG_SAMPLE_MAX 2048
#endif
constexpr int kSegSampleMin = 512, kSegSampleMax = GRACE_SEG_SAMPLE_MAX;
// segments up to this size are selected whole in one prep workgroup (the prep kernel supports up to
// kSmallN); larger ones take the bracket / main / finalize path.  A 16 K or 32 K segment in one
// workgroup (four serial rounds of loads, an LDS select over 32 K keys) ended the prep launch
// ~6 us after the last large segment's bracket, delaying the main pass by that much.
constexpr int kSegSmallMax = 8192;
static_assert(kSegSmallMax <= kSmallN, "small segments fit the prep workgroup");

struct SegPlan {
  const float* g;
  float* r;
  float* out;          // dense world-1 output (kDenseFused) or null (kDenseRes)
  float* vals;
  int32_t* idx;
  float beta, gamma;
  const int64_t* seg_off;   // [nseg + 1] element offsets
  const int64_t* k_off;     // [nseg + 1] payload offsets (k_i prefix sums)
  const int32_t* large;     // [nL] segments with n > kSegSmallMax (any order: the host sorts by size)
  const int32_t* small;     // [nS] the others
  const int64_t* chk_off;   // [nL + 1] main-pass chunk offsets of the large segments
  const int32_t* chunk_li;  // [nchunks] large-segment slot of every main-pass chunk
  const int64_t* ws_off;    // [nL] byte offsets of the large segments' workspaces
  const int64_t* fin_off;   // [nL + 1] finalize workgroups of each large segment (prefix sums)
  const int32_t* fin_li;    // [nfin] large-segment slot of every finalize workgroup
  char* ws;
  int32_t nL, nS;
  // residual-sample carry per large segment (grace_topk_residual_step_carry's, per segment): the
  // prep writes the segment's t at its sample positions to carry + carry_off[li], the finalize the
  // segment's selection threshold after them; with carry_valid the next prep derives r' there from
  // them and reads only g (one random read per sample instead of two).  carry may be null.
  float* carry;
  const int64_t* carry_off;
  int32_t carry_valid;
};

__device__ __forceinline__ StepArgs seg_step_args(const SegPlan& p, int s) {
  const int64_t o = p.seg_off[s], ko = p.k_off[s];
  StepArgs a{};
  a.g = p.g + o;
  a.r = p.r + o;
  a.r_in = a.r;
  a.beta = p.beta;
  a.gamma = p.gamma;
  a.n = p.seg_off[s + 1] - o;
  a.k = p.k_off[s + 1] - ko;
  a.vals = p.vals + ko;
  a.idx = p.idx + ko;
  a.out = p.out ? p.out + o : nullptr;
  a.idx_base = o;
  return a;
}

__host__ __device__ __forceinline__ int64_t seg_cap(int64_t n, int64_t k) {
  const int64_t c = 2 * k + 65536;
  return c < n ? c : n;
}
__host__ __device__ __forceinline__ int64_t seg_al(int64_t x) { return (x + 255) & ~(int64_t)255; }
// one large segment's workspace: ctl | candidate histogram | candidate list | boundary list
__host__ __device__ __forceinline__ int64_t seg_ws_bytes_one(int64_t n, int64_t k) {
  return 256 + seg_al(4 * kHistBins) + 2 * seg_al(8 * seg_cap(n, k));
}
__device__ __forceinline__ TopkWs seg_ws(const SegPlan& p, int li, int64_t n, int64_t k) {
  char* q = p.ws + p.ws_off[li];
  TopkWs w{};
  w.cap = seg_cap(n, k);
  w.ctl = reinterpret_cast<TopkCtl*>(q);
  w.hist = reinterpret_cast<uint32_t*>(q + 256);
  w.cand = reinterpret_cast<int2*>(q + 256 + seg_al(4 * kHistBins));
  w.bnd = reinterpret_cast<int2*>(q + 256 + seg_al(4 * kHistBins) + seg_al(8 * w.cap));
  w.shist = nullptr;   // the segment bracket keeps its sample histogram in LDS
  w.chist = nullptr;
  return w;
}
__host__ __device__ __forceinline__ int64_t seg_sample_n(int64_t n) {
  int64_t S = n / 256;
  S = S < kSegSampleMin ? kSegSampleMin : (S > kSegSampleMax ? kSegSampleMax : S);
  return S < n / 4 ? S : n / 4;
}
// the step arguments of large segment slot li, with its carry (prep and finalize)
__device__ __forceinline__ StepArgs seg_large_args(const SegPlan& p, int li) {
  StepArgs a = seg_step_args(p, p.large[li]);
  if (p.carry) {
    a.sample_n = seg_sample_n(a.n);
    a.rs_out = p.carry + p.carry_off[li];
    a.rs_in = p.carry_valid ? a.rs_out : nullptr;
  }
  return a;
}


// A small segment (n <= kSegSmallMax) in one workgroup, built for throughput next to many others in the
// same launch: t staged in LDS with 8 loads per array in flight per thread, the exact threshold by
// block_select_comp over LDS, then every element written from LDS with independent coalesced
// stores and the payload placed by one LDS atomic per wave (order within the segment is free: the
// exchange and the decode are order-independent).  small_body's ordered one-round-per-1024
// writes and serial loads made 116 ResNet-50 tensors a 46 us launch.
template <bool HAS_RES, int MODE>
__device__ void seg_small_body(const StepArgs& a, float* s_t, uint32_t* hist, uint32_t* s_w, uint32_t* s_res) {
  constexpr int kU = 8;
  const int tid = threadIdx.x;
  const int64_t n = a.n;
  for (int64_t j0 = tid; j0 < n; j0 += (int64_t)kU * kSelBlock) {
    float t[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t i = j0 + (int64_t)u * kSelBlock;
      t[u] = compensate<HAS_RES>(a, i < n ? i : j0);   // clamped, unconditional
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t i = j0 + (int64_t)u * kSelBlock;
      if (i < n) s_t[i] = t[u];
    }
  }
  __syncthreads();
  const float* st = s_t;
  auto src = [st](int64_t i) { return comp_key(abs_key(st[i]), (uint32_t)i); };
  const uint32_t k = (uint32_t)a.k;
  uint64_t T = 0;
  if ((int64_t)k < n) T = block_select_comp(src, n, k, hist, s_w, s_res);
  if (tid == 0) s_res[0] = 0u;
  __syncthreads();
  for (int64_t i = tid; i < n; i += kSelBlock) {
    const float v = st[i];
    const bool sel = comp_key(abs_key(v), (uint32_t)i) >= T;
    if constexpr (kWritesR<MODE>) a.r[i] = sel ? v - v : v;
    if constexpr (kWritesOut<MODE>) a.out[i] = sel ? 0.f + v : 0.f;
    const uint64_t m = __ballot(sel);
    uint32_t base = 0;
    if (m && lane_rank(m) == 0 && sel) base = atomicAdd(&s_res[0], (uint32_t)__popcll(m));
    base = __shfl(base, m ? __builtin_ctzll(m) : 0, 64);
    if (sel) {
      const uint32_t pos = base + lane_rank(m);
      a.vals[pos] = v;
      a.idx[pos] = (int32_t)(i + a.idx_base);
    }
  }
}

template <bool HAS_RES, int MODE>
__global__ __launch_bounds__(kSelBlock) void seg_prep_kernel(SegPlan p) {
  // bracket: the fine sample histogram [kBracketBins]; small segment: t [kSmallN] + select histogram
  __shared__ uint32_t lds[kSmallN + 2048];
  __shared__ uint32_t s_w[kSelBlock / kWave + 1];
  __shared__ uint32_t s_res[8];
  static_assert(kBracketBins + kBracketBins / 32 <= kSmallN + 2048, "padded bracket histogram fits the shared block");
  const int b = blockIdx.x, tid = threadIdx.x;
  if (b >= p.nL) {   // a small segment, selected and written completely by this workgroup
#ifdef GRACE_SEG_NOSMALL   // diagnostic timing build only (small segments left unwritten)
    return;
#endif
    const StepArgs a = seg_step_args(p, p.small[b - p.nL]);
    seg_small_body<HAS_RES, MODE>(a, reinterpret_cast<float*>(lds), lds + kSmallN, s_w, s_res);
    return;
  }
  const StepArgs a = seg_large_args(p, b);
  const TopkWs w = seg_ws(p, b, a.n, a.k);
  STAMP_IF(true, w.ctl, 13);
#ifdef GRACE_STAMPS
  if (tid == 0) {   // main-pass span of this segment: first chunk start (min), last chunk end (max)
    reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(w.ctl) + 64)[16] = ~0ull;
    reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(w.ctl) + 64)[17] = 0ull;
    reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(w.ctl) + 64)[18] = 0ull;
    reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(w.ctl) + 64)[19] = 0ull;
  }
#endif
  const int64_t S = seg_sample_n(a.n);
  const uint32_t st = (uint32_t)(a.n / S);
  constexpr int kPer = kSegSampleMax / kSelBlock;
  float t[kPer];
#pragma unroll
  for (int q = 0; q < kPer; ++q) {   // every sample load issued before any is used (clamped index)
    const int64_t sidx = (int64_t)q * kSelBlock + tid;
    const int64_t sc = sidx < S ? sidx : S - 1;
    const int64_t pos = sample_pos(sc, st);
    if (HAS_RES && a.rs_in) {
      // the segment's carried t'(pos) and threshold: r'(pos) as the last step left it, and one
      // random read (g) per sample instead of two (the headline bracket's carry, per segment)
      const float tp = a.rs_in[sc];
      const uint64_t Tp = *reinterpret_cast<const uint64_t*>(a.rs_in + carry_thr_off(S));
      const float rp = comp_key(abs_key(tp), (uint32_t)pos) >= Tp ? tp - tp : tp;
      t[q] = a.beta * rp + a.gamma * a.g[pos];
    } else {
      t[q] = compensate<HAS_RES>(a, pos);
    }
  }
  if (a.rs_out) {
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int64_t sidx = (int64_t)q * kSelBlock + tid;
      if (sidx < S) a.rs_out[sidx] = t[q];
    }
  }
  // this step's counters and candidate histogram (the segment's previous finalize has completed)
  if (tid >= 3 && tid < 12) reinterpret_cast<uint32_t*>(w.ctl)[tid] = 0u;
  for (int j = tid; j < kHistBins; j += kSelBlock) w.hist[j] = 0u;
  for (int j = tid; j < kBracketBins + kBracketBins / 32; j += kSelBlock) lds[j] = 0u;   // padded layout
  __syncthreads();
  STAMP_IF(true, w.ctl, 14);
#pragma unroll
  for (int q = 0; q < kPer; ++q)
    if ((int64_t)q * kSelBlock + tid < S) atomicAdd(&lds[hist_pad(abs_key(t[q]) >> 16)], 1u);
  __syncthreads();
  const BracketRanks br = bracket_ranks(S, a.k, a.n);
  int d[3];
  uint32_t above[3];
  find_bins_desc<kSelBlock, kBracketBins, 3, true>(lds, br.r1, s_w, s_res, d, above);
  if (tid == 0) bracket_publish(w.ctl, bracket_thresholds(br, S, (uint32_t)d[0], (uint32_t)d[1], (uint32_t)d[2]));
  STAMP_IF(true, w.ctl, 15);
}

template <bool HAS_RES, int MODE, bool VEC>
__global__ __launch_bounds__(kMainBlock, 4) void seg_main_kernel(SegPlan p) {
  __shared__ MainShared sm;
  const int tid = threadIdx.x;
  const int li = p.chunk_li[blockIdx.x];
  const int s = p.large[li];
  const StepArgs a = seg_step_args(p, s);
  const TopkWs w = seg_ws(p, li, a.n, a.k);
  const int64_t chunk = (int64_t)blockIdx.x - p.chk_off[li];
#ifdef GRACE_STAMPS
  if (tid == 0)
    atomicMin(reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(w.ctl) + 64) + 16,
              (unsigned long long)__builtin_amdgcn_s_memrealtime());
#endif
  for (int b = tid; b < kHistBins; b += kMainBlock) sm.hist[b] = 0;
  const uint32_t lo = w.ctl->thr_lo, hi = w.ctl->thr_hi, sh = w.ctl->shift, mid = w.ctl->thr_mid;
  __syncthreads();
  uint32_t wfill;
  // (no beta = gamma = 1 instantiation here: next to the segment bookkeeping it pushed this kernel
  // to 128 VGPRs and 96 B of scratch per lane)
  if (VEC && (p.seg_off[s] & 3) == 0 && (chunk + 1) * kChunkOf<HAS_RES, MODE> <= a.n) {
    wfill = main_chunk_v2<HAS_RES, MODE, VEC>(a, w, sm, lo, hi, sh, mid, chunk);
  } else {
    wfill = main_chunk_v2<HAS_RES, MODE, false>(a, w, sm, lo, hi, sh, mid, chunk);
  }
  flush_staged(a, w, sm, lo, hi, sh, mid, wfill);
  __syncthreads();
  for (int b = tid; b < kHistBins; b += kMainBlock) {
    const uint32_t h = sm.hist[b];
    if (h) atomicAdd(&w.hist[b * kHistStride], h);
  }
#ifdef GRACE_STAMPS
  if (tid == 0)
    atomicMax(reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(w.ctl) + 64) + 17,
              (unsigned long long)__builtin_amdgcn_s_memrealtime());
#endif
}

// the engine's finalize per large segment, with the segment's fin_off[li + 1] - fin_off[li]
// workgroups (sized on the host for ~2 k_i candidates, one round of kSelBlock * kFinPer each) and
// its own last arriver; no parallel exact fallback (its grid barrier would span segments): a missed
// bracket falls back to the last workgroup's exact select over the segment
template <int MODE>
__global__ __launch_bounds__(kSelBlock) void seg_fin_kernel(SegPlan p) {
  __shared__ FinShared<kSelBlock> fs;
  const int li = p.fin_li[blockIdx.x];
  const int fi = (int)((int64_t)blockIdx.x - p.fin_off[li]);
  const int fcnt = (int)(p.fin_off[li + 1] - p.fin_off[li]);
  const StepArgs a = seg_large_args(p, li);
  const TopkWs w = seg_ws(p, li, a.n, a.k);
  STAMP_IF(fi == 0, w.ctl, 8);
  finalize_run<MODE, kSelBlock, false>(a, w, fi, fcnt, fs, false);
}

template <bool HAS_RES, int MODE>
static grace_status_t run_segmented(const SegPlan& p, int64_t nchunks, int64_t nfin, bool vec, hipStream_t s) {
  seg_prep_kernel<HAS_RES, MODE><<<(unsigned)(p.nL + p.nS), kSelBlock, 0, s>>>(p);
  GRACE_CHECK_LAUNCH("grace_topk_segmented_step");
  if (p.nL == 0) return GRACE_OK;
  if (vec)
    launch_timed(seg_main_kernel<HAS_RES, MODE, true>, dim3((unsigned)nchunks), dim3(kMainBlock), s, p);
  else
    launch_timed(seg_main_kernel<HAS_RES, MODE, false>, dim3((unsigned)nchunks), dim3(kMainBlock), s, p);
  GRACE_CHECK_LAUNCH("grace_topk_segmented_step");
  seg_fin_kernel<MODE><<<(unsigned)nfin, kSelBlock, 0, s>>>(p);
  GRACE_CHECK_LAUNCH("grace_topk_segmented_step");
  return GRACE_OK;
}

}  // namespace grace

using namespace grace;

extern "C" {

grace_status_t grace_read_status(const void* workspace, int32_t* status_host, void* stream) {
  GRACE_REQUIRE(workspace && status_host, "grace_read_status: bad arguments");
  const TopkCtl* c = reinterpret_cast<const TopkCtl*>(workspace);
  hipError_t e = hipMemcpyAsync(status_host, &c->status, sizeof(int32_t), hipMemcpyDeviceToHost,
                                as_stream(stream));
  if (e == hipSuccess) e = hipStreamSynchronize(as_stream(stream));
  if (e != hipSuccess) {
    set_error("grace_read_status", e);
    return GRACE_ERR_HIP;
  }
  return GRACE_OK;
}

size_t grace_topk_stream_probe_workspace_bytes(int64_t n) { return ws_bytes(n, 1); }

// Placement spacers (ops.pick_pair): device memory taken straight from the HIP runtime between the
// residual and output candidate allocations and given straight back, so the caller's allocator
// cache keeps none of it
grace_status_t grace_spacer_alloc(size_t bytes, void** ptr) {
  GRACE_REQUIRE(ptr, "grace_spacer_alloc: null ptr");
  *ptr = nullptr;
  if (bytes == 0) return GRACE_OK;
  if (hipMalloc(ptr, bytes) != hipSuccess) {
    *ptr = nullptr;
    (void)hipGetLastError();
    set_error_msg("grace_spacer_alloc: hipMalloc failed");
    return GRACE_ERR_HIP;
  }
  return GRACE_OK;
}

grace_status_t grace_spacer_free(void* ptr) {
  if (ptr && hipFree(ptr) != hipSuccess) {
    (void)hipGetLastError();
    set_error_msg("grace_spacer_free: hipFree failed");
    return GRACE_ERR_HIP;
  }
  return GRACE_OK;
}

grace_status_t grace_topk_stream_probe(const float* g, float* r, float* out, int64_t n, int32_t sparse, void* ws,
                                       size_t ws_bytes_, void* stream) {
  GRACE_REQUIRE(g && r && out && ws && n >= 1 && n < ((int64_t)1 << 31) &&
                    ((reinterpret_cast<uintptr_t>(g) | reinterpret_cast<uintptr_t>(r) |
                      reinterpret_cast<uintptr_t>(out)) & 15u) == 0,
                "grace_topk_stream_probe: bad arguments (16-B aligned device buffers, 1 <= n < 2^31)");
  GRACE_REQUIRE(ws_bytes_ >= ws_bytes(n, 1), "grace_topk_stream_probe: workspace too small");
  TopkWs w = carve(ws, n, 1);
  StepArgs a{g, r, 1.f, 1.f, n, 1, nullptr, nullptr, out};
  a.r_in = r;
  const unsigned nblk = (unsigned)((n + kChunkOf<true, kDenseFused> - 1) / kChunkOf<true, kDenseFused>);
  // timed like the real pass (the event timer rides on the dispatch packet when it is enabled)
  if (sparse)   // the recycled-output layout: g, r read, r' written, out untouched
    launch_timed(topk_main<true, kDenseFused, true, true, true>, dim3(nblk), dim3(kMainBlock), as_stream(stream), a, w);
  else
    launch_timed(topk_main<true, kDenseFused, true, true>, dim3(nblk), dim3(kMainBlock), as_stream(stream), a, w);
  GRACE_CHECK_LAUNCH("grace_topk_stream_probe");
  return GRACE_OK;
}

int32_t grace_status_take(int32_t* host_word) {
  // a host-side atomic exchange: a device fetch_or (system scope, over PCIe) that lands between
  // a plain read and a plain clear would otherwise be lost
  return host_word ? __atomic_exchange_n(host_word, 0, __ATOMIC_SEQ_CST) : 0;
}

grace_status_t grace_topk_status_word(int32_t* host_word) {
  g_topk_hstatus = host_word;
  return GRACE_OK;
}

int64_t grace_topk_fallback_spin_limit(int64_t limit) {
  const int64_t prev = g_fb_spin_max;
  if (limit >= 0) g_fb_spin_max = limit > 0xFFFFFFFFll ? 0xFFFFFFFFu : (uint32_t)limit;
  return prev;
}

grace_status_t grace_timer_enable(int enable) {
  if (enable && !g_ev_created) {
    for (int i = 0; i < 2 * kMaxEv; ++i) {
      hipError_t e = hipEventCreateWithFlags(&g_ev[i], hipEventDisableSystemFence);
      if (e != hipSuccess) {
        set_error("grace_timer_enable", e);
        return GRACE_ERR_HIP;
      }
    }
    g_ev_created = 1;
  }
  g_timer_on = enable ? 1 : 0;
  g_ev_used = 0;
  return GRACE_OK;
}

grace_status_t grace_event_create(void** event) {
  GRACE_REQUIRE(event, "grace_event_create: bad arguments");
  hipEvent_t ev = nullptr;
  const hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableSystemFence | hipEventDisableTiming);
  if (e != hipSuccess) {
    set_error("grace_event_create", e);
    return GRACE_ERR_HIP;
  }
  *event = ev;
  return GRACE_OK;
}

grace_status_t grace_event_destroy(void* event) {
  GRACE_REQUIRE(event, "grace_event_destroy: bad arguments");
  const hipError_t e = hipEventDestroy(static_cast<hipEvent_t>(event));
  if (e != hipSuccess) {
    set_error("grace_event_destroy", e);
    return GRACE_ERR_HIP;
  }
  return GRACE_OK;
}

grace_status_t grace_topk_arm_main_event(void* event) {
  t_main_ev = static_cast<hipEvent_t>(event);
  return GRACE_OK;
}

grace_status_t grace_stream_wait_event(void* stream, void* event) {
  GRACE_REQUIRE(event, "grace_stream_wait_event: bad arguments");
  const hipError_t e = hipStreamWaitEvent(static_cast<hipStream_t>(stream), static_cast<hipEvent_t>(event), 0);
  if (e != hipSuccess) {
    set_error("grace_stream_wait_event", e);
    return GRACE_ERR_HIP;
  }
  return GRACE_OK;
}

grace_status_t grace_timer_collect(float* total_ms, int32_t* launches) {
  GRACE_REQUIRE(total_ms && launches, "grace_timer_collect: bad arguments");
  float tot = 0.f;
  for (int i = 0; i < g_ev_used; ++i) {
    hipError_t e = hipEventSynchronize(g_ev[2 * i + 1]);
    float ms = 0.f;
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, g_ev[2 * i], g_ev[2 * i + 1]);
    if (e != hipSuccess) {
      set_error("grace_timer_collect", e);
      return GRACE_ERR_HIP;
    }
    tot += ms;
  }
  *total_ms = tot;
  *launches = g_ev_used;
  g_ev_used = 0;
  return GRACE_OK;
}

size_t grace_topk_workspace_bytes(int64_t n, int64_t k) { return ws_bytes(n, k); }

grace_status_t grace_topk_compress(const float* x, int64_t n, int64_t k, float* vals, int32_t* idx,
                                   void* ws, size_t ws_bytes_, void* stream) {
  GRACE_REQUIRE(x && vals && idx && n > 0 && k >= 1 && k <= n && n < (int64_t)1 << 31,
                "grace_topk_compress: bad arguments");
  GRACE_REQUIRE(n <= kSmallN || ws, "grace_topk_compress: workspace required");
  StepArgs a{x, nullptr, 1.f, 1.f, n, k, vals, idx, nullptr};
  return run_topk<false, kDenseNone>(a, ws, ws_bytes_, as_stream(stream));
}

grace_status_t grace_topk_step_dense(const float* x, int64_t n, int64_t k, float* vals, int32_t* idx, float* out,
                                     const int32_t* prev_idx, int64_t prev_count, void* ws, size_t ws_bytes_,
                                     void* stream) {
  GRACE_REQUIRE(x && vals && idx && out && n > 0 && k >= 1 && k <= n && n < (int64_t)1 << 31,
                "grace_topk_step_dense: bad arguments");
  GRACE_REQUIRE(n <= kSmallN || ws, "grace_topk_step_dense: workspace required");
  StepArgs a{x, nullptr, 1.f, 1.f, n, k, vals, idx, out};
  a.prev_idx = prev_idx;
  a.prev_count = prev_idx ? prev_count : 0;
  return run_topk<false, kDenseOut>(a, ws, ws_bytes_, as_stream(stream));
}

grace_status_t grace_topk_residual_step(const float* g, float* residual, int32_t has_residual,
                                        float beta, float gamma, int64_t n, int64_t k, float* vals,
                                        int32_t* idx, float* out, void* ws, size_t ws_bytes_,
                                        void* stream) {
  GRACE_REQUIRE(g && residual && vals && idx && n > 0 && k >= 1 && k <= n && n < (int64_t)1 << 31,
                "grace_topk_residual_step: bad arguments");
  GRACE_REQUIRE(n <= kSmallN || ws, "grace_topk_residual_step: workspace required");
  StepArgs a{g, residual, beta, gamma, n, k, vals, idx, out};
  hipStream_t s = as_stream(stream);
  if (out) {
    return has_residual ? run_topk<true, kDenseFused>(a, ws, ws_bytes_, s)
                        : run_topk<false, kDenseFused>(a, ws, ws_bytes_, s);
  }
  return has_residual ? run_topk<true, kDenseRes>(a, ws, ws_bytes_, s)
                      : run_topk<false, kDenseRes>(a, ws, ws_bytes_, s);
}

int64_t grace_topk_carry_size(int64_t n, int64_t k) {
  if (n <= kSmallN || k >= n || n >= (int64_t)1 << 31) return 0;   // no sampled bracket on these paths
  const int64_t sn = bracket_sample_n(n);
  return n / sn >= kCarryMinStratum ? carry_thr_off(sn) + 2 : 0;   // t at the sample positions + the u64 threshold
}

grace_status_t grace_topk_residual_step_carry(const float* g, float* residual, int32_t has_residual,
                                              float beta, float gamma, int64_t n, int64_t k, float* vals,
                                              int32_t* idx, float* out, float* carry, int64_t carry_len,
                                              int32_t carry_valid, const int32_t* prev_idx, int64_t prev_count,
                                              void* ws, size_t ws_bytes_, void* stream) {
  GRACE_REQUIRE(g && residual && vals && idx && n > 0 && k >= 1 && k <= n && n < (int64_t)1 << 31,
                "grace_topk_residual_step_carry: bad arguments");
  GRACE_REQUIRE(!carry || carry_len >= grace_topk_carry_size(n, k),
                "grace_topk_residual_step_carry: carry shorter than grace_topk_carry_size(n, k)");
  GRACE_REQUIRE(n <= kSmallN || ws, "grace_topk_residual_step_carry: workspace required");
  StepArgs a{g, residual, beta, gamma, n, k, vals, idx, out};
  a.prev_idx = prev_idx;
  a.prev_count = prev_idx ? prev_count : 0;
  if (carry && grace_topk_carry_size(n, k) > 0) {
    a.rs_out = carry;
    a.rs_in = has_residual && carry_valid ? carry : nullptr;   // read by the bracket, rewritten by main
  }
  hipStream_t s = as_stream(stream);
  if (out) {
    return has_residual ? run_topk<true, kDenseFused>(a, ws, ws_bytes_, s)
                        : run_topk<false, kDenseFused>(a, ws, ws_bytes_, s);
  }
  return has_residual ? run_topk<true, kDenseRes>(a, ws, ws_bytes_, s)
                      : run_topk<false, kDenseRes>(a, ws, ws_bytes_, s);
}

grace_status_t grace_topk_residual_step_swap(const float* g, const float* r_in, int32_t has_residual, float beta,
                                             float gamma, int64_t n, int64_t k, float* vals, int32_t* idx,
                                             float* r_out, float* carry, int64_t carry_len, int32_t carry_valid,
                                             void* ws, size_t ws_bytes_, void* stream) {
  GRACE_REQUIRE(g && r_out && (!has_residual || r_in) && r_in != r_out && vals && idx && n > 0 && k >= 1 &&
                    k <= n && n < (int64_t)1 << 31,
                "grace_topk_residual_step_swap: bad arguments (r_in and r_out distinct)");
  GRACE_REQUIRE(!carry || carry_len >= grace_topk_carry_size(n, k),
                "grace_topk_residual_step_swap: carry shorter than grace_topk_carry_size(n, k)");
  GRACE_REQUIRE(n <= kSmallN || ws, "grace_topk_residual_step_swap: workspace required");
  StepArgs a{g, r_out, beta, gamma, n, k, vals, idx, nullptr};
  a.r_in = has_residual ? r_in : nullptr;
  if (carry && grace_topk_carry_size(n, k) > 0) {
    a.rs_out = carry;
    a.rs_in = has_residual && carry_valid ? carry : nullptr;
  }
  hipStream_t s = as_stream(stream);
  if (has_residual) return run_topk<true, kResSwap>(a, ws, ws_bytes_, s);
  a.r_in = a.r;   // (never read without a residual; distinct from nothing)
  return run_topk<false, kResSwap>(a, ws, ws_bytes_, s);
}

grace_status_t grace_sparse_decode(const float* vals, const int32_t* idx, int64_t count, float* out,
                                   int64_t n, void* stream) {
  GRACE_REQUIRE(out && n >= 0 && count >= 0 && (count == 0 || (vals && idx)),
                "grace_sparse_decode: bad arguments");
  grace_status_t st = grace_fill(out, 0.f, n, stream);
  if (st != GRACE_OK || count == 0) return st;
  scatter_kernel<<<stream_grid(count, 256, 1024), 256, 0, as_stream(stream)>>>(vals, idx, count, out);
  GRACE_CHECK_LAUNCH("grace_sparse_decode");
  return GRACE_OK;
}

grace_status_t grace_sparse_decode_i64(const float* vals, const int64_t* idx, int64_t count,
                                       float* out, int64_t n, void* stream) {
  GRACE_REQUIRE(out && n >= 0 && count >= 0 && (count == 0 || (vals && idx)),
                "grace_sparse_decode_i64: bad arguments");
  grace_status_t st = grace_fill(out, 0.f, n, stream);
  if (st != GRACE_OK || count == 0) return st;
  scatter_kernel_i64<<<stream_grid(count, 256, 1024), 256, 0, as_stream(stream)>>>(vals, idx, count, out);
  GRACE_CHECK_LAUNCH("grace_sparse_decode_i64");
  return GRACE_OK;
}

grace_status_t grace_sparse_aggregate_into(const float* vals, const int32_t* idx, int64_t stride,
                                           const int64_t* counts_host, int32_t world, float divisor,
                                           float* out, int32_t* tags, int64_t n, void* stream) {
  GRACE_REQUIRE(vals && idx && counts_host && out && tags && world >= 1 && world <= kMaxAggWorld && n >= 0,
                "grace_sparse_aggregate: bad arguments (1 <= world <= 64)");
  hipStream_t s = as_stream(stream);
  for (int w = 0; w < world; ++w) {
    const int64_t c = counts_host[w];
    if (c <= 0) continue;
    scatter_add_tag_kernel<<<stream_grid(c, 256, 1024), 256, 0, s>>>(vals + w * stride, idx + w * stride,
                                                                      c, w, out, tags);
    GRACE_CHECK_LAUNCH("grace_sparse_aggregate");
  }
  if (divisor != 1.0f) {
    for (int w0 = 0; w0 < world; w0 += kMaxAggWorld) {   // one launch per 64 ranks
      const int nw = min(kMaxAggWorld, world - w0);
      AggCum cum;
      int64_t total = 0;
      for (int w = 0; w < nw; ++w) {
        cum.v[w] = total;
        total += counts_host[w0 + w] > 0 ? counts_host[w0 + w] : 0;
      }
      cum.v[nw] = total;
      if (total == 0) continue;
      // tags hold absolute ranks: shift the tag base by w0 through the idx/tags comparison below
      tag_divide_kernel<<<stream_grid(total, 256, 2048), 256, 0, s>>>(idx + w0 * stride, stride, cum, nw, divisor,
                                                                       out, tags);
      GRACE_CHECK_LAUNCH("grace_sparse_aggregate");
      if (w0 + nw < world) {
        set_error_msg("grace_sparse_aggregate: more than 64 ranks per divide launch is not supported");
        return GRACE_ERR_ARG;
      }
    }
  }
  return GRACE_OK;
}

grace_status_t grace_sparse_aggregate(const float* vals, const int32_t* idx, int64_t stride,
                                      const int64_t* counts_host, int32_t world, float divisor,
                                      float* out, int32_t* tags, int64_t n, void* stream) {
  GRACE_REQUIRE(vals && idx && counts_host && out && tags && world >= 1 && n >= 0,
                "grace_sparse_aggregate: bad arguments");
  grace_status_t st = grace_fill(out, 0.f, n, stream);
  if (st != GRACE_OK) return st;
  return grace_sparse_aggregate_into(vals, idx, stride, counts_host, world, divisor, out, tags, n, stream);
}



int32_t grace_topk_segmented_small_max(void) { return kSegSmallMax; }

int64_t grace_topk_segmented_chunk(int32_t has_residual, int32_t dense_out) {
  if (has_residual) return dense_out ? kChunkOf<true, kDenseFused> : kChunkOf<true, kDenseRes>;
  return dense_out ? kChunkOf<false, kDenseFused> : kChunkOf<false, kDenseRes>;
}

int64_t grace_topk_segmented_seg_ws_bytes(int64_t n, int64_t k) { return seg_ws_bytes_one(n, k); }

// f32 words of a large segment's carry: t at its sample positions + the u64 threshold
int64_t grace_topk_segmented_carry_len(int64_t n) { return carry_thr_off(seg_sample_n(n)) + 2; }

// finalize workgroups for a large segment: one round (kSelBlock * kFinPer candidates) each for the
// ~2-3 k a segment's small-sample band holds, plus one.  4 k budgeted: at 2 k a second round per
// workgroup made the largest tensors' routing 8-10 us instead of 3 (ddp_segmented 110.7 -> 106.3 us,
// profiles/r04_seg_fin_ab.txt).  A/B knob: budget GRACE_SEG_FIN_MULT k
#ifndef GRACE_SEG_FIN_MULT
#define GRACE_SEG_FIN_MULT 4
#endif
int64_t grace_topk_segmented_workspace_bytes(const int64_t* sizes, const int64_t* ks, int32_t count) {
  if (!sizes || !ks || count < 0) return -1;
  int64_t total = 0;
  for (int32_t i = 0; i < count; ++i)
    total += (int64_t)align256((size_t)seg_ws_bytes_one(sizes[i] < 1 ? 1 : sizes[i], ks[i] < 1 ? 1 : ks[i]));
  return total;
}

int32_t grace_topk_segmented_fin_blocks(int64_t n, int64_t k) {
  const int64_t per = (int64_t)kSelBlock * kFinPer;
  int64_t c = GRACE_SEG_FIN_MULT * k < n ? GRACE_SEG_FIN_MULT * k : n;
  c = (c + per - 1) / per + 1;
  return (int32_t)(c > kFinBlocks ? kFinBlocks : c);
}

grace_status_t grace_topk_segmented_step(const float* g, float* residual, int32_t has_residual, float beta,
                                         float gamma, const int64_t* seg_off, const int64_t* k_off,
                                         const int32_t* large, int32_t n_large, const int32_t* small,
                                         int32_t n_small, const int64_t* chk_off, const int32_t* chunk_li,
                                         int64_t nchunks, const int64_t* ws_off, const int64_t* fin_off,
                                         const int32_t* fin_li, int64_t nfin, int64_t n_total, float* vals,
                                         int32_t* idx, float* out, float* carry, const int64_t* carry_off,
                                         int32_t carry_valid, void* ws, size_t ws_bytes, int64_t ws_need,
                                         void* stream) {
  GRACE_REQUIRE(g && residual && seg_off && k_off && vals && idx && n_large >= 0 && n_small >= 0 &&
                    n_large + n_small >= 1 && n_total >= 1 && n_total < ((int64_t)1 << 31) &&
                    (n_large == 0 || (large && chk_off && chunk_li && ws_off && fin_off && fin_li && ws &&
                                      nchunks >= 1 && nfin >= n_large)) &&
                    (n_small == 0 || small),
                "grace_topk_segmented_step: bad arguments");
  SegPlan p{};
  p.g = g;
  p.r = residual;
  p.out = out;
  p.vals = vals;
  p.idx = idx;
  p.beta = beta;
  p.gamma = gamma;
  p.seg_off = seg_off;
  p.k_off = k_off;
  p.large = large;
  p.small = small;
  p.chk_off = chk_off;
  p.chunk_li = chunk_li;
  p.ws_off = ws_off;
  p.fin_off = fin_off;
  p.fin_li = fin_li;
  p.ws = reinterpret_cast<char*>(ws);
  p.nL = n_large;
  p.nS = n_small;
  GRACE_REQUIRE(!carry || carry_off, "grace_topk_segmented_step: carry without carry_off");
  // written by every step (a first step without a residual records t = g), read only with a
  // residual whose previous step wrote it
  p.carry = carry;
  p.carry_off = carry_off;
  p.carry_valid = carry && has_residual && carry_valid ? 1 : 0;
  GRACE_REQUIRE(n_large == 0 || (ws_need > 0 && ws_bytes >= (size_t)ws_need),
                "grace_topk_segmented_step: workspace smaller than grace_topk_segmented_workspace_bytes");
  const bool vec = ((reinterpret_cast<uintptr_t>(g) | reinterpret_cast<uintptr_t>(residual) |
                     reinterpret_cast<uintptr_t>(out)) & 15u) == 0;
  hipStream_t s = as_stream(stream);
  if (has_residual)
    return out ? run_segmented<true, kDenseFused>(p, nchunks, nfin, vec, s)
               : run_segmented<true, kDenseRes>(p, nchunks, nfin, vec, s);
  return out ? run_segmented<false, kDenseFused>(p, nchunks, nfin, vec, s)
             : run_segmented<false, kDenseRes>(p, nchunks, nfin, vec, s);
}

}  // extern "C"
