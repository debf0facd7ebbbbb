// Per-tensor top-k + residual over a whole model's gradients in one launch sequence (CDNA4).
//
// The reference's DDP loop calls Communicator.step once per parameter tensor
// (examples/dist/CIFAR10-dawndist/core.py:203-206), each a TopKCompressor(ratio) with its own
// k_i = max(1, int(n_i * ratio)) (grace_dl/dist/compressor/topk.py:34) and its own residual
// (grace_dl/dist/memory/residual.py:10-20).  At ResNet-50's 161 tensors (64 .. 2.4 M elements) that
// loop is launch-bound.  Here all tensors sit back to back in one flat buffer (the segments) and
// ONE sequence of four launches runs every tensor's exact top-k with exactly those semantics:
//
//   p1      (chunks)    t = beta r + gamma g, r' = t, per-segment 2048-bin histogram of |t| >> 20
//                       (per-wave LDS histograms, one global atomic per non-zero bin per chunk)
//   find    (segments)  the bin B_i holding segment i's k_i-th largest key, the count above it
//                       (re-zeroes the histogram for the next call)
//   p2      (chunks)    reads t back: key bin > B_i -> selected (payload, dense out = 0 + t,
//                       r' = t - t); bin == B_i -> candidate list; dense out = 0 elsewhere
//   select  (segments)  exact choice of the remaining need_i candidates of bin B_i by
//                       (|t| desc, index asc) -- the single-bucket engine's tie rule
//
// No sampling, so no miss path: a degenerate tensor (all ties) only makes its candidate list long.
// Traffic 20 B per element (p1: read g, r, write r'; p2: read r', write out) against the single-bucket
// engine's 16; the point of this path is the per-tensor k, not the last 20 %.
// Payload indices are GLOBAL (flat-buffer) int32 indices; per-tensor local index = global - seg_off.
#include "common.h"
#include "select.h"

namespace grace {

typedef float f32x4v __attribute__((ext_vector_type(4)));
constexpr int kSegBlock = 256;
#ifndef GRACE_SEG_CHUNK
#define GRACE_SEG_CHUNK 8192
#endif
// elements per p1 / p2 workgroup: p1's per-wave histograms are cleared and reduced once per chunk,
// so longer chunks amortise them (ResNet-50 set, 161 tensors: 4096 -> 8192 elements, step 0.211 /
// 0.214 -> 0.186 / 0.194 ms, A/B on one box)
constexpr int kSegChunk = GRACE_SEG_CHUNK;
constexpr int kSegQ = kSegChunk / (4 * kSegBlock);    // quads per thread
static_assert(kSegQ * 4 <= 32, "one mask bit per element of a thread");
constexpr int kSegBins = 2048;                        // histogram of key >> 20
constexpr int kSegSelBlock = 1024;
constexpr int kSelR = 16;                             // candidates per thread held in registers

struct SegCtl {
  int32_t B;        // boundary bin (-1: every element selected)
  uint32_t above;   // elements in bins > B
  uint32_t need;    // how many of bin B are still selected
  uint32_t n_sel;   // p2 payload fill counter
  uint32_t n_cand;  // p2 candidate-list fill counter
  uint32_t pad[3];
};
static_assert(sizeof(SegCtl) == 32, "ctl slot");

struct SegArgs {
  const float* g;
  float* r;
  int has_res;
  float beta, gamma;
  const int64_t* seg_off;    // [nseg + 1] element offsets
  const int64_t* k_off;      // [nseg + 1] payload offsets (k_i prefix sums)
  const int64_t* chk_off;    // [nseg + 1] chunk offsets
  const int32_t* chunk_seg;  // [nchunks] segment of each chunk
  float* vals;
  int32_t* idx;
  float* out;                // dense world-1 output (may alias g), or null
  uint32_t* hist;            // [nseg][kSegBins]
  SegCtl* ctl;               // [nseg]
  int2* cand;                // [n_total]: segment i's candidates at seg_off[i]
};

// this workgroup's chunk [c0, c1) of segment s; `aligned`: 16-B quads (segment start and bases)
struct SegChunk {
  int s;
  int64_t c0, c1;
};
__device__ __forceinline__ SegChunk seg_chunk(const SegArgs& a, int64_t chunk) {
  SegChunk c;
  c.s = a.chunk_seg[chunk];
  const int64_t s0 = a.seg_off[c.s], s1 = a.seg_off[c.s + 1];
  c.c0 = s0 + (chunk - a.chk_off[c.s]) * kSegChunk;
  c.c1 = min(c.c0 + (int64_t)kSegChunk, s1);
  return c;
}
__device__ __forceinline__ SegChunk seg_chunk(const SegArgs& a) { return seg_chunk(a, blockIdx.x); }

#ifndef GRACE_SEG_P1_CHUNKS
#define GRACE_SEG_P1_CHUNKS 4
#endif
// p1 chunks per workgroup: the per-segment histogram leaves with one global atomic per non-zero
// bin per flush, and a workgroup flushes once per segment it covers instead of once per chunk
// (the atomics of one flush per 8192-element chunk kept the memory-side atomic unit busy ~20 us
// past p1's end: the find kernel's first loads waited for them)
constexpr int kSegP1Chunks = GRACE_SEG_P1_CHUNKS;

__device__ __forceinline__ void seg_quad(const float* p, int64_t e, int64_t end, bool vec, float (&v)[4]) {
  if (vec && e + 3 < end) {
    const f32x4v q = __builtin_nontemporal_load(reinterpret_cast<const f32x4v*>(p + e));
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = e + j < end ? p[e + j] : 0.f;
  }
}
__device__ __forceinline__ void seg_store(float* p, int64_t e, int64_t end, bool vec, const float (&v)[4]) {
  if (vec && e + 3 < end) {
    __builtin_nontemporal_store(f32x4v{v[0], v[1], v[2], v[3]}, reinterpret_cast<f32x4v*>(p + e));
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (e + j < end) p[e + j] = v[j];
  }
}

// ---- p1: compensate, residual = t, per-segment histogram
__global__ __launch_bounds__(kSegBlock) void seg_p1_kernel(SegArgs a, int vec_base, int64_t nchunks) {
  __shared__ uint32_t lh[kSegBlock / kWave][kSegBins];   // one histogram per wave: fewer same-bin conflicts
  const int tid = threadIdx.x, w = tid >> 6;
  for (int b = tid; b < (kSegBlock / kWave) * kSegBins; b += kSegBlock) (&lh[0][0])[b] = 0u;
  const int64_t ch0 = (int64_t)blockIdx.x * kSegP1Chunks, ch1 = min(ch0 + (int64_t)kSegP1Chunks, nchunks);
  for (int64_t ch = ch0; ch < ch1; ++ch) {
    const SegChunk c = seg_chunk(a, ch);
    const bool vec = vec_base && (c.c0 & 3) == 0;
    float gv[kSegQ][4], rv[kSegQ][4] = {};
#pragma unroll
    for (int u = 0; u < kSegQ; ++u) {
      const int64_t e = c.c0 + 4 * ((int64_t)u * kSegBlock + tid);
      seg_quad(a.g, e, c.c1, vec, gv[u]);
      if (a.has_res) seg_quad(a.r, e, c.c1, vec, rv[u]);
    }
    __syncthreads();   // (first chunk: the histogram clear)
#pragma unroll
    for (int u = 0; u < kSegQ; ++u) {
      const int64_t e = c.c0 + 4 * ((int64_t)u * kSegBlock + tid);
      float t[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        t[j] = a.has_res ? a.beta * rv[u][j] + a.gamma * gv[u][j] : gv[u][j];
        if (e + j < c.c1) atomicAdd(&lh[w][abs_key(t[j]) >> 20], 1u);
      }
      seg_store(a.r, e, c.c1, vec, t);
    }
    // flush when the next chunk belongs to another segment (or this is the last one)
    if (ch + 1 == ch1 || a.chunk_seg[ch + 1] != c.s) {
      __syncthreads();
      uint32_t* gh = a.hist + (int64_t)c.s * kSegBins;
      for (int b = tid; b < kSegBins; b += kSegBlock) {
        uint32_t v = 0;
#pragma unroll
        for (int ww = 0; ww < kSegBlock / kWave; ++ww) { v += lh[ww][b]; lh[ww][b] = 0u; }
        if (v) atomicAdd(&gh[b], v);
      }
    }
  }
}

// ---- find: per segment, the boundary bin of its k-th largest key (one workgroup per segment)
__global__ __launch_bounds__(kSegBlock) void seg_find_kernel(SegArgs a) {
  __shared__ uint32_t s_w[kSegBlock / kWave + 1];
  __shared__ uint32_t s_res[2];
  const int s = blockIdx.x;
  const int64_t n_s = a.seg_off[s + 1] - a.seg_off[s];
  const int64_t k_s = a.k_off[s + 1] - a.k_off[s];
  uint32_t* gh = a.hist + (int64_t)s * kSegBins;
  SegCtl c{};
  if (k_s >= n_s) {
    c.B = -1;
    c.above = (uint32_t)n_s;
    c.need = 0;
  } else {
    uint32_t above = 0;
    c.B = find_bin_desc<kSegBlock, kSegBins>(gh, (uint32_t)k_s, s_w, s_res, &above);
    c.above = above;
    c.need = (uint32_t)k_s - above;
  }
  __syncthreads();
  for (int b = threadIdx.x; b < kSegBins; b += kSegBlock) gh[b] = 0u;   // zeroed for the next call
  if (threadIdx.x == 0) a.ctl[s] = c;                                   // n_sel = n_cand = 0
}

// ---- p2: route every element of the segment by its key bin
__global__ __launch_bounds__(kSegBlock) void seg_p2_kernel(SegArgs a, int vec_base) {
  __shared__ uint32_t s_w[kSegBlock / kWave + 1];
  __shared__ uint32_t s_base[2];
  const SegChunk c = seg_chunk(a);
  const int tid = threadIdx.x;
  const SegCtl ct = a.ctl[c.s];
  const bool vec = vec_base && (c.c0 & 3) == 0;
  float tv[kSegQ][4];
#pragma unroll
  for (int u = 0; u < kSegQ; ++u) {
    const int64_t e = c.c0 + 4 * ((int64_t)u * kSegBlock + tid);
    if (vec && e + 3 < c.c1) {   // t was written by p1 moments ago: plain loads can hit the caches
      const f32x4v q = *reinterpret_cast<const f32x4v*>(a.r + e);
      tv[u][0] = q.x; tv[u][1] = q.y; tv[u][2] = q.z; tv[u][3] = q.w;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) tv[u][j] = e + j < c.c1 ? a.r[e + j] : 0.f;
    }
  }
  uint32_t msel = 0, mcand = 0;   // bit u * 4 + j
#pragma unroll
  for (int u = 0; u < kSegQ; ++u) {
    const int64_t e = c.c0 + 4 * ((int64_t)u * kSegBlock + tid);
    float o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const bool valid = e + j < c.c1;
      const int bin = (int)(abs_key(tv[u][j]) >> 20);
      const bool sel = valid && bin > ct.B;
      const bool cnd = valid && bin == ct.B;
      msel |= (uint32_t)sel << (u * 4 + j);
      mcand |= (uint32_t)cnd << (u * 4 + j);
      o[j] = sel ? 0.f + tv[u][j] : 0.f;
      if (sel) a.r[e + j] = tv[u][j] - tv[u][j];
    }
    if (a.out) seg_store(a.out, e, c.c1, vec, o);
  }
  const uint32_t packed = (uint32_t)__popc(msel) | ((uint32_t)__popc(mcand) << 16);
  uint32_t tot;
  const uint32_t ex = block_excl_scan<kSegBlock>(packed, s_w, &tot);
  if (tid == 0) {
    s_base[0] = (tot & 0xFFFFu) ? atomicAdd(&a.ctl[c.s].n_sel, tot & 0xFFFFu) : 0u;
    s_base[1] = (tot >> 16) ? atomicAdd(&a.ctl[c.s].n_cand, tot >> 16) : 0u;
  }
  __syncthreads();
  uint32_t ps = s_base[0] + (ex & 0xFFFFu), pc = s_base[1] + (ex >> 16);
  const int64_t kbase = a.k_off[c.s], cbase = a.seg_off[c.s];
#pragma unroll
  for (int u = 0; u < kSegQ; ++u) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int b = u * 4 + j;
      const int64_t i = c.c0 + 4 * ((int64_t)u * kSegBlock + tid) + j;
      if ((msel >> b) & 1u) {
        a.vals[kbase + ps] = tv[u][j];
        a.idx[kbase + ps] = (int32_t)i;
        ++ps;
      } else if ((mcand >> b) & 1u) {
        a.cand[cbase + pc] = make_int2((int)i, (int)f2u(tv[u][j]));
        ++pc;
      }
    }
  }
}

// ---- select: the need_i best of segment i's boundary-bin candidates (one workgroup per segment)
__global__ __launch_bounds__(kSegSelBlock) void seg_select_kernel(SegArgs a) {
  __shared__ uint32_t hist[2048];
  __shared__ uint32_t s_w[kSegSelBlock / kWave + 1];
  __shared__ uint32_t s_res[2];
  __shared__ uint32_t s_pos;
  const int s = blockIdx.x;
  const SegCtl ct = a.ctl[s];
  if (ct.need == 0) return;
  const int2* list = a.cand + a.seg_off[s];
  const uint32_t nc = ct.n_cand;
  if (nc <= (uint32_t)(kSegSelBlock * kSelR)) {
    // the list held in registers for every radix pass (the global-list select below re-reads it
    // from memory once per pass, a dependent round trip per round of loads)
    int2 e[kSelR];
#pragma unroll
    for (int u = 0; u < kSelR; ++u) {
      const uint32_t j = threadIdx.x + (uint32_t)u * kSegSelBlock;
      e[u] = j < nc ? list[j] : make_int2(0, 0);
    }
    auto comp = [&](int u) { return comp_key(abs_key(u2f((uint32_t)e[u].y)), (uint32_t)e[u].x); };
    uint64_t prefix = (uint64_t)((uint32_t)ct.B >> 1) << 53, pmask = (uint64_t)2047u << 53;
    uint32_t rem = ct.need;
    for (int pass = 1; pass < 6; ++pass) {   // block_select_comp's passes, from the second digit
      const int shift = pass < 5 ? 53 - 11 * pass : 0;
      const uint32_t dmask = pass < 5 ? 2047u : 511u;
      for (int b = threadIdx.x; b < 2048; b += kSegSelBlock) hist[b] = 0;
      __syncthreads();
#pragma unroll
      for (int u = 0; u < kSelR; ++u) {
        const uint64_t c = comp(u);
        if (threadIdx.x + (uint32_t)u * kSegSelBlock < nc && (c & pmask) == prefix)
          atomicAdd(&hist[(c >> shift) & dmask], 1u);
      }
      __syncthreads();
      uint32_t above;
      const int d = find_bin_desc<kSegSelBlock, 2048>(hist, rem, s_w, s_res, &above);
      rem -= above;
      prefix |= (uint64_t)d << shift;
      pmask |= (uint64_t)dmask << shift;
      const bool whole = hist[d] == rem;
      __syncthreads();
      if (whole) break;
    }
    if (threadIdx.x == 0) s_pos = 0;
    __syncthreads();
    const int64_t kb = a.k_off[s] + ct.above;
#pragma unroll
    for (int u = 0; u < kSelR; ++u) {
      if (threadIdx.x + (uint32_t)u * kSegSelBlock < nc && comp(u) >= prefix) {
        const float v = u2f((uint32_t)e[u].y);
        const uint32_t p = atomicAdd(&s_pos, 1u);
        a.vals[kb + p] = v;
        a.idx[kb + p] = e[u].x;
        a.r[e[u].x] = v - v;
        if (a.out) a.out[e[u].x] = 0.f + v;
      }
    }
    return;
  }
  auto src = [list](int64_t j) {
    const int2 e = list[j];
    return comp_key(abs_key(u2f((uint32_t)e.y)), (uint32_t)e.x);
  };
  // every candidate's key is in bin B (key >> 20 == B), so the top digit of the composite (its
  // bits 53..63 = key bits 21..31) is B >> 1 for all of them: start at the second pass
  const uint64_t T = block_select_comp<kSegSelBlock>(src, nc, ct.need, hist, s_w, s_res, 1,
                                                     (uint64_t)((uint32_t)ct.B >> 1) << 53, (uint64_t)2047u << 53);
  if (threadIdx.x == 0) s_pos = 0;
  __syncthreads();
  const int64_t kb = a.k_off[s] + ct.above;
  for (uint32_t j = threadIdx.x; j < nc; j += kSegSelBlock) {
    const int2 e = list[j];
    const float v = u2f((uint32_t)e.y);
    if (comp_key(abs_key(v), (uint32_t)e.x) >= T) {
      const uint32_t p = atomicAdd(&s_pos, 1u);
      a.vals[kb + p] = v;
      a.idx[kb + p] = e.x;
      a.r[e.x] = v - v;
      if (a.out) a.out[e.x] = 0.f + v;
    }
  }
}

static inline size_t seg_align(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace grace

using namespace grace;

extern "C" {

size_t grace_topk_segmented_workspace_bytes(int64_t n_total, int32_t nseg) {
  return seg_align(sizeof(uint32_t) * kSegBins * (size_t)nseg) + seg_align(sizeof(SegCtl) * (size_t)nseg) +
         seg_align(sizeof(int2) * (size_t)n_total);
}

int32_t grace_topk_segmented_chunk(void) { return kSegChunk; }

grace_status_t grace_topk_segmented_step(const float* g, float* residual, int32_t has_residual, float beta,
                                         float gamma, const int64_t* seg_off, const int64_t* k_off,
                                         const int64_t* chk_off, const int32_t* chunk_seg, int32_t nseg,
                                         int64_t n_total, int64_t nchunks, float* vals, int32_t* idx, float* out,
                                         void* ws, size_t ws_bytes, void* stream) {
  GRACE_REQUIRE(g && residual && seg_off && k_off && chk_off && chunk_seg && vals && idx && ws && nseg >= 1 &&
                    n_total >= 1 && n_total < ((int64_t)1 << 31) && nchunks >= 1,
                "grace_topk_segmented_step: bad arguments");
  GRACE_REQUIRE(ws_bytes >= grace_topk_segmented_workspace_bytes(n_total, nseg),
                "grace_topk_segmented_step: workspace too small");
  char* p = reinterpret_cast<char*>(ws);
  SegArgs a{};
  a.g = g;
  a.r = residual;
  a.has_res = has_residual ? 1 : 0;
  a.beta = beta;
  a.gamma = gamma;
  a.seg_off = seg_off;
  a.k_off = k_off;
  a.chk_off = chk_off;
  a.chunk_seg = chunk_seg;
  a.vals = vals;
  a.idx = idx;
  a.out = out;
  a.hist = reinterpret_cast<uint32_t*>(p);
  p += seg_align(sizeof(uint32_t) * kSegBins * (size_t)nseg);
  a.ctl = reinterpret_cast<SegCtl*>(p);
  p += seg_align(sizeof(SegCtl) * (size_t)nseg);
  a.cand = reinterpret_cast<int2*>(p);
  const int vec = ((reinterpret_cast<uintptr_t>(g) | reinterpret_cast<uintptr_t>(residual) |
                    reinterpret_cast<uintptr_t>(out)) & 15u) == 0;
  hipStream_t st = as_stream(stream);
  seg_p1_kernel<<<(unsigned)((nchunks + kSegP1Chunks - 1) / kSegP1Chunks), kSegBlock, 0, st>>>(a, vec, nchunks);
  GRACE_CHECK_LAUNCH("grace_topk_segmented_step");
  seg_find_kernel<<<(unsigned)nseg, kSegBlock, 0, st>>>(a);
  GRACE_CHECK_LAUNCH("grace_topk_segmented_step");
  seg_p2_kernel<<<(unsigned)nchunks, kSegBlock, 0, st>>>(a, vec);
  GRACE_CHECK_LAUNCH("grace_topk_segmented_step");
  seg_select_kernel<<<(unsigned)nseg, kSegSelBlock, 0, st>>>(a);
  GRACE_CHECK_LAUNCH("grace_topk_segmented_step");
  return GRACE_OK;
}

}  // extern "C"
