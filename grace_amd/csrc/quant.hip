// Quantisation codecs for CDNA4: QSGD (bucketed stochastic levels), TernGrad (ternary with a
// clipped max scale), natural compression (cupy and cnat_cuda encodings) and fp16.
//
// Every codec works on a SEGMENTED bucket: one flat f32 buffer holding `nseg` tensors back to
// back, described by a device offset table seg_off[nseg + 1].  A single tensor is one segment.
// This is what lets the 161-tensor ResNet-50 gradient set run as one launch per stage instead of
// 161 (SURVEY.md §7 "small-tensor overhead").
//
// Randomness: `u` (uniform [0,1) floats) or `ri` (natural's random ints) may be injected (parity
// mode, the reference's own generator streams); when NULL a counter-based device generator
// (common.h uniform01) keyed by `seed` is used.
#include <hip/hip_fp16.h>
#include <math.h>

#include "common.h"

namespace grace {

constexpr int kQBlock = 256;
// Row kernels: buckets (chunks) per 16-lane row per iteration, and grid caps.  A/B on the ResNet-50
// set (tools/exp_tern_ab.py, two boxes): 2 buckets per row beat 4 for every row kernel (fewer
// registers, more rows in flight); the QSGD encoder is best at <= 4096 workgroups (a few
// iterations per row: 38 -> 34 us), the decoders at <= 8192 (QSGD 24 -> 22 us, TernGrad 25 -> 21 us).
#ifndef GRACE_QNB
#define GRACE_QNB 2
#endif
constexpr int kQNB = GRACE_QNB;
#ifndef GRACE_QGRID
#define GRACE_QGRID 8192
#endif
constexpr int kQGridCap = GRACE_QGRID;      // decoders
#ifndef GRACE_QENC_GRID
#define GRACE_QENC_GRID 4096
#endif
constexpr int kQEncGridCap = GRACE_QENC_GRID;   // QSGD encoder
constexpr int kSegLds = 512;     // offset tables up to this many segments are staged in LDS

// segment containing flat element / bucket index `x`: largest s with off[s] <= x
__device__ __forceinline__ int find_seg(const int64_t* off, int nseg, int64_t x) {
  int lo = 0, hi = nseg - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (off[mid] <= x) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// Offset tables (seg_off and the per-segment sub-block table) staged once per workgroup, so the
// per-bucket / per-quad segment search runs on LDS instead of dependent global loads.
struct SegTables {
  int64_t seg[kSegLds + 1];
  int64_t sub[kSegLds + 1];
};

struct SegView {
  const int64_t* seg;
  const int64_t* sub;
};

__device__ __forceinline__ SegView stage_tables(SegTables& t, const int64_t* seg, const int64_t* sub, int nseg) {
  if (nseg <= kSegLds) {
    for (int i = threadIdx.x; i <= nseg; i += blockDim.x) {
      t.seg[i] = seg[i];
      if (sub) t.sub[i] = sub[i];
    }
    __syncthreads();
    return SegView{t.seg, sub ? t.sub : nullptr};
  }
  return SegView{seg, sub};
}

// advance a segment cursor monotonically: largest s' >= s with off[s'] <= x
__device__ __forceinline__ int seg_advance(const int64_t* off, int nseg, int s, int64_t x) {
  while (s + 1 < nseg && off[s + 1] <= x) ++s;
  return s;
}

// contiguous per-workgroup range [lo, hi) of `total` items, in multiples of `step`
__device__ __forceinline__ void block_range(int64_t total, int64_t step, int64_t& lo, int64_t& hi) {
  int64_t per = (total + gridDim.x - 1) / gridDim.x;
  per = (per + step - 1) / step * step;
  lo = min((int64_t)blockIdx.x * per, total);
  hi = min(lo + per, total);
}

// float -> int16 exactly as torch CPU on x86 (cvttss2si to int32, low 16 bits): NaN / out of
// int32 range -> 0x80000000 -> 0.  Used by QSGD's .type(torch.int16) (qsgd.py:36).
__device__ __forceinline__ int32_t f2i16_x86(float v) {
  if (!(fabsf(v) < 2147483648.0f)) return 0;   // NaN, inf, |v| >= 2^31
  return (int32_t)(int16_t)(int32_t)v;
}

typedef float f4v __attribute__((ext_vector_type(4)));

// 4 consecutive floats from p[e .. e+3], zero past `end`; one 16-B load when aligned and full
__device__ __forceinline__ void load_quad(const float* __restrict__ p, int64_t e, int64_t end, bool aligned,
                                          float (&v)[4]) {
  if (aligned && e + 3 < end) {
    const f4v q = *reinterpret_cast<const f4v*>(p + e);
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = e + j < end ? p[e + j] : 0.f;
  }
}

// ================================================================================================
// QSGD (grace_dl/dist/compressor/qsgd.py:12-51)
//   norm_b   = sqrt(sum over the zero-padded bucket of x^2)          (f32 result; f64 accumulate)
//   level    = (reciprocal(norm) * q) * |x|   -- Tensor.__rdiv__ is reciprocal() * q
//   new      = floor(level) + (u < level - floor(level))
//   code     = int16(new * sign(x)) -> int8 (q < 128) or fp16 (q >= 128)
// A half-wave (32 lanes x 4 elements) owns one bucket of up to 128: one 16-B load per lane, the
// bucket norm is a 5-step xor-shuffle reduction, then the lane encodes the 4 values it holds and
// stores them with one 4-B (int8) / 8-B (fp16) write.  x is read exactly once.  Buckets larger
// than 128 loop over 128-element slices (two passes, the second hitting L2).
// VARIANT 0: QSGDCompressor (qsgd.py:12-39).  VARIANT 1: QSGDCompressor_CUDA / qsgd_cuda.cu:320-388
// (f64 norms over finite elements, level = q / norm * |x| by one division, NaN/Inf -> -128).
template <typename CodeT, int VARIANT>
__device__ __forceinline__ CodeT qsgd_code(float xv, float level, float ui, float norm) {
  const float prev = floorf(level);
  if constexpr (VARIANT == 0) {
    const float nl = prev + ((ui < level - prev) ? 1.0f : 0.0f);
    // nl * torch.sign(x) == copysign(nl, x) on every input: nl >= 0 or NaN, and where sign(x) is
    // 0 or NaN the product is 0 / NaN, which the int16 conversion maps to 0 either way
    const int32_t c16 = f2i16_x86(copysignf(nl, xv));
    if constexpr (sizeof(CodeT) == 1) return (CodeT)(int8_t)c16;
    else return (CodeT)__float2half((float)(int16_t)c16);
  } else {
    int8_t c = -128;
    if (isfinite(norm) && isfinite(xv)) {
      const int8_t pl = (int8_t)prev;
      c = (ui < level - prev) ? (int8_t)(pl + 1) : pl;
      if (xv < 0.f) c = (int8_t)-c;
    }
    return (CodeT)c;
  }
}

template <typename CodeT>
__device__ __forceinline__ void store_codes4(CodeT* __restrict__ codes, int64_t e, int64_t end, bool aligned,
                                             const CodeT (&c)[4]) {
  if (aligned && e + 3 < end) {
    if constexpr (sizeof(CodeT) == 1) {
      const uint32_t w = (uint32_t)(uint8_t)c[0] | ((uint32_t)(uint8_t)c[1] << 8) |
                         ((uint32_t)(uint8_t)c[2] << 16) | ((uint32_t)(uint8_t)c[3] << 24);
      *reinterpret_cast<uint32_t*>(codes + e) = w;
    } else {
      uint2 w;
      w.x = (uint32_t)__half_as_ushort(c[0]) | ((uint32_t)__half_as_ushort(c[1]) << 16);
      w.y = (uint32_t)__half_as_ushort(c[2]) | ((uint32_t)__half_as_ushort(c[3]) << 16);
      *reinterpret_cast<uint2*>(codes + e) = w;
    }
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (e + j < end) codes[e + j] = c[j];
  }
}

// ---- 32-bit fast path (n < 2^31, nseg <= kSegLds, bucket 128): every index is an int32, the offset
// tables sit in LDS as int32 and the generator key is hoisted, which roughly halves the VALU work
// per element against the general kernels (64-bit index math was a third of their instructions).
struct SegTables32 {
  int32_t seg[kSegLds + 1];
  int32_t sub[kSegLds + 1];
};

__device__ __forceinline__ void stage_tables32(SegTables32& t, const int64_t* seg, const int64_t* sub, int nseg) {
  for (int i = threadIdx.x; i <= nseg; i += blockDim.x) {
    t.seg[i] = (int32_t)seg[i];
    t.sub[i] = (int32_t)sub[i];
  }
  __syncthreads();
}

__device__ __forceinline__ int find_seg32(const int32_t* off, int nseg, int32_t x) {
  int lo = 0, hi = nseg - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (off[mid] <= x) lo = mid; else hi = mid - 1;
  }
  return lo;
}

__device__ __forceinline__ int seg_advance32(const int32_t* off, int nseg, int s, int32_t x) {
  while (s + 1 < nseg && off[s + 1] <= x) ++s;
  return s;
}

__device__ __forceinline__ void block_range32(int32_t total, int32_t step, int32_t& lo, int32_t& hi) {
  int32_t per = (total + (int32_t)gridDim.x - 1) / (int32_t)gridDim.x;
  per = (per + step - 1) / step * step;
  lo = min((int32_t)blockIdx.x * per, total);
  hi = min(lo + per, total);
}

// uniform01x4 for i < 2^32 with the key mix64(seed) precomputed: identical values
__device__ __forceinline__ void uniform01x4_k(uint64_t key, uint32_t i, float (&u)[4]) {
  uint32_t h = fmix32(((i * 0x9E3779B1u) ^ (uint32_t)key) + (uint32_t)(key >> 32));
  u[0] = (float)(h >> 8) * (1.0f / 16777216.0f);
  h = h ? h : 0x9E3779B9u;
#pragma unroll
  for (int j = 1; j < 4; ++j) {
    h ^= h << 13;
    h ^= h >> 17;
    h ^= h << 5;
    u[j] = (float)(h >> 8) * (1.0f / 16777216.0f);
  }
}

// A 16-lane row owns a bucket of 128: each lane two quads (l16, l16 + 16; two 16-B loads), the norm is
// one DPP row reduction; kQNB buckets per row per iteration with every load issued first.
// FUSED: the world-1 Allgather step (qsgd.py:41-51 decompress, allgather.py:44 sum from 0, division by
// 1 omitted) in the same pass: out = 0 + (norm / q) * code, written instead of the codes and norms --
// the same arithmetic as qsgd_decode_bkt_kernel, so the result is bit-identical to compress + decode.
template <typename CodeT, int VARIANT, bool FUSED = false>
__global__ __launch_bounds__(kQBlock) void qsgd_encode128_kernel(
    const float* __restrict__ x, const int64_t* __restrict__ seg_off, const int64_t* __restrict__ bkt_off,
    int nseg, int32_t nbuckets, float qf, const float* __restrict__ u, uint64_t seed,
    const float* __restrict__ norms_in, float* __restrict__ norms_out, CodeT* __restrict__ codes,
    float* __restrict__ fused_out = nullptr, uint32_t xoff = 0) {
  // xoff: the bucket element of x[0] for the device generator (a shard of a larger bucket,
  // grace_qsgd_compress_at): the draws are keyed by the bucket's element index
  __shared__ SegTables32 tab;
  // int8 codes leave as 16-B stores: each row stages its kQNB buckets' codes (128 B each) here and
  // every lane stores 16 contiguous bytes (a 4-B store per quad covered four 64-B pieces per wave
  // instruction: 10 of the encoder's 33 us)
#ifdef GRACE_QSGD_STORE4   // A/B build only: the per-quad 4-B code stores
  constexpr bool kStage16 = false;
#else
  constexpr bool kStage16 = !FUSED && sizeof(CodeT) == 1;
#endif
  const bool codes16 = (reinterpret_cast<uintptr_t>(codes) & 15) == 0;
  __shared__ uint32_t cst[kStage16 ? kQBlock / 16 : 1][kQNB * 32];
  stage_tables32(tab, seg_off, bkt_off, nseg);
  const int l16 = threadIdx.x & 15;
  constexpr int kRows = kQBlock / 16;
  const uint64_t key = mix64(seed);
  int32_t blo, bhi;
  block_range32(nbuckets, kRows, blo, bhi);
  const int32_t b_first = blo + (int32_t)(threadIdx.x >> 4);
  int s = b_first < bhi ? find_seg32(tab.sub, nseg, b_first) : 0;
  for (int32_t b = b_first; b < bhi; b += kQNB * kRows) {
    int32_t bb[kQNB], e[kQNB][2], end[kQNB];
    bool ok[kQNB], fast[kQNB][2];
    float v[kQNB][2][4];
#pragma unroll
    for (int h = 0; h < kQNB; ++h) {
      bb[h] = b + h * kRows;
      ok[h] = bb[h] < bhi;
      if (ok[h]) s = seg_advance32(tab.sub, nseg, s, bb[h]);
      const int32_t base = tab.seg[s] + (bb[h] - tab.sub[s]) * 128;
      end[h] = ok[h] ? min(base + 128, tab.seg[s + 1]) : base;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        e[h][q] = base + 4 * l16 + 64 * q;   // quads l16 and l16 + 16: each instruction covers 256 contiguous bytes per row
        fast[h][q] = ok[h] && (base & 3) == 0 && e[h][q] + 3 < end[h];
        // unconditional 16-B load (element 0 stands in for a slow quad): a load under a divergent
        // branch makes the compiler wait vmcnt(0) at the join, serialising the loads
        const f4v t = *reinterpret_cast<const f4v*>(x + (fast[h][q] ? e[h][q] : 0));
        v[h][q][0] = t.x; v[h][q][1] = t.y; v[h][q][2] = t.z; v[h][q][3] = t.w;
      }
    }
#pragma unroll
    for (int h = 0; h < kQNB; ++h)   // quads at a segment edge / unaligned segment (rare)
#pragma unroll
      for (int q = 0; q < 2; ++q)
        if (!fast[h][q]) {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[h][q][j] = ok[h] && e[h][q] + j < end[h] ? x[e[h][q] + j] : 0.f;
        }
    float norm[kQNB];
    if (norms_in) {
#pragma unroll
      for (int h = 0; h < kQNB; ++h) norm[h] = ok[h] ? norms_in[bb[h]] : 1.f;
    } else {
#pragma unroll
      for (int h = 0; h < kQNB; ++h) {
        // squares of f32 values are exact in f64, so fma == add of the exact product
        double acc = 0.0;
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (VARIANT == 0 || isfinite(v[h][q][j])) acc = fma((double)v[h][q][j], (double)v[h][q][j], acc);
        acc = row16_sum(acc);
        norm[h] = VARIANT == 0 ? sqrtf((float)acc) : (float)sqrt(acc);
      }
    }
    bool st16[kQNB];   // row-uniform: bucket h is whole (128 elements), 16-B aligned codes
#pragma unroll
    for (int h = 0; h < kQNB; ++h) {
      const int32_t bbase = e[h][0] - 4 * l16;
      st16[h] = kStage16 && codes16 && ok[h] && (bbase & 15) == 0 && bbase + 128 <= end[h];
    }
#pragma unroll
    for (int h = 0; h < kQNB; ++h) {
      if (!ok[h]) continue;
      if (!FUSED && l16 == 0) norms_out[bb[h]] = norm[h];
      const float scale = VARIANT == 0 ? (1.0f / norm[h]) * qf : qf / norm[h];
      const float dsc = norm[h] / qf;   // the decoder's scale
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int32_t eq = e[h][q];
        float uu[4];
        if (u) {   // parity mode (injected stream): not the fast path
#pragma unroll
          for (int j = 0; j < 4; ++j) uu[j] = eq + j < end[h] ? u[eq + j] : 0.f;
        } else {
#ifdef GRACE_DIAG_NORNG   // diagnostic A/B build only: constant u
          uu[0] = uu[1] = uu[2] = uu[3] = 0.5f + 0.f * (float)key;
#else
          uniform01x4_k(key, (uint32_t)eq + xoff, uu);
#endif
        }
        CodeT c[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float level = VARIANT == 0 ? scale * fabsf(v[h][q][j]) : qf / norm[h] * fabsf(v[h][q][j]);
          c[j] = qsgd_code<CodeT, VARIANT>(v[h][q][j], level, uu[j], norm[h]);
        }
        if constexpr (FUSED) {
          float o[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float cf = (float)c[j];
            float d = dsc * cf;
            if (VARIANT == 1 && cf == -128.0f) d = __int_as_float(0x7FC00000);
            o[j] = 0.f + d;
          }
          if (fast[h][q]) {
            __builtin_nontemporal_store(f4v{o[0], o[1], o[2], o[3]}, reinterpret_cast<f4v*>(fused_out + eq));
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (eq + j < end[h]) fused_out[eq + j] = o[j];
          }
        } else if (kStage16 && st16[h]) {
          cst[threadIdx.x >> 4][h * 32 + q * 16 + l16] =
              (uint32_t)(uint8_t)c[0] | ((uint32_t)(uint8_t)c[1] << 8) | ((uint32_t)(uint8_t)c[2] << 16) |
              ((uint32_t)(uint8_t)c[3] << 24);
        } else {
#ifdef GRACE_DIAG_NOSTORE   // diagnostic A/B build only: no code stores (a never-true runtime guard)
          if (norm[h] < 0.f)
#endif
          store_codes4(codes, eq, end[h], fast[h][q], c);
        }
      }
    }
    if constexpr (kStage16) {
      // the row's staged buckets: lane l16 stores bytes [16 (l16 % 8), +16) of bucket l16 / 8 (same
      // wave wrote them: LDS keeps the wave's order, no barrier)
#pragma unroll
      for (int h0 = 0; h0 < kQNB; h0 += 2) {
        const int h = h0 + (l16 >> 3);
        if (h < kQNB && ok[h] && st16[h]) {
          const uint4 wv = *reinterpret_cast<const uint4*>(&cst[threadIdx.x >> 4][h * 32 + 4 * (l16 & 7)]);
#ifdef GRACE_DIAG_NOSTORE
          if (norm[h] < 0.f)
#endif
          *reinterpret_cast<uint4*>(codes + (e[h][0] - 4 * l16) + 16 * (l16 & 7)) = wv;
        }
      }
    }
  }
}

// The device-generator fast path of qsgd_encode128_kernel (no injected u, no injected norms): the
// same codes and norms bit for bit (tests/test_gpu_quant.py feeds the injected-stream kernel the
// generator's uniforms, tests/device_rng.py).  Per element the non-pipelined kernel spent ~38 VALU
// instructions (SQ_INSTS_VALU): the kernel is issue-bound, its 128 MB moving at 3.5 TB/s against
// the 5.5 TB/s the same read-4-B / write-1-B mix streams at (grace_hbm_probe variants 6-9: 20.8 us).
// What this kernel removes:
//  * the per-stage segment walk: each workgroup tabulates its buckets' base offsets in LDS once;
//  * f2i16_x86's NaN / range selects on the int8 path: with a finite norm and scale every level is
//    <= q (1 + 3 eps), so the code is the low byte of the exact integer (rows with a non-finite
//    scale take qsgd_code);
//  * half the bucket scalar work: even lanes of a row compute bucket 0's correctly rounded sqrt and
//    divisions, odd lanes bucket 1's, and quad_perm DPP moves hand every lane both;
//  * the index multiply of the generator (formed once per bucket).
// Software pipelined as well: a row owns buckets row, row + 16, ... of the workgroup's range, kQNB
// per stage, and stage i + 1's loads are issued before stage i is reduced, encoded and stored.
// Every load is unconditional (a stage past the range loads x[0..3] and is discarded), so hipcc never
// has to assume a skipped load and wait vmcnt(0) for the prefetched stage.  Buckets that are not
// whole, 16-B aligned 128-element blocks (a segment's partial last bucket, unaligned segments) are
// skipped by the pipeline and encoded afterwards by their row with per-element loads.
// ResNet-50 set (25.5 M elements, 199,672 buckets): 36.7 -> 34.2 us.
#ifndef GRACE_QENC_PIPE
#define GRACE_QENC_PIPE 1
#endif
#ifndef GRACE_QENC_PIPE_GRID
#define GRACE_QENC_PIPE_GRID 4096   // A/B on the ResNet-50 set: 1024 35.6, 2048 34.6, 4096 34.2 us
#endif
constexpr int kQEncPipeGridCap = GRACE_QENC_PIPE_GRID;
#ifndef GRACE_QENC_PIPE_FUSED
#define GRACE_QENC_PIPE_FUSED 0
#endif
constexpr int kQBkMax = 1024;   // buckets per workgroup of the pipelined encoder (its LDS table)
#ifndef GRACE_QENC_NT
#define GRACE_QENC_NT 1
#endif

template <typename CodeT, int VARIANT, bool FUSED>
struct QsgdPipe {
  static constexpr bool kStage16 = !FUSED && sizeof(CodeT) == 1;
  static constexpr int kRows = kQBlock / 16;
  struct Tile {
    f4v v[kQNB][2];
    int32_t base[kQNB], bb[kQNB];
    bool full[kQNB];
  };

  // uniform01x4_k with i * 0x9E3779B1 supplied (the kernel forms it from a per-bucket product)
  __device__ static __forceinline__ void uniform4(uint32_t ic, uint32_t klo, uint32_t khi, float (&u)[4]) {
    uint32_t h = fmix32((ic ^ klo) + khi);
    u[0] = (float)(h >> 8) * (1.0f / 16777216.0f);
    h = h ? h : 0x9E3779B9u;
#pragma unroll
    for (int j = 1; j < 4; ++j) {
      h ^= h << 13;
      h ^= h >> 17;
      h ^= h << 5;
      u[j] = (float)(h >> 8) * (1.0f / 16777216.0f);
    }
  }

  __device__ static __forceinline__ float bucket_norm(double acc) {
    acc = row16_sum(acc);
    return VARIANT == 0 ? sqrtf((float)acc) : (float)sqrt(acc);
  }

  __device__ static __forceinline__ double sq_acc(const float (&v)[4], double acc) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (VARIANT == 0 || isfinite(v[j])) acc = fma((double)v[j], (double)v[j], acc);
    return acc;
  }
};

template <typename CodeT, int VARIANT, bool FUSED = false>
__global__ __launch_bounds__(kQBlock) void qsgd_encode128_pipe_kernel(
    const float* __restrict__ x, const int64_t* __restrict__ seg_off, const int64_t* __restrict__ bkt_off,
    int nseg, int32_t nbuckets, float qf, uint64_t seed, float* __restrict__ norms_out,
    CodeT* __restrict__ codes, float* __restrict__ fused_out) {
  using P = QsgdPipe<CodeT, VARIANT, FUSED>;
  using Tile = typename P::Tile;
  constexpr int kRows = P::kRows;
  constexpr int kStride = kQNB * kRows;
  constexpr bool kStage16 = P::kStage16;
  constexpr bool kI8 = VARIANT == 0 && sizeof(CodeT) == 1;
  constexpr uint32_t kC = 0x9E3779B1u;
  __shared__ SegTables32 tab;
  __shared__ uint32_t cst[kStage16 ? kRows : 1][kQNB * 32];
  // the workgroup's buckets: base element offset, bit 31 set when not a whole 16-B-aligned bucket
  // (one binary search per bucket here instead of a segment walk in every stage)
  __shared__ int32_t bkt[kQBkMax];
  stage_tables32(tab, seg_off, bkt_off, nseg);
  const bool codes16 = (reinterpret_cast<uintptr_t>(codes) & 15) == 0;
  const int l16 = threadIdx.x & 15;
  const int row = threadIdx.x >> 4;
  const bool odd = (l16 & 1) != 0;
  const uint64_t key = mix64(seed);
  const uint32_t klo = (uint32_t)key, khi = (uint32_t)(key >> 32);
  const uint32_t lane_c = (uint32_t)(4 * l16) * kC;
  int32_t blo, bhi;
  block_range32(nbuckets, kRows, blo, bhi);
  const int32_t nbk = bhi - blo;   // <= kQBkMax (host grid)
  if (nbk <= 0) return;
  for (int32_t j = threadIdx.x; j < nbk; j += kQBlock) {
    const int32_t b = blo + j;
    const int sj = find_seg32(tab.sub, nseg, b);
    const int32_t base = tab.seg[sj] + (b - tab.sub[sj]) * 128;
    const bool full = (base & 3) == 0 && base + 128 <= tab.seg[sj + 1];
    bkt[j] = full ? base : (int32_t)((uint32_t)base | 0x80000000u);
  }
  __syncthreads();

  auto issue = [&](int32_t j0, Tile& T) {   // j0: the stage's first bucket, relative to blo
#pragma unroll
    for (int h = 0; h < kQNB; ++h) {
      const int32_t j = j0 + row + h * kRows;
      const bool ok = j < nbk;
      const int32_t ent = bkt[ok ? j : 0];
      const bool full = ok && ent >= 0;
      const int32_t base = ent & 0x7FFFFFFF;
      T.bb[h] = blo + j;
      T.base[h] = base;
      T.full[h] = full;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        int32_t e = full ? base + 4 * l16 + 64 * q : 0;
        asm volatile("" : "+v"(e));   // opaque: hipcc would otherwise split the load into a branch
#if GRACE_QENC_NT
        T.v[h][q] = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(x + e));
#else
        T.v[h][q] = *reinterpret_cast<const f4v*>(x + e);
#endif
      }
    }
  };

  auto encode = [&](Tile& T) {
    double acc[kQNB];
#pragma unroll
    for (int h = 0; h < kQNB; ++h) {   // all 16 lanes of every row take part in the row reductions
      acc[h] = 0.0;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const float v4[4] = {T.v[h][q][0], T.v[h][q][1], T.v[h][q][2], T.v[h][q][3]};
#ifdef GRACE_DIAG_NONORM   // diagnostic A/B build only: no bucket reduction
        acc[h] += (double)v4[0];
#else
        acc[h] = P::sq_acc(v4, acc[h]);
#endif
      }
      acc[h] = row16_sum(acc[h]);
    }
    // bucket scalars: norm, scale (level = scale |x|, the same expression as qsgd_code's callers)
    // and the decoder's norm / q.  With two buckets a stage, the even lanes of a row compute bucket
    // 0's and the odd lanes bucket 1's (one correctly rounded sqrt and divisions per lane instead of
    // two), then quad_perm DPP moves hand each lane both.
    float norm[kQNB], scale[kQNB], dsc[kQNB];
    auto scalars = [&](double a, float& nm, float& sc, float& ds) {
      nm = VARIANT == 0 ? sqrtf((float)a) : (float)sqrt(a);
      sc = VARIANT == 0 ? (1.0f / nm) * qf : qf / nm;
      ds = nm / qf;
    };
    if constexpr (kQNB == 2) {
      float nm, sc, ds;
      scalars(odd ? acc[1] : acc[0], nm, sc, ds);
      auto even = [](float v) {   // quad_perm [0,0,2,2]
        return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xA0, 0xF, 0xF, false));
      };
      auto oddl = [](float v) {   // quad_perm [1,1,3,3]
        return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xF5, 0xF, 0xF, false));
      };
      norm[0] = even(nm); norm[1] = oddl(nm);
      scale[0] = even(sc); scale[1] = oddl(sc);
      if constexpr (FUSED) { dsc[0] = even(ds); dsc[1] = oddl(ds); }
      if (!FUSED && l16 < 2) {   // lane h of the row stores bucket h's norm
        const bool f = odd ? T.full[1] : T.full[0];
        if (f) norms_out[odd ? T.bb[1] : T.bb[0]] = nm;
      }
    } else {
#pragma unroll
      for (int h = 0; h < kQNB; ++h) {
        scalars(acc[h], norm[h], scale[h], dsc[h]);
        if (!FUSED && l16 == 0 && T.full[h]) norms_out[T.bb[h]] = norm[h];
      }
    }
#ifdef GRACE_DIAG_NONORM
#pragma unroll
    for (int h = 0; h < kQNB; ++h) { norm[h] = (float)acc[h] + 1.f; scale[h] = qf / norm[h]; dsc[h] = norm[h] / qf; }
#endif
#pragma unroll
    for (int h = 0; h < kQNB; ++h) {
      if (!T.full[h]) continue;   // row-uniform
      const int32_t base = T.base[h];
      const bool st16 = kStage16 && codes16 && (base & 15) == 0;
      const bool fin = scale[h] < __builtin_inff() && norm[h] < __builtin_inff();   // row-uniform
      const uint32_t bc = (uint32_t)base * kC + lane_c;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int32_t eq = base + 4 * l16 + 64 * q;
        float uu[4];
#ifdef GRACE_DIAG_NORNG   // diagnostic A/B build only: constant u
        uu[0] = uu[1] = uu[2] = uu[3] = 0.5f + 0.f * (float)bc;
#else
        P::uniform4(bc + (uint32_t)(64 * q) * kC, klo, khi, uu);
#endif
        CodeT c[4];
        uint32_t cw = 0;   // the int8 codes packed (kI8)
        float cf[4];       // the codes as floats (FUSED)
        if (kI8 && fin) {
          // qsgd_code<int8, 0> for a finite norm and scale: then every x is finite and
          // level <= q (1 + 3 eps), so f2i16_x86's NaN / range test never fires and the codeword
          // is the low byte of the exact integer copysign(nl, x)
          int32_t ni[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float xv = T.v[h][q][j];
            const float level = scale[h] * fabsf(xv);
            const float prev = floorf(level);
            const float nl = uu[j] < level - prev ? prev + 1.0f : prev;
            ni[j] = (int32_t)copysignf(nl, xv);
            cf[j] = (float)(int8_t)ni[j];
          }
          cw = __builtin_amdgcn_perm(__builtin_amdgcn_perm((uint32_t)ni[3], (uint32_t)ni[2], 0x0c0c0400u),
                                     __builtin_amdgcn_perm((uint32_t)ni[1], (uint32_t)ni[0], 0x0c0c0400u),
                                     0x05040100u);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float xv = T.v[h][q][j];
            const float level = scale[h] * fabsf(xv);   // VARIANT 1: scale = q / norm
            c[j] = qsgd_code<CodeT, VARIANT>(xv, level, uu[j], norm[h]);
            cf[j] = (float)c[j];
          }
          if constexpr (sizeof(CodeT) == 1)
            cw = (uint32_t)(uint8_t)c[0] | ((uint32_t)(uint8_t)c[1] << 8) | ((uint32_t)(uint8_t)c[2] << 16) |
                 ((uint32_t)(uint8_t)c[3] << 24);
        }
        if constexpr (FUSED) {
          f4v o;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float d = dsc[h] * cf[j];
            if (VARIANT == 1 && cf[j] == -128.0f) d = __int_as_float(0x7FC00000);
            o[j] = 0.f + d;
          }
          __builtin_nontemporal_store(o, reinterpret_cast<f4v*>(fused_out + eq));
        } else if (kStage16 && st16) {
#ifdef GRACE_DIAG_NOSTORE   // diagnostic A/B build only: no code stores (a never-true runtime guard)
          if (norm[h] < 0.f)
#endif
          cst[row][h * 32 + q * 16 + l16] = cw;
        } else if constexpr (sizeof(CodeT) == 1) {
          *reinterpret_cast<uint32_t*>(codes + eq) = cw;
        } else {
          store_codes4(codes, eq, eq + 4, true, c);
        }
      }
    }
    if constexpr (kStage16) {   // the row's staged buckets, 16 B per lane (same wave wrote them)
#pragma unroll
      for (int h0 = 0; h0 < kQNB; h0 += 2) {
        const bool hi = (l16 >> 3) != 0;   // lanes 8..15 store bucket h0 + 1 (selects, not an index)
        const bool has = h0 + 1 < kQNB;
        const bool fl = hi ? (has && T.full[has ? h0 + 1 : h0]) : T.full[h0];
        const int32_t bs = hi ? T.base[has ? h0 + 1 : h0] : T.base[h0];
        if (fl && codes16 && (bs & 15) == 0) {
          const uint4 wv = *reinterpret_cast<const uint4*>(&cst[row][(h0 + (hi ? 1 : 0)) * 32 + 4 * (l16 & 7)]);
#ifdef GRACE_DIAG_NOSTORE
          if (wv.x == 0x12345678u && wv.y == 0x9abcdef0u)
#endif
          *reinterpret_cast<uint4*>(codes + bs + 16 * (l16 & 7)) = wv;
        }
      }
    }
  };

  // block-uniform trip count; two tiles used alternately (static registers, no copies)
  Tile A, B;
  issue(0, A);
  for (int32_t j0 = 0; j0 < nbk; j0 += 2 * kStride) {
    issue(j0 + kStride, B);
    encode(A);
    issue(j0 + 2 * kStride, A);
    encode(B);
  }

  // the buckets the pipeline skipped: partial or unaligned, per-element loads (no prefetch pending)
  for (int32_t j = row; j < nbk; j += kRows) {
    if (bkt[j] >= 0) continue;   // row-uniform: done by the pipeline
    const int32_t bb = blo + j;
    const int sj = find_seg32(tab.sub, nseg, bb);
    const int32_t base = tab.seg[sj] + (bb - tab.sub[sj]) * 128;
    const int32_t end = min(base + 128, tab.seg[sj + 1]);
    float v[2][4];
    double acc = 0.0;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int32_t eq = base + 4 * l16 + 64 * q;
#pragma unroll
      for (int j = 0; j < 4; ++j) v[q][j] = eq + j < end ? x[eq + j] : 0.f;
      acc = P::sq_acc(v[q], acc);
    }
    const float norm = P::bucket_norm(acc);
    if (!FUSED && l16 == 0) norms_out[bb] = norm;
    const float scale = VARIANT == 0 ? (1.0f / norm) * qf : qf / norm;
    const float dsc = norm / qf;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int32_t eq = base + 4 * l16 + 64 * q;
      float uu[4];
      P::uniform4((uint32_t)eq * kC, klo, khi, uu);
      CodeT c[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float level = VARIANT == 0 ? scale * fabsf(v[q][j]) : qf / norm * fabsf(v[q][j]);
        c[j] = qsgd_code<CodeT, VARIANT>(v[q][j], level, uu[j], norm);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (eq + j >= end) continue;
        if constexpr (FUSED) {
          const float cf = (float)c[j];
          float d = dsc * cf;
          if (VARIANT == 1 && cf == -128.0f) d = __int_as_float(0x7FC00000);
          fused_out[eq + j] = 0.f + d;
        } else {
          codes[eq + j] = c[j];
        }
      }
    }
  }
}

template <typename CodeT, int VARIANT>
__global__ __launch_bounds__(kQBlock) void qsgd_encode_kernel(
    const float* __restrict__ x, const int64_t* __restrict__ seg_off, const int64_t* __restrict__ bkt_off,
    int nseg, int64_t nbuckets, int bucket, float qf, const float* __restrict__ u, uint64_t seed,
    const float* __restrict__ norms_in, float* __restrict__ norms_out, CodeT* __restrict__ codes, int64_t xoff = 0) {
  __shared__ SegTables tab;
  const SegView sv = stage_tables(tab, seg_off, bkt_off, nseg);
  const int l32 = threadIdx.x & 31;
  constexpr int kHalves = kQBlock / 32;
  int64_t blo, bhi;
  block_range(nbuckets, kHalves, blo, bhi);
  const int64_t b_first = blo + (threadIdx.x >> 5);
  int s = b_first < bhi ? find_seg(sv.sub, nseg, b_first) : 0;
  if (bucket <= 128) {
    // kQNB buckets per half-wave per iteration: every 16-B load is in flight before any bucket
    // reduces, and the kQNB shuffle reductions interleave
    for (int64_t b = b_first; b < bhi; b += kQNB * kHalves) {
      int64_t bb[kQNB], base[kQNB], end[kQNB];
      bool ok[kQNB], aligned[kQNB];
      float v[kQNB][4];
#pragma unroll
      for (int h = 0; h < kQNB; ++h) {
        bb[h] = b + h * kHalves;
        ok[h] = bb[h] < bhi;
        if (ok[h]) s = seg_advance(sv.sub, nseg, s, bb[h]);
        base[h] = sv.seg[s] + (bb[h] - sv.sub[s]) * bucket;
        end[h] = ok[h] ? min(base[h] + (int64_t)bucket, sv.seg[s + 1]) : base[h];
        aligned[h] = (base[h] & 3) == 0;
        load_quad(x, base[h] + 4 * l32, end[h], aligned[h], v[h]);
      }
      float norm[kQNB];
      if (norms_in) {
#pragma unroll
        for (int h = 0; h < kQNB; ++h) norm[h] = ok[h] ? norms_in[bb[h]] : 1.f;
      } else {
        double acc[kQNB];
#pragma unroll
        for (int h = 0; h < kQNB; ++h) {
          acc[h] = 0.0;
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (VARIANT == 0 || isfinite(v[h][j])) acc[h] += (double)v[h][j] * (double)v[h][j];
        }
#pragma unroll
        for (int o = 16; o > 0; o >>= 1) {
#pragma unroll
          for (int h = 0; h < kQNB; ++h) acc[h] += __shfl_xor(acc[h], o, 64);
        }
#pragma unroll
        for (int h = 0; h < kQNB; ++h) norm[h] = VARIANT == 0 ? sqrtf((float)acc[h]) : (float)sqrt(acc[h]);
      }
#pragma unroll
      for (int h = 0; h < kQNB; ++h) {
        if (!ok[h]) continue;
        const int64_t e = base[h] + 4 * l32;
        if (l32 == 0) norms_out[bb[h]] = norm[h];
        const float scale = VARIANT == 0 ? (1.0f / norm[h]) * qf : qf / norm[h];
        float uu[4];
        if (u) load_quad(u, e, end[h], aligned[h], uu);
        else uniform01x4(seed, (uint64_t)(e + xoff), uu);
        CodeT c[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float level = VARIANT == 0 ? scale * fabsf(v[h][j]) : qf / norm[h] * fabsf(v[h][j]);
          c[j] = qsgd_code<CodeT, VARIANT>(v[h][j], level, uu[j], norm[h]);
        }
        store_codes4(codes, e, end[h], aligned[h], c);
      }
    }
    return;
  }
  for (int64_t b = b_first; b < bhi; b += kHalves) {
    s = seg_advance(sv.sub, nseg, s, b);
    const int64_t base = sv.seg[s] + (b - sv.sub[s]) * bucket;
    const int64_t end = min(base + (int64_t)bucket, sv.seg[s + 1]);
    float norm;
    if (norms_in) {
      norm = norms_in[b];
    } else {
      double acc = 0.0;
      for (int64_t i = base + l32; i < end; i += 32) {
        const float v = x[i];
        if (VARIANT == 0 || isfinite(v)) acc += (double)v * (double)v;
      }
      acc = half_sum(acc);
      norm = VARIANT == 0 ? sqrtf((float)acc) : (float)sqrt(acc);
    }
    if (l32 == 0) norms_out[b] = norm;
    const float scale = VARIANT == 0 ? (1.0f / norm) * qf : qf / norm;
    for (int64_t i = base + l32; i < end; i += 32) {
      const float v = x[i];
      const float ui = u ? u[i] : uniform01(seed, (uint64_t)(i + xoff));
      const float level = VARIANT == 0 ? scale * fabsf(v) : qf / norm * fabsf(v);
      codes[i] = qsgd_code<CodeT, VARIANT>(v, level, ui, norm);
    }
  }
}

// 4 codes of one rank at p[0 .. 3] as floats (vec: one 4-B / 8-B load)
template <typename CodeT>
__device__ __forceinline__ void load_codes4(const CodeT* __restrict__ p, bool vec, float (&c)[4]) {
  if constexpr (sizeof(CodeT) == 1) {
    uint32_t wd;
    if (vec) wd = *reinterpret_cast<const uint32_t*>(p);
    else wd = (uint32_t)(uint8_t)p[0] | ((uint32_t)(uint8_t)p[1] << 8) | ((uint32_t)(uint8_t)p[2] << 16) |
              ((uint32_t)(uint8_t)p[3] << 24);
#pragma unroll
    for (int j = 0; j < 4; ++j) c[j] = (float)(int8_t)(wd >> (8 * j));
  } else {
    uint2 wd;
    if (vec) {
      wd = *reinterpret_cast<const uint2*>(p);
    } else {
      wd.x = (uint32_t)__half_as_ushort(p[0]) | ((uint32_t)__half_as_ushort(p[1]) << 16);
      wd.y = (uint32_t)__half_as_ushort(p[2]) | ((uint32_t)__half_as_ushort(p[3]) << 16);
    }
    c[0] = __half2float(__ushort_as_half((unsigned short)wd.x));
    c[1] = __half2float(__ushort_as_half((unsigned short)(wd.x >> 16)));
    c[2] = __half2float(__ushort_as_half((unsigned short)wd.y));
    c[3] = __half2float(__ushort_as_half((unsigned short)(wd.y >> 16)));
  }
}

template <typename CodeT>
__device__ __forceinline__ float load_code1(const CodeT* __restrict__ p) {
  if constexpr (sizeof(CodeT) == 1) return (float)(int8_t)*p;
  else return __half2float(*p);
}

// Decoders: each workgroup walks a contiguous range in rounds of kDecRound elements; per round a
// thread owns kDecQuads quads spaced one workgroup-width (1024 elements) apart, so every load and
// 16-B store instruction of a wave is contiguous, and all of the round's loads are issued before
// any of its results is needed.  The segment cursor only advances.
constexpr int kDecQuads = 4;
constexpr int64_t kDecRound = (int64_t)kQBlock * 4 * kDecQuads;

// element-wise decode of [i0, i1) (quads that straddle a segment end; kept out of line so the
// fast path's register budget stays small)
template <typename CodeT, int VARIANT, bool B128>
__device__ __attribute__((noinline)) void qsgd_decode_slow(
    const CodeT* __restrict__ codes, const float* __restrict__ norms, int64_t code_stride, int64_t norm_stride,
    int world, const int64_t* seg, const int64_t* sub, int nseg, int64_t i0, int64_t i1, int bucket, float qf,
    float divisor, int aggregate, float* __restrict__ out) {
  for (int64_t i = i0; i < i1; ++i) {
    const int sj = find_seg(seg, nseg, i);
    const uint32_t off = (uint32_t)(i - seg[sj]);
    const int64_t bk = sub[sj] + (B128 ? (off >> 7) : off / (uint32_t)bucket);
    float a = 0.f;
    for (int w = 0; w < world; ++w) {
      const float c = load_code1(codes + w * code_stride + i);
      float d = (norms[w * norm_stride + bk] / qf) * c;
      if (VARIANT == 1 && c == -128.0f) d = __int_as_float(0x7FC00000);
      a = (aggregate || w > 0) ? a + d : d;
    }
    out[i] = divisor == 1.0f ? a : a / divisor;
  }
}

// decode (+ rank-ordered aggregate of W payloads): out = ((0 + d_0) + d_1 ...) / divisor with
// d_w = (norm_w / q) * code_w  (qsgd.py:44-49).  W = 1, divisor = 1 is plain decompress.
template <typename CodeT, int VARIANT, bool B128>
__global__ __launch_bounds__(kQBlock) void qsgd_decode_kernel(
    const CodeT* __restrict__ codes, const float* __restrict__ norms, int64_t code_stride,
    int64_t norm_stride, int world, const int64_t* __restrict__ seg_off,
    const int64_t* __restrict__ bkt_off, int nseg, int64_t n, int bucket, float qf, float divisor,
    int aggregate, int vec, float* __restrict__ out) {
  __shared__ SegTables tab;
  const SegView sv = stage_tables(tab, seg_off, bkt_off, nseg);
  int64_t lo, hi;
  block_range(n, kDecRound, lo, hi);
  int s = lo < hi ? find_seg(sv.seg, nseg, lo + 4 * threadIdx.x < hi ? lo + 4 * threadIdx.x : lo) : 0;
  for (int64_t r0 = lo; r0 < hi; r0 += kDecRound) {
    int64_t e[kDecQuads], b0[kDecQuads];
    int split[kDecQuads];
    bool fast[kDecQuads];
#pragma unroll
    for (int k = 0; k < kDecQuads; ++k) {
      e[k] = r0 + (int64_t)k * kQBlock * 4 + 4 * threadIdx.x;
      const int64_t ec = e[k] < hi ? e[k] : hi - 1;
      s = seg_advance(sv.seg, nseg, s, ec);
      fast[k] = e[k] + 3 < hi && e[k] + 3 < sv.seg[s + 1] && bucket >= 4;
      const uint32_t off = (uint32_t)(ec - sv.seg[s]);
      const uint32_t bo = B128 ? (off >> 7) : off / (uint32_t)bucket;
      const uint32_t in_b = B128 ? (off & 127u) : off - bo * (uint32_t)bucket;
      split[k] = (int)min((uint32_t)bucket - in_b, 4u);
      b0[k] = sv.sub[s] + bo;
    }
    float acc[kDecQuads][4] = {};
    for (int w = 0; w < world; ++w) {
      float c[kDecQuads][4], na[kDecQuads], nb[kDecQuads];
#pragma unroll
      for (int k = 0; k < kDecQuads; ++k) {
        if (fast[k]) {
          load_codes4(codes + w * code_stride + e[k], vec != 0, c[k]);
          na[k] = norms[w * norm_stride + b0[k]];
          nb[k] = split[k] < 4 ? norms[w * norm_stride + b0[k] + 1] : na[k];
        }
      }
#pragma unroll
      for (int k = 0; k < kDecQuads; ++k) {
        if (!fast[k]) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float d = ((j < split[k] ? na[k] : nb[k]) / qf) * c[k][j];
          if (VARIANT == 1 && c[k][j] == -128.0f) d = __int_as_float(0x7FC00000);
          acc[k][j] = (aggregate || w > 0) ? acc[k][j] + d : d;   // Python sum: 0 + d_0 + d_1 ...
        }
      }
    }
#pragma unroll
    for (int k = 0; k < kDecQuads; ++k) {
      if (fast[k]) {
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[k][j] = divisor == 1.0f ? acc[k][j] : acc[k][j] / divisor;
        __builtin_nontemporal_store(f4v{acc[k][0], acc[k][1], acc[k][2], acc[k][3]},
                                    reinterpret_cast<f4v*>(out + e[k]));
      } else {
        qsgd_decode_slow<CodeT, VARIANT, B128>(codes, norms, code_stride, norm_stride, world, sv.seg, sv.sub, nseg,
                                               e[k], min(e[k] + 4, hi), bucket, qf, divisor, aggregate, out);
      }
    }
  }
}

// Bucket-of-128 decode, mirroring the encoder's layout: a 16-lane row owns a bucket (each lane two
// quads), kQNB buckets per row per iteration, every load issued before any is used.  The segment
// walk and the scale norm_w / q (one division) are per bucket and lane-pair of quads instead of
// per quad.  Same arithmetic as qsgd_decode_kernel.
// Sharded records (grace_qsgd_decompress_records, sharded_quant.py): the codes and norms of the
// bucket's buckets [w U, (w + 1) U) sit in rank w's gathered record -- codes from the record's
// start (element rank_lo[w] first), norms from rec_norms floats further -- so bucket b reads
// through rank w = b / U's record.  units == 0: the plain flat layout.
struct QShardRec {
  int64_t units;       // buckets per rank U (0: off)
  int64_t rec_codes;   // record stride in codes
  int64_t rec_norms;   // record stride in floats
  int64_t norm_off;    // the norms' offset inside a record, in floats
  const int64_t* lo;   // rank_lo[w]: the first element of rank w's range
};

template <typename CodeT, int VARIANT>
__global__ __launch_bounds__(kQBlock) void qsgd_decode_bkt_kernel(
    const CodeT* __restrict__ codes, const float* __restrict__ norms, int64_t code_stride,
    int64_t norm_stride, int world, const int64_t* __restrict__ seg_off,
    const int64_t* __restrict__ bkt_off, int nseg, float qf, float divisor, int aggregate, int vec,
    float* __restrict__ out, QShardRec sr = QShardRec{0, 0, 0, 0, nullptr}) {
  __shared__ SegTables32 tab;
  stage_tables32(tab, seg_off, bkt_off, nseg);
  const int l16 = threadIdx.x & 15;
  constexpr int kRows = kQBlock / 16;
  const int32_t nbuckets = tab.sub[nseg];
  int32_t blo, bhi;
  block_range32(nbuckets, kRows, blo, bhi);
  const int32_t b_first = blo + (int32_t)(threadIdx.x >> 4);
  int s = b_first < bhi ? find_seg32(tab.sub, nseg, b_first) : 0;
  for (int32_t b = b_first; b < bhi; b += kQNB * kRows) {
    int32_t bb[kQNB], e[kQNB][2], end[kQNB];
    bool ok[kQNB], full[kQNB][2];
    const CodeT* cp[kQNB];   // codes / norms of bucket bb[h] (a rank's record with sharded records)
    const float* np[kQNB];
#pragma unroll
    for (int h = 0; h < kQNB; ++h) {
      bb[h] = b + h * kRows;
      ok[h] = bb[h] < bhi;
      if (ok[h]) s = seg_advance32(tab.sub, nseg, s, bb[h]);
      const int32_t base = tab.seg[s] + (bb[h] - tab.sub[s]) * 128;
      end[h] = ok[h] ? min(base + 128, tab.seg[s + 1]) : base;
      cp[h] = codes;
      np[h] = norms;
      bool al = true;
      if (sr.units && ok[h]) {
        const int64_t w = bb[h] / sr.units;
        const int64_t lo = sr.lo[w];
        cp[h] = codes + w * sr.rec_codes - lo;
        np[h] = norms + w * sr.rec_norms + sr.norm_off - w * sr.units;
        al = ((base - lo) & 3) == 0;   // the record's codes start at rank_lo[w]
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        e[h][q] = base + 4 * l16 + 64 * q;   // quads l16 and l16 + 16: each instruction covers 256 contiguous bytes per row
        full[h][q] = ok[h] && vec && al && (base & 3) == 0 && e[h][q] + 3 < end[h];
      }
    }
    float acc[kQNB][2][4] = {};
    for (int w = 0; w < world; ++w) {
      float c[kQNB][2][4], nrm[kQNB];
      // unconditional loads first (see qsgd_encode128_kernel), edge quads fixed up after
#pragma unroll
      for (int h = 0; h < kQNB; ++h) {
#pragma unroll
        for (int q = 0; q < 2; ++q)
          load_codes4(full[h][q] ? cp[h] + w * code_stride + e[h][q] : codes, true, c[h][q]);
        nrm[h] = ok[h] ? np[h][w * norm_stride + bb[h]] : norms[0];
      }
#pragma unroll
      for (int h = 0; h < kQNB; ++h) {
#pragma unroll
        for (int q = 0; q < 2; ++q)
          if (ok[h] && !full[h][q]) {
            const CodeT* p = cp[h] + w * code_stride + e[h][q];
#pragma unroll
            for (int j = 0; j < 4; ++j) c[h][q][j] = e[h][q] + j < end[h] ? load_code1(p + j) : 0.f;
          }
        const float sc = nrm[h] / qf;
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float d = sc * c[h][q][j];
            if (VARIANT == 1 && c[h][q][j] == -128.0f) d = __int_as_float(0x7FC00000);
            acc[h][q][j] = (aggregate || w > 0) ? acc[h][q][j] + d : d;   // Python sum: 0 + d_0 + ...
          }
      }
    }
#pragma unroll
    for (int h = 0; h < kQNB; ++h) {
      if (!ok[h]) continue;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        float* a4 = acc[h][q];
        if (divisor != 1.0f) {
#pragma unroll
          for (int j = 0; j < 4; ++j) a4[j] = a4[j] / divisor;
        }
        const int32_t eq = e[h][q];
        if (full[h][q]) {
          __builtin_nontemporal_store(f4v{a4[0], a4[1], a4[2], a4[3]}, reinterpret_cast<f4v*>(out + eq));
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (eq + j < end[h]) out[eq + j] = a4[j];
        }
      }
    }
  }
}

// ================================================================================================
// TernGrad (grace_dl/dist/compressor/terngrad.py:7-30)
//   std    = sqrt(mean((x - mean x)^2))        (here: f64 sums of x and x^2, one read)
//   c      = f32(2.5 * (double)f32(std))       clamp bound as torch rounds the Python double
//   scalar = max |clamp(x, -c, c)| = min(max|x|, c)
//   code   = (u * scalar >= |clamp x|) ? 0 : sign(x)          int8 in {-1, 0, 1}
// Stage 1 writes f64 partials per work unit (16384 elements); stage 2 (encode) reduces its
// segment's partials with the whole workgroup in a fixed order (every unit of a segment derives
// the identical scale), then encodes its unit.  Both stages move 16 B per lane.
// Where the segment scale is reduced (A/B knob): 0 = the last stats unit of each segment to arrive
// (agent-scope partials + arrival ticket), 1 = every encode unit of the segment, from the stats
// kernel's plain partials, at the start of the encode while its first x loads are in flight (the
// stats kernel then has no arrival tail).  Both sum the partials in unit order: identical scales.
#ifndef GRACE_TERN_ENC_REDUCE
#define GRACE_TERN_ENC_REDUCE 1
#endif
constexpr bool kTernEncReduce = GRACE_TERN_ENC_REDUCE != 0;
#ifndef GRACE_TERN_UNIT
#define GRACE_TERN_UNIT 16384   // A/B, ResNet-50 set compress: 4096 / 8192 / 16384 / 32768 -> 64.7 /
#endif                          // 56.5 / 54.0 / 60.6 us (tools/ab_quant.py, one process)
constexpr int kTernUnit = GRACE_TERN_UNIT;

struct TernPartial { double sum, sq; float amax; uint32_t nan; };

// [base, end) split into a scalar head, 16-B aligned quads and a scalar tail
struct QuadSplit {
  int64_t a0, a1;   // aligned quad range [a0, a1), a0 % 4 == a1 % 4 == 0
};
__device__ __forceinline__ QuadSplit quad_split(int64_t base, int64_t end) {
  int64_t a0 = (base + 3) & ~(int64_t)3;
  if (a0 > end) a0 = end;
  int64_t a1 = end & ~(int64_t)3;
  if (a1 < a0) a1 = a0;
  return QuadSplit{a0, a1};
}
// the same with quads at the indices congruent to ph mod 4 (a shard whose element xoff sits at its
// 16-B aligned start: ph = xoff & 3)
__device__ __forceinline__ QuadSplit quad_split_ph(int64_t base, int64_t end, int64_t ph) {
  int64_t a0 = base + ((ph - base) & 3);
  if (a0 > end) a0 = end;
  int64_t a1 = end - ((end - ph) & 3);
  if (a1 < a0) a1 = a0;
  return QuadSplit{a0, a1};
}

__device__ __forceinline__ void tern_acc(float v, double& sum, double& sq, float& amax, uint32_t& nan) {
  sum += (double)v;
  sq += (double)v * (double)v;
  if (v != v) nan = 1; else amax = fmaxf(amax, fabsf(v));
}

// workgroup reduction of a TernPartial in a fixed order (deterministic)
template <int BLOCK = kQBlock>
__device__ __forceinline__ TernPartial block_tern_reduce(double sum, double sq, float amax, uint32_t nan) {
  __shared__ double sh_s[BLOCK / kWave], sh_q[BLOCK / kWave];
  __shared__ float sh_m[BLOCK / kWave];
  __shared__ uint32_t sh_n[BLOCK / kWave];
  sum = wave_sum(sum);
  sq = wave_sum(sq);
  amax = wave_max(amax);
  nan = __ballot(nan != 0) != 0;
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { sh_s[w] = sum; sh_q[w] = sq; sh_m[w] = amax; sh_n[w] = nan; }
  __syncthreads();
  TernPartial p{0.0, 0.0, 0.f, 0u};
  for (int j = 0; j < BLOCK / kWave; ++j) {
    p.sum += sh_s[j]; p.sq += sh_q[j]; p.amax = fmaxf(p.amax, sh_m[j]); p.nan |= sh_n[j];
  }
  return p;
}

// per-segment scale slot, kept at the segment's first unit (empty segments have none)
struct TernScale { float c, scalar; };

// Per-unit workspace slot, an array of structs indexed by unit: a unit's counter sits at the same
// address whatever nunits a call uses and no call's partials overlap another call's counters, so one
// zero-initialised buffer serves calls of any shape (each segment's last unit leaves its counter
// zeroed).  A struct-of-arrays layout sized by nunits let a smaller call's partials land on a larger
// call's counters.
struct TernSlot {
  TernPartial part;    // the unit's partial (agent-scope stores)
  TernScale scale;     // the segment's (c, scalar), at its first unit
  uint32_t tick, pad;  // arrivals, at the segment's first unit
};
static_assert(sizeof(TernSlot) == 40, "TernSlot layout");
__host__ __device__ inline size_t tern_ws_bytes(int64_t nunits) { return sizeof(TernSlot) * (size_t)(nunits + 1); }

// Stage 1: per-unit f64 partials; the LAST unit of a segment to arrive reduces the segment's
// partials in a fixed order (the same block reduction whichever unit it is, so the scale is
// deterministic) and publishes (c, scalar) for stage 2.  Partials cross workgroups -- and XCDs,
// whose L2s are not coherent -- so they are written and read back at agent scope (write-through),
// ordered by vmcnt(0) before the arrival ticket: no cache-wide fences.
// unit0 / xoff (sharded TernGrad, grace_terngrad_shard_*): this launch runs the global units unit0,
// unit0 + 1, ... and x points at global element xoff (its shard); 0 / 0 for a whole bucket
__global__ __launch_bounds__(kQBlock) void tern_stats_kernel(const float* __restrict__ x,
                                                            const int64_t* __restrict__ seg_off,
                                                            const int64_t* __restrict__ unit_off, int nseg,
                                                            const float* __restrict__ clip_in, TernSlot* __restrict__ w,
                                                            float* __restrict__ scalars, int64_t unit0 = 0,
                                                            int64_t xoff = 0) {
  __shared__ SegTables tab;
  __shared__ uint32_t s_last;
  const SegView sv = stage_tables(tab, seg_off, unit_off, nseg);
  const int64_t unit = unit0 + blockIdx.x;
  const int s = find_seg(sv.sub, nseg, unit);
  const int64_t base = sv.seg[s] + (unit - sv.sub[s]) * kTernUnit;
  const int64_t end = min(base + (int64_t)kTernUnit, sv.seg[s + 1]);
  const QuadSplit qs = quad_split_ph(base, end, xoff & 3);
  x -= xoff;   // indexed by global element from here on (never below xoff)
  double sum = 0.0, sq = 0.0;
  float amax = 0.f;
  uint32_t nan = 0;
  const int t = threadIdx.x;
  if (base + t < qs.a0) tern_acc(x[base + t], sum, sq, amax, nan);
  if (qs.a1 + t < end) tern_acc(x[qs.a1 + t], sum, sq, amax, nan);
  const f4v* xq = reinterpret_cast<const f4v*>(x + qs.a0);
  const int64_t nq = (qs.a1 - qs.a0) >> 2;
#pragma unroll 4
  for (int64_t j = t; j < nq; j += kQBlock) {
    const f4v v = xq[j];   // a plain load (allocates in the caches): the encoder re-reads x (A/B: -4 %)
    tern_acc(v.x, sum, sq, amax, nan);
    tern_acc(v.y, sum, sq, amax, nan);
    tern_acc(v.z, sum, sq, amax, nan);
    tern_acc(v.w, sum, sq, amax, nan);
  }
  const TernPartial p = block_tern_reduce(sum, sq, amax, nan);
  uint64_t* pw = reinterpret_cast<uint64_t*>(&w[unit].part);
  if constexpr (kTernEncReduce) {
    // the encode kernel reduces the segment's partials itself (next launch: plain stores suffice)
    if (t == 0) w[unit].part = p;
    return;
  }
  if (t == 0) {
    __hip_atomic_store(pw, (uint64_t)__double_as_longlong(p.sum), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(pw + 1, (uint64_t)__double_as_longlong(p.sq), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(pw + 2, (uint64_t)__float_as_uint(p.amax) | ((uint64_t)p.nan << 32), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int64_t first = sv.sub[s], units = sv.sub[s + 1] - first;
    s_last = atomicAdd(&w[first].tick, 1u) == (uint32_t)(units - 1);
  }
  __syncthreads();
  if (!s_last) return;
  // last arrival: the segment's statistics from its units' partials, in a fixed order
  const int64_t first = sv.sub[s];
  sum = 0.0; sq = 0.0; amax = 0.f; nan = 0;
  for (int64_t j = first + t; j < sv.sub[s + 1]; j += kQBlock) {
    const uint64_t* pj = reinterpret_cast<const uint64_t*>(&w[j].part);
    sum += __longlong_as_double((long long)__hip_atomic_load(pj, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    sq += __longlong_as_double((long long)__hip_atomic_load(pj + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    const uint64_t mn = __hip_atomic_load(pj + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    amax = fmaxf(amax, __uint_as_float((uint32_t)mn));
    nan |= (uint32_t)(mn >> 32);
  }
  const TernPartial q = block_tern_reduce(sum, sq, amax, nan);
  if (t == 0) {
    float c;
    if (clip_in) {
      c = clip_in[s];
    } else {
      const double nn = (double)(sv.seg[s + 1] - sv.seg[s]);
      const double mean = q.sum / nn;
      double var = q.sq / nn - mean * mean;
      if (var < 0.0) var = 0.0;
      c = (float)(2.5 * (double)(float)sqrt(var));
    }
    // torch.clamp propagates a NaN bound (an injected NaN clip, or std = NaN when x holds an inf):
    // every clamped element and the scalar are then NaN, as for a NaN element
    const float scalar = (q.nan || c != c) ? __int_as_float(0x7FC00000) : fminf(q.amax, c);
    w[first].scale = TernScale{c, scalar};
    scalars[s] = scalar;
    w[first].tick = 0u;   // left zeroed for the next call
  }
}

#ifndef GRACE_TERN_BLOCK
#define GRACE_TERN_BLOCK 256
#endif
constexpr int kTernBlock = GRACE_TERN_BLOCK;
#ifndef GRACE_TERN_SUB
#define GRACE_TERN_SUB 4
#endif   // encode workgroup (A/B: 256 beats 512 and 1024)

// FUSED: the world-1 Allgather step in the same pass -- out = 0 + code * scalar (the decoder's
// arithmetic, division by 1 omitted) written instead of the codes: bit-identical to encode + decode.
// HAS_U: an injected uniform stream (parity tests); a separate instantiation, so the device-
// generator path has no load under a branch (hipcc would wait vmcnt(0) at the join, i.e. also for
// the prefetched next sub-chunk)
template <bool FUSED = false, bool HAS_U = false>
__global__ __launch_bounds__(kTernBlock) void tern_encode_kernel(
    const float* __restrict__ x, const int64_t* __restrict__ seg_off, const int64_t* __restrict__ unit_off,
    int nseg, const TernSlot* __restrict__ w, const float* __restrict__ u, uint64_t seed,
    int8_t* __restrict__ codes, float* __restrict__ out, const float* __restrict__ clip_in,
    float* __restrict__ scalars, int64_t unit0 = 0, int64_t xoff = 0) {
  __shared__ SegTables tab;
  const SegView sv = stage_tables(tab, seg_off, unit_off, nseg);
  const int64_t unit = unit0 + blockIdx.x;
  const int s = find_seg(sv.sub, nseg, unit);
  const int64_t base = sv.seg[s] + (unit - sv.sub[s]) * kTernUnit;
  const int64_t end = min(base + (int64_t)kTernUnit, sv.seg[s + 1]);
  const QuadSplit qs = quad_split_ph(base, end, xoff & 3);
  // x, u, codes and out hold the elements from global xoff on (a shard); indexed globally below
  x -= xoff;
  if constexpr (HAS_U) u -= xoff;
  if constexpr (FUSED) out -= xoff;
  else codes -= xoff;
  const int t = threadIdx.x;
  const int64_t nq = (qs.a1 - qs.a0) >> 2;
  // The unit's quads in kTernSteps sub-chunks of kTernSub per thread, software pipelined: the next
  // sub-chunk's loads are issued before the current one is encoded and stored.  (All 1560 units of
  // the ResNet-50 set are co-resident, so loading the whole unit first made the chip load, then
  // compute, then store in lockstep, with HBM idle in between.)
  constexpr int kPer = kTernUnit / 4 / kTernBlock;
  constexpr int kTernSub = GRACE_TERN_SUB;
  constexpr int kTernSteps = kPer / kTernSub;
  static_assert(kPer % kTernSub == 0, "sub-chunks tile the unit");
  const f4v* xq = reinterpret_cast<const f4v*>(x + qs.a0);
  auto load_sub = [&](int st, f4v (&dst)[kTernSub]) {
#pragma unroll
    for (int k = 0; k < kTernSub; ++k) {
      const int64_t j = t + (int64_t)(st * kTernSub + k) * kTernBlock;
      // plain (cache-allocating) loads: part of the re-read of x hits the Infinity Cache the
      // statistics pass filled (A/B r04, one box: encode 29.6 us with non-temporal loads, 27.8 us
      // plain; 32.5 us when a 512 MiB write stream between the two passes evicts x first)
#ifdef GRACE_TERN_ENC_NT   // A/B build only: the non-temporal re-read
      if (nq > 0) dst[k] = __builtin_nontemporal_load(xq + (j < nq ? j : 0));
#else
      if (nq > 0) dst[k] = xq[j < nq ? j : 0];
#endif
    }
  };
  f4v cur[kTernSub], nxt[kTernSub];
  load_sub(0, cur);
  float c, scalar;
  if constexpr (kTernEncReduce) {
    // the segment's statistics from its units' partials, in unit order (every unit of the segment
    // computes the identical scale); the first unit publishes the scalar
    double ps = 0.0, pq = 0.0;
    float pm = 0.f;
    uint32_t pn = 0;
    for (int64_t j = sv.sub[s] + t; j < sv.sub[s + 1]; j += kTernBlock) {
      const TernPartial pj = w[j].part;
      ps += pj.sum; pq += pj.sq; pm = fmaxf(pm, pj.amax); pn |= pj.nan;
    }
    const TernPartial q = block_tern_reduce<kTernBlock>(ps, pq, pm, pn);
    if (clip_in) {
      c = clip_in[s];
    } else {
      const double nn = (double)(sv.seg[s + 1] - sv.seg[s]);
      const double mean = q.sum / nn;
      double var = q.sq / nn - mean * mean;
      if (var < 0.0) var = 0.0;
      c = (float)(2.5 * (double)(float)sqrt(var));
    }
    scalar = (q.nan || c != c) ? __int_as_float(0x7FC00000) : fminf(q.amax, c);   // (NaN bound: NaN)
    if (t == 0 && unit == sv.sub[s] && scalars) scalars[s] = scalar;
  } else {
    const TernScale sc = w[sv.sub[s]].scale;   // published by the segment's last stats unit
    c = sc.c;
    scalar = sc.scalar;
  }

  auto enc = [&](float xv, float ui) -> int8_t {
    const float cl = fminf(fmaxf(xv, -c), c);
    const float ab = fabsf(cl);
    const float rnd = ui * scalar;
    int8_t code = 0;
    if (!(rnd >= ab)) {
      const float sg = cl > 0.f ? scalar : (cl < 0.f ? -scalar : 0.f);
      code = sg > 0.f ? 1 : (sg < 0.f ? -1 : 0);
    }
    return code;
  };
  auto put1 = [&](int64_t i, int8_t cd) {
    if constexpr (FUSED) out[i] = 0.f + (float)cd * scalar;
    else codes[i] = cd;
  };
  // The device generator draws a quad's four uniforms at once (uniform01x4 at the GLOBAL quad index,
  // a multiple of 4) and a unit's head / tail elements one by one: so element e's draw depends on
  // the unit's globally aligned split, not on where a shard's quads fall.  u1(e) is that draw; a
  // shard whose quads are out of phase with the global quads (ph != 0) composes each of its quads
  // from the two global quads it straddles.
  const QuadSplit gq = quad_split(base, end);   // the single-GPU encoder's split of this unit
  const int64_t ph = xoff & 3;
  const bool key32 = qs.a1 <= ((int64_t)1 << 32) && gq.a1 <= ((int64_t)1 << 32);
  const uint64_t key = mix64(seed);
  auto quad_u = [&](int64_t q, float (&r4)[4]) {
    if (key32) uniform01x4_k(key, (uint32_t)q, r4);
    else uniform01x4(seed, (uint64_t)q, r4);
  };
  // lane j of a register quad by selects (a dynamic index would put the array in scratch memory)
  auto pick = [](const float (&a)[4], int64_t j) { return j == 0 ? a[0] : (j == 1 ? a[1] : (j == 2 ? a[2] : a[3])); };
  auto u1 = [&](int64_t e) -> float {
    if (e < gq.a0 || e >= gq.a1) return uniform01(seed, (uint64_t)e);
    float r4[4];
    quad_u(e & ~(int64_t)3, r4);
    return pick(r4, e & 3);
  };
  if (base + t < qs.a0) {
    const int64_t i = base + t;
    put1(i, enc(x[i], HAS_U ? u[i] : u1(i)));
  }
  if (qs.a1 + t < end) {
    const int64_t i = qs.a1 + t;
    put1(i, enc(x[i], HAS_U ? u[i] : u1(i)));
  }
  // The quads: the same codes as enc() with fewer instructions.  With s = scalar > 0 (then
  // c >= scalar > 0): enc() is sign(x) where u s < min(|x|, c) and 0 elsewhere (x = +-0 never
  // passes the test; NaN x cannot occur, it makes the scalar NaN).  With scalar 0 or NaN every code
  // is 0: using NaN for the product makes the test fail there too.  The code byte of a selected x is
  // 0x01 or 0xFF from its sign bit.  32-bit quad offsets; the generator key is hoisted
  // (uniform01x4_k = uniform01x4 for element indices below 2^32).
  const float sc_eff = scalar > 0.f ? scalar : __int_as_float(0x7FC00000);
  auto codes4 = [&](const f4v& v, const f4v& uu) -> uint32_t {
    uint32_t cw = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const bool sel = uu[j] * sc_eff < fminf(fabsf(v[j]), c);
      const uint32_t byte = ((uint32_t)((int32_t)__float_as_uint(v[j]) >> 31) | 1u) & 0xFFu;
      cw |= (sel ? byte : 0u) << (8 * j);   // (the shifts fold into v_lshl_or)
    }
    return cw;
  };
  auto encode_quad = [&](int jq, const f4v& v) {
    const int64_t i = qs.a0 + 4 * (int64_t)jq;
    f4v uu;
    if constexpr (HAS_U) {
      uu = *reinterpret_cast<const f4v*>(u + i);
    } else {
      float r4[4];
      if (ph == 0) {   // (the whole-bucket encoder: its quads are the global quads)
        quad_u(i, r4);
      } else {
        float ra[4], rb[4];
        quad_u(i - ph, ra);
        quad_u(i - ph + 4, rb);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int64_t e = i + j;
          const float qv = j < 4 - ph ? pick(ra, (ph + j) & 3) : pick(rb, (j + ph) & 3);
          r4[j] = (e < gq.a0 || e >= gq.a1) ? uniform01(seed, (uint64_t)e) : qv;
        }
      }
      uu = f4v{r4[0], r4[1], r4[2], r4[3]};
    }
    const uint32_t cw = codes4(v, uu);
    if constexpr (FUSED) {
      f4v o;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = 0.f + (float)(int8_t)(uint8_t)(cw >> (8 * j)) * scalar;
      __builtin_nontemporal_store(o, reinterpret_cast<f4v*>(out + i));
    } else {
      *reinterpret_cast<uint32_t*>(codes + i) = cw;
    }
  };
  // two sub-chunk buffers, used alternately in the fully unrolled loop (static registers, no copies)
  const int nqi = (int)nq;
#pragma unroll
  for (int st = 0; st < kTernSteps; ++st) {
    f4v (&curb)[kTernSub] = (st & 1) ? nxt : cur;
    f4v (&nxtb)[kTernSub] = (st & 1) ? cur : nxt;
    if (st + 1 < kTernSteps) load_sub(st + 1, nxtb);
#pragma unroll
    for (int k = 0; k < kTernSub; ++k) {
      const int jq = t + (st * kTernSub + k) * kTernBlock;
      if (jq < nqi) encode_quad(jq, curb[k]);
    }
  }
}

// Every segment's scalar from the per-unit partials in w -- the encoder's reduction verbatim (a
// kTernBlock workgroup, the units in the same thread order, block_tern_reduce), so the scalars are
// bit-identical to the ones the single-GPU encoder publishes.  Sharded TernGrad: every rank derives
// all scalars after the slot all-gather, none travels.
__global__ __launch_bounds__(kTernBlock) void tern_scalars_kernel(const int64_t* __restrict__ seg_off,
                                                                  const int64_t* __restrict__ unit_off,
                                                                  const TernSlot* __restrict__ w,
                                                                  const float* __restrict__ clip_in,
                                                                  float* __restrict__ scalars) {
  const int s = blockIdx.x;
  const int t = threadIdx.x;
  const int64_t u0 = unit_off[s], u1 = unit_off[s + 1];
  if (u0 == u1) return;   // an empty segment has no units (the encoder publishes nothing either)
  double ps = 0.0, pq = 0.0;
  float pm = 0.f;
  uint32_t pn = 0;
  for (int64_t j = u0 + t; j < u1; j += kTernBlock) {
    const TernPartial pj = w[j].part;
    ps += pj.sum; pq += pj.sq; pm = fmaxf(pm, pj.amax); pn |= pj.nan;
  }
  const TernPartial q = block_tern_reduce<kTernBlock>(ps, pq, pm, pn);
  float c;
  if (clip_in) {
    c = clip_in[s];
  } else {
    const double nn = (double)(seg_off[s + 1] - seg_off[s]);
    const double mean = q.sum / nn;
    double var = q.sq / nn - mean * mean;
    if (var < 0.0) var = 0.0;
    c = (float)(2.5 * (double)(float)sqrt(var));
  }
  if (t == 0) scalars[s] = (q.nan || c != c) ? __int_as_float(0x7FC00000) : fminf(q.amax, c);
}

// Row decoder: a 16-lane row owns a 128-element chunk of the flat buffer (each lane the quads l16
// and l16 + 16), kQNB chunks per row per iteration, every load issued before any is used.  A chunk
// inside one segment uses one scalar per rank; the few quads of a chunk that straddles a segment
// boundary are decoded element-wise.  Same arithmetic as tern_decode_kernel.
__global__ __launch_bounds__(kQBlock) void tern_decode_row_kernel(const int8_t* __restrict__ codes,
                                                                 const float* __restrict__ scalars,
                                                                 int64_t code_stride, int64_t scal_stride,
                                                                 int world, const int64_t* __restrict__ seg_off,
                                                                 int nseg, int32_t n, float divisor, int aggregate,
                                                                 int vec, float* __restrict__ out) {
  __shared__ int32_t seg[kSegLds + 1];
  for (int i = threadIdx.x; i <= nseg; i += blockDim.x) seg[i] = (int32_t)seg_off[i];
  __syncthreads();
  const int l16 = threadIdx.x & 15;
  constexpr int kRows = kQBlock / 16;
  const int32_t nchunks = (n + 127) / 128;
  int32_t blo, bhi;
  block_range32(nchunks, kRows, blo, bhi);
  const int32_t c_first = blo + (int32_t)(threadIdx.x >> 4);
  int s = c_first < bhi ? find_seg32(seg, nseg, c_first * 128) : 0;
  for (int32_t c = c_first; c < bhi; c += kQNB * kRows) {
    int32_t e[kQNB][2], ce[kQNB];
    int sidx[kQNB];
    bool ok[kQNB], full[kQNB][2];
#pragma unroll
    for (int h = 0; h < kQNB; ++h) {
      const int32_t cc = c + h * kRows;
      ok[h] = cc < bhi;
      const int32_t i0 = cc * 128;
      if (ok[h]) s = seg_advance32(seg, nseg, s, i0);
      sidx[h] = s;
      ce[h] = ok[h] ? min(i0 + 128, n) : i0;
      const bool uni = seg[s + 1] >= ce[h];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        e[h][q] = i0 + 4 * l16 + 64 * q;
        full[h][q] = ok[h] && uni && vec && e[h][q] + 3 < ce[h];
      }
    }
    float acc[kQNB][2][4] = {};
    for (int w = 0; w < world; ++w) {
      float cv[kQNB][2][4], sc[kQNB];
#pragma unroll
      for (int h = 0; h < kQNB; ++h) {
#pragma unroll
        for (int q = 0; q < 2; ++q)
          load_codes4(codes + (full[h][q] ? w * code_stride + e[h][q] : 0), true, cv[h][q]);
        sc[h] = scalars[w * scal_stride + sidx[h]];
      }
#pragma unroll
      for (int h = 0; h < kQNB; ++h)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          if (full[h][q]) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const float d = cv[h][q][j] * sc[h];
              acc[h][q][j] = (aggregate || w > 0) ? acc[h][q][j] + d : d;
            }
          } else if (ok[h]) {   // chunk edge / segment boundary / unaligned codes: per element
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int32_t i = e[h][q] + j;
              if (i < ce[h]) {
                const int sj = seg_advance32(seg, nseg, sidx[h], i);
                const float d = (float)codes[w * code_stride + i] * scalars[w * scal_stride + sj];
                acc[h][q][j] = (aggregate || w > 0) ? acc[h][q][j] + d : d;
              }
            }
          }
        }
    }
#pragma unroll
    for (int h = 0; h < kQNB; ++h) {
      if (!ok[h]) continue;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        float* a4 = acc[h][q];
        if (divisor != 1.0f) {
#pragma unroll
          for (int j = 0; j < 4; ++j) a4[j] = a4[j] / divisor;
        }
        const int32_t eq = e[h][q];
        if (full[h][q]) {
          __builtin_nontemporal_store(f4v{a4[0], a4[1], a4[2], a4[3]}, reinterpret_cast<f4v*>(out + eq));
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (eq + j < ce[h]) out[eq + j] = a4[j];
        }
      }
    }
  }
}

__device__ __attribute__((noinline)) void tern_decode_slow(const int8_t* __restrict__ codes,
                                                           const float* __restrict__ scalars, int64_t code_stride,
                                                           int64_t scal_stride, int world, const int64_t* seg,
                                                           int nseg, int64_t i0, int64_t i1, float divisor,
                                                           int aggregate, float* __restrict__ out) {
  for (int64_t i = i0; i < i1; ++i) {
    const int sj = find_seg(seg, nseg, i);
    float a = 0.f;
    for (int w = 0; w < world; ++w) {
      const float d = (float)codes[w * code_stride + i] * scalars[w * scal_stride + sj];
      a = (aggregate || w > 0) ? a + d : d;
    }
    out[i] = divisor == 1.0f ? a : a / divisor;
  }
}

__global__ __launch_bounds__(kQBlock) void tern_decode_kernel(const int8_t* __restrict__ codes,
                                                             const float* __restrict__ scalars,
                                                             int64_t code_stride, int64_t scal_stride,
                                                             int world, const int64_t* __restrict__ seg_off,
                                                             int nseg, int64_t n, float divisor, int aggregate,
                                                             int vec, float* __restrict__ out) {
  __shared__ SegTables tab;
  const SegView sv = stage_tables(tab, seg_off, nullptr, nseg);
  int64_t lo, hi;
  block_range(n, kDecRound, lo, hi);
  int s = lo < hi ? find_seg(sv.seg, nseg, lo + 4 * threadIdx.x < hi ? lo + 4 * threadIdx.x : lo) : 0;
  for (int64_t r0 = lo; r0 < hi; r0 += kDecRound) {
    int64_t e[kDecQuads];
    int sk[kDecQuads];
    bool fast[kDecQuads];
#pragma unroll
    for (int k = 0; k < kDecQuads; ++k) {
      e[k] = r0 + (int64_t)k * kQBlock * 4 + 4 * threadIdx.x;
      s = seg_advance(sv.seg, nseg, s, e[k] < hi ? e[k] : hi - 1);
      sk[k] = s;
      fast[k] = e[k] + 3 < hi && e[k] + 3 < sv.seg[s + 1];
    }
    float acc[kDecQuads][4] = {};
    for (int w = 0; w < world; ++w) {
      float c[kDecQuads][4], sc[kDecQuads];
#pragma unroll
      for (int k = 0; k < kDecQuads; ++k) {
        if (fast[k]) {
          load_codes4(codes + w * code_stride + e[k], vec != 0, c[k]);
          sc[k] = scalars[w * scal_stride + sk[k]];
        }
      }
#pragma unroll
      for (int k = 0; k < kDecQuads; ++k) {
        if (!fast[k]) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float d = c[k][j] * sc[k];
          acc[k][j] = (aggregate || w > 0) ? acc[k][j] + d : d;
        }
      }
    }
#pragma unroll
    for (int k = 0; k < kDecQuads; ++k) {
      if (fast[k]) {
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[k][j] = divisor == 1.0f ? acc[k][j] : acc[k][j] / divisor;
        __builtin_nontemporal_store(f4v{acc[k][0], acc[k][1], acc[k][2], acc[k][3]},
                                    reinterpret_cast<f4v*>(out + e[k]));
      } else {
        tern_decode_slow(codes, scalars, code_stride, scal_stride, world, sv.seg, nseg, e[k], min(e[k] + 4, hi),
                         divisor, aggregate, out);
      }
    }
  }
}

// A/B knob (r06): a tile decoder -- one 16-B output quad per lane and QPT quads per lane, i.e. a
// contiguous 4 KB x QPT output tile per workgroup (r05's write probes: a workgroup writing 4 KB runs
// at the box's write rate, 16 KB tiles at 0.87 of it) -- instead of the 16-lane row decoder.  World 1.
// Measured slower (tools/ab_decode.py, ResNet-50 set, one process): row decoder 22.4 us, tiles of
// 4 / 8 / 16 KB 26.6 / 24.1 / 24.2 us (the per-workgroup segment-table staging and search); off.
#ifndef GRACE_TERN_TILE_QPT
#define GRACE_TERN_TILE_QPT 0
#endif
constexpr int kTernTileQpt = GRACE_TERN_TILE_QPT;

template <int QPT>
__global__ __launch_bounds__(kQBlock) void tern_decode_tile_kernel(const int8_t* __restrict__ codes,
                                                                  const float* __restrict__ scalars,
                                                                  const int64_t* __restrict__ seg_off, int nseg,
                                                                  int64_t n, float divisor, int aggregate,
                                                                  float* __restrict__ out) {
  __shared__ int64_t sg[kSegLds + 1];
  for (int i = threadIdx.x; i <= nseg; i += blockDim.x) sg[i] = seg_off[i];
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kQBlock * 4 * QPT + 4 * threadIdx.x;
  uint32_t cw[QPT];
  int sq[QPT];
  bool fast[QPT];
#pragma unroll
  for (int q = 0; q < QPT; ++q) {   // every load issued first, unconditionally (clamped address)
    const int64_t e = base + (int64_t)q * kQBlock * 4;
    sq[q] = find_seg(sg, nseg, e < n ? e : n - 1);
    fast[q] = e + 3 < n && e + 3 < sg[sq[q] + 1];
    cw[q] = *reinterpret_cast<const uint32_t*>(codes + (fast[q] ? e : 0));
  }
#pragma unroll
  for (int q = 0; q < QPT; ++q) {
    const int64_t e = base + (int64_t)q * kQBlock * 4;
    if (e >= n) continue;
    if (fast[q]) {
      const float sc = scalars[sq[q]];
      float a[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float d = (float)(int8_t)((cw[q] >> (8 * j)) & 0xFFu) * sc;
        a[j] = aggregate ? 0.f + d : d;
        if (divisor != 1.0f) a[j] = a[j] / divisor;
      }
      __builtin_nontemporal_store(f4v{a[0], a[1], a[2], a[3]}, reinterpret_cast<f4v*>(out + e));
    } else {
      for (int64_t x = e; x < e + 4 && x < n; ++x) {
        const float d = (float)codes[x] * scalars[find_seg(sg, nseg, x)];
        float v = aggregate ? 0.f + d : d;
        out[x] = divisor == 1.0f ? v : v / divisor;
      }
    }
  }
}

// Sharded TernGrad (grace_amd/dist/sharded_terngrad.py): the whole bucket decoded straight from the
// gathered per-rank records.  Rank w's codes of its elements [rank_lo[w], rank_lo[w + 1]) sit in
// its record at w * rec_bytes, as int8 or (packed) in the 2-bit planar layout of the reference's
// packing (grace_dl/tensorflow/compressor/packing.py:4-29, code + 1: element i of an L-element
// block in byte i % Q at bits 2 (i / Q), Q = grace_pack2_bytes(L)) -- no unpack pass, no copy into
// a flat code buffer.  out = code * scalar, tern_decode_kernel's arithmetic at world 1.
constexpr int kRecRanksMax = 64;

__device__ __forceinline__ float tern_rec_code(const uint8_t* __restrict__ r, uint32_t i, uint32_t L, int packed) {
  if (!packed) return (float)(int8_t)r[i];
  const uint32_t Q = (L + (4u - L % 4u)) / 4u;
  const uint32_t pl = i / Q;
  return (float)((int)((r[i - pl * Q] >> (2u * pl)) & 3u) - 1);
}

__global__ __launch_bounds__(kQBlock) void tern_decode_records_kernel(const uint8_t* __restrict__ rec, int64_t rec_bytes,
                                                                     int world, const int64_t* __restrict__ rank_lo,
                                                                     int packed, const float* __restrict__ scalars,
                                                                     const int64_t* __restrict__ seg_off, int nseg,
                                                                     int64_t n, float* __restrict__ out) {
  __shared__ SegTables tab;
  __shared__ int64_t rlo[kRecRanksMax + 1];
  for (int i = threadIdx.x; i <= world; i += blockDim.x) rlo[i] = rank_lo[i];
  // the segment table in LDS only (nseg <= kSegLds, checked at launch): a SegView may point to global
  // memory, so its reads compile to flat loads with a vmcnt(0) lgkmcnt(0) wait in every table walk
  for (int i = threadIdx.x; i <= nseg; i += blockDim.x) tab.seg[i] = seg_off[i];
  __syncthreads();
  const int64_t* sg = tab.seg;
  // a contiguous range per workgroup, so that a thread's rank and segment only step forward a little
  // (a grid-stride walk jumped over whole segments: a linear segment walk of up to nseg per quad)
  int64_t lo, hi;
  block_range(n, 4 * kQBlock, lo, hi);
  const int64_t e0 = lo + 4 * threadIdx.x;
  int w = 0;
  while (w + 1 < world && rlo[w + 1] <= e0) ++w;
  int s = lo < hi ? find_seg(sg, nseg, e0 < hi ? e0 : lo) : 0;
  // the element's place in its rank's block: plane pl, byte j (packed: i = pl Q + j), advanced
  // incrementally -- one division per rank a thread enters, not one per quad
  int wc = -1;
  uint32_t L = 0, Q = 1, pl = 0, j = 0;
  const uint32_t lim = (uint32_t)min(rec_bytes, (int64_t)0xFFFFFFFF);
  constexpr int kU = 4;   // quads per thread per round: every load issued before any is used
  const uint32_t wlast = lim / 4u - 1u;   // the record's last dword (rec_bytes: a 16-B multiple)
  for (int64_t eb = e0; eb < hi; eb += 4 * kQBlock * kU) {
    uint32_t w0[kU], w1[kU], jb[kU], plu[kU];
    float sc[kU];
    bool fast[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t e = eb + (int64_t)u * 4 * kQBlock;
      const bool in = e < hi;
      if (in) {
        while (w + 1 < world && rlo[w + 1] <= e) ++w;   // e grows: the rank and segment only advance
        s = seg_advance(sg, nseg, s, e);
        const uint32_t i = (uint32_t)(e - rlo[w]);
        if (w != wc) {
          wc = w;
          L = (uint32_t)(rlo[w + 1] - rlo[w]);
          Q = packed ? (L + (4u - L % 4u)) / 4u : 0xFFFFFFFFu;
          pl = packed ? i / Q : 0u;
          j = i - pl * (packed ? Q : 0u);
        } else {
          j = packed ? j + 4u * kQBlock : i;
          while (j >= Q) { j -= Q; ++pl; }
        }
      }
      fast[u] = in && e + 3 < hi && e + 3 < rlo[w + 1] && e + 3 < sg[s + 1] && j + 3u < Q;
      jb[u] = fast[u] ? j : 0u;
      plu[u] = pl;
      // unconditional loads (a load under a branch makes the compiler wait for it at the join):
      // the two dwords holding bytes [j, j + 3] of the rank's record, and the segment's scalar
      const uint32_t* rp = reinterpret_cast<const uint32_t*>(rec + w * rec_bytes);
      w0[u] = rp[jb[u] >> 2];
      w1[u] = rp[min((jb[u] >> 2) + 1u, wlast)];
      sc[u] = scalars[s];
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t e = eb + (int64_t)u * 4 * kQBlock;
      if (e >= hi) continue;
      if (fast[u]) {
        const uint32_t b = __builtin_amdgcn_alignbyte(w1[u], w0[u], jb[u] & 3u);   // bytes j .. j + 3
        float c[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const uint32_t by = (b >> (8 * t)) & 0xFFu;
          c[t] = packed ? (float)((int)((by >> (2u * plu[u])) & 3u) - 1) : (float)(int8_t)by;
        }
        __builtin_nontemporal_store(f4v{c[0] * sc[u], c[1] * sc[u], c[2] * sc[u], c[3] * sc[u]},
                                    reinterpret_cast<f4v*>(out + e));
      } else {
        // the quad crosses the bucket's end, a rank's range, a segment or a plane: element by element
        for (int64_t x = e; x < e + 4 && x < hi; ++x) {
          int wx = 0;
          while (wx + 1 < world && rlo[wx + 1] <= x) ++wx;
          const int sx = find_seg(sg, nseg, x);
          out[x] = tern_rec_code(rec + wx * rec_bytes, (uint32_t)(x - rlo[wx]), (uint32_t)(rlo[wx + 1] - rlo[wx]),
                                 packed) * scalars[sx];
        }
      }
    }
  }
}

// ================================================================================================
// Elementwise byte codecs (natural, cnat, fp16).  Every thread handles quads of 4 consecutive
// elements: one 16-B load of x (and of an injected random stream), one 4-B code store (8-B for
// fp16), grid-stride over the quads; a ragged tail or unaligned views fall back to per-element
// accesses inside the same quad.
__device__ __forceinline__ bool quad_fast(int64_t e, int64_t n, bool aligned) { return aligned && e + 3 < n; }

// natural compression, cupy flavour (grace_dl/dist/compressor/natural.py:12-40): exponent
// rounded up when mantissa > randint(0, 2^23 - 1), clipped to [18, 145], code = sign | (E - 18).
__device__ __forceinline__ uint32_t natural_code(float xv, int32_t r) {
  const int32_t bits = __float_as_int(xv);
  const int32_t sign = bits & (int32_t)0x80000000;
  int32_t e = bits & 0x7F800000;
  const int32_t mant = bits & 0x007FFFFF;
  if (mant > r) e += 0x00800000;
  e = min(max(e, (int32_t)0x09000000), (int32_t)0x48800000);
  return (uint32_t)(uint8_t)((sign >> 24) | ((e >> 23) - 18));
}

// device generator of the natural codec: one rand32 hash per quad plus xorshift32 steps
// (uniform01x4's stream), mapped onto [0, 0x7FFFFF) by a high multiply (the reference's randint
// range; the per-element 64-bit mixes and 64-bit modulo this replaced made the encoder ALU-bound)
__device__ __forceinline__ void natural_rand4(uint64_t seed, int64_t e, int32_t (&r)[4]) {
  uint32_t hq = rand32(seed, (uint64_t)e);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (j) { hq = hq ? hq : 0x9E3779B9u; hq ^= hq << 13; hq ^= hq >> 17; hq ^= hq << 5; }
    r[j] = (int32_t)__umulhi(hq, 0x7FFFFFu);
  }
}

__global__ __launch_bounds__(kQBlock) void natural_encode_kernel(const float* __restrict__ x, int64_t n,
                                                                const int32_t* __restrict__ ri, uint64_t seed,
                                                                uint8_t* __restrict__ codes, int aligned,
                                                                int64_t xoff) {
  const int64_t nq = (n + 3) >> 2;
  for (int64_t q = (int64_t)blockIdx.x * kQBlock + threadIdx.x; q < nq; q += (int64_t)gridDim.x * kQBlock) {
    const int64_t e = q << 2;
    const bool fast = quad_fast(e, n, aligned != 0);
    float v[4];
    int32_t r[4];
    load_quad(x, e, n, fast, v);
    if (ri) {
      if (fast) {
        const int4 t = *reinterpret_cast<const int4*>(ri + e);
        r[0] = t.x; r[1] = t.y; r[2] = t.z; r[3] = t.w;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) r[j] = e + j < n ? ri[e + j] : 0;
      }
    } else {
      natural_rand4(seed, e + xoff, r);   // (xoff % 4 == 0: the bucket's quads)
    }
    uint32_t c[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) c[j] = natural_code(v[j], r[j]);
    if (fast) {
      *reinterpret_cast<uint32_t*>(codes + e) = c[0] | (c[1] << 8) | (c[2] << 16) | (c[3] << 24);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (e + j < n) codes[e + j] = (uint8_t)c[j];
    }
  }
}

__device__ __forceinline__ float natural_dec(uint32_t c) {
  const uint32_t e = c & 0x7F;
  const float mag = __uint_as_float((e + 18u) << 23);
  const float v = c > 127 ? -mag : mag;
  return v * (e >= 1 ? 1.0f : 0.0f);   // 0x80 decodes to -0.0 as in the reference
}

// cnat_cuda flavour (cnat_cuda.cu:68-134): frexp mantissa m in [0.5, 1); exponent kept w.p.
// 2|m| - 1; LUT: biased E <= 17 -> 0, E -> E - 17 saturating at 127, +128 if negative.
__device__ __forceinline__ uint32_t cnat_code(float v, float r) {
  if (v == 0.f) return 0u;
  int ex;
  const float prob = fabsf(frexpf(v, &ex)) / 0.5f - 1.0f;
  if (r >= prob) ex -= 1;
  const int biased = ex + 127;
  int code = biased <= 17 ? 0 : min(biased - 17, 127);
  if (v < 0.f) code += 128;
  return (uint32_t)code;
}

__global__ __launch_bounds__(kQBlock) void cnat_encode_kernel(const float* __restrict__ x, int64_t n,
                                                             const float* __restrict__ rnd, int deterministic,
                                                             uint64_t seed, uint8_t* __restrict__ codes,
                                                             int aligned, int64_t xoff) {
  const int64_t nq = (n + 3) >> 2;
  for (int64_t q = (int64_t)blockIdx.x * kQBlock + threadIdx.x; q < nq; q += (int64_t)gridDim.x * kQBlock) {
    const int64_t e = q << 2;
    const bool fast = quad_fast(e, n, aligned != 0);
    float v[4], r[4];
    load_quad(x, e, n, fast, v);
    if (deterministic) {
#pragma unroll
      for (int j = 0; j < 4; ++j) r[j] = 0.5f;
    } else if (rnd) {
      load_quad(rnd, e, n, fast, r);
    } else {
      uniform01x4(seed, (uint64_t)(e + xoff), r);   // one hash per quad (device generator)
    }
    uint32_t c[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) c[j] = cnat_code(v[j], r[j]);
    if (fast) {
      *reinterpret_cast<uint32_t*>(codes + e) = c[0] | (c[1] << 8) | (c[2] << 16) | (c[3] << 24);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (e + j < n) codes[e + j] = (uint8_t)c[j];
    }
  }
}

__device__ __forceinline__ float cnat_dec(uint32_t c) {
  const uint32_t m = c & 0x7F;
  const uint32_t e = m == 0 ? 0u : m + 17u;
  return __uint_as_float(((c >> 7) << 31) | (e << 23));
}

// decode (+ rank-ordered aggregate of W payloads at `stride`): 4 codes per 4-B load per rank,
// one 16-B store
template <int FLAVOUR>   // 0 = cupy natural, 1 = cnat
__global__ __launch_bounds__(kQBlock) void natural_decode_kernel(const uint8_t* __restrict__ codes,
                                                                int64_t stride, int world, int64_t n,
                                                                float divisor, int aggregate,
                                                                float* __restrict__ out, int aligned) {
  const int64_t nq = (n + 3) >> 2;
  for (int64_t q = (int64_t)blockIdx.x * kQBlock + threadIdx.x; q < nq; q += (int64_t)gridDim.x * kQBlock) {
    const int64_t e = q << 2;
    const bool fast = quad_fast(e, n, aligned != 0);
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int w = 0; w < world; ++w) {
      const uint8_t* c = codes + w * stride + e;
      uint32_t wd;
      if (fast) {
        wd = *reinterpret_cast<const uint32_t*>(c);
      } else {
        wd = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (e + j < n) wd |= (uint32_t)c[j] << (8 * j);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t cj = (wd >> (8 * j)) & 0xFFu;
        const float d = FLAVOUR == 0 ? natural_dec(cj) : cnat_dec(cj);
        acc[j] = (aggregate || w > 0) ? acc[j] + d : d;
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = divisor == 1.0f ? acc[j] : acc[j] / divisor;
    if (fast) {
      *reinterpret_cast<f4v*>(out + e) = f4v{acc[0], acc[1], acc[2], acc[3]};
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (e + j < n) out[e + j] = acc[j];
    }
  }
}

// ================================================================================================
// fp16 (grace_dl/dist/compressor/fp16.py): round-to-nearest-even cast and back, 4 per quad
__global__ __launch_bounds__(kQBlock) void f32_to_f16_kernel(const float* __restrict__ x, __half* __restrict__ h,
                                                            int64_t n, int aligned) {
  const int64_t nq = (n + 3) >> 2;
  for (int64_t q = (int64_t)blockIdx.x * kQBlock + threadIdx.x; q < nq; q += (int64_t)gridDim.x * kQBlock) {
    const int64_t e = q << 2;
    const bool fast = quad_fast(e, n, aligned != 0);
    float v[4];
    load_quad(x, e, n, fast, v);
    if (fast) {
      uint2 wd;
      wd.x = (uint32_t)__half_as_ushort(__float2half_rn(v[0])) | ((uint32_t)__half_as_ushort(__float2half_rn(v[1])) << 16);
      wd.y = (uint32_t)__half_as_ushort(__float2half_rn(v[2])) | ((uint32_t)__half_as_ushort(__float2half_rn(v[3])) << 16);
      *reinterpret_cast<uint2*>(h + e) = wd;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (e + j < n) h[e + j] = __float2half_rn(v[j]);
    }
  }
}
// f16 -> f32; with `aggregate` the W rank-major payloads at `stride` are summed in rank order from
// 0 (Python's sum: 0 + d0 + d1 ..., allgather.py:44) and divided by `divisor` unless it is 1 --
// the Allgather step's decompress + aggregate + divide in one pass
__global__ __launch_bounds__(kQBlock) void f16_to_f32_kernel(const __half* __restrict__ h, float* __restrict__ x,
                                                            int64_t n, int aligned, int64_t stride, int world,
                                                            int aggregate, float divisor) {
  const int64_t nq = (n + 3) >> 2;
  for (int64_t q = (int64_t)blockIdx.x * kQBlock + threadIdx.x; q < nq; q += (int64_t)gridDim.x * kQBlock) {
    const int64_t e = q << 2;
    const bool fast = quad_fast(e, n, aligned != 0);
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int w = 0; w < world; ++w) {
      const __half* hw = h + w * stride;
      float d[4];
      if (fast) {
        const uint2 wd = *reinterpret_cast<const uint2*>(hw + e);
        d[0] = __half2float(__ushort_as_half((unsigned short)wd.x));
        d[1] = __half2float(__ushort_as_half((unsigned short)(wd.x >> 16)));
        d[2] = __half2float(__ushort_as_half((unsigned short)wd.y));
        d[3] = __half2float(__ushort_as_half((unsigned short)(wd.y >> 16)));
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) d[j] = e + j < n ? __half2float(hw[e + j]) : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = (aggregate || w > 0) ? acc[j] + d[j] : d[j];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = divisor == 1.0f ? acc[j] : acc[j] / divisor;
    if (fast) {
      *reinterpret_cast<f4v*>(x + e) = f4v{acc[0], acc[1], acc[2], acc[3]};
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (e + j < n) x[e + j] = acc[j];
    }
  }
}

// World-1 Allgather(Natural | Natural_CUDA | FP16, NoneMemory).step in ONE pass: out = 0 + dec(enc(x))
// (the division by world size 1 is exact and omitted), with the same codes as the separate encode
// kernels on the device generator -- the codes never reach memory (8 B per element instead of 10 / 12).
enum CastMode : int { kCastNatural = 0, kCastCnat = 1, kCastCnatDet = 2, kCastF16 = 3 };
template <int MODE>
__device__ __forceinline__ float cast_round_trip(float v, float u, int32_t ri) {
  if constexpr (MODE == kCastNatural) return 0.f + natural_dec(natural_code(v, ri));
  else if constexpr (MODE == kCastCnat || MODE == kCastCnatDet) return 0.f + cnat_dec(cnat_code(v, u));
  else return 0.f + __half2float(__float2half_rn(v));
}

template <int MODE>
__global__ __launch_bounds__(kQBlock) void cast_step_w1_kernel(const float* __restrict__ x, float* __restrict__ o,
                                                              int64_t n, uint64_t seed) {
  const int64_t n4 = n >> 2;
  const int64_t q = (int64_t)blockIdx.x * kQBlock + threadIdx.x;
  const int64_t qq = q < n4 ? q : (n4 > 0 ? n4 - 1 : 0);
  const f4v v = n4 > 0 ? reinterpret_cast<const f4v*>(x)[qq] : f4v{0.f, 0.f, 0.f, 0.f};
  const int64_t e = q << 2;
  float u[4] = {0.5f, 0.5f, 0.5f, 0.5f};
  int32_t r[4] = {0, 0, 0, 0};
  if constexpr (MODE == kCastNatural) natural_rand4(seed, e, r);
  if constexpr (MODE == kCastCnat) uniform01x4(seed, (uint64_t)e, u);
  if (q < n4) {
    reinterpret_cast<f4v*>(o)[q] = f4v{cast_round_trip<MODE>(v.x, u[0], r[0]), cast_round_trip<MODE>(v.y, u[1], r[1]),
                                       cast_round_trip<MODE>(v.z, u[2], r[2]), cast_round_trip<MODE>(v.w, u[3], r[3])};
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && (n & 3)) {   // the scalar tail: one quad's generator
    const int64_t t0 = n4 << 2;
    float ut[4] = {0.5f, 0.5f, 0.5f, 0.5f};
    int32_t rt[4] = {0, 0, 0, 0};
    if constexpr (MODE == kCastNatural) natural_rand4(seed, t0, rt);
    if constexpr (MODE == kCastCnat) uniform01x4(seed, (uint64_t)t0, ut);
    for (int j = 0; j < (int)(n & 3); ++j) o[t0 + j] = cast_round_trip<MODE>(x[t0 + j], ut[j], rt[j]);
  }
}

// ================================================================================================
// QSGD, Horovod flavour (grace_dl/torch/compressor/qsgd.py:12-39): ONE norm over the whole tensor
// (tensor.norm(), no buckets, no padding), then the same codeword rule as above.  Three launches:
// f64 partial sums of x^2 per workgroup, one workgroup sums them in workgroup order and writes
// norm = (float)sqrt(total) (or passes an injected norm through), and an elementwise encoder that
// reads the norm once per thread.
constexpr int kQgBlocks = 1024;

__global__ __launch_bounds__(kQBlock) void qsgd_global_sumsq_kernel(const float* __restrict__ x, int64_t n,
                                                                   double* __restrict__ part) {
  double acc = 0.0;
  const int64_t n4 = ((reinterpret_cast<uintptr_t>(x) & 15) == 0) ? n >> 2 : 0;
  for (int64_t i = (int64_t)blockIdx.x * kQBlock + threadIdx.x; i < n4; i += (int64_t)gridDim.x * kQBlock) {
    const f4v v = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(x) + i);
    acc = fma((double)v.x, (double)v.x, acc);
    acc = fma((double)v.y, (double)v.y, acc);
    acc = fma((double)v.z, (double)v.z, acc);
    acc = fma((double)v.w, (double)v.w, acc);
  }
  for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * kQBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kQBlock)
    acc = fma((double)x[i], (double)x[i], acc);
  __shared__ double sh[kQBlock / kWave];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int w = 0; w < kQBlock / kWave; ++w) t += sh[w];
    part[blockIdx.x] = t;
  }
}

__global__ __launch_bounds__(kQBlock) void qsgd_global_norm_kernel(const double* __restrict__ part, int nparts,
                                                                  const float* __restrict__ norm_in,
                                                                  float* __restrict__ norm_out) {
  __shared__ double sh[kQBlock];
  double t = 0.0;
  for (int b = threadIdx.x; b < nparts; b += kQBlock) t += part[b];
  sh[threadIdx.x] = t;
  __syncthreads();
  if (threadIdx.x == 0) {
    if (norm_in) {
      norm_out[0] = norm_in[0];
    } else {
      double tot = 0.0;
      for (int b = 0; b < kQBlock; ++b) tot += sh[b];
      norm_out[0] = (float)sqrt(tot);
    }
  }
}

template <typename CodeT>
__global__ __launch_bounds__(kQBlock) void qsgd_global_encode_kernel(const float* __restrict__ x, int64_t n,
                                                                    const float* __restrict__ norm_p, float qf,
                                                                    const float* __restrict__ u, uint64_t seed,
                                                                    CodeT* __restrict__ codes, int aligned) {
  const float norm = norm_p[0];
  const float scale = (1.0f / norm) * qf;   // q / norm as torch's __rdiv__: reciprocal(norm) * q
  const int64_t nq = (n + 3) >> 2;
  for (int64_t q = (int64_t)blockIdx.x * kQBlock + threadIdx.x; q < nq; q += (int64_t)gridDim.x * kQBlock) {
    const int64_t e = q << 2;
    float v[4], uu[4];
    load_quad(x, e, n, aligned != 0, v);
    if (u) load_quad(u, e, n, aligned != 0, uu);
    else uniform01x4(seed, (uint64_t)e, uu);
    CodeT c[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) c[j] = qsgd_code<CodeT, 0>(v[j], scale * fabsf(v[j]), uu[j], norm);
    store_codes4(codes, e, n, aligned != 0, c);
  }
}

}  // namespace grace

using namespace grace;

// the pipelined encoder's grid: the cap, or more workgroups when a workgroup's bucket range would
// outgrow its LDS table (block_range32 rounds a range up to a multiple of 16 rows)
static unsigned qenc_pipe_grid(int64_t nbuckets) {
  const int64_t need = (nbuckets + (kQBkMax - 32) - 1) / (kQBkMax - 32);
  return (unsigned)std::max<int64_t>(stream_grid(nbuckets, kQNB * kQBlock / 16, kQEncPipeGridCap), need);
}

#ifdef GRACE_TERN_FLUSH
__global__ void tern_flush_kernel(float* p, int64_t n) {
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n; i += (int64_t)gridDim.x * blockDim.x * 4)
    *reinterpret_cast<float4*>(p + i) = make_float4(1.f, 2.f, 3.f, 4.f);
}
#endif

extern "C" {

grace_status_t grace_qsgd_step_w1(const float* x, const int64_t* seg_off, const int64_t* bkt_off, int32_t nseg,
                                  int64_t nbuckets, int32_t quantum_num, int32_t variant, const float* u,
                                  uint64_t seed, float* out, void* stream) {
  GRACE_REQUIRE(x && seg_off && bkt_off && nseg >= 1 && nseg <= kSegLds && nbuckets >= 0 &&
                    nbuckets < (int64_t(1) << 24) && quantum_num >= 1 && out &&
                    (variant == 0 || (variant == 1 && quantum_num < 128)),
                "grace_qsgd_step_w1: bad arguments (bucket 128, <= kSegLds segments)");
  if (nbuckets == 0) return GRACE_OK;
  hipStream_t st = as_stream(stream);
  // the fused step keeps the non-pipelined kernel: it writes 4 B per element, and the A/B on the
  // ResNet-50 set had the pipelined one slower there (43.1 / 40.6 us at 1024 / 2048 workgroups vs 40.3)
  const bool pipe = GRACE_QENC_PIPE_FUSED && !u;
  const unsigned grid16 = pipe ? qenc_pipe_grid(nbuckets) : stream_grid(nbuckets, kQNB * kQBlock / 16, kQEncGridCap);
#define GRACE_QSTEP128(CT, V)                                                                        \
  do { if (pipe)                                                                                          \
    qsgd_encode128_pipe_kernel<CT, V, true><<<grid16, kQBlock, 0, st>>>(                             \
        x, seg_off, bkt_off, nseg, (int32_t)nbuckets, (float)quantum_num, seed, nullptr, nullptr, out); \
  else                                                                                               \
    qsgd_encode128_kernel<CT, V, true><<<grid16, kQBlock, 0, st>>>(x, seg_off, bkt_off, nseg, (int32_t)nbuckets, \
                                                                (float)quantum_num, u, seed, nullptr, nullptr, \
                                                                nullptr, out); } while (0)
  if (variant == 1) GRACE_QSTEP128(int8_t, 1);
  else if (quantum_num < 128) GRACE_QSTEP128(int8_t, 0);
  else GRACE_QSTEP128(__half, 0);
#undef GRACE_QSTEP128
  GRACE_CHECK_LAUNCH("grace_qsgd_step_w1");
  return GRACE_OK;
}

int32_t grace_qsgd_seg_max(void) { return kSegLds; }

grace_status_t grace_qsgd_compress_at(const float* x, int64_t xoff, const int64_t* seg_off, const int64_t* bkt_off,
                                      int32_t nseg, int64_t nbuckets, int32_t quantum_num, int32_t bucket_size,
                                      int32_t variant, const float* u, uint64_t seed, const float* norms_in,
                                      float* norms_out, void* codes, void* stream) {
  GRACE_REQUIRE(x && seg_off && bkt_off && nseg >= 1 && nbuckets >= 0 && bucket_size >= 1 &&
                    quantum_num >= 1 && norms_out && codes && xoff >= 0 && xoff < ((int64_t)1 << 31),
                "grace_qsgd_compress: bad arguments");
  if (nbuckets == 0) return GRACE_OK;
  GRACE_REQUIRE(variant == 0 || (variant == 1 && quantum_num < 128), "grace_qsgd_compress: bad variant");
  const unsigned grid = stream_grid(nbuckets, kQNB * kQBlock / 32, kQGridCap);
  hipStream_t st = as_stream(stream);
  if (bucket_size == 128 && nseg <= kSegLds && nbuckets < (int64_t(1) << 24)) {   // n < 2^31
    const bool pipe = GRACE_QENC_PIPE && !u && !norms_in && xoff == 0;
    const unsigned grid16 = pipe ? qenc_pipe_grid(nbuckets) : stream_grid(nbuckets, kQNB * kQBlock / 16, kQEncGridCap);
#define GRACE_QENC128(CT, V)                                                                         \
  do { if (pipe)                                                                                          \
    qsgd_encode128_pipe_kernel<CT, V><<<grid16, kQBlock, 0, st>>>(x, seg_off, bkt_off, nseg, (int32_t)nbuckets, \
                                                               (float)quantum_num, seed, norms_out,  \
                                                               reinterpret_cast<CT*>(codes), nullptr); \
  else                                                                                               \
    qsgd_encode128_kernel<CT, V><<<grid16, kQBlock, 0, st>>>(x, seg_off, bkt_off, nseg, (int32_t)nbuckets, \
                                                          (float)quantum_num, u, seed, norms_in,      \
                                                          norms_out, reinterpret_cast<CT*>(codes),    \
                                                          nullptr, (uint32_t)xoff); } while (0)
    if (variant == 1) GRACE_QENC128(int8_t, 1);
    else if (quantum_num < 128) GRACE_QENC128(int8_t, 0);
    else GRACE_QENC128(__half, 0);
#undef GRACE_QENC128
    GRACE_CHECK_LAUNCH("grace_qsgd_compress");
    return GRACE_OK;
  }
  if (variant == 1) {
    qsgd_encode_kernel<int8_t, 1><<<grid, kQBlock, 0, st>>>(x, seg_off, bkt_off, nseg, nbuckets, bucket_size,
                                                           (float)quantum_num, u, seed, norms_in, norms_out,
                                                           reinterpret_cast<int8_t*>(codes), xoff);
  } else if (quantum_num < 128) {
    qsgd_encode_kernel<int8_t, 0><<<grid, kQBlock, 0, st>>>(x, seg_off, bkt_off, nseg, nbuckets, bucket_size,
                                                           (float)quantum_num, u, seed, norms_in, norms_out,
                                                           reinterpret_cast<int8_t*>(codes), xoff);
  } else {
    qsgd_encode_kernel<__half, 0><<<grid, kQBlock, 0, st>>>(x, seg_off, bkt_off, nseg, nbuckets, bucket_size,
                                                           (float)quantum_num, u, seed, norms_in, norms_out,
                                                           reinterpret_cast<__half*>(codes), xoff);
  }
  GRACE_CHECK_LAUNCH("grace_qsgd_compress");
  return GRACE_OK;
}

grace_status_t grace_qsgd_compress(const float* x, const int64_t* seg_off, const int64_t* bkt_off,
                                   int32_t nseg, int64_t nbuckets, int32_t quantum_num, int32_t bucket_size,
                                   int32_t variant, const float* u, uint64_t seed, const float* norms_in,
                                   float* norms_out, void* codes, void* stream) {
  return grace_qsgd_compress_at(x, 0, seg_off, bkt_off, nseg, nbuckets, quantum_num, bucket_size, variant, u, seed,
                                norms_in, norms_out, codes, stream);
}

size_t grace_qsgd_global_workspace_bytes(void) { return sizeof(double) * kQgBlocks; }

grace_status_t grace_qsgd_global_compress(const float* x, int64_t n, int32_t quantum_num, const float* u,
                                          uint64_t seed, const float* norm_in, float* norm_out, void* codes,
                                          void* ws, void* stream) {
  GRACE_REQUIRE(x && n >= 1 && quantum_num >= 1 && norm_out && codes && ws,
                "grace_qsgd_global_compress: bad arguments");
  hipStream_t st = as_stream(stream);
  double* part = reinterpret_cast<double*>(ws);
  int nparts = 0;
  if (!norm_in) {
    nparts = (int)stream_grid((n + 3) / 4, kQBlock, kQgBlocks);
    qsgd_global_sumsq_kernel<<<nparts, kQBlock, 0, st>>>(x, n, part);
    GRACE_CHECK_LAUNCH("grace_qsgd_global_compress");
  }
  qsgd_global_norm_kernel<<<1, kQBlock, 0, st>>>(part, nparts, norm_in, norm_out);
  GRACE_CHECK_LAUNCH("grace_qsgd_global_compress");
  const unsigned grid = stream_grid((n + 3) / 4, kQBlock, 4096);
  const int aligned = ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(u)) & 15) == 0 &&
                      (reinterpret_cast<uintptr_t>(codes) & (quantum_num < 128 ? 3 : 7)) == 0;
  if (quantum_num < 128)
    qsgd_global_encode_kernel<int8_t><<<grid, kQBlock, 0, st>>>(x, n, norm_out, (float)quantum_num, u, seed,
                                                                reinterpret_cast<int8_t*>(codes), aligned);
  else
    qsgd_global_encode_kernel<__half><<<grid, kQBlock, 0, st>>>(x, n, norm_out, (float)quantum_num, u, seed,
                                                                reinterpret_cast<__half*>(codes), aligned);
  GRACE_CHECK_LAUNCH("grace_qsgd_global_compress");
  return GRACE_OK;
}

grace_status_t grace_qsgd_decompress(const void* codes, const float* norms, int64_t code_stride,
                                     int64_t norm_stride, int32_t world, const int64_t* seg_off,
                                     const int64_t* bkt_off, int32_t nseg, int64_t n, int32_t quantum_num,
                                     int32_t bucket_size, int32_t variant, int32_t aggregate, float divisor,
                                     float* out, void* stream) {
  GRACE_REQUIRE(codes && norms && seg_off && bkt_off && out && world >= 1 && nseg >= 1 && n >= 0,
                "grace_qsgd_decompress: bad arguments");
  if (n == 0) return GRACE_OK;
  const unsigned grid = stream_grid((n + kDecRound - 1) / kDecRound, 1, 4096);
  hipStream_t st = as_stream(stream);
  // 4 codes per load: one 4-B (int8) / 8-B (fp16) load when every rank's slice is aligned
  const int64_t cbytes = variant == 0 && quantum_num >= 128 ? 2 : 1;
  const int vec = (code_stride % 4 == 0) && ((uintptr_t)codes % (4 * cbytes) == 0);
#define GRACE_QDEC(CT, V, B)                                                                         \
  qsgd_decode_kernel<CT, V, B><<<grid, kQBlock, 0, st>>>(reinterpret_cast<const CT*>(codes), norms,  \
                                                         code_stride, norm_stride, world, seg_off,   \
                                                         bkt_off, nseg, n, bucket_size,              \
                                                         (float)quantum_num, divisor, aggregate, vec, out)
  const bool b128 = bucket_size == 128;
  if (b128 && nseg <= kSegLds && n < (int64_t(1) << 31)) {
    const unsigned bgrid = stream_grid((n + 127) / 128 + nseg, kQNB * kQBlock / 16, kQGridCap);
#define GRACE_QDECB(CT, V)                                                                          \
  qsgd_decode_bkt_kernel<CT, V><<<bgrid, kQBlock, 0, st>>>(reinterpret_cast<const CT*>(codes), norms, \
                                                          code_stride, norm_stride, world, seg_off,  \
                                                          bkt_off, nseg, (float)quantum_num, divisor, \
                                                          aggregate, vec, out)
    if (variant == 1) GRACE_QDECB(int8_t, 1);
    else if (quantum_num < 128) GRACE_QDECB(int8_t, 0);
    else GRACE_QDECB(__half, 0);
#undef GRACE_QDECB
    GRACE_CHECK_LAUNCH("grace_qsgd_decompress");
    return GRACE_OK;
  }
  if (variant == 1) {
    if (b128) GRACE_QDEC(int8_t, 1, true); else GRACE_QDEC(int8_t, 1, false);
  } else if (quantum_num < 128) {
    if (b128) GRACE_QDEC(int8_t, 0, true); else GRACE_QDEC(int8_t, 0, false);
  } else {
    if (b128) GRACE_QDEC(__half, 0, true); else GRACE_QDEC(__half, 0, false);
  }
#undef GRACE_QDEC
  GRACE_CHECK_LAUNCH("grace_qsgd_decompress");
  return GRACE_OK;
}

grace_status_t grace_qsgd_decompress_records(const void* records, int64_t rec_bytes, int64_t norm_off_bytes,
                                             int32_t world, int64_t units_per_rank, const int64_t* rank_lo,
                                             const int64_t* seg_off, const int64_t* bkt_off, int32_t nseg, int64_t n,
                                             int32_t quantum_num, int32_t variant, float* out, void* stream) {
  const int64_t cbytes = variant == 0 && quantum_num >= 128 ? 2 : 1;
  GRACE_REQUIRE(records && rank_lo && seg_off && bkt_off && out && world >= 1 && nseg >= 1 && n >= 0 &&
                    units_per_rank >= 1 && nseg <= kSegLds && n < (int64_t(1) << 31) && rec_bytes % 16 == 0 &&
                    norm_off_bytes % 16 == 0 && norm_off_bytes < rec_bytes && (uintptr_t)records % 16 == 0,
                "grace_qsgd_decompress_records: bad arguments (16-B aligned records and norms, nseg <= 512)");
  GRACE_REQUIRE(variant == 0 || (variant == 1 && quantum_num < 128), "grace_qsgd_decompress_records: bad variant");
  if (n == 0) return GRACE_OK;
  const char* rec = reinterpret_cast<const char*>(records);
  const QShardRec sr{units_per_rank, rec_bytes / cbytes, rec_bytes / 4, norm_off_bytes / 4, rank_lo};
  const float* norms = reinterpret_cast<const float*>(rec);
  const unsigned bgrid = stream_grid((n + 127) / 128 + nseg, kQNB * kQBlock / 16, kQGridCap);
  hipStream_t st = as_stream(stream);
#define GRACE_QDECR(CT, V)                                                                           \
  qsgd_decode_bkt_kernel<CT, V><<<bgrid, kQBlock, 0, st>>>(reinterpret_cast<const CT*>(rec), norms, 0, 0, 1, \
                                                          seg_off, bkt_off, nseg, (float)quantum_num, 1.0f, 0, \
                                                          1, out, sr)
  if (variant == 1) GRACE_QDECR(int8_t, 1);
  else if (quantum_num < 128) GRACE_QDECR(int8_t, 0);
  else GRACE_QDECR(__half, 0);
#undef GRACE_QDECR
  GRACE_CHECK_LAUNCH("grace_qsgd_decompress_records");
  return GRACE_OK;
}

grace_status_t grace_terngrad_decompress_records(const void* records, int64_t rec_bytes, int32_t world,
                                                 const int64_t* rank_lo, int32_t packed, const float* scalars,
                                                 const int64_t* seg_off, int32_t nseg, int64_t n, float* out,
                                                 void* stream) {
  GRACE_REQUIRE(records && rank_lo && scalars && seg_off && out && world >= 1 && world <= kRecRanksMax && nseg >= 1 &&
                    nseg <= kSegLds && n >= 0 && n < (int64_t(1) << 31) && rec_bytes >= 16 && rec_bytes % 16 == 0 &&
                    (uintptr_t)records % 16 == 0 && (uintptr_t)out % 16 == 0,
                "grace_terngrad_decompress_records: bad arguments (1 <= world <= 64, nseg <= 512, n < 2^31, "
                "16-B aligned records of a 16-B multiple, 16-B aligned out)");
  if (n == 0) return GRACE_OK;
  tern_decode_records_kernel<<<stream_grid((n + 15) / 16, kQBlock, 8192), kQBlock, 0, as_stream(stream)>>>(
      reinterpret_cast<const uint8_t*>(records), rec_bytes, world, rank_lo, packed ? 1 : 0, scalars, seg_off, nseg, n,
      out);
  GRACE_CHECK_LAUNCH("grace_terngrad_decompress_records");
  return GRACE_OK;
}

size_t grace_terngrad_workspace_bytes(int64_t nunits) { return tern_ws_bytes(nunits); }
int32_t grace_terngrad_unit(void) { return kTernUnit; }

grace_status_t grace_terngrad_compress(const float* x, const int64_t* seg_off, const int64_t* unit_off,
                                       int32_t nseg, int64_t nunits, const float* clip_in, const float* u,
                                       uint64_t seed, int8_t* codes, float* scalars, void* ws,
                                       void* stream) {
  GRACE_REQUIRE(x && seg_off && unit_off && nseg >= 1 && nunits >= 1 && codes && scalars && ws,
                "grace_terngrad_compress: bad arguments");
  TernSlot* const w = reinterpret_cast<TernSlot*>(ws);
  tern_stats_kernel<<<(unsigned)nunits, kQBlock, 0, as_stream(stream)>>>(x, seg_off, unit_off, nseg, clip_in, w,
                                                                       scalars);
  GRACE_CHECK_LAUNCH("grace_terngrad_compress");
#ifdef GRACE_TERN_FLUSH
  // diagnostic A/B build only: stream 512 MiB of writes between the statistics pass and the
  // encoder, so the encoder's re-read of x cannot be served by the 256 MiB Infinity Cache
  {
    static float* junk = nullptr;
    constexpr int64_t kJunk = (int64_t)1 << 27;
    if (!junk && hipMalloc(&junk, kJunk * sizeof(float)) != hipSuccess) junk = nullptr;
    if (junk) tern_flush_kernel<<<4096, 256, 0, as_stream(stream)>>>(junk, kJunk);
  }
#endif
  if (u)
    tern_encode_kernel<false, true><<<(unsigned)nunits, kTernBlock, 0, as_stream(stream)>>>(
        x, seg_off, unit_off, nseg, w, u, seed, codes, nullptr, clip_in, scalars);
  else
    tern_encode_kernel<false, false><<<(unsigned)nunits, kTernBlock, 0, as_stream(stream)>>>(
        x, seg_off, unit_off, nseg, w, u, seed, codes, nullptr, clip_in, scalars);
  GRACE_CHECK_LAUNCH("grace_terngrad_compress");
  return GRACE_OK;
}

int32_t grace_terngrad_slot_bytes(void) { return (int32_t)sizeof(TernSlot); }

grace_status_t grace_terngrad_shard_stats(const float* x, int64_t xoff, const int64_t* seg_off,
                                          const int64_t* unit_off, int32_t nseg, int64_t unit0, int64_t nunits_local,
                                          void* ws, void* stream) {
  GRACE_REQUIRE(kTernEncReduce, "grace_terngrad_shard_stats: needs the encode-side scale reduction "
                "(a GRACE_TERN_ENC_REDUCE=0 build has no global slot protocol)");
  GRACE_REQUIRE(x && seg_off && unit_off && nseg >= 1 && unit0 >= 0 && nunits_local >= 0 && xoff >= 0 && ws &&
                    (reinterpret_cast<uintptr_t>(x) & 15) == 0,
                "grace_terngrad_shard_stats: bad arguments (16-B aligned shard)");
  if (nunits_local == 0) return GRACE_OK;
  tern_stats_kernel<<<(unsigned)nunits_local, kQBlock, 0, as_stream(stream)>>>(
      x, seg_off, unit_off, nseg, nullptr, reinterpret_cast<TernSlot*>(ws), nullptr, unit0, xoff);
  GRACE_CHECK_LAUNCH("grace_terngrad_shard_stats");
  return GRACE_OK;
}

grace_status_t grace_terngrad_shard_encode(const float* x, int64_t xoff, const int64_t* seg_off,
                                           const int64_t* unit_off, int32_t nseg, int64_t unit0,
                                           int64_t nunits_local, const float* clip_in, const float* u, uint64_t seed,
                                           int8_t* codes, const void* ws, void* stream) {
  GRACE_REQUIRE(kTernEncReduce, "grace_terngrad_shard_encode: needs the encode-side scale reduction "
                "(a GRACE_TERN_ENC_REDUCE=0 build has no global slot protocol)");
  GRACE_REQUIRE(x && seg_off && unit_off && nseg >= 1 && unit0 >= 0 && nunits_local >= 0 && xoff >= 0 && codes &&
                    ws && ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(u) |
                            reinterpret_cast<uintptr_t>(codes)) & 15) == 0,
                "grace_terngrad_shard_encode: bad arguments (16-B aligned shard, u and codes)");
  if (nunits_local == 0) return GRACE_OK;
  const TernSlot* w = reinterpret_cast<const TernSlot*>(ws);
  if (u)
    tern_encode_kernel<false, true><<<(unsigned)nunits_local, kTernBlock, 0, as_stream(stream)>>>(
        x, seg_off, unit_off, nseg, w, u, seed, codes, nullptr, clip_in, nullptr, unit0, xoff);
  else
    tern_encode_kernel<false, false><<<(unsigned)nunits_local, kTernBlock, 0, as_stream(stream)>>>(
        x, seg_off, unit_off, nseg, w, u, seed, codes, nullptr, clip_in, nullptr, unit0, xoff);
  GRACE_CHECK_LAUNCH("grace_terngrad_shard_encode");
  return GRACE_OK;
}

grace_status_t grace_terngrad_scalars(const int64_t* seg_off, const int64_t* unit_off, int32_t nseg,
                                      const float* clip_in, const void* ws, float* scalars, void* stream) {
  GRACE_REQUIRE(seg_off && unit_off && nseg >= 1 && ws && scalars, "grace_terngrad_scalars: bad arguments");
  tern_scalars_kernel<<<(unsigned)nseg, kTernBlock, 0, as_stream(stream)>>>(
      seg_off, unit_off, reinterpret_cast<const TernSlot*>(ws), clip_in, scalars);
  GRACE_CHECK_LAUNCH("grace_terngrad_scalars");
  return GRACE_OK;
}

grace_status_t grace_terngrad_step_w1(const float* x, const int64_t* seg_off, const int64_t* unit_off, int32_t nseg,
                                     int64_t nunits, const float* clip_in, const float* u, uint64_t seed,
                                     float* scalars, void* ws, float* out, void* stream) {
  GRACE_REQUIRE(x && seg_off && unit_off && nseg >= 1 && nunits >= 1 && scalars && ws && out &&
                    ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(out)) & 15) == 0,
                "grace_terngrad_step_w1: bad arguments (16-B aligned x and out)");
  TernSlot* const w = reinterpret_cast<TernSlot*>(ws);
  tern_stats_kernel<<<(unsigned)nunits, kQBlock, 0, as_stream(stream)>>>(x, seg_off, unit_off, nseg, clip_in, w,
                                                                       scalars);
  GRACE_CHECK_LAUNCH("grace_terngrad_step_w1");
  if (u)
    tern_encode_kernel<true, true><<<(unsigned)nunits, kTernBlock, 0, as_stream(stream)>>>(
        x, seg_off, unit_off, nseg, w, u, seed, nullptr, out, clip_in, scalars);
  else
    tern_encode_kernel<true, false><<<(unsigned)nunits, kTernBlock, 0, as_stream(stream)>>>(
        x, seg_off, unit_off, nseg, w, u, seed, nullptr, out, clip_in, scalars);
  GRACE_CHECK_LAUNCH("grace_terngrad_step_w1");
  return GRACE_OK;
}

grace_status_t grace_terngrad_decompress(const int8_t* codes, const float* scalars, int64_t code_stride,
                                         int64_t scal_stride, int32_t world, const int64_t* seg_off,
                                         int32_t nseg, int64_t n, int32_t aggregate, float divisor, float* out,
                                         void* stream) {
  GRACE_REQUIRE(codes && scalars && seg_off && out && world >= 1 && nseg >= 1 && n >= 0,
                "grace_terngrad_decompress: bad arguments");
  if (n == 0) return GRACE_OK;
  const int vec = (code_stride % 4 == 0) && ((uintptr_t)codes % 4 == 0);
  if constexpr (kTernTileQpt > 0) {
    if (world == 1 && vec && nseg <= kSegLds && (uintptr_t)out % 16 == 0) {
      constexpr int64_t kTile = (int64_t)kQBlock * 4 * (kTernTileQpt > 0 ? kTernTileQpt : 1);
      tern_decode_tile_kernel<(kTernTileQpt > 0 ? kTernTileQpt : 1)><<<(unsigned)((n + kTile - 1) / kTile), kQBlock, 0,
                                                                     as_stream(stream)>>>(
          codes, scalars, seg_off, nseg, n, divisor, aggregate, out);
      GRACE_CHECK_LAUNCH("grace_terngrad_decompress");
      return GRACE_OK;
    }
  }
  if (nseg <= kSegLds && n < (int64_t(1) << 31)) {
    tern_decode_row_kernel<<<stream_grid((n + 127) / 128, kQNB * kQBlock / 16, kQGridCap), kQBlock, 0,
                             as_stream(stream)>>>(codes, scalars, code_stride, scal_stride, world, seg_off, nseg,
                                                  (int32_t)n, divisor, aggregate, vec, out);
    GRACE_CHECK_LAUNCH("grace_terngrad_decompress");
    return GRACE_OK;
  }
  tern_decode_kernel<<<stream_grid((n + kDecRound - 1) / kDecRound, 1, 4096), kQBlock, 0, as_stream(stream)>>>(
      codes, scalars, code_stride, scal_stride, world, seg_off, nseg, n, divisor, aggregate, vec, out);
  GRACE_CHECK_LAUNCH("grace_terngrad_decompress");
  return GRACE_OK;
}

grace_status_t grace_natural_compress_at(const float* x, int64_t xoff, int64_t n, const int32_t* rand_int,
                                         uint64_t seed, uint8_t* codes, void* stream) {
  GRACE_REQUIRE(x && codes && n >= 0 && xoff >= 0 && (xoff & 3) == 0, "grace_natural_compress: bad arguments");
  if (n == 0) return GRACE_OK;
  const int al = ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(rand_int)) & 15) == 0 &&
                 (reinterpret_cast<uintptr_t>(codes) & 3) == 0;
  natural_encode_kernel<<<stream_grid((n + 3) / 4, kQBlock, 4096), kQBlock, 0, as_stream(stream)>>>(
      x, n, rand_int, seed, codes, al, xoff);
  GRACE_CHECK_LAUNCH("grace_natural_compress");
  return GRACE_OK;
}

grace_status_t grace_natural_compress(const float* x, int64_t n, const int32_t* rand_int, uint64_t seed,
                                      uint8_t* codes, void* stream) {
  return grace_natural_compress_at(x, 0, n, rand_int, seed, codes, stream);
}

grace_status_t grace_cnat_compress_at(const float* x, int64_t xoff, int64_t n, const float* rand,
                                      int32_t deterministic, uint64_t seed, uint8_t* codes, void* stream) {
  GRACE_REQUIRE(x && codes && n >= 0 && xoff >= 0 && (xoff & 3) == 0, "grace_cnat_compress: bad arguments");
  if (n == 0) return GRACE_OK;
  const int al = ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(rand)) & 15) == 0 &&
                 (reinterpret_cast<uintptr_t>(codes) & 3) == 0;
  cnat_encode_kernel<<<stream_grid((n + 3) / 4, kQBlock, 4096), kQBlock, 0, as_stream(stream)>>>(
      x, n, rand, deterministic, seed, codes, al, xoff);
  GRACE_CHECK_LAUNCH("grace_cnat_compress");
  return GRACE_OK;
}

grace_status_t grace_cnat_compress(const float* x, int64_t n, const float* rand, int32_t deterministic,
                                   uint64_t seed, uint8_t* codes, void* stream) {
  return grace_cnat_compress_at(x, 0, n, rand, deterministic, seed, codes, stream);
}

grace_status_t grace_natural_decompress(const uint8_t* codes, int64_t stride, int32_t world, int64_t n,
                                        int32_t flavour, int32_t aggregate, float divisor, float* out,
                                        void* stream) {
  GRACE_REQUIRE(codes && out && world >= 1 && n >= 0 && (flavour == 0 || flavour == 1),
                "grace_natural_decompress: bad arguments");
  if (n == 0) return GRACE_OK;
  const unsigned grid = stream_grid((n + 3) / 4, kQBlock, 4096);
  const int al = (reinterpret_cast<uintptr_t>(codes) & 3) == 0 && (stride % 4 == 0 || world == 1) &&
                 (reinterpret_cast<uintptr_t>(out) & 15) == 0;
  if (flavour == 0)
    natural_decode_kernel<0><<<grid, kQBlock, 0, as_stream(stream)>>>(codes, stride, world, n, divisor,
                                                                      aggregate, out, al);
  else
    natural_decode_kernel<1><<<grid, kQBlock, 0, as_stream(stream)>>>(codes, stride, world, n, divisor,
                                                                      aggregate, out, al);
  GRACE_CHECK_LAUNCH("grace_natural_decompress");
  return GRACE_OK;
}

grace_status_t grace_fp16_compress(const float* x, void* half_out, int64_t n, void* stream) {
  GRACE_REQUIRE(x && half_out && n >= 0, "grace_fp16_compress: bad arguments");
  if (n == 0) return GRACE_OK;
  const int al = (reinterpret_cast<uintptr_t>(x) & 15) == 0 && (reinterpret_cast<uintptr_t>(half_out) & 7) == 0;
  f32_to_f16_kernel<<<stream_grid((n + 3) / 4, kQBlock, 4096), kQBlock, 0, as_stream(stream)>>>(
      x, reinterpret_cast<__half*>(half_out), n, al);
  GRACE_CHECK_LAUNCH("grace_fp16_compress");
  return GRACE_OK;
}

grace_status_t grace_fp16_decompress(const void* half_in, float* out, int64_t n, void* stream) {
  GRACE_REQUIRE(half_in && out && n >= 0, "grace_fp16_decompress: bad arguments");
  if (n == 0) return GRACE_OK;
  const int al = (reinterpret_cast<uintptr_t>(half_in) & 7) == 0 && (reinterpret_cast<uintptr_t>(out) & 15) == 0;
  f16_to_f32_kernel<<<stream_grid((n + 3) / 4, kQBlock, 4096), kQBlock, 0, as_stream(stream)>>>(
      reinterpret_cast<const __half*>(half_in), out, n, al, 0, 1, 0, 1.0f);
  GRACE_CHECK_LAUNCH("grace_fp16_decompress");
  return GRACE_OK;
}

grace_status_t grace_cast_step_w1(const float* x, int64_t n, int32_t mode, uint64_t seed, float* out,
                                  void* stream) {
  GRACE_REQUIRE(x && out && n >= 0 && mode >= 0 && mode <= 3 &&
                ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(out)) & 15) == 0,
                "grace_cast_step_w1: bad arguments (16-B aligned x and out)");
  if (n == 0) return GRACE_OK;
  const unsigned grid = (unsigned)(((n >> 2) + kQBlock - 1) / kQBlock > 0 ? ((n >> 2) + kQBlock - 1) / kQBlock : 1);
  const hipStream_t st = as_stream(stream);
  switch (mode) {
    case kCastNatural: cast_step_w1_kernel<kCastNatural><<<grid, kQBlock, 0, st>>>(x, out, n, seed); break;
    case kCastCnat: cast_step_w1_kernel<kCastCnat><<<grid, kQBlock, 0, st>>>(x, out, n, seed); break;
    case kCastCnatDet: cast_step_w1_kernel<kCastCnatDet><<<grid, kQBlock, 0, st>>>(x, out, n, seed); break;
    default: cast_step_w1_kernel<kCastF16><<<grid, kQBlock, 0, st>>>(x, out, n, seed); break;
  }
  GRACE_CHECK_LAUNCH("grace_cast_step_w1");
  return GRACE_OK;
}

grace_status_t grace_fp16_decompress_aggregate(const void* half_in, int64_t stride, int32_t world, int64_t n,
                                               float divisor, float* out, void* stream) {
  GRACE_REQUIRE(half_in && out && n >= 0 && world >= 1 && stride >= n && divisor != 0.0f,
                "grace_fp16_decompress_aggregate: bad arguments");
  if (n == 0) return GRACE_OK;
  const int al = (reinterpret_cast<uintptr_t>(half_in) & 7) == 0 && (stride & 3) == 0 &&
                 (reinterpret_cast<uintptr_t>(out) & 15) == 0;
  f16_to_f32_kernel<<<stream_grid((n + 3) / 4, kQBlock, 4096), kQBlock, 0, as_stream(stream)>>>(
      reinterpret_cast<const __half*>(half_in), out, n, al, stride, world, 1, divisor);
  GRACE_CHECK_LAUNCH("grace_fp16_decompress_aggregate");
  return GRACE_OK;
}

}  // extern "C"
