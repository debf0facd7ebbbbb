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

// segment containing flat element / bucket index `x`: largest s with off[s] <= x
__device__ __forceinline__ int find_seg(const int64_t* off, int nseg, int64_t x) {
  int lo = 0, hi = nseg - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (off[mid] <= x) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// float -> int16 exactly as torch CPU on x86 (cvttss2si to int32, low 16 bits): NaN / out of
// int32 range -> 0x80000000 -> 0.  Used by QSGD's .type(torch.int16) (qsgd.py:36).
__device__ __forceinline__ int32_t f2i16_x86(float v) {
  if (!(fabsf(v) < 2147483648.0f)) return 0;   // NaN, inf, |v| >= 2^31
  return (int32_t)(int16_t)(int32_t)v;
}

// ================================================================================================
// QSGD (grace_dl/dist/compressor/qsgd.py:12-51)
//   norm_b   = sqrt(sum over the zero-padded bucket of x^2)          (f32 result; f64 accumulate)
//   level    = (reciprocal(norm) * q) * |x|   -- Tensor.__rdiv__ is reciprocal() * q
//   new      = floor(level) + (u < level - floor(level))
//   code     = int16(new * sign(x)) -> int8 (q < 128) or fp16 (q >= 128)
// One wave per group of buckets: each lane loads its slice of the bucket, the bucket norm is a
// shuffle reduction, then the same lane encodes its elements.  Reads x once.
// VARIANT 0: QSGDCompressor (qsgd.py:12-39).  VARIANT 1: QSGDCompressor_CUDA / qsgd_cuda.cu:320-388
// (f64 norms over finite elements, level = q / norm * |x| by one division, NaN/Inf -> -128).
template <typename CodeT, int VARIANT>
__global__ __launch_bounds__(kQBlock) void qsgd_encode_kernel(
    const float* __restrict__ x, const int64_t* __restrict__ seg_off, const int64_t* __restrict__ bkt_off,
    int nseg, int64_t nbuckets, int bucket, float qf, const float* __restrict__ u, uint64_t seed,
    const float* __restrict__ norms_in, float* __restrict__ norms_out, CodeT* __restrict__ codes) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * kQBlock + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * kQBlock) >> 6;
  for (int64_t b = wave; b < nbuckets; b += nwaves) {
    const int s = find_seg(bkt_off, nseg, b);
    const int64_t base = seg_off[s] + (b - bkt_off[s]) * bucket;
    const int64_t end = min(base + (int64_t)bucket, seg_off[s + 1]);
    float norm;
    if (norms_in) {
      norm = norms_in[b];
    } else {
      double acc = 0.0;
      for (int64_t i = base + lane; i < end; i += 64) {
        const double v = (double)x[i];
        if (VARIANT == 0 || isfinite(v)) acc += v * v;
      }
      acc = wave_sum(acc);
      norm = VARIANT == 0 ? sqrtf((float)acc) : (float)sqrt(acc);
    }
    if (lane == 0) norms_out[b] = norm;
    const float scale = VARIANT == 0 ? (1.0f / norm) * qf : qf / norm;
    for (int64_t i = base + lane; i < end; i += 64) {
      const float xv = x[i];
      const float level = scale * fabsf(xv);
      const float prev = floorf(level);
      const float ui = u ? u[i] : uniform01(seed, (uint64_t)i);
      const float nl = prev + ((ui < level - prev) ? 1.0f : 0.0f);
      if constexpr (VARIANT == 0) {
        const float sg = xv > 0.f ? 1.f : (xv < 0.f ? -1.f : (xv == 0.f ? 0.f : xv));   // torch.sign
        const int32_t c16 = f2i16_x86(nl * sg);
        if constexpr (sizeof(CodeT) == 1) codes[i] = (CodeT)(int8_t)c16;
        else codes[i] = (CodeT)__float2half((float)(int16_t)c16);
      } else {
        int8_t c = -128;
        if (isfinite(norm) && isfinite(xv)) {
          const int8_t pl = (int8_t)floorf(level);
          c = (ui < level - prev) ? (int8_t)(pl + 1) : pl;
          if (xv < 0.f) c = (int8_t)-c;
        }
        codes[i] = (CodeT)c;
      }
    }
  }
}

// decode (+ rank-ordered aggregate of W payloads): out = ((0 + d_0) + d_1 ...) / divisor with
// d_w = (norm_w / q) * code_w  (qsgd.py:44-49).  W = 1, divisor = 1 is plain decompress.
template <typename CodeT, int VARIANT>
__global__ __launch_bounds__(kQBlock) void qsgd_decode_kernel(
    const CodeT* __restrict__ codes, const float* __restrict__ norms, int64_t code_stride,
    int64_t norm_stride, int world, const int64_t* __restrict__ seg_off,
    const int64_t* __restrict__ bkt_off, int nseg, int64_t n, int bucket, float qf, float divisor,
    int aggregate, float* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * kQBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kQBlock) {
    const int s = find_seg(seg_off, nseg, i);
    const int64_t b = bkt_off[s] + (i - seg_off[s]) / bucket;
    float acc = 0.f;
    for (int w = 0; w < world; ++w) {
      float c;
      if constexpr (sizeof(CodeT) == 1) c = (float)(int8_t)codes[w * code_stride + i];
      else c = __half2float(codes[w * code_stride + i]);
      float d = (norms[w * norm_stride + b] / qf) * c;
      if (VARIANT == 1 && c == -128.0f) d = __int_as_float(0x7FC00000);
      acc = (aggregate || w > 0) ? acc + d : d;   // Python sum: 0 + d_0 + d_1 ...
    }
    out[i] = divisor == 1.0f ? acc : acc / divisor;
  }
}

// ================================================================================================
// TernGrad (grace_dl/dist/compressor/terngrad.py:7-30)
//   std    = sqrt(mean((x - mean x)^2))        (here: f64 sums of x and x^2, one read)
//   c      = f32(2.5 * (double)f32(std))       clamp bound as torch rounds the Python double
//   scalar = max |clamp(x, -c, c)| = min(max|x|, c)
//   code   = (u * scalar >= |clamp x|) ? 0 : sign(x)          int8 in {-1, 0, 1}
// Stage 1 writes f64 partials per work unit; stage 2 (encode) reduces its segment's partials in
// fixed order (deterministic), derives the scale and encodes its unit.
constexpr int kTernUnit = 16384;

struct TernPartial { double sum, sq; float amax; uint32_t nan; };

__global__ __launch_bounds__(kQBlock) void tern_stats_kernel(const float* __restrict__ x,
                                                            const int64_t* __restrict__ seg_off,
                                                            const int64_t* __restrict__ unit_off, int nseg,
                                                            TernPartial* __restrict__ part) {
  const int64_t unit = blockIdx.x;
  const int s = find_seg(unit_off, nseg, unit);
  const int64_t base = seg_off[s] + (unit - unit_off[s]) * kTernUnit;
  const int64_t end = min(base + (int64_t)kTernUnit, seg_off[s + 1]);
  double sum = 0.0, sq = 0.0;
  float amax = 0.f;
  uint32_t nan = 0;
  for (int64_t i = base + threadIdx.x; i < end; i += kQBlock) {
    const float v = x[i];
    sum += (double)v;
    sq += (double)v * (double)v;
    if (v != v) nan = 1; else amax = fmaxf(amax, fabsf(v));
  }
  __shared__ double sh_s[kQBlock / kWave], sh_q[kQBlock / kWave];
  __shared__ float sh_m[kQBlock / kWave];
  __shared__ uint32_t sh_n[kQBlock / kWave];
  sum = wave_sum(sum);
  sq = wave_sum(sq);
  amax = wave_max(amax);
  nan = __ballot(nan != 0) != 0;
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { sh_s[w] = sum; sh_q[w] = sq; sh_m[w] = amax; sh_n[w] = nan; }
  __syncthreads();
  if (threadIdx.x == 0) {
    TernPartial p{0.0, 0.0, 0.f, 0u};
    for (int j = 0; j < kQBlock / kWave; ++j) {
      p.sum += sh_s[j]; p.sq += sh_q[j]; p.amax = fmaxf(p.amax, sh_m[j]); p.nan |= sh_n[j];
    }
    part[unit] = p;
  }
}

__device__ __forceinline__ void tern_scale(const TernPartial* part, int64_t u0, int64_t u1, int64_t n,
                                           const float* clip_in, int s, float* scalar) {
  double sum = 0.0, sq = 0.0;
  float amax = 0.f;
  uint32_t nan = 0;
  for (int64_t j = u0; j < u1; ++j) {
    sum += part[j].sum; sq += part[j].sq; amax = fmaxf(amax, part[j].amax); nan |= part[j].nan;
  }
  float c;
  if (clip_in) {
    c = clip_in[s];
  } else {
    const double mean = sum / (double)n;
    double var = sq / (double)n - mean * mean;
    if (var < 0.0) var = 0.0;
    const float stdf = (float)sqrt(var);
    c = (float)(2.5 * (double)stdf);
  }
  *scalar = nan ? __int_as_float(0x7FC00000) : fminf(amax, c);
}

__global__ __launch_bounds__(kQBlock) void tern_encode_kernel(
    const float* __restrict__ x, const int64_t* __restrict__ seg_off, const int64_t* __restrict__ unit_off,
    int nseg, const TernPartial* __restrict__ part, const float* __restrict__ clip_in,
    const float* __restrict__ u, uint64_t seed, int8_t* __restrict__ codes, float* __restrict__ scalars) {
  const int64_t unit = blockIdx.x;
  const int s = find_seg(unit_off, nseg, unit);
  __shared__ float s_scalar, s_clip;
  if (threadIdx.x == 0) {
    float sc;
    tern_scale(part, unit_off[s], unit_off[s + 1], seg_off[s + 1] - seg_off[s], clip_in, s, &sc);
    s_scalar = sc;
    if (unit == unit_off[s]) scalars[s] = sc;
    // clamp bound: the injected / derived c (scalar = min(max|x|, c))
    if (clip_in) {
      s_clip = clip_in[s];
    } else {
      double sum = 0.0, sq = 0.0;
      for (int64_t j = unit_off[s]; j < unit_off[s + 1]; ++j) { sum += part[j].sum; sq += part[j].sq; }
      const double nn = (double)(seg_off[s + 1] - seg_off[s]);
      const double mean = sum / nn;
      double var = sq / nn - mean * mean;
      if (var < 0.0) var = 0.0;
      s_clip = (float)(2.5 * (double)(float)sqrt(var));
    }
  }
  __syncthreads();
  const float scalar = s_scalar, c = s_clip;
  const int64_t base = seg_off[s] + (unit - unit_off[s]) * kTernUnit;
  const int64_t end = min(base + (int64_t)kTernUnit, seg_off[s + 1]);
  for (int64_t i = base + threadIdx.x; i < end; i += kQBlock) {
    const float xv = x[i];
    const float cl = fminf(fmaxf(xv, -c), c);
    const float ab = fabsf(cl);
    const float ui = u ? u[i] : uniform01(seed, (uint64_t)i);
    const float rnd = ui * scalar;
    int8_t code = 0;
    if (!(rnd >= ab)) {
      const float sg = cl > 0.f ? scalar : (cl < 0.f ? -scalar : 0.f);
      code = sg > 0.f ? 1 : (sg < 0.f ? -1 : 0);
    }
    codes[i] = code;
  }
}

__global__ __launch_bounds__(kQBlock) void tern_decode_kernel(const int8_t* __restrict__ codes,
                                                             const float* __restrict__ scalars,
                                                             int64_t code_stride, int64_t scal_stride,
                                                             int world, const int64_t* __restrict__ seg_off,
                                                             int nseg, int64_t n, float divisor, int aggregate,
                                                             float* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * kQBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kQBlock) {
    const int s = find_seg(seg_off, nseg, i);
    float acc = 0.f;
    for (int w = 0; w < world; ++w) {
      const float d = (float)codes[w * code_stride + i] * scalars[w * scal_stride + s];
      acc = (aggregate || w > 0) ? acc + d : d;
    }
    out[i] = divisor == 1.0f ? acc : acc / divisor;
  }
}

// ================================================================================================
// natural compression, cupy flavour (grace_dl/dist/compressor/natural.py:12-40): exponent
// rounded up when mantissa > randint(0, 2^23 - 1), clipped to [18, 145], code = sign | (E - 18).
__global__ __launch_bounds__(kQBlock) void natural_encode_kernel(const float* __restrict__ x, int64_t n,
                                                                const int32_t* __restrict__ ri, uint64_t seed,
                                                                uint8_t* __restrict__ codes) {
  for (int64_t i = (int64_t)blockIdx.x * kQBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kQBlock) {
    const int32_t bits = __float_as_int(x[i]);
    const int32_t sign = bits & (int32_t)0x80000000;
    int32_t e = bits & 0x7F800000;
    const int32_t mant = bits & 0x007FFFFF;
    const int32_t r = ri ? ri[i] : (int32_t)(mix64(seed ^ mix64((uint64_t)i)) % 0x7FFFFFull);
    if (mant > r) e += 0x00800000;
    e = min(max(e, (int32_t)0x09000000), (int32_t)0x48800000);
    codes[i] = (uint8_t)((sign >> 24) | ((e >> 23) - 18));
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
__global__ __launch_bounds__(kQBlock) void cnat_encode_kernel(const float* __restrict__ x, int64_t n,
                                                             const float* __restrict__ rnd, int deterministic,
                                                             uint64_t seed, uint8_t* __restrict__ codes) {
  for (int64_t i = (int64_t)blockIdx.x * kQBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kQBlock) {
    const float v = x[i];
    if (v == 0.f) { codes[i] = 0; continue; }
    int ex;
    const float prob = fabsf(frexpf(v, &ex)) / 0.5f - 1.0f;
    const float r = deterministic ? 0.5f : (rnd ? rnd[i] : uniform01(seed, (uint64_t)i));
    if (r >= prob) ex -= 1;
    const int biased = ex + 127;
    int code = biased <= 17 ? 0 : min(biased - 17, 127);
    if (v < 0.f) code += 128;
    codes[i] = (uint8_t)code;
  }
}

__device__ __forceinline__ float cnat_dec(uint32_t c) {
  const uint32_t m = c & 0x7F;
  const uint32_t e = m == 0 ? 0u : m + 17u;
  return __uint_as_float(((c >> 7) << 31) | (e << 23));
}

template <int FLAVOUR>   // 0 = cupy natural, 1 = cnat
__global__ __launch_bounds__(kQBlock) void natural_decode_kernel(const uint8_t* __restrict__ codes,
                                                                int64_t stride, int world, int64_t n,
                                                                float divisor, int aggregate,
                                                                float* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * kQBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kQBlock) {
    float acc = 0.f;
    for (int w = 0; w < world; ++w) {
      const uint32_t c = codes[w * stride + i];
      const float d = FLAVOUR == 0 ? natural_dec(c) : cnat_dec(c);
      acc = (aggregate || w > 0) ? acc + d : d;
    }
    out[i] = divisor == 1.0f ? acc : acc / divisor;
  }
}

// ================================================================================================
// fp16 (grace_dl/dist/compressor/fp16.py): round-to-nearest-even cast and back
__global__ __launch_bounds__(kQBlock) void f32_to_f16_kernel(const float* __restrict__ x, __half* __restrict__ h,
                                                            int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * kQBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kQBlock)
    h[i] = __float2half_rn(x[i]);
}
__global__ __launch_bounds__(kQBlock) void f16_to_f32_kernel(const __half* __restrict__ h, float* __restrict__ x,
                                                            int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * kQBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kQBlock)
    x[i] = __half2float(h[i]);
}

}  // namespace grace

using namespace grace;

extern "C" {

grace_status_t grace_qsgd_compress(const float* x, const int64_t* seg_off, const int64_t* bkt_off,
                                   int32_t nseg, int64_t nbuckets, int32_t quantum_num, int32_t bucket_size,
                                   int32_t variant, const float* u, uint64_t seed, const float* norms_in,
                                   float* norms_out, void* codes, void* stream) {
  GRACE_REQUIRE(x && seg_off && bkt_off && nseg >= 1 && nbuckets >= 0 && bucket_size >= 1 &&
                    quantum_num >= 1 && norms_out && codes,
                "grace_qsgd_compress: bad arguments");
  if (nbuckets == 0) return GRACE_OK;
  GRACE_REQUIRE(variant == 0 || (variant == 1 && quantum_num < 128), "grace_qsgd_compress: bad variant");
  const unsigned grid = stream_grid(nbuckets, kQBlock / 64, 4096);
  hipStream_t st = as_stream(stream);
  if (variant == 1) {
    qsgd_encode_kernel<int8_t, 1><<<grid, kQBlock, 0, st>>>(x, seg_off, bkt_off, nseg, nbuckets, bucket_size,
                                                           (float)quantum_num, u, seed, norms_in, norms_out,
                                                           reinterpret_cast<int8_t*>(codes));
  } else if (quantum_num < 128) {
    qsgd_encode_kernel<int8_t, 0><<<grid, kQBlock, 0, st>>>(x, seg_off, bkt_off, nseg, nbuckets, bucket_size,
                                                           (float)quantum_num, u, seed, norms_in, norms_out,
                                                           reinterpret_cast<int8_t*>(codes));
  } else {
    qsgd_encode_kernel<__half, 0><<<grid, kQBlock, 0, st>>>(x, seg_off, bkt_off, nseg, nbuckets, bucket_size,
                                                           (float)quantum_num, u, seed, norms_in, norms_out,
                                                           reinterpret_cast<__half*>(codes));
  }
  GRACE_CHECK_LAUNCH("grace_qsgd_compress");
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
  const unsigned grid = stream_grid(n, kQBlock, 4096);
  hipStream_t st = as_stream(stream);
  if (variant == 1) {
    qsgd_decode_kernel<int8_t, 1><<<grid, kQBlock, 0, st>>>(reinterpret_cast<const int8_t*>(codes), norms,
                                                           code_stride, norm_stride, world, seg_off, bkt_off,
                                                           nseg, n, bucket_size, (float)quantum_num, divisor,
                                                           aggregate, out);
  } else if (quantum_num < 128) {
    qsgd_decode_kernel<int8_t, 0><<<grid, kQBlock, 0, st>>>(reinterpret_cast<const int8_t*>(codes), norms,
                                                           code_stride, norm_stride, world, seg_off, bkt_off,
                                                           nseg, n, bucket_size, (float)quantum_num, divisor,
                                                           aggregate, out);
  } else {
    qsgd_decode_kernel<__half, 0><<<grid, kQBlock, 0, st>>>(reinterpret_cast<const __half*>(codes), norms,
                                                           code_stride, norm_stride, world, seg_off, bkt_off,
                                                           nseg, n, bucket_size, (float)quantum_num, divisor,
                                                           aggregate, out);
  }
  GRACE_CHECK_LAUNCH("grace_qsgd_decompress");
  return GRACE_OK;
}

size_t grace_terngrad_workspace_bytes(int64_t nunits) { return sizeof(TernPartial) * (size_t)(nunits + 1); }
int32_t grace_terngrad_unit(void) { return kTernUnit; }

grace_status_t grace_terngrad_compress(const float* x, const int64_t* seg_off, const int64_t* unit_off,
                                       int32_t nseg, int64_t nunits, const float* clip_in, const float* u,
                                       uint64_t seed, int8_t* codes, float* scalars, void* ws,
                                       void* stream) {
  GRACE_REQUIRE(x && seg_off && unit_off && nseg >= 1 && nunits >= 1 && codes && scalars && ws,
                "grace_terngrad_compress: bad arguments");
  TernPartial* part = reinterpret_cast<TernPartial*>(ws);
  tern_stats_kernel<<<(unsigned)nunits, kQBlock, 0, as_stream(stream)>>>(x, seg_off, unit_off, nseg, part);
  GRACE_CHECK_LAUNCH("grace_terngrad_compress");
  tern_encode_kernel<<<(unsigned)nunits, kQBlock, 0, as_stream(stream)>>>(x, seg_off, unit_off, nseg, part,
                                                                         clip_in, u, seed, codes, scalars);
  GRACE_CHECK_LAUNCH("grace_terngrad_compress");
  return GRACE_OK;
}

grace_status_t grace_terngrad_decompress(const int8_t* codes, const float* scalars, int64_t code_stride,
                                         int64_t scal_stride, int32_t world, const int64_t* seg_off,
                                         int32_t nseg, int64_t n, int32_t aggregate, float divisor, float* out,
                                         void* stream) {
  GRACE_REQUIRE(codes && scalars && seg_off && out && world >= 1 && nseg >= 1 && n >= 0,
                "grace_terngrad_decompress: bad arguments");
  if (n == 0) return GRACE_OK;
  tern_decode_kernel<<<stream_grid(n, kQBlock, 4096), kQBlock, 0, as_stream(stream)>>>(
      codes, scalars, code_stride, scal_stride, world, seg_off, nseg, n, divisor, aggregate, out);
  GRACE_CHECK_LAUNCH("grace_terngrad_decompress");
  return GRACE_OK;
}

grace_status_t grace_natural_compress(const float* x, int64_t n, const int32_t* rand_int, uint64_t seed,
                                      uint8_t* codes, void* stream) {
  GRACE_REQUIRE(x && codes && n >= 0, "grace_natural_compress: bad arguments");
  if (n == 0) return GRACE_OK;
  natural_encode_kernel<<<stream_grid(n, kQBlock, 4096), kQBlock, 0, as_stream(stream)>>>(x, n, rand_int, seed,
                                                                                        codes);
  GRACE_CHECK_LAUNCH("grace_natural_compress");
  return GRACE_OK;
}

grace_status_t grace_cnat_compress(const float* x, int64_t n, const float* rand, int32_t deterministic,
                                   uint64_t seed, uint8_t* codes, void* stream) {
  GRACE_REQUIRE(x && codes && n >= 0, "grace_cnat_compress: bad arguments");
  if (n == 0) return GRACE_OK;
  cnat_encode_kernel<<<stream_grid(n, kQBlock, 4096), kQBlock, 0, as_stream(stream)>>>(x, n, rand, deterministic,
                                                                                     seed, codes);
  GRACE_CHECK_LAUNCH("grace_cnat_compress");
  return GRACE_OK;
}

grace_status_t grace_natural_decompress(const uint8_t* codes, int64_t stride, int32_t world, int64_t n,
                                        int32_t flavour, int32_t aggregate, float divisor, float* out,
                                        void* stream) {
  GRACE_REQUIRE(codes && out && world >= 1 && n >= 0 && (flavour == 0 || flavour == 1),
                "grace_natural_decompress: bad arguments");
  if (n == 0) return GRACE_OK;
  const unsigned grid = stream_grid(n, kQBlock, 4096);
  if (flavour == 0)
    natural_decode_kernel<0><<<grid, kQBlock, 0, as_stream(stream)>>>(codes, stride, world, n, divisor,
                                                                      aggregate, out);
  else
    natural_decode_kernel<1><<<grid, kQBlock, 0, as_stream(stream)>>>(codes, stride, world, n, divisor,
                                                                      aggregate, out);
  GRACE_CHECK_LAUNCH("grace_natural_decompress");
  return GRACE_OK;
}

grace_status_t grace_fp16_compress(const float* x, void* half_out, int64_t n, void* stream) {
  GRACE_REQUIRE(x && half_out && n >= 0, "grace_fp16_compress: bad arguments");
  if (n == 0) return GRACE_OK;
  f32_to_f16_kernel<<<stream_grid(n, kQBlock, 4096), kQBlock, 0, as_stream(stream)>>>(
      x, reinterpret_cast<__half*>(half_out), n);
  GRACE_CHECK_LAUNCH("grace_fp16_compress");
  return GRACE_OK;
}

grace_status_t grace_fp16_decompress(const void* half_in, float* out, int64_t n, void* stream) {
  GRACE_REQUIRE(half_in && out && n >= 0, "grace_fp16_decompress: bad arguments");
  if (n == 0) return GRACE_OK;
  f16_to_f32_kernel<<<stream_grid(n, kQBlock, 4096), kQBlock, 0, as_stream(stream)>>>(
      reinterpret_cast<const __half*>(half_in), out, n);
  GRACE_CHECK_LAUNCH("grace_fp16_decompress");
  return GRACE_OK;
}

}  // extern "C"
