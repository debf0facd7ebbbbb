// Elementwise codecs and memory arithmetic: residual axpby/sub, the signSGD family, one-bit,
// and the small reductions they need.  All kernels stream 16 B per lane (float4 loads of the
// f32 gradient, one 32-bit word of four u8 codewords per lane) and grid-stride over the bucket.
#include <math.h>
#include <stdio.h>
#include <string.h>

#include "common.h"

namespace grace {

static thread_local char g_err[512] = "";

void set_error(const char* where, hipError_t e) {
  snprintf(g_err, sizeof(g_err), "%s: %s", where, hipGetErrorString(e));
}
void set_error_msg(const char* msg) { snprintf(g_err, sizeof(g_err), "%s", msg); }

static inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }
static inline bool aligned4(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 3u) == 0; }

constexpr int kBlock = 256;

// ------------------------------------------------------------------------------------------------
// Generic 4-wide streaming driver: Op::vec(i, i4) handles elements [4*i4, 4*i4+4), Op::one(i)
// a single element.  VEC=false runs the scalar loop (unaligned views).
template <bool VEC, typename Op>
__global__ __launch_bounds__(kBlock) void stream_kernel(Op op, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if constexpr (VEC) {
    const int64_t n4 = n >> 2;
    for (int64_t i = gid; i < n4; i += stride) op.vec(i);
    for (int64_t i = (n4 << 2) + gid; i < n; i += stride) op.one(i);
  } else {
    for (int64_t i = gid; i < n; i += stride) op.one(i);
  }
}

template <typename Op>
static grace_status_t launch_stream(const char* name, Op op, int64_t n, bool vec_ok, void* stream) {
  if (n <= 0) return GRACE_OK;
  if (vec_ok) {
    stream_kernel<true, Op><<<stream_grid((n + 3) / 4, kBlock), kBlock, 0, as_stream(stream)>>>(op, n);
  } else {
    stream_kernel<false, Op><<<stream_grid(n, kBlock), kBlock, 0, as_stream(stream)>>>(op, n);
  }
  GRACE_CHECK_LAUNCH(name);
  return GRACE_OK;
}

// t = beta*r + gamma*g, two roundings then the add (no contraction: -ffp-contract=off)
struct AxpbyOp {
  const float* r; const float* g; float beta, gamma; float* t;
  __device__ void vec(int64_t i) const {
    float4 a = reinterpret_cast<const float4*>(r)[i];
    float4 b = reinterpret_cast<const float4*>(g)[i];
    float4 o;
    o.x = beta * a.x + gamma * b.x; o.y = beta * a.y + gamma * b.y;
    o.z = beta * a.z + gamma * b.z; o.w = beta * a.w + gamma * b.w;
    reinterpret_cast<float4*>(t)[i] = o;
  }
  __device__ void one(int64_t i) const { t[i] = beta * r[i] + gamma * g[i]; }
};

struct SubOp {
  const float* a; const float* b; float* o;
  __device__ void vec(int64_t i) const {
    float4 x = reinterpret_cast<const float4*>(a)[i];
    float4 y = reinterpret_cast<const float4*>(b)[i];
    reinterpret_cast<float4*>(o)[i] = make_float4(x.x - y.x, x.y - y.y, x.z - y.z, x.w - y.w);
  }
  __device__ void one(int64_t i) const { o[i] = a[i] - b[i]; }
};

struct DivOp {
  const float* a; float d; float* o;
  __device__ void vec(int64_t i) const {
    float4 x = reinterpret_cast<const float4*>(a)[i];
    reinterpret_cast<float4*>(o)[i] = make_float4(x.x / d, x.y / d, x.z / d, x.w / d);
  }
  __device__ void one(int64_t i) const { o[i] = a[i] / d; }
};

struct AccOp {
  float* acc; const float* x; int first;
  __device__ void vec(int64_t i) const {
    float4 b = reinterpret_cast<const float4*>(x)[i];
    float4 a = first ? make_float4(0.f, 0.f, 0.f, 0.f) : reinterpret_cast<const float4*>(acc)[i];
    reinterpret_cast<float4*>(acc)[i] = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
  }
  __device__ void one(int64_t i) const { acc[i] = (first ? 0.f : acc[i]) + x[i]; }
};

struct FillOp {
  float v; float* o;
  __device__ void vec(int64_t i) const {   // write-only stream: non-temporal 16-B stores
    typedef float f4v __attribute__((ext_vector_type(4)));
    __builtin_nontemporal_store(f4v{v, v, v, v}, reinterpret_cast<f4v*>(o) + i);
  }
  __device__ void one(int64_t i) const { o[i] = v; }
};

__device__ __forceinline__ uint32_t pack_ge0(float4 x) {
  return (uint32_t)(x.x >= 0.f) | ((uint32_t)(x.y >= 0.f) << 8) | ((uint32_t)(x.z >= 0.f) << 16) |
         ((uint32_t)(x.w >= 0.f) << 24);
}

struct SignEncOp {
  const float* x; uint8_t* c;
  __device__ void vec(int64_t i) const {
    reinterpret_cast<uint32_t*>(c)[i] = pack_ge0(reinterpret_cast<const float4*>(x)[i]);
  }
  __device__ void one(int64_t i) const { c[i] = (uint8_t)(x[i] >= 0.f); }
};

// decode: (float)c * 2 - 1, then optional * scale (EF-signSGD multiplies mean * decode)
struct SignDecOp {
  const uint8_t* c; const float* scale; float* o;
  __device__ float dec(uint32_t b, float s, bool has_s) const {
    float v = (float)b * 2.0f - 1.0f;
    return has_s ? s * v : v;
  }
  __device__ void vec(int64_t i) const {
    uint32_t w = reinterpret_cast<const uint32_t*>(c)[i];
    const bool hs = scale != nullptr;
    const float s = hs ? scale[0] : 1.f;
    reinterpret_cast<float4*>(o)[i] = make_float4(dec(w & 0xFF, s, hs), dec((w >> 8) & 0xFF, s, hs),
                                                  dec((w >> 16) & 0xFF, s, hs), dec(w >> 24, s, hs));
  }
  __device__ void one(int64_t i) const {
    const bool hs = scale != nullptr;
    o[i] = dec(c[i], hs ? scale[0] : 1.f, hs);
  }
};

// majority: Python sum over ranks ((0 + d0) + d1 ...) then >= 0 -> +-1.  The partial sums of
// +-1 are small integers, exact in f32, so summing in rank order is trivially reproduced.
struct SignMajOp {
  const uint8_t* c; int world; int64_t n; float* o;
  __device__ void vec(int64_t i) const {
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    for (int w = 0; w < world; ++w) {
      uint32_t v = reinterpret_cast<const uint32_t*>(c + (int64_t)w * n)[i];
      s0 += (float)(v & 0xFF) * 2.f - 1.f; s1 += (float)((v >> 8) & 0xFF) * 2.f - 1.f;
      s2 += (float)((v >> 16) & 0xFF) * 2.f - 1.f; s3 += (float)(v >> 24) * 2.f - 1.f;
    }
    reinterpret_cast<float4*>(o)[i] = make_float4(s0 >= 0.f ? 1.f : -1.f, s1 >= 0.f ? 1.f : -1.f,
                                                  s2 >= 0.f ? 1.f : -1.f, s3 >= 0.f ? 1.f : -1.f);
  }
  __device__ void one(int64_t i) const {
    float s = 0.f;
    for (int w = 0; w < world; ++w) s += (float)c[(int64_t)w * n + i] * 2.f - 1.f;
    o[i] = s >= 0.f ? 1.f : -1.f;
  }
};

// Signum: m = (1-beta)*g + beta*m_prev.  The reference computes (1.0 - momentum) in double and
// torch casts both Python scalars to f32 before the multiplies; the caller passes beta and the
// kernel forms the same two f32 coefficients.
struct SignumOp {
  const float* g; float* m; int has_prev; float a, b; uint8_t* c;
  __device__ float upd(float gv, float mv) const { return has_prev ? a * gv + b * mv : gv; }
  __device__ void vec(int64_t i) const {
    float4 gv = reinterpret_cast<const float4*>(g)[i];
    float4 mv = has_prev ? reinterpret_cast<const float4*>(m)[i] : make_float4(0, 0, 0, 0);
    float4 o = make_float4(upd(gv.x, mv.x), upd(gv.y, mv.y), upd(gv.z, mv.z), upd(gv.w, mv.w));
    reinterpret_cast<float4*>(m)[i] = o;
    reinterpret_cast<uint32_t*>(c)[i] = pack_ge0(o);
  }
  __device__ void one(int64_t i) const {
    float o = upd(g[i], has_prev ? m[i] : 0.f);
    m[i] = o;
    c[i] = (uint8_t)(o >= 0.f);
  }
};

struct SignStepOp {
  const float* x; uint8_t* c; float* o;
  __device__ void vec(int64_t i) const {
    float4 v = reinterpret_cast<const float4*>(x)[i];
    if (c) reinterpret_cast<uint32_t*>(c)[i] = pack_ge0(v);   // codes optional (W=1 step)
    reinterpret_cast<float4*>(o)[i] =
        make_float4(v.x >= 0.f ? 1.f : -1.f, v.y >= 0.f ? 1.f : -1.f, v.z >= 0.f ? 1.f : -1.f,
                    v.w >= 0.f ? 1.f : -1.f);
  }
  __device__ void one(int64_t i) const {
    bool p = x[i] >= 0.f;
    if (c) c[i] = (uint8_t)p;
    o[i] = p ? 1.f : -1.f;
  }
};

// World-1 sign step without codes (the launch-bound 4 MiB configs[0] step): U float4 per thread,
// every load issued before any store (one HBM latency per thread), no grid-stride loop; the scalar
// tail (n % 4) is handled by the first workgroup.
#ifndef GRACE_SIGN_NT
#define GRACE_SIGN_NT 0
#endif
#ifndef GRACE_SIGN_BLOCK
#define GRACE_SIGN_BLOCK 256
#endif
constexpr int kSignBlock = GRACE_SIGN_BLOCK;
typedef float sf4v __attribute__((ext_vector_type(4)));
template <int U>
__global__ __launch_bounds__(kSignBlock) void sign_step_w1_kernel(const float* __restrict__ x, float* __restrict__ o,
                                                                 int64_t n) {
  const int64_t n4 = n >> 2;
  const int64_t base = (int64_t)blockIdx.x * kSignBlock * U + threadIdx.x;
  sf4v v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + (int64_t)u * kSignBlock;
    const sf4v* src = reinterpret_cast<const sf4v*>(x) + (i < n4 ? i : 0);
    if constexpr (GRACE_SIGN_NT & 1) v[u] = __builtin_nontemporal_load(src);
    else v[u] = *src;
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + (int64_t)u * kSignBlock;
    if (i < n4) {
      const sf4v r = {v[u].x >= 0.f ? 1.f : -1.f, v[u].y >= 0.f ? 1.f : -1.f, v[u].z >= 0.f ? 1.f : -1.f,
                      v[u].w >= 0.f ? 1.f : -1.f};
      if constexpr (GRACE_SIGN_NT & 2) __builtin_nontemporal_store(r, reinterpret_cast<sf4v*>(o) + i);
      else reinterpret_cast<sf4v*>(o)[i] = r;
    }
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    const int64_t i = (n4 << 2) + threadIdx.x;
    o[i] = x[i] >= 0.f ? 1.f : -1.f;
  }
}

// one-bit decode: mask0 * mean0 + notmask * mean1 (two products, then the add)
struct OneBitDecOp {
  const uint8_t* m; const float* mean0; const float* mean1; int quirk; float* o;
  __device__ float dec(uint32_t b, float m0, float m1) const {
    float nb = quirk ? (float)(255u - b) : (float)(1u - b);
    return (float)b * m0 + nb * m1;
  }
  __device__ void vec(int64_t i) const {
    const float m0 = mean0[0], m1 = mean1[0];
    uint32_t w = reinterpret_cast<const uint32_t*>(m)[i];
    reinterpret_cast<float4*>(o)[i] = make_float4(dec(w & 0xFF, m0, m1), dec((w >> 8) & 0xFF, m0, m1),
                                                  dec((w >> 16) & 0xFF, m0, m1), dec(w >> 24, m0, m1));
  }
  __device__ void one(int64_t i) const { o[i] = dec(m[i], mean0[0], mean1[0]); }
};

// ------------------------------------------------------------------------------------------------
// Reductions: block partials in f64 (deterministic order per block), then one finishing block
// that sums the partials in block order.  Used off the headline path (EF-sign mean, one-bit).
constexpr int kRedBlocks = 1024;

template <int K>
struct Partials { double v[K]; };

template <typename Acc>
__global__ __launch_bounds__(kBlock) void reduce_partials(const float* x, int64_t n, Acc acc,
                                                           double* part) {
  constexpr int K = Acc::K;
  double s[K];
#pragma unroll
  for (int j = 0; j < K; ++j) s[j] = 0.0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) acc.add(x[i], s);
  __shared__ double sh[K][kBlock / kWave];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    double v = wave_sum(s[j]);
    if ((threadIdx.x & 63) == 0) sh[j][threadIdx.x >> 6] = v;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int j = 0; j < K; ++j) {
      double t = 0.0;
      for (int w = 0; w < kBlock / kWave; ++w) t += sh[j][w];
      part[(int64_t)j * gridDim.x + blockIdx.x] = t;
    }
  }
}

template <typename Fin>
__global__ __launch_bounds__(kBlock) void reduce_finish(const double* part, int nparts, Fin fin) {
  constexpr int K = Fin::K;
  __shared__ double sh[K][kBlock];
  for (int j = 0; j < K; ++j) {
    double t = 0.0;
    for (int b = threadIdx.x; b < nparts; b += blockDim.x) t += part[(int64_t)j * nparts + b];
    sh[j][threadIdx.x] = t;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double tot[K];
    for (int j = 0; j < K; ++j) {
      double t = 0.0;
      for (int b = 0; b < kBlock; ++b) t += sh[j][b];
      tot[j] = t;
    }
    fin.finish(tot);
  }
}

struct AbsSumAcc {
  static constexpr int K = 1;
  __device__ void add(float v, double* s) const { s[0] += fabs((double)v); }
};
struct AbsMeanFin {
  static constexpr int K = 1;
  int64_t n; float* out;
  __device__ void finish(const double* t) const { out[0] = (float)t[0] / (float)n; }
};

// one-bit: sum0 over x<0, num0, sum1 over !(x<0) (NaN included, as ~mask0 in onebit.py:18)
struct OneBitAcc {
  static constexpr int K = 3;
  __device__ void add(float v, double* s) const {
    if (v < 0.f) { s[0] += (double)v; s[1] += 1.0; } else { s[2] += (double)v; }
  }
};
struct OneBitFin {
  static constexpr int K = 3;
  int64_t n; float* out;
  __device__ void finish(const double* t) const {
    const float sum0 = (float)t[0], num0 = (float)t[1], sum1 = (float)t[2];
    const float num1 = (float)n - num0;
    out[0] = num0 > 0.f ? sum0 / num0 : sum0;
    out[1] = num1 > 0.f ? sum1 / num1 : sum1;
  }
};

template <typename Acc, typename Fin>
static grace_status_t run_reduce(const char* name, const float* x, int64_t n, Acc acc, Fin fin,
                                 void* ws, void* stream) {
  const int blocks = (int)stream_grid(n, kBlock, kRedBlocks);
  double* part = reinterpret_cast<double*>(ws);
  reduce_partials<Acc><<<blocks, kBlock, 0, as_stream(stream)>>>(x, n, acc, part);
  GRACE_CHECK_LAUNCH(name);
  reduce_finish<Fin><<<1, kBlock, 0, as_stream(stream)>>>(part, blocks, fin);
  GRACE_CHECK_LAUNCH(name);
  return GRACE_OK;
}

// ------------------------------------------------------------------------------------------------
// HBM ceiling probe (bench.py's measured roofline): the headline step's dense traffic
// mix without any of its arithmetic -- read r, g; write r' = r + g and o = 0 -- with non-temporal
// 16-B loads and stores.  A family of pure streaming layouts; bench.py reports the fastest as the
// box's ceiling.  Variants 0-2: one chunk of 256 x 4 x VEC elements per 256-thread workgroup
// (VEC = 8 / 12 / 16 float4 per lane per array; 12 is the top-k main pass's residual layout), the
// lane's float4s loaded in groups of 4 with the next group in flight while the current one is
// stored; at most 4 workgroups per CU as the main pass.  Variants 3-5: a grid-stride loop over
// 1024 / 2048 / 4096 workgroups.  Chunk variants cover floor(n / chunk) chunks.
typedef float f32x4v __attribute__((ext_vector_type(4)));
template <int VEC>
__global__ __launch_bounds__(256, 4) void probe_2r2w_chunk(f32x4v* __restrict__ r, const f32x4v* __restrict__ g,
                                                          f32x4v* __restrict__ o) {
  constexpr int G = 4, NG = VEC / G;
  const int64_t base = (int64_t)blockIdx.x * (256 * VEC) + threadIdx.x;
  f32x4v a[G], b[G];
#pragma unroll
  for (int u = 0; u < G; ++u) {
    a[u] = __builtin_nontemporal_load(r + base + u * 256);
    b[u] = __builtin_nontemporal_load(g + base + u * 256);
  }
#pragma unroll
  for (int q = 0; q < NG; ++q) {
    f32x4v an[G], bn[G];
    if (q + 1 < NG) {
#pragma unroll
      for (int u = 0; u < G; ++u) {
        an[u] = __builtin_nontemporal_load(r + base + ((q + 1) * G + u) * 256);
        bn[u] = __builtin_nontemporal_load(g + base + ((q + 1) * G + u) * 256);
      }
    }
#pragma unroll
    for (int u = 0; u < G; ++u) {
      __builtin_nontemporal_store(a[u] + b[u], r + base + (q * G + u) * 256);
      __builtin_nontemporal_store(f32x4v{0.f, 0.f, 0.f, 0.f}, o + base + (q * G + u) * 256);
    }
    if (q + 1 < NG) {
#pragma unroll
      for (int u = 0; u < G; ++u) { a[u] = an[u]; b[u] = bn[u]; }
    }
  }
}
__global__ __launch_bounds__(256) void probe_2r2w_stride(f32x4v* __restrict__ r, const f32x4v* __restrict__ g,
                                                        f32x4v* __restrict__ o, int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const f32x4v a = __builtin_nontemporal_load(r + i), b = __builtin_nontemporal_load(g + i);
    __builtin_nontemporal_store(a + b, r + i);
    __builtin_nontemporal_store(f32x4v{0.f, 0.f, 0.f, 0.f}, o + i);
  }
}
// Variants 6-9: the encoders' mix (QSGD / TernGrad / natural compress: read f32, write one byte per
// element) -- read g, write o's bytes (the top byte of each element).  6 / 7: one chunk of
// 256 x 4 x VEC elements per workgroup (VEC 8 / 16), every load issued first; 8 / 9: grid-stride over
// 2048 / 4096 workgroups.
__device__ __forceinline__ uint32_t probe_pack(const f32x4v v) {
  return __builtin_amdgcn_perm(__builtin_amdgcn_perm(__float_as_uint(v.w), __float_as_uint(v.z), 0x0c0c0703u),
                               __builtin_amdgcn_perm(__float_as_uint(v.y), __float_as_uint(v.x), 0x0c0c0703u),
                               0x05040100u);
}
template <int VEC>
__global__ __launch_bounds__(256) void probe_4r1w_chunk(const f32x4v* __restrict__ g, uint32_t* __restrict__ o) {
  const int64_t base = (int64_t)blockIdx.x * (256 * VEC) + threadIdx.x;
  f32x4v a[VEC];
#pragma unroll
  for (int u = 0; u < VEC; ++u) a[u] = __builtin_nontemporal_load(g + base + u * 256);
#pragma unroll
  for (int u = 0; u < VEC; ++u) __builtin_nontemporal_store(probe_pack(a[u]), o + base + u * 256);
}
__global__ __launch_bounds__(256) void probe_4r1w_stride(const f32x4v* __restrict__ g, uint32_t* __restrict__ o,
                                                        int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256)
    __builtin_nontemporal_store(probe_pack(__builtin_nontemporal_load(g + i)), o + i);
}
constexpr int kProbeVariants = 10;
static int64_t probe_chunk(int variant) {
  return variant == 0 ? 8192 : variant == 1 ? 12288 : variant == 2 ? 16384 : variant == 6 ? 8192 : variant == 7 ? 16384 : 0;
}

}  // namespace grace

using namespace grace;

// ================================================================================================
extern "C" {

int grace_version(void) { return 100; }
const char* grace_last_error(void) { return g_err; }

grace_status_t grace_axpby(const float* r, const float* g, float beta, float gamma, float* t,
                           int64_t n, void* stream) {
  GRACE_REQUIRE(n >= 0 && r && g && t, "grace_axpby: bad arguments");
  return launch_stream("grace_axpby", AxpbyOp{r, g, beta, gamma, t}, n,
                       aligned16(r) && aligned16(g) && aligned16(t), stream);
}

grace_status_t grace_sub(const float* t, const float* d, float* r, int64_t n, void* stream) {
  GRACE_REQUIRE(n >= 0 && t && d && r, "grace_sub: bad arguments");
  return launch_stream("grace_sub", SubOp{t, d, r}, n, aligned16(t) && aligned16(d) && aligned16(r),
                       stream);
}

grace_status_t grace_div_scalar(const float* x, float divisor, float* out, int64_t n, void* stream) {
  GRACE_REQUIRE(n >= 0 && x && out, "grace_div_scalar: bad arguments");
  return launch_stream("grace_div_scalar", DivOp{x, divisor, out}, n, aligned16(x) && aligned16(out),
                       stream);
}

int64_t grace_hbm_probe_elems(int64_t n, int32_t variant) {
  if (variant < 0 || variant >= kProbeVariants || n < 0) return -1;
  const int64_t c = probe_chunk(variant);
  return c ? n / c * c : n / 4 * 4;
}

grace_status_t grace_hbm_probe(float* r, const float* g, float* o, int64_t n, int32_t variant, void* stream) {
  GRACE_REQUIRE(r && g && o && n >= 16384 && variant >= 0 && variant < kProbeVariants && aligned16(r) &&
                    aligned16(g) && aligned16(o),
                "grace_hbm_probe: bad arguments (n >= 16384, 16-B aligned buffers, variant 0..9)");
  f32x4v* r4 = reinterpret_cast<f32x4v*>(r);
  const f32x4v* g4 = reinterpret_cast<const f32x4v*>(g);
  f32x4v* o4 = reinterpret_cast<f32x4v*>(o);
  const hipStream_t s = as_stream(stream);
  const unsigned chunks = (unsigned)(grace_hbm_probe_elems(n, variant) / (probe_chunk(variant) ? probe_chunk(variant) : 1));
  switch (variant) {
    case 0: probe_2r2w_chunk<8><<<chunks, 256, 0, s>>>(r4, g4, o4); break;
    case 1: probe_2r2w_chunk<12><<<chunks, 256, 0, s>>>(r4, g4, o4); break;
    case 2: probe_2r2w_chunk<16><<<chunks, 256, 0, s>>>(r4, g4, o4); break;
    case 6: probe_4r1w_chunk<8><<<chunks, 256, 0, s>>>(g4, reinterpret_cast<uint32_t*>(o)); break;
    case 7: probe_4r1w_chunk<16><<<chunks, 256, 0, s>>>(g4, reinterpret_cast<uint32_t*>(o)); break;
    case 8: case 9: probe_4r1w_stride<<<2048u << (variant - 8), 256, 0, s>>>(g4, reinterpret_cast<uint32_t*>(o), n / 4); break;
    default: probe_2r2w_stride<<<1024u << (variant - 3), 256, 0, s>>>(r4, g4, o4, n / 4); break;
  }
  GRACE_CHECK_LAUNCH("grace_hbm_probe");
  return GRACE_OK;
}

// A fill is the runtime's 32-bit memset: it writes 256 MiB at 6.1 TB/s on MI355X against 4.6 TB/s for
// a grid-stride float4 kernel and 5.4 TB/s for one 16 KiB tile per workgroup (tools/write_probe.hip,
// profiles/r05_write_probe.txt) -- bit-identical, the word is the float's bits.
#ifndef GRACE_FILL_MEMSET
#define GRACE_FILL_MEMSET 1
#endif
grace_status_t grace_fill(float* x, float value, int64_t n, void* stream) {
  GRACE_REQUIRE(n >= 0 && x, "grace_fill: bad arguments");
  if (GRACE_FILL_MEMSET) {
    if (n == 0) return GRACE_OK;
    const hipError_t e = hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(x), (int)__builtin_bit_cast(uint32_t, value),
                                           (size_t)n, as_stream(stream));
    if (e != hipSuccess) { set_error("grace_fill", e); return GRACE_ERR_HIP; }
    return GRACE_OK;
  }
  return launch_stream("grace_fill", FillOp{value, x}, n, aligned16(x), stream);
}

grace_status_t grace_accumulate(float* acc, const float* x, int64_t n, int32_t first, void* stream) {
  GRACE_REQUIRE(n >= 0 && acc && x, "grace_accumulate: bad arguments");
  return launch_stream("grace_accumulate", AccOp{acc, x, first}, n, aligned16(acc) && aligned16(x),
                       stream);
}

grace_status_t grace_sign_encode(const float* x, uint8_t* codes, int64_t n, void* stream) {
  GRACE_REQUIRE(n >= 0 && x && codes, "grace_sign_encode: bad arguments");
  return launch_stream("grace_sign_encode", SignEncOp{x, codes}, n, aligned16(x) && aligned4(codes),
                       stream);
}

grace_status_t grace_sign_decode(const uint8_t* codes, const float* scale_dev, float* out, int64_t n,
                                 void* stream) {
  GRACE_REQUIRE(n >= 0 && codes && out, "grace_sign_decode: bad arguments");
  return launch_stream("grace_sign_decode", SignDecOp{codes, scale_dev, out}, n,
                       aligned4(codes) && aligned16(out), stream);
}

grace_status_t grace_sign_majority(const uint8_t* codes_wn, int32_t world, float* out, int64_t n,
                                   void* stream) {
  GRACE_REQUIRE(n >= 0 && world >= 1 && codes_wn && out, "grace_sign_majority: bad arguments");
  return launch_stream("grace_sign_majority", SignMajOp{codes_wn, world, n, out}, n,
                       aligned4(codes_wn) && (n % 4 == 0) && aligned16(out), stream);
}

grace_status_t grace_signum_encode(const float* g, float* momentum, int32_t has_prev, float coef_g,
                                   float coef_m, uint8_t* codes, int64_t n, void* stream) {
  GRACE_REQUIRE(n >= 0 && g && momentum && codes, "grace_signum_encode: bad arguments");
  return launch_stream("grace_signum_encode", SignumOp{g, momentum, has_prev, coef_g, coef_m, codes}, n,
                       aligned16(g) && aligned16(momentum) && aligned4(codes), stream);
}

grace_status_t grace_sign_step_w1(const float* x, uint8_t* codes, float* out, int64_t n, void* stream) {
  GRACE_REQUIRE(n >= 0 && x && out, "grace_sign_step_w1: bad arguments");
  if (!codes && n >= 4 && aligned16(x) && aligned16(out)) {
#ifndef GRACE_SIGN_U
#define GRACE_SIGN_U 1   // A/B over 200 steps: U = 1, 2 -> 5.1 us/step, U = 4 -> 5.7, U = 8 -> 5.5
#endif
    constexpr int U = GRACE_SIGN_U;
    const int64_t grid = ((n >> 2) + kSignBlock * U - 1) / (kSignBlock * U);
    sign_step_w1_kernel<U><<<(unsigned)grid, kSignBlock, 0, as_stream(stream)>>>(x, out, n);
    GRACE_CHECK_LAUNCH("grace_sign_step_w1");
    return GRACE_OK;
  }
  return launch_stream("grace_sign_step_w1", SignStepOp{x, codes, out}, n,
                       aligned16(x) && (!codes || aligned4(codes)) && aligned16(out), stream);
}

size_t grace_reduce_workspace_bytes(int64_t n) {
  (void)n;
  return sizeof(double) * 4 * kRedBlocks;
}

grace_status_t grace_abs_mean(const float* x, int64_t n, float* out_dev, void* ws, void* stream) {
  GRACE_REQUIRE(n > 0 && x && out_dev && ws, "grace_abs_mean: bad arguments");
  return run_reduce("grace_abs_mean", x, n, AbsSumAcc{}, AbsMeanFin{n, out_dev}, ws, stream);
}

grace_status_t grace_onebit_encode(const float* x, int64_t n, uint8_t* mask0, float* means_dev,
                                   void* ws, void* stream) {
  GRACE_REQUIRE(n > 0 && x && mask0 && means_dev && ws, "grace_onebit_encode: bad arguments");
  // mask0 = (x < 0) is the complement of (x >= 0) only for non-NaN; compute it directly
  struct LtOp {
    const float* x; uint8_t* c;
    __device__ void vec(int64_t i) const {
      float4 v = reinterpret_cast<const float4*>(x)[i];
      reinterpret_cast<uint32_t*>(c)[i] = (uint32_t)(v.x < 0.f) | ((uint32_t)(v.y < 0.f) << 8) |
                                           ((uint32_t)(v.z < 0.f) << 16) | ((uint32_t)(v.w < 0.f) << 24);
    }
    __device__ void one(int64_t i) const { c[i] = (uint8_t)(x[i] < 0.f); }
  };
  grace_status_t s = launch_stream("grace_onebit_encode", LtOp{x, mask0}, n,
                                   aligned16(x) && aligned4(mask0), stream);
  if (s != GRACE_OK) return s;
  return run_reduce("grace_onebit_encode", x, n, OneBitAcc{}, OneBitFin{n, means_dev}, ws, stream);
}

grace_status_t grace_onebit_decode(const uint8_t* mask0, const float* mean0_dev, const float* mean1_dev,
                                   int32_t quirk, float* out, int64_t n, void* stream) {
  GRACE_REQUIRE(n >= 0 && mask0 && mean0_dev && mean1_dev && out, "grace_onebit_decode: bad arguments");
  return launch_stream("grace_onebit_decode", OneBitDecOp{mask0, mean0_dev, mean1_dev, quirk, out}, n,
                       aligned4(mask0) && aligned16(out), stream);
}

}  // extern "C"
