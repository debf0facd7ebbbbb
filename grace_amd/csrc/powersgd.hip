// PowerSGD rank-r compression (grace_dl/dist/compressor/powersgd.py:7-65) for CDNA4.
//
//   P = M q        (n x m) . (m x r)  -- f32 MFMA v_mfma_f32_16x16x4_f32, K split over 8 waves
//   orthogonalize(P)                  -- modified Gram-Schmidt, one workgroup
//   Q = M^T P      (m x n) . (n x r)  -- f32 MFMA, rows split into slabs, deterministic reduce
//   out = P Q^T, residual = M - P Q^T -- one streaming pass (decompress + ResidualMemory update)
//
// At r = 4 the contractions are HBM-bound (2 flop per byte of M against an f32 ridge near 20), so
// the MFMA tiles use only r of their 16 columns and the kernels are sized for bandwidth: every
// load of M is a 16-B (float4) load and M is read exactly once per product.
#include <math.h>

#include "common.h"

namespace grace {

typedef float f32x4v __attribute__((ext_vector_type(4)));

constexpr int kPWaves = 8;                  // K split of P = M q
constexpr int kPBlock = kPWaves * kWave;
constexpr int kQWaves = 4;                  // 4 x 64 columns per workgroup of Q = M^T P
constexpr int kQBlock = kQWaves * kWave;
constexpr int kMaxRank = 16;

__device__ __forceinline__ f32x4v mfma4(float a, float b, f32x4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// ------------------------------------------------------------------------------------------------
// P[n x r] = M[n x m] q[m x r].  One workgroup per 16-row tile; wave w covers the K range
// [w*kspan, (w+1)*kspan) in steps of 16: lane l loads M[i0 + (l&15)][k + 4(l>>4) .. +3] (float4)
// and issues 4 MFMAs, MFMA s taking element s (the k-slice {k + 4g + s}) with the matching q rows.
template <bool VEC>
__global__ __launch_bounds__(kPBlock) void psgd_p_kernel(const float* __restrict__ M, int64_t n, int64_t m,
                                                        const float* __restrict__ q, int r,
                                                        float* __restrict__ P) {
  __shared__ float red[kPWaves][16][17];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t i0 = (int64_t)blockIdx.x * 16;
  const int64_t row = i0 + (lane & 15);
  const int g = lane >> 4;
  const int col = lane & 15;
  const int64_t ksteps = (m + 15) / 16;
  const int64_t per = (ksteps + kPWaves - 1) / kPWaves;
  const int64_t s0 = w * per, s1 = min(ksteps, s0 + per);
  f32x4v acc = {0.f, 0.f, 0.f, 0.f};
  for (int64_t st = s0; st < s1; ++st) {
    const int64_t k = st * 16 + 4 * g;
    float a[4];
    if (VEC && row < n && k + 3 < m) {
      const f32x4v v = __builtin_nontemporal_load(reinterpret_cast<const f32x4v*>(M + row * m + k));
      a[0] = v.x; a[1] = v.y; a[2] = v.z; a[3] = v.w;
    } else {
#pragma unroll
      for (int s = 0; s < 4; ++s) a[s] = (row < n && k + s < m) ? M[row * m + k + s] : 0.f;
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const float b = (col < r && k + s < m) ? q[(k + s) * r + col] : 0.f;
      acc = mfma4(a[s], b, acc);
    }
  }
  // D layout: col = lane & 15, row = (lane >> 4) * 4 + j
#pragma unroll
  for (int j = 0; j < 4; ++j) red[w][(lane >> 4) * 4 + j][lane & 15] = acc[j];
  __syncthreads();
  if (threadIdx.x < 16 * 16) {
    const int rr = threadIdx.x / 16, cc = threadIdx.x % 16;
    float s = 0.f;
#pragma unroll
    for (int ww = 0; ww < kPWaves; ++ww) s += red[ww][rr][cc];
    if (cc < r && i0 + rr < n) P[(i0 + rr) * r + cc] = s;
  }
}

// ------------------------------------------------------------------------------------------------
// Q partials: part[slab][m x r] = M[slab rows]^T P[slab rows].  Workgroup = 4 waves x 64 columns;
// per 4-row step lane l loads M[i + (l>>4)][j0 + 4(l&15) .. +3] (1 KB per wave-instruction) and
// issues 4 MFMAs (tile s = columns j0 + 4jj + s) against A = P^T[c = l&15][k = l>>4].
template <bool VEC>
__global__ __launch_bounds__(kQBlock) void psgd_qt_kernel(const float* __restrict__ M, int64_t n, int64_t m,
                                                         const float* __restrict__ P, int r, int64_t slab,
                                                         float* __restrict__ part) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t j0 = ((int64_t)blockIdx.x * kQWaves + w) * 64;
  const int64_t ilo = (int64_t)blockIdx.y * slab, ihi = min(n, ilo + slab);
  const int kk = lane >> 4, jj = lane & 15;
  const int64_t jc = j0 + 4 * jj;
  f32x4v acc[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) acc[s] = f32x4v{0.f, 0.f, 0.f, 0.f};
  if (j0 < m) {
    for (int64_t i = ilo; i < ihi; i += 4) {
      const int64_t row = i + kk;
      const bool rv = row < ihi;
      const float a = (rv && jj < r) ? P[row * r + jj] : 0.f;
      float b[4];
      if (VEC && rv && jc + 3 < m) {
        const f32x4v v = __builtin_nontemporal_load(reinterpret_cast<const f32x4v*>(M + row * m + jc));
        b[0] = v.x; b[1] = v.y; b[2] = v.z; b[3] = v.w;
      } else {
#pragma unroll
        for (int s = 0; s < 4; ++s) b[s] = (rv && jc + s < m) ? M[row * m + jc + s] : 0.f;
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) acc[s] = mfma4(a, b[s], acc[s]);
    }
  }
  // tile s, lane l, reg j: column j0 + 4 (l & 15) + s, rank row c = (l >> 4) * 4 + j
  float* pp = part + (int64_t)blockIdx.y * m * r;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int64_t j = j0 + 4 * (lane & 15) + s;
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) {
      const int c = (lane >> 4) * 4 + q4;
      if (j < m && c < r) pp[j * r + c] = acc[s][q4];
    }
  }
}

__global__ __launch_bounds__(256) void psgd_qreduce_kernel(const float* __restrict__ part, int64_t nslab,
                                                          int64_t mr, float* __restrict__ Q) {
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < mr; e += (int64_t)gridDim.x * 256) {
    float s = 0.f;
    for (int64_t sl = 0; sl < nslab; ++sl) s += part[sl * mr + e];
    Q[e] = s;
  }
}

// ------------------------------------------------------------------------------------------------
// Modified Gram-Schmidt on the columns of A[n x r] in place (powersgd.py:7-18): one workgroup,
// column norms and projections reduced in f64 through LDS.
__global__ __launch_bounds__(1024) void psgd_orth_kernel(float* __restrict__ A, int64_t n, int r) {
  __shared__ double sh[1024 / kWave][kMaxRank];
  __shared__ float sres[kMaxRank];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int c = 0; c < r; ++c) {
    double s = 0.0;
    for (int64_t i = threadIdx.x; i < n; i += 1024) {
      const double v = A[i * r + c];
      s += v * v;
    }
    s = wave_sum(s);
    if (lane == 0) sh[w][0] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
      double t = 0.0;
      for (int ww = 0; ww < 1024 / kWave; ++ww) t += sh[ww][0];
      sres[0] = sqrtf((float)t);
    }
    __syncthreads();
    const float norm = sres[0];
    for (int64_t i = threadIdx.x; i < n; i += 1024) A[i * r + c] = A[i * r + c] / norm;
    __syncthreads();
    if (c + 1 < r) {
      double d[kMaxRank];
      for (int c2 = c + 1; c2 < r; ++c2) d[c2] = 0.0;
      for (int64_t i = threadIdx.x; i < n; i += 1024) {
        const double col = A[i * r + c];
        for (int c2 = c + 1; c2 < r; ++c2) d[c2] += col * (double)A[i * r + c2];
      }
      for (int c2 = c + 1; c2 < r; ++c2) {
        const double t = wave_sum(d[c2]);
        if (lane == 0) sh[w][c2] = t;
      }
      __syncthreads();
      if (threadIdx.x < r && threadIdx.x > c) {
        double t = 0.0;
        for (int ww = 0; ww < 1024 / kWave; ++ww) t += sh[ww][threadIdx.x];
        sres[threadIdx.x] = (float)t;
      }
      __syncthreads();
      for (int64_t i = threadIdx.x; i < n; i += 1024) {
        const float col = A[i * r + c];
        for (int c2 = c + 1; c2 < r; ++c2) A[i * r + c2] = A[i * r + c2] - sres[c2] * col;
      }
      __syncthreads();
    }
  }
}

// ------------------------------------------------------------------------------------------------
// out = P Q^T (decompress, powersgd.py:58-65); optionally residual = M - out (PowerSGDMemory
// update, memory/powersgd.py:32-37) in the same pass.  Thread = 4 consecutive columns of a row.
template <bool VEC>
__global__ __launch_bounds__(256) void psgd_outer_kernel(const float* __restrict__ P, const float* __restrict__ Q,
                                                        int64_t n, int64_t m, int r, float* __restrict__ out,
                                                        const float* __restrict__ M, float* __restrict__ res) {
  const int64_t m4 = (m + 3) / 4;
  const int64_t total = n * m4;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
    const int64_t i = t / m4;
    const int64_t j = (t - i * m4) * 4;
    float o[4] = {0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < r; ++c) {
      const float p = P[i * r + c];
#pragma unroll
      for (int s = 0; s < 4; ++s)
        if (j + s < m) o[s] = o[s] + p * Q[(j + s) * r + c];
    }
    if (VEC && j + 3 < m) {
      if (out) __builtin_nontemporal_store(f32x4v{o[0], o[1], o[2], o[3]}, reinterpret_cast<f32x4v*>(out + i * m + j));
      if (res) {
        const f32x4v mv = __builtin_nontemporal_load(reinterpret_cast<const f32x4v*>(M + i * m + j));
        __builtin_nontemporal_store(f32x4v{mv.x - o[0], mv.y - o[1], mv.z - o[2], mv.w - o[3]},
                                    reinterpret_cast<f32x4v*>(res + i * m + j));
      }
    } else {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        if (j + s >= m) break;
        if (out) out[i * m + j + s] = o[s];
        if (res) res[i * m + j + s] = M[i * m + j + s] - o[s];
      }
    }
  }
}

// standard normal draws (Box-Muller on the counter-based generator), for q (powersgd.py:41)
__global__ __launch_bounds__(256) void normal_kernel(float* __restrict__ x, int64_t n, uint64_t seed) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const uint64_t h = mix64(seed ^ mix64((uint64_t)i * 2 + 1));
    const float u1 = ((float)(uint32_t)(h >> 40) + 1.0f) * (1.0f / 16777217.0f);   // (0, 1]
    const float u2 = (float)(uint32_t)(h & 0xFFFFFF) * (1.0f / 16777216.0f);
    x[i] = sqrtf(-2.0f * logf(u1)) * cosf(6.2831853071795864f * u2);
  }
}

}  // namespace grace

using namespace grace;

extern "C" {

grace_status_t grace_powersgd_p(const float* M, int64_t n, int64_t m, const float* q, int32_t r, float* P,
                                void* stream) {
  GRACE_REQUIRE(M && q && P && n >= 1 && m >= 1 && r >= 1 && r <= kMaxRank, "grace_powersgd_p: bad arguments");
  const bool vec = (m % 4 == 0) && ((reinterpret_cast<uintptr_t>(M) & 15u) == 0);
  const unsigned grid = (unsigned)((n + 15) / 16);
  if (vec) psgd_p_kernel<true><<<grid, kPBlock, 0, as_stream(stream)>>>(M, n, m, q, r, P);
  else psgd_p_kernel<false><<<grid, kPBlock, 0, as_stream(stream)>>>(M, n, m, q, r, P);
  GRACE_CHECK_LAUNCH("grace_powersgd_p");
  return GRACE_OK;
}

static int64_t qt_slabs(int64_t n, int64_t m) {
  const int64_t cgroups = (m + 255) / 256;
  int64_t s = 512 / cgroups;
  if (s < 1) s = 1;
  const int64_t maxs = (n + 3) / 4;
  return s < maxs ? s : maxs;
}

size_t grace_powersgd_workspace_bytes(int64_t n, int64_t m, int32_t r) {
  return sizeof(float) * (size_t)(qt_slabs(n, m) * m * r) + 256;
}

grace_status_t grace_powersgd_qt(const float* M, int64_t n, int64_t m, const float* P, int32_t r, float* Q,
                                 void* ws, void* stream) {
  GRACE_REQUIRE(M && P && Q && ws && n >= 1 && m >= 1 && r >= 1 && r <= kMaxRank,
                "grace_powersgd_qt: bad arguments");
  const int64_t ns = qt_slabs(n, m);
  int64_t slab = (n + ns - 1) / ns;
  slab = (slab + 3) / 4 * 4;
  const int64_t nslab = (n + slab - 1) / slab;
  const bool vec = (m % 4 == 0) && ((reinterpret_cast<uintptr_t>(M) & 15u) == 0);
  dim3 grid((unsigned)((m + 255) / 256), (unsigned)nslab);
  float* part = reinterpret_cast<float*>(ws);
  if (vec) psgd_qt_kernel<true><<<grid, kQBlock, 0, as_stream(stream)>>>(M, n, m, P, r, slab, part);
  else psgd_qt_kernel<false><<<grid, kQBlock, 0, as_stream(stream)>>>(M, n, m, P, r, slab, part);
  GRACE_CHECK_LAUNCH("grace_powersgd_qt");
  psgd_qreduce_kernel<<<stream_grid(m * r, 256, 1024), 256, 0, as_stream(stream)>>>(part, nslab, m * r, Q);
  GRACE_CHECK_LAUNCH("grace_powersgd_qt");
  return GRACE_OK;
}

grace_status_t grace_orthogonalize(float* A, int64_t n, int32_t r, void* stream) {
  GRACE_REQUIRE(A && n >= 1 && r >= 1 && r <= kMaxRank, "grace_orthogonalize: bad arguments");
  psgd_orth_kernel<<<1, 1024, 0, as_stream(stream)>>>(A, n, r);
  GRACE_CHECK_LAUNCH("grace_orthogonalize");
  return GRACE_OK;
}

grace_status_t grace_powersgd_outer(const float* P, const float* Q, int64_t n, int64_t m, int32_t r, float* out,
                                    const float* M, float* residual, void* stream) {
  GRACE_REQUIRE(P && Q && n >= 1 && m >= 1 && r >= 1 && (out || (M && residual)) && (!residual || M),
                "grace_powersgd_outer: bad arguments");
  const bool vec = (m % 4 == 0) &&
                   (((reinterpret_cast<uintptr_t>(out) | reinterpret_cast<uintptr_t>(M) |
                      reinterpret_cast<uintptr_t>(residual)) & 15u) == 0);
  const unsigned grid = stream_grid(n * ((m + 3) / 4), 256, 4096);
  if (vec) psgd_outer_kernel<true><<<grid, 256, 0, as_stream(stream)>>>(P, Q, n, m, r, out, M, residual);
  else psgd_outer_kernel<false><<<grid, 256, 0, as_stream(stream)>>>(P, Q, n, m, r, out, M, residual);
  GRACE_CHECK_LAUNCH("grace_powersgd_outer");
  return GRACE_OK;
}

grace_status_t grace_normal_fill(float* x, int64_t n, uint64_t seed, void* stream) {
  GRACE_REQUIRE(x && n >= 0, "grace_normal_fill: bad arguments");
  if (n == 0) return GRACE_OK;
  normal_kernel<<<stream_grid(n, 256, 1024), 256, 0, as_stream(stream)>>>(x, n, seed);
  GRACE_CHECK_LAUNCH("grace_normal_fill");
  return GRACE_OK;
}

}  // extern "C"
