// PowerSGD rank-r compression (grace_dl/dist/compressor/powersgd.py:7-65) for CDNA4.
//
//   P = M q        (n x m) . (m x r)  -- f32 MFMA v_mfma_f32_16x16x4_f32, K split over 8 waves
//   orthogonalize(P)                  -- Cholesky-QR in f64 (= MGS's Q), one workgroup
//   Q = M^T P      (m x n) . (n x r)  -- f32 MFMA, rows split into slabs, deterministic reduce
//   out = P Q^T, residual = M - P Q^T -- one streaming pass (decompress + ResidualMemory update)
//
// At r = 4 the contractions are HBM-bound (2 flop per byte of M against an f32 ridge near 20), so
// the MFMA tiles use only r of their 16 columns and the kernels are sized for bandwidth: every
// load of M is a 16-B (float4) load and M is read exactly once per product.
#include <math.h>

#include <atomic>

#include "common.h"

namespace grace {

typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef float f32x2v __attribute__((ext_vector_type(2)));

constexpr int kMaxRank = 16;

__device__ __forceinline__ f32x4v mfma4(float a, float b, f32x4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// ------------------------------------------------------------------------------------------------
// Workspace: [tickets u32 x kTickets | partials f32].  Split-K / split-row partial products are
// summed by the LAST workgroup to finish a tile (ticket counter), in a fixed order, so results
// are deterministic and no separate reduce launch is needed; that workgroup re-zeroes its ticket,
// so the workspace stays zeroed between calls.
constexpr int64_t kTickets = 65536;
constexpr size_t kTicketBytes = sizeof(uint32_t) * kTickets;

// Cross-workgroup partials.  The workgroups of one tile run on different XCDs, whose L2s are not
// coherent with each other, so the partials are written with agent-scope (sc1, write-through)
// stores and read back with agent-scope loads.  That makes the usual release/acquire fences --
// a full L2 writeback (buffer_wbl2) and invalidate (buffer_inv) per workgroup -- unnecessary:
// the ticket increment only has to wait for the workgroup's own partial stores (vmcnt(0)).
__device__ __forceinline__ void st_agent(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_agent(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// sum of p[0], p[stride], ... p[(cnt-1) stride] in that order, 8 loads in flight
__device__ __forceinline__ float sum_partials(const float* __restrict__ p, int64_t stride, int cnt) {
  float t = 0.f;
  int k = 0;
  for (; k + 8 <= cnt; k += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = ld_agent(p + (k + u) * stride);
#pragma unroll
    for (int u = 0; u < 8; ++u) t += v[u];
  }
  for (; k < cnt; ++k) t += ld_agent(p + k * stride);
  return t;
}

#ifdef GRACE_KFAN
constexpr int kFan = GRACE_KFAN;
#else
constexpr int kFan = 8;                     // slabs per first-level reduction group
#endif
#ifdef GRACE_PS_OCC
#define PS_OCC __attribute__((amdgpu_waves_per_eu(GRACE_PS_OCC, 8)))
#else
#define PS_OCC
#endif

// t[i] = sum over k < cnt (in order) of p[k * stride + f0 + threadIdx.x + i * 256], i < 4, for
// entries below `nent`; 4 x 8 loads in flight per round
__device__ __forceinline__ void sum_partials4(const float* __restrict__ p, int64_t stride, int cnt, int f0,
                                              int nent, float (&t)[4]) {
  int fi[4];
  bool ok[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    fi[i] = f0 + (int)threadIdx.x + i * 256;
    ok[i] = fi[i] < nent;
    t[i] = 0.f;
  }
  for (int k = 0; k < cnt; k += 8) {
    float v[4][8];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int u = 0; u < 8; ++u)
        v[i][u] = ld_agent(p + (k + u < cnt ? k + u : 0) * stride + (ok[i] ? fi[i] : 0));   // clamped, unconditional
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (k + u < cnt) t[i] += v[i][u];
  }
}

// 16-B write-through partials: buffer ops with the sc1 cache policy (common.h kSc1)
// elementwise sum over k < cnt (in order) of the 16-B runs at byte offset off + k * sb of `rs`,
// 8 loads in flight
__device__ __forceinline__ f32x4v sum_partials_v4(__amdgpu_buffer_rsrc_t rs, int sb, int cnt, int off) {
  f32x4v t = {0.f, 0.f, 0.f, 0.f};
  for (int k = 0; k < cnt; k += 8) {
    f32x4v v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, off + (k + u < cnt ? k + u : 0) * sb, 0, kSc1);
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (k + u < cnt) t += v[u];
  }
  return t;
}

// returns true in exactly one (the last-arriving) workgroup of the tile; every thread's partial
// stores (st_agent) are complete before the workgroup takes its ticket
__device__ __forceinline__ bool last_arrival(uint32_t* ticket, uint32_t expected) {
  __shared__ uint32_t s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = (t == expected - 1) ? 1u : 0u;
    if (s_last) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  return s_last != 0;
}

// standard normal draws: Box-Muller on the counter-based generator, one (cos, sin) pair per two
// consecutive elements; element e is component e & 1 of pair e >> 1 (normal_kernel, the generic and
// the rank-4 fused draws all produce the same stream)
__device__ __forceinline__ void normal_pair(uint64_t seed, uint64_t pair, float& z0, float& z1) {
  const uint64_t h = mix64(seed ^ mix64(pair * 2 + 1));
  const float u1 = ((float)(uint32_t)(h >> 40) + 1.0f) * (1.0f / 16777217.0f);   // (0, 1]
  const float u2 = (float)(uint32_t)(h & 0xFFFFFF) * (1.0f / 16777216.0f);
  // hardware transcendentals (v_log_f32 = log2, v_sin/v_cos_f32 take revolutions, v_sqrt_f32):
  // a few ulp, irrelevant for a random draw, and ~5x fewer instructions than the correctly
  // rounded libm calls -- the fused draw runs on one workgroup, so they were 4 us of its 9
  const float rad = __builtin_amdgcn_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u1));   // -2 ln 2 log2(u1)
  z0 = rad * __builtin_amdgcn_cosf(u2);
  z1 = rad * __builtin_amdgcn_sinf(u2);
}
__device__ __forceinline__ float normal_at(uint64_t seed, uint64_t i) {
  float z0, z1;
  normal_pair(seed, i >> 1, z0, z1);
  return (i & 1) ? z1 : z0;
}

// ------------------------------------------------------------------------------------------------
// Both contractions stream M through LDS in tiles of 16 rows x 256·CPL columns: every global load
// is one row's 1 KB contiguous run (64 lanes x 16 B) and a lane's CPL loads of a row
// are adjacent, so a wave reads CPL KB of each row back to back (wide runs keep DRAM pages open:
// 1-KB runs at a 16-KB row stride read at about half the rate of 4-KB runs).  The next tile's loads
// are in flight while the MFMAs consume the current one, and the MFMA operand reads come from LDS
// (rows padded by 4 floats so the 16-row operand reads spread over the banks).
constexpr int kTileR = 16;
constexpr int kPW = 4;                      // waves per workgroup (both kernels)
constexpr int kPBlockT = kPW * kWave;
#ifdef GRACE_TILE_CPL
constexpr int kCPL = GRACE_TILE_CPL;        // columns per lane / 4 of the streamed tiles
#else
constexpr int kCPL = 1;
#endif
template <int CPL> struct Tile {
  static constexpr int C = 256 * CPL;       // tile columns
  static constexpr int LD = C + 4;          // padded LDS row
};

// prefetch tile (row0, col0) of M into registers: wave w loads rows w, w+4, w+8, w+12, each as CPL
// consecutive 1-KB runs
template <int CPL, bool VEC>
__device__ __forceinline__ void tile_load(const float* __restrict__ M, int64_t n, int64_t m, int64_t rlo,
                                          int64_t rhi, int64_t row0, int64_t col0, f32x4v (&pre)[4 * CPL]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t row = row0 + w + 4 * j;
    const bool rv = row >= rlo && row < rhi && row < n;
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      const int64_t col = col0 + 256 * c + 4 * lane;
      if (VEC) {
        const int64_t rc = rv ? row : rlo;
        const int64_t cc = col < m ? col : m - 4;
        // plain (cache-allocating) load: P's pass leaves part of M in the MALL for Qt's re-read
        // (A/B with 5 rotated 64 MiB matrices: step 67.2 -> 65.9 us against non-temporal loads)
        const f32x4v v = *reinterpret_cast<const f32x4v*>(M + rc * m + cc);
        const bool in = rv && col < m;
        pre[j * CPL + c] = in ? v : f32x4v{0.f, 0.f, 0.f, 0.f};
      } else {
        f32x4v v;
        v.x = (rv && col + 0 < m) ? M[row * m + col + 0] : 0.f;
        v.y = (rv && col + 1 < m) ? M[row * m + col + 1] : 0.f;
        v.z = (rv && col + 2 < m) ? M[row * m + col + 2] : 0.f;
        v.w = (rv && col + 3 < m) ? M[row * m + col + 3] : 0.f;
        pre[j * CPL + c] = v;
      }
    }
  }
}

template <int CPL>
__device__ __forceinline__ void tile_store(float (*tile)[Tile<CPL>::LD], const f32x4v (&pre)[4 * CPL]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int c = 0; c < CPL; ++c)
      *reinterpret_cast<f32x4v*>(&tile[w + 4 * j][256 * c + 4 * lane]) = pre[j * CPL + c];
}

// prefetch `cnt` rows [row0, row0 + cnt) of a small row-major [rows x r] factor (q or P) as a
// flat run of cnt * r floats, zero past row `rhi`; thread t holds flat entries t, t + 256, ...
template <int PER>
__device__ __forceinline__ void fac_load(const float* __restrict__ F, int r, int64_t row0, int64_t rhi, int cnt,
                                         float (&pre)[PER]) {
  const int64_t total = (int64_t)cnt * r;
  const int64_t lim = (rhi - row0) * r;        // valid flat entries
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int64_t e = threadIdx.x + (int64_t)j * kPBlockT;
    const bool ok = e < total && e < lim;
    const float v = F[row0 * r + (ok ? e : 0)];
    pre[j] = ok ? v : 0.f;
  }
}
template <int PER>
__device__ __forceinline__ void fac_store(float* fs, int r, int cnt, const float (&pre)[PER]) {
  const int total = cnt * r;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int e = threadIdx.x + j * kPBlockT;
    if (e < total) fs[e] = pre[j];
  }
}
// rank 4: thread t holds rows row0 + t + 256 c (c < CPL) of a [rows x 4] factor, one 16-B load each
// (zero past `rhi`)
template <int CPL>
__device__ __forceinline__ void fac_load_r4(const float* __restrict__ F, int64_t row0, int64_t rhi,
                                            f32x4v (&pre)[CPL]) {
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int64_t row = row0 + threadIdx.x + 256 * c;
    const f32x4v v = *reinterpret_cast<const f32x4v*>(F + 4 * (row < rhi ? row : row0));
    pre[c] = row < rhi ? v : f32x4v{0.f, 0.f, 0.f, 0.f};
  }
}
// the same rows of a fresh standard-normal [rows x 4] factor, drawn instead of loaded: entry
// (row, c) = element row * 4 + c of the normal_kernel stream, i.e. Box-Muller pairs 2 row, 2 row + 1
template <int CPL>
__device__ __forceinline__ void fac_draw_r4(uint64_t seed, int64_t row0, int64_t rhi, f32x4v (&pre)[CPL]) {
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int64_t row = row0 + threadIdx.x + 256 * c;
    float z0, z1, z2, z3;
    normal_pair(seed, (uint64_t)row * 2, z0, z1);
    normal_pair(seed, (uint64_t)row * 2 + 1, z2, z3);
    pre[c] = row < rhi ? f32x4v{z0, z1, z2, z3} : f32x4v{0.f, 0.f, 0.f, 0.f};
  }
}
template <int PER>
__device__ __forceinline__ void fac_draw(uint64_t seed, int r, int64_t row0, int64_t rhi, int cnt, float (&pre)[PER]) {
  const int64_t total = (int64_t)cnt * r;
  const int64_t lim = (rhi - row0) * r;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int64_t e = threadIdx.x + (int64_t)j * kPBlockT;
    pre[j] = (e < total && e < lim) ? normal_at(seed, (uint64_t)(row0 * r + e)) : 0.f;
  }
}
constexpr int kPPer = kTileR * kMaxRank / kPBlockT;   // 1: P rows of one row tile

// ------------------------------------------------------------------------------------------------
// P[n x r] = M[n x m] q[m x r].  Grid = (K chunks, 16-row tiles).  Per tile wave w owns columns
// [64·CPL·w, 64·CPL·(w + 1)): per 16-wide k-step lane l reads A = M[l&15][k + 4(l>>4) .. +3] and
// B = the matching q rows from LDS and issues 4 MFMAs (MFMA s = k-slice {k + 4g + s}).  The only
// global loads in the loop are the NEXT tile's (M and its q rows), so they overlap the MFMAs
// instead of being serialised behind in-loop loads.  The 4 waves and the K chunks are reduced
// deterministically (LDS, then the last workgroup of the row tile).  R4: q staged as 16-B rows,
// wide tiles; otherwise one 1-KB run per row and flat scalar q staging.
// DRAWQ: q is not read but drawn on the fly (standard normal, counter-based, keyed by `seed`; the
// same values grace_normal_fill writes), so PowerSGD's fresh q needs no buffer and no launch.
template <bool VEC, bool R4, bool DRAWQ = false>
__global__ __launch_bounds__(kPBlockT) PS_OCC void psgd_p_kernel(const float* __restrict__ M, int64_t n, int64_t m,
                                                         const float* __restrict__ q, int r,
                                                         float* __restrict__ P, float* __restrict__ part,
                                                         uint32_t* __restrict__ tickets, uint64_t seed = 0) {
  constexpr int CPL = R4 ? kCPL : 1;
  constexpr int TC = Tile<CPL>::C;
  constexpr int QPER = TC * kMaxRank / kPBlockT;
  __shared__ float tile[kTileR][Tile<CPL>::LD];
  __shared__ float qs[TC * (R4 ? 4 : kMaxRank)];
  __shared__ float red[kPW][16][17];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int ks = blockIdx.x, nks = gridDim.x;
  const int64_t rt = blockIdx.y;
  const int64_t i0 = rt * kTileR;
  const int g = lane >> 4;
  const int col = lane & 15;
  const int64_t nkt = (m + TC - 1) / TC;
  const int64_t per = (nkt + nks - 1) / nks;
  const int64_t kt0 = ks * per, kt1 = min(nkt, kt0 + per);
  f32x4v acc = {0.f, 0.f, 0.f, 0.f};
  f32x4v pre[4 * CPL];
  float qpre[R4 ? 1 : QPER];
  f32x4v q4[CPL];
  auto q_tile = [&](int64_t row0) {
    if constexpr (R4) {
      if constexpr (DRAWQ) fac_draw_r4<CPL>(seed, row0, m, q4);
      else fac_load_r4<CPL>(q, row0, m, q4);
    } else {
      if constexpr (DRAWQ) fac_draw(seed, r, row0, m, TC, qpre);
      else fac_load(q, r, row0, m, TC, qpre);
    }
  };
  if (kt0 < kt1) {
    tile_load<CPL, VEC>(M, n, m, i0, i0 + kTileR, i0, kt0 * TC, pre);
    q_tile(kt0 * TC);
  }
  for (int64_t kt = kt0; kt < kt1; ++kt) {
    tile_store<CPL>(tile, pre);
    if constexpr (R4) {
#pragma unroll
      for (int c = 0; c < CPL; ++c) *reinterpret_cast<f32x4v*>(&qs[4 * (threadIdx.x + 256 * c)]) = q4[c];
    } else {
      fac_store(qs, r, TC, qpre);
    }
    __syncthreads();
    if (kt + 1 < kt1) {
      tile_load<CPL, VEC>(M, n, m, i0, i0 + kTileR, i0, (kt + 1) * TC, pre);
      q_tile((kt + 1) * TC);
    }
#pragma unroll
    for (int st = 0; st < 4 * CPL; ++st) {
      const int kl = 64 * CPL * w + 16 * st + 4 * g;
      const f32x4v av = *reinterpret_cast<const f32x4v*>(&tile[lane & 15][kl]);
      if constexpr (R4) {
#pragma unroll
        for (int s = 0; s < 4; ++s) acc = mfma4(av[s], col < 4 ? qs[(kl + s) * 4 + col] : 0.f, acc);
      } else {
#pragma unroll
        for (int s = 0; s < 4; ++s) acc = mfma4(av[s], col < r ? qs[(kl + s) * r + col] : 0.f, acc);
      }
    }
    __syncthreads();
  }
  // D layout: col = lane & 15, row = (lane >> 4) * 4 + j
#pragma unroll
  for (int j = 0; j < 4; ++j) red[w][(lane >> 4) * 4 + j][lane & 15] = acc[j];
  __syncthreads();
  const int rr = threadIdx.x / 16, cc = threadIdx.x % 16;   // 256 threads = the 16 x 16 tile
  float sum = 0.f;
#pragma unroll
  for (int ww = 0; ww < kPW; ++ww) sum += red[ww][rr][cc];
  const bool valid = cc < r && i0 + rr < n;
  if (nks == 1) {
    if (valid) P[(i0 + rr) * r + cc] = sum;
    return;
  }
  if constexpr (R4) {
    // rank 4: the tile's 16 x 4 partial is 16 rows of 16 B, written through (sc1) and summed as
    // 16-B runs by the last K chunk to arrive (same per-entry order as the scalar path)
    __syncthreads();
    float* stg = &tile[0][0];
    if (cc < 4) stg[rr * 4 + cc] = sum;
    __syncthreads();
    const int64_t rows = min((int64_t)kTileR, n - i0);
    const int sb = (int)(n * 4 * sizeof(float));
    if (threadIdx.x < rows) {
      const auto rs = __builtin_amdgcn_make_buffer_rsrc(part + ((int64_t)ks * n + i0) * 4, (short)0,
                                                        (int)(rows * 16), 0x00020000);
      __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const f32x4v*>(&stg[4 * threadIdx.x]), rs,
                                             threadIdx.x * 16, 0, kSc1);
    }
    if (!last_arrival(tickets + rt, (uint32_t)nks)) return;
    if (threadIdx.x < rows) {
      const auto rs = __builtin_amdgcn_make_buffer_rsrc(part + i0 * 4, (short)0, sb * (nks - 1) + (int)(rows * 16),
                                                        0x00020000);
      *reinterpret_cast<f32x4v*>(P + (i0 + threadIdx.x) * 4) = sum_partials_v4(rs, sb, nks, threadIdx.x * 16);
    }
    return;
  }
  if (valid) st_agent(part + ((int64_t)ks * n + i0 + rr) * r + cc, sum);
  if (!last_arrival(tickets + rt, (uint32_t)nks)) return;
  if (valid) P[(i0 + rr) * r + cc] = sum_partials(part + (i0 + rr) * r + cc, (int64_t)n * r, nks);
}

// The slabs' [TC columns x r] results (staged in LDS as stg[column * r + rank]) are reduced over
// the slabs in two fixed-order levels (groups of kFan slabs, then the groups), each by the last
// workgroup to arrive; the partials travel as 16-B write-through runs.  Grid = (column groups of TC,
// slabs).
template <int TC, int BLOCK = kPBlockT>
__device__ __forceinline__ void qt_reduce_slabs(const float* stg, int64_t m, int r, int64_t j0, int64_t cg,
                                                float* __restrict__ Q, float* __restrict__ part,
                                                uint32_t* __restrict__ tickets) {
  const int nslab = gridDim.y;
  const int64_t ncol = min((int64_t)TC, m - j0);
  const int nent = (int)(ncol * r);
  if (nslab == 1) {
    for (int f = threadIdx.x; f < nent; f += BLOCK) Q[j0 * r + f] = stg[f];
    return;
  }
  const int64_t sstride = (int64_t)m * r;
  // 16-B write-through runs when every slab's run is 16-B aligned and short enough for 32-bit offsets
  const bool v4 = (nent % 4) == 0 && (sstride % 4) == 0 && (((reinterpret_cast<uintptr_t>(part) | reinterpret_cast<uintptr_t>(Q)) & 15u) == 0) &&
                  sstride * (int64_t)sizeof(float) * kFan < (1ll << 31) &&
                  sstride * (int64_t)sizeof(float) * ((nslab + kFan - 1) / kFan) < (1ll << 31);
  float* mine = part + (int64_t)blockIdx.y * sstride + j0 * r;
  if (v4) {
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(mine, (short)0, nent * (int)sizeof(float), 0x00020000);
    for (int f4 = threadIdx.x; f4 < nent / 4; f4 += BLOCK)
      __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const f32x4v*>(&stg[4 * f4]), rs, f4 * 16, 0, kSc1);
  } else {
    for (int f = threadIdx.x; f < nent; f += BLOCK) st_agent(mine + f, stg[f]);
  }
  // two-level deterministic reduction over the slabs: groups of kFan slabs, then the groups
  const int ngroups = (nslab + kFan - 1) / kFan;
  const int sg = blockIdx.y / kFan;
  const int in_group = min(kFan, nslab - sg * kFan);
  if (!last_arrival(tickets + cg * ngroups + sg, (uint32_t)in_group)) return;
  float* part2 = part + (int64_t)nslab * m * r;
  if (v4) {
    const float* src = part + ((int64_t)sg * kFan) * sstride + j0 * r;
    const int sb = (int)(sstride * sizeof(float));
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(src), (short)0,
                                                      sb * (in_group - 1) + nent * (int)sizeof(float), 0x00020000);
    const auto rd = __builtin_amdgcn_make_buffer_rsrc(part2 + (int64_t)sg * sstride + j0 * r, (short)0,
                                                      nent * (int)sizeof(float), 0x00020000);
    for (int f4 = threadIdx.x; f4 < nent / 4; f4 += BLOCK) {
      const f32x4v t = sum_partials_v4(rs, sb, in_group, f4 * 16);
      if (ngroups == 1) *reinterpret_cast<f32x4v*>(Q + j0 * r + 4 * f4) = t;
      else __builtin_amdgcn_raw_buffer_store_b128(t, rd, f4 * 16, 0, kSc1);
    }
    if (ngroups == 1) return;
    if (!last_arrival(tickets + kTickets / 2 + cg, (uint32_t)ngroups)) return;
    const auto r2 = __builtin_amdgcn_make_buffer_rsrc(part2 + j0 * r, (short)0,
                                                      sb * (ngroups - 1) + nent * (int)sizeof(float), 0x00020000);
    for (int f4 = threadIdx.x; f4 < nent / 4; f4 += BLOCK)
      *reinterpret_cast<f32x4v*>(Q + j0 * r + 4 * f4) = sum_partials_v4(r2, sb, ngroups, f4 * 16);
    return;
  }
  // the group's entries are one contiguous run of (columns x r) floats per slab; each thread
  // sums up to 4 of them at once so all of their partial loads are in flight together
  for (int f0 = 0; f0 < nent; f0 += 4 * BLOCK) {
    float t[4];
    sum_partials4(part + ((int64_t)sg * kFan) * sstride + j0 * r, sstride, in_group, f0, nent, t);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int f = f0 + threadIdx.x + i * BLOCK;
      if (f < nent) {
        if (ngroups == 1) Q[j0 * r + f] = t[i];
        else st_agent(part2 + (int64_t)sg * sstride + j0 * r + f, t[i]);
      }
    }
  }
  if (ngroups == 1) return;
  if (!last_arrival(tickets + kTickets / 2 + cg, (uint32_t)ngroups)) return;
  for (int f0 = 0; f0 < nent; f0 += 4 * BLOCK) {
    float t[4];
    sum_partials4(part2 + j0 * r, sstride, ngroups, f0, nent, t);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int f = f0 + threadIdx.x + i * BLOCK;
      if (f < nent) Q[j0 * r + f] = t[i];
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Q = M^T P.  Grid = (256·CPL-column groups, row slabs).  Per 16-row tile wave w owns columns
// [64·CPL·w, 64·CPL·(w + 1)) of the group: per 4-row step lane l reads B = M[4st + (l>>4)][64·CPL·w
// + 64c + 4(l&15) .. +3] and A = P^T[c = l&15][row] from LDS and issues 4 MFMAs per 64-column
// block c (tile 4c + s = columns 64c + 4jj + s).  As in P, the loop's only global loads are the
// next tile's (M rows and their P rows).  The slabs are reduced in two fixed-order levels (groups
// of kFan slabs, then the groups), each by the last workgroup to arrive.
template <bool VEC>
__global__ __launch_bounds__(kPBlockT) PS_OCC void psgd_qt_kernel(const float* __restrict__ M, int64_t n, int64_t m,
                                                          const float* __restrict__ P, int r, int64_t slab,
                                                          float* __restrict__ Q, float* __restrict__ part,
                                                          uint32_t* __restrict__ tickets) {
  constexpr int CPL = kCPL;
  constexpr int TC = Tile<CPL>::C;
  __shared__ float tile[kTileR][Tile<CPL>::LD];
  __shared__ float ps[kTileR * kMaxRank];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t cg = blockIdx.x;
  const int64_t j0 = cg * TC;
  const int64_t ilo = (int64_t)blockIdx.y * slab, ihi = min(n, ilo + slab);
  const int kk = lane >> 4, jj = lane & 15;
  f32x4v acc[4 * CPL];
#pragma unroll
  for (int s = 0; s < 4 * CPL; ++s) acc[s] = f32x4v{0.f, 0.f, 0.f, 0.f};
  f32x4v pre[4 * CPL];
  float ppre[kPPer];
  if (ilo < ihi) {
    tile_load<CPL, VEC>(M, n, m, ilo, ihi, ilo, j0, pre);
    fac_load(P, r, ilo, ihi, kTileR, ppre);
  }
  for (int64_t i = ilo; i < ihi; i += kTileR) {
    tile_store<CPL>(tile, pre);
    fac_store(ps, r, kTileR, ppre);
    __syncthreads();
    if (i + kTileR < ihi) {
      tile_load<CPL, VEC>(M, n, m, ilo, ihi, i + kTileR, j0, pre);
      fac_load(P, r, i + kTileR, ihi, kTileR, ppre);
    }
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      const int rl = 4 * st + kk;
      const float a = jj < r ? ps[rl * r + jj] : 0.f;
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        const f32x4v bv = *reinterpret_cast<const f32x4v*>(&tile[rl][64 * CPL * w + 64 * c + 4 * jj]);
#pragma unroll
        for (int s = 0; s < 4; ++s) acc[4 * c + s] = mfma4(a, bv[s], acc[4 * c + s]);
      }
    }
    __syncthreads();
  }
  // the slab's [TC columns x r] result goes through LDS (the tile is free after the loop's last
  // barrier) so that it leaves as flat 16-B runs: tile 4c + s, lane l, reg q4 is column
  // 64·CPL·w + 64c + 4 (l & 15) + s of the group, rank row (l >> 4) * 4 + q4
  static_assert(TC * kMaxRank <= kTileR * Tile<CPL>::LD, "staging fits the tile");
  float* stg = &tile[0][0];
#pragma unroll
  for (int c = 0; c < CPL; ++c)
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int jl = 64 * CPL * w + 64 * c + 4 * (lane & 15) + s;
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4) {
        const int cr = (lane >> 4) * 4 + q4;
        if (cr < r) stg[jl * r + cr] = acc[4 * c + s][q4];
      }
    }
  __syncthreads();
  qt_reduce_slabs<TC>(stg, m, r, j0, cg, Q, part, tickets);
}

// Rank-4 Q = M^T P on the vector ALUs (4 FMAs per element of M: the contraction needs no matrix
// cores).  A 1024-thread workgroup owns 1024 columns and a slab of rows: column wave cw = w & 3
// holds the 256 columns [256cw, 256cw + 256) (one 16-B quad per lane per row, so the workgroup
// reads 4 KB of each row) and row wave rw = w >> 2 a quarter of the slab.  Every lane issues kQ4D
// rows' loads before any is used (no LDS, no barriers in the loop) and accumulates its 4 columns x
// 4 ranks in registers, row by row in order; P's row is a wave-uniform 16-B load.  The 4 row waves
// are summed in LDS in a fixed order, then the slabs as in psgd_qt_kernel.  The big workgroups
// exist for that last step: the slab reduction was the kernel's critical path (streaming alone:
// ~9 us; with 512 small workgroups' partials, 22 us), and 4x fewer slabs make it one round of
// loads per level.
constexpr int kQ4C = 1024;
constexpr int kQ4D = 16;
constexpr int kQ4Block = 1024;
__global__ __launch_bounds__(kQ4Block) void psgd_qt4_kernel(const float* __restrict__ M, int64_t n, int64_t m,
                                                           const float* __restrict__ P, int64_t slab,
                                                           float* __restrict__ Q, float* __restrict__ part,
                                                           uint32_t* __restrict__ tickets) {
  __shared__ float stg[kQ4C * 4];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int cw = w & 3, rw = w >> 2;
  const int64_t cg = blockIdx.x, j0 = cg * kQ4C;
  const int64_t jc = j0 + 256 * cw + 4 * lane;       // this lane's 4 columns (m % 4 == 0)
  const float* mp = M + (jc < m ? jc : 0);
  const int64_t slo = (int64_t)blockIdx.y * slab, shi = min(n, slo + slab);
  const int64_t quarter = slab / 4;                   // slab is a multiple of 4 * kQ4D
  const int64_t ilo = min(shi, slo + rw * quarter), ihi = min(shi, ilo + quarter);
  float acc[4][4];
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[s][c] = 0.f;
  for (int64_t i = ilo; i < ihi; i += kQ4D) {
    f32x4v v[kQ4D];
#pragma unroll
    for (int d = 0; d < kQ4D; ++d) {
      const int64_t row = i + d < ihi ? i + d : ilo;  // unconditional loads: a clamped row stands in
      v[d] = *reinterpret_cast<const f32x4v*>(mp + row * m);
    }
#pragma unroll
    for (int d = 0; d < kQ4D; ++d) {
      if (i + d < ihi) {
        const f32x4v pr = *reinterpret_cast<const f32x4v*>(P + (i + d) * 4);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int c = 0; c < 4; ++c) acc[s][c] = fmaf(v[d][s], pr[c], acc[s][c]);
      }
    }
  }
  // row waves 0, 1, 2, 3 in order: column jl = 256cw + 4 lane + s, rank c -> stg[jl * 4 + c]
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (rw == q) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        f32x4v* dst = reinterpret_cast<f32x4v*>(&stg[(256 * cw + 4 * lane + s) * 4]);
        const f32x4v mine = f32x4v{acc[s][0], acc[s][1], acc[s][2], acc[s][3]};
        *dst = q == 0 ? mine : *dst + mine;
      }
    }
    __syncthreads();
  }
#ifdef GRACE_QT4_NORED   // diagnostic A/B build only: no slab reduction (wrong Q)
  if (blockIdx.y == 0) for (int f = threadIdx.x; f < kQ4C * 4 && j0 * 4 + f < m * 4; f += kQ4Block) Q[j0 * 4 + f] = stg[f];
  return;
#endif
  qt_reduce_slabs<kQ4C, kQ4Block>(stg, m, 4, j0, cg, Q, part, tickets);
}

// ------------------------------------------------------------------------------------------------
// orthogonalize(A[n x r]) in place (powersgd.py:7-18), one workgroup, as Cholesky-QR in f64:
//   G = A^T A (f64 accumulation of the f32 entries, one read of A)
//   R = chol(G)  (upper, positive diagonal)  -- the R of modified Gram-Schmidt
//   A <- A R^-1  (row-wise forward substitution in f64, one write of A)
// In exact arithmetic this is the reference's MGS result.  One Cholesky-QR pass loses
// orthogonality like kappa(A)^2 * eps64, so the Cholesky pivots are checked: when the smallest
// relative pivot d_c / G_cc falls below kOrthPivotMin (kappa(A) above ~1e4), or a pivot is not
// finite, the workgroup switches to modified Gram-Schmidt with re-orthogonalisation in f64
// (orth_mgs2, below).  That returns the exact QR factor of the f32 input to ~1e-7 for ANY
// input, including near-rank-deficient ones (P = M q of a low-rank gradient), where the
// reference's f32 MGS itself is only determined to ~kappa * eps32.  A column that is EXACTLY
// dependent (residual exactly 0) comes out as zeros, where the reference's 0/0 gives NaN
// (DESIGN.md section 2).
constexpr int kOrthBlock = 1024;
constexpr double kOrthPivotMin = 1e-8;

// Robust path: MGS2 (every column projected twice against the finished ones, then normalised).
// Register version: the rows a thread holds (row threadIdx.x + j * kOrthBlock) stay in f64
// registers for the whole factorisation, so the result is the exact factor of the f32 input to
// f64 accuracy; only the dot products meet in LDS.
template <int R, int ROWS>
__device__ void orth_mgs2_regs(double (&x)[ROWS][R], int r) {
  constexpr int NW = kOrthBlock / kWave;
  __shared__ double red[NW][R];
  __shared__ double coef[R];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int c = 0; c < R; ++c) {
    if (c >= r) break;
    for (int pass = 0; pass < 2 && c > 0; ++pass) {
#pragma unroll
      for (int j = 0; j < R; ++j) {
        if (j < c) {
          double d = 0.0;
#pragma unroll
          for (int q = 0; q < ROWS; ++q) d = fma(x[q][j], x[q][c], d);
          d = wave_sum(d);
          if (lane == 0) red[w][j] = d;
        }
      }
      __syncthreads();
      if (threadIdx.x < c) {
        double t = 0.0;
        for (int ww = 0; ww < NW; ++ww) t += red[ww][threadIdx.x];
        coef[threadIdx.x] = t;
      }
      __syncthreads();
#pragma unroll
      for (int q = 0; q < ROWS; ++q)
#pragma unroll
        for (int j = 0; j < R; ++j)
          if (j < c) x[q][c] -= coef[j] * x[q][j];
      __syncthreads();   // red / coef are reused
    }
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < ROWS; ++q) s = fma(x[q][c], x[q][c], s);
    s = wave_sum(s);
    if (lane == 0) red[w][0] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
      double t = 0.0;
      for (int ww = 0; ww < NW; ++ww) t += red[ww][0];
      coef[0] = t;
    }
    __syncthreads();
    const double nrm = sqrt(coef[0]);
    const double inv = nrm > 0.0 ? 1.0 / nrm : 0.0;   // exactly dependent column -> zeros
#pragma unroll
    for (int q = 0; q < ROWS; ++q) x[q][c] *= inv;
    __syncthreads();
  }
}

// Global version (A taller than the register chunk): f64 arithmetic on A in place in global
// memory, f32 storage between sweeps (still well inside the reference's own f32 error).  Each thread owns rows threadIdx.x + j *
// kOrthBlock for every sweep, so a thread only ever re-reads what it wrote itself; the column dot
// products meet in LDS.  Rare (ill-conditioned inputs only), so simplicity over speed: 3 sweeps
// and 3 block reductions per column.
template <int R>
__device__ void orth_mgs2(float* __restrict__ A, int64_t n, int r) {
  constexpr int NW = kOrthBlock / kWave;
  __shared__ double red[NW][R];
  __shared__ double coef[R];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  auto block_sums = [&](double (&v)[R], int cnt) {   // coef[j] = sum over the block of v[j], j < cnt
#pragma unroll
    for (int j = 0; j < R; ++j) {
      if (j < cnt) {
        const double t = wave_sum(v[j]);
        if (lane == 0) red[w][j] = t;
      }
    }
    __syncthreads();
    if (threadIdx.x < cnt) {
      double t = 0.0;
      for (int ww = 0; ww < NW; ++ww) t += red[ww][threadIdx.x];
      coef[threadIdx.x] = t;
    }
    __syncthreads();
  };
  for (int c = 0; c < r; ++c) {
    for (int pass = 0; pass < 2 && c > 0; ++pass) {
      double d[R];
#pragma unroll
      for (int j = 0; j < R; ++j) d[j] = 0.0;
      for (int64_t i = threadIdx.x; i < n; i += kOrthBlock) {
        const double ac = (double)A[i * r + c];
#pragma unroll
        for (int j = 0; j < R; ++j)
          if (j < c) d[j] += (double)A[i * r + j] * ac;
      }
      block_sums(d, c);
      for (int64_t i = threadIdx.x; i < n; i += kOrthBlock) {
        double ac = (double)A[i * r + c];
#pragma unroll
        for (int j = 0; j < R; ++j)
          if (j < c) ac -= coef[j] * (double)A[i * r + j];
        A[i * r + c] = (float)ac;
      }
      __syncthreads();   // coef is reused
    }
    double s2[R];
#pragma unroll
    for (int j = 0; j < R; ++j) s2[j] = 0.0;
    for (int64_t i = threadIdx.x; i < n; i += kOrthBlock) {
      const double v = (double)A[i * r + c];
      s2[0] += v * v;
    }
    block_sums(s2, 1);
    const double nrm = sqrt(coef[0]);
    const double inv = nrm > 0.0 ? 1.0 / nrm : 0.0;   // exactly dependent column -> zeros
    for (int64_t i = threadIdx.x; i < n; i += kOrthBlock) A[i * r + c] = (float)((double)A[i * r + c] * inv);
    __syncthreads();
  }
}

// R = r rounded up to a power of two (the Gram accumulators live in registers: R(R+1)/2 doubles).
// DRAW: fill A with normal draws first (powersgd.py:41 q = normal_(); orthogonalize(q)) -- one
// launch instead of two.  A with n <= kOrthBlock * kOrthRows rows (4096 at r <= 4) is read (or drawn) once into
// registers and written once; taller A is streamed twice in chunks whose loads are all issued
// together.
template <int R, bool DRAW>
__global__ __launch_bounds__(kOrthBlock) void psgd_orth_kernel(float* __restrict__ A, int64_t n, int r,
                                                              uint64_t seed) {
  constexpr int kGram = R * (R + 1) / 2;
  constexpr int kOrthRows = R <= 4 ? 4 : (R <= 8 ? 2 : 1);   // rows per thread held in registers
  __shared__ double sh[kOrthBlock / kWave][kGram];
  __shared__ double Rs[R][R];
  __shared__ double Rinv[R];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const bool single = n <= (int64_t)kOrthBlock * kOrthRows;
  float a[kOrthRows][R];
  auto load_chunk = [&](int64_t base) {
#pragma unroll
    for (int j = 0; j < kOrthRows; ++j) {
      const int64_t i = base + threadIdx.x + (int64_t)j * kOrthBlock;
      const bool rv = i < n;
#pragma unroll
      for (int c = 0; c < R; ++c) {
        float v;
        if (DRAW) {
          v = normal_at(seed, (uint64_t)(i * r + c));
        } else {
          const float t = A[(rv ? i : 0) * r + (c < r ? c : 0)];   // clamped, unconditional
          v = t;
        }
        a[j][c] = (rv && c < r) ? v : 0.f;
      }
    }
  };
  double g[kGram];
#pragma unroll
  for (int e = 0; e < kGram; ++e) g[e] = 0.0;
  for (int64_t base = 0; base < n; base += (int64_t)kOrthBlock * kOrthRows) {
    load_chunk(base);
#pragma unroll
    for (int j = 0; j < kOrthRows; ++j) {
      int e = 0;
#pragma unroll
      for (int c = 0; c < R; ++c)
#pragma unroll
        for (int c2 = c; c2 < R; ++c2, ++e) g[e] += (double)a[j][c] * (double)a[j][c2];
    }
    if (DRAW && !single) {   // tall draw: store the draws, the solve pass re-reads them
#pragma unroll
      for (int j = 0; j < kOrthRows; ++j) {
        const int64_t i = base + threadIdx.x + (int64_t)j * kOrthBlock;
#pragma unroll
        for (int c = 0; c < R; ++c)
          if (i < n && c < r) A[i * r + c] = a[j][c];
      }
    }
  }
#pragma unroll
  for (int e = 0; e < kGram; ++e) {
    const double t = wave_sum(g[e]);
    if (lane == 0) sh[w][e] = t;
  }
  __syncthreads();
  __shared__ double Gs[kGram];
  if (threadIdx.x < kGram) {
    double t = 0.0;
    for (int ww = 0; ww < kOrthBlock / kWave; ++ww) t += sh[ww][threadIdx.x];
    Gs[threadIdx.x] = t;
  }
  __syncthreads();
  __shared__ int s_robust;
  if (threadIdx.x == 0) {
    // packed upper-triangle index of (c, c2), c <= c2
    auto gi = [](int c, int c2) { return c * R - c * (c - 1) / 2 + (c2 - c); };
    int robust = 0;
    for (int c = 0; c < R; ++c) {
      double d = Gs[gi(c, c)];
      for (int k = 0; k < c; ++k) d -= Rs[k][c] * Rs[k][c];
      if (c < r && !(d > kOrthPivotMin * Gs[gi(c, c)] && isfinite(d))) robust = 1;
      const double rcc = c < r ? sqrt(d) : 1.0;
      const double inv = 1.0 / rcc;
      Rs[c][c] = rcc;
      Rinv[c] = inv;
      for (int c2 = c + 1; c2 < R; ++c2) {
        double t = Gs[gi(c, c2)];
        for (int k = 0; k < c; ++k) t -= Rs[k][c] * Rs[k][c2];
        Rs[c][c2] = c2 < r ? t * inv : 0.0;
      }
    }
    s_robust = robust;
  }
  __syncthreads();
  if (s_robust) {   // ill-conditioned: MGS2 (in f64 registers when A fits the register chunk)
    if (single) {
      double x[kOrthRows][R];
#pragma unroll
      for (int j = 0; j < kOrthRows; ++j)
#pragma unroll
        for (int c = 0; c < R; ++c) x[j][c] = (double)a[j][c];
      orth_mgs2_regs<R, kOrthRows>(x, r);
#pragma unroll
      for (int j = 0; j < kOrthRows; ++j) {
        const int64_t i = threadIdx.x + (int64_t)j * kOrthBlock;
#pragma unroll
        for (int c = 0; c < R; ++c)
          if (i < n && c < r) A[i * r + c] = (float)x[j][c];
      }
    } else {
      orth_mgs2<R>(A, n, r);
    }
    return;
  }
  // A <- A R^-1, row-wise forward substitution
  for (int64_t base = 0; base < n; base += (int64_t)kOrthBlock * kOrthRows) {
    if (!single) load_chunk(base);   // single chunk: the rows are still in registers
    if (DRAW && !single) {
      // re-read what pass 1 stored (load_chunk would redraw the identical values; reading is cheaper)
#pragma unroll
      for (int j = 0; j < kOrthRows; ++j) {
        const int64_t i = base + threadIdx.x + (int64_t)j * kOrthBlock;
#pragma unroll
        for (int c = 0; c < R; ++c) a[j][c] = (i < n && c < r) ? A[i * r + c] : 0.f;
      }
    }
#pragma unroll
    for (int j = 0; j < kOrthRows; ++j) {
      const int64_t i = base + threadIdx.x + (int64_t)j * kOrthBlock;
      double x[R];
#pragma unroll
      for (int c = 0; c < R; ++c) {
        double t = (double)a[j][c];
#pragma unroll
        for (int k = 0; k < c; ++k) t -= x[k] * Rs[k][c];   // LDS broadcast reads
        x[c] = t * Rinv[c];
      }
#pragma unroll
      for (int c = 0; c < R; ++c)
        if (i < n && c < r) A[i * r + c] = (float)x[c];
    }
  }
}

// Rank-4 fast path (r == 4, n <= 4096 rows, 16-B aligned A: PowerSGD's P and q at rank 4): the
// same Cholesky-QR with one 16-B load and store per row, the Gram entries reduced by DPP row
// butterflies (no ds_bpermute chains) and, for DRAW, one Box-Muller pair per two entries.
constexpr int kOrth4Rows = kOrthBlock * 4;

template <bool DRAW>
__global__ __launch_bounds__(kOrthBlock) void psgd_orth4_kernel(float* __restrict__ A, int64_t n, uint64_t seed) {
  constexpr int R = 4, kGram = 10;
  __shared__ double sh[kOrthBlock / 16][kGram];
  __shared__ double Gs[kGram];
  __shared__ double Rs[R][R];
  __shared__ double Rinv[R];
  float a[4][R];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t i = threadIdx.x + (int64_t)j * kOrthBlock;
    const bool rv = i < n;
    if constexpr (DRAW) {
      normal_pair(seed, (uint64_t)i * 2, a[j][0], a[j][1]);
      normal_pair(seed, (uint64_t)i * 2 + 1, a[j][2], a[j][3]);
    } else {
      const f32x4v v = *reinterpret_cast<const f32x4v*>(A + (rv ? i : 0) * R);   // unconditional
      a[j][0] = v.x; a[j][1] = v.y; a[j][2] = v.z; a[j][3] = v.w;
    }
    if (!rv) a[j][0] = a[j][1] = a[j][2] = a[j][3] = 0.f;
  }
  double g[kGram];
#pragma unroll
  for (int e = 0; e < kGram; ++e) g[e] = 0.0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    int e = 0;
#pragma unroll
    for (int c = 0; c < R; ++c)
#pragma unroll
      for (int c2 = c; c2 < R; ++c2, ++e) g[e] = fma((double)a[j][c], (double)a[j][c2], g[e]);
  }
#pragma unroll
  for (int e = 0; e < kGram; ++e) g[e] = row16_sum(g[e]);
  if ((threadIdx.x & 15) == 0) {
#pragma unroll
    for (int e = 0; e < kGram; ++e) sh[threadIdx.x >> 4][e] = g[e];
  }
  __syncthreads();
  if (threadIdx.x < kGram) {
    double t = 0.0;
    for (int k = 0; k < kOrthBlock / 16; ++k) t += sh[k][threadIdx.x];
    Gs[threadIdx.x] = t;
  }
  __syncthreads();
  __shared__ int s_robust;
  if (threadIdx.x == 0) {
    auto gi = [](int c, int c2) { return c * R - c * (c - 1) / 2 + (c2 - c); };
    int robust = 0;
    for (int c = 0; c < R; ++c) {
      double d = Gs[gi(c, c)];
      for (int k = 0; k < c; ++k) d -= Rs[k][c] * Rs[k][c];
      if (!(d > kOrthPivotMin * Gs[gi(c, c)] && isfinite(d))) robust = 1;
      const double rcc = sqrt(d);
      const double inv = 1.0 / rcc;
      Rs[c][c] = rcc;
      Rinv[c] = inv;
      for (int c2 = c + 1; c2 < R; ++c2) {
        double t = Gs[gi(c, c2)];
        for (int k = 0; k < c; ++k) t -= Rs[k][c] * Rs[k][c2];
        Rs[c][c2] = t * inv;
      }
    }
    s_robust = robust;
  }
  __syncthreads();
  if (s_robust) {   // ill-conditioned: MGS2 in f64 registers
    double x[4][R];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int c = 0; c < R; ++c) x[j][c] = (double)a[j][c];
    orth_mgs2_regs<R, 4>(x, R);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t i = threadIdx.x + (int64_t)j * kOrthBlock;
      if (i < n)
        *reinterpret_cast<f32x4v*>(A + i * R) = f32x4v{(float)x[j][0], (float)x[j][1], (float)x[j][2], (float)x[j][3]};
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t i = threadIdx.x + (int64_t)j * kOrthBlock;
    double x[R];
#pragma unroll
    for (int c = 0; c < R; ++c) {
      double t = (double)a[j][c];
#pragma unroll
      for (int k = 0; k < c; ++k) t -= x[k] * Rs[k][c];
      x[c] = t * Rinv[c];
    }
    if (i < n) *reinterpret_cast<f32x4v*>(A + i * R) = f32x4v{(float)x[0], (float)x[1], (float)x[2], (float)x[3]};
  }
}

// ------------------------------------------------------------------------------------------------
// out = P Q^T (decompress, powersgd.py:58-65); optionally residual = M - out (PowerSGDMemory
// update, memory/powersgd.py:32-37) in the same pass.  A workgroup owns 1024 columns x kOuterRows
// rows: each thread keeps Q[j .. j+3][0 .. r) in registers, P's rows for the band sit in LDS, and
// the band is streamed with 16-B non-temporal stores (and loads of M for the residual).
constexpr int kOuterRows = 16;
#ifdef GRACE_OUTER_ROWS
constexpr int kOuter4Rows = GRACE_OUTER_ROWS;
#else
constexpr int kOuter4Rows = 4;   // A/B (tools/exp_psgd.py): 4-row bands 12.3 us, 2: 12.7, 8-32: 13.4
#endif

template <bool VEC>
__global__ __launch_bounds__(256) void psgd_outer_kernel(const float* __restrict__ P, const float* __restrict__ Q,
                                                        int64_t n, int64_t m, int r, float* __restrict__ out,
                                                        const float* __restrict__ M, float* __restrict__ res) {
  __shared__ float sp[kOuterRows][kMaxRank];
  const int64_t i0 = (int64_t)blockIdx.y * kOuterRows;
  for (int e = threadIdx.x; e < kOuterRows * kMaxRank; e += 256) {
    const int rr = e / kMaxRank, c = e % kMaxRank;
    sp[rr][c] = (i0 + rr < n && c < r) ? P[(i0 + rr) * r + c] : 0.f;
  }
  const int64_t j = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  float qr[4][kMaxRank];
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int c = 0; c < kMaxRank; ++c) qr[s][c] = (j + s < m && c < r) ? Q[(j + s) * r + c] : 0.f;
  __syncthreads();
  if (j >= m) return;
  const int64_t rows = min((int64_t)kOuterRows, n - i0);
  for (int rr = 0; rr < rows; ++rr) {
    const int64_t i = i0 + rr;
    float o[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < kMaxRank; ++c) {
      if (c < r) {
        const float p = sp[rr][c];
#pragma unroll
        for (int s = 0; s < 4; ++s) o[s] = o[s] + p * qr[s][c];
      }
    }
    if (VEC && j + 3 < m) {
#ifdef GRACE_OUTER_PLAIN
      if (out) *reinterpret_cast<f32x4v*>(out + i * m + j) = f32x4v{o[0], o[1], o[2], o[3]};
#else
      if (out) __builtin_nontemporal_store(f32x4v{o[0], o[1], o[2], o[3]}, reinterpret_cast<f32x4v*>(out + i * m + j));
#endif
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

// Rank 4, 16-B aligned, m % 4 == 0: Q's four rows per thread are four 16-B loads (a thread's 64 B
// are contiguous across the wave), the band's P rows are workgroup-uniform 16-B loads; the same
// f32 operation order as psgd_outer_kernel, so both give identical bits.
template <int ROWS>
__global__ __launch_bounds__(256) void psgd_outer4_kernel(const float* __restrict__ P, const float* __restrict__ Q,
                                                         int64_t n, int64_t m, float* __restrict__ out,
                                                         const float* __restrict__ M, float* __restrict__ res) {
  const int64_t i0 = (int64_t)blockIdx.y * ROWS;
  const int64_t j = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (j >= m) return;
  f32x4v qv[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) qv[s] = *reinterpret_cast<const f32x4v*>(Q + (j + s) * 4);
  const int64_t rows = min((int64_t)ROWS, n - i0);
#pragma unroll 4
  for (int rr = 0; rr < rows; ++rr) {
    const int64_t i = i0 + rr;
    const f32x4v p = *reinterpret_cast<const f32x4v*>(P + i * 4);
    f32x4v mv;
    if (res) mv = __builtin_nontemporal_load(reinterpret_cast<const f32x4v*>(M + i * m + j));
    float o[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      float t = 0.f;
#pragma unroll
      for (int c = 0; c < 4; ++c) t = t + p[c] * qv[s][c];
      o[s] = t;
    }
    if (out) __builtin_nontemporal_store(f32x4v{o[0], o[1], o[2], o[3]}, reinterpret_cast<f32x4v*>(out + i * m + j));
    if (res)
      __builtin_nontemporal_store(f32x4v{mv.x - o[0], mv.y - o[1], mv.z - o[2], mv.w - o[3]},
                                  reinterpret_cast<f32x4v*>(res + i * m + j));
  }
}

// ------------------------------------------------------------------------------------------------
// World-1 rank-4 compress in ONE pass over M (psgd_w1_pass + psgd_w1_fin).
//
// At world size 1 nothing is all-reduced between the contractions (powersgd.py:44-52), so
//   P = orth(M q) = P_raw R^-1           (R = chol(P_raw^T P_raw), the R of the reference's MGS)
//   Q = M^T P      = (M^T P_raw) R^-1
// and both P_raw = M q and Qraw = M^T P_raw come out of a single read of M: P_raw's row i needs
// only row i of M, which is still in registers when Qraw accumulates M[i, j] P_raw[i, :].  Qraw is
// accumulated in f64 (f32 x f32 products are exact in f64), so the triangular solve by R^-1 does
// not amplify rounding by kappa(R) the way an f32 Qraw would: Q matches M^T P to f32 accuracy.
// M is read once instead of twice (8 nm bytes per step with the decompression instead of 12 nm).
//
// psgd_w1_pass: a 1024-thread workgroup owns a 1024-column group of a 64-row slab -- column wave
// cw = w & 3 holds 256 columns (4 per lane), row wave rw = w >> 2 holds 16 rows, all 16 rows'
// loads issued at once (the grid is sized to one workgroup per CU, so the whole of M is in
// flight).  Per row the lane's 4 x 4 products are summed over its DPP row (16 lanes), the 16
// (column wave, DPP row) partials of the group in LDS, and the G = ceil(m / 1024) column groups of
// the slab exchange their 64 x 4 partials through write-through (sc1) 16-B records and one
// arrival counter per slab; every group sums the G records in the same order, so they all hold
// bit-identical P_raw rows.  Then Qraw[j, c] += M[i, j] P_raw[i, c] in f64 from the registers; the
// row waves are summed in LDS and each workgroup writes one f64 [1024 x 4] partial.  Group 0 of
// each slab writes P_raw and accumulates the slab's Gram matrix (f64).
// psgd_w1_fin: every workgroup sums the Gram partials (fixed order), factors R = chol(G) and
// solves its share of rows: P = P_raw R^-1 in place, Q = (sum of the Qraw partials) R^-1.  When the
// pivots say P_raw is ill-conditioned (as psgd_orth4_kernel), workgroup 0 runs MGS2 on P_raw,
// publishes its R (write-through + flag) and the others solve Q with that R.
// Requirements (checked by grace_powersgd_w1_ok): r == 4, m % 4 == 0, m <= 16384, 16-B aligned M,
// q, P, Q; the launch keeps the grid within one workgroup per CU (co-resident: the exchange waits).
constexpr int kW1Block = 1024;
constexpr int kW1Rows = 16;                   // rows per lane (per row wave)
constexpr int kW1Slab = 4 * kW1Rows;          // 64 rows per slab
constexpr int kW1Cols = 1024;                 // columns per workgroup
constexpr int kW1MaxG = 16;                   // m <= 16384
constexpr int kW1FinBlock = 1024;
constexpr uint32_t kW1SpinMax = 1u << 22;     // bounded waits (never expected to run out)
#ifndef GRACE_W1_SPLIT
#define GRACE_W1_SPLIT 0   // A/B knob (0: all 16 rows' loads in flight at once)
#endif
#ifndef GRACE_W1_NT
#define GRACE_W1_NT 1      // non-temporal loads of M (A/B, one process: compress 34.9 -> 33.7 us)
#endif
#ifndef GRACE_W1_XCD
#define GRACE_W1_XCD 0     // A/B knob: the G column groups of a slab on one XCD
#endif
#ifndef GRACE_W1_QNT
#define GRACE_W1_QNT 1     // non-temporal stores of the Qraw partials (A/B: compress 34.0 -> 32.9 us)
#endif

#ifdef GRACE_STAMPS   // diagnostic build only: s_memrealtime phase stamps of psgd_w1_pass
#define W1_STAMP(ws, slot) do { if (threadIdx.x == 0) { if (blockIdx.x == 0 && blockIdx.y == 0) (ws).dbg[slot] = __builtin_amdgcn_s_memrealtime(); \
    if ((slot) >= 1 && (slot) <= 4) (ws).dbg[8 + 4 * (blockIdx.y * gridDim.x + blockIdx.x) + (slot) - 1] = __builtin_amdgcn_s_memrealtime(); \
    if ((slot) == 0 && blockIdx.y * gridDim.x + blockIdx.x < 512) (ws).dbg[1200 + blockIdx.y * gridDim.x + blockIdx.x] = __builtin_amdgcn_s_memrealtime(); } } while (0)
#define W1_SPAN(ws) do { if (threadIdx.x == 0) { atomicMin((unsigned long long*)&(ws).dbg[6], (unsigned long long)__builtin_amdgcn_s_memrealtime()); } } while (0)
#define W1_END(ws) do { if (threadIdx.x == 0) { atomicMax((unsigned long long*)&(ws).dbg[7], (unsigned long long)__builtin_amdgcn_s_memrealtime()); } } while (0)
#define FIN_STAMP(ws, slot) do { if (threadIdx.x == 0 && blockIdx.x == 0) (ws).dbg[1800 + (slot)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#define FIN_SPAN(ws) do { if (threadIdx.x == 0) { atomicMin((unsigned long long*)&(ws).dbg[1810], (unsigned long long)__builtin_amdgcn_s_memrealtime()); } } while (0)
#define FIN_END(ws) do { if (threadIdx.x == 0) { atomicMax((unsigned long long*)&(ws).dbg[1811], (unsigned long long)__builtin_amdgcn_s_memrealtime()); } } while (0)
#else
#define FIN_STAMP(ws, slot) do { } while (0)
#define FIN_SPAN(ws) do { } while (0)
#define FIN_END(ws) do { } while (0)
#define W1_STAMP(ws, slot) do { } while (0)
#define W1_SPAN(ws) do { } while (0)
#define W1_END(ws) do { } while (0)
#endif

struct W1Ws {
  uint32_t* arr;      // [S] exchange arrivals
  uint32_t* done;     // [S] exchange reads
  uint32_t* ctl;      // [0] robust-path flag (= this call's tag), [2] waits that ran out (count)
  uint32_t* status;   // optional host-mapped word: bit 1 = a wait ran out (the call's P, Q invalid)
  uint64_t* dbg;      // diagnostic stamps (GRACE_STAMPS builds only)
  f32x4v* xp;         // [S][G][64] partial P rows
  double* qpart;      // [S][m][4] one f64 partial of Qraw per slab
  double* gpart;      // [4 S][16] four Gram partials per slab
};

__device__ __forceinline__ float row16_sum_f32(float v) {
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x141, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x140, 0xF, 0xF, false));
  return v;
}

// bounded wait for *p >= target (or == target when EQ); a wait that runs out is counted in ctl[2]
// and flagged in the host-mapped status word (bit `bit`): the call's P and Q are then not valid and
// the host raises (grace_amd/ops.py).  Never expected: the grid is one workgroup per CU
// (occupancy-checked) and the Python layer never lets two of these grids run at once.
template <bool EQ = false>
__device__ __forceinline__ bool spin_until(const uint32_t* p, uint32_t target, const W1Ws& ws, uint32_t bit) {
  uint32_t spins = 0;
  while (true) {
    const uint32_t v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (EQ ? v == target : v >= target) return true;
    __builtin_amdgcn_s_sleep(2);
    if (++spins > kW1SpinMax) {
      __hip_atomic_fetch_add(ws.ctl + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (ws.status) __hip_atomic_fetch_or(ws.status, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return false;
    }
  }
}

template <bool DRAWQ>
__global__ __launch_bounds__(kW1Block) void psgd_w1_pass(const float* __restrict__ M, int64_t n, int64_t m,
                                                        const float* __restrict__ q, uint64_t seed,
                                                        float* __restrict__ P, W1Ws ws, int S) {
  __shared__ float pp[4][kW1Rows][4][4];       // [rw][d][cw][rank]: the column waves' partials
  __shared__ double prow[kW1Slab][4];          // P_raw rows of the slab, f64
  __shared__ double qred[2][16 * 256];         // row-wave pair sums, [e][column-wave lane]
  __shared__ f32x4v qsh[kW1Cols];               // q rows of this column group
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int cw = w & 3, rw = w >> 2;
  const int G = gridDim.x, SG = gridDim.y;
  int cg = blockIdx.x, sy = blockIdx.y;
#if GRACE_W1_XCD
  {  // XCD-aware placement (A/B): workgroups are dealt to the 8 XCDs round-robin by linear id; the G
     // column groups of one slab row get ids 8 apart, i.e. one XCD, so the slab's exchange waits on
     // workgroups that share an L2 and a fabric port rather than on the slowest of G XCDs
    const int NB = G * SG, L = blockIdx.y * G + blockIdx.x;
    if (NB % (8 * G) == 0) {
      const int x = L & 7, j = L >> 3;
      cg = j % G;
      sy = x * (NB / 8 / G) + j / G;
    }
  }
#endif
  W1_STAMP(ws, 0);
  W1_SPAN(ws);
  const int64_t jc = (int64_t)cg * kW1Cols + 256 * cw + 4 * lane;
  const bool colv = jc < m;                    // m % 4 == 0: all 4 columns or none
  const uint32_t jo = colv ? (uint32_t)jc : 0u; // lane offset within a row (m <= 16384)
  const auto xrs = __builtin_amdgcn_make_buffer_rsrc(ws.xp, (short)0, 0x7FFFFFFF, 0x00020000);
  // Row interleave: slab s is row lanes 4 s + rw, and row lane l holds rows l + L d (L = 4 S), so at
  // load step d every workgroup reads inside one contiguous band of L rows (a sequential sweep of M
  // rather than 4 S scattered 16-row runs)
  const int64_t L = 4 * (int64_t)S;
  bool qstaged = false;
  // q rows of this column group: loaded BEFORE M's rows, so that staging them into LDS waits only
  // for this one older load (vmcnt counts in order).  Loaded after them (r04), the staging waited
  // for all 16 rows of M first, and the q load was issued only then (a spilled address reload
  // with vmcnt(0) in front of it): one full memory latency per workgroup on the critical path.
  f32x4v qr = {0.f, 0.f, 0.f, 0.f};
  {
    const int64_t jq = (int64_t)cg * kW1Cols + threadIdx.x;
    if (jq < m) {
      if constexpr (DRAWQ) {
        float z0, z1, z2, z3;
        normal_pair(seed, (uint64_t)jq * 2, z0, z1);
        normal_pair(seed, (uint64_t)jq * 2 + 1, z2, z3);
        qr = f32x4v{z0, z1, z2, z3};
      } else {
        qr = *reinterpret_cast<const f32x4v*>(q + 4 * jq);
      }
    }
  }
  for (int s = sy; s < S; s += SG) {
    const int64_t lrow = 4 * (int64_t)s + rw;
    f32x4v v[kW1Rows];
#pragma unroll
    for (int d = 0; d < kW1Rows; ++d) {        // every load issued before any is used
      // wave-uniform row base (scalar) + 32-bit lane offset; a row past n re-reads row n - 1
      const int64_t row = lrow + L * d;
      const float* rowp = M + (row < n ? row : n - 1) * m;
#if GRACE_W1_SPLIT > 0   // A/B knob: issue the first rows, wait for them, then the rest
      if (d == GRACE_W1_SPLIT) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
#if GRACE_W1_NT
      v[d] = __builtin_nontemporal_load(reinterpret_cast<const f32x4v*>(rowp + jo));
#else
      v[d] = *reinterpret_cast<const f32x4v*>(rowp + jo);
#endif
    }
    if (!qstaged) {   // q rows of the group into LDS while M's loads are in flight
      qstaged = true;
      qsh[threadIdx.x] = qr;
    }
    // no masking of v (a masked copy would double the rows' registers): a column past m has zero
    // q rows (qsh), and a row past n re-reads row n - 1 but gets a zero P_raw row (prow) below
    // partial P of each row over the lane's 4 columns, summed over the DPP row
    __syncthreads();   // qsh written (first slab)
    // Partial P over the wave's 256 columns, 4 rows (16 values: row dd, rank c at 4 dd + c) at a
    // time, by a 64-lane reduce-scatter: permlane32 swap (+8), permlane16 swap (+4), row mirror
    // (+2) and half-row mirror (+1) each halve the values a lane holds while summing over lane
    // pairs, then a quad allreduce; lane l ends with value l >> 2 summed over all 64 lanes.
    // ~40 VALU ops per 4 rows instead of 4 DPP stages for every value.
    const f32x4v* qrow = &qsh[256 * cw + 4 * lane];   // the lane's 4 q rows (LDS)
    const bool b3 = (lane >> 3) & 1, b2 = (lane >> 2) & 1;
#pragma unroll
    for (int b4 = 0; b4 < kW1Rows / 4; ++b4) {
      const f32x4v q0 = qrow[0], q1 = qrow[1], q2 = qrow[2], q3 = qrow[3];
      float u[16];
#pragma unroll
      for (int dd = 0; dd < 4; ++dd) {   // ranks in pairs: packed f32 FMAs
        const f32x4v mv = v[4 * b4 + dd];
#pragma unroll
        for (int c = 0; c < 4; c += 2) {
          f32x2v x = f32x2v{mv.x, mv.x} * f32x2v{q0[c], q0[c + 1]};
          x = __builtin_elementwise_fma(f32x2v{mv.y, mv.y}, f32x2v{q1[c], q1[c + 1]}, x);
          x = __builtin_elementwise_fma(f32x2v{mv.z, mv.z}, f32x2v{q2[c], q2[c + 1]}, x);
          x = __builtin_elementwise_fma(f32x2v{mv.w, mv.w}, f32x2v{q3[c], q3[c + 1]}, x);
          u[4 * dd + c] = x.x;
          u[4 * dd + c + 1] = x.y;
        }
      }
      float z[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(u[k]), __float_as_uint(u[k + 8]), false, false);
        z[k] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
      }
      float y[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(z[k]), __float_as_uint(z[k + 4]), false, false);
        y[k] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
      }
      float x2[2];
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const float send = b3 ? y[k] : y[k + 2], keep = b3 ? y[k + 2] : y[k];
        x2[k] = keep + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(send), 0x140, 0xF, 0xF, false));   // row_mirror
      }
      const float send = b2 ? x2[0] : x2[1], keep = b2 ? x2[1] : x2[0];
      float w1 = keep + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(send), 0x141, 0xF, 0xF, false));   // half mirror
      w1 += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(w1), 0x4E, 0xF, 0xF, false));
      w1 += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(w1), 0xB1, 0xF, 0xF, false));
      if ((lane & 3) == 0) pp[rw][4 * b4 + (lane >> 4)][cw][(lane >> 2) & 3] = w1;
    }
    __syncthreads();
    W1_STAMP(ws, 1);
    const int t = threadIdx.x;
    f32x4v part = {0.f, 0.f, 0.f, 0.f};
    if (t < kW1Slab) {
#pragma unroll
      for (int k = 0; k < 4; ++k) part += *reinterpret_cast<const f32x4v*>(pp[t >> 4][t & 15][k]);
      if (G > 1) __builtin_amdgcn_raw_buffer_store_b128(part, xrs, (int)((((int64_t)s * G + cg) * kW1Slab + t) * 16), 0, kSc1);
    }
    if (G > 1) {
      // every wave's write-through record stores complete, then one arrival per workgroup; wait
      // for the slab's G groups (co-resident grid) and read all G records in group order
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (t == 0) {
        __hip_atomic_fetch_add(ws.arr + s, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        spin_until(ws.arr + s, (uint32_t)G, ws, 2u);   // runs out: flagged invalid (status bit 1)
      }
      __syncthreads();
      W1_STAMP(ws, 2);
      if (t < kW1Slab) {   // the G records in group order, 4 loads in flight per round (clamped)
        part = f32x4v{0.f, 0.f, 0.f, 0.f};
        for (int g0 = 0; g0 < G; g0 += 4) {
          f32x4v rec[4];
#pragma unroll
          for (int u = 0; u < 4; ++u)
            rec[u] = __builtin_amdgcn_raw_buffer_load_b128(
                xrs, (int)((((int64_t)s * G + (g0 + u < G ? g0 + u : G - 1)) * kW1Slab + t) * 16), 0, kSc1);
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if (g0 + u < G) part += rec[u];
        }
      }
    }
    if (t < kW1Slab) {
      const int64_t row = 4 * (int64_t)s + (t >> 4) + L * (t & 15);   // slab row t = (rw, d)
#pragma unroll
      for (int c = 0; c < 4; ++c) prow[t][c] = row < n ? (double)part[c] : 0.0;
      if (cg == 0) {
        // group 0 writes P_raw and the slab's Gram partials: wave 0 holds the 64 slab rows, each
        // DPP row of 16 sums its rows' products (f64, symmetric butterflies) -> 4 partials per slab
        const f32x4v pr = part;
        if (row < n) *reinterpret_cast<f32x4v*>(P + row * 4) = pr;
        double gv[10];
        int e = 0;
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int c2 = c; c2 < 4; ++c2, ++e) gv[e] = row < n ? (double)pr[c] * (double)pr[c2] : 0.0;
#pragma unroll
        for (int k = 0; k < 10; ++k) gv[k] = row16_sum(gv[k]);
        if ((t & 15) == 0) {
#pragma unroll
          for (int k = 0; k < 10; ++k) ws.gpart[((int64_t)s * 4 + (t >> 4)) * 16 + k] = gv[k];
        }
      }
    }
    __syncthreads();
    if (G > 1 && t == 0) {   // the last group to finish reading re-zeroes the slab's counters
      if (__hip_atomic_fetch_add(ws.done + s, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (uint32_t)G - 1) {
        __hip_atomic_store(ws.arr + s, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(ws.done + s, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    W1_STAMP(ws, 3);
    // Qraw += M[i, j] P_raw[i, :] in f64, rows in order
    double acc[4][4];
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[s4][c] = 0.0;
#ifdef GRACE_W1_NOQ   // diagnostic A/B build only: no Qraw FMAs (wrong Q)
    for (int s4 = 0; s4 < 4; ++s4) acc[s4][0] = (double)v[s4][s4];
#else
#pragma unroll
    for (int d = 0; d < kW1Rows; ++d) {
      const double* pr = prow[rw * kW1Rows + d];   // wave-uniform: LDS broadcast
      const double p0 = pr[0], p1 = pr[1], p2 = pr[2], p3 = pr[3];
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        const double mv = (double)v[d][s4];
        acc[s4][0] = fma(mv, p0, acc[s4][0]);
        acc[s4][1] = fma(mv, p1, acc[s4][1]);
        acc[s4][2] = fma(mv, p2, acc[s4][2]);
        acc[s4][3] = fma(mv, p3, acc[s4][3]);
      }
    }
#endif
    // row waves summed as (rw0 + rw1) + (rw2 + rw3) through two LDS regions laid out element-major
    // (qred[buf][e][256 cw-lanes]: consecutive lanes on consecutive banks), e = 4 s4 + rank
    double* q16a = &qred[0][64 * cw + lane];
    double* q16b = &qred[1][64 * cw + lane];
    if (rw & 1) {
      double* dst = rw == 1 ? q16a : q16b;
#pragma unroll
      for (int e = 0; e < 16; ++e) dst[e * 256] = acc[e >> 2][e & 3];
    }
    __syncthreads();
    if (!(rw & 1)) {
      const double* src = rw == 0 ? q16a : q16b;
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[e >> 2][e & 3] += src[e * 256];
    }
    __syncthreads();
    if (rw == 2) {
#pragma unroll
      for (int e = 0; e < 16; ++e) q16a[e * 256] = acc[e >> 2][e & 3];
    }
    __syncthreads();
    if (rw == 0) {   // the final sums, element-major, into the second region
#pragma unroll
      for (int e = 0; e < 16; ++e) q16b[e * 256] = acc[e >> 2][e & 3] + q16a[e * 256];
    }
    __syncthreads();
    {
      // the slab's f64 [columns x 4] partial of Qraw (psgd_w1_fin sums the S slabs in order),
      // 32 KB stored by all 1024 threads as 16-B pieces contiguous across the workgroup:
      // piece q = column q / 2 of the group, ranks 2 (q & 1) and 2 (q & 1) + 1
      const int64_t gbase = ((int64_t)s * m + (int64_t)cg * kW1Cols) * 4;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int qp = threadIdx.x + 1024 * h, jl = qp >> 1;
        if ((int64_t)cg * kW1Cols + jl < m) {
          const int cwl = 64 * (jl >> 8) + ((jl & 255) >> 2), e0 = 4 * (jl & 3) + 2 * (qp & 1);
#if GRACE_W1_QNT   // A/B knob: non-temporal stores of the Qraw partials
          typedef double f64x2v __attribute__((ext_vector_type(2)));
          __builtin_nontemporal_store(f64x2v{qred[1][e0 * 256 + cwl], qred[1][(e0 + 1) * 256 + cwl]},
                                      reinterpret_cast<f64x2v*>(ws.qpart + gbase + 2 * qp));
#else
          *reinterpret_cast<double2*>(ws.qpart + gbase + 2 * qp) =
              make_double2(qred[1][e0 * 256 + cwl], qred[1][(e0 + 1) * 256 + cwl]);
#endif
        }
      }
    }
    __syncthreads();   // prow / pp / qred are rewritten by the next slab
  }
  W1_STAMP(ws, 4);
  W1_END(ws);
}

// row solve x = a R^-1 (forward substitution, f64)
__device__ __forceinline__ void w1_solve(const double (&a)[4], const double (&Rs)[4][4], const double (&Rinv)[4],
                                         double (&x)[4]) {
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    double t = a[c];
#pragma unroll
    for (int k = 0; k < c; ++k) t -= x[k] * Rs[k][c];
    x[c] = t * Rinv[c];
  }
}

// Q[j0 .. j1) = M^T P directly (robust path): thread (row lane rl = t >> 4, column quad cq = t & 15)
// accumulates rows rl, rl + 64, ... of its 4 columns in f64; the 64 row lanes are summed in a fixed
// order (cross-row shuffles, then the 16 waves in LDS).
__device__ void w1_direct_q(const float* __restrict__ M, const float* __restrict__ P, int64_t n, int64_t m,
                            int64_t j0, int64_t j1, float* __restrict__ Q) {
  __shared__ double red[kW1FinBlock / kWave][16][16];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int rl = t >> 4, cq = t & 15;
  for (int64_t jb = j0; jb < j1; jb += 64) {
    const int64_t j = jb + 4 * cq;
    const bool jv = j < j1;
    double acc[4][4] = {};
    for (int64_t i = rl; i < n; i += kW1FinBlock / 16) {
      const f32x4v mv = *reinterpret_cast<const f32x4v*>(M + i * m + (jv ? j : j0));
      const f32x4v pv = *reinterpret_cast<const f32x4v*>(P + i * 4);
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[s4][c] = fma((double)mv[s4], (double)pv[c], acc[s4][c]);
    }
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        double v = acc[s4][c];
        v += __shfl_xor(v, 16, 64);
        v += __shfl_xor(v, 32, 64);
        if (lane < 16) red[w][cq][s4 * 4 + c] = v;
      }
    __syncthreads();
    if (t < 256) {
      const int cq2 = t >> 4, e = t & 15;
      double v = 0.0;
      for (int ww = 0; ww < kW1FinBlock / kWave; ++ww) v += red[ww][cq2][e];
      const int64_t jj = jb + 4 * cq2 + (e >> 2);
      if (jj < j1) Q[jj * 4 + (e & 3)] = (float)v;
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(kW1FinBlock) void psgd_w1_fin(const float* __restrict__ M, float* __restrict__ P,
                                                          int64_t n, int64_t m, float* __restrict__ Q, W1Ws ws,
                                                          int S, uint32_t tag) {
  __shared__ double Gs[10];
  __shared__ double Rs[4][4];
  __shared__ double Rinv[4];
  __shared__ int s_robust;
  const int t = threadIdx.x, NB = gridDim.x, b = blockIdx.x;
  FIN_STAMP(ws, 0);
  FIN_SPAN(ws);
  // this workgroup's Q rows (16 per round)
  const int64_t qper = ((m + NB - 1) / NB + 15) / 16 * 16;
  const int64_t q0 = min(m, (int64_t)b * qper), q1 = min(m, q0 + qper);
  // This workgroup's P_raw rows and its first Q round's partials are loaded first: their latency
  // overlaps the Gram sum and the factorisation below.  Q: wave w owns column q0 + w of a round
  // (16 per round), lane sl sums slabs sl, sl + 64, ... in order; then a fixed-order butterfly
  // over the 64 lanes.
  const int64_t pper = (n + NB - 1) / NB;
  const int64_t prow_i = (int64_t)b * pper + t;
  const bool pv_ok = t < pper && prow_i < n;
  // The Gram partials' loads go first: vmcnt is in order, so the Gram sum below waits for them
  // only, not for the 8 MB of Qraw partials prefetched after them (A/B in the stamps build).
  // Gram: wave e < 10 sums slot e, lane k taking slabs k, k + 64, ... (loads in flight together),
  // then a fixed-order butterfly over the lanes
  const int ge = t >> 6, gk = t & 63;
  const int NG = 4 * S;   // 4 Gram partials per slab
  double gv[4];
  if (ge < 10) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int su = gk + u * kWave;
      gv[u] = ws.gpart[(int64_t)(su < NG ? su : 0) * 16 + ge];   // clamped to partial 0
    }
  }
  const f32x4v pv = *reinterpret_cast<const f32x4v*>(P + (pv_ok ? prow_i : 0) * 4);
  const int col = t >> 6, sl = t & 63;
  double2 pre_lo[4], pre_hi[4];
  {
    const int64_t j = q0 + col < q1 ? q0 + col : 0;
    if (S <= 64) {   // one slab per lane (the common case): no clamped duplicate loads
      const double2* src = reinterpret_cast<const double2*>(ws.qpart + ((int64_t)(sl < S ? sl : 0) * m + j) * 4);
      pre_lo[0] = src[0];
      pre_hi[0] = src[1];
#pragma unroll
      for (int u = 1; u < 4; ++u) pre_lo[u] = pre_hi[u] = make_double2(0.0, 0.0);
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int su = sl + 64 * u < S ? sl + 64 * u : 0;   // clamped to slab 0
        const double2* src = reinterpret_cast<const double2*>(ws.qpart + ((int64_t)su * m + j) * 4);
        pre_lo[u] = src[0];
        pre_hi[u] = src[1];
      }
    }
  }
  FIN_STAMP(ws, 1);
  if (ge < 10) {
    double g = 0.0;
#pragma unroll
    for (int u = 0; u < 4; ++u) g += gk + u * kWave < NG ? gv[u] : 0.0;
    for (int s0 = gk + 4 * kWave; s0 < NG; s0 += 4 * kWave) {   // S > 64: further rounds
      double v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int su = s0 + u * kWave;
        v[u] = ws.gpart[(int64_t)(su < NG ? su : 0) * 16 + ge];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) g += s0 + u * kWave < NG ? v[u] : 0.0;
    }
    g = wave_sum(g);
    if (gk == 0) Gs[ge] = g;
  }
  __syncthreads();
  FIN_STAMP(ws, 2);
  if (t == 0) {   // Cholesky with the pivot check of psgd_orth4_kernel
    auto gi = [](int c, int c2) { return c * 4 - c * (c - 1) / 2 + (c2 - c); };
    int robust = 0;
    for (int c = 0; c < 4; ++c) {
      double d = Gs[gi(c, c)];
      for (int k = 0; k < c; ++k) d -= Rs[k][c] * Rs[k][c];
      if (!(d > kOrthPivotMin * Gs[gi(c, c)] && isfinite(d))) robust = 1;
      const double rcc = sqrt(d);
      const double inv = 1.0 / rcc;
      Rs[c][c] = rcc;
      Rinv[c] = inv;
      for (int c2 = c + 1; c2 < 4; ++c2) {
        double u = Gs[gi(c, c2)];
        for (int k = 0; k < c; ++k) u -= Rs[k][c] * Rs[k][c2];
        Rs[c][c2] = u * inv;
      }
    }
    s_robust = robust;
  }
  __syncthreads();
  if (s_robust) {
    // ill-conditioned P_raw (kappa above ~1e4): Qraw R^-1 would amplify rounding by kappa, so
    // workgroup 0 orthogonalises P_raw in place by MGS2 (psgd_orth4_kernel's robust path) and
    // publishes it (release fence + flag); every workgroup then computes its Q rows as M^T P
    // directly (a second read of M, on this rare path only)
    if (b == 0) {
      if (n <= (int64_t)kOrth4Rows) {
        double x[4][4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int64_t i = t + (int64_t)j * kOrthBlock;
          const f32x4v v = *reinterpret_cast<const f32x4v*>(P + (i < n ? i : 0) * 4);
#pragma unroll
          for (int c = 0; c < 4; ++c) x[j][c] = i < n ? (double)v[c] : 0.0;
        }
        orth_mgs2_regs<4, 4>(x, 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int64_t i = t + (int64_t)j * kOrthBlock;
          if (i < n) *reinterpret_cast<f32x4v*>(P + i * 4) = f32x4v{(float)x[j][0], (float)x[j][1], (float)x[j][2], (float)x[j][3]};
        }
      } else {
        orth_mgs2<4>(P, n, 4);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (t == 0 && NB > 1) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(ws.ctl, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    } else {
      if (t == 0) {
        // the flag holds the tag of the call that set it, so a flag left by an earlier call never
        // matches and nothing has to reset it (a run-out wait is flagged to the host: bit 1)
        spin_until<true>(ws.ctl, tag, ws, 2u);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __syncthreads();
    }
    w1_direct_q(M, P, n, m, q0, q1, Q);
    return;
  }
  FIN_STAMP(ws, 3);
  // P = P_raw R^-1 in place: this workgroup's rows
  for (int64_t i = prow_i; i < min(n, (int64_t)(b + 1) * pper); i += kW1FinBlock) {
    const f32x4v v = i == prow_i ? pv : *reinterpret_cast<const f32x4v*>(P + i * 4);
    const double a[4] = {(double)v.x, (double)v.y, (double)v.z, (double)v.w};
    double x[4];
    w1_solve(a, Rs, Rinv, x);
    *reinterpret_cast<f32x4v*>(P + i * 4) = f32x4v{(float)x[0], (float)x[1], (float)x[2], (float)x[3]};
  }
  // Q rows, 16 columns per round (wave = column, lane = slab lane), x = Qraw R^-1
  for (int64_t jb = q0; jb < q1; jb += 16) {
    const int64_t j = jb + col;
    const bool jv = j < q1;
    double a[4] = {0.0, 0.0, 0.0, 0.0};
    for (int s0 = sl; s0 < S; s0 += 4 * 64) {   // up to 4 slabs' loads in flight
      double2 lo[4], hi[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (jb == q0 && s0 == sl) {   // prefetched at the top
          lo[u] = pre_lo[u];
          hi[u] = pre_hi[u];
          continue;
        }
        const int su = s0 + 64 * u < S ? s0 + 64 * u : 0;   // clamped to slab 0
        const double2* src = reinterpret_cast<const double2*>(ws.qpart + ((int64_t)su * m + (jv ? j : 0)) * 4);
        lo[u] = src[0];
        hi[u] = src[1];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (s0 + 64 * u < S) { a[0] += lo[u].x; a[1] += lo[u].y; a[2] += hi[u].x; a[3] += hi[u].y; }
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      double v = row16_sum(a[c]);
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      a[c] = v;
    }
    if (jv && sl == 0) {
      double x[4];
      w1_solve(a, Rs, Rinv, x);
      *reinterpret_cast<f32x4v*>(Q + j * 4) = f32x4v{(float)x[0], (float)x[1], (float)x[2], (float)x[3]};
    }
  }
  FIN_STAMP(ws, 4);
  FIN_END(ws);
}

// standard normal draws (Box-Muller on the counter-based generator), for q (powersgd.py:41)
__global__ __launch_bounds__(256) void normal_kernel(float* __restrict__ x, int64_t n, uint64_t seed) {
  for (int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x; 2 * p < n; p += (int64_t)gridDim.x * 256) {
    float z0, z1;
    normal_pair(seed, (uint64_t)p, z0, z1);
    x[2 * p] = z0;
    if (2 * p + 1 < n) x[2 * p + 1] = z1;
  }
}

}  // namespace grace

using namespace grace;

namespace grace {
template <bool DRAW>
static void launch_orth(float* A, int64_t n, int32_t r, uint64_t seed, hipStream_t st) {
  if (r == 4 && n <= kOrth4Rows && (reinterpret_cast<uintptr_t>(A) & 15) == 0) {
    psgd_orth4_kernel<DRAW><<<1, kOrthBlock, 0, st>>>(A, n, seed);
    return;
  }
  if (r <= 1) psgd_orth_kernel<1, DRAW><<<1, kOrthBlock, 0, st>>>(A, n, r, seed);
  else if (r <= 2) psgd_orth_kernel<2, DRAW><<<1, kOrthBlock, 0, st>>>(A, n, r, seed);
  else if (r <= 4) psgd_orth_kernel<4, DRAW><<<1, kOrthBlock, 0, st>>>(A, n, r, seed);
  else if (r <= 8) psgd_orth_kernel<8, DRAW><<<1, kOrthBlock, 0, st>>>(A, n, r, seed);
  else psgd_orth_kernel<16, DRAW><<<1, kOrthBlock, 0, st>>>(A, n, r, seed);
}
}  // namespace grace


extern "C" {

static int p_ksplit(int64_t n, int64_t m, int64_t tc) {
  const int64_t tiles = (n + kTileR - 1) / kTileR;
  if (tiles > kTickets) return 1;
  const int64_t nkt = (m + tc - 1) / tc;
#ifdef GRACE_P_KS
  return (int)min((int64_t)GRACE_P_KS, nkt);
#endif
  int64_t ks = (2048 + tiles - 1) / tiles;                  // aim for >= 2048 workgroups
  if (ks > nkt) ks = nkt;
  if (ks > 64) ks = 64;
  return ks < 1 ? 1 : (int)ks;
}

#ifndef GRACE_QT_WG
#define GRACE_QT_WG 1024
#endif
static int64_t qt_slab(int64_t n, int64_t m) {
  const int64_t groups = (m + Tile<kCPL>::C - 1) / Tile<kCPL>::C;
  if (groups * 128 > kTickets / 2) return n;
#ifdef GRACE_QT_SLAB
  return GRACE_QT_SLAB;
#endif
  const int64_t ns = (GRACE_QT_WG + groups - 1) / groups;   // aim for >= GRACE_QT_WG workgroups
  int64_t slab = (n + ns - 1) / ns;
  slab = (slab + kTileR - 1) / kTileR * kTileR;
  if (slab < 2 * kTileR) slab = 2 * kTileR;                 // keep the prefetch pipeline busy
  while ((n + slab - 1) / slab > 16 * kFan) slab *= 2;      // <= 16 groups of kFan slabs
  return slab;
}

// psgd_qt4_kernel: slabs of 4 x kQ4D-multiples, aiming at >= 256 workgroups, <= 16 groups of kFan
static bool qt4_ok(int64_t m) { return ((m + kQ4C - 1) / kQ4C) * 16 <= kTickets / 2; }
static int64_t qt4_slab(int64_t n, int64_t m) {
  const int64_t groups = (m + kQ4C - 1) / kQ4C;
#ifndef GRACE_QT4_WG
#define GRACE_QT4_WG 256
#endif
  const int64_t ns = (GRACE_QT4_WG + groups - 1) / groups;
  int64_t slab = (n + ns - 1) / ns;
  slab = (slab + 4 * kQ4D - 1) / (4 * kQ4D) * (4 * kQ4D);   // four row waves of whole batches
  while ((n + slab - 1) / slab > 16 * kFan) slab *= 2;
  return slab;
}

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

size_t grace_powersgd_workspace_bytes(int64_t n, int64_t m, int32_t r) {
  const size_t pp = sizeof(float) * (size_t)p_ksplit(n, m, Tile<1>::C) * n * r;   // >= the R4 split
  // the larger of the two Qt kernels' slab partials (the rank-4 kernel needs 16-B aligned M and P)
  int64_t nslab = (n + qt_slab(n, m) - 1) / qt_slab(n, m);
  if (r == 4 && qt4_ok(m)) nslab = max(nslab, (n + qt4_slab(n, m) - 1) / qt4_slab(n, m));
  const size_t qp = sizeof(float) * (size_t)(nslab + (nslab + kFan - 1) / kFan) * m * r;
  return kTicketBytes + align256(pp > qp ? pp : qp);
}

extern "C++" template <bool DRAWQ>
static grace_status_t launch_p(const float* M, int64_t n, int64_t m, const float* q, uint64_t seed, int32_t r,
                               float* P, void* ws, hipStream_t st) {
  const bool vec = (m % 4 == 0) && ((reinterpret_cast<uintptr_t>(M) & 15u) == 0);
  const bool r4 = r == 4 &&
                  ((reinterpret_cast<uintptr_t>(q) | reinterpret_cast<uintptr_t>(P) | reinterpret_cast<uintptr_t>(ws)) & 15u) == 0 &&
                  n * 16 * 64 < (1ll << 31);   // partial offsets: <= 64 K chunks of n 16-B rows
  const dim3 grid((unsigned)p_ksplit(n, m, vec && r4 ? Tile<kCPL>::C : Tile<1>::C), (unsigned)((n + kTileR - 1) / kTileR));
  uint32_t* tickets = reinterpret_cast<uint32_t*>(ws);
  float* part = reinterpret_cast<float*>(reinterpret_cast<char*>(ws) + kTicketBytes);
  if (vec && r4) psgd_p_kernel<true, true, DRAWQ><<<grid, kPBlockT, 0, st>>>(M, n, m, q, r, P, part, tickets, seed);
  else if (vec) psgd_p_kernel<true, false, DRAWQ><<<grid, kPBlockT, 0, st>>>(M, n, m, q, r, P, part, tickets, seed);
  else psgd_p_kernel<false, false, DRAWQ><<<grid, kPBlockT, 0, st>>>(M, n, m, q, r, P, part, tickets, seed);
  GRACE_CHECK_LAUNCH("grace_powersgd_p");
  return GRACE_OK;
}

grace_status_t grace_powersgd_p(const float* M, int64_t n, int64_t m, const float* q, int32_t r, float* P,
                                void* ws, void* stream) {
  GRACE_REQUIRE(M && q && P && ws && n >= 1 && m >= 1 && r >= 1 && r <= kMaxRank,
                "grace_powersgd_p: bad arguments");
  return launch_p<false>(M, n, m, q, 0, r, P, ws, as_stream(stream));
}

grace_status_t grace_powersgd_p_draw(const float* M, int64_t n, int64_t m, uint64_t seed, int32_t r, float* P,
                                     void* ws, void* stream) {
  GRACE_REQUIRE(M && P && ws && n >= 1 && m >= 1 && r >= 1 && r <= kMaxRank,
                "grace_powersgd_p_draw: bad arguments");
  return launch_p<true>(M, n, m, nullptr, seed, r, P, ws, as_stream(stream));
}

grace_status_t grace_powersgd_qt(const float* M, int64_t n, int64_t m, const float* P, int32_t r, float* Q,
                                 void* ws, void* stream) {
  GRACE_REQUIRE(M && P && Q && ws && n >= 1 && m >= 1 && r >= 1 && r <= kMaxRank,
                "grace_powersgd_qt: bad arguments");
  const bool vec = (m % 4 == 0) && ((reinterpret_cast<uintptr_t>(M) & 15u) == 0);
  uint32_t* tickets = reinterpret_cast<uint32_t*>(ws);
  float* part = reinterpret_cast<float*>(reinterpret_cast<char*>(ws) + kTicketBytes);
#ifndef GRACE_QT_MFMA
  if (r == 4 && vec && qt4_ok(m) && ((reinterpret_cast<uintptr_t>(P) & 15u) == 0)) {
    const int64_t slab = qt4_slab(n, m);
    const dim3 grid((unsigned)((m + kQ4C - 1) / kQ4C), (unsigned)((n + slab - 1) / slab));
    psgd_qt4_kernel<<<grid, kQ4Block, 0, as_stream(stream)>>>(M, n, m, P, slab, Q, part, tickets);
    GRACE_CHECK_LAUNCH("grace_powersgd_qt");
    return GRACE_OK;
  }
#endif
  const int64_t slab = qt_slab(n, m);
  const int64_t nslab = (n + slab - 1) / slab;
  const dim3 grid((unsigned)((m + Tile<kCPL>::C - 1) / Tile<kCPL>::C), (unsigned)nslab);
  if (vec) psgd_qt_kernel<true><<<grid, kPBlockT, 0, as_stream(stream)>>>(M, n, m, P, r, slab, Q, part, tickets);
  else psgd_qt_kernel<false><<<grid, kPBlockT, 0, as_stream(stream)>>>(M, n, m, P, r, slab, Q, part, tickets);
  GRACE_CHECK_LAUNCH("grace_powersgd_qt");
  return GRACE_OK;
}

grace_status_t grace_orthogonalize(float* A, int64_t n, int32_t r, void* stream) {
  GRACE_REQUIRE(A && n >= 1 && r >= 1 && r <= kMaxRank, "grace_orthogonalize: bad arguments");
  launch_orth<false>(A, n, r, 0, as_stream(stream));
  GRACE_CHECK_LAUNCH("grace_orthogonalize");
  return GRACE_OK;
}

grace_status_t grace_normal_orthogonal(float* A, int64_t n, int32_t r, uint64_t seed, void* stream) {
  GRACE_REQUIRE(A && n >= 1 && r >= 1 && r <= kMaxRank, "grace_normal_orthogonal: bad arguments");
  launch_orth<true>(A, n, r, seed, as_stream(stream));
  GRACE_CHECK_LAUNCH("grace_normal_orthogonal");
  return GRACE_OK;
}

grace_status_t grace_powersgd_outer(const float* P, const float* Q, int64_t n, int64_t m, int32_t r, float* out,
                                    const float* M, float* residual, void* stream) {
  GRACE_REQUIRE(P && Q && n >= 1 && m >= 1 && r >= 1 && (out || (M && residual)) && (!residual || M),
                "grace_powersgd_outer: bad arguments");
  const bool vec = (m % 4 == 0) &&
                   (((reinterpret_cast<uintptr_t>(out) | reinterpret_cast<uintptr_t>(M) |
                      reinterpret_cast<uintptr_t>(residual)) & 15u) == 0);
  if (vec && r == 4 && ((reinterpret_cast<uintptr_t>(P) | reinterpret_cast<uintptr_t>(Q)) & 15u) == 0) {
    const dim3 g4((unsigned)((m + 1023) / 1024), (unsigned)((n + kOuter4Rows - 1) / kOuter4Rows));
    psgd_outer4_kernel<kOuter4Rows><<<g4, 256, 0, as_stream(stream)>>>(P, Q, n, m, out, M, residual);
    GRACE_CHECK_LAUNCH("grace_powersgd_outer");
    return GRACE_OK;
  }
  const dim3 grid((unsigned)((m + 1023) / 1024), (unsigned)((n + kOuterRows - 1) / kOuterRows));
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

// ------------------------------------------------------------------------------------------------
// world-1 rank-4 compress (psgd_w1_pass + psgd_w1_fin).  Workspace: [ctl 256 B | arrivals and
// read counters for kW1MaxSlabs slabs | R 256 B] at fixed offsets (the counters are left zeroed,
// whatever the shape of the call that shares the workspace), then the shape-sized data regions.
namespace grace {
constexpr int64_t kW1MaxSlabs = 16384;        // n <= 1 Mi rows
constexpr int kW1MaxCUs = 256;                // partial slots sized for <= 256 CUs (MI355X)

static int64_t w1_S(int64_t n) { return (n + kW1Slab - 1) / kW1Slab; }
static int w1_G(int64_t m) { return (int)((m + kW1Cols - 1) / kW1Cols); }
static int64_t w1_SG_max(int64_t n, int64_t m) {
  const int64_t cap = kW1MaxCUs / w1_G(m);
  return min(w1_S(n), cap < 1 ? 1 : cap);
}
static size_t w1_align(size_t x) { return (x + 255) & ~(size_t)255; }
static size_t w1_bytes(int64_t n, int64_t m) {
  const int64_t S = w1_S(n);
  return 256 + 2 * w1_align(4 * kW1MaxSlabs) + 16384 + w1_align((size_t)S * w1_G(m) * kW1Slab * 16) +
         w1_align((size_t)S * 4 * 16 * 8) + (size_t)S * m * 32;
}
static W1Ws w1_carve(void* base, int64_t n, int64_t m) {
  char* p = reinterpret_cast<char*>(base);
  W1Ws w;
  w.status = nullptr;
  w.ctl = reinterpret_cast<uint32_t*>(p); p += 256;
  w.arr = reinterpret_cast<uint32_t*>(p); p += w1_align(4 * kW1MaxSlabs);
  w.done = reinterpret_cast<uint32_t*>(p); p += w1_align(4 * kW1MaxSlabs);
  w.dbg = reinterpret_cast<uint64_t*>(p); p += 16384;   // diagnostic stamps only
  w.xp = reinterpret_cast<f32x4v*>(p); p += w1_align((size_t)w1_S(n) * w1_G(m) * kW1Slab * 16);
  w.gpart = reinterpret_cast<double*>(p); p += w1_align((size_t)w1_S(n) * 4 * 16 * 8);
  w.qpart = reinterpret_cast<double*>(p);
  return w;
}
// CUs of the current device and whether both kernels fit one workgroup per CU (cached per device)
static int w1_cus() {
  static int cached[64];
  static bool init[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  if (!init[dev]) {
    int a = 0, b = 0, c = 0, cus = 0;
    const bool ok = hipOccupancyMaxActiveBlocksPerMultiprocessor(&a, psgd_w1_pass<true>, kW1Block, 0) == hipSuccess &&
                    hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, psgd_w1_pass<false>, kW1Block, 0) == hipSuccess &&
                    hipOccupancyMaxActiveBlocksPerMultiprocessor(&c, psgd_w1_fin, kW1FinBlock, 0) == hipSuccess &&
                    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess;
    cached[dev] = ok && a >= 1 && b >= 1 && c >= 1 ? cus : 0;
    init[dev] = true;
  }
  return cached[dev];
}
}  // namespace grace

extern "C" {

int32_t grace_powersgd_w1_ok(int64_t n, int64_t m, int32_t r) {
  return r == 4 && n >= 1 && m >= 4 && m % 4 == 0 && m <= (int64_t)kW1Cols * kW1MaxG && w1_S(n) <= kW1MaxSlabs &&
                 w1_cus() >= w1_G(m)
             ? 1 : 0;
}

size_t grace_powersgd_w1_workspace_bytes(int64_t n, int64_t m) { return w1_bytes(n, m); }

grace_status_t grace_powersgd_w1_compress(const float* M, int64_t n, int64_t m, const float* q, uint64_t seed,
                                          float* P, float* Q, void* ws, size_t ws_bytes, uint32_t* status_host,
                                          void* stream) {
  GRACE_REQUIRE(M && P && Q && ws && grace_powersgd_w1_ok(n, m, 4), "grace_powersgd_w1_compress: bad arguments");
  GRACE_REQUIRE(((reinterpret_cast<uintptr_t>(M) | reinterpret_cast<uintptr_t>(q) | reinterpret_cast<uintptr_t>(P) |
                  reinterpret_cast<uintptr_t>(Q) | reinterpret_cast<uintptr_t>(ws)) & 15u) == 0,
                "grace_powersgd_w1_compress: M, q, P, Q and the workspace must be 16-B aligned");
  if (ws_bytes < w1_bytes(n, m)) {
    set_error_msg("grace_powersgd_w1_compress: workspace too small");
    return GRACE_ERR_WORKSPACE;
  }
  const hipStream_t st = as_stream(stream);
  W1Ws w = w1_carve(ws, n, m);
  w.status = nullptr;
  if (status_host) {   // pinned host word; the kernels write it through its device mapping
    void* dp = nullptr;
    w.status = hipHostGetDevicePointer(&dp, status_host, 0) == hipSuccess && dp ? reinterpret_cast<uint32_t*>(dp)
                                                                                 : status_host;
  }
  // per-call tag of the robust path's flag: never equal to a flag an earlier call left behind
  static std::atomic<uint32_t> g_w1_tag{0};
  uint32_t tag = ++g_w1_tag;
  if (tag == 0) tag = ++g_w1_tag;
  const int G = w1_G(m);
  const int64_t S = w1_S(n);
  int64_t SG = min((int64_t)w1_cus() / G, w1_SG_max(n, m));   // one workgroup per CU: co-resident
  if (SG < 1) SG = 1;
  const dim3 grid((unsigned)G, (unsigned)SG);
  if (q) psgd_w1_pass<false><<<grid, kW1Block, 0, st>>>(M, n, m, q, seed, P, w, (int)S);
  else psgd_w1_pass<true><<<grid, kW1Block, 0, st>>>(M, n, m, q, seed, P, w, (int)S);
  GRACE_CHECK_LAUNCH("psgd_w1_pass");
  int64_t nb = (max(n, m) + 15) / 16;
  nb = min(nb, min((int64_t)256, (int64_t)w1_cus()));   // one per CU at most: co-resident (robust path)
  if (nb < 1) nb = 1;
  psgd_w1_fin<<<(unsigned)nb, kW1FinBlock, 0, st>>>(M, P, n, m, Q, w, (int)S, tag);   // one partial per slab
  GRACE_CHECK_LAUNCH("psgd_w1_fin");
  return GRACE_OK;
}

}  // extern "C"
