// Read + sparse-write probe (r06): what does the no-memory top-k's recycled output cost?  The main
// pass of Allgather(TopK 1 %, NoneMemory).step reads g (256 MiB) and writes only the ~1 % of
// elements it selects into an output that already holds zeros elsewhere; the previous step's picks
// are cleared by scattered 4-B stores.  This probe streams g in the main pass's exact layout (2048
// workgroups x 256 lanes, 32 float4 per lane in groups of 4, two groups ahead, non-temporal 16-B
// loads) and writes the picks (|g| > thr, ~1 % of uniform(-1, 1) data) at different granules:
//   0 nothing written (the read ceiling of this layout)
//   1 a 4-B store per pick (the r05 recycled mode)
//   2 the whole 16-B quad of a lane that holds a pick (zeros elsewhere)
//   3 the 32-B granule (2 lanes) holding a pick
//   4 the 64-B granule (4 lanes)
//   5 the 128-B line (8 lanes)
//   6 every quad (the dense output)
//   7 granule 3, and also every 32-B granule the PREVIOUS step wrote (a bitmap, 1 bit per 32 B,
//     read per lane): the clear folded into the main pass
// and the clear kernels: k scattered 4-B zero stores from an index list in ascending order (as the
// payload lists come out, chunk by chunk) or in random order.
// Build: hipcc --offload-arch=gfx950 -O3 tools/scatter_probe.hip -o tools/scatter_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int kBlock = 256, kNV = 32, kGroup = 4;
constexpr long kChunk = (long)kBlock * 4 * kNV;   // 32768 elements

__device__ __forceinline__ unsigned hash32(unsigned x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}
__global__ void init_uniform(float* x, long n, unsigned seed) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    x[i] = (float)(hash32((unsigned)i * 2654435761u + seed) >> 8) * (2.f / 16777216.f) - 1.f;
}

template <int MODE>
__device__ __forceinline__ void handle(const f4& v, f4* out4, float* out, long q, float thr, unsigned prev_bits) {
  const int lane = threadIdx.x & 63;
  const bool p0 = fabsf(v.x) > thr, p1 = fabsf(v.y) > thr, p2 = fabsf(v.z) > thr, p3 = fabsf(v.w) > thr;
  const bool any = p0 | p1 | p2 | p3;
  if constexpr (MODE == 1) {
    const long i = q * 4;
    if (p0) out[i] = v.x;
    if (p1) out[i + 1] = v.y;
    if (p2) out[i + 2] = v.z;
    if (p3) out[i + 3] = v.w;
  } else if constexpr (MODE >= 2 && MODE <= 5 || MODE == 7) {
    constexpr int G = MODE == 2 ? 1 : MODE == 3 || MODE == 7 ? 2 : MODE == 4 ? 4 : 8;
    const unsigned long long m = __ballot(any);
    const unsigned gm = (unsigned)(m >> (lane & ~(G - 1))) & ((1u << G) - 1u);
    bool w = gm != 0;
    if constexpr (MODE == 7) w = w || prev_bits;
    if (w) {
      const f4 o = {p0 ? v.x : 0.f, p1 ? v.y : 0.f, p2 ? v.z : 0.f, p3 ? v.w : 0.f};
      __builtin_nontemporal_store(o, out4 + q);
    }
  } else if constexpr (MODE == 6) {
    const f4 o = {p0 ? v.x : 0.f, p1 ? v.y : 0.f, p2 ? v.z : 0.f, p3 ? v.w : 0.f};
    __builtin_nontemporal_store(o, out4 + q);
  }
  (void)prev_bits;
}

// bitmap: 1 bit per 32-B granule (8 floats): word w covers floats [256 w, 256 w + 256)
template <int MODE>
__global__ __launch_bounds__(kBlock, 4) void stream_pick(const f4* __restrict__ g4, float* out, const unsigned* bits,
                                                          float thr, float* sink) {
  f4* out4 = reinterpret_cast<f4*>(out);
  const long base = (long)blockIdx.x * (kChunk / 4) + threadIdx.x;   // in float4
  f4 a[kGroup], b[kGroup], c[kGroup];
#pragma unroll
  for (int u = 0; u < kGroup; ++u) a[u] = __builtin_nontemporal_load(g4 + base + u * kBlock);
#pragma unroll
  for (int u = 0; u < kGroup; ++u) b[u] = __builtin_nontemporal_load(g4 + base + (kGroup + u) * kBlock);
  float acc = 0.f;
#pragma unroll 1
  for (int q = 0; q < kNV / kGroup; ++q) {
    if (q + 2 < kNV / kGroup) {
#pragma unroll
      for (int u = 0; u < kGroup; ++u)
        c[u] = __builtin_nontemporal_load(g4 + base + ((q + 2) * kGroup + u) * kBlock);
    }
#pragma unroll
    for (int u = 0; u < kGroup; ++u) {
      const long qi = base + (q * kGroup + u) * kBlock;
      unsigned pb = 0;
      if constexpr (MODE == 7) pb = (bits[qi >> 6] >> ((qi >> 1) & 31)) & 1u;
      if constexpr (MODE == 0) acc += a[u].x + a[u].y + a[u].z + a[u].w;
      else handle<MODE>(a[u], out4, out, qi, thr, pb);
    }
#pragma unroll
    for (int u = 0; u < kGroup; ++u) { a[u] = b[u]; b[u] = c[u]; }
  }
  if (acc == 12345.678f) sink[0] = acc;
}

__global__ void clear_list(float* out, const int* idx, long k) {
  for (long j = (long)blockIdx.x * blockDim.x + threadIdx.x; j < k; j += (long)gridDim.x * blockDim.x)
    out[idx[j]] = 0.f;
}

int main() {
  const long n = 1L << 26, k = n / 100;
  const int sets = 3, reps = 20;
  const float thr = 0.99f;   // |u| > 0.99 on uniform(-1, 1): 1 %
  float *g[sets], *out[sets], *sink;
  unsigned* bits[sets];
  int *idx_sorted, *idx_rand;
  for (int s = 0; s < sets; ++s) {
    hipMalloc(&g[s], n * 4);
    hipMalloc(&out[s], n * 4);
    hipMalloc(&bits[s], n / 8);   // n / 256 words... 1 bit per 8 floats = n / 64 bytes (over-allocated)
    init_uniform<<<4096, 256>>>(g[s], n, 17u + s);
    hipMemset(out[s], 0, n * 4);
  }
  hipMalloc(&sink, 4);
  // a previous selection's granule bitmap: mark the granules of another uniform draw's picks
  {
    std::vector<unsigned> hb(n / 256, 0u);
    std::vector<int> si, ri;
    srand(5);
    for (long i = 0; i < n; ++i) {
      const unsigned h = (unsigned)(((unsigned long long)i * 0x9E3779B97F4A7C15ull) >> 40) ^ (unsigned)rand();
      if ((h % 1000u) < 10u) {   // ~1 %
        hb[i >> 8] |= 1u << ((i >> 3) & 31);
        si.push_back((int)i);
      }
    }
    ri = si;
    std::random_shuffle(ri.begin(), ri.end());
    for (int s = 0; s < sets; ++s) hipMemcpy(bits[s], hb.data(), hb.size() * 4, hipMemcpyHostToDevice);
    const long kk = std::min<long>(k, (long)si.size());
    hipMalloc(&idx_sorted, kk * 4);
    hipMalloc(&idx_rand, kk * 4);
    hipMemcpy(idx_sorted, si.data(), kk * 4, hipMemcpyHostToDevice);
    hipMemcpy(idx_rand, ri.data(), kk * 4, hipMemcpyHostToDevice);
    printf("prev picks %zu, clear list %ld\n", si.size(), kk);
  }
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int grid = (int)(n / kChunk);
  const char* names[] = {"read only", "4-B store per pick", "16-B quad with a pick", "32-B granule with a pick",
                         "64-B granule with a pick", "128-B line with a pick", "dense (every quad)",
                         "32-B granule: new picks + previous bitmap", "clear 1 % (ascending idx)",
                         "clear 1 % (random idx)"};
  for (int v = 0; v < 10; ++v) {
    std::vector<float> ts;
    for (int r = 0; r < reps + sets; ++r) {
      const int s = r % sets;
      hipEventRecord(e0);
      switch (v) {
        case 0: stream_pick<0><<<grid, kBlock>>>((const f4*)g[s], out[s], bits[s], thr, sink); break;
        case 1: stream_pick<1><<<grid, kBlock>>>((const f4*)g[s], out[s], bits[s], thr, sink); break;
        case 2: stream_pick<2><<<grid, kBlock>>>((const f4*)g[s], out[s], bits[s], thr, sink); break;
        case 3: stream_pick<3><<<grid, kBlock>>>((const f4*)g[s], out[s], bits[s], thr, sink); break;
        case 4: stream_pick<4><<<grid, kBlock>>>((const f4*)g[s], out[s], bits[s], thr, sink); break;
        case 5: stream_pick<5><<<grid, kBlock>>>((const f4*)g[s], out[s], bits[s], thr, sink); break;
        case 6: stream_pick<6><<<grid, kBlock>>>((const f4*)g[s], out[s], bits[s], thr, sink); break;
        case 7: stream_pick<7><<<grid, kBlock>>>((const f4*)g[s], out[s], bits[s], thr, sink); break;
        case 8: clear_list<<<1024, 256>>>(out[s], idx_sorted, k); break;
        case 9: clear_list<<<1024, 256>>>(out[s], idx_rand, k); break;
      }
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (r >= sets) ts.push_back(ms * 1e3f);
    }
    std::sort(ts.begin(), ts.end());
    printf("%d %-44s median %7.1f us  min %7.1f us  (read %.2f TB/s at the median)\n", v, names[v], ts[ts.size() / 2],
           ts[0], v < 8 ? n * 4.0 / (ts[ts.size() / 2] * 1e-6) / 1e12 : 0.0);
  }
  return 0;
}
