// Write-only 256 MiB stream probe (r05): which store shape reaches the box's write rate?  Variants,
// each over 3 rotated buffers, hipEvent-timed medians of 20 launches:
//   0 grid-stride float4 non-temporal stores, 256-thread blocks, 4 x #CU x 8 blocks (grace_fill's shape)
//   1 the same with plain stores
//   2 one 16 KiB tile per 256-thread block (each lane 4 x 16 B, lane-interleaved), non-temporal
//   3 the same, plain stores
//   4 one 32 KiB tile per block, 8 x 16 B per lane (the W > 1 decode's write shape), non-temporal
//   5 the same, plain
//   6 hipMemsetD32Async (the runtime's fill); 7-11 other tile / block shapes
//   12-14 wave-contiguous tiles (each wave's stores one contiguous span); 15-19 the tile shapes read
// Build: hipcc --offload-arch=gfx950 -O3 tools/write_probe.hip -o tools/write_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));

template <bool NT>
__global__ __launch_bounds__(256) void fill_stride(f4* o, long n4, float v) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    if (NT) __builtin_nontemporal_store(f4{v, v, v, v}, o + i);
    else o[i] = f4{v, v, v, v};
  }
}
template <bool NT, int PER, int BS = 256>
__global__ __launch_bounds__(BS) void fill_tile(f4* o, float v) {
  f4* base = o + (long)blockIdx.x * BS * PER;
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    if (NT) __builtin_nontemporal_store(f4{v, v, v, v}, base + u * BS + threadIdx.x);
    else base[u * BS + threadIdx.x] = f4{v, v, v, v};
  }
}
// wave-contiguous: wave w of the block writes its own contiguous 64 x PER x 16 B piece of the tile
// (store u of lane l at w * 64 * PER + 64 u + l), so each wave's stores burst into one span
template <int PER, int BS = 256>
__global__ __launch_bounds__(BS) void fill_tile_wc(f4* o, float v) {
  f4* base = o + (long)blockIdx.x * BS * PER + (threadIdx.x >> 6) * 64 * PER + (threadIdx.x & 63);
#pragma unroll
  for (int u = 0; u < PER; ++u) __builtin_nontemporal_store(f4{v, v, v, v}, base + 64 * u);
}
// read probes: the same two tile layouts read (non-temporal loads), a per-thread sum kept live
template <int PER, bool WC, int BS = 256>
__global__ __launch_bounds__(BS) void read_tile(const f4* x, float* sink) {
  const f4* base = WC ? x + (long)blockIdx.x * BS * PER + (threadIdx.x >> 6) * 64 * PER + (threadIdx.x & 63)
                      : x + (long)blockIdx.x * BS * PER + threadIdx.x;
  f4 v[PER];
#pragma unroll
  for (int u = 0; u < PER; ++u) v[u] = __builtin_nontemporal_load(base + (WC ? 64 : BS) * u);
  float acc = 0.f;
#pragma unroll
  for (int u = 0; u < PER; ++u) acc += v[u].x + v[u].y + v[u].z + v[u].w;
  if (acc == 12345.678f) sink[0] = acc;
}

int main() {
  const long n = 1L << 26, n4 = n / 4;
  f4* buf[3];
  for (int b = 0; b < 3; ++b)
    if (hipMalloc(&buf[b], n * 4) != hipSuccess) { printf("alloc failed\n"); return 1; }
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const char* names[] = {"stride nt", "stride plain", "tile16K nt", "tile16K plain", "tile32K nt", "tile32K plain",
                         "hipMemsetD32Async", "tile4K nt", "tile8K nt", "tile64K/1024 nt", "tile32K/512 nt",
                         "tile16K/1024 nt", "tile32K wave-contig nt", "tile16K wave-contig nt",
                         "tile8K wave-contig nt", "read tile32K interleaved", "read tile32K wave-contig",
                         "read tile16K interleaved", "read tile16K wave-contig", "read tile4K"};
  float* sink = nullptr;
  if (hipMalloc(&sink, 64) != hipSuccess) { printf("alloc failed\n"); return 1; }
  const int first = getenv("WP_FIRST") ? atoi(getenv("WP_FIRST")) : 0;
  for (int v = first; v < 20; ++v) {
    std::vector<float> ts;
    for (int r = 0; r < 25; ++r) {
      f4* o = buf[r % 3];
      hipEventRecord(e0, 0);
      switch (v) {
        case 0: fill_stride<true><<<cus * 8 * 4, 256>>>(o, n4, 0.f); break;
        case 1: fill_stride<false><<<cus * 8 * 4, 256>>>(o, n4, 0.f); break;
        case 2: fill_tile<true, 4><<<(unsigned)(n4 / (256 * 4)), 256>>>(o, 0.f); break;
        case 3: fill_tile<false, 4><<<(unsigned)(n4 / (256 * 4)), 256>>>(o, 0.f); break;
        case 4: fill_tile<true, 8><<<(unsigned)(n4 / (256 * 8)), 256>>>(o, 0.f); break;
        case 5: fill_tile<false, 8><<<(unsigned)(n4 / (256 * 8)), 256>>>(o, 0.f); break;
        case 6: hipMemsetD32Async((hipDeviceptr_t)o, 0, n, 0); break;
        case 7: fill_tile<true, 1><<<(unsigned)(n4 / 256), 256>>>(o, 0.f); break;
        case 8: fill_tile<true, 2><<<(unsigned)(n4 / 512), 256>>>(o, 0.f); break;
        case 9: fill_tile<true, 4, 1024><<<(unsigned)(n4 / 4096), 1024>>>(o, 0.f); break;
        case 10: fill_tile<true, 4, 512><<<(unsigned)(n4 / 2048), 512>>>(o, 0.f); break;
        case 11: fill_tile<true, 1, 1024><<<(unsigned)(n4 / 1024), 1024>>>(o, 0.f); break;
        case 12: fill_tile_wc<8><<<(unsigned)(n4 / (256 * 8)), 256>>>(o, 0.f); break;
        case 13: fill_tile_wc<4><<<(unsigned)(n4 / (256 * 4)), 256>>>(o, 0.f); break;
        case 14: fill_tile_wc<2><<<(unsigned)(n4 / (256 * 2)), 256>>>(o, 0.f); break;
        case 15: read_tile<8, false><<<(unsigned)(n4 / (256 * 8)), 256>>>(o, sink); break;
        case 16: read_tile<8, true><<<(unsigned)(n4 / (256 * 8)), 256>>>(o, sink); break;
        case 17: read_tile<4, false><<<(unsigned)(n4 / (256 * 4)), 256>>>(o, sink); break;
        case 18: read_tile<4, true><<<(unsigned)(n4 / (256 * 4)), 256>>>(o, sink); break;
        case 19: read_tile<1, false><<<(unsigned)(n4 / 256), 256>>>(o, sink); break;
      }
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      if (r >= 5) ts.push_back(ms * 1000.f);
    }
    std::sort(ts.begin(), ts.end());
    const float med = ts[ts.size() / 2];
    printf("%-18s median %.1f us  %.2f TB/s  (min %.1f)\n", names[v], med, 4.0 * n / med / 1e6, ts.front());
  }
  return 0;
}
