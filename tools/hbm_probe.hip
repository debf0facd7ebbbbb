// HBM ceiling probe for the codec kernels' traffic mixes on MI355X (standalone; not part of the
// library).  Build: hipcc --offload-arch=gfx950 -O3 tools/hbm_probe.hip -o tools/hbm_probe
// Prints one JSON object per line: {"probe": ..., "gbps": ...}.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr int B = 256;

__global__ __launch_bounds__(B) void copy_k(const float4* __restrict__ a, float4* __restrict__ o, int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * B + threadIdx.x; i < n4; i += (int64_t)gridDim.x * B) o[i] = a[i];
}
__global__ __launch_bounds__(B) void read_k(const float4* __restrict__ a, float* out, int64_t n4) {
  float s = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * B + threadIdx.x; i < n4; i += (int64_t)gridDim.x * B) {
    float4 v = a[i];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 123.456f) out[0] = s;
}
// the fused top-k step's dense traffic: read r, g; write r' = r + g and out = 0
__global__ __launch_bounds__(B) void r2w2_k(float4* __restrict__ r, const float4* __restrict__ g,
                                           float4* __restrict__ o, int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * B + threadIdx.x; i < n4; i += (int64_t)gridDim.x * B) {
    float4 a = r[i], b = g[i];
    r[i] = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
    o[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
}
// same, one chunk of 16384 elements per workgroup, 16 float4 per thread, unrolled x4
template <int U>
__global__ __launch_bounds__(B) void r2w2_chunk_k(float4* __restrict__ r, const float4* __restrict__ g,
                                                 float4* __restrict__ o, int64_t n4) {
  const int64_t base = (int64_t)blockIdx.x * (B * 16) + threadIdx.x;
  for (int it = 0; it < 16; it += U) {
    float4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) { a[u] = r[base + (it + u) * B]; b[u] = g[base + (it + u) * B]; }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      r[base + (it + u) * B] = make_float4(a[u].x + b[u].x, a[u].y + b[u].y, a[u].z + b[u].z, a[u].w + b[u].w);
      o[base + (it + u) * B] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
}
// nontemporal variants (NT_LD: loads, NT_ST: stores)
typedef float f4 __attribute__((ext_vector_type(4)));
template <bool NT_LD, bool NT_ST>
__global__ __launch_bounds__(B) void r2w2_nt_k(f4* __restrict__ r, const f4* __restrict__ g,
                                              f4* __restrict__ o, int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * B + threadIdx.x; i < n4; i += (int64_t)gridDim.x * B) {
    f4 a, b;
    if (NT_LD) { a = __builtin_nontemporal_load(r + i); b = __builtin_nontemporal_load(g + i); }
    else { a = r[i]; b = g[i]; }
    f4 x = a + b, z = {0.f, 0.f, 0.f, 0.f};
    if (NT_ST) { __builtin_nontemporal_store(x, r + i); __builtin_nontemporal_store(z, o + i); }
    else { r[i] = x; o[i] = z; }
  }
}
// the top-k main pass's layout without its classification: one 16384-element chunk per workgroup,
// groups of G float4 per lane per array, the next group's nt loads issued before the current group
// is added and stored (nt); dynamic LDS pins the workgroups per CU (occupancy)
template <int G>
__global__ __launch_bounds__(B) void r2w2_nt_chunk_k(f4* __restrict__ r, const f4* __restrict__ g,
                                                    f4* __restrict__ o, int64_t n4) {
  extern __shared__ float pin[];
  if (n4 < 0) pin[threadIdx.x] = 0.f;   // never: keeps the LDS allocation
  constexpr int NG = 16 / G;
  const int64_t base = (int64_t)blockIdx.x * (B * 16) + threadIdx.x;
  f4 a[G], b[G];
#pragma unroll
  for (int u = 0; u < G; ++u) { a[u] = __builtin_nontemporal_load(r + base + u * B); b[u] = __builtin_nontemporal_load(g + base + u * B); }
#pragma unroll 1
  for (int q = 0; q < NG; ++q) {
    f4 an[G], bn[G];
    if (q + 1 < NG) {
#pragma unroll
      for (int u = 0; u < G; ++u) {
        an[u] = __builtin_nontemporal_load(r + base + ((q + 1) * G + u) * B);
        bn[u] = __builtin_nontemporal_load(g + base + ((q + 1) * G + u) * B);
      }
    }
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const f4 z = {0.f, 0.f, 0.f, 0.f};
      __builtin_nontemporal_store(a[u] + b[u], r + base + (q * G + u) * B);
      __builtin_nontemporal_store(z, o + base + (q * G + u) * B);
    }
#pragma unroll
    for (int u = 0; u < G; ++u) { a[u] = an[u]; b[u] = bn[u]; }
  }
}
__global__ __launch_bounds__(B) void r2w2_nt_gs_lds_k(f4* __restrict__ r, const f4* __restrict__ g,
                                                     f4* __restrict__ o, int64_t n4) {
  extern __shared__ float pin[];
  if (n4 < 0) pin[threadIdx.x] = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * B + threadIdx.x; i < n4; i += (int64_t)gridDim.x * B) {
    f4 a = __builtin_nontemporal_load(r + i), b = __builtin_nontemporal_load(g + i);
    const f4 z = {0.f, 0.f, 0.f, 0.f};
    __builtin_nontemporal_store(a + b, r + i);
    __builtin_nontemporal_store(z, o + i);
  }
}
__global__ void scatter_k(const int* __restrict__ idx, int64_t k, float* __restrict__ o) {
  for (int64_t j = (int64_t)blockIdx.x * B + threadIdx.x; j < k; j += (int64_t)gridDim.x * B) o[idx[j]] = 1.f;
}
__global__ void empty_k() {}

template <typename F>
float time_ms(F f, int reps = 10) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) f();
  std::vector<float> v;
  for (int i = 0; i < reps; ++i) {
    CK(hipEventRecord(a));
    f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b)); v.push_back(ms);
  }
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main() {
  const int64_t n = 64ll * 1024 * 1024, n4 = n / 4;
  float *r, *g, *o, *x;
  CK(hipMalloc(&r, n * 4)); CK(hipMalloc(&g, n * 4)); CK(hipMalloc(&o, n * 4)); CK(hipMalloc(&x, n * 4));
  CK(hipMemset(r, 0, n * 4)); CK(hipMemset(g, 0, n * 4)); CK(hipMemset(o, 0, n * 4)); CK(hipMemset(x, 0, n * 4));
  float* sink; CK(hipMalloc(&sink, 4));
  for (int grid : {1024, 2048, 4096, 8192}) {
    float ms = time_ms([&] { copy_k<<<grid, B>>>((float4*)g, (float4*)o, n4); });
    printf("{\"probe\": \"copy 1R1W grid %d\", \"gbps\": %.1f}\n", grid, 8.0 * n / ms / 1e6);
    ms = time_ms([&] { read_k<<<grid, B>>>((float4*)g, sink, n4); });
    printf("{\"probe\": \"read 1R grid %d\", \"gbps\": %.1f}\n", grid, 4.0 * n / ms / 1e6);
    ms = time_ms([&] { r2w2_k<<<grid, B>>>((float4*)r, (float4*)g, (float4*)o, n4); });
    printf("{\"probe\": \"r2w2 grid-stride grid %d\", \"gbps\": %.1f}\n", grid, 16.0 * n / ms / 1e6);
  }
  for (int grid : {1024, 2048}) {
    float ms = time_ms([&] { r2w2_nt_k<false, true><<<grid, B>>>((f4*)r, (f4*)g, (f4*)o, n4); });
    printf("{\"probe\": \"r2w2 nt-store grid %d\", \"gbps\": %.1f}\n", grid, 16.0 * n / ms / 1e6);
    ms = time_ms([&] { r2w2_nt_k<true, true><<<grid, B>>>((f4*)r, (f4*)g, (f4*)o, n4); });
    printf("{\"probe\": \"r2w2 nt-load+store grid %d\", \"gbps\": %.1f}\n", grid, 16.0 * n / ms / 1e6);
    ms = time_ms([&] { r2w2_nt_k<true, false><<<grid, B>>>((f4*)r, (f4*)g, (f4*)o, n4); });
    printf("{\"probe\": \"r2w2 nt-load grid %d\", \"gbps\": %.1f}\n", grid, 16.0 * n / ms / 1e6);
  }
  {
    float ms = time_ms([&] { r2w2_chunk_k<4><<<n / 4096 / 4, B>>>((float4*)r, (float4*)g, (float4*)o, n4); });
    printf("{\"probe\": \"r2w2 chunk16384 U4\", \"gbps\": %.1f, \"us\": %.1f}\n", 16.0 * n / ms / 1e6, ms * 1e3);
    ms = time_ms([&] { r2w2_chunk_k<8><<<n / 4096 / 4, B>>>((float4*)r, (float4*)g, (float4*)o, n4); });
    printf("{\"probe\": \"r2w2 chunk16384 U8\", \"gbps\": %.1f, \"us\": %.1f}\n", 16.0 * n / ms / 1e6, ms * 1e3);
  }
  for (int lds : {0, 20 * 1024, 40 * 1024}) {   // 8+ / 8 / 4 workgroups per CU
    float ms = time_ms([&] { r2w2_nt_chunk_k<4><<<n / 4096 / 4, B, lds>>>((f4*)r, (f4*)g, (f4*)o, n4); });
    printf("{\"probe\": \"r2w2 nt chunk16384 G4 lds %d\", \"gbps\": %.1f, \"us\": %.1f}\n", lds, 16.0 * n / ms / 1e6, ms * 1e3);
    ms = time_ms([&] { r2w2_nt_chunk_k<2><<<n / 4096 / 4, B, lds>>>((f4*)r, (f4*)g, (f4*)o, n4); });
    printf("{\"probe\": \"r2w2 nt chunk16384 G2 lds %d\", \"gbps\": %.1f, \"us\": %.1f}\n", lds, 16.0 * n / ms / 1e6, ms * 1e3);
    for (int grid : {1024, 2048}) {
      ms = time_ms([&] { r2w2_nt_gs_lds_k<<<grid, B, lds>>>((f4*)r, (f4*)g, (f4*)o, n4); });
      printf("{\"probe\": \"r2w2 nt grid-stride grid %d lds %d\", \"gbps\": %.1f, \"us\": %.1f}\n", grid, lds, 16.0 * n / ms / 1e6, ms * 1e3);
    }
  }
  for (int64_t k : {100000ll, 227000ll, 671088ll}) {
    std::vector<int> h(k);
    srand(1);
    for (auto& v : h) v = (int)(((int64_t)rand() << 16 ^ rand()) % n);
    int* d; CK(hipMalloc(&d, k * 4)); CK(hipMemcpy(d, h.data(), k * 4, hipMemcpyHostToDevice));
    float ms = time_ms([&] { scatter_k<<<1024, B>>>(d, k, x); });
    printf("{\"probe\": \"scatter %lld random 4B writes\", \"us\": %.2f}\n", (long long)k, ms * 1e3);
    CK(hipFree(d));
  }
  {
    float ms = time_ms([&] { empty_k<<<1, 64>>>(); empty_k<<<1, 64>>>(); }, 50);
    printf("{\"probe\": \"two empty dependent launches\", \"us\": %.2f}\n", ms * 1e3);
  }
  return 0;
}
