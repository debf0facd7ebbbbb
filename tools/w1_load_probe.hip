// Load-phase floor of psgd_w1_pass's access shape (DESIGN §4 "PowerSGD one-pass phases"):
// 64 MiB of M (4096 x 4096 f32), one read, no arithmetic beyond a sum that keeps the loads live.
//   v0  the pass's shape: grid (4 column groups, 64 slabs), 1024 threads, 16 row-interleaved
//       16-B non-temporal loads per lane, all issued at once
//   v1  v0 with plain loads
//   v2  2 workgroups per CU: grid (4, 128) x 512 threads, 16 rows per lane
//   v3  v0's grid with the rows issued in two halves (8 loads, wait, 8 loads)
//   v4  a grid-stride stream: 2048 workgroups x 256 threads, 4 x 16 B in flight per lane
//   v5  4 workgroups per CU: grid (4, 256) x 256 threads, 16 rows per lane
//   v6  2 workgroups per CU: grid (4, 128) x 1024 threads, 8 rows per lane
//   v7  4 workgroups per CU: grid (4, 256) x 512 threads, 8 rows per lane
// Five rotated M buffers (320 MiB > the 256 MiB Infinity Cache), hipEvent median of 15 launches.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/w1_load_probe tools/w1_load_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <algorithm>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int N = 4096, Mc = 4096;

template <int ROWS, int BLOCK, bool NT, int SPLIT>
__global__ __launch_bounds__(BLOCK) void shape_load(const float* __restrict__ M, float* __restrict__ sink, int S) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  constexpr int CW = 4;                       // column waves (256 columns each)
  const int cw = w % CW, rw = w / CW, RW = BLOCK / 64 / CW;
  const int cg = blockIdx.x, s = blockIdx.y;
  const int jo = cg * 1024 + 256 * cw + 4 * lane;
  const long L = (long)RW * S;
  const long lrow = (long)RW * s + rw;
  f4 v[ROWS];
#pragma unroll
  for (int d = 0; d < ROWS; ++d) {
    if (SPLIT && d == SPLIT) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const long row = lrow + L * d;
    const f4* p = reinterpret_cast<const f4*>(M + row * Mc + jo);
    v[d] = NT ? __builtin_nontemporal_load(p) : *p;
  }
  f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int d = 0; d < ROWS; ++d) acc += v[d];
  const float t = acc.x + acc.y + acc.z + acc.w;
  if (t == 12345.f) sink[0] = t;
}

__global__ __launch_bounds__(256) void stream_load(const f4* __restrict__ M, float* __restrict__ sink, long nq) {
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  const long stride = (long)gridDim.x * 256;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < nq; i += 4 * stride) {
    f4 a[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) a[u] = i + u * stride < nq ? __builtin_nontemporal_load(M + i + u * stride) : f4{0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < 4; ++u) acc += a[u];
  }
  const float t = acc.x + acc.y + acc.z + acc.w;
  if (t == 12345.f) sink[0] = t;
}

int main() {
  const size_t bytes = (size_t)N * Mc * 4;
  std::vector<float*> bufs(5);
  for (auto& b : bufs) { hipMalloc(&b, bytes); hipMemset(b, 0, bytes); }
  float* sink;
  hipMalloc(&sink, 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[] = {"v0 pass shape nt", "v1 pass shape plain", "v2 2 WG/CU 512 thr", "v3 two halves",
                         "v4 grid-stride stream", "v5 4 WG/CU 256 thr", "v6 2 WG/CU 1024 thr 8r", "v7 4 WG/CU 512 thr 8r"};
  for (int v = 0; v < 8; ++v) {
    std::vector<float> ts;
    for (int rep = 0; rep < 20; ++rep) {
      const float* M = bufs[rep % 5];
      hipEventRecord(e0, 0);
      switch (v) {
        case 0: shape_load<16, 1024, true, 0><<<dim3(4, 64), 1024>>>(M, sink, 64); break;
        case 1: shape_load<16, 1024, false, 0><<<dim3(4, 64), 1024>>>(M, sink, 64); break;
        case 2: shape_load<16, 512, true, 0><<<dim3(4, 128), 512>>>(M, sink, 128); break;
        case 3: shape_load<16, 1024, true, 8><<<dim3(4, 64), 1024>>>(M, sink, 64); break;
        case 4: stream_load<<<2048, 256>>>(reinterpret_cast<const f4*>(M), sink, (long)N * Mc / 4); break;
        case 5: shape_load<16, 256, true, 0><<<dim3(4, 256), 256>>>(M, sink, 256); break;
        case 6: shape_load<8, 1024, true, 0><<<dim3(4, 128), 1024>>>(M, sink, 128); break;
        case 7: shape_load<8, 512, true, 0><<<dim3(4, 256), 512>>>(M, sink, 256); break;
      }
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      if (rep >= 5) ts.push_back(ms * 1000.f);
    }
    std::sort(ts.begin(), ts.end());
    printf("%-24s median %7.2f us  min %7.2f us  -> %6.2f TB/s (median)\n", names[v], ts[ts.size() / 2], ts[0],
           bytes / (ts[ts.size() / 2] * 1e-6) / 1e12);
  }
  return 0;
}
