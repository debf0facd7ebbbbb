// Packed wire formats for the sign / ternary codecs.
//
//   1-bit: sign codes u8 {0,1} (signsgd.py:13-16) -> bit i of byte i/8 (LSB first), 8x smaller
//          on the wire; a layout of the same codewords, unpacking to the identical u8 tensor.
//          Majority decode (signsgd.py:24-30: sum of +-1 >= 0) runs directly on W packed
//          payloads with popcounts.
//   2-bit: grace_dl/tensorflow/compressor/packing.py:4-29 exactly: values 0..3 padded with
//          range(0, 4 - n % 4) (4 pad values when n % 4 == 0), split into four planar quarters,
//          byte j = a[j] + 4 a[q + j] + 16 a[2q + j] + 64 a[3q + j] (q = padded / 4).  TernGrad
//          codes travel as code + 1.
#include "common.h"

namespace grace {

constexpr int kWBlock = 256;

// 32 codes -> one u32 word (thread per word; two 16-B loads per thread)
__global__ __launch_bounds__(kWBlock) void pack_bits_kernel(const uint8_t* __restrict__ codes, int64_t n,
                                                           uint32_t* __restrict__ words, int64_t nw) {
  for (int64_t w = (int64_t)blockIdx.x * kWBlock + threadIdx.x; w < nw; w += (int64_t)gridDim.x * kWBlock) {
    const int64_t e = w * 32;
    uint32_t bits = 0;
    if (e + 31 < n && (reinterpret_cast<uintptr_t>(codes) & 15u) == 0) {
      const uint4 a = reinterpret_cast<const uint4*>(codes + e)[0];
      const uint4 b = reinterpret_cast<const uint4*>(codes + e)[1];
      const uint32_t v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
      for (int q = 0; q < 8; ++q)
#pragma unroll
        for (int j = 0; j < 4; ++j) bits |= (((v[q] >> (8 * j)) & 1u) ? 1u : 0u) << (4 * q + j);
    } else {
      for (int j = 0; j < 32 && e + j < n; ++j) bits |= (codes[e + j] ? 1u : 0u) << j;
    }
    words[w] = bits;
  }
}

__global__ __launch_bounds__(kWBlock) void unpack_bits_kernel(const uint32_t* __restrict__ words, int64_t n,
                                                             uint8_t* __restrict__ codes, int64_t nw) {
  for (int64_t w = (int64_t)blockIdx.x * kWBlock + threadIdx.x; w < nw; w += (int64_t)gridDim.x * kWBlock) {
    const uint32_t bits = words[w];
    const int64_t e = w * 32;
    if (e + 31 < n && (reinterpret_cast<uintptr_t>(codes) & 15u) == 0) {
      uint32_t v[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        uint32_t x = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) x |= ((bits >> (4 * q + j)) & 1u) << (8 * j);
        v[q] = x;
      }
      reinterpret_cast<uint4*>(codes + e)[0] = make_uint4(v[0], v[1], v[2], v[3]);
      reinterpret_cast<uint4*>(codes + e)[1] = make_uint4(v[4], v[5], v[6], v[7]);
    } else {
      for (int j = 0; j < 32 && e + j < n; ++j) codes[e + j] = (uint8_t)((bits >> j) & 1u);
    }
  }
}

// majority over W packed payloads (rank w's words at + w * stride): +1 where 2 * ones >= W.
// Lane l of a wave owns elements base + 4 l .. + 3 (the 4-bit nibble l % 8 of word base / 32 + l / 8;
// the 8 lanes of a word read it together), counts its 4 bits over the ranks and stores one float4:
// every store instruction writes 1 KB contiguous.  (A thread per word storing its 32 floats one by
// one touched 64 lines per instruction: 0.24 ms for a 256 MiB decode + encode.)
constexpr int kMajU = 4;   // 256-element wave slices per lane per round
__global__ __launch_bounds__(kWBlock) void majority_bits_kernel(const uint32_t* __restrict__ words, int64_t stride,
                                                               int world, int64_t n, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = (int64_t)gridDim.x * (kWBlock / 64);
  const int64_t wave = (int64_t)blockIdx.x * (kWBlock / 64) + (threadIdx.x >> 6);
  const bool vec = (reinterpret_cast<uintptr_t>(out) & 15u) == 0;
  for (int64_t base = wave * 256 * kMajU; base < n; base += nwaves * 256 * kMajU) {
    uint32_t ones[kMajU][4] = {};
    for (int r = 0; r < world; ++r) {
      uint32_t wv[kMajU];
#pragma unroll
      for (int u = 0; u < kMajU; ++u) {   // every word of the round in flight before any is used
        const int64_t e = base + 256 * u + 4 * lane;
        wv[u] = e < n ? words[r * stride + (e >> 5)] : 0u;
      }
#pragma unroll
      for (int u = 0; u < kMajU; ++u) {
        const uint32_t nib = wv[u] >> (4 * (lane & 7));
#pragma unroll
        for (int j = 0; j < 4; ++j) ones[u][j] += (nib >> j) & 1u;
      }
    }
#pragma unroll
    for (int u = 0; u < kMajU; ++u) {
      const int64_t e = base + 256 * u + 4 * lane;
      float v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = 2 * (int)ones[u][j] - world >= 0 ? 1.f : -1.f;
      if (vec && e + 3 < n) {
        *reinterpret_cast<float4*>(out + e) = make_float4(v[0], v[1], v[2], v[3]);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (e + j < n) out[e + j] = v[j];
      }
    }
  }
}

// sign encode straight into the 1-bit layout (signsgd.py:13-16, code = x >= 0: -0 -> 1, NaN -> 0):
// lane l reads elements base + 4 l .. + 3 as one float4, four wave ballots collect the codes, and
// lanes 0..7 assemble and store the wave's 8 words (bit e % 32 of word e / 32, LSB first, as
// pack_bits_kernel).  The u8 codes are never stored.
__device__ __forceinline__ uint32_t spread4(uint32_t b) {   // bit i of b (i < 8) -> bit 4 i
  b = (b | (b << 12)) & 0x000F000Fu;
  b = (b | (b << 6)) & 0x03030303u;
  b = (b | (b << 3)) & 0x11111111u;
  return b;
}
constexpr int kEncU = 4;
__global__ __launch_bounds__(kWBlock) void sign_encode_bits_kernel(const float* __restrict__ x, int64_t n,
                                                                  uint32_t* __restrict__ words) {
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = (int64_t)gridDim.x * (kWBlock / 64);
  const int64_t wave = (int64_t)blockIdx.x * (kWBlock / 64) + (threadIdx.x >> 6);
  const bool vec = (reinterpret_cast<uintptr_t>(x) & 15u) == 0;
  const int64_t nw = (n + 31) >> 5;
  for (int64_t base = wave * 256 * kEncU; base < n; base += nwaves * 256 * kEncU) {
    float v[kEncU][4];
#pragma unroll
    for (int u = 0; u < kEncU; ++u) {
      const int64_t e = base + 256 * u + 4 * lane;
      if (vec && e + 3 < n) {
        typedef float f4v __attribute__((ext_vector_type(4)));
        const f4v q = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(x + e));
        v[u][0] = q.x; v[u][1] = q.y; v[u][2] = q.z; v[u][3] = q.w;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[u][j] = e + j < n ? x[e + j] : -1.f;   // past n: code 0
      }
    }
#pragma unroll
    for (int u = 0; u < kEncU; ++u) {
      uint64_t bal[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) bal[j] = __ballot(v[u][j] >= 0.f);
      if (lane < 8) {
        uint32_t wd = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) wd |= spread4((uint32_t)(bal[j] >> (8 * lane)) & 0xFFu) << j;
        const int64_t wi = ((base + 256 * u) >> 5) + lane;
        if (wi < nw) words[wi] = wd;
      }
    }
  }
}

// packing.py encode_byte: values 0..3 (u8), planar quarters
__global__ __launch_bounds__(kWBlock) void pack2_kernel(const uint8_t* __restrict__ a, int64_t n, int64_t q,
                                                       uint8_t* __restrict__ out) {
  for (int64_t j = (int64_t)blockIdx.x * kWBlock + threadIdx.x; j < q; j += (int64_t)gridDim.x * kWBlock) {
    uint32_t b = 0;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int64_t i = s * q + j;
      const uint32_t v = i < n ? (uint32_t)(a[i] & 3u) : (uint32_t)(i - n);   // pad = range(0, pad_size)
      b |= v << (2 * s);
    }
    out[j] = (uint8_t)b;
  }
}

__global__ __launch_bounds__(kWBlock) void unpack2_kernel(const uint8_t* __restrict__ packed, int64_t n, int64_t q,
                                                         uint8_t* __restrict__ a) {
  for (int64_t j = (int64_t)blockIdx.x * kWBlock + threadIdx.x; j < q; j += (int64_t)gridDim.x * kWBlock) {
    const uint32_t b = packed[j];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int64_t i = s * q + j;
      if (i < n) a[i] = (uint8_t)((b >> (2 * s)) & 3u);
    }
  }
}

// TernGrad codes int8 {-1,0,1} <-> packing values code + 1
__global__ __launch_bounds__(kWBlock) void tern_to_pack_kernel(const int8_t* __restrict__ c, int64_t n, int64_t q,
                                                              uint8_t* __restrict__ out) {
  for (int64_t j = (int64_t)blockIdx.x * kWBlock + threadIdx.x; j < q; j += (int64_t)gridDim.x * kWBlock) {
    uint32_t b = 0;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int64_t i = s * q + j;
      const uint32_t v = i < n ? (uint32_t)(c[i] + 1) & 3u : (uint32_t)(i - n);
      b |= v << (2 * s);
    }
    out[j] = (uint8_t)b;
  }
}

__global__ __launch_bounds__(kWBlock) void pack_to_tern_kernel(const uint8_t* __restrict__ packed, int64_t n, int64_t q,
                                                              int8_t* __restrict__ c) {
  for (int64_t j = (int64_t)blockIdx.x * kWBlock + threadIdx.x; j < q; j += (int64_t)gridDim.x * kWBlock) {
    const uint32_t b = packed[j];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int64_t i = s * q + j;
      if (i < n) c[i] = (int8_t)((int)((b >> (2 * s)) & 3u) - 1);
    }
  }
}

}  // namespace grace

using namespace grace;

extern "C" {

int64_t grace_pack2_bytes(int64_t n) { return (n + (4 - n % 4)) / 4; }

grace_status_t grace_pack_bits(const uint8_t* codes, int64_t n, uint32_t* words, void* stream) {
  GRACE_REQUIRE(codes && words && n >= 0, "grace_pack_bits: bad arguments");
  const int64_t nw = (n + 31) / 32;
  if (nw == 0) return GRACE_OK;
  pack_bits_kernel<<<stream_grid(nw, kWBlock, 2048), kWBlock, 0, as_stream(stream)>>>(codes, n, words, nw);
  GRACE_CHECK_LAUNCH("grace_pack_bits");
  return GRACE_OK;
}

grace_status_t grace_sign_encode_bits(const float* x, int64_t n, uint32_t* words, void* stream) {
  GRACE_REQUIRE(x && words && n >= 0, "grace_sign_encode_bits: bad arguments");
  if (n == 0) return GRACE_OK;
  sign_encode_bits_kernel<<<stream_grid((n + 1023) / 1024, kEncU, 4096), kWBlock, 0, as_stream(stream)>>>(x, n, words);
  GRACE_CHECK_LAUNCH("grace_sign_encode_bits");
  return GRACE_OK;
}

grace_status_t grace_unpack_bits(const uint32_t* words, int64_t n, uint8_t* codes, void* stream) {
  GRACE_REQUIRE(codes && words && n >= 0, "grace_unpack_bits: bad arguments");
  const int64_t nw = (n + 31) / 32;
  if (nw == 0) return GRACE_OK;
  unpack_bits_kernel<<<stream_grid(nw, kWBlock, 2048), kWBlock, 0, as_stream(stream)>>>(words, n, codes, nw);
  GRACE_CHECK_LAUNCH("grace_unpack_bits");
  return GRACE_OK;
}

grace_status_t grace_sign_majority_bits(const uint32_t* words, int64_t stride_words, int32_t world, int64_t n,
                                        float* out, void* stream) {
  GRACE_REQUIRE(words && out && world >= 1 && world <= 63 && n >= 0, "grace_sign_majority_bits: bad arguments");
  const int64_t nw = (n + 31) / 32;
  if (nw == 0) return GRACE_OK;
  majority_bits_kernel<<<stream_grid((n + 1023) / 1024, kMajU, 4096), kWBlock, 0, as_stream(stream)>>>(
      words, stride_words, world, n, out);
  GRACE_CHECK_LAUNCH("grace_sign_majority_bits");
  return GRACE_OK;
}

grace_status_t grace_pack2(const uint8_t* values, int64_t n, uint8_t* packed, void* stream) {
  GRACE_REQUIRE(values && packed && n >= 0, "grace_pack2: bad arguments");
  const int64_t q = grace_pack2_bytes(n);
  pack2_kernel<<<stream_grid(q, kWBlock, 2048), kWBlock, 0, as_stream(stream)>>>(values, n, q, packed);
  GRACE_CHECK_LAUNCH("grace_pack2");
  return GRACE_OK;
}

grace_status_t grace_unpack2(const uint8_t* packed, int64_t n, uint8_t* values, void* stream) {
  GRACE_REQUIRE(values && packed && n >= 0, "grace_unpack2: bad arguments");
  const int64_t q = grace_pack2_bytes(n);
  unpack2_kernel<<<stream_grid(q, kWBlock, 2048), kWBlock, 0, as_stream(stream)>>>(packed, n, q, values);
  GRACE_CHECK_LAUNCH("grace_unpack2");
  return GRACE_OK;
}

grace_status_t grace_tern_pack(const int8_t* codes, int64_t n, uint8_t* packed, void* stream) {
  GRACE_REQUIRE(codes && packed && n >= 0, "grace_tern_pack: bad arguments");
  const int64_t q = grace_pack2_bytes(n);
  tern_to_pack_kernel<<<stream_grid(q, kWBlock, 2048), kWBlock, 0, as_stream(stream)>>>(codes, n, q, packed);
  GRACE_CHECK_LAUNCH("grace_tern_pack");
  return GRACE_OK;
}

grace_status_t grace_tern_unpack(const uint8_t* packed, int64_t n, int8_t* codes, void* stream) {
  GRACE_REQUIRE(codes && packed && n >= 0, "grace_tern_unpack: bad arguments");
  const int64_t q = grace_pack2_bytes(n);
  pack_to_tern_kernel<<<stream_grid(q, kWBlock, 2048), kWBlock, 0, as_stream(stream)>>>(packed, n, q, codes);
  GRACE_CHECK_LAUNCH("grace_tern_unpack");
  return GRACE_OK;
}

}  // extern "C"
