// bf16x6 Winograd filter transform shared by wino_x6.hip (standalone launch)
// and prep.hip (the batched per-step re-layout).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mfma_util.h"

namespace gk {
namespace {

// 16-byte chunk q of a U row r (32 bf16 input channels) lives at chunk
// q ^ wx6_swz(r): a fragment read of 16 rows x one chunk spreads over all
// bank slots (the x62 GEMM image, gemm_kern.h x62_swz)
__host__ __device__ __forceinline__ int wx6_swz(int r) { return ((r >> 3) & 1) << 1; }

__device__ __forceinline__ uint16_t wx6_bf16(float f) { return (uint16_t)(pack_bf16x2(f, 0.f) & 0xffffu); }

// Filter transform G g G^T of one (co, ci) pair of the convolution being run
// (flip: the grad-input filter W'[c][kh][kw][k] = W[k][2-kh][2-kw][c] of the
// forward w = [K][3][3][C]), each of the 16 values split exactly into three
// bf16 parts (hi, mid, lo: round-to-nearest-even of the remaining residual),
// into u3 element (((s * 16 + xi) * 3 + plane) * Co + co) * 32 + chunk' * 8 +
// (ci & 7) with s = ci / 32, chunk' = ((ci & 31) >> 3) ^ wx6_swz(co).
__device__ __forceinline__ void wino_x6_pair(const float* __restrict__ w, uint16_t* __restrict__ u3, int Co, int Ci,
                                             int flip, int co, int ci) {
  float g[3][3];
#pragma unroll
  for (int kh = 0; kh < 3; ++kh)
#pragma unroll
    for (int kw = 0; kw < 3; ++kw)
      g[kh][kw] = flip ? w[((int64_t)ci * 9 + (2 - kh) * 3 + (2 - kw)) * Co + co]
                       : w[((int64_t)co * 9 + kh * 3 + kw) * Ci + ci];
  float t[4][3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    t[0][j] = g[0][j];
    t[1][j] = 0.5f * (g[0][j] + g[1][j] + g[2][j]);
    t[2][j] = 0.5f * (g[0][j] - g[1][j] + g[2][j]);
    t[3][j] = g[2][j];
  }
  float uv[16];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    uv[4 * i + 0] = t[i][0];
    uv[4 * i + 1] = 0.5f * (t[i][0] + t[i][1] + t[i][2]);
    uv[4 * i + 2] = 0.5f * (t[i][0] - t[i][1] + t[i][2]);
    uv[4 * i + 3] = t[i][2];
  }
  const int s = ci >> 5;
  const int col = ((((ci & 31) >> 3) ^ wx6_swz(co)) << 3) | (ci & 7);
  const int64_t ps = (int64_t)Co * 32;
#pragma unroll
  for (int xi = 0; xi < 16; ++xi) {
    const float v = uv[xi];
    const uint16_t hi = wx6_bf16(v);
    const float r1 = v - __uint_as_float((uint32_t)hi << 16);
    const uint16_t mi = wx6_bf16(r1);
    const uint16_t lo = wx6_bf16(r1 - __uint_as_float((uint32_t)mi << 16));
    uint16_t* dst = u3 + (((int64_t)(s * 16 + xi) * 3) * Co + co) * 32 + col;
    dst[0] = hi;
    dst[ps] = mi;
    dst[2 * ps] = lo;
  }
}

}  // namespace
}  // namespace gk
