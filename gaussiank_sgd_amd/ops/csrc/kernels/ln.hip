// Fused residual-add (+ dropout) + LayerNorm for transformer blocks, gfx950.
//
//   forward : h = x + dropout(a);  y = (h - mean) * rstd * gamma + beta
//   backward: dh = rstd * (g - mean(g) - xhat * mean(g * xhat)),  g = dy * gamma
//             dx = dh (residual branch), da = dh * mask / (1 - p)
//             dgamma = sum_rows dy * xhat, dbeta = sum_rows dy
// The post-LN BERT layer (x = LN(x + drop(W a + b))) otherwise runs a
// dropout kernel, an add, bf16->fp32 casts, an fp32 LayerNorm and a cast back
// in the forward and the mirror image in the backward (profiles/
// r01_bert_kernel_stats.csv).  Here each direction is one row pass (one wave
// per row, bf16 I/O, fp32 math, 16-byte vector accesses) plus, backward, a
// tiny column-partials finalize for dgamma / dbeta.  The dropout mask is kept
// as 1 bit per element and regenerated from nothing: it is a hash of
// (seed, row, column), so the backward needs no mask tensor at all.
#include <hip/hip_runtime.h>

#include "common.h"
#include "gk_kernels.h"

namespace gk {
namespace {

constexpr int kLnMaxChunks = 8;          // per lane: H <= 64 * 8 * 8 = 4096
constexpr int kLnRowsPerWave = 8;        // backward: rows per wave before column partials are flushed

__device__ __forceinline__ void load8(const uint16_t* p, float* v) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

__device__ __forceinline__ uint32_t bf16r(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x7fffffu)) return (u >> 16) | 0x40u;
  u += 0x7fffu + ((u >> 16) & 1u);
  return u >> 16;
}

__device__ __forceinline__ void store8(uint16_t* p, const float* v) {
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = bf16r(v[2 * i]) | (bf16r(v[2 * i + 1]) << 16);
  *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
}

// keep element (row, col) with probability 1 - p: hash < keep threshold
__device__ __forceinline__ bool keep(uint32_t seed, int64_t row, int col, uint32_t thr) {
  return hash_u32((uint32_t)(row * 8191 + col), seed ^ (uint32_t)(row >> 19)) < thr;
}

template <int CH>
__global__ __launch_bounds__(kBlock) void add_ln_fwd_kernel(const uint16_t* __restrict__ a,
                                                            const uint16_t* __restrict__ x,
                                                            const float* __restrict__ gamma,
                                                            const float* __restrict__ beta, uint16_t* __restrict__ y,
                                                            uint16_t* __restrict__ hsave, float* __restrict__ mean,
                                                            float* __restrict__ rstd, int64_t R, int H, float eps,
                                                            uint32_t seed, uint32_t thr, float scale) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  if (row >= R) return;
  const int nc = H >> 3;
  float h[CH][8];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < CH; ++j) {
    const int c = lane + j * 64;
    if (c < nc) {
      float av[8], xv[8];
      load8(a + row * H + c * 8, av);
      load8(x + row * H + c * 8, xv);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float ad = thr ? (keep(seed, row, c * 8 + i, thr) ? av[i] * scale : 0.f) : av[i];
        h[j][i] = xv[i] + ad;
        s += h[j][i];
      }
    }
  }
  const float mu = wave_sum(s) / (float)H;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < CH; ++j)
    if (lane + j * 64 < nc)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float d = h[j][i] - mu;
        q = fmaf(d, d, q);
      }
  const float rs = rsqrtf(wave_sum(q) / (float)H + eps);
#pragma unroll
  for (int j = 0; j < CH; ++j) {
    const int c = lane + j * 64;
    if (c < nc) {
      float o[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int col = c * 8 + i;
        o[i] = (h[j][i] - mu) * rs * (gamma ? gamma[col] : 1.f) + (beta ? beta[col] : 0.f);
      }
      store8(y + row * H + c * 8, o);
      store8(hsave + row * H + c * 8, h[j]);
    }
  }
  if (lane == 0) {
    mean[row] = mu;
    rstd[row] = rs;
  }
}

// one wave walks kLnRowsPerWave rows; lane owns columns (lane + 64 j)*8 .. +7
// and accumulates dgamma / dbeta partials for them in registers
template <int CH>
__global__ __launch_bounds__(kBlock) void add_ln_bwd_kernel(
    const uint16_t* __restrict__ dy, const uint16_t* __restrict__ hsave, const float* __restrict__ mean,
    const float* __restrict__ rstd, const float* __restrict__ gamma, uint16_t* __restrict__ dx,
    uint16_t* __restrict__ da, float* __restrict__ pg, float* __restrict__ pb, int64_t R, int H, uint32_t seed,
    uint32_t thr, float scale) {
  const int lane = threadIdx.x & 63;
  const int64_t wave_g = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  const int nc = H >> 3;
  float accg[CH][8], accb[CH][8];
#pragma unroll
  for (int j = 0; j < CH; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) accg[j][i] = accb[j][i] = 0.f;
  for (int rr = 0; rr < kLnRowsPerWave; ++rr) {
    const int64_t row = wave_g * kLnRowsPerWave + rr;
    if (row >= R) break;
    const float mu = mean[row], rs = rstd[row];
    float g[CH][8], xh[CH][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const int c = lane + j * 64;
      if (c < nc) {
        float dv[8], hv[8];
        load8(dy + row * H + c * 8, dv);
        load8(hsave + row * H + c * 8, hv);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int col = c * 8 + i;
          xh[j][i] = (hv[i] - mu) * rs;
          g[j][i] = dv[i] * (gamma ? gamma[col] : 1.f);
          s1 += g[j][i];
          s2 = fmaf(g[j][i], xh[j][i], s2);
          accg[j][i] = fmaf(dv[i], xh[j][i], accg[j][i]);
          accb[j][i] += dv[i];
        }
      }
    }
    const float m1 = wave_sum(s1) / (float)H, m2 = wave_sum(s2) / (float)H;
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const int c = lane + j * 64;
      if (c < nc) {
        float o[8], od[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          o[i] = rs * (g[j][i] - m1 - xh[j][i] * m2);
          if (da) od[i] = thr ? (keep(seed, row, c * 8 + i, thr) ? o[i] * scale : 0.f) : o[i];
        }
        store8(dx + row * H + c * 8, o);
        if (da) store8(da + row * H + c * 8, od);
      }
    }
  }
  // per-wave column partials: row wave_g of [nwaves][H]
#pragma unroll
  for (int j = 0; j < CH; ++j) {
    const int c = lane + j * 64;
    if (c < nc) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        pg[wave_g * H + c * 8 + i] = accg[j][i];
        pb[wave_g * H + c * 8 + i] = accb[j][i];
      }
    }
  }
}

// dgamma / dbeta (+)= column sums of the [P][H] partials.  A workgroup owns
// kFinCols columns; its threads split the P rows kFinParts ways with 8 loads
// in flight each (the partials are L2-resident: an un-pipelined loop is
// latency-bound), then combine in fp64 through LDS.
constexpr int kFinCols = 16;
constexpr int kFinParts = kBlock / kFinCols;

__global__ __launch_bounds__(kBlock) void ln_param_finalize_kernel(const float* __restrict__ pg,
                                                                   const float* __restrict__ pb, int64_t P, int H,
                                                                   float* __restrict__ dgamma,
                                                                   float* __restrict__ dbeta, int accumulate) {
  __shared__ double sh[2][kFinParts][kFinCols];
  const int cl = threadIdx.x % kFinCols;
  const int part = threadIdx.x / kFinCols;
  const int col = blockIdx.x * kFinCols + cl;
  double sg = 0.0, sb = 0.0;
  if (col < H) {
    int64_t r = part;
    for (; r + 7 * kFinParts < P; r += 8 * kFinParts) {
      float vg[8], vb[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        vg[u] = pg[(r + u * kFinParts) * H + col];
        vb[u] = pb[(r + u * kFinParts) * H + col];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        sg += vg[u];
        sb += vb[u];
      }
    }
    for (; r < P; r += kFinParts) {
      sg += pg[r * H + col];
      sb += pb[r * H + col];
    }
  }
  sh[0][part][cl] = sg;
  sh[1][part][cl] = sb;
  __syncthreads();
  if (part == 0 && col < H) {
    double tg = 0.0, tb = 0.0;
#pragma unroll
    for (int q = 0; q < kFinParts; ++q) {
      tg += sh[0][q][cl];
      tb += sh[1][q][cl];
    }
    if (dgamma) dgamma[col] = (accumulate ? dgamma[col] : 0.f) + (float)tg;
    if (dbeta) dbeta[col] = (accumulate ? dbeta[col] : 0.f) + (float)tb;
  }
}

}  // namespace

bool add_ln_supported(int H) { return H % 8 == 0 && H >= 8 && H <= 64 * 8 * kLnMaxChunks; }

int64_t add_ln_partial_rows(int64_t R) {
  const int64_t waves = (R + kLnRowsPerWave - 1) / kLnRowsPerWave;
  return (waves + kWavesPerBlock - 1) / kWavesPerBlock * kWavesPerBlock;
}

void add_ln_forward(const void* a, const void* x, const float* gamma, const float* beta, void* y, void* hsave,
                    float* mean, float* rstd, int64_t R, int H, float eps, float p, uint32_t seed,
                    hipStream_t stream) {
  const uint32_t thr = p > 0.f ? (uint32_t)((1.0 - (double)p) * 4294967295.0) : 0u;
  const float scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const unsigned grid = (unsigned)((R + kWavesPerBlock - 1) / kWavesPerBlock);
#define GK_LNF(CH)                                                                                                 \
  hipLaunchKernelGGL(add_ln_fwd_kernel<CH>, dim3(grid), dim3(kBlock), 0, stream, (const uint16_t*)a,              \
                     (const uint16_t*)x, gamma, beta, (uint16_t*)y, (uint16_t*)hsave, mean, rstd, R, H, eps, seed, \
                     thr, scale)
  const int ch = ((H >> 3) + 63) / 64;
  if (ch <= 1) GK_LNF(1);
  else if (ch <= 2) GK_LNF(2);
  else if (ch <= 4) GK_LNF(4);
  else GK_LNF(8);
#undef GK_LNF
}

void add_ln_backward(const void* dy, const void* hsave, const float* mean, const float* rstd, const float* gamma,
                     void* dx, void* da, float* dgamma, float* dbeta, int accumulate, float* ws, int64_t R, int H,
                     float p, uint32_t seed, hipStream_t stream) {
  const uint32_t thr = p > 0.f ? (uint32_t)((1.0 - (double)p) * 4294967295.0) : 0u;
  const float scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const int64_t P = add_ln_partial_rows(R);
  float* pg = ws;
  float* pb = ws + P * H;
  const unsigned grid = (unsigned)(P / kWavesPerBlock);
#define GK_LNB(CH)                                                                                                  \
  hipLaunchKernelGGL(add_ln_bwd_kernel<CH>, dim3(grid), dim3(kBlock), 0, stream, (const uint16_t*)dy,               \
                     (const uint16_t*)hsave, mean, rstd, gamma, (uint16_t*)dx, (uint16_t*)da, pg, pb, R, H, seed, \
                     thr, scale)
  const int ch = ((H >> 3) + 63) / 64;
  if (ch <= 1) GK_LNB(1);
  else if (ch <= 2) GK_LNB(2);
  else if (ch <= 4) GK_LNB(4);
  else GK_LNB(8);
#undef GK_LNB
  if (dgamma || dbeta)
    hipLaunchKernelGGL(ln_param_finalize_kernel, dim3((H + kFinCols - 1) / kFinCols), dim3(kBlock), 0, stream, pg,
                       pb, P, H, dgamma, dbeta, accumulate);
}

}  // namespace gk
