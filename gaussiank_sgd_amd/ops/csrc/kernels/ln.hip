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
// tiny column-partials finalize for dgamma / dbeta.  Storage bf16 (autocast)
// or fp32 (the reference's precision), fp32 math either way.  The dropout mask is kept
// as 1 bit per element and regenerated from nothing: it is a hash of
// (seed, row, column), so the backward needs no mask tensor at all.
#include <hip/hip_runtime.h>

#include "common.h"
#include "gk_kernels.h"

namespace gk {
namespace {

constexpr int kLnMaxChunks = 8;          // per lane: H <= 64 * 8 * 8 = 4096
constexpr int kLnRowsPerWave = 4;        // backward: rows per wave (RPW at a time)
constexpr int kLnRowsPerBlock = kLnRowsPerWave * kWavesPerBlock;   // backward: one partial row per block

__device__ __forceinline__ void load8(const uint16_t* p, float* v) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

__device__ __forceinline__ void load8f(const float* p, float* v) {
  const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
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

// 8-element chunks of either storage type: 16 bytes of bf16 or 32 of fp32
__device__ __forceinline__ void ld8(const uint16_t* p, float* v) { load8(p, v); }
__device__ __forceinline__ void ld8(const float* p, float* v) { load8f(p, v); }
__device__ __forceinline__ void st8(uint16_t* p, const float* v) { store8(p, v); }
__device__ __forceinline__ void st8(float* p, const float* v) {
  reinterpret_cast<float4*>(p)[0] = make_float4(v[0], v[1], v[2], v[3]);
  reinterpret_cast<float4*>(p)[1] = make_float4(v[4], v[5], v[6], v[7]);
}

// keep element (row, col) with probability 1 - p: hash < keep threshold
__device__ __forceinline__ bool keep(uint32_t seed, int64_t row, int col, uint32_t thr) {
  return hash_u32((uint32_t)(row * 8191 + col), seed ^ (uint32_t)(row >> 19)) < thr;
}

// sum over the L lanes of one row (L = 64 / rows-per-wave, a power of two)
template <int L>
__device__ __forceinline__ float row_sum(float v) {
#pragma unroll
  for (int off = L / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// RPW rows per wave, L = 64 / RPW lanes per row; lane sl owns 16-byte chunks
// sl + L j (j < CH) of its row.  BERT's H = 768 is 96 chunks: 2 rows per wave
// x 32 lanes x 3 chunks, every lane busy (one row per wave left half the
// lanes idle on the second chunk)
template <int CH, int RPW, typename T>
__global__ __launch_bounds__(kBlock) void add_ln_fwd_kernel(const T* __restrict__ a,
                                                            const T* __restrict__ x,
                                                            const float* __restrict__ gamma,
                                                            const float* __restrict__ beta, T* __restrict__ y,
                                                            T* __restrict__ hsave, float* __restrict__ mean,
                                                            float* __restrict__ rstd, int64_t R, int H, float eps,
                                                            uint32_t seed, uint32_t thr, float scale,
                                                            const uint32_t* __restrict__ seed_dev) {
  if (seed_dev != nullptr) seed = hash_u32(__builtin_amdgcn_readfirstlane(*seed_dev), seed);
  constexpr int L = 64 / RPW;
  const int lane = threadIdx.x & 63, sl = lane % L;
  const int64_t row0 = ((int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * RPW;
  if (row0 >= R) return;
  const int64_t row = row0 + lane / L;
  const bool rv = row < R;
  const int nc = H >> 3;
  float h[CH][8];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < CH; ++j) {
    const int c = sl + j * L;
#pragma unroll
    for (int i = 0; i < 8; ++i) h[j][i] = 0.f;
    if (rv && c < nc) {
      float av[8], xv[8];
      ld8(a + row * H + c * 8, av);
      ld8(x + row * H + c * 8, xv);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float ad = thr ? (keep(seed, row, c * 8 + i, thr) ? av[i] * scale : 0.f) : av[i];
        h[j][i] = xv[i] + ad;
        s += h[j][i];
      }
    }
  }
  const float mu = row_sum<L>(s) / (float)H;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < CH; ++j)
    if (rv && sl + j * L < nc)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float d = h[j][i] - mu;
        q = fmaf(d, d, q);
      }
  const float rs = rsqrtf(row_sum<L>(q) / (float)H + eps);
#pragma unroll
  for (int j = 0; j < CH; ++j) {
    const int c = sl + j * L;
    if (rv && c < nc) {
      float gv[8], bv[8], o[8];
      if (gamma) load8f(gamma + c * 8, gv);
      if (beta) load8f(beta + c * 8, bv);
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = (h[j][i] - mu) * rs * (gamma ? gv[i] : 1.f) + (beta ? bv[i] : 0.f);
      st8(y + row * H + c * 8, o);
      st8(hsave + row * H + c * 8, h[j]);
    }
  }
  if (rv && sl == 0) {
    mean[row] = mu;
    rstd[row] = rs;
  }
}

// A block walks kLnRowsPerBlock rows (each wave kLnRowsPerWave, RPW at a
// time); lanes accumulate dgamma / dbeta partials of their columns in
// registers, the block adds its waves' partials in a fixed order through LDS
// and writes ONE partial row (deterministic, no atomics).
template <int CH, int RPW, typename T>
__global__ __launch_bounds__(kBlock) void add_ln_bwd_kernel(
    const T* __restrict__ dy, const T* __restrict__ hsave, const float* __restrict__ mean,
    const float* __restrict__ rstd, const float* __restrict__ gamma, T* __restrict__ dx,
    T* __restrict__ da, float* __restrict__ pg, float* __restrict__ pb, int64_t R, int H, uint32_t seed,
    uint32_t thr, float scale, const uint32_t* __restrict__ seed_dev) {
  if (seed_dev != nullptr) seed = hash_u32(__builtin_amdgcn_readfirstlane(*seed_dev), seed);
  constexpr int L = 64 / RPW;
  __shared__ float red[2][64 * 8 * kLnMaxChunks];
  const int lane = threadIdx.x & 63, sl = lane % L, wave = threadIdx.x >> 6;
  const int nc = H >> 3;
  float accg[CH][8], accb[CH][8];
#pragma unroll
  for (int j = 0; j < CH; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) accg[j][i] = accb[j][i] = 0.f;
  const int64_t wrow = ((int64_t)blockIdx.x * kWavesPerBlock + wave) * kLnRowsPerWave;
#pragma unroll 1
  for (int rr = 0; rr < kLnRowsPerWave; rr += RPW) {
    const int64_t row = wrow + rr + lane / L;
    const bool rv = row < R;
    const float mu = rv ? mean[row] : 0.f, rs = rv ? rstd[row] : 0.f;
    float g[CH][8], xh[CH][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const int c = sl + j * L;
#pragma unroll
      for (int i = 0; i < 8; ++i) g[j][i] = xh[j][i] = 0.f;
      if (rv && c < nc) {
        float dv[8], hv[8], gv[8];
        ld8(dy + row * H + c * 8, dv);
        ld8(hsave + row * H + c * 8, hv);
        if (gamma) load8f(gamma + c * 8, gv);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          xh[j][i] = (hv[i] - mu) * rs;
          g[j][i] = gamma ? dv[i] * gv[i] : dv[i];
          s1 += g[j][i];
          s2 = fmaf(g[j][i], xh[j][i], s2);
          accg[j][i] = fmaf(dv[i], xh[j][i], accg[j][i]);
          accb[j][i] += dv[i];
        }
      }
    }
    const float m1 = row_sum<L>(s1) / (float)H, m2 = row_sum<L>(s2) / (float)H;
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const int c = sl + j * L;
      if (rv && c < nc) {
        float o[8], od[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          o[i] = rs * (g[j][i] - m1 - xh[j][i] * m2);
          if (da) od[i] = thr ? (keep(seed, row, c * 8 + i, thr) ? o[i] * scale : 0.f) : o[i];
        }
        st8(dx + row * H + c * 8, o);
        if (da) st8(da + row * H + c * 8, od);
      }
    }
  }
  // the row halves of a wave own the same columns: fold them first
  if (RPW == 2) {
#pragma unroll
    for (int j = 0; j < CH; ++j)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        accg[j][i] += __shfl_xor(accg[j][i], 32, 64);
        accb[j][i] += __shfl_xor(accb[j][i], 32, 64);
      }
  }
  // waves 0, 1, 2, 3 in turn into the block's LDS row (fixed order)
  for (int w = 0; w < kWavesPerBlock; ++w) {
    if (wave == w && lane < L) {
#pragma unroll
      for (int j = 0; j < CH; ++j) {
        const int c = sl + j * L;
        if (c < nc)
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            red[0][c * 8 + i] = w ? red[0][c * 8 + i] + accg[j][i] : accg[j][i];
            red[1][c * 8 + i] = w ? red[1][c * 8 + i] + accb[j][i] : accb[j][i];
          }
      }
    }
    __syncthreads();
  }
  for (int c4 = threadIdx.x; c4 < (H >> 2); c4 += kBlock) {
    reinterpret_cast<float4*>(pg + (int64_t)blockIdx.x * H)[c4] = reinterpret_cast<const float4*>(red[0])[c4];
    reinterpret_cast<float4*>(pb + (int64_t)blockIdx.x * H)[c4] = reinterpret_cast<const float4*>(red[1])[c4];
  }
}

// dgamma / dbeta (+)= column sums of the [P][H] partials, in two levels so
// the 6 MB of BERT partials stream at full width: level 1 (grid: 64-column
// slabs x kFinSplits row ranges) writes [kFinSplits][H] sums, level 2 adds
// those kFinSplits rows in order (fp64 within each level, deterministic).
constexpr int kFinSplits = 32;
constexpr int kFinParts = kBlock / 64;   // row interleave inside a level-1 block

__global__ __launch_bounds__(kBlock) void ln_param_partial_kernel(const float* __restrict__ pg,
                                                                  const float* __restrict__ pb, int64_t P, int H,
                                                                  float* __restrict__ q) {
  __shared__ double sh[2][kFinParts][64];
  const int cl = threadIdx.x & 63, part = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + cl;
  const int64_t per = (P + kFinSplits - 1) / kFinSplits;
  const int64_t r0 = blockIdx.y * per, r1 = r0 + per < P ? r0 + per : P;
  double sg = 0.0, sb = 0.0;
  if (col < H) {
    int64_t r = r0 + part;
    for (; r + 3 * kFinParts < r1; r += 4 * kFinParts) {
      float vg[4], vb[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        vg[u] = pg[(r + u * kFinParts) * H + col];
        vb[u] = pb[(r + u * kFinParts) * H + col];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        sg += vg[u];
        sb += vb[u];
      }
    }
    for (; r < r1; r += kFinParts) {
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
    for (int k = 0; k < kFinParts; ++k) {
      tg += sh[0][k][cl];
      tb += sh[1][k][cl];
    }
    q[(int64_t)blockIdx.y * H + col] = (float)tg;
    q[(int64_t)(kFinSplits + blockIdx.y) * H + col] = (float)tb;
  }
}

__global__ __launch_bounds__(kBlock) void ln_param_finalize_kernel(const float* __restrict__ q, int H,
                                                                   float* __restrict__ dgamma,
                                                                   float* __restrict__ dbeta, int accumulate) {
  const int col = blockIdx.x * kBlock + threadIdx.x;
  if (col >= H) return;
  double tg = 0.0, tb = 0.0;
#pragma unroll 8
  for (int k = 0; k < kFinSplits; ++k) {
    tg += q[(int64_t)k * H + col];
    tb += q[(int64_t)(kFinSplits + k) * H + col];
  }
  if (dgamma) dgamma[col] = (accumulate ? dgamma[col] : 0.f) + (float)tg;
  if (dbeta) dbeta[col] = (accumulate ? dbeta[col] : 0.f) + (float)tb;
}

// (CH, RPW) for a row of nc 16-byte chunks: two rows per wave up to 256
// chunks (H <= 2048), the fewest chunks per lane that cover the row
template <template <int, int> class Launch>
void ln_dispatch(int nc, Launch<1, 2> l12, Launch<2, 2> l22, Launch<3, 2> l32, Launch<4, 2> l42, Launch<6, 2> l62,
                 Launch<8, 2> l82, Launch<8, 1> l81) {
  if (nc <= 32) l12();
  else if (nc <= 64) l22();
  else if (nc <= 96) l32();
  else if (nc <= 128) l42();
  else if (nc <= 192) l62();
  else if (nc <= 256) l82();
  else l81();
}

}  // namespace

bool add_ln_supported(int H) { return H % 8 == 0 && H >= 8 && H <= 64 * 8 * kLnMaxChunks; }

int64_t add_ln_partial_rows(int64_t R) {
  // per-block partial rows + the [2][kFinSplits] level-1 sums (in rows of H)
  return (R + kLnRowsPerBlock - 1) / kLnRowsPerBlock + kFinSplits;
}

namespace {
struct LnFwdArgs {
  const void *a, *x;
  const float *gamma, *beta;
  void *y, *hsave;
  float *mean, *rstd;
  int64_t R;
  int H;
  float eps;
  uint32_t seed, thr;
  float scale;
  const uint32_t* seed_dev;
  hipStream_t stream;
  bool f32;
};

template <int CH, int RPW>
struct LnFwdLaunch {
  const LnFwdArgs* p;
  template <typename T>
  void go() const {
    const int64_t waves = (p->R + RPW - 1) / RPW;
    const unsigned grid = (unsigned)((waves + kWavesPerBlock - 1) / kWavesPerBlock);
    hipLaunchKernelGGL((add_ln_fwd_kernel<CH, RPW, T>), dim3(grid), dim3(kBlock), 0, p->stream,
                       static_cast<const T*>(p->a), static_cast<const T*>(p->x), p->gamma, p->beta,
                       static_cast<T*>(p->y), static_cast<T*>(p->hsave), p->mean, p->rstd, p->R, p->H, p->eps, p->seed,
                       p->thr, p->scale, p->seed_dev);
  }
  void operator()() const {
    if (p->f32) go<float>();
    else go<uint16_t>();
  }
};

struct LnBwdArgs {
  const void *dy, *hsave;
  const float *mean, *rstd, *gamma;
  void *dx, *da;
  float *pg, *pb;
  int64_t R;
  int H;
  uint32_t seed, thr;
  float scale;
  const uint32_t* seed_dev;
  hipStream_t stream;
  bool f32;
};

template <int CH, int RPW>
struct LnBwdLaunch {
  const LnBwdArgs* p;
  template <typename T>
  void go() const {
    hipLaunchKernelGGL((add_ln_bwd_kernel<CH, RPW, T>), dim3((unsigned)((p->R + kLnRowsPerBlock - 1) / kLnRowsPerBlock)),
                       dim3(kBlock), 0, p->stream, static_cast<const T*>(p->dy), static_cast<const T*>(p->hsave),
                       p->mean, p->rstd, p->gamma, static_cast<T*>(p->dx), static_cast<T*>(p->da), p->pg, p->pb, p->R,
                       p->H, p->seed, p->thr, p->scale, p->seed_dev);
  }
  void operator()() const {
    if (p->f32) go<float>();
    else go<uint16_t>();
  }
};
}  // namespace

void add_ln_forward(const void* a, const void* x, const float* gamma, const float* beta, void* y, void* hsave,
                    float* mean, float* rstd, int64_t R, int H, float eps, float p, uint32_t seed,
                    const uint32_t* seed_dev, hipStream_t stream, bool f32) {
  const uint32_t thr = p > 0.f ? (uint32_t)((1.0 - (double)p) * 4294967295.0) : 0u;
  const float scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const LnFwdArgs args{a, x, gamma, beta, y, hsave, mean, rstd, R, H, eps, seed, thr, scale, seed_dev, stream, f32};
  ln_dispatch<LnFwdLaunch>(H >> 3, {&args}, {&args}, {&args}, {&args}, {&args}, {&args}, {&args});
}

void add_ln_backward(const void* dy, const void* hsave, const float* mean, const float* rstd, const float* gamma,
                     void* dx, void* da, float* dgamma, float* dbeta, int accumulate, float* ws, int64_t R, int H,
                     float p, uint32_t seed, const uint32_t* seed_dev, hipStream_t stream, bool f32) {
  const uint32_t thr = p > 0.f ? (uint32_t)((1.0 - (double)p) * 4294967295.0) : 0u;
  const float scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const int64_t P = (R + kLnRowsPerBlock - 1) / kLnRowsPerBlock;
  float* pg = ws;
  float* pb = ws + P * H;
  float* q = ws + 2 * P * H;   // [2][kFinSplits][H]: fits the 2 * add_ln_partial_rows(R) * H of the workspace
  const LnBwdArgs args{dy, hsave, mean, rstd, gamma, dx, da, pg, pb, R, H, seed, thr, scale, seed_dev, stream, f32};
  ln_dispatch<LnBwdLaunch>(H >> 3, {&args}, {&args}, {&args}, {&args}, {&args}, {&args}, {&args});
  if (dgamma || dbeta) {
    hipLaunchKernelGGL(ln_param_partial_kernel, dim3((H + 63) / 64, kFinSplits), dim3(kBlock), 0, stream, pg, pb, P, H,
                       q);
    hipLaunchKernelGGL(ln_param_finalize_kernel, dim3((H + kBlock - 1) / kBlock), dim3(kBlock), 0, stream, q, H,
                       dgamma, dbeta, accumulate);
  }
}

}  // namespace gk
