// Fused batch-norm (training) + residual add + ReLU for channels-last (NHWC)
// activations on gfx950.
//
// ResNet-style blocks spend ~1/3 of a training step in MIOpen's NHWC batch
// norm plus separate ReLU / residual-add passes (profiles/r01_*).  Here one
// BN layer is:
//   forward : stats (grid)  -> per-block per-channel sum / sum^2 (fp32)
//             finalize      -> mean, invstd, scale, shift, running stats
//             apply (grid)  -> y = act(x*scale + shift [+ residual])
//   backward: reduce (grid) -> sum dz, sum dz*xhat   (dz = dy * relu mask)
//             finalize      -> dgamma, dbeta
//             apply (grid)  -> dx = scale*(dz - dbeta/M - xhat*dgamma/M),
//                              dresidual = dz
// so the ReLU mask, the residual gradient and the normalisation share the
// same streaming passes.  The forward writes the ReLU mask as 1 bit per
// element (1 byte per 16-byte vector); the backward reads it instead of y,
// cutting the backward's read traffic by a third.  Activations are viewed as [M = N*H*W, C]; each
// thread owns 16 contiguous bytes of channels (8 bf16 / 4 fp32) and walks
// rows, so every wave reads whole 1-KiB contiguous runs.  Statistics are
// accumulated in fp32 per thread and combined in fp64.
#include <hip/hip_runtime.h>

#include "common.h"
#include "gk_kernels.h"

namespace gk {
namespace {

__device__ __forceinline__ float bf16_to_f32(uint16_t h) { return __uint_as_float(((uint32_t)h) << 16); }

__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x7fffffu)) return (uint16_t)((u >> 16) | 0x40);  // NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

// 16-byte vector of VEC elements of T, converted to/from fp32.
template <typename T>
struct Vec;

template <>
struct Vec<uint16_t> {  // bf16
  static constexpr int N = 8;
  __device__ static void load(const uint16_t* p, float* v) {
    const uint4 u = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(w[i] << 16);
      v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
  __device__ static void store(uint16_t* p, const float* v) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = (uint32_t)f32_to_bf16(v[2 * i]) | ((uint32_t)f32_to_bf16(v[2 * i + 1]) << 16);
    *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
  }
};

template <>
struct Vec<float> {
  static constexpr int N = 4;
  __device__ static void load(const float* p, float* v) {
    const float4 f = *reinterpret_cast<const float4*>(p);
    v[0] = f.x; v[1] = f.y; v[2] = f.z; v[3] = f.w;
  }
  __device__ static void store(float* p, const float* v) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  }
};

struct Geo {
  int tpr;      // threads across the channel tile
  int rl;       // row lanes per block
  int ct;       // channels per tile
  int gx;       // channel tiles
  int gy;       // row chunks
  int64_t rows_per_block;
};

template <typename T>
Geo make_geo(int64_t M, int C, int target_blocks) {
  constexpr int V = Vec<T>::N;
  Geo g;
  int cv = C / V;
  g.tpr = cv < 64 ? cv : 64;
  while (cv % g.tpr) --g.tpr;  // tpr divides C/V
  g.ct = g.tpr * V;
  g.rl = kBlock / g.tpr;
  g.gx = C / g.ct;
  int64_t gy = (target_blocks + g.gx - 1) / g.gx;
  const int64_t max_gy = (M + g.rl - 1) / g.rl;
  if (gy > max_gy) gy = max_gy;
  if (gy < 1) gy = 1;
  g.gy = (int)gy;
  g.rows_per_block = (M + g.gy - 1) / g.gy;
  return g;
}

// ---------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(kBlock) void bn_stats_kernel(const T* __restrict__ x, int64_t M, int C, Geo g,
                                                          float* __restrict__ psum, float* __restrict__ psq) {
  constexpr int V = Vec<T>::N;
  const int tc = threadIdx.x % g.tpr;
  const int lane_r = threadIdx.x / g.tpr;
  const int c0 = blockIdx.x * g.ct + tc * V;
  const int64_t r0 = (int64_t)blockIdx.y * g.rows_per_block;
  int64_t r1 = r0 + g.rows_per_block;
  if (r1 > M) r1 = M;
  float s[V], q[V];
#pragma unroll
  for (int i = 0; i < V; ++i) s[i] = q[i] = 0.f;
  for (int64_t r = (lane_r < g.rl ? r0 + lane_r : r1); r < r1; r += g.rl) {
    float v[V];
    Vec<T>::load(x + r * C + c0, v);
#pragma unroll
    for (int i = 0; i < V; ++i) {
      s[i] += v[i];
      q[i] = fmaf(v[i], v[i], q[i]);
    }
  }
  __shared__ float sh[2][kBlock * 8];
#pragma unroll
  for (int i = 0; i < V; ++i) {
    sh[0][threadIdx.x * V + i] = s[i];
    sh[1][threadIdx.x * V + i] = q[i];
  }
  __syncthreads();
  // reduce over row lanes: thread t < ct handles channel (tile-local) t
  for (int cl = threadIdx.x; cl < g.ct; cl += kBlock) {
    const int t = cl / V, i = cl % V;
    float a = 0.f, b = 0.f;
    for (int l = 0; l < g.rl; ++l) {
      a += sh[0][(l * g.tpr + t) * V + i];
      b += sh[1][(l * g.tpr + t) * V + i];
    }
    const int c = blockIdx.x * g.ct + cl;
    psum[(int64_t)blockIdx.y * C + c] = a;
    psq[(int64_t)blockIdx.y * C + c] = b;
  }
}

// Per-channel reduction of the [gy][C] partials: a workgroup owns kFinC
// channels; its 256 threads split the gy rows kFinParts ways and keep 8 loads
// in flight per thread (the partials are L2-resident; an un-pipelined loop is
// latency-bound), then combine the partial sums in fp64 through LDS.
constexpr int kFinC = 16;
constexpr int kFinParts = kBlock / kFinC;

__device__ __forceinline__ void reduce_partials2(const float* __restrict__ pa, const float* __restrict__ pb, int gy,
                                                 int C, double* out_a, double* out_b, bool* owner, int* c_out) {
  __shared__ double sh[2][kFinParts][kFinC];
  const int cl = threadIdx.x % kFinC;
  const int part = threadIdx.x / kFinC;
  const int c = blockIdx.x * kFinC + cl;
  double a = 0.0, b = 0.0;
  if (c < C) {
    int j = part;
    for (; j + 7 * kFinParts < gy; j += 8 * kFinParts) {
      float va[8], vb[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        va[u] = pa[(int64_t)(j + u * kFinParts) * C + c];
        vb[u] = pb[(int64_t)(j + u * kFinParts) * C + c];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        a += va[u];
        b += vb[u];
      }
    }
    for (; j < gy; j += kFinParts) {
      a += pa[(int64_t)j * C + c];
      b += pb[(int64_t)j * C + c];
    }
  }
  sh[0][part][cl] = a;
  sh[1][part][cl] = b;
  __syncthreads();
  *owner = part == 0 && c < C;
  *c_out = c;
  if (part == 0) {
    double sa = 0.0, sb = 0.0;
#pragma unroll
    for (int p = 0; p < kFinParts; ++p) {
      sa += sh[0][p][cl];
      sb += sh[1][p][cl];
    }
    *out_a = sa;
    *out_b = sb;
  }
}

__global__ __launch_bounds__(kBlock) void bn_finalize_kernel(const float* __restrict__ psum,
                                                             const float* __restrict__ psq, int gy, int64_t M, int C,
                                                             const float* __restrict__ w, const float* __restrict__ b,
                                                             float eps, float momentum, float* __restrict__ run_mean,
                                                             float* __restrict__ run_var, float* __restrict__ save_mean,
                                                             float* __restrict__ save_invstd, float* __restrict__ scale,
                                                             float* __restrict__ shift) {
  double s = 0.0, q = 0.0;
  bool owner;
  int c;
  reduce_partials2(psum, psq, gy, C, &s, &q, &owner, &c);
  if (!owner) return;
  const double mean = s / (double)M;
  double var = q / (double)M - mean * mean;
  if (var < 0.0) var = 0.0;
  const float invstd = (float)(1.0 / sqrt(var + (double)eps));
  const float gam = w ? w[c] : 1.f;
  const float bet = b ? b[c] : 0.f;
  save_mean[c] = (float)mean;
  save_invstd[c] = invstd;
  scale[c] = gam * invstd;
  shift[c] = bet - (float)mean * gam * invstd;
  if (run_mean) {
    const double unbiased = M > 1 ? var * (double)M / (double)(M - 1) : var;
    run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * (float)mean;
    run_var[c] = (1.f - momentum) * run_var[c] + momentum * (float)unbiased;
  }
}

template <typename T, bool RELU, bool RES>
__global__ __launch_bounds__(kBlock) void bn_apply_kernel(const T* __restrict__ x, const T* __restrict__ res,
                                                          T* __restrict__ y, uint8_t* __restrict__ mask, int64_t M,
                                                          int C, Geo g, const float* __restrict__ scale,
                                                          const float* __restrict__ shift) {
  constexpr int V = Vec<T>::N;
  const int tc = threadIdx.x % g.tpr;
  const int lane_r = threadIdx.x / g.tpr;
  const int c0 = blockIdx.x * g.ct + tc * V;
  float sc[V], sf[V];
#pragma unroll
  for (int i = 0; i < V; ++i) { sc[i] = scale[c0 + i]; sf[i] = shift[c0 + i]; }
  const int64_t r0 = (int64_t)blockIdx.y * g.rows_per_block;
  int64_t r1 = r0 + g.rows_per_block;
  if (r1 > M) r1 = M;
  for (int64_t r = (lane_r < g.rl ? r0 + lane_r : r1); r < r1; r += g.rl) {
    float v[V];
    Vec<T>::load(x + r * C + c0, v);
    float rv[V];
    if (RES) Vec<T>::load(res + r * C + c0, rv);
    uint32_t bits = 0;
#pragma unroll
    for (int i = 0; i < V; ++i) {
      float o = fmaf(v[i], sc[i], sf[i]);
      if (RES) o += rv[i];
      if (RELU) {
        bits |= (o > 0.f ? 1u : 0u) << i;
        o = fmaxf(o, 0.f);
      }
      v[i] = o;
    }
    Vec<T>::store(y + r * C + c0, v);
    if (RELU) mask[r * (C / V) + c0 / V] = (uint8_t)bits;
  }
}

// ---------------------------------------------------------------------------
// backward
// ---------------------------------------------------------------------------
template <typename T, bool RELU>
__global__ __launch_bounds__(kBlock) void bn_bwd_reduce_kernel(const T* __restrict__ dy, const uint8_t* __restrict__ mask,
                                                               const T* __restrict__ x, int64_t M, int C, Geo g,
                                                               const float* __restrict__ mean,
                                                               const float* __restrict__ invstd,
                                                               float* __restrict__ pdb, float* __restrict__ pdg) {
  constexpr int V = Vec<T>::N;
  const int tc = threadIdx.x % g.tpr;
  const int lane_r = threadIdx.x / g.tpr;
  const int c0 = blockIdx.x * g.ct + tc * V;
  float mu[V], is[V], sb[V], sg[V];
#pragma unroll
  for (int i = 0; i < V; ++i) { mu[i] = mean[c0 + i]; is[i] = invstd[c0 + i]; sb[i] = sg[i] = 0.f; }
  const int64_t r0 = (int64_t)blockIdx.y * g.rows_per_block;
  int64_t r1 = r0 + g.rows_per_block;
  if (r1 > M) r1 = M;
  for (int64_t r = (lane_r < g.rl ? r0 + lane_r : r1); r < r1; r += g.rl) {
    float d[V], xv[V];
    Vec<T>::load(dy + r * C + c0, d);
    Vec<T>::load(x + r * C + c0, xv);
    const uint32_t bits = RELU ? (uint32_t)mask[r * (C / V) + c0 / V] : 0xffu;
#pragma unroll
    for (int i = 0; i < V; ++i) {
      const float dz = ((bits >> i) & 1u) ? d[i] : 0.f;
      sb[i] += dz;
      sg[i] = fmaf(dz, (xv[i] - mu[i]) * is[i], sg[i]);
    }
  }
  __shared__ float sh[2][kBlock * 8];
#pragma unroll
  for (int i = 0; i < V; ++i) {
    sh[0][threadIdx.x * V + i] = sb[i];
    sh[1][threadIdx.x * V + i] = sg[i];
  }
  __syncthreads();
  for (int cl = threadIdx.x; cl < g.ct; cl += kBlock) {
    const int t = cl / V, i = cl % V;
    float a = 0.f, b = 0.f;
    for (int l = 0; l < g.rl; ++l) {
      a += sh[0][(l * g.tpr + t) * V + i];
      b += sh[1][(l * g.tpr + t) * V + i];
    }
    const int c = blockIdx.x * g.ct + cl;
    pdb[(int64_t)blockIdx.y * C + c] = a;
    pdg[(int64_t)blockIdx.y * C + c] = b;
  }
}

__global__ __launch_bounds__(kBlock) void bn_bwd_finalize_kernel(const float* __restrict__ pdb,
                                                                 const float* __restrict__ pdg, int gy, int C,
                                                                 float* __restrict__ dbeta, float* __restrict__ dgamma,
                                                                 float* __restrict__ gb_acc,
                                                                 float* __restrict__ gw_acc) {
  double a = 0.0, b = 0.0;
  bool owner;
  int c;
  reduce_partials2(pdb, pdg, gy, C, &a, &b, &owner, &c);
  if (!owner) return;
  dbeta[c] = (float)a;
  dgamma[c] = (float)b;
  // direct-to-arena parameter gradients (AccumulateGrad semantics)
  if (gb_acc) gb_acc[c] += (float)a;
  if (gw_acc) gw_acc[c] += (float)b;
}

template <typename T, bool RELU, bool DRES>
__global__ __launch_bounds__(kBlock) void bn_bwd_apply_kernel(const T* __restrict__ dy, const uint8_t* __restrict__ mask,
                                                              const T* __restrict__ x, T* __restrict__ dx,
                                                              T* __restrict__ dres, int64_t M, int C, Geo g,
                                                              const float* __restrict__ w,
                                                              const float* __restrict__ mean,
                                                              const float* __restrict__ invstd,
                                                              const float* __restrict__ dbeta,
                                                              const float* __restrict__ dgamma) {
  constexpr int V = Vec<T>::N;
  const int tc = threadIdx.x % g.tpr;
  const int lane_r = threadIdx.x / g.tpr;
  const int c0 = blockIdx.x * g.ct + tc * V;
  const float invM = 1.f / (float)M;
  float mu[V], is[V], k1[V], k2[V], k3[V];
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int c = c0 + i;
    mu[i] = mean[c];
    is[i] = invstd[c];
    const float gam = w ? w[c] : 1.f;
    k1[i] = gam * is[i];                 // scale
    k2[i] = dbeta[c] * invM;             // mean of dz
    k3[i] = dgamma[c] * invM;            // mean of dz * xhat
  }
  const int64_t r0 = (int64_t)blockIdx.y * g.rows_per_block;
  int64_t r1 = r0 + g.rows_per_block;
  if (r1 > M) r1 = M;
  for (int64_t r = (lane_r < g.rl ? r0 + lane_r : r1); r < r1; r += g.rl) {
    float d[V], xv[V], o[V];
    Vec<T>::load(dy + r * C + c0, d);
    Vec<T>::load(x + r * C + c0, xv);
    const uint32_t bits = RELU ? (uint32_t)mask[r * (C / V) + c0 / V] : 0xffu;
#pragma unroll
    for (int i = 0; i < V; ++i) {
      const float dz = ((bits >> i) & 1u) ? d[i] : 0.f;
      d[i] = dz;
      const float xh = (xv[i] - mu[i]) * is[i];
      o[i] = k1[i] * (dz - k2[i] - xh * k3[i]);
    }
    Vec<T>::store(dx + r * C + c0, o);
    if (DRES) Vec<T>::store(dres + r * C + c0, d);
  }
}

constexpr int kTargetBlocks = 1024;

}  // namespace

size_t bn_workspace_floats(int64_t M, int C, int elem_bytes) {
  const Geo g = elem_bytes == 2 ? make_geo<uint16_t>(M, C, kTargetBlocks) : make_geo<float>(M, C, kTargetBlocks);
  return (size_t)2 * g.gy * C;
}

bool bn_supported(int C, int elem_bytes) {
  const int V = elem_bytes == 2 ? 8 : 4;
  return C % V == 0 && C >= V;
}

template <typename T>
void bn_forward_t(const T* x, const T* res, T* y, uint8_t* mask, int64_t M, int C, const float* w, const float* b, float eps,
                  float momentum, float* run_mean, float* run_var, float* save_mean, float* save_invstd,
                  float* scale, float* shift, float* ws, int relu, hipStream_t s) {
  const Geo g = make_geo<T>(M, C, kTargetBlocks);
  float* psum = ws;
  float* psq = ws + (int64_t)g.gy * C;
  hipLaunchKernelGGL(bn_stats_kernel<T>, dim3(g.gx, g.gy), dim3(kBlock), 0, s, x, M, C, g, psum, psq);
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + kFinC - 1) / kFinC), dim3(kBlock), 0, s, psum, psq, g.gy, M, C,
                     w, b, eps, momentum, run_mean, run_var, save_mean, save_invstd, scale, shift);
  if (relu && res)
    hipLaunchKernelGGL((bn_apply_kernel<T, true, true>), dim3(g.gx, g.gy), dim3(kBlock), 0, s, x, res, y, mask, M, C, g,
                       scale, shift);
  else if (relu)
    hipLaunchKernelGGL((bn_apply_kernel<T, true, false>), dim3(g.gx, g.gy), dim3(kBlock), 0, s, x, res, y, mask, M, C, g,
                       scale, shift);
  else if (res)
    hipLaunchKernelGGL((bn_apply_kernel<T, false, true>), dim3(g.gx, g.gy), dim3(kBlock), 0, s, x, res, y, mask, M, C, g,
                       scale, shift);
  else
    hipLaunchKernelGGL((bn_apply_kernel<T, false, false>), dim3(g.gx, g.gy), dim3(kBlock), 0, s, x, res, y, mask, M, C, g,
                       scale, shift);
}

template <typename T>
void bn_backward_t(const T* dy, const uint8_t* mask, const T* x, T* dx, T* dres, int64_t M, int C, const float* w,
                   const float* mean, const float* invstd, float* dgamma, float* dbeta, float* ws, int relu,
                   float* gw_acc, float* gb_acc, hipStream_t s) {
  const Geo g = make_geo<T>(M, C, kTargetBlocks);
  float* pdb = ws;
  float* pdg = ws + (int64_t)g.gy * C;
  if (relu)
    hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, true>), dim3(g.gx, g.gy), dim3(kBlock), 0, s, dy, mask, x, M, C, g,
                       mean, invstd, pdb, pdg);
  else
    hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, false>), dim3(g.gx, g.gy), dim3(kBlock), 0, s, dy, mask, x, M, C, g,
                       mean, invstd, pdb, pdg);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + kFinC - 1) / kFinC), dim3(kBlock), 0, s, pdb, pdg, g.gy, C,
                     dbeta, dgamma, gb_acc, gw_acc);
#define GK_BWD_APPLY(R, D)                                                                                       \
  hipLaunchKernelGGL((bn_bwd_apply_kernel<T, R, D>), dim3(g.gx, g.gy), dim3(kBlock), 0, s, dy, mask, x, dx, dres, M, \
                     C, g, w, mean, invstd, dbeta, dgamma)
  if (relu && dres) GK_BWD_APPLY(true, true);
  else if (relu) GK_BWD_APPLY(true, false);
  else if (dres) GK_BWD_APPLY(false, true);
  else GK_BWD_APPLY(false, false);
#undef GK_BWD_APPLY
}

size_t bn_mask_bytes(int64_t M, int C, int elem_bytes) { return (size_t)M * (size_t)(C / (elem_bytes == 2 ? 8 : 4)); }

void bn_act_forward(const void* x, const void* res, void* y, uint8_t* mask, int64_t M, int C, int elem_bytes,
                    const float* w, const float* b, float eps, float momentum, float* run_mean, float* run_var,
                    float* save_mean, float* save_invstd, float* scale, float* shift, float* ws, int relu,
                    hipStream_t s) {
  if (elem_bytes == 2)
    bn_forward_t<uint16_t>((const uint16_t*)x, (const uint16_t*)res, (uint16_t*)y, mask, M, C, w, b, eps, momentum,
                           run_mean, run_var, save_mean, save_invstd, scale, shift, ws, relu, s);
  else
    bn_forward_t<float>((const float*)x, (const float*)res, (float*)y, mask, M, C, w, b, eps, momentum, run_mean,
                        run_var, save_mean, save_invstd, scale, shift, ws, relu, s);
}

void bn_act_backward(const void* dy, const uint8_t* mask, const void* x, void* dx, void* dres, int64_t M, int C,
                     int elem_bytes, const float* w, const float* mean, const float* invstd, float* dgamma,
                     float* dbeta, float* ws, int relu, float* gw_acc, float* gb_acc, hipStream_t s) {
  if (elem_bytes == 2)
    bn_backward_t<uint16_t>((const uint16_t*)dy, mask, (const uint16_t*)x, (uint16_t*)dx, (uint16_t*)dres, M, C, w,
                            mean, invstd, dgamma, dbeta, ws, relu, gw_acc, gb_acc, s);
  else
    bn_backward_t<float>((const float*)dy, mask, (const float*)x, (float*)dx, (float*)dres, M, C, w, mean, invstd,
                         dgamma, dbeta, ws, relu, gw_acc, gb_acc, s);
}

}  // namespace gk
