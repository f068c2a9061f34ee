// Fused optimizer kernels over flat parameter / momentum / gradient arenas.
//
//   fused_sgd        K12: torch.optim.SGD semantics (weight decay, momentum,
//                    dampening, nesterov; first step buf = d) for every param
//                    group in ONE launch, plus optional gradient zeroing and a
//                    device-side gradient scale (clip coefficient, K14).
//                    Reference: dl_trainer.py:212-228 (two param groups),
//                    dl_trainer.py:839-873 (_step), torch SGD via
//                    distributed_optimizer.py:546.
//   segmented_sumsq  per-tensor ||w||^2, ||g||^2 (LARS trust ratios)
//   fused_lars       K13: lars.py:67-134 (trust ratio clamp [0,50], grad clamp
//                    +-10, acceleration buffer initialised to ones)
//   clip_grad_norm   K14: global-norm clip with no host sync
//                    (dist_trainer.py:80-85 clip after synchronize()).
//
// The arenas are float4-aligned per tensor (the Python arena pads every tensor
// to 64 elements), so each workgroup streams one <=16K-element chunk with
// 16-byte loads.
#include "common.h"
#include "gk_kernels.h"

namespace gk {
namespace {

__device__ __forceinline__ uint16_t f2bf(float f) {  // round-to-nearest-even, NaN kept quiet
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x7fffffu)) return (uint16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

__device__ __forceinline__ float sgd_elem(float w, float& m, float g, const SgdGroup& p, float gs) {
  float d = g * gs;
  if (p.weight_decay != 0.f) d = fmaf(p.weight_decay, w, d);
  if (p.momentum != 0.f) {
    if (p.first_step) m = d;
    else m = fmaf(p.momentum, m, (1.f - p.dampening) * d);
    d = p.nesterov ? fmaf(p.momentum, m, d) : m;
  }
  return fmaf(-p.lr, d, w);
}

__global__ __launch_bounds__(kBlock) void fused_sgd_kernel(SgdArgs a) {
  const Chunk c = a.chunks[blockIdx.x];
  SgdGroup p = a.groups[c.group];
  if (a.lr_mult) p.lr *= *a.lr_mult;   // lr schedule of a captured graph, read at replay time
  const float gs = a.grad_scale ? *a.grad_scale : 1.f;
  float* w = a.w + c.start;
  float* m = a.m ? a.m + c.start : nullptr;
  float* g = a.g + c.start;
  const bool use_m = p.momentum != 0.f;
  const int n4 = c.len >> 2;
  float4* w4 = reinterpret_cast<float4*>(w);
  float4* g4 = reinterpret_cast<float4*>(g);
  float4* m4 = reinterpret_cast<float4*>(m);
  for (int i = threadIdx.x; i < n4; i += kBlock) {
    float4 wv = w4[i];
    const float4 gv = g4[i];
    float4 mv = make_float4(0.f, 0.f, 0.f, 0.f);
    if (use_m && !p.first_step) mv = m4[i];
    wv.x = sgd_elem(wv.x, mv.x, gv.x, p, gs);
    wv.y = sgd_elem(wv.y, mv.y, gv.y, p, gs);
    wv.z = sgd_elem(wv.z, mv.z, gv.z, p, gs);
    wv.w = sgd_elem(wv.w, mv.w, gv.w, p, gs);
    w4[i] = wv;
    if (use_m) m4[i] = mv;
    if (a.zero_grad) g4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (a.w_bf16) {
      const uint32_t lo = (uint32_t)f2bf(wv.x) | ((uint32_t)f2bf(wv.y) << 16);
      const uint32_t hi = (uint32_t)f2bf(wv.z) | ((uint32_t)f2bf(wv.w) << 16);
      reinterpret_cast<uint2*>(a.w_bf16 + c.start)[i] = make_uint2(lo, hi);
    }
  }
  for (int i = (n4 << 2) + threadIdx.x; i < c.len; i += kBlock) {
    float mv = (use_m && !p.first_step) ? m[i] : 0.f;
    w[i] = sgd_elem(w[i], mv, g[i], p, gs);
    if (use_m) m[i] = mv;
    if (a.zero_grad) g[i] = 0.f;
    if (a.w_bf16) a.w_bf16[c.start + i] = f2bf(w[i]);
  }
}

// DGC momentum correction: u = mu*u + (g + wd*w); g = u (the compressor then
// sparsifies the locally accumulated velocity instead of the raw gradient).
__global__ __launch_bounds__(kBlock) void momentum_correct_kernel(McArgs a) {
  const Chunk c = a.chunks[blockIdx.x];
  const float mu = a.momentum[c.group];
  const float wd = a.weight_decay[c.group];
  float* u = a.u + c.start;
  float* g = a.g + c.start;
  const float* w = a.w + c.start;
  const int n4 = c.len >> 2;
  for (int i = threadIdx.x; i < n4; i += kBlock) {
    float4 uv = reinterpret_cast<float4*>(u)[i];
    const float4 gv = reinterpret_cast<const float4*>(g)[i];
    const float4 wv = reinterpret_cast<const float4*>(w)[i];
    uv.x = fmaf(mu, uv.x, fmaf(wd, wv.x, gv.x));
    uv.y = fmaf(mu, uv.y, fmaf(wd, wv.y, gv.y));
    uv.z = fmaf(mu, uv.z, fmaf(wd, wv.z, gv.z));
    uv.w = fmaf(mu, uv.w, fmaf(wd, wv.w, gv.w));
    reinterpret_cast<float4*>(u)[i] = uv;
    reinterpret_cast<float4*>(g)[i] = uv;
  }
  for (int i = (n4 << 2) + threadIdx.x; i < c.len; i += kBlock) {
    const float uv = fmaf(mu, u[i], fmaf(wd, w[i], g[i]));
    u[i] = uv;
    g[i] = uv;
  }
}

// Momentum factor masking: u[idx] = 0 for every index this rank sent.
__global__ __launch_bounds__(kBlock) void mask_records_kernel(float* __restrict__ u, const int32_t* __restrict__ rec,
                                                              int64_t k_cap) {
  const int64_t sent = rec[0];
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < sent && i < k_cap;
       i += (int64_t)gridDim.x * kBlock)
    u[rec[kRecHdr + i]] = 0.f;
}

__global__ __launch_bounds__(kBlock) void accum_grad_bf16_kernel(float* __restrict__ dst,
                                                                 const uint16_t* __restrict__ src, int64_t n,
                                                                 int vec) {
  const int64_t tid = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  const int64_t n8 = vec ? (n >> 3) : 0;
  for (int64_t i = tid; i < n8; i += stride) {
    const uint4 u = reinterpret_cast<const uint4*>(src)[i];
    float4 a = reinterpret_cast<float4*>(dst)[2 * i];
    float4 b = reinterpret_cast<float4*>(dst)[2 * i + 1];
    a.x += __uint_as_float(u.x << 16); a.y += __uint_as_float(u.x & 0xffff0000u);
    a.z += __uint_as_float(u.y << 16); a.w += __uint_as_float(u.y & 0xffff0000u);
    b.x += __uint_as_float(u.z << 16); b.y += __uint_as_float(u.z & 0xffff0000u);
    b.z += __uint_as_float(u.w << 16); b.w += __uint_as_float(u.w & 0xffff0000u);
    reinterpret_cast<float4*>(dst)[2 * i] = a;
    reinterpret_cast<float4*>(dst)[2 * i + 1] = b;
  }
  for (int64_t i = (n8 << 3) + tid; i < n; i += stride) dst[i] += __uint_as_float(((uint32_t)src[i]) << 16);
}

__global__ __launch_bounds__(kBlock) void accum_grad_f32_kernel(float* __restrict__ dst, const float* __restrict__ src,
                                                                int64_t n) {
  const int64_t tid = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = tid; i < n; i += stride) dst[i] += src[i];
}

__global__ __launch_bounds__(kBlock) void cast_bf16_kernel(uint16_t* __restrict__ dst, const float* __restrict__ src,
                                                           int64_t n) {
  const int64_t tid = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = tid; i < n; i += stride) dst[i] = f2bf(src[i]);
}

__global__ __launch_bounds__(kBlock) void segmented_sumsq_kernel(const float* __restrict__ w,
                                                                 const float* __restrict__ g,
                                                                 const Chunk* __restrict__ chunks,
                                                                 double* __restrict__ out) {
  const Chunk c = chunks[blockIdx.x];
  const float* wp = w + c.start;
  const float* gp = g + c.start;
  float sw = 0.f, sg = 0.f;
  const int n4 = c.len >> 2;
  for (int i = threadIdx.x; i < n4; i += kBlock) {
    const float4 a = reinterpret_cast<const float4*>(wp)[i];
    const float4 b = reinterpret_cast<const float4*>(gp)[i];
    sw += (a.x * a.x + a.y * a.y) + (a.z * a.z + a.w * a.w);
    sg += (b.x * b.x + b.y * b.y) + (b.z * b.z + b.w * b.w);
  }
  for (int i = (n4 << 2) + threadIdx.x; i < c.len; i += kBlock) {
    sw += wp[i] * wp[i];
    sg += gp[i] * gp[i];
  }
  __shared__ double sh[kWavesPerBlock];
  const double bw = block_sum((double)sw, sh);
  const double bg = block_sum((double)sg, sh);
  if (threadIdx.x == 0) {
    atomicAdd(out + 2 * c.seg, bw);
    atomicAdd(out + 2 * c.seg + 1, bg);
  }
}

__device__ __forceinline__ float lars_elem(float w, float& acc, float g, float wd, float mom, float slr) {
  float d = fmaf(wd, w, g);
  d = fminf(fmaxf(d, -10.f), 10.f);
  acc = fmaf(mom, acc, slr * d);
  return w - acc;
}

__global__ __launch_bounds__(kBlock) void fused_lars_kernel(LarsArgs a) {
  const Chunk c = a.chunks[blockIdx.x];
  const int gi = c.group;
  const float lr = a.lr[gi], mom = a.momentum[gi], wd = a.weight_decay[gi], eeta = a.eeta[gi], eps = a.epsilon[gi];
  const float wn = (float)sqrt(a.seg_sumsq[2 * c.seg]);
  const float gn = (float)sqrt(a.seg_sumsq[2 * c.seg + 1]);
  float trust = 1.f;
  if (wn > 0.f && gn > 0.f) trust = eeta * wn / (gn + wd * wn + eps);
  trust = fminf(fmaxf(trust, 0.f), 50.f);
  const float slr = lr * trust;
  float* w = a.w + c.start;
  float* m = a.m + c.start;
  const float* g = a.g + c.start;
  const int n4 = c.len >> 2;
  for (int i = threadIdx.x; i < n4; i += kBlock) {
    float4 wv = reinterpret_cast<float4*>(w)[i];
    float4 mv = reinterpret_cast<float4*>(m)[i];
    const float4 gv = reinterpret_cast<const float4*>(g)[i];
    wv.x = lars_elem(wv.x, mv.x, gv.x, wd, mom, slr);
    wv.y = lars_elem(wv.y, mv.y, gv.y, wd, mom, slr);
    wv.z = lars_elem(wv.z, mv.z, gv.z, wd, mom, slr);
    wv.w = lars_elem(wv.w, mv.w, gv.w, wd, mom, slr);
    reinterpret_cast<float4*>(w)[i] = wv;
    reinterpret_cast<float4*>(m)[i] = mv;
  }
  for (int i = (n4 << 2) + threadIdx.x; i < c.len; i += kBlock) {
    float mv = m[i];
    w[i] = lars_elem(w[i], mv, g[i], wd, mom, slr);
    m[i] = mv;
  }
}

// ---- global-norm clip -------------------------------------------------------
__global__ __launch_bounds__(kBlock) void sumsq_kernel(const float* __restrict__ x, int64_t n, double* __restrict__ part) {
  float s = 0.f;
  const int64_t tid = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  if ((reinterpret_cast<uintptr_t>(x) & 15) == 0) {
    const int64_t n4 = n >> 2;
    for (int64_t i = tid; i < n4; i += stride) {
      const float4 v = reinterpret_cast<const float4*>(x)[i];
      s += (v.x * v.x + v.y * v.y) + (v.z * v.z + v.w * v.w);
    }
    for (int64_t i = (n4 << 2) + tid; i < n; i += stride) s += x[i] * x[i];
  } else {
    for (int64_t i = tid; i < n; i += stride) s += x[i] * x[i];
  }
  __shared__ double sh[kWavesPerBlock];
  const double b = block_sum((double)s, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = b;
}

__global__ __launch_bounds__(kBlock) void clip_coef_kernel(const double* __restrict__ part, int nparts, float max_norm,
                                                           float* __restrict__ coef, float* __restrict__ norm_out) {
  double s = 0.0;
  for (int b = threadIdx.x; b < nparts; b += kBlock) s += part[b];
  __shared__ double sh[kWavesPerBlock];
  s = block_sum(s, sh);
  if (threadIdx.x == 0) {
    const float nrm = (float)sqrt(s);
    float c = max_norm / (nrm + 1e-6f);
    if (c > 1.f) c = 1.f;
    *coef = c;
    if (norm_out) *norm_out = nrm;
  }
}

__global__ __launch_bounds__(kBlock) void scale_kernel(float* __restrict__ x, int64_t n, const float* __restrict__ coef) {
  const float c = *coef;
  if (c == 1.f) return;
  const int64_t tid = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = tid; i < n; i += stride) x[i] *= c;
}

}  // namespace

void fused_sgd(const SgdArgs& a, hipStream_t s) {
  if (a.nchunks <= 0) return;
  hipLaunchKernelGGL(fused_sgd_kernel, dim3(a.nchunks), dim3(kBlock), 0, s, a);
}

void momentum_correct(const McArgs& a, hipStream_t s) {
  if (a.nchunks <= 0) return;
  hipLaunchKernelGGL(momentum_correct_kernel, dim3(a.nchunks), dim3(kBlock), 0, s, a);
}

void mask_records(float* u, const int32_t* record, int64_t k_cap, hipStream_t s) {
  int64_t G = ceil_div(k_cap, (int64_t)kBlock);
  if (G < 1) G = 1;
  if (G > 1024) G = 1024;
  hipLaunchKernelGGL(mask_records_kernel, dim3((int)G), dim3(kBlock), 0, s, u, record, k_cap);
}

void accum_grad(float* dst, const void* src, int64_t n, int src_bytes, hipStream_t s) {
  if (n <= 0) return;
  int64_t G = ceil_div(n, (int64_t)kBlock * 8);
  if (G < 1) G = 1;
  if (G > 2048) G = 2048;
  const bool vec = ((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) & 15) == 0;
  if (src_bytes == 2)  // unaligned pointers: the scalar tail loop covers every element
    hipLaunchKernelGGL(accum_grad_bf16_kernel, dim3((int)G), dim3(kBlock), 0, s, dst, (const uint16_t*)src, n,
                       vec ? 1 : 0);
  else
    hipLaunchKernelGGL(accum_grad_f32_kernel, dim3((int)G), dim3(kBlock), 0, s, dst, (const float*)src, n);
}

void cast_bf16(uint16_t* dst, const float* src, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  int64_t G = ceil_div(n, (int64_t)kBlock * 8);
  if (G < 1) G = 1;
  if (G > 2048) G = 2048;
  hipLaunchKernelGGL(cast_bf16_kernel, dim3((int)G), dim3(kBlock), 0, s, dst, src, n);
}

void segmented_sumsq(const float* w, const float* g, const Chunk* chunks, int nchunks, double* out, hipStream_t s) {
  if (nchunks <= 0) return;
  hipLaunchKernelGGL(segmented_sumsq_kernel, dim3(nchunks), dim3(kBlock), 0, s, w, g, chunks, out);
}

void fused_lars(const LarsArgs& a, hipStream_t s) {
  if (a.nchunks <= 0) return;
  hipLaunchKernelGGL(fused_lars_kernel, dim3(a.nchunks), dim3(kBlock), 0, s, a);
}

void clip_grad_norm(float* g, int64_t n, float max_norm, double* ws, float* coef_out, float* norm_out,
                    hipStream_t s) {
  int G = (int)ceil_div(n, (int64_t)kBlock * 16);
  if (G < 1) G = 1;
  if (G > 1024) G = 1024;
  hipLaunchKernelGGL(sumsq_kernel, dim3(G), dim3(kBlock), 0, s, g, n, ws);
  hipLaunchKernelGGL(clip_coef_kernel, dim3(1), dim3(kBlock), 0, s, ws, G, max_norm, coef_out, norm_out);
  int Gs = (int)ceil_div(n, (int64_t)kBlock * 8);
  if (Gs < 1) Gs = 1;
  if (Gs > 2048) Gs = 2048;
  hipLaunchKernelGGL(scale_kernel, dim3(Gs), dim3(kBlock), 0, s, g, n, coef_out);
}

}  // namespace gk
