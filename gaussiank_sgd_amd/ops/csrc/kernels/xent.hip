// Fused softmax cross-entropy over bf16 logits rows (the BERT MLM loss:
// 2560 masked rows x 30522 vocabulary per bs32 x 512 step).
//
// PyTorch's path casts the bf16 logits to fp32 (a 312 MB write), runs
// log_softmax forward / backward over the fp32 copy, the nll gather /
// scatter, and casts the gradient back: ~0.6 ms of a 20 ms BERT step
// (profiles/r02_bert_kernel_stats_latest.csv).  Here one workgroup per row:
//   forward : max pass + sum-of-exp pass over the bf16 row (fp32 math), the
//             row's log-sum-exp saved, loss_r = lse - x[label] (0 for an
//             ignored row);
//   backward: dlogits = (exp(x - lse) - [v == label]) * scale, written in bf16
//             (scale = upstream gradient / number of counted rows).
#include <hip/hip_runtime.h>

#include "common.h"
#include "gk_kernels.h"

namespace gk {
namespace {

__device__ __forceinline__ float bf(uint16_t h) { return __uint_as_float(((uint32_t)h) << 16); }

__device__ __forceinline__ float block_reduce_max(float v, float* sh) {
  v = wave_max(v);
  __syncthreads();
  if (lane_id() == 0) sh[wave_id()] = v;
  __syncthreads();
  float r = sh[0];
#pragma unroll
  for (int w = 1; w < kWavesPerBlock; ++w) r = fmaxf(r, sh[w]);
  return r;
}

__device__ __forceinline__ float block_reduce_sum(float v, float* sh) {
  v = wave_sum(v);
  __syncthreads();
  if (lane_id() == 0) sh[wave_id()] = v;
  __syncthreads();
  float r = 0.f;
#pragma unroll
  for (int w = 0; w < kWavesPerBlock; ++w) r += sh[w];
  return r;
}

// rows of V bf16, V even (BERT: 30522 -- rows are only 4-byte aligned): each
// thread walks bf16 pairs
__global__ __launch_bounds__(kBlock) void xent_fwd_kernel(const uint16_t* __restrict__ logits,
                                                          const int64_t* __restrict__ labels, float* __restrict__ lse,
                                                          float* __restrict__ loss, int V, int64_t ignore) {
  __shared__ float sh[kWavesPerBlock];
  const int64_t r = blockIdx.x;
  const uint32_t* row = reinterpret_cast<const uint32_t*>(logits + r * V);
  const int nv = V / 2;
  float m = -INFINITY;
  for (int i = threadIdx.x; i < nv; i += kBlock) {
    const uint32_t w = row[i];
    m = fmaxf(m, fmaxf(__uint_as_float(w << 16), __uint_as_float(w & 0xffff0000u)));
  }
  m = block_reduce_max(m, sh);
  float s = 0.f;
  for (int i = threadIdx.x; i < nv; i += kBlock) {
    const uint32_t w = row[i];
    s += __expf(__uint_as_float(w << 16) - m) + __expf(__uint_as_float(w & 0xffff0000u) - m);
  }
  s = block_reduce_sum(s, sh);
  if (threadIdx.x == 0) {
    const float l = m + __logf(s);
    lse[r] = l;
    const int64_t y = labels[r];
    loss[r] = (y == ignore || y < 0 || y >= V) ? 0.f : l - bf(logits[r * V + y]);
  }
}

__global__ __launch_bounds__(kBlock) void xent_bwd_kernel(const uint16_t* __restrict__ logits,
                                                          const int64_t* __restrict__ labels,
                                                          const float* __restrict__ lse, const float* __restrict__ scale,
                                                          uint16_t* __restrict__ grad, int V, int64_t ignore) {
  const int64_t r = blockIdx.x;
  const int64_t y = labels[r];
  const bool skip = y == ignore || y < 0 || y >= V;
  const float l = lse[r];
  const float sc = *scale;
  const uint32_t* row = reinterpret_cast<const uint32_t*>(logits + r * V);
  uint32_t* out = reinterpret_cast<uint32_t*>(grad + r * V);
  const int nv = V / 2;
  for (int i = threadIdx.x; i < nv; i += kBlock) {
    uint32_t o = 0u;
    if (!skip) {
      const uint32_t w = row[i];
      const int v0 = 2 * i;
      const float g0 = __expf(__uint_as_float(w << 16) - l) - (v0 == y ? 1.f : 0.f);
      const float g1 = __expf(__uint_as_float(w & 0xffff0000u) - l) - (v0 + 1 == y ? 1.f : 0.f);
      o = __builtin_bit_cast(uint32_t, __builtin_convertvector(
              (float __attribute__((ext_vector_type(2)))){g0 * sc, g1 * sc}, __bf16 __attribute__((ext_vector_type(2)))));
    }
    out[i] = o;
  }
}

}  // namespace

bool xent_supported(int V) { return V % 2 == 0 && V >= 2; }

void xent_forward(const void* logits, const int64_t* labels, float* lse, float* loss, int64_t R, int V, int64_t ignore,
                  hipStream_t s) {
  hipLaunchKernelGGL(xent_fwd_kernel, dim3((unsigned)R), dim3(kBlock), 0, s, (const uint16_t*)logits, labels, lse, loss,
                     V, ignore);
}

void xent_backward(const void* logits, const int64_t* labels, const float* lse, const float* scale, void* grad,
                   int64_t R, int V, int64_t ignore, hipStream_t s) {
  hipLaunchKernelGGL(xent_bwd_kernel, dim3((unsigned)R), dim3(kBlock), 0, s, (const uint16_t*)logits, labels, lse,
                     scale, (uint16_t*)grad, V, ignore);
}

}  // namespace gk
