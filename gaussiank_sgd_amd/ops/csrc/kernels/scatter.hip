// Sparse aggregation (K11) and the sign-bucket-mean compressor (K9).
//
// Reference aggregation (distributed_optimizer.py:468-482) loops over ranks in
// Python and index_puts half-chunks, which is wrong for unequal counts (SURVEY
// 2.3).  Here every rank's packed record {sent, total, chosen, thr | idx[k_cap]
// | val[k_cap]} is scattered in ONE launch with hardware fp32 atomics
// (global_atomic_add_f32), the 1/P average folded in; the deterministic mode
// applies the ranks in order with plain read-modify-writes (indices inside one
// record are unique, so one launch per rank is race-free and reproducible).
#include "common.h"
#include "gk_kernels.h"

namespace gk {
namespace {

__global__ __launch_bounds__(kBlock) void scatter_atomic_kernel(float* __restrict__ dst, int64_t n,
                                                                const int32_t* __restrict__ records, int64_t k_cap,
                                                                int64_t rec_words, float scale) {
  const int r = blockIdx.y;
  const int32_t* rec = records + (int64_t)r * rec_words;
  const int64_t cnt = rec[0];
  const int32_t* idx = rec + 4;
  const float* val = reinterpret_cast<const float*>(rec + 4 + k_cap);
  for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < cnt; j += (int64_t)gridDim.x * kBlock) {
    const int64_t i = idx[j];
    if (i >= 0 && i < n) atomicAdd(dst + i, val[j] * scale);
  }
}

__global__ __launch_bounds__(kBlock) void scatter_rank_kernel(float* __restrict__ dst, int64_t n,
                                                              const int32_t* __restrict__ rec, int64_t k_cap,
                                                              float scale) {
  const int64_t cnt = rec[0];
  const int32_t* idx = rec + 4;
  const float* val = reinterpret_cast<const float*>(rec + 4 + k_cap);
  for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < cnt; j += (int64_t)gridDim.x * kBlock) {
    const int64_t i = idx[j];
    if (i >= 0 && i < n) dst[i] += val[j] * scale;
  }
}

__global__ __launch_bounds__(kBlock) void fill_zero_kernel(float* __restrict__ dst, int64_t n) {
  const int64_t tid = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
    const int64_t n4 = n >> 2;
    float4* d4 = reinterpret_cast<float4*>(dst);
    for (int64_t i = tid; i < n4; i += stride) d4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int64_t i = (n4 << 2) + tid; i < n; i += stride) dst[i] = 0.f;
  } else {
    for (int64_t i = tid; i < n; i += stride) dst[i] = 0.f;
  }
}

// ---- sign-bucket mean -------------------------------------------------------
__global__ __launch_bounds__(kBlock) void sign_stats_kernel(const float* __restrict__ x, int64_t n,
                                                            double* __restrict__ partials) {
  double sp = 0.0, sn = 0.0;
  double cp = 0.0, cn = 0.0;
  const int64_t tid = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  float fsp = 0.f, fsn = 0.f;
  uint32_t icp = 0, icn = 0;
  for (int64_t i = tid; i < n; i += stride) {
    const float v = x[i];
    if (v >= 0.f) { fsp += v; ++icp; } else { fsn += v; ++icn; }
  }
  sp = fsp; sn = fsn; cp = icp; cn = icn;
  __shared__ double sh[kWavesPerBlock];
  sp = block_sum(sp, sh);
  sn = block_sum(sn, sh);
  cp = block_sum(cp, sh);
  cn = block_sum(cn, sh);
  if (threadIdx.x == 0) {
    partials[blockIdx.x * 4 + 0] = sp;
    partials[blockIdx.x * 4 + 1] = cp;
    partials[blockIdx.x * 4 + 2] = sn;
    partials[blockIdx.x * 4 + 3] = cn;
  }
}

__global__ __launch_bounds__(kBlock) void sign_finalize_kernel(const double* __restrict__ partials, int nparts,
                                                               float* __restrict__ means) {
  double sp = 0, cp = 0, sn = 0, cn = 0;
  for (int b = threadIdx.x; b < nparts; b += kBlock) {
    sp += partials[b * 4 + 0]; cp += partials[b * 4 + 1];
    sn += partials[b * 4 + 2]; cn += partials[b * 4 + 3];
  }
  __shared__ double sh[kWavesPerBlock];
  sp = block_sum(sp, sh); cp = block_sum(cp, sh);
  sn = block_sum(sn, sh); cn = block_sum(cn, sh);
  if (threadIdx.x == 0) {
    means[0] = cp > 0 ? (float)(sp / cp) : 0.f;
    means[1] = cn > 0 ? (float)(sn / cn) : 0.f;
  }
}

__global__ __launch_bounds__(kBlock) void sign_apply_kernel(float* __restrict__ x, int64_t n,
                                                            uint8_t* __restrict__ mask, const float* __restrict__ means,
                                                            int decompress) {
  const float mp = means[0], mn = means[1];
  const int64_t tid = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = tid; i < n; i += stride) {
    if (decompress) {
      x[i] += mask[i] ? mp : mn;
    } else {
      const float v = x[i];
      const bool pos = v >= 0.f;
      mask[i] = pos ? 1 : 0;
      x[i] = v + (pos ? -mp : -mn);
    }
  }
}

int grid_for(int64_t n, int cap) {
  int64_t g = ceil_div(n, (int64_t)kBlock * 8);
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

}  // namespace

void scatter_add_records(float* dst, int64_t n, const int32_t* records, int P, int64_t k_cap, float scale,
                         int deterministic, hipStream_t s) {
  const int64_t rec_words = 4 + 2 * k_cap;
  int gx = (int)ceil_div(k_cap, (int64_t)kBlock);
  if (gx < 1) gx = 1;
  if (gx > 1024) gx = 1024;
  if (deterministic) {
    for (int r = 0; r < P; ++r)
      hipLaunchKernelGGL(scatter_rank_kernel, dim3(gx), dim3(kBlock), 0, s, dst, n, records + (int64_t)r * rec_words,
                         k_cap, scale);
  } else {
    hipLaunchKernelGGL(scatter_atomic_kernel, dim3(gx, P), dim3(kBlock), 0, s, dst, n, records, k_cap, rec_words,
                       scale);
  }
}

void fill_zero(float* dst, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(fill_zero_kernel, dim3(grid_for(n / 4 + 1, 2048)), dim3(kBlock), 0, s, dst, n);
}

size_t sign_bucket_workspace_bytes(int64_t) { return sizeof(double) * 4 * 1024; }

void sign_bucket_compress(float* x, int64_t n, uint8_t* mask, float* means, void* ws, hipStream_t s) {
  double* partials = reinterpret_cast<double*>(ws);
  const int G = grid_for(n, 1024);
  hipLaunchKernelGGL(sign_stats_kernel, dim3(G), dim3(kBlock), 0, s, x, n, partials);
  hipLaunchKernelGGL(sign_finalize_kernel, dim3(1), dim3(kBlock), 0, s, partials, G, means);
  hipLaunchKernelGGL(sign_apply_kernel, dim3(grid_for(n, 2048)), dim3(kBlock), 0, s, x, n, mask, means, 0);
}

void sign_bucket_decompress(float* x, int64_t n, const uint8_t* mask, const float* means, hipStream_t s) {
  hipLaunchKernelGGL(sign_apply_kernel, dim3(grid_for(n, 2048)), dim3(kBlock), 0, s, x, n,
                     const_cast<uint8_t*>(mask), means, 1);
}

}  // namespace gk
