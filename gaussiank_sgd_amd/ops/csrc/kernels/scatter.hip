// Sparse aggregation (K11) and the sign-bucket-mean compressor (K9).
//
// Reference aggregation (distributed_optimizer.py:468-482) loops over ranks in
// Python, index_puts half-chunks (wrong for unequal counts), then
// divides the sum by P.  Here the P packed records {sent, total, chosen, thr |
// idx[k_cap] | val[k_cap]} are reduced in ONE launch:
//
//   reduce_records (default): every index is owned by the first rank whose
//     record holds it; the owner sums the P contributions IN RANK ORDER
//     (fp32, like the reference loop) and applies the 1/P average once to the
//     sum.  No atomics, so every replica computes bit-identical gradients for
//     any P and any duplicate pattern.  Records are sorted (the compressor
//     emits ascending indices): a workgroup takes 1024 consecutive entries of
//     one rank, finds the matching index window of every other rank with two
//     binary searches, stages those windows in LDS and resolves each entry
//     with LDS binary searches.
//   APPLY variant (DGC momentum correction, where the global update is plain
//     SGD on the aggregate): w[idx] -= lr * avg and the bf16 shadow weight is
//     refreshed at idx -- the dense gradient pass of the optimizer disappears.
//   scatter_atomic: hardware fp32 atomics (global_atomic_add_f32), for the
//     explicit non-deterministic request only.
#include "common.h"
#include "gk_kernels.h"

namespace gk {
namespace {

constexpr int kRedPer = 4;                       // entries per thread
constexpr int kRedTile = kBlock * kRedPer;       // entries of the owner rank per workgroup
constexpr int kRedWin = 1024;                    // LDS window per other rank (int32 indices)
constexpr int kRedMaxP = 16;                     // ranks staged in LDS; more go through global memory

__device__ __forceinline__ int lower_bound_i32(const int32_t* a, int lo, int hi, int32_t key) {
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a[mid] < key) lo = mid + 1; else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ uint16_t f2bf_rne(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x7fffffu)) return (uint16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

template <bool APPLY>
__global__ __launch_bounds__(kBlock) void reduce_records_kernel(float* __restrict__ dst, int64_t n,
                                                                const int32_t* __restrict__ records, int P,
                                                                int64_t k_cap, int64_t rec_words, float scale,
                                                                const float* __restrict__ lr_ptr, float lr,
                                                                uint16_t* __restrict__ shadow) {
  // two roundings (product, then sum) exactly as the reference / CPU mirror:
  // this file is compiled with -ffp-contract=off (ops/build.py), hipcc's
  // default would fuse them into one FMA
  __shared__ int32_t win[kRedMaxP][kRedWin];
  __shared__ int s_lo[kRedMaxP], s_len[kRedMaxP];
  const int r = blockIdx.y;
  const int32_t* rec = records + (int64_t)r * rec_words;
  int64_t cnt = rec[0];
  if (cnt > k_cap) cnt = k_cap;
  const int64_t t0 = (int64_t)blockIdx.x * kRedTile;
  if (t0 >= cnt) return;                                       // block-uniform
  const int64_t t1 = t0 + kRedTile < cnt ? t0 + kRedTile : cnt;
  const int32_t* idx = rec + kRecHdr;
  const float* val = reinterpret_cast<const float*>(rec + kRecHdr + k_cap);
  const int32_t key_lo = idx[t0], key_hi = idx[t1 - 1];
  // window [lo, lo+len) of every other rank holding keys in [key_lo, key_hi]
  if (threadIdx.x < P && threadIdx.x < kRedMaxP) {
    const int q = threadIdx.x;
    const int32_t* rq = records + (int64_t)q * rec_words;
    int cq = rq[0];
    if (cq > k_cap) cq = (int)k_cap;
    const int lo = lower_bound_i32(rq + kRecHdr, 0, cq, key_lo);
    const int hi = lower_bound_i32(rq + kRecHdr, lo, cq, key_hi + 1);
    s_lo[q] = lo;
    s_len[q] = hi - lo;
  }
  __syncthreads();
  const int Ps = P < kRedMaxP ? P : kRedMaxP;
  for (int q = 0; q < Ps; ++q) {
    if (q == r || s_len[q] > kRedWin) continue;
    const int32_t* src = records + (int64_t)q * rec_words + kRecHdr + s_lo[q];
    for (int i = threadIdx.x; i < s_len[q]; i += kBlock) win[q][i] = src[i];
  }
  __syncthreads();
  const float lr_eff = APPLY ? (lr_ptr ? lr * *lr_ptr : lr) : 0.f;
#pragma unroll
  for (int e = 0; e < kRedPer; ++e) {
    const int64_t j = t0 + (int64_t)e * kBlock + threadIdx.x;
    if (j >= t1) continue;
    const int32_t key = idx[j];
    bool owner = true;
    float s = 0.f;
    for (int q = 0; q < P && owner; ++q) {
      float v = 0.f;
      if (q == r) {
        v = val[j];
      } else {
        const int32_t* rq = records + (int64_t)q * rec_words;
        int pos, len, lo;
        bool hit;
        if (q < kRedMaxP) {
          lo = s_lo[q];
          len = s_len[q];
          if (len <= kRedWin) {
            pos = lower_bound_i32(win[q], 0, len, key);
            hit = pos < len && win[q][pos] == key;
          } else {
            pos = lower_bound_i32(rq + kRecHdr + lo, 0, len, key);
            hit = pos < len && rq[kRecHdr + lo + pos] == key;
          }
        } else {
          int cq = rq[0];
          if (cq > k_cap) cq = (int)k_cap;
          lo = 0;
          len = cq;
          pos = lower_bound_i32(rq + kRecHdr, 0, len, key);
          hit = pos < len && rq[kRecHdr + pos] == key;
        }
        if (hit) {
          if (q < r) owner = false;                      // an earlier rank owns this index
          else v = reinterpret_cast<const float*>(rq + kRecHdr + k_cap)[lo + pos];
        }
      }
      s = s + v;                                         // rank order: ((0 + v0) + v1) + ...
    }
    if (!owner || key < 0 || key >= n) continue;
    const float avg = s * scale;
    if (APPLY) {
      const float wn = dst[key] - lr_eff * avg;
      dst[key] = wn;
      if (shadow) shadow[key] = f2bf_rne(wn);
    } else {
      dst[key] = dst[key] + avg;
    }
  }
}

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

// ---- replica digest ----------------------------------------------------------
// fp64 sum (fixed reduction tree -> reproducible) and a wrapping 64-bit sum of
// a position-keyed mix of every element's bits (order-independent, so exact).
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

__global__ __launch_bounds__(kBlock) void digest_partial_kernel(const float* __restrict__ x, int64_t n,
                                                                uint64_t* __restrict__ part) {
  double s = 0.0;
  uint64_t h = 0;
  const int64_t tid = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = tid; i < n; i += stride) {
    const float v = x[i];
    s += (double)v;
    h += mix64(((uint64_t)__float_as_uint(v) << 32) ^ (uint64_t)i * 0x9e3779b97f4a7c15ull);
  }
  __shared__ double sh[kWavesPerBlock];
  __shared__ uint64_t shh[kWavesPerBlock];
  s = block_sum(s, sh);
  h = wave_sum(h);
  if (lane_id() == 0) shh[wave_id()] = h;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t t = 0;
    for (int w = 0; w < kWavesPerBlock; ++w) t += shh[w];
    part[2 * blockIdx.x] = (uint64_t)__double_as_longlong(s);
    part[2 * blockIdx.x + 1] = t;
  }
}

__global__ __launch_bounds__(kBlock) void digest_final_kernel(const uint64_t* __restrict__ part, int G,
                                                              uint64_t* __restrict__ out) {
  if (threadIdx.x != 0) return;
  double s = 0.0;
  uint64_t h = 0;
  for (int b = 0; b < G; ++b) {
    s += __longlong_as_double((long long)part[2 * b]);
    h += part[2 * b + 1];
  }
  out[0] = (uint64_t)__double_as_longlong(s);
  out[1] = h;
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
  if (P == 1) {  // one record: indices are unique, a plain scatter is already deterministic
    int gx = (int)ceil_div(k_cap, (int64_t)kBlock);
    if (gx < 1) gx = 1;
    if (gx > 1024) gx = 1024;
    hipLaunchKernelGGL(scatter_rank_kernel, dim3(gx), dim3(kBlock), 0, s, dst, n, records, k_cap, scale);
  } else if (deterministic) {
    const int gx = (int)ceil_div(k_cap, (int64_t)kRedTile);
    hipLaunchKernelGGL((reduce_records_kernel<false>), dim3(gx < 1 ? 1 : gx, P), dim3(kBlock), 0, s, dst, n, records,
                       P, k_cap, rec_words, scale, (const float*)nullptr, 0.f, (uint16_t*)nullptr);
  } else {
    int gx = (int)ceil_div(k_cap, (int64_t)kBlock);
    if (gx < 1) gx = 1;
    if (gx > 1024) gx = 1024;
    hipLaunchKernelGGL(scatter_atomic_kernel, dim3(gx, P), dim3(kBlock), 0, s, dst, n, records, k_cap, rec_words,
                       scale);
  }
}

void apply_records_sgd(float* w, uint16_t* w_bf16, int64_t n, const int32_t* records, int P, int64_t k_cap,
                       float scale, float lr, const float* lr_mult, hipStream_t s) {
  const int64_t rec_words = 4 + 2 * k_cap;
  const int gx = (int)ceil_div(k_cap, (int64_t)kRedTile);
  hipLaunchKernelGGL((reduce_records_kernel<true>), dim3(gx < 1 ? 1 : gx, P), dim3(kBlock), 0, s, w, n, records, P,
                     k_cap, rec_words, scale, lr_mult, lr, w_bf16);
}

void arena_digest(const float* x, int64_t n, uint64_t* out, uint64_t* ws, hipStream_t s) {
  const int G = grid_for(n, 1024);
  hipLaunchKernelGGL(digest_partial_kernel, dim3(G), dim3(kBlock), 0, s, x, n, ws);
  hipLaunchKernelGGL(digest_final_kernel, dim3(1), dim3(64), 0, s, ws, G, out);
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
