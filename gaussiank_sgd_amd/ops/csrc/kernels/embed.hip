// Fused BERT input embedding: x[m] = word[ids[m]] + pos[m % T] + type[tt[m]]
// (fp32 tables and output, rows of H = 4k floats) and its backward.
//
// PyTorch runs this as three gathers + two adds forward and, backward, three
// sort-based embedding_dense_backward passes (rocprim radix sort, segment
// offsets, sum_and_scatter: ~0.8 ms of a 21 ms BERT-base bs32 x 512 step,
// profiles/r02_bert_*).  Here:
//   forward : one pass, one float4 per thread of each output row;
//   backward: word rows scatter-added into a zeroed [V, H] gradient with fp32
//             atomics (the ids of one step are spread over the vocabulary;
//             the order of the adds into one row is not fixed -- the
//             deterministic mode keeps PyTorch's sort-based path),
//             position rows summed over the batch (one thread per (t, h4)
//             walks the B rows: deterministic, written not accumulated),
//             type rows summed per block in fixed order into [blocks][NT][H]
//             partials and finalized in block order (deterministic).
// Reference model: the BERT MLM config of SURVEY.md (configs/bert.conf);
// the reference repo has no BERT code of its own (parity unpinned).
#include <hip/hip_runtime.h>

#include "common.h"
#include "gk_kernels.h"

namespace gk {
namespace {

constexpr int kEmbTypes = 2;   // token types (BERT: segment A / B)

__global__ __launch_bounds__(kBlock) void emb_fwd_kernel(const int64_t* __restrict__ ids,
                                                         const int64_t* __restrict__ tt, const float* __restrict__ Ww,
                                                         const float* __restrict__ Wp, const float* __restrict__ Wt,
                                                         float* __restrict__ out, int64_t M, int T, int H4) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= M * H4) return;
  const int64_t m = i / H4;
  const int h = (int)(i - m * H4);
  const int64_t w = ids[m];
  const int t = (int)(m % T);
  const int64_t ty = tt ? tt[m] : 0;
  const float4 a = reinterpret_cast<const float4*>(Ww + w * (int64_t)H4 * 4)[h];
  const float4 b = reinterpret_cast<const float4*>(Wp + (int64_t)t * H4 * 4)[h];
  const float4 c = reinterpret_cast<const float4*>(Wt + ty * (int64_t)H4 * 4)[h];
  // (word + pos) + type: the order of the reference composition
  reinterpret_cast<float4*>(out)[i] = make_float4(a.x + b.x + c.x, a.y + b.y + c.y, a.z + b.z + c.z, a.w + b.w + c.w);
}

__global__ __launch_bounds__(kBlock) void emb_word_bwd_kernel(const int64_t* __restrict__ ids,
                                                              const float* __restrict__ dx, float* __restrict__ dWw,
                                                              int64_t M, int H4) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= M * H4) return;
  const int64_t m = i / H4;
  const int h = (int)(i - m * H4);
  const float4 g = reinterpret_cast<const float4*>(dx)[i];
  float* dst = dWw + ids[m] * (int64_t)H4 * 4 + h * 4;
  atomicAdd(dst + 0, g.x);
  atomicAdd(dst + 1, g.y);
  atomicAdd(dst + 2, g.z);
  atomicAdd(dst + 3, g.w);
}

// dWp[t] = sum_b dx[b * T + t] for t < T; rows T..P-1 are zero
__global__ __launch_bounds__(kBlock) void emb_pos_bwd_kernel(const float* __restrict__ dx, float* __restrict__ dWp,
                                                             int B, int T, int P, int H4) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= (int64_t)P * H4) return;
  const int t = (int)(i / H4);
  const int h = (int)(i - (int64_t)t * H4);
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (t < T) {
    for (int b = 0; b < B; ++b) {
      const float4 g = reinterpret_cast<const float4*>(dx)[((int64_t)b * T + t) * H4 + h];
      s.x += g.x; s.y += g.y; s.z += g.z; s.w += g.w;
    }
  }
  reinterpret_cast<float4*>(dWp)[i] = s;
}

// type partials: block (bx, by) sums rows by*rows_per .. of column group bx
// per token type into part[by][type][H]
__global__ __launch_bounds__(kBlock) void emb_type_partial_kernel(const int64_t* __restrict__ tt,
                                                                  const float* __restrict__ dx,
                                                                  float* __restrict__ part, int64_t M, int H4,
                                                                  int64_t rows_per) {
  // threads: kBlock / 64 row lanes x 64 column float4 groups (H4 <= 64 * gridDim.x)
  const int hc = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rl = threadIdx.x >> 6;   // 0..3
  const int64_t r0 = (int64_t)blockIdx.y * rows_per;
  int64_t r1 = r0 + rows_per;
  if (r1 > M) r1 = M;
  float4 s[kEmbTypes];
#pragma unroll
  for (int k = 0; k < kEmbTypes; ++k) s[k] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (hc < H4) {
    for (int64_t m = r0 + rl; m < r1; m += kBlock / 64) {
      const float4 g = reinterpret_cast<const float4*>(dx)[m * H4 + hc];
      const int ty = tt ? (int)tt[m] : 0;
#pragma unroll
      for (int k = 0; k < kEmbTypes; ++k)
        if (ty == k) { s[k].x += g.x; s[k].y += g.y; s[k].z += g.z; s[k].w += g.w; }
    }
  }
  __shared__ float4 sh[kBlock / 64][kEmbTypes][64];
#pragma unroll
  for (int k = 0; k < kEmbTypes; ++k) sh[rl][k][threadIdx.x & 63] = s[k];
  __syncthreads();
  if (rl == 0 && hc < H4) {
#pragma unroll
    for (int k = 0; k < kEmbTypes; ++k) {
      float4 a = sh[0][k][threadIdx.x];
      for (int l = 1; l < kBlock / 64; ++l) {
        const float4 b = sh[l][k][threadIdx.x];
        a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
      }
      reinterpret_cast<float4*>(part)[((int64_t)blockIdx.y * kEmbTypes + k) * H4 + hc] = a;
    }
  }
}

__global__ __launch_bounds__(kBlock) void emb_type_final_kernel(const float* __restrict__ part, float* __restrict__ dWt,
                                                                int nparts, int NT, int H4) {
  const int i = blockIdx.x * kBlock + threadIdx.x;   // over NT * H4
  if (i >= NT * H4) return;
  const int k = i / H4, h = i - k * H4;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (k < kEmbTypes) {
    for (int p = 0; p < nparts; ++p) {
      const float4 b = reinterpret_cast<const float4*>(part)[((int64_t)p * kEmbTypes + k) * H4 + h];
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
  }
  reinterpret_cast<float4*>(dWt)[i] = a;
}

constexpr int kEmbTypeParts = 256;

}  // namespace

int emb_type_parts() { return kEmbTypeParts; }
bool emb_supported(int H, int NT) { return H % 4 == 0 && H / 4 <= 64 * 64 && NT <= kEmbTypes; }

void emb_forward(const int64_t* ids, const int64_t* tt, const float* Ww, const float* Wp, const float* Wt, float* out,
                 int64_t M, int T, int H, hipStream_t s) {
  const int H4 = H / 4;
  const int64_t n = M * H4;
  hipLaunchKernelGGL(emb_fwd_kernel, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, ids, tt, Ww, Wp,
                     Wt, out, M, T, H4);
}

void emb_backward(const int64_t* ids, const int64_t* tt, const float* dx, float* dWw, float* dWp, float* dWt,
                  float* part, int64_t M, int B, int T, int P, int NT, int H, hipStream_t s) {
  const int H4 = H / 4;
  const int64_t n = M * H4;
  if (dWw)   // zeroed by the caller
    hipLaunchKernelGGL(emb_word_bwd_kernel, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, ids, dx,
                       dWw, M, H4);
  if (dWp)
    hipLaunchKernelGGL(emb_pos_bwd_kernel, dim3((unsigned)(((int64_t)P * H4 + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                       s, dx, dWp, B, T, P, H4);
  if (dWt) {
    const int64_t rows_per = (M + kEmbTypeParts - 1) / kEmbTypeParts;
    const int nparts = (int)((M + rows_per - 1) / rows_per);
    hipLaunchKernelGGL(emb_type_partial_kernel, dim3((unsigned)((H4 + 63) / 64), (unsigned)nparts), dim3(kBlock), 0, s,
                       tt, dx, part, M, H4, rows_per);
    hipLaunchKernelGGL(emb_type_final_kernel, dim3((unsigned)((NT * H4 + kBlock - 1) / kBlock)), dim3(kBlock), 0, s,
                       part, dWt, nparts, NT, H4);
  }
}

}  // namespace gk
