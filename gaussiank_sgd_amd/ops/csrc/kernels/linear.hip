// Column passes of bf16 linear layers (BERT encoder / MLM head, LSTM softmax),
// accumulating straight into the optimizer's fp32 gradient arena:
//   colsum_acc  db[n] += sum_m dy[m, n]                       (bias gradient)
//   gelu_bwd    dpre = dy * gelu'(pre) (erf GELU, as F.gelu) and, with db,
//               db[n] += sum_m dpre[m, n] -- the GELU backward and the bias
//               gradient of the producing linear in ONE pass over dy / pre.
// torch computes the bias gradient as a separate bf16 reduction at ~1 TB/s
// (profiles/r01_bert_kernel_stats.csv: 49 calls, 1.3 ms per BERT step) plus a
// cast-and-add into the fp32 arena; here it is a streaming pass at HBM rate.
//
// Layout: [M, N] row-major bf16, N % 8 == 0, rows 16-byte aligned.  Lane
// (rl, cl) of a 256-thread block owns columns 8*cl .. 8*cl+7 of the block's
// 256-column slab (one 16-byte load per row, kUnroll rows in flight) and rows
// rl, rl + 8, ... of the block's row range.  The 8 row lanes' fp32 sums are
// folded through LDS and each column receives ONE float atomic per block
// (a wave's atomics cover 256 contiguous bytes: the full-rate shape).
#include "common.h"
#include "gk_kernels.h"

namespace gk {
namespace {

constexpr int kCL = 32;               // column lanes: 32 x 8 = 256 columns per block
constexpr int kRL = kBlock / kCL;     // row lanes
constexpr int kUnroll = 4;            // rows in flight per lane

__device__ __forceinline__ float lo_bf(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float hi_bf(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }

__device__ __forceinline__ uint32_t bf_bits(float f) {  // round-to-nearest-even, NaN kept quiet
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x7fffffu)) return (u >> 16) | 0x40u;
  u += 0x7fffu + ((u >> 16) & 1u);
  return u >> 16;
}

// d/dx [x * Phi(x)] = Phi(x) + x * phi(x)   (F.gelu, approximate='none')
__device__ __forceinline__ float gelu_grad(float x) {
  const float cdf = 0.5f * (1.f + erff(x * 0.70710678118654752f));
  const float pdf = 0.39894228040143268f * __expf(-0.5f * x * x);
  return fmaf(x, pdf, cdf);
}

template <bool GELU>
__global__ __launch_bounds__(kBlock) void colsum_kernel(const uint16_t* __restrict__ dy,
                                                        const uint16_t* __restrict__ pre,
                                                        uint16_t* __restrict__ dpre, float* __restrict__ db,
                                                        int64_t M, int N) {
  __shared__ float red[kRL][kCL * 8];
  const int cl = threadIdx.x % kCL, rl = threadIdx.x / kCL;
  const int c0 = (blockIdx.x * kCL + cl) * 8;
  float s[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) s[i] = 0.f;
  if (c0 < N) {
    const int64_t step = (int64_t)gridDim.y * kRL;
    for (int64_t r = (int64_t)blockIdx.y * kRL + rl; r < M; r += kUnroll * step) {
      uint4 u[kUnroll], p[kUnroll];
#pragma unroll
      for (int j = 0; j < kUnroll; ++j) {
        const int64_t rr = r + j * step;
        u[j] = make_uint4(0u, 0u, 0u, 0u);
        p[j] = make_uint4(0u, 0u, 0u, 0u);
        if (rr < M) {
          u[j] = *reinterpret_cast<const uint4*>(dy + rr * N + c0);
          if (GELU) p[j] = *reinterpret_cast<const uint4*>(pre + rr * N + c0);
        }
      }
#pragma unroll
      for (int j = 0; j < kUnroll; ++j) {
        uint32_t w[4] = {u[j].x, u[j].y, u[j].z, u[j].w};
        if (GELU) {
          const uint32_t q[4] = {p[j].x, p[j].y, p[j].z, p[j].w};
#pragma unroll
          for (int h = 0; h < 4; ++h) {
            const float d0 = lo_bf(w[h]) * gelu_grad(lo_bf(q[h]));
            const float d1 = hi_bf(w[h]) * gelu_grad(hi_bf(q[h]));
            w[h] = bf_bits(d0) | (bf_bits(d1) << 16);
          }
          const int64_t rr = r + j * step;
          if (rr < M) *reinterpret_cast<uint4*>(dpre + rr * N + c0) = make_uint4(w[0], w[1], w[2], w[3]);
        }
        // sums of the values as stored (the bf16 the weight / input GEMMs consume)
#pragma unroll
        for (int h = 0; h < 4; ++h) {
          s[2 * h] += lo_bf(w[h]);
          s[2 * h + 1] += hi_bf(w[h]);
        }
      }
    }
  }
  if (db == nullptr) return;   // kernel argument: uniform over the block
#pragma unroll
  for (int i = 0; i < 8; ++i) red[rl][cl * 8 + i] = s[i];
  __syncthreads();
  const int col = blockIdx.x * (kCL * 8) + threadIdx.x;
  if (col < N) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < kRL; ++k) t += red[k][threadIdx.x];
    atomicAdd(db + col, t);
  }
}

template <bool GELU>
void launch_colsum(const uint16_t* dy, const uint16_t* pre, uint16_t* dpre, float* db, int64_t M, int N,
                   hipStream_t s) {
  if (M <= 0 || N <= 0) return;
  const int gx = (int)ceil_div(N, kCL * 8);
  // >= two unrolled passes per lane; about eight blocks per CU in total
  int64_t gy = ceil_div(M, (int64_t)kRL * kUnroll * 2);
  const int64_t cap = 2048 / gx > 0 ? 2048 / gx : 1;
  if (gy > cap) gy = cap;
  if (gy < 1) gy = 1;
  hipLaunchKernelGGL((colsum_kernel<GELU>), dim3((unsigned)gx, (unsigned)gy), dim3(kBlock), 0, s, dy, pre, dpre, db,
                     M, N);
}

}  // namespace

void colsum_acc_bf16(const uint16_t* dy, float* db, int64_t M, int N, hipStream_t stream) {
  if (db == nullptr) return;
  launch_colsum<false>(dy, nullptr, nullptr, db, M, N, stream);
}

void gelu_bwd_colsum_bf16(const uint16_t* dy, const uint16_t* pre, uint16_t* dpre, float* db, int64_t M, int N,
                          hipStream_t stream) {
  launch_colsum<true>(dy, pre, dpre, db, M, N, stream);
}

}  // namespace gk
