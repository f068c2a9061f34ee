// Column passes of bf16 / fp32 linear layers (BERT encoder / MLM head, LSTM softmax),
// accumulating straight into the optimizer's fp32 gradient arena:
//   colsum_acc  db[n] += sum_m dy[m, n]                       (bias gradient)
//   gelu_bwd    dpre = dy * gelu'(pre) (erf GELU, as F.gelu) and, with db,
//               db[n] += sum_m dpre[m, n] -- the GELU backward and the bias
//               gradient of the producing linear in ONE pass over dy / pre.
// torch computes the bias gradient as a separate bf16 reduction at ~1 TB/s
// (profiles/r01_bert_kernel_stats.csv: 49 calls, 1.3 ms per BERT step) plus a
// cast-and-add into the fp32 arena; here it is a streaming pass at HBM rate.
//
// Layout: [M, N] row-major bf16 or fp32, N % 8 == 0, rows 16-byte aligned.  Lane
// (rl, cl) of a 256-thread block owns columns 8*cl .. 8*cl+7 of the block's
// 256-column slab (one 16-byte load per row in bf16, two in fp32; kUnroll rows in flight) and rows
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

// 8 consecutive elements of a row as fp32, and back (bf16: one 16-byte
// access, fp32: two)
template <typename T>
struct Row8;
template <>
struct Row8<uint16_t> {
  static __device__ __forceinline__ void load(const uint16_t* p, float v[8]) {
    const uint4 u = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      v[2 * h] = lo_bf(w[h]);
      v[2 * h + 1] = hi_bf(w[h]);
    }
  }
  // rounds v to the stored precision (the values the consumers read) and stores
  static __device__ __forceinline__ void store(uint16_t* p, float v[8]) {
    uint32_t w[4];
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      w[h] = bf_bits(v[2 * h]) | (bf_bits(v[2 * h + 1]) << 16);
      v[2 * h] = lo_bf(w[h]);
      v[2 * h + 1] = hi_bf(w[h]);
    }
    *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
  }
};
template <>
struct Row8<float> {
  static __device__ __forceinline__ void load(const float* p, float v[8]) {
    const float4 a = *reinterpret_cast<const float4*>(p);
    const float4 b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
  static __device__ __forceinline__ void store(float* p, float v[8]) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
};

template <bool GELU, typename T>
__global__ __launch_bounds__(kBlock) void colsum_kernel(const T* __restrict__ dy, const T* __restrict__ pre,
                                                        T* __restrict__ dpre, float* __restrict__ db, int64_t M,
                                                        int N) {
  __shared__ float red[kRL][kCL * 8];
  const int cl = threadIdx.x % kCL, rl = threadIdx.x / kCL;
  const int c0 = (blockIdx.x * kCL + cl) * 8;
  float s[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) s[i] = 0.f;
  if (c0 < N) {
    const int64_t step = (int64_t)gridDim.y * kRL;
    for (int64_t r = (int64_t)blockIdx.y * kRL + rl; r < M; r += kUnroll * step) {
      float u[kUnroll][8], q[kUnroll][8];
#pragma unroll
      for (int j = 0; j < kUnroll; ++j) {
        const int64_t rr = r + j * step;
#pragma unroll
        for (int i = 0; i < 8; ++i) u[j][i] = q[j][i] = 0.f;
        if (rr < M) {
          Row8<T>::load(dy + rr * N + c0, u[j]);
          if (GELU) Row8<T>::load(pre + rr * N + c0, q[j]);
        }
      }
#pragma unroll
      for (int j = 0; j < kUnroll; ++j) {
        if (GELU) {
#pragma unroll
          for (int i = 0; i < 8; ++i) u[j][i] *= gelu_grad(q[j][i]);
          const int64_t rr = r + j * step;
          if (rr < M) Row8<T>::store(dpre + rr * N + c0, u[j]);   // u: now the stored values
        }
        // sums of the values as stored (what the weight / input GEMMs consume)
#pragma unroll
        for (int i = 0; i < 8; ++i) s[i] += u[j][i];
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

template <bool GELU, typename T>
void launch_colsum(const T* dy, const T* pre, T* dpre, float* db, int64_t M, int N, hipStream_t s) {
  if (M <= 0 || N <= 0) return;
  const int gx = (int)ceil_div(N, kCL * 8);
  // >= two unrolled passes per lane; about eight blocks per CU in total
  int64_t gy = ceil_div(M, (int64_t)kRL * kUnroll * 2);
  const int64_t cap = 2048 / gx > 0 ? 2048 / gx : 1;
  if (gy > cap) gy = cap;
  if (gy < 1) gy = 1;
  hipLaunchKernelGGL((colsum_kernel<GELU, T>), dim3((unsigned)gx, (unsigned)gy), dim3(kBlock), 0, s, dy, pre, dpre,
                     db, M, N);
}

}  // namespace

void colsum_acc_bf16(const uint16_t* dy, float* db, int64_t M, int N, hipStream_t stream) {
  if (db == nullptr) return;
  launch_colsum<false, uint16_t>(dy, nullptr, nullptr, db, M, N, stream);
}

void gelu_bwd_colsum_bf16(const uint16_t* dy, const uint16_t* pre, uint16_t* dpre, float* db, int64_t M, int N,
                          hipStream_t stream) {
  launch_colsum<true, uint16_t>(dy, pre, dpre, db, M, N, stream);
}

void colsum_acc_f32(const float* dy, float* db, int64_t M, int N, hipStream_t stream) {
  if (db == nullptr) return;
  launch_colsum<false, float>(dy, nullptr, nullptr, db, M, N, stream);
}

void gelu_bwd_colsum_f32(const float* dy, const float* pre, float* dpre, float* db, int64_t M, int N,
                         hipStream_t stream) {
  launch_colsum<true, float>(dy, pre, dpre, db, M, N, stream);
}

}  // namespace gk
