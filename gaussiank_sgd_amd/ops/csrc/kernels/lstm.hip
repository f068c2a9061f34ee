// LSTM cell kernels for a bf16 LSTM layer whose GEMMs run on hipBLASLt
// (ops/lstm.py; BASELINE config 4: PTB 2 x LSTM-1500, reference
// models/lstm.py:5-47).  MIOpen's RNN -- what nn.LSTM dispatches to on ROCm --
// computes in fp16 under bf16 autocast and spends ~10 us per step in two
// hidden-update kernels (profiles/r01_lstm_kernel_stats.csv); here each step
// is one GEMM plus ONE of these element-wise kernels.
//
//   fwd: G = xg[t] + hg  (xg = x W_ih^T + b_ih + b_hh for every t, one GEMM;
//        hg = h_{t-1} W_hh^T, the step's split-K GEMM);  i, f, o = sigmoid, g = tanh
//        (PyTorch gate order i, f, g, o: gate k of unit j is column k*H + j);
//        c = f c_prev + i g;  h = o tanh(c).
//        Writes h (bf16: the layer output and the next step's GEMM operand),
//        c (fp32) and the activated gates (fp32, for the backward).
//   bwd: dh = dout[t] + dh_rec (dh_rec = dG_{t+1} W_hh, the step's GEMM),
//        dc = dc_next + dh o (1 - tanh(c)^2);
//        dG = [dc g i(1-i), dc c_prev f(1-f), dc i (1-g^2), dh tanh(c) o(1-o)]
//        (bf16: the operand of the dh_rec and weight-gradient GEMMs),
//        dc_prev = dc f (fp32 carry).
// One thread per (row, unit) owns its four gates; consecutive threads take
// consecutive units, so every gate row is read coalesced.  The step GEMMs run
// split-K on rec_gemm_kernel below over 64-padded operands (h_pad, dG_pad and
// padded copies of W_hh); the cell kernels sum its fp32 K-slices on load.
#include "common.h"
#include "gk_kernels.h"
#include "mfma_util.h"

namespace gk {
namespace {

__device__ __forceinline__ float bf2f(uint16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

__device__ __forceinline__ uint16_t f2bf16(float f) {  // round-to-nearest-even, NaN kept quiet
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x7fffffu)) return (uint16_t)((u >> 16) | 0x40u);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// Split-K recurrent GEMM  P[s][m][n] = sum_{k in slice s} A[m][k] B[n][k]
// (fp32 partial slabs; the cell kernel that consumes them sums the S slices,
// so there are no atomics and no inter-block hand-off).  The per-step LSTM
// GEMM has M = batch (<= 128 per tile), N = 4H, K = H: as one GEMM it is
// latency-bound on its K loop (~20 us for H = 1500 with hipBLASLt or the
// gemm_nt kernel, bench/lstm_gemm_probe.py); split over S K-slices every
// block runs only kslice / 32 MFMA steps.  Block = 4 waves; wave w owns rows
// m0 + 32w .. +31 (two 16-row MFMA subtiles) x 64 columns (four subtiles).
// Fragments load straight from global into registers, up to eight 32-deep K
// steps in flight (A rows are L2-resident, each B row is read by one block per
// slice).
// Requirements (checked on the host): K % (64 S) == 0, N % 64 == 0, rows
// 16-byte aligned.
template <int D>
__global__ __launch_bounds__(kBlock) void rec_gemm_kernel(const uint16_t* __restrict__ A, int64_t lda,
                                                          const uint16_t* __restrict__ B, int64_t ldb,
                                                          float* __restrict__ P, int M, int N, int kslice) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int n0 = blockIdx.x * 64;
  const int s = blockIdx.y;
  const int m0 = blockIdx.z * 128 + w * 32;
  if (m0 >= M) return;  // no LDS / barriers: a wave past the last row just leaves
  const int64_t kb = (int64_t)s * kslice + fq * 8;
  const uint16_t* ap[2];
  const uint16_t* bp[4];
#pragma unroll
  for (int ms = 0; ms < 2; ++ms) {
    int r = m0 + ms * 16 + fr;
    r = r < M ? r : M - 1;
    ap[ms] = A + (int64_t)r * lda + kb;
  }
#pragma unroll
  for (int ns = 0; ns < 4; ++ns) bp[ns] = B + (int64_t)(n0 + ns * 16 + fr) * ldb + kb;
  f32x4 acc[2][4];
#pragma unroll
  for (int ms = 0; ms < 2; ++ms)
#pragma unroll
    for (int ns = 0; ns < 4; ++ns) acc[ms][ns] = f32x4{0.f, 0.f, 0.f, 0.f};
  // D 32-deep K steps per batch: all 6 D fragment loads are issued before the
  // first MFMA, so each wave keeps 6 D KB in flight (the kernel is bound by
  // load latency, not by MFMA issue)
  for (int k = 0; k < kslice; k += 32 * D) {
    bf16x8 a[D][2], b[D][4];
#pragma unroll
    for (int d = 0; d < D; ++d) {
#pragma unroll
      for (int ns = 0; ns < 4; ++ns) b[d][ns] = *reinterpret_cast<const bf16x8*>(bp[ns] + k + 32 * d);
#pragma unroll
      for (int ms = 0; ms < 2; ++ms) a[d][ms] = *reinterpret_cast<const bf16x8*>(ap[ms] + k + 32 * d);
    }
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
      for (int ms = 0; ms < 2; ++ms)
#pragma unroll
        for (int ns = 0; ns < 4; ++ns)
          acc[ms][ns] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[d][ms], b[d][ns], acc[ms][ns], 0, 0, 0);
  }
  // D[row = 4 fq + r][col = fr] of every 16x16 subtile
  float* Ps = P + (int64_t)s * M * N;
#pragma unroll
  for (int ms = 0; ms < 2; ++ms)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + ms * 16 + fq * 4 + r;
      if (m < M) {
#pragma unroll
        for (int ns = 0; ns < 4; ++ns) Ps[(int64_t)m * N + n0 + ns * 16 + fr] = acc[ms][ns][r];
      }
    }
}

// fp32 twin (the reference's precision, v_mfma_f32_16x16x4_f32): lane (fr, fq)
// loads 4 consecutive K elements of its row as one float4 and MFMA j contracts
// element j of every lane group (the same permutation on both operands), so
// each 16-deep K step is 4 MFMAs per 16x16 subtile; D such steps in flight.
template <int D>
__global__ __launch_bounds__(kBlock) void rec_gemm_f32_kernel(const float* __restrict__ A, int64_t lda,
                                                              const float* __restrict__ B, int64_t ldb,
                                                              float* __restrict__ P, int M, int N, int kslice) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int n0 = blockIdx.x * 64;
  const int s = blockIdx.y;
  const int m0 = blockIdx.z * 128 + w * 32;
  if (m0 >= M) return;
  const int64_t kb = (int64_t)s * kslice + fq * 4;
  const float* ap[2];
  const float* bp[4];
#pragma unroll
  for (int ms = 0; ms < 2; ++ms) {
    int r = m0 + ms * 16 + fr;
    r = r < M ? r : M - 1;
    ap[ms] = A + (int64_t)r * lda + kb;
  }
#pragma unroll
  for (int ns = 0; ns < 4; ++ns) bp[ns] = B + (int64_t)(n0 + ns * 16 + fr) * ldb + kb;
  f32x4 acc[2][4];
#pragma unroll
  for (int ms = 0; ms < 2; ++ms)
#pragma unroll
    for (int ns = 0; ns < 4; ++ns) acc[ms][ns] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int k = 0; k < kslice; k += 16 * D) {
    f32x4 a[D][2], b[D][4];
#pragma unroll
    for (int d = 0; d < D; ++d) {
#pragma unroll
      for (int ns = 0; ns < 4; ++ns) b[d][ns] = *reinterpret_cast<const f32x4*>(bp[ns] + k + 16 * d);
#pragma unroll
      for (int ms = 0; ms < 2; ++ms) a[d][ms] = *reinterpret_cast<const f32x4*>(ap[ms] + k + 16 * d);
    }
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int ms = 0; ms < 2; ++ms)
#pragma unroll
          for (int ns = 0; ns < 4; ++ns)
            acc[ms][ns] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[d][ms][j], b[d][ns][j], acc[ms][ns], 0, 0, 0);
  }
  float* Ps = P + (int64_t)s * M * N;
#pragma unroll
  for (int ms = 0; ms < 2; ++ms)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + ms * 16 + fq * 4 + r;
      if (m < M) {
#pragma unroll
        for (int ns = 0; ns < 4; ++ns) Ps[(int64_t)m * N + n0 + ns * 16 + fr] = acc[ms][ns][r];
      }
    }
}

// bf16x6 twin (fp32-accurate, the reference's precision, on the bf16 matrix
// cores): A is the fp32 [M][K] operand (h_pad / dG_pad), split exactly into
// bf16 parts hi + mid + lo in registers (mfma_util.h split3x8); B arrives
// pre-split as three bf16 planes [3][N][K] (W_hh is constant over the
// sequence: split ONCE per forward / backward on the host side).  The six part
// products of order <= 2 are accumulated in fp32, smallest first (the dropped
// mid*lo, lo*mid, lo*lo are each < 2^-24 |a b|) -- six 16-cycle bf16 MFMAs per
// 32-deep step against eight 32-cycle fp32 ones (2.67x on the matrix pipe).
// Lane (fr, fq) holds K elements 8 fq .. 8 fq + 7 of its row in both operands.
template <int D>
__global__ __launch_bounds__(kBlock) void rec_gemm_x6_kernel(const float* __restrict__ A, int64_t lda,
                                                             const uint16_t* __restrict__ B3, int64_t ldb,
                                                             int64_t bplane, float* __restrict__ P, int M, int N,
                                                             int kslice) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int n0 = blockIdx.x * 64;
  const int s = blockIdx.y;
  const int m0 = blockIdx.z * 128 + w * 32;
  if (m0 >= M) return;  // no LDS / barriers: a wave past the last row just leaves
  const int64_t kb = (int64_t)s * kslice + fq * 8;
  const float* ap[2];
  const uint16_t* bp[4];
#pragma unroll
  for (int ms = 0; ms < 2; ++ms) {
    int r = m0 + ms * 16 + fr;
    r = r < M ? r : M - 1;
    ap[ms] = A + (int64_t)r * lda + kb;
  }
#pragma unroll
  for (int ns = 0; ns < 4; ++ns) bp[ns] = B3 + (int64_t)(n0 + ns * 16 + fr) * ldb + kb;
  f32x4 acc[2][4];
#pragma unroll
  for (int ms = 0; ms < 2; ++ms)
#pragma unroll
    for (int ns = 0; ns < 4; ++ns) acc[ms][ns] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int k = 0; k < kslice; k += 32 * D) {
    f32x4 a[D][2][2];
    bf16x8 bh[D][4], bm[D][4], bl[D][4];
#pragma unroll
    for (int d = 0; d < D; ++d) {
#pragma unroll
      for (int ns = 0; ns < 4; ++ns) {
        const uint16_t* q = bp[ns] + k + 32 * d;
        bh[d][ns] = *reinterpret_cast<const bf16x8*>(q);
        bm[d][ns] = *reinterpret_cast<const bf16x8*>(q + bplane);
        bl[d][ns] = *reinterpret_cast<const bf16x8*>(q + 2 * bplane);
      }
#pragma unroll
      for (int ms = 0; ms < 2; ++ms) {
        a[d][ms][0] = *reinterpret_cast<const f32x4*>(ap[ms] + k + 32 * d);
        a[d][ms][1] = *reinterpret_cast<const f32x4*>(ap[ms] + k + 32 * d + 4);
      }
    }
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
      for (int ms = 0; ms < 2; ++ms) {
        bf16x8 ah, am, al;
        split3x8(a[d][ms][0], a[d][ms][1], ah, am, al);
#pragma unroll
        for (int ns = 0; ns < 4; ++ns) {
          f32x4 c = acc[ms][ns];
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh[d][ns], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl[d][ns], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bm[d][ns], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bm[d][ns], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bh[d][ns], c, 0, 0, 0);
          acc[ms][ns] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh[d][ns], c, 0, 0, 0);
        }
      }
  }
  // D[row = 4 fq + r][col = fr] of every 16x16 subtile
  float* Ps = P + (int64_t)s * M * N;
#pragma unroll
  for (int ms = 0; ms < 2; ++ms)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + ms * 16 + fq * 4 + r;
      if (m < M) {
#pragma unroll
        for (int ns = 0; ns < 4; ++ns) Ps[(int64_t)m * N + n0 + ns * 16 + fr] = acc[ms][ns][r];
      }
    }
}

// element storage of the cell kernels' bf16 / fp32 operands
__device__ __forceinline__ float ld_e(const uint16_t* p, int64_t i) { return bf2f(p[i]); }
__device__ __forceinline__ float ld_e(const float* p, int64_t i) { return p[i]; }
__device__ __forceinline__ uint16_t cvt_e(float v, uint16_t*) { return f2bf16(v); }
__device__ __forceinline__ float cvt_e(float v, float*) { return v; }

// Cell kernels.  Gate k of unit j: column k*H + j of the [B][4H] rows (xg,
// gates, dG), column k*Hp + j of the 64-padded [B][4Hp] rows (P, dG_pad).
template <typename T>
__global__ __launch_bounds__(kBlock) void lstm_fwd_kernel(const T* __restrict__ xg, const T* __restrict__ hg,
                                                          const float* __restrict__ P, int S,
                                                          const float* __restrict__ c_prev, float* __restrict__ c,
                                                          T* __restrict__ h, T* __restrict__ h_pad,
                                                          float* __restrict__ gates, int B, int H, int Hp) {
  const int64_t idx = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (idx >= (int64_t)B * H) return;
  const int b = (int)(idx / H), j = (int)(idx - (int64_t)b * H);
  const int64_t g0 = (int64_t)b * 4 * H + j;
  const int64_t p0 = (int64_t)b * 4 * Hp + j;
  const int64_t slab = (int64_t)B * 4 * Hp;
  float a[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) a[k] = ld_e(xg, g0 + k * H);
  if (hg)
#pragma unroll
    for (int k = 0; k < 4; ++k) a[k] += ld_e(hg, g0 + k * H);
  for (int s = 0; s < S; ++s)
#pragma unroll
    for (int k = 0; k < 4; ++k) a[k] += P[s * slab + p0 + k * Hp];
  const float i = sigm(a[0]), f = sigm(a[1]), g = tanhf(a[2]), o = sigm(a[3]);
  const float cn = fmaf(f, c_prev[idx], i * g);
  c[idx] = cn;
  const T hv = cvt_e(o * tanhf(cn), h);
  h[idx] = hv;
  if (h_pad) h_pad[(int64_t)b * Hp + j] = hv;
  gates[g0] = i;
  gates[g0 + H] = f;
  gates[g0 + 2 * H] = g;
  gates[g0 + 3 * H] = o;
}

template <typename T>
__global__ __launch_bounds__(kBlock) void lstm_bwd_kernel(const T* __restrict__ dout, const T* __restrict__ dh_rec,
                                                          const float* __restrict__ P, int S,
                                                          const float* __restrict__ dc_next,
                                                          const float* __restrict__ gates,
                                                          const float* __restrict__ c, const float* __restrict__ c_prev,
                                                          T* __restrict__ dG, T* __restrict__ dG_pad,
                                                          float* __restrict__ dc_prev, int B, int H, int Hp) {
  const int64_t idx = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (idx >= (int64_t)B * H) return;
  const int b = (int)(idx / H), j = (int)(idx - (int64_t)b * H);
  const int64_t g0 = (int64_t)b * 4 * H + j;
  const float i = gates[g0], f = gates[g0 + H], g = gates[g0 + 2 * H], o = gates[g0 + 3 * H];
  float dh = dout ? ld_e(dout, idx) : 0.f;
  if (dh_rec) dh += ld_e(dh_rec, idx);
  if (P) {
    const int64_t p0 = (int64_t)b * Hp + j, slab = (int64_t)B * Hp;
    for (int s = 0; s < S; ++s) dh += P[s * slab + p0];
  }
  const float tc = tanhf(c[idx]);
  const float dc = (dc_next ? dc_next[idx] : 0.f) + dh * o * (1.f - tc * tc);
  const T d[4] = {cvt_e(dc * g * i * (1.f - i), dG), cvt_e(dc * c_prev[idx] * f * (1.f - f), dG),
                  cvt_e(dc * i * (1.f - g * g), dG), cvt_e(dh * tc * o * (1.f - o), dG)};
#pragma unroll
  for (int k = 0; k < 4; ++k) dG[g0 + k * H] = d[k];
  if (dG_pad) {
    const int64_t q0 = (int64_t)b * 4 * Hp + j;
#pragma unroll
    for (int k = 0; k < 4; ++k) dG_pad[q0 + k * Hp] = d[k];
  }
  dc_prev[idx] = dc * f;
}

}  // namespace

void lstm_rec_gemm(const uint16_t* A, int64_t lda, const uint16_t* B, int64_t ldb, float* P, int M, int N, int K,
                   int S, hipStream_t stream) {
  if (M <= 0 || N <= 0 || S <= 0) return;
  dim3 grid((unsigned)(N / 64), (unsigned)S, (unsigned)ceil_div(M, 128));
  const int ks = K / S;
  if (ks % 256 == 0)
    hipLaunchKernelGGL(rec_gemm_kernel<8>, grid, dim3(kBlock), 0, stream, A, lda, B, ldb, P, M, N, ks);
  else if (ks % 128 == 0)
    hipLaunchKernelGGL(rec_gemm_kernel<4>, grid, dim3(kBlock), 0, stream, A, lda, B, ldb, P, M, N, ks);
  else
    hipLaunchKernelGGL(rec_gemm_kernel<2>, grid, dim3(kBlock), 0, stream, A, lda, B, ldb, P, M, N, ks);
}

void lstm_rec_gemm_f32(const float* A, int64_t lda, const float* B, int64_t ldb, float* P, int M, int N, int K, int S,
                       hipStream_t stream) {
  if (M <= 0 || N <= 0 || S <= 0) return;
  dim3 grid((unsigned)(N / 64), (unsigned)S, (unsigned)ceil_div(M, 128));
  const int ks = K / S;
  if (ks % 128 == 0)
    hipLaunchKernelGGL(rec_gemm_f32_kernel<8>, grid, dim3(kBlock), 0, stream, A, lda, B, ldb, P, M, N, ks);
  else
    hipLaunchKernelGGL(rec_gemm_f32_kernel<4>, grid, dim3(kBlock), 0, stream, A, lda, B, ldb, P, M, N, ks);
}

void lstm_rec_gemm_x6(const float* A, int64_t lda, const uint16_t* B3, int64_t ldb, int64_t bplane, float* P, int M,
                      int N, int K, int S, hipStream_t stream) {
  if (M <= 0 || N <= 0 || S <= 0) return;
  dim3 grid((unsigned)(N / 64), (unsigned)S, (unsigned)ceil_div(M, 128));
  const int ks = K / S;
  if (ks % 64 == 0)
    hipLaunchKernelGGL(rec_gemm_x6_kernel<2>, grid, dim3(kBlock), 0, stream, A, lda, B3, ldb, bplane, P, M, N, ks);
  else
    hipLaunchKernelGGL(rec_gemm_x6_kernel<1>, grid, dim3(kBlock), 0, stream, A, lda, B3, ldb, bplane, P, M, N, ks);
}

template <typename T>
void cell_fwd(const T* xg, const T* hg, const float* P, int S, const float* c_prev, float* c, T* h, T* h_pad,
              float* gates, int B, int H, int Hp, hipStream_t stream) {
  const int64_t n = (int64_t)B * H;
  if (n <= 0) return;
  hipLaunchKernelGGL(lstm_fwd_kernel<T>, dim3((unsigned)ceil_div(n, (int64_t)kBlock)), dim3(kBlock), 0, stream, xg, hg,
                     P, S, c_prev, c, h, h_pad, gates, B, H, Hp);
}

template <typename T>
void cell_bwd(const T* dout, const T* dh_rec, const float* P, int S, const float* dc_next, const float* gates,
              const float* c, const float* c_prev, T* dG, T* dG_pad, float* dc_prev, int B, int H, int Hp,
              hipStream_t stream) {
  const int64_t n = (int64_t)B * H;
  if (n <= 0) return;
  hipLaunchKernelGGL(lstm_bwd_kernel<T>, dim3((unsigned)ceil_div(n, (int64_t)kBlock)), dim3(kBlock), 0, stream, dout,
                     dh_rec, P, S, dc_next, gates, c, c_prev, dG, dG_pad, dc_prev, B, H, Hp);
}

void lstm_cell_fwd(const uint16_t* xg, const uint16_t* hg, const float* P, int S, const float* c_prev, float* c, uint16_t* h,
                   uint16_t* h_pad, float* gates, int B, int H, int Hp, hipStream_t stream) {
  cell_fwd<uint16_t>(xg, hg, P, S, c_prev, c, h, h_pad, gates, B, H, Hp, stream);
}

void lstm_cell_bwd(const uint16_t* dout, const uint16_t* dh_rec, const float* P, int S, const float* dc_next, const float* gates,
                   const float* c, const float* c_prev, uint16_t* dG, uint16_t* dG_pad, float* dc_prev, int B, int H,
                   int Hp, hipStream_t stream) {
  cell_bwd<uint16_t>(dout, dh_rec, P, S, dc_next, gates, c, c_prev, dG, dG_pad, dc_prev, B, H, Hp, stream);
}

void lstm_cell_fwd_f32(const float* xg, const float* hg, const float* P, int S, const float* c_prev, float* c, float* h,
                       float* h_pad, float* gates, int B, int H, int Hp, hipStream_t stream) {
  cell_fwd<float>(xg, hg, P, S, c_prev, c, h, h_pad, gates, B, H, Hp, stream);
}

void lstm_cell_bwd_f32(const float* dout, const float* dh_rec, const float* P, int S, const float* dc_next,
                       const float* gates, const float* c, const float* c_prev, float* dG, float* dG_pad, float* dc_prev,
                       int B, int H, int Hp, hipStream_t stream) {
  cell_bwd<float>(dout, dh_rec, P, S, dc_next, gates, c, c_prev, dG, dG_pad, dc_prev, B, H, Hp, stream);
}

}  // namespace gk
