// LSTM cell kernels for a bf16 LSTM layer whose GEMMs run on hipBLASLt
// (ops/lstm.py; BASELINE config 4: PTB 2 x LSTM-1500, reference
// models/lstm.py:5-47).  MIOpen's RNN -- what nn.LSTM dispatches to on ROCm --
// computes in fp16 under bf16 autocast and spends ~10 us per step in two
// hidden-update kernels (profiles/r01_lstm_kernel_stats.csv); here each step
// is one GEMM plus ONE of these element-wise kernels.
//
//   fwd: G = xg[t] + hg  (xg = x W_ih^T + b_ih + b_hh for every t, one GEMM;
//        hg = h_{t-1} W_hh^T, the step's GEMM);  i, f, o = sigmoid, g = tanh
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
// consecutive units, so every gate row is read coalesced.
#include "common.h"
#include "gk_kernels.h"

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

__global__ __launch_bounds__(kBlock) void lstm_fwd_kernel(const uint16_t* __restrict__ xg,
                                                          const uint16_t* __restrict__ hg,
                                                          const float* __restrict__ c_prev, float* __restrict__ c,
                                                          uint16_t* __restrict__ h, float* __restrict__ gates, int B,
                                                          int H) {
  const int64_t idx = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (idx >= (int64_t)B * H) return;
  const int b = (int)(idx / H), j = (int)(idx - (int64_t)b * H);
  const int64_t g0 = (int64_t)b * 4 * H + j;
  float a[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) a[k] = bf2f(xg[g0 + k * H]) + bf2f(hg[g0 + k * H]);
  const float i = sigm(a[0]), f = sigm(a[1]), g = tanhf(a[2]), o = sigm(a[3]);
  const float cn = fmaf(f, c_prev[idx], i * g);
  c[idx] = cn;
  h[idx] = f2bf16(o * tanhf(cn));
  gates[g0] = i;
  gates[g0 + H] = f;
  gates[g0 + 2 * H] = g;
  gates[g0 + 3 * H] = o;
}

__global__ __launch_bounds__(kBlock) void lstm_bwd_kernel(const uint16_t* __restrict__ dout,
                                                          const uint16_t* __restrict__ dh_rec,
                                                          const float* __restrict__ dc_next,
                                                          const float* __restrict__ gates,
                                                          const float* __restrict__ c, const float* __restrict__ c_prev,
                                                          uint16_t* __restrict__ dG, float* __restrict__ dc_prev, int B,
                                                          int H) {
  const int64_t idx = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (idx >= (int64_t)B * H) return;
  const int b = (int)(idx / H), j = (int)(idx - (int64_t)b * H);
  const int64_t g0 = (int64_t)b * 4 * H + j;
  const float i = gates[g0], f = gates[g0 + H], g = gates[g0 + 2 * H], o = gates[g0 + 3 * H];
  float dh = 0.f;
  if (dout) dh += bf2f(dout[idx]);
  if (dh_rec) dh += bf2f(dh_rec[idx]);
  const float tc = tanhf(c[idx]);
  const float dc = (dc_next ? dc_next[idx] : 0.f) + dh * o * (1.f - tc * tc);
  dG[g0] = f2bf16(dc * g * i * (1.f - i));
  dG[g0 + H] = f2bf16(dc * c_prev[idx] * f * (1.f - f));
  dG[g0 + 2 * H] = f2bf16(dc * i * (1.f - g * g));
  dG[g0 + 3 * H] = f2bf16(dh * tc * o * (1.f - o));
  dc_prev[idx] = dc * f;
}

}  // namespace

void lstm_cell_fwd(const uint16_t* xg, const uint16_t* hg, const float* c_prev, float* c, uint16_t* h, float* gates,
                   int B, int H, hipStream_t stream) {
  const int64_t n = (int64_t)B * H;
  if (n <= 0) return;
  hipLaunchKernelGGL(lstm_fwd_kernel, dim3((unsigned)ceil_div(n, (int64_t)kBlock)), dim3(kBlock), 0, stream, xg, hg,
                     c_prev, c, h, gates, B, H);
}

void lstm_cell_bwd(const uint16_t* dout, const uint16_t* dh_rec, const float* dc_next, const float* gates,
                   const float* c, const float* c_prev, uint16_t* dG, float* dc_prev, int B, int H,
                   hipStream_t stream) {
  const int64_t n = (int64_t)B * H;
  if (n <= 0) return;
  hipLaunchKernelGGL(lstm_bwd_kernel, dim3((unsigned)ceil_div(n, (int64_t)kBlock)), dim3(kBlock), 0, stream, dout,
                     dh_rec, dc_next, gates, c, c_prev, dG, dc_prev, B, H);
}

}  // namespace gk
