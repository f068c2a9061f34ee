// The ImageNet-ResNet stem convolution (7x7, stride 2, padding 3, 3 -> 64
// channels) at fp32 -- the reference's precision -- on v_mfma_f32_16x16x4_f32.
// stem.hip is the bf16 path (bf16 MFMA on packed 4-channel pixels); at fp32
// MIOpen was the fallback, 1.4 ms forward + 2.2 ms grad-weight per bs512 step
// (profiles/r03_resnet50_bs512_fp32_kernel_stats.csv, igemm_fwd / igemm_wrw
// rows): its implicit GEMM handles the 3-channel input badly.
//
// K = 7 x 7 x 3 = 147 taps, ordered (kh, kw, c) like the NHWC input, padded to
// 148; a tap's offset inside an LDS input band is koff(k) = (kh * PW + kw) * 3
// + c (tap_off, computed per k-step), so an MFMA operand element is one
// ds_read_b32 at pixel_base + koff.
//
// forward: a persistent block walks bands of 4 output rows of one image; the
//   band's 13 input rows (zero padding materialised, 230 pixels x 3 channels)
//   and the whole [64][148] weight matrix sit in LDS.  Wave w owns output row
//   w of the band: 7 16-pixel subtiles x 4 16-channel subtiles (112 fp32
//   accumulators), 37 k-steps of 4 taps, weights as the MFMA A operand so a
//   lane ends with 4 consecutive channels of one pixel (16-byte stores); the
//   epilogue reduces the following BatchNorm's batch statistics per block
//   (stats row = block, as gemm.hip's conv epilogue).
// grad-weight: dW[n][k] = sum_px dY[px][n] A[px][k], contraction over pixels
//   4 at a time: dY fragments straight from global (lane = channel, coalesced),
//   A fragments gathered from the LDS band; each wave accumulates 64 x 160
//   (4 x 10 subtiles, 160 registers) over its rows of every band of the
//   block; the 4 waves are summed through LDS and every block writes one
//   partial; stem_f32_wgrad_reduce sums the partials in a fixed order
//   (deterministic) into the (arena) gradient.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "common.h"
#include "gk_kernels.h"
#include "mfma_util.h"

namespace gk {
namespace {

constexpr int kFR = 4;                    // output rows per band (one per wave)
constexpr int kFIn = 2 * kFR + 5;         // input rows per band
constexpr int kFK = 147, kFKP = 148;      // taps, padded
constexpr int kFOW = 112;                 // output width the kernels are built for (224 input)
constexpr int kFPW = 2 * kFOW + 6;        // padded input band width (pixels)
constexpr int kFBand = kFIn * kFPW * 3;   // floats of one input band
constexpr int kFWg = 64 * kFKP;           // floats of the weight matrix
constexpr int kFKS = 10;                  // grad-weight k subtiles (160 >= 148)

struct StemF32Geo {
  int N, H, W, OH, OW, nbands;   // nbands = N * OH / kFR
};

// input rows 2 orow0 - 3 .. + 12 of image n, columns -3 .. 226, zero outside.
// An NHWC image row is 224 x 3 contiguous floats (16-byte aligned: 2688 B),
// copied as float4; the 3-pixel borders are zero.
__device__ __forceinline__ void load_band(float* band, const float* __restrict__ x, const StemF32Geo& g, int n,
                                          int orow0) {
  constexpr int RV = 2 * kFOW * 3 / 4;   // float4 per input row
  constexpr int RW = kFPW * 3;           // floats per band row
  const int ih0 = 2 * orow0 - 3;
  for (int i = threadIdx.x; i < kFIn * RV; i += blockDim.x) {
    const int rr = i / RV, j = i - rr * RV;
    const int ih = ih0 + rr;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if ((unsigned)ih < (unsigned)g.H) v = reinterpret_cast<const float4*>(x + ((int64_t)n * g.H + ih) * g.W * 3)[j];
    float* d = band + rr * RW + 9 + 4 * j;
    d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
  }
  for (int i = threadIdx.x; i < kFIn * 18; i += blockDim.x) {
    const int rr = i / 18, j = i - rr * 18;
    band[rr * RW + (j < 9 ? j : RW - 18 + j)] = 0.f;
  }
}

// LDS offset of tap k inside the band (koff table, computed: one fewer LDS
// round trip per k-step); the padded tap 147 reads offset 0 (weight 0)
__device__ __forceinline__ int tap_off(int k) {
  const int kh = k / 21, r = k - kh * 21, kw = r / 3, c = r - kw * 3;
  return k < kFK ? (kh * kFPW + kw) * 3 + c : 0;
}

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
stem_f32_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w, int64_t s0, int64_t s1, int64_t s2,
                    int64_t s3, float* __restrict__ y, StemF32Geo g, float* __restrict__ stats, int64_t stats_ld) {
  extern __shared__ __attribute__((aligned(16))) float fl[];
  float* band = fl;
  float* wl = fl + kFBand;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fi = lane & 15, fq = lane >> 4;
  // weights [n][k], k = (kh * 7 + kw) * 3 + c, k = 147 zero
  for (int i = threadIdx.x; i < kFWg; i += blockDim.x) {
    const int n = i / kFKP, k = i - n * kFKP;
    float v = 0.f;
    if (k < kFK) {
      const int kh = k / 21, r = k - kh * 21, kw = r / 3, c = r - kw * 3;
      v = w[n * s0 + c * s1 + kh * s2 + kw * s3];
    }
    wl[i] = v;
  }
  float ssum[4][4], ssq[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int r = 0; r < 4; ++r) ssum[a][r] = ssq[a][r] = 0.f;
  const int bpi = g.OH / kFR;   // bands per image
  for (int b = blockIdx.x; b < g.nbands; b += gridDim.x) {
    const int n = b / bpi, orow0 = (b - n * bpi) * kFR;
    __syncthreads();   // the previous band's reads are done
    load_band(band, x, g, n, orow0);
    __syncthreads();
    f32x4 acc[7][4];
#pragma unroll
    for (int t = 0; t < 7; ++t)
#pragma unroll
      for (int a = 0; a < 4; ++a) acc[t][a] = f32x4{0.f, 0.f, 0.f, 0.f};
    int pb[7];
#pragma unroll
    for (int t = 0; t < 7; ++t) pb[t] = (2 * wave * kFPW + 2 * (t * 16 + fi)) * 3;
    // operands of k-step s + 1 read while the 28 MFMAs of step s run
    auto ldop = [&](int st, float (&bwv)[4], float (&axv)[7]) __attribute__((always_inline)) {
      const int k = 4 * st + fq;
      const int ko = tap_off(k);
#pragma unroll
      for (int a = 0; a < 4; ++a) bwv[a] = wl[(a * 16 + fi) * kFKP + k];
#pragma unroll
      for (int t = 0; t < 7; ++t) axv[t] = band[pb[t] + ko];
    };
    float bw[4], ax[7];
    ldop(0, bw, ax);
    for (int st = 0; st < kFKP / 4; ++st) {
      float bn[4], an[7];
      if (st + 1 < kFKP / 4) ldop(st + 1, bn, an);
#pragma unroll
      for (int t = 0; t < 7; ++t)
#pragma unroll
        for (int a = 0; a < 4; ++a) acc[t][a] = __builtin_amdgcn_mfma_f32_16x16x4f32(bw[a], ax[t], acc[t][a], 0, 0, 0);
#pragma unroll
      for (int a = 0; a < 4; ++a) bw[a] = bn[a];
#pragma unroll
      for (int t = 0; t < 7; ++t) ax[t] = an[t];
    }
    // lane: channels a * 16 + 4 fq + r of pixel t * 16 + fi of output row orow0 + wave
    const int orow = orow0 + wave;
#pragma unroll
    for (int t = 0; t < 7; ++t) {
      const int ocol = t * 16 + fi;
      float* yp = y + (((int64_t)n * g.OH + orow) * g.OW + ocol) * 64;
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const f32x4 v = acc[t][a];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          ssum[a][r] += v[r];
          ssq[a][r] = fmaf(v[r], v[r], ssq[a][r]);
        }
        *reinterpret_cast<f32x4*>(yp + a * 16 + 4 * fq) = v;
      }
    }
  }
  if (stats) {
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) {
          ssum[a][r] += __shfl_xor(ssum[a][r], off, 64);
          ssq[a][r] += __shfl_xor(ssq[a][r], off, 64);
        }
    __syncthreads();
    float* red = fl;   // [sum | sq][wave][64]
    if (fi == 0) {
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          red[wave * 64 + a * 16 + 4 * fq + r] = ssum[a][r];
          red[(4 + wave) * 64 + a * 16 + 4 * fq + r] = ssq[a][r];
        }
    }
    __syncthreads();
    if (threadIdx.x < 64) {
      float sa = 0.f, sb = 0.f;
#pragma unroll
      for (int w2 = 0; w2 < 4; ++w2) {
        sa += red[w2 * 64 + threadIdx.x];
        sb += red[(4 + w2) * 64 + threadIdx.x];
      }
      stats[(int64_t)blockIdx.x * 64 + threadIdx.x] = sa;
      stats[stats_ld + (int64_t)blockIdx.x * 64 + threadIdx.x] = sb;
    }
  }
}

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
stem_f32_wgrad_kernel(const float* __restrict__ x, const float* __restrict__ dy, float* __restrict__ part,
                      StemF32Geo g) {
  extern __shared__ __attribute__((aligned(16))) float fl[];
  float* band = fl;                                  // also the cross-wave reduction area [64][160]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fi = lane & 15, fq = lane >> 4;
  int ko[kFKS];
#pragma unroll
  for (int ks = 0; ks < kFKS; ++ks) ko[ks] = tap_off(ks * 16 + fi);   // taps >= 147: gradient dropped
  f32x4 acc[4][kFKS];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int ks = 0; ks < kFKS; ++ks) acc[a][ks] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int bpi = g.OH / kFR;
  for (int b = blockIdx.x; b < g.nbands; b += gridDim.x) {
    const int n = b / bpi, orow0 = (b - n * bpi) * kFR;
    __syncthreads();
    load_band(band, x, g, n, orow0);
    __syncthreads();
    const int orow = orow0 + wave;
    const float* dyr = dy + (((int64_t)n * g.OH + orow) * g.OW) * 64;
    // dY (global) and A (LDS) fragments of pixel step s + 1 in flight while
    // the 40 MFMAs of step s run
    auto ldop = [&](int st, float (&gav)[4], float (&xbv)[kFKS]) __attribute__((always_inline)) {
      const int ocol = 4 * st + fq;   // the pixel this lane's contraction slot holds
#pragma unroll
      for (int a = 0; a < 4; ++a) gav[a] = dyr[(int64_t)ocol * 64 + a * 16 + fi];
      const int pb = (2 * wave * kFPW + 2 * ocol) * 3;
#pragma unroll
      for (int ks = 0; ks < kFKS; ++ks) xbv[ks] = band[pb + ko[ks]];
    };
    float ga[4], xb[kFKS];
    ldop(0, ga, xb);
    for (int st = 0; st < kFOW / 4; ++st) {
      float gn[4], xn[kFKS];
      if (st + 1 < kFOW / 4) ldop(st + 1, gn, xn);
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int ks = 0; ks < kFKS; ++ks)
          acc[a][ks] = __builtin_amdgcn_mfma_f32_16x16x4f32(ga[a], xb[ks], acc[a][ks], 0, 0, 0);
#pragma unroll
      for (int a = 0; a < 4; ++a) ga[a] = gn[a];
#pragma unroll
      for (int ks = 0; ks < kFKS; ++ks) xb[ks] = xn[ks];
    }
  }
  // lane: dW[n = a * 16 + 4 fq + r][k = ks * 16 + fi]; sum the 4 waves in order through LDS
  float* red = fl;
  for (int w2 = 0; w2 < 4; ++w2) {
    __syncthreads();
    if (wave == w2) {
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int ks = 0; ks < kFKS; ++ks)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float* p = red + (a * 16 + 4 * fq + r) * 160 + ks * 16 + fi;
            *p = (w2 == 0 ? 0.f : *p) + acc[a][ks][r];
          }
    }
  }
  __syncthreads();
  float* dst = part + (int64_t)blockIdx.x * 64 * kFKP;
  for (int i = threadIdx.x; i < 64 * kFKP; i += blockDim.x) {
    const int nn = i / kFKP, k = i - nn * kFKP;
    dst[i] = red[nn * 160 + k];
  }
}

// ---------------------------------------------------------------------------
// bf16x6 forward (fp32-accurate on the bf16 matrix cores, as gemm_kern.h X6):
// the weights are split ONCE per call into three exact bf16 planes [3][64][160]
// (stem_w_split3_kernel; taps >= 147 zero), the band's activations are split
// in registers (mfma_util.h split3x8), and the six part products of order
// <= 2 are accumulated in fp32, smallest first.  K = 160 taps = five 32-deep
// v_mfma_f32_16x16x32_bf16 steps (6 x 16 cycles each) against 37 4-deep fp32
// steps (32 cycles each): 2.5x fewer matrix-pipe cycles.  Same band walk,
// output layout and statistics epilogue as stem_f32_fwd_kernel; the weight
// fragments come straight from global memory (61 KiB, L2-resident), so LDS
// holds the input band only.
// ---------------------------------------------------------------------------
constexpr int kXK = 160;                  // taps padded to five 32-deep steps
constexpr int kXPlane = 64 * kXK;         // elements of one weight plane

__device__ __forceinline__ uint16_t bf16_rne(float v) { return (uint16_t)(pack_bf16x2(v, 0.f) & 0xffffu); }

__global__ void __launch_bounds__(256) stem_w_split3_kernel(const float* __restrict__ w, int64_t s0, int64_t s1,
                                                            int64_t s2, int64_t s3, uint16_t* __restrict__ wp3) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= kXPlane) return;
  const int n = i / kXK, k = i - n * kXK;
  float v = 0.f;
  if (k < kFK) {
    const int kh = k / 21, r = k - kh * 21, kw = r / 3, c = r - kw * 3;
    v = w[n * s0 + c * s1 + kh * s2 + kw * s3];
  }
  const uint16_t hi = bf16_rne(v);
  const float r1 = v - __uint_as_float((uint32_t)hi << 16);
  const uint16_t mid = bf16_rne(r1);
  const float r2 = r1 - __uint_as_float((uint32_t)mid << 16);
  wp3[i] = hi;
  wp3[kXPlane + i] = mid;
  wp3[2 * kXPlane + i] = bf16_rne(r2);
}

// OCC: waves per SIMD the register budget is set for (1: 179 VGPR + 112 AGPR,
// no spills; 2: 256 registers with a 40-byte spill) -- GKSGD_STEM_X6_OCC picks;
// default 2: bs128 0.249 ms vs 0.309 (OCC 1) vs 0.339 for the fp32-MFMA kernel
// (bench/stem_x6_probe.py, profiles/r06_stem_x6.txt)
template <int OCC>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC)))
stem_f32x6_fwd_kernel(const float* __restrict__ x, const uint16_t* __restrict__ wp3, float* __restrict__ y,
                      StemF32Geo g, float* __restrict__ stats, int64_t stats_ld) {
  extern __shared__ __attribute__((aligned(16))) float fl[];
  float* band = fl;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fi = lane & 15, fq = lane >> 4;
  float ssum[4][4], ssq[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int r = 0; r < 4; ++r) ssum[a][r] = ssq[a][r] = 0.f;
  const int bpi = g.OH / kFR;
  for (int b = blockIdx.x; b < g.nbands; b += gridDim.x) {
    const int n = b / bpi, orow0 = (b - n * bpi) * kFR;
    __syncthreads();   // the previous band's reads are done
    load_band(band, x, g, n, orow0);
    __syncthreads();
    f32x4 acc[7][4];
#pragma unroll
    for (int t = 0; t < 7; ++t)
#pragma unroll
      for (int a = 0; a < 4; ++a) acc[t][a] = f32x4{0.f, 0.f, 0.f, 0.f};
    int pb[7];
#pragma unroll
    for (int t = 0; t < 7; ++t) pb[t] = (2 * wave * kFPW + 2 * (t * 16 + fi)) * 3;
    for (int c = 0; c < kXK / 32; ++c) {
      // lane (fi, fq): taps 32 c + 8 fq + e, e = 0..7, of output channel a * 16 + fi
      // (first operand) and of pixel t * 16 + fi (second operand)
      const int k0 = 32 * c + 8 * fq;
      bf16x8 wh[4], wm[4], wl[4];
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const uint16_t* q = wp3 + (a * 16 + fi) * kXK + k0;
        wh[a] = *reinterpret_cast<const bf16x8*>(q);
        wm[a] = *reinterpret_cast<const bf16x8*>(q + kXPlane);
        wl[a] = *reinterpret_cast<const bf16x8*>(q + 2 * kXPlane);
      }
      int ko[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) ko[e] = tap_off(k0 + e);
#pragma unroll
      for (int t = 0; t < 7; ++t) {
        f32x4 x0, x1;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          x0[e] = band[pb[t] + ko[e]];
          x1[e] = band[pb[t] + ko[4 + e]];
        }
        bf16x8 xh, xm, xl;
        split3x8(x0, x1, xh, xm, xl);
#pragma unroll
        for (int a = 0; a < 4; ++a) {
          f32x4 cc = acc[t][a];
          cc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wl[a], xh, cc, 0, 0, 0);
          cc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh[a], xl, cc, 0, 0, 0);
          cc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wm[a], xm, cc, 0, 0, 0);
          cc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wm[a], xh, cc, 0, 0, 0);
          cc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh[a], xm, cc, 0, 0, 0);
          acc[t][a] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh[a], xh, cc, 0, 0, 0);
        }
      }
    }
    // lane: channels a * 16 + 4 fq + r of pixel t * 16 + fi of output row orow0 + wave
    const int orow = orow0 + wave;
#pragma unroll
    for (int t = 0; t < 7; ++t) {
      const int ocol = t * 16 + fi;
      float* yp = y + (((int64_t)n * g.OH + orow) * g.OW + ocol) * 64;
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const f32x4 v = acc[t][a];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          ssum[a][r] += v[r];
          ssq[a][r] = fmaf(v[r], v[r], ssq[a][r]);
        }
        *reinterpret_cast<f32x4*>(yp + a * 16 + 4 * fq) = v;
      }
    }
  }
  if (stats) {
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) {
          ssum[a][r] += __shfl_xor(ssum[a][r], off, 64);
          ssq[a][r] += __shfl_xor(ssq[a][r], off, 64);
        }
    __syncthreads();
    float* red = fl;   // [sum | sq][wave][64]
    if (fi == 0) {
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          red[wave * 64 + a * 16 + 4 * fq + r] = ssum[a][r];
          red[(4 + wave) * 64 + a * 16 + 4 * fq + r] = ssq[a][r];
        }
    }
    __syncthreads();
    if (threadIdx.x < 64) {
      float sa = 0.f, sb = 0.f;
#pragma unroll
      for (int w2 = 0; w2 < 4; ++w2) {
        sa += red[w2 * 64 + threadIdx.x];
        sb += red[(4 + w2) * 64 + threadIdx.x];
      }
      stats[(int64_t)blockIdx.x * 64 + threadIdx.x] = sa;
      stats[stats_ld + (int64_t)blockIdx.x * 64 + threadIdx.x] = sb;
    }
  }
}

// bf16x6 grad-weight: the contraction over pixels runs 32 at a time on
// v_mfma_f32_16x16x32_bf16.  Lane (fi, fq) holds pixels 32 s + 8 fq .. + 7 of
// its wave's output row: dY of channel a * 16 + fi (straight from global, as
// the fp32 kernel) and the band values of tap ks * 16 + fi, each split once
// into three exact bf16 parts; six part products per (a, ks) subtile, smallest
// first.  112 pixels = three full steps and a half step (lanes fq >= 2 hold
// zeros).  The next step's dY loads are issued before this step's MFMAs and
// the next band's loads before this band's (double-buffered band in LDS).  Same band walk, accumulator layout and per-block partials as
// stem_f32_wgrad_kernel (stem_f32_wgrad_reduce sums them).
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1)))
stem_f32x6_wgrad_kernel(const float* __restrict__ x, const float* __restrict__ dy, float* __restrict__ part,
                        StemF32Geo g) {
  extern __shared__ __attribute__((aligned(16))) float fl[];
  // two band buffers (the next band is loaded into registers during this
  // band's MFMAs and stored to the other buffer after them); buffer 0 is also
  // the cross-wave reduction area [64][160]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fi = lane & 15, fq = lane >> 4;
  int ko[kFKS];
#pragma unroll
  for (int ks = 0; ks < kFKS; ++ks) ko[ks] = tap_off(ks * 16 + fi);   // taps >= 147: gradient dropped
  f32x4 acc[4][kFKS];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int ks = 0; ks < kFKS; ++ks) acc[a][ks] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int bpi = g.OH / kFR;
  constexpr int kSteps = (kFOW + 31) / 32;
  constexpr int RV = 2 * kFOW * 3 / 4;               // float4 per input row
  constexpr int RW = kFPW * 3;                       // floats per band row
  constexpr int kBandV = kFIn * RV;
  constexpr int kBandPer = (kBandV + 255) / 256;
  // the zero borders of both buffers, once
  for (int i = threadIdx.x; i < 2 * kFIn * 18; i += blockDim.x) {
    const int bf = i / (kFIn * 18), q = i - bf * (kFIn * 18);
    const int rr = q / 18, j = q - rr * 18;
    fl[bf * kFBand + rr * RW + (j < 9 ? j : RW - 18 + j)] = 0.f;
  }
  float4 bv[kBandPer];
  auto fetch_band = [&](int bb) __attribute__((always_inline)) {
    const int n = bb / bpi, ih0 = 2 * ((bb - n * bpi) * kFR) - 3;
#pragma unroll
    for (int j = 0; j < kBandPer; ++j) {
      const int i = threadIdx.x + 256 * j;
      const int rr = i / RV, jj = i - rr * RV;
      const int ih = ih0 + rr;
      bv[j] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (i < kBandV && (unsigned)ih < (unsigned)g.H)
        bv[j] = reinterpret_cast<const float4*>(x + ((int64_t)n * g.H + ih) * g.W * 3)[jj];
    }
  };
  auto store_band = [&](float* band) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < kBandPer; ++j) {
      const int i = threadIdx.x + 256 * j;
      if (i < kBandV) {
        const int rr = i / RV, jj = i - rr * RV;
        float* d = band + rr * RW + 9 + 4 * jj;
        d[0] = bv[j].x; d[1] = bv[j].y; d[2] = bv[j].z; d[3] = bv[j].w;
      }
    }
  };
  // dY of the NEXT pixel step is loaded while this step's MFMAs run (the
  // global round trip would otherwise stall every step)
  float dn[4][8];
  auto load_dy = [&](int bb, int s) __attribute__((always_inline)) {
    const int n = bb / bpi, orow = (bb - n * bpi) * kFR + wave;
    const float* dyr = dy + (((int64_t)n * g.OH + orow) * g.OW) * 64;
    const int px = 32 * s + 8 * fq;
    const int pxc = px < kFOW ? px : 0;              // dead lanes read valid addresses (zeroed at use)
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int e = 0; e < 8; ++e) dn[a][e] = dyr[(int64_t)(pxc + e) * 64 + a * 16 + fi];
  };
  int cur = 0;
  if (blockIdx.x < g.nbands) {
    load_dy(blockIdx.x, 0);
    fetch_band(blockIdx.x);
    store_band(fl);
  }
  __syncthreads();
  for (int b = blockIdx.x; b < g.nbands; b += gridDim.x) {
    const int bnext = b + (int)gridDim.x;
    if (bnext < g.nbands) fetch_band(bnext);
    const float* band = fl + cur * kFBand;
    for (int s = 0; s < kSteps; ++s) {
      const int px = 32 * s + 8 * fq;
      const bool live = px < kFOW;                   // kFOW % 8 == 0: a lane's 8 pixels are all in or all out
      const int pxc = live ? px : 0;
      bf16x8 gh[4], gm[4], gl[4];
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        f32x4 d0, d1;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          d0[e] = live ? dn[a][e] : 0.f;
          d1[e] = live ? dn[a][4 + e] : 0.f;
        }
        split3x8(d0, d1, gh[a], gm[a], gl[a]);
      }
      if (s + 1 < kSteps) load_dy(b, s + 1);
      else if (bnext < g.nbands) load_dy(bnext, 0);
      const int pb = (2 * wave * kFPW + 2 * pxc) * 3;
      // band operand of tap subtile ks (dead lanes read valid band values:
      // their dY parts are zero, so the products vanish)
      auto rd = [&](int ks, float (&xv)[8]) __attribute__((always_inline)) {
#pragma unroll
        for (int e = 0; e < 8; ++e) xv[e] = band[pb + 6 * e + ko[ks]];
      };
      // one wave per SIMD issues in order, so a VALU run behind an MFMA run
      // waits for the matrix pipe: the split of subtile ks + 1 is cut into 20
      // one-to-two-instruction stages placed between the 24 MFMAs of subtile ks
      // (sched_barrier fixes the order), and the band values of ks + 2 are read
      // meanwhile (a whole subtile of LDS latency)
      float xr[2][8];
      uint32_t sh[4], sm[4], sl[4];
      float s1[8], s2[8];
      auto split_stage = [&](const float (&xv)[8], int j) __attribute__((always_inline)) {
        const int p = j / 5, stg = j % 5;
        if (stg == 0) {
          sh[p] = pack_bf16x2(xv[2 * p], xv[2 * p + 1]);
        } else if (stg == 1) {
          s1[2 * p] = xv[2 * p] - __uint_as_float(sh[p] << 16);
          s1[2 * p + 1] = xv[2 * p + 1] - __uint_as_float(sh[p] & 0xffff0000u);
        } else if (stg == 2) {
          sm[p] = pack_bf16x2(s1[2 * p], s1[2 * p + 1]);
        } else if (stg == 3) {
          s2[2 * p] = s1[2 * p] - __uint_as_float(sm[p] << 16);
          s2[2 * p + 1] = s1[2 * p + 1] - __uint_as_float(sm[p] & 0xffff0000u);
        } else {
          sl[p] = pack_bf16x2(s2[2 * p], s2[2 * p + 1]);
        }
      };
      auto planes = [&](bf16x8& h, bf16x8& m, bf16x8& l) __attribute__((always_inline)) {
        h = __builtin_bit_cast(bf16x8, u32x4{sh[0], sh[1], sh[2], sh[3]});
        m = __builtin_bit_cast(bf16x8, u32x4{sm[0], sm[1], sm[2], sm[3]});
        l = __builtin_bit_cast(bf16x8, u32x4{sl[0], sl[1], sl[2], sl[3]});
      };
      rd(0, xr[0]);
      rd(1, xr[1]);
      bf16x8 xh, xm, xl;
#pragma unroll
      for (int j = 0; j < 20; ++j) split_stage(xr[0], j);
      planes(xh, xm, xl);
#pragma unroll
      for (int ks = 0; ks < kFKS; ++ks) {
        const int nx = (ks + 1) & 1;                 // buffer of subtile ks + 1
        if (ks + 2 < kFKS) rd(ks + 2, xr[ks & 1]);   // subtile ks's buffer is free: its split is done
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 24; ++i) {
          const int a = i / 6, t = i % 6;
          const bf16x8 ga = t == 0 ? gl[a] : (t == 1 || t == 5 || t == 4 ? gh[a] : gm[a]);
          const bf16x8 xb = t == 0 ? xh : (t == 1 ? xl : (t == 2 || t == 4 ? xm : xh));
          acc[a][ks] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ga, xb, acc[a][ks], 0, 0, 0);
          if (ks + 1 < kFKS && i >= 2 && i < 22) split_stage(xr[nx], i - 2);
          __builtin_amdgcn_sched_barrier(0);
        }
        if (ks + 1 < kFKS) planes(xh, xm, xl);
      }
    }
    // the other buffer was last read before the previous barrier
    if (bnext < g.nbands) store_band(fl + (cur ^ 1) * kFBand);
    __syncthreads();
    cur ^= 1;
  }
  // lane: dW[n = a * 16 + 4 fq + r][k = ks * 16 + fi]; sum the 4 waves in order through LDS
  float* red = fl;
  for (int w2 = 0; w2 < 4; ++w2) {
    __syncthreads();
    if (wave == w2) {
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int ks = 0; ks < kFKS; ++ks)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float* p = red + (a * 16 + 4 * fq + r) * 160 + ks * 16 + fi;
            *p = (w2 == 0 ? 0.f : *p) + acc[a][ks][r];
          }
    }
  }
  __syncthreads();
  float* dst = part + (int64_t)blockIdx.x * 64 * kFKP;
  for (int i = threadIdx.x; i < 64 * kFKP; i += blockDim.x) {
    const int nn = i / kFKP, k = i - nn * kFKP;
    dst[i] = red[nn * 160 + k];
  }
}

// out[n][c][kh][kw] (strided fp32, the (arena) gradient) += sum over blocks.
// A workgroup owns 16 consecutive outputs of the padded [64][148] partial
// rows; its 16 lane groups each sum every 16th block (independent loads in
// flight instead of one serial chain of `blocks` loads per output: 130 us ->
// a few us at bs512), then lane group 0 adds the 16 group sums in order --
// a fixed order, so the result is deterministic.
constexpr int kRedOut = 16, kRedSplit = 16;
__global__ void __launch_bounds__(256) stem_f32_wgrad_reduce_kernel(const float* __restrict__ part, int blocks,
                                                                    float* __restrict__ out, int64_t s0, int64_t s1,
                                                                    int64_t s2, int64_t s3) {
  __shared__ float sh[kRedSplit][kRedOut];
  const int ol = threadIdx.x % kRedOut, sp = threadIdx.x / kRedOut;
  const int o = blockIdx.x * kRedOut + ol;          // < 64 * kFKP (grid covers it exactly)
  float acc = 0.f;
#pragma unroll 8
  for (int b = sp; b < blocks; b += kRedSplit) acc += part[(int64_t)b * 64 * kFKP + o];
  sh[sp][ol] = acc;
  __syncthreads();
  if (sp == 0) {
    float t = 0.f;
#pragma unroll
    for (int j = 0; j < kRedSplit; ++j) t += sh[j][ol];
    const int n = o / kFKP, k = o - n * kFKP;
    if (k < kFK) {
      const int kh = k / 21, r = k - kh * 21, kw = r / 3, c = r - kw * 3;
      out[n * s0 + c * s1 + kh * s2 + kw * s3] += t;
    }
  }
}
static_assert((64 * kFKP) % kRedOut == 0, "reduce grid covers the partial rows exactly");

constexpr int kFFwdLds = (kFBand + kFWg) * 4;
constexpr int kFWgLds = (kFBand > 64 * 160 ? kFBand : 64 * 160) * 4;
constexpr int kFWg6Lds = (2 * kFBand > 64 * 160 ? 2 * kFBand : 64 * 160) * 4;

}  // namespace

bool stem_f32_supported(int H, int W) { return H == 224 && W == 224; }

int stem_f32_wgrad_blocks(int N) { return N * (kFOW / kFR) < 512 ? N * (kFOW / kFR) : 512; }

int stem_f32_forward(const float* x, int N, int H, int W, const float* w, int64_t s0, int64_t s1, int64_t s2,
                     int64_t s3, float* y, float* stats, int stats_rows, hipStream_t stream) {
  StemF32Geo g{N, H, W, kFOW, kFOW, N * (kFOW / kFR)};
  int grid = g.nbands < 512 ? g.nbands : 512;
  if (stats && grid > stats_rows) grid = stats_rows;
  static bool attr = [] {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&stem_f32_fwd_kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, kFFwdLds) == hipSuccess;
  }();
  (void)attr;
  hipLaunchKernelGGL(stem_f32_fwd_kernel, dim3((unsigned)grid), dim3(256), kFFwdLds, stream, x, w, s0, s1, s2, s3, y, g,
                     stats, (int64_t)stats_rows * 64);
  return grid;
}

int stem_f32x6_wplanes() { return 3 * kXPlane; }

int stem_f32x6_forward(const float* x, int N, int H, int W, const float* w, int64_t s0, int64_t s1, int64_t s2,
                       int64_t s3, uint16_t* wp3, float* y, float* stats, int stats_rows, hipStream_t stream) {
  StemF32Geo g{N, H, W, kFOW, kFOW, N * (kFOW / kFR)};
  int grid = g.nbands < 512 ? g.nbands : 512;
  if (stats && grid > stats_rows) grid = stats_rows;
  constexpr int lds = kFBand * 4;
  hipLaunchKernelGGL(stem_w_split3_kernel, dim3((kXPlane + 255) / 256), dim3(256), 0, stream, w, s0, s1, s2, s3, wp3);
  static const int occ = [] {
    const char* e = getenv("GKSGD_STEM_X6_OCC");
    return (e != nullptr && e[0] == '1') ? 1 : 2;
  }();
  if (occ == 2)
    hipLaunchKernelGGL(stem_f32x6_fwd_kernel<2>, dim3((unsigned)grid), dim3(256), lds, stream, x, wp3, y, g, stats,
                       (int64_t)stats_rows * 64);
  else
    hipLaunchKernelGGL(stem_f32x6_fwd_kernel<1>, dim3((unsigned)grid), dim3(256), lds, stream, x, wp3, y, g, stats,
                       (int64_t)stats_rows * 64);
  return grid;
}

void stem_f32_wgrad(const float* x, const float* dy, int N, int H, int W, float* part, float* out, int64_t s0,
                    int64_t s1, int64_t s2, int64_t s3, bool x6, hipStream_t stream) {
  StemF32Geo g{N, H, W, kFOW, kFOW, N * (kFOW / kFR)};
  const int grid = stem_f32_wgrad_blocks(N);
  static bool attr = [] {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&stem_f32_wgrad_kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, kFWgLds) == hipSuccess;
  }();
  (void)attr;
  // bf16x6: one wave per SIMD (the prefetched dY and next band live in
  // registers beside the 160 accumulators)
  static bool attr6 = [] {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&stem_f32x6_wgrad_kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, kFWg6Lds) == hipSuccess;
  }();
  (void)attr6;
  if (x6)
    hipLaunchKernelGGL(stem_f32x6_wgrad_kernel, dim3((unsigned)grid), dim3(256), kFWg6Lds, stream, x, dy, part, g);
  else
    hipLaunchKernelGGL(stem_f32_wgrad_kernel, dim3((unsigned)grid), dim3(256), kFWgLds, stream, x, dy, part, g);
  hipLaunchKernelGGL(stem_f32_wgrad_reduce_kernel, dim3(64 * kFKP / kRedOut), dim3(256), 0, stream, part, grid, out,
                     s0, s1, s2, s3);
}

}  // namespace gk
