// The ImageNet-ResNet stem convolution (7x7, stride 2, padding 3, 3 -> 64
// channels) on gfx950: forward with the BatchNorm statistics in the epilogue,
// and grad-weight.  MIOpen runs it at ~0.7 ms per direction at bs512
// (profiles/r01_resnet50_conv_roofline_bs512.txt: 16-19 % of roofline) -- the
// 3-channel input defeats its implicit-GEMM tiling.
//
// Both kernels walk "bands" of kSR output rows of one image.  The band's input
// rows are staged once in LDS as bf16 pixels of 4 channels (the 4th zero), the
// image's zero padding materialised, converting from the fp32 (or bf16) NHWC
// batch on the fly (no separate cast pass).  The GEMM K dimension is packed as
// kh * 32 + kw * 4 + c (kw < 8, c < 4; the kw = 7 / c = 3 slots multiply zero
// weights), so one 16x16x32 MFMA k-step is one filter row kh and a lane's 8
// k-values are two adjacent input pixels -- one aligned ds_read_b128 (LDS
// pixel j = input column + 3 makes 2*ow + 2*q even).
//
// forward : 7 waves; each 64-pixel output tile is 4x4 MFMA 16x16 subtiles x 7
//           k-steps against the packed weights resident in LDS; the epilogue is
//           gemm.hip's (8 channels per lane per 16-byte store) plus per-block
//           BatchNorm partials of the stored bf16 values.
// wgrad   : 7 waves, wave w owns filter row kh = w (two 16-wide k tiles) x 64
//           output channels; the band's output gradient is staged [pixel][64]
//           with the transposed-read swizzle and read as dY^T fragments
//           (ds_read_b64_tr_b16), the input patches as 8 strided bf16 per
//           fragment.  Per-block partials [blocks][64 * 224] are summed in a
//           fixed order by stem_wgrad_reduce_kernel (deterministic, no atomics)
//           and added into the (arena) gradient.
#include <hip/hip_runtime.h>

#include "common.h"
#include "gk_kernels.h"
#include "mfma_util.h"

namespace gk {
namespace {

constexpr int kSR = 8;               // output rows per band
constexpr int kSRows = 2 * kSR + 5;  // input rows per band
constexpr int kSK = 224;             // packed K
constexpr int kSKP = 232;            // LDS pitch of a packed weight row (conflict-free b128 reads)
constexpr int kFwdWaves = 7;        // 14 64-pixel tiles per 8 x 112 band: 2 per wave
constexpr int kWgWaves = 7;
constexpr int kDyB = 16;             // wgrad: staged 16-byte dy chunks per thread per band

struct StemGeo {
  int N, H, W, OH, OW;
  int WL;       // LDS band row length in pixels (>= 2*OW + 6, even)
  int nbands;   // bands per image
};

__device__ __forceinline__ uint16_t bf16_of(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x7fffffu)) return (uint16_t)((u >> 16) | 0x40);  // NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
__device__ __forceinline__ uint16_t ld_bf16(const float* p) { return bf16_of(*p); }
__device__ __forceinline__ uint16_t ld_bf16(const uint16_t* p) { return *p; }

// one input pixel's 3 channels, loaded with one 12-byte (fp32) / 6-byte access
template <typename T>
struct Px3 { T c0, c1, c2; };

__device__ __forceinline__ uint2 to_lds(const Px3<float>& v) {
  return make_uint2(pack_bf16x2(v.c0, v.c1), pack_bf16x2(v.c2, 0.f));
}
__device__ __forceinline__ uint2 to_lds(const Px3<uint16_t>& v) {
  return make_uint2((uint32_t)v.c0 | ((uint32_t)v.c1 << 16), (uint32_t)v.c2);
}

// Band staging, split into a register phase and an LDS phase so the next band's
// loads can be in flight while the current band is multiplied: input rows
// 2*oh0-3 .. of image n -> band[i * WL + j] = 4 bf16 (c0, c1, c2, 0) of input
// pixel (2*oh0 - 3 + i, j - 3), zeros outside the image.  Thread t stages band
// pixels t, t + T, t + 2T, ... (T threads); its (row, column) advance by a fixed
// (T / WL, T % WL) step, so no division per pixel.  B pixels per call; the host
// checks kSRows * WL <= kStageB * T for the single-call (prefetch) form.
constexpr int kStageB = 12;
template <typename T, int B>
struct InputRegs {
  Px3<T> v[B];
  uint32_t in;   // bit u: pixel u inside the image
};

struct BandIter {
  int i0, j0, di, dj;   // this thread's first band pixel and the per-pixel step
  __device__ BandIter(const StemGeo& g) {
    i0 = threadIdx.x / g.WL;
    j0 = threadIdx.x - i0 * g.WL;
    di = blockDim.x / g.WL;
    dj = blockDim.x - di * g.WL;
  }
};

// pixels u = 0..B-1 of this thread starting at band pixel index `first` (row fi, column fj)
template <typename T, int B>
__device__ __forceinline__ void load_input(const T* __restrict__ x, const StemGeo& g, const BandIter& it, int n,
                                           int oh0, int fi, int fj, InputRegs<T, B>& r) {
  const T* img = x + (int64_t)n * g.H * g.W * 3;
  int i = fi, j = fj;
  r.in = 0;
#pragma unroll
  for (int u = 0; u < B; ++u) {
    const int ih = 2 * oh0 - 3 + i, iw = j - 3;
    const bool in = i < kSRows && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
    r.in |= (in ? 1u : 0u) << u;
    r.v[u] = *reinterpret_cast<const Px3<T>*>(in ? img + (ih * g.W + iw) * 3 : img);
    j += it.dj;
    i += it.di;
    if (j >= g.WL) {
      j -= g.WL;
      ++i;
    }
  }
}

template <typename T, int B>
__device__ __forceinline__ void store_input(const StemGeo& g, int first, const InputRegs<T, B>& r, uint2* band) {
  const int total = kSRows * g.WL;
#pragma unroll
  for (int u = 0; u < B; ++u) {
    const int pix = first + u * blockDim.x;
    if (pix < total) band[pix] = ((r.in >> u) & 1u) ? to_lds(r.v[u]) : make_uint2(0u, 0u);
  }
}

// synchronous staging, B loads in flight per thread per round
template <int B, typename T>
__device__ __forceinline__ void stage_input_sync(const T* __restrict__ x, const StemGeo& g, const BandIter& it, int n,
                                                 int oh0, uint2* band) {
  const int total = kSRows * g.WL;
  int fi = it.i0, fj = it.j0;
  for (int first = threadIdx.x; first < total; first += B * blockDim.x) {
    InputRegs<T, B> r;
    load_input<T, B>(x, g, it, n, oh0, fi, fj, r);
    store_input<T, B>(g, first, r, band);
#pragma unroll
    for (int u = 0; u < B; ++u) {
      fj += it.dj;
      fi += it.di;
      if (fj >= g.WL) {
        fj -= g.WL;
        ++fi;
      }
    }
  }
}

// one 7-wave block per CU (the 64 accumulators, the fragments, the BatchNorm
// partials and the next band's prefetched pixels need ~250 VGPRs)
template <typename T>
__global__ void __launch_bounds__(64 * kFwdWaves)
stem_fwd_kernel(const T* __restrict__ x, const uint16_t* __restrict__ wp, uint16_t* __restrict__ y,
                float* __restrict__ stats, int64_t stats_ld, StemGeo g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* wl = smem;                                             // [64][kSKP] bf16
  uint2* bands = reinterpret_cast<uint2*>(smem + 64 * kSKP * 2);   // two band buffers
  const int bstride = kSRows * g.WL;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const bool odd = fq & 1;
  for (int i = threadIdx.x; i < 64 * (kSK / 8); i += blockDim.x) {
    const int nn = i / (kSK / 8), q = i - nn * (kSK / 8);
    *reinterpret_cast<uint4*>(wl + (nn * kSKP + q * 8) * 2) = *reinterpret_cast<const uint4*>(wp + nn * kSK + q * 8);
  }
  float ssum[4][4], ssq[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) ssum[a][b] = ssq[a][b] = 0.f;
  const int64_t total = (int64_t)g.N * g.nbands;
  const int ppb = kSR * g.OW;
  const int mtiles = (ppb + 63) / 64;
  const BandIter it(g);
  InputRegs<T, kStageB> pre;
  if (blockIdx.x < total) {
    const int n = (int)(blockIdx.x / g.nbands);
    load_input<T, kStageB>(x, g, it, n, (int)(blockIdx.x - (int64_t)n * g.nbands) * kSR, it.i0, it.j0, pre);
  }
  int cur = 0;
  for (int64_t bi = blockIdx.x; bi < total; bi += gridDim.x) {
    const int n = (int)(bi / g.nbands);
    const int oh0 = (int)(bi - (int64_t)n * g.nbands) * kSR;
    uint2* band = bands + cur * bstride;
    store_input<T, kStageB>(g, threadIdx.x, pre, band);   // buffer `cur` was last read two bands ago
    __syncthreads();
    const int64_t nb = bi + gridDim.x;
    if (nb < total) {            // next band's loads in flight during this band's MFMAs
      const int n2 = (int)(nb / g.nbands);
      load_input<T, kStageB>(x, g, it, n2, (int)(nb - (int64_t)n2 * g.nbands) * kSR, it.i0, it.j0, pre);
    }
    cur ^= 1;
    for (int mt = wave; mt < mtiles; mt += kFwdWaves) {
      int aoff[4];
      int64_t orow[4];
      bool ok[4];
#pragma unroll
      for (int ms = 0; ms < 4; ++ms) {
        const int p = mt * 64 + ms * 16 + fr;
        int r = p / g.OW, ow = p - r * g.OW;
        ok[ms] = p < ppb && oh0 + r < g.OH;
        if (!ok[ms]) r = ow = 0;
        aoff[ms] = ((2 * r) * g.WL + 2 * ow + 2 * fq) * 8;
        orow[ms] = ((int64_t)n * g.OH + oh0 + r) * g.OW + ow;
      }
      f32x4 acc[4][4];
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
      // not unrolled: fully unrolled, the compiler hoists all 7 k-steps' LDS reads
      // (224 VGPRs) and spills; the second wave per SIMD covers the read latency
#pragma unroll 1
      for (int kh = 0; kh < 7; ++kh) {
        bf16x8 av[4], bv[4];
#pragma unroll
        for (int ms = 0; ms < 4; ++ms)
          av[ms] = *reinterpret_cast<const bf16x8*>(reinterpret_cast<const char*>(band) + aoff[ms] + kh * g.WL * 8);
#pragma unroll
        for (int ns = 0; ns < 4; ++ns)
          bv[ns] = *reinterpret_cast<const bf16x8*>(wl + ((ns * 16 + fr) * kSKP + kh * 32 + fq * 8) * 2);
#pragma unroll
        for (int ms = 0; ms < 4; ++ms)
#pragma unroll
          for (int ns = 0; ns < 4; ++ns)
            acc[ms][ns] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bv[ns], av[ms], acc[ms][ns], 0, 0, 0);
      }
      // lane holds C[pixel fr][channel 16 ns + 4 fq + r]; lanes fq, fq^1 swap halves
      // of the subtile pair so each lane stores 8 consecutive channels (gemm.hip)
#pragma unroll
      for (int ms = 0; ms < 4; ++ms) {
#pragma unroll
        for (int pr = 0; pr < 2; ++pr) {
          const f32x4 va = acc[ms][2 * pr], vb = acc[ms][2 * pr + 1];
          const uint32_t a0 = pack_bf16x2(va[0], va[1]), a1 = pack_bf16x2(va[2], va[3]);
          const uint32_t b0 = pack_bf16x2(vb[0], vb[1]), b1 = pack_bf16x2(vb[2], vb[3]);
          if (stats && ok[ms]) {
            const uint32_t pk[4] = {a0, a1, b0, b1};
#pragma unroll
            for (int h = 0; h < 4; ++h) {
              const float lo = __uint_as_float(pk[h] << 16), hi = __uint_as_float(pk[h] & 0xffff0000u);
              const int nsx = 2 * pr + (h >> 1), rr = (h & 1) * 2;
              ssum[nsx][rr] += lo;
              ssq[nsx][rr] = fmaf(lo, lo, ssq[nsx][rr]);
              ssum[nsx][rr + 1] += hi;
              ssq[nsx][rr + 1] = fmaf(hi, hi, ssq[nsx][rr + 1]);
            }
          }
          const uint32_t r0 = (uint32_t)__shfl_xor((int)(odd ? a0 : b0), 16, 64);
          const uint32_t r1 = (uint32_t)__shfl_xor((int)(odd ? a1 : b1), 16, 64);
          const uint4 v = odd ? make_uint4(r0, r1, b0, b1) : make_uint4(a0, a1, r0, r1);
          const int ch = pr * 32 + (odd ? 16 + 4 * (fq - 1) : 4 * fq);
          if (ok[ms]) *reinterpret_cast<uint4*>(y + orow[ms] * 64 + ch) = v;
        }
      }
    }
  }
  if (stats) {
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) {
          ssum[a][b] += __shfl_xor(ssum[a][b], off, 64);
          ssq[a][b] += __shfl_xor(ssq[a][b], off, 64);
        }
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);   // [2][kFwdWaves][64] (the weights are no longer read)
    if (fr == 0) {
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int col = a * 16 + fq * 4 + b;
          red[wave * 64 + col] = ssum[a][b];
          red[(kFwdWaves + wave) * 64 + col] = ssq[a][b];
        }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < 64; c += blockDim.x) {
      float sa = 0.f, sb = 0.f;
#pragma unroll
      for (int w = 0; w < kFwdWaves; ++w) {
        sa += red[w * 64 + c];
        sb += red[(kFwdWaves + w) * 64 + c];
      }
      stats[(int64_t)blockIdx.x * 64 + c] = sa;
      stats[stats_ld + (int64_t)blockIdx.x * 64 + c] = sb;
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(64 * kWgWaves)
stem_wgrad_kernel(const T* __restrict__ x, const uint16_t* __restrict__ dy, float* __restrict__ part, StemGeo g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int ppb = kSR * g.OW;                                   // multiple of 32 (host check)
  char* dyt = smem;                                             // [ppb][128 B]
  uint2* band = reinterpret_cast<uint2*>(smem + ppb * 128);
  const uint16_t* bandh = reinterpret_cast<const uint16_t*>(band);
  const int lane = threadIdx.x & 63, kh = threadIdx.x >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  f32x4 acc[4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a) acc[a][0] = acc[a][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  // this lane's k column per k tile: k = 32 kh + 16 kt + fr -> (kw, c)
  int kcol[2];
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    const int kq = 16 * kt + fr;
    kcol[kt] = (kq >> 2) * 4 + (kq & 3);   // LDS element offset of tap kw, channel c within a pixel row
  }
  // dY^T fragment halves for rows 0..31 (a step adds 32 rows = p0 * 128 bytes;
  // the transposed-read swizzle repeats every 16 rows)
  const char* ta0[4];
  const char* ta1[4];
  {
    const int gq = lane >> 4, li = lane & 15;
    const int q = li >> 2, pp = li & 3;
    const int ra = 8 * gq + q, rb = ra + 4;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int col = nt * 16 + 4 * pp;
      ta0[nt] = dyt + ra * 128 + ((((col >> 3) ^ tr_swz<128>(ra)) << 4) | ((col & 7) << 1));
      ta1[nt] = dyt + rb * 128 + ((((col >> 3) ^ tr_swz<128>(rb)) << 4) | ((col & 7) << 1));
    }
  }
  const int64_t total = (int64_t)g.N * g.nbands;
  const BandIter it(g);
  // the band's output gradient: its pixels are contiguous in dy (rows oh0 .. of
  // image n), kDyB 16-byte chunks per thread (host check), rows past OH read 0
  // (only dy is prefetched across the MFMAs -- the input patch registers on top
  // would spill; the input rows are staged at the band start, one batch of loads)
  uint4 dv[kDyB];
  int valid = 0;
  auto load_band = [&](int64_t b) {
    const int n = (int)(b / g.nbands);
    const int oh0 = (int)(b - (int64_t)n * g.nbands) * kSR;
    const int64_t dbase = ((int64_t)n * g.OH + oh0) * g.OW * 64;
    valid = (g.OH - oh0 < kSR ? g.OH - oh0 : kSR) * g.OW * 8;
#pragma unroll
    for (int u = 0; u < kDyB; ++u) {
      const int i = u * blockDim.x + threadIdx.x;
      dv[u] = *reinterpret_cast<const uint4*>(dy + dbase + (int64_t)(i < valid ? i : 0) * 8);
    }
  };
  if (blockIdx.x < total) load_band(blockIdx.x);
  for (int64_t bi = blockIdx.x; bi < total; bi += gridDim.x) {
    const int n = (int)(bi / g.nbands);
    const int oh0 = (int)(bi - (int64_t)n * g.nbands) * kSR;
    __syncthreads();   // the previous band's fragments are read
#pragma unroll
    for (int u = 0; u < kDyB; ++u) {
      const int i = u * blockDim.x + threadIdx.x;
      if (i < ppb * 8) {
        const int p = i >> 3, ck = i & 7;
        *reinterpret_cast<uint4*>(dyt + p * 128 + ((ck ^ tr_swz<128>(p)) << 4)) =
            i < valid ? dv[u] : make_uint4(0u, 0u, 0u, 0u);
      }
    }
    stage_input_sync<6>(x, g, it, n, oh0, band);   // after the dy registers are free
    __syncthreads();
    if (bi + gridDim.x < total) load_band(bi + gridDim.x);   // in flight during the MFMAs
    // step p0 reads pixels p0 + 8 fq + 0..7: their output row / column advance
    // incrementally (OW % 8 == 0 keeps the 8 in one row)
    int pr_ = (8 * fq) / g.OW, pw = 8 * fq - ((8 * fq) / g.OW) * g.OW;
#pragma unroll 2
    for (int p0 = 0; p0 < ppb; p0 += 32) {
      bf16x8 av[4], bv[2];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((GK_LDS bf16x4*)(GK_LDS char*)(ta0[nt] + p0 * 128));
        const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((GK_LDS bf16x4*)(GK_LDS char*)(ta1[nt] + p0 * 128));
        av[nt] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
      const int base = ((2 * pr_ + kh) * g.WL + 2 * pw) * 4;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        const uint16_t* sp = bandh + base + kcol[kt];
        bf16x8 bb;
#pragma unroll
        for (int j = 0; j < 8; ++j) bb[j] = (short)sp[8 * j];
        bv[kt] = bb;
      }
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
          acc[nt][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[nt], bv[kt], acc[nt][kt], 0, 0, 0);
      pw += 32;
      while (pw >= g.OW) {
        pw -= g.OW;
        ++pr_;
      }
    }
  }
  // lane holds D[channel 16 nt + 4 fq + r][k = 32 kh + 16 kt + fr]
  float* out = part + (int64_t)blockIdx.x * 64 * kSK;
#pragma unroll
  for (int nt = 0; nt < 4; ++nt)
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) out[(nt * 16 + 4 * fq + r) * kSK + 32 * kh + 16 * kt + fr] = acc[nt][kt][r];
}

// out[n][c][kh][kw] (element strides so) += sum over blocks of part[b][n][kh*32 + kw*4 + c]
__global__ void __launch_bounds__(256) stem_wgrad_reduce_kernel(const float* __restrict__ part, int blocks,
                                                                float* __restrict__ out, int64_t s0, int64_t s1,
                                                                int64_t s2, int64_t s3) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 64 * 147) return;
  const int n = i / 147, rem = i - n * 147;
  const int c = rem / 49, t = rem - c * 49;
  const int kh = t / 7, kw = t - kh * 7;
  const int k = kh * 32 + kw * 4 + c;
  float s = 0.f;
  for (int b = 0; b < blocks; ++b) s += part[(int64_t)b * 64 * kSK + n * kSK + k];
  out[n * s0 + c * s1 + kh * s2 + kw * s3] += s;
}

// [64][3][7][7] weights (element strides) -> packed bf16 [64][224]
__global__ void __launch_bounds__(256) stem_pack_kernel(const float* __restrict__ w, int64_t s0, int64_t s1,
                                                        int64_t s2, int64_t s3, uint16_t* __restrict__ wp) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 64 * kSK) return;
  const int n = i / kSK, k = i - n * kSK;
  const int kh = k >> 5, kw = (k >> 2) & 7, c = k & 3;
  wp[i] = (kw < 7 && c < 3) ? bf16_of(w[n * s0 + c * s1 + kh * s2 + kw * s3]) : (uint16_t)0;
}

StemGeo stem_geo(int N, int H, int W) {
  StemGeo g;
  g.N = N;
  g.H = H;
  g.W = W;
  g.OH = (H + 6 - 7) / 2 + 1;
  g.OW = (W + 6 - 7) / 2 + 1;
  g.WL = (2 * g.OW + 6 + 1) & ~1;
  g.nbands = (g.OH + kSR - 1) / kSR;
  return g;
}

int lds_fwd(const StemGeo& g) { return 64 * kSKP * 2 + 2 * kSRows * g.WL * 8; }
int lds_wgrad(const StemGeo& g) { return kSR * g.OW * 128 + kSRows * g.WL * 8; }

}  // namespace

bool stem_supported(int H, int W) {
  const StemGeo g = stem_geo(1, H, W);
  return H >= 8 && W >= 8 && g.OW % 8 == 0 && lds_fwd(g) <= 160 * 1024 && lds_wgrad(g) <= 160 * 1024 &&
         kSRows * g.WL <= kStageB * 64 * kFwdWaves && kSR * g.OW * 8 <= kDyB * 64 * kWgWaves;
}

void stem_pack_weight(const float* w, int64_t s0, int64_t s1, int64_t s2, int64_t s3, uint16_t* wp,
                      hipStream_t stream) {
  hipLaunchKernelGGL(stem_pack_kernel, dim3((64 * kSK + 255) / 256), dim3(256), 0, stream, w, s0, s1, s2, s3, wp);
}

int stem_forward(const void* x, bool x_f32, int N, int H, int W, const uint16_t* wp, uint16_t* y, float* stats,
                 int stats_rows, hipStream_t stream) {
  const StemGeo g = stem_geo(N, H, W);
  const int64_t total = (int64_t)N * g.nbands;
  int64_t gx = 256;
  if (gx > total) gx = total;
  if (stats && gx > stats_rows) gx = stats_rows;
  const int lds = lds_fwd(g);
  const int64_t ld = (int64_t)stats_rows * 64;
  if (x_f32) {
    static bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&stem_fwd_kernel<float>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
    (void)attr;
    hipLaunchKernelGGL(stem_fwd_kernel<float>, dim3((unsigned)gx), dim3(64 * kFwdWaves), lds, stream,
                       static_cast<const float*>(x), wp, y, stats, ld, g);
  } else {
    static bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&stem_fwd_kernel<uint16_t>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
    (void)attr;
    hipLaunchKernelGGL(stem_fwd_kernel<uint16_t>, dim3((unsigned)gx), dim3(64 * kFwdWaves), lds, stream,
                       static_cast<const uint16_t*>(x), wp, y, stats, ld, g);
  }
  return (int)gx;
}

int stem_wgrad_blocks(int N, int H, int W) {
  const StemGeo g = stem_geo(N, H, W);
  const int64_t total = (int64_t)N * g.nbands;
  return (int)(total < 256 ? total : 256);
}

void stem_wgrad(const void* x, bool x_f32, int N, int H, int W, const uint16_t* dy, float* part, float* out,
                int64_t s0, int64_t s1, int64_t s2, int64_t s3, hipStream_t stream) {
  const StemGeo g = stem_geo(N, H, W);
  const int gx = stem_wgrad_blocks(N, H, W);
  const int lds = lds_wgrad(g);
  if (x_f32) {
    static bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&stem_wgrad_kernel<float>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
    (void)attr;
    hipLaunchKernelGGL(stem_wgrad_kernel<float>, dim3(gx), dim3(64 * kWgWaves), lds, stream,
                       static_cast<const float*>(x), dy, part, g);
  } else {
    static bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&stem_wgrad_kernel<uint16_t>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
    (void)attr;
    hipLaunchKernelGGL(stem_wgrad_kernel<uint16_t>, dim3(gx), dim3(64 * kWgWaves), lds, stream,
                       static_cast<const uint16_t*>(x), dy, part, g);
  }
  hipLaunchKernelGGL(stem_wgrad_reduce_kernel, dim3((64 * 147 + 255) / 256), dim3(256), 0, stream, part, gx, out, s0,
                     s1, s2, s3);
}

}  // namespace gk
