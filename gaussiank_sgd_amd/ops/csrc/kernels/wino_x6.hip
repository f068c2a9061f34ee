// Winograd F(2x2, 3x3), stride 1, pad 1, fp32-accurate on bf16 MFMAs ("bf16x6")
// for gfx950.
//
// winograd.hip runs the 16 element-wise GEMMs M[xi] = V[xi] U[xi] on the fp32
// MFMA (v_mfma_f32_16x16x4_f32: 1024 MACs per 32 cycles per SIMD).  Here every
// fp32 operand is split exactly into three bf16 parts (split3x8, mfma_util.h)
// and the six part products of order <= 2 are accumulated in fp32 on
// v_mfma_f32_16x16x32_bf16 (8192 MACs per 16 cycles): 6 x 16 cycles per 8192
// MACs against 8 x 32 -- 2.7x the fp32 MFMA rate, with the same error class
// as the other bf16x6 kernels (tests vs fp64 and vs the fp32-MFMA Winograd).
// The transforms are unchanged fp32 VALU arithmetic.
//
// Why a new kernel and not the fp32 one with another MFMA: a 32-deep bf16 K
// step needs 32 input channels per stage, and with 16 xi, 3 planes of 2 bytes
// per value, a stage of V (64 tiles) and U (64 output channels) is 384 KiB --
// beyond the 160 KiB of LDS.  So V never goes through LDS: the B operand of
// the MFMA (lane (t, q): tile t, channels 8q .. 8q + 7) is exactly what one
// lane transforms from its own tile's 4x4 patch, so each lane loads its patch
// (16 pixels x 8 channels: 32 x 16-byte loads), forms t = B^T d in registers
// and, per xi, V = t B, splits it and feeds the MFMAs directly.  Only U is
// staged in LDS: pre-transformed and pre-split per step ([C/32][16][3][Co][32]
// bf16, 16-byte chunks swizzled by row), half a slice (8 xi) per LDS stage by
// LDS-DMA, two stages.
//
// Block: 256 threads = 4 waves, one per SIMD; 64 tiles (16 per wave) x 32
// output channels (two 16-row A fragments) x all 16 xi: 128 fp32 accumulators
// per lane, the output transform A^T M A is register-only.  The A operand is
// U (rows = output channels), so a lane ends with 4 consecutive channels of
// one tile: 16-byte stores.  Persistent over tile blocks (x extent a multiple
// of 8: all channel blocks of a tile block on one XCD, sharing its patches in
// L2); the next slice's patch is loaded during the current slice (two
// register sets).  Epilogues: plain, BatchNorm statistics, BN-backward dz
// (the operands of winograd.hip).
//
// (GK_WX6_PROBE_* macros: timing-only A/B builds that drop the patch loads or
// the U LDS-DMA; never defined in the extension build.)
#include <hip/hip_runtime.h>

#include "common.h"
#include "gk_kernels.h"
#include "mfma_util.h"
#include "wino_x6_common.h"

namespace gk {
namespace {

constexpr int XT = 64;                     // tiles per block (16 per wave)
constexpr int XK = 32;                     // output channels per block
constexpr int XC = 32;                     // input channels per slice (one bf16 K step)
constexpr int XROW = 64;                   // bytes of one U row (32 bf16 channels)
constexpr int XPLANE = XK * XROW;          // one (xi, plane) piece of a block: 2 KiB
constexpr int XSTAGE = 8 * 3 * XPLANE;     // half a slice: 8 xi x 3 planes = 48 KiB
constexpr int XLDS = 2 * XSTAGE;

__host__ __device__ __forceinline__ int xsw(int r) { return wx6_swz(r); }

struct X6Geo {
  int H, W, Ci, Co, TH, TW, ntiles;
  uint32_t xbytes, ybytes;
};

struct X6Bnb {
  const float* h;
  const float* dy2;
  const uint8_t* mask;
};

// the filter transform + split (wino_x6_common.h), one thread per (co, ci);
// consecutive threads take consecutive rows co
__global__ void __launch_bounds__(256) wino_x6_wt_kernel(const float* __restrict__ w, uint16_t* __restrict__ u3,
                                                         int Co, int Ci, int flip) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (int64_t)Co * Ci) return;
  wino_x6_pair(w, u3, Co, Ci, flip, (int)(idx % Co), (int)(idx / Co));
}

template <bool STATS, bool BNB>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1)))
wino_x6_kernel(const float* __restrict__ x, const uint16_t* __restrict__ u3, float* __restrict__ y, X6Geo g,
               float* __restrict__ stats, int64_t stats_ld, X6Bnb bb) {
  extern __shared__ __attribute__((aligned(16))) char xl[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fi = lane & 15, fq = lane >> 4;
  const int k0 = blockIdx.y * XK;
  const int ntb = (g.ntiles + XT - 1) / XT;
  const int nsl = g.Ci / XC;
  const int my_tb = (int)blockIdx.x < ntb ? (ntb - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  const int total = my_tb * nsl;
  const int THW = g.TH * g.TW;

  f32x4 acc[16][2];
#pragma unroll
  for (int xi = 0; xi < 16; ++xi) acc[xi][0] = acc[xi][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  float ssum[2][4], ssq[2][4];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int r = 0; r < 4; ++r) ssum[a][r] = ssq[a][r] = 0.f;

  // patch addressing: this lane's tile of a tile block, channels 8 fq .. 8 fq + 7
  // of the slice; an out-of-image pixel gets an offset past the buffer's range,
  // which the hardware turns into zero loads (winograd.hip)
  const auto xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x), (short)0, (int)g.xbytes, 0x00020000);
  uint32_t voff[16];
  auto set_tile = [&](int tb) __attribute__((always_inline)) {
    const int tt = tb * XT + wave * 16 + fi;
    const bool tv = tt < g.ntiles;
    const int ttc = tv ? tt : 0;
    const int n = ttc / THW, r = ttc - n * THW, th = r / g.TW, tw = r - th * g.TW;
    const int ih0 = 2 * th - 1, iw0 = 2 * tw - 1;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool v = tv && (unsigned)(ih0 + i) < (unsigned)g.H && (unsigned)(iw0 + j) < (unsigned)g.W;
        voff[4 * i + j] =
            v ? (uint32_t)((((int64_t)n * g.H + ih0 + i) * g.W + iw0 + j) * g.Ci + 8 * fq) * 4u : 0x80000000u;
      }
  };
  // patch rows (4 pixels x channels 0-3 / 4-7 each): row i of slice s
  typedef f32x4 Row[4][2];
  auto gload_row = [&](Row& d, int i, int s) __attribute__((always_inline)) {
    const int so = __builtin_amdgcn_readfirstlane(s * XC * 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#ifdef GK_WX6_PROBE_NOLOAD
      d[j][0] = f32x4{(float)(voff[4 * i + j] & 7), 1.f, 2.f, (float)so};
      d[j][1] = f32x4{1.f, (float)(voff[4 * i + j] & 3), 2.f, 3.f};
#else
      d[j][0] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, (int)voff[4 * i + j], so, 0));
      d[j][1] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, (int)voff[4 * i + j], so + 16, 0));
#endif
    }
  };
  // U half-slice (slice s, xi 8 h .. 8 h + 7) into LDS stage b: 24 pieces of
  // 2 KiB (rows k0 .. k0 + 31 of one (xi, plane)), 12 x 1 KiB LDS-DMA per wave
  auto uload = [&](int s, int h, int b) __attribute__((always_inline)) {
    GK_LDS char* ub = (GK_LDS char*)xl + b * XSTAGE;
#pragma unroll
    for (int i = 0; i < 12; ++i) {
      const int q = wave * 12 + i, piece = q >> 1, half = q & 1;   // piece = xl_ * 3 + plane
      const int64_t src = (((int64_t)(s * 16 + 8 * h) * 3 + piece) * g.Co + k0) * 32 + half * 512 + lane * 8;
#ifndef GK_WX6_PROBE_NODMA
      glds16(u3 + src, ub + piece * XPLANE + half * 1024);
#endif
    }
  };
  // A fragments (U) of xi slot xl_ (0..7) of stage b, plane pl, fragment kf
  const int aoff0 = fi * XROW + ((fq ^ xsw(fi)) << 4);   // rows kf*16 + fi: xsw(kf*16 + fi) == xsw(fi)
  auto afrag = [&](int b, int xl_, int pl, int kf) __attribute__((always_inline)) -> bf16x8 {
    const char* p = xl + b * XSTAGE + (xl_ * 3 + pl) * XPLANE + kf * 16 * XROW + aoff0;
    return *reinterpret_cast<const bf16x8*>(p);
  };

  // xi = 4 i + j of t row i (= row i of B^T d): V = (t B)[j], split, 2 x 6 MFMAs
  auto xi_mfma = [&](const Row& t, int xi, int b) __attribute__((always_inline)) {
    const int j = xi & 3, xl_ = xi & 7;
    f32x4 v0, v1;
    if (j == 0) { v0 = t[0][0] - t[2][0]; v1 = t[0][1] - t[2][1]; }
    else if (j == 1) { v0 = t[1][0] + t[2][0]; v1 = t[1][1] + t[2][1]; }
    else if (j == 2) { v0 = t[2][0] - t[1][0]; v1 = t[2][1] - t[1][1]; }
    else { v0 = t[1][0] - t[3][0]; v1 = t[1][1] - t[3][1]; }
    bf16x8 vh, vm, vl;
    split3x8(v0, v1, vh, vm, vl);
#pragma unroll
    for (int kf = 0; kf < 2; ++kf) {
      const bf16x8 ah = afrag(b, xl_, 0, kf), am = afrag(b, xl_, 1, kf), al = afrag(b, xl_, 2, kf);
      f32x4 c = acc[xi][kf];
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, vh, c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, vl, c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, vm, c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, vh, c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, vm, c, 0, 0, 0);
      acc[xi][kf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, vh, c, 0, 0, 0);
    }
  };
  auto rsub = [&](Row& o, const Row& a, const Row& b) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 4; ++j) { o[j][0] = a[j][0] - b[j][0]; o[j][1] = a[j][1] - b[j][1]; }
  };
  auto radd = [&](Row& o, const Row& a, const Row& b) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 4; ++j) { o[j][0] = a[j][0] + b[j][0]; o[j][1] = a[j][1] + b[j][1]; }
  };

  const auto hr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(bb.h), (short)0, BNB ? (int)g.ybytes : 0,
                                                    0x00020000);
  const auto dr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(bb.dy2), (short)0,
                                                    (BNB && bb.dy2) ? (int)g.ybytes : 0, 0x00020000);
  const auto mr = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(bb.mask), (short)0,
                                                    (BNB && bb.mask) ? (int)(g.ybytes / 16) : 0, 0x00020000);
  // output transform A^T M A of this lane's tile, 4 channels per fragment
  auto epilogue = [&](int tb) __attribute__((always_inline)) {
    const int tt = tb * XT + wave * 16 + fi;
    const bool tv = tt < g.ntiles;
    const int ttc = tv ? tt : 0;
    const int n = ttc / THW, rr = ttc - n * THW, th = rr / g.TW, tw = rr - th * g.TW;
    bool pv[4];
    int64_t row[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int oh = 2 * th + (p >> 1), ow = 2 * tw + (p & 1);
      pv[p] = tv && oh < g.H && ow < g.W;
      row[p] = ((int64_t)n * g.H + oh) * g.W + ow;
    }
#pragma unroll
    for (int kf = 0; kf < 2; ++kf) {
      const int kk = k0 + kf * 16 + 4 * fq;
      f32x4 o[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float s0[4], s1[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          s0[j] = acc[j][kf][r] + acc[4 + j][kf][r] + acc[8 + j][kf][r];
          s1[j] = acc[4 + j][kf][r] - acc[8 + j][kf][r] - acc[12 + j][kf][r];
        }
        o[0][r] = s0[0] + s0[1] + s0[2];
        o[1][r] = s0[1] - s0[2] - s0[3];
        o[2][r] = s1[0] + s1[1] + s1[2];
        o[3][r] = s1[1] - s1[2] - s1[3];
      }
#pragma unroll
      for (int xi = 0; xi < 16; ++xi) acc[xi][kf] = f32x4{0.f, 0.f, 0.f, 0.f};
      f32x4 hv[4], d2[4];
      uint32_t bits[4];
      if constexpr (BNB) {
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const uint32_t off = pv[p] ? (uint32_t)(row[p] * g.Co + kk) * 4u : 0x80000000u;
          hv[p] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(hr, (int)off, 0, 0));
          d2[p] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(dr, (int)off, 0, 0));
          const uint32_t moff = pv[p] ? (uint32_t)(row[p] * (g.Co >> 2) + (kk >> 2)) : 0x80000000u;
          bits[p] = bb.mask ? (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(mr, (int)moff, 0, 0) : 0xfu;
        }
      }
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        f32x4 v = o[p];
        if constexpr (BNB) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float dz = pv[p] && ((bits[p] >> r) & 1u) ? v[r] + d2[p][r] : 0.f;
            v[r] = dz;
            ssum[kf][r] += dz;
            ssq[kf][r] = fmaf(dz, hv[p][r], ssq[kf][r]);
          }
        } else if constexpr (STATS) {
          const float m = pv[p] ? 1.f : 0.f;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            ssum[kf][r] = fmaf(m, v[r], ssum[kf][r]);
            ssq[kf][r] = fmaf(m * v[r], v[r], ssq[kf][r]);
          }
        }
        if (pv[p]) *reinterpret_cast<f32x4*>(y + row[p] * g.Co + kk) = v;
      }
    }
  };

  if (total > 0) {
    int tb = blockIdx.x, s = 0;     // compute cursor
    int lb = blockIdx.x, ls = 0;    // patch-load cursor (one slice ahead)
    auto adv = [&](int& t, int& st) __attribute__((always_inline)) {
      if (++st == nsl) {
        st = 0;
        t += gridDim.x;
      }
    };
    // Patch rows in registers (the budget: 128 accumulators + 256 VGPRs):
    // rows d0-d2 of a slice are prefetched during the previous slice's second
    // half; at the top t0 = d0 - d2, t1 = d1 + d2, t2 = d2 - d1 are formed and
    // d3 is loaded (landing during the first half, which needs t0, t1 only);
    // t3 = d1 - d3 at the middle, where the next slice's d0-d2 go out.  Peak
    // ~160 patch registers instead of two full 128-register patches.
    Row p0, p1, p2;
    set_tile(lb);
    uload(0, 0, 0);
    gload_row(p0, 0, 0);
    gload_row(p1, 1, 0);
    gload_row(p2, 2, 0);
    for (int it = 0; it < total; ++it) {
      const bool more = it + 1 < total;
      // this slice's d0-d2 and U half 0 have landed; stage 1 is free
      asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
      uload(s, 1, 1);
      Row d3, t0, t1, t2, t3;
      gload_row(d3, 3, s);
      rsub(t0, p0, p2);
      radd(t1, p1, p2);
      rsub(t2, p2, p1);
      const Row& d1 = p1;
#pragma unroll
      for (int xi = 0; xi < 4; ++xi) xi_mfma(t0, xi, 0);
#pragma unroll
      for (int xi = 4; xi < 8; ++xi) xi_mfma(t1, xi, 0);
      // d3 and U half 1 have landed; stage 0 is free
      asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
      rsub(t3, d1, d3);
      if (more) {
        int ns = s + 1;
        if (ns == nsl) ns = 0;
        uload(ns, 0, 0);
        adv(lb, ls);
        if (ls == 0) set_tile(lb);
        gload_row(p0, 0, ls);
        gload_row(p1, 1, ls);
        gload_row(p2, 2, ls);
      }
#pragma unroll
      for (int xi = 8; xi < 12; ++xi) xi_mfma(t2, xi, 1);
#pragma unroll
      for (int xi = 12; xi < 16; ++xi) xi_mfma(t3, xi, 1);
      if (s == nsl - 1) epilogue(tb);
      adv(tb, s);
    }
  }

  if constexpr (STATS || BNB) {
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) {
          ssum[a][r] += __shfl_xor(ssum[a][r], off, 64);
          ssq[a][r] += __shfl_xor(ssq[a][r], off, 64);
        }
    __syncthreads();
    float* red = reinterpret_cast<float*>(xl);   // [sum | sq][wave][32]
    if (fi == 0) {
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int col = a * 16 + 4 * fq + r;
          red[wave * XK + col] = ssum[a][r];
          red[(4 + wave) * XK + col] = ssq[a][r];
        }
    }
    __syncthreads();
    if (tid < XK) {
      float sa = 0.f, sb = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        sa += red[w * XK + tid];
        sb += red[(4 + w) * XK + tid];
      }
      stats[(int64_t)blockIdx.x * g.Co + k0 + tid] = sa;
      stats[stats_ld + (int64_t)blockIdx.x * g.Co + k0 + tid] = sb;
    }
  }
}

template <bool STATS, bool BNB>
int launch_x6(const float* x, const uint16_t* u3, float* y, const X6Geo& g, int max_blocks, float* stats,
              int stats_rows, const X6Bnb& bb, hipStream_t stream) {
  const int ntb = (g.ntiles + XT - 1) / XT;
  const int nkb = g.Co / XK;
  // persistent along tiles, one block per CU, x extent a multiple of 8
  int gx = max_blocks > 0 ? max_blocks : ((256 + nkb - 1) / nkb + 7) / 8 * 8;
  if (gx > ntb) gx = ntb;
  if ((STATS || BNB) && gx > stats_rows) gx = stats_rows;
  if (gx < 1) gx = 1;
  static bool attr = [] {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&wino_x6_kernel<STATS, BNB>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, XLDS) == hipSuccess;
  }();
  (void)attr;
  hipLaunchKernelGGL((wino_x6_kernel<STATS, BNB>), dim3((unsigned)gx, (unsigned)nkb), dim3(256), XLDS, stream, x, u3, y,
                     g, stats, (int64_t)stats_rows * g.Co, bb);
  return gx;
}

}  // namespace

void wino_x6_weights(const float* w, uint16_t* u3, int Co, int Ci, int flip, hipStream_t stream) {
  const int64_t n = (int64_t)Co * Ci;
  hipLaunchKernelGGL(wino_x6_wt_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, w, u3, Co, Ci, flip);
}

int wino_x6_conv(const float* x, const uint16_t* u3, float* y, int N, int H, int W, int Ci, int Co, int max_blocks,
                 float* stats, int stats_rows, const BnBwdArgs* bn, hipStream_t stream) {
  if (Ci % XC != 0 || Co % XK != 0) return -1;
  X6Geo g{H, W, Ci, Co, (H + 1) / 2, (W + 1) / 2, 0, 0, 0};
  g.ntiles = N * g.TH * g.TW;
  g.xbytes = (uint32_t)((int64_t)N * H * W * Ci * 4);
  g.ybytes = (uint32_t)((int64_t)N * H * W * Co * 4);
  const X6Bnb bb = bn ? X6Bnb{static_cast<const float*>(bn->h), static_cast<const float*>(bn->dy2), bn->mask}
                      : X6Bnb{nullptr, nullptr, nullptr};
  if (bn) return launch_x6<false, true>(x, u3, y, g, max_blocks, stats, stats_rows, bb, stream);
  if (stats) return launch_x6<true, false>(x, u3, y, g, max_blocks, stats, stats_rows, bb, stream);
  return launch_x6<false, false>(x, u3, y, g, max_blocks, nullptr, 0, bb, stream);
}

}  // namespace gk
