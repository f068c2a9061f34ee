// Grad-weight of a 3x3 / stride-1 / padding-1 convolution over channels-last
// bf16 activations, tap-parallel (gfx950).
//
//   dW[k][kh][kw][c] += sum_p dY[p][k] * X[p shifted by (kh-1, kw-1)][c]
//
// The implicit-GEMM grad-weight (gemm.hip gemm_tn, GATHER) streams the output
// gradient once per 64-wide K tile, i.e. once per filter tap: 9x the dY traffic
// at C = 64 (ResNet-50 layer1: 340-430 us against a 65 us roofline).  Here a
// workgroup owns one (64 input channels) x (64 output channels) pair and a run
// of "bands" of R output rows; per band it stages dY and X ONCE in LDS and its 9
// waves -- one per tap -- read their shifted X window from the same image.
//
// Pixels are walked in padded coordinates: output pixel (r, w) of the band is
// q = r * WP + w + 1 with WP = W + 2; the two pad columns per row carry dY = 0,
// so every run of 8 consecutive q maps to 8 consecutive staged rows for every
// tap (X row index q + kh * WP + kw; the X image carries one leading zero row
// and the zero padding of the convolution).  Both operands are [pixel][64 ch]
// images with 128-byte rows read as transposed MFMA fragments
// (ds_read_b64_tr_b16, the swizzle of gemm.hip's TN kernel), so the reduction
// runs over pixels: per 32-pixel step a wave issues 16 transposed reads and 16
// v_mfma_f32_16x16x32_bf16 into its 64 x 64 tap tile.
//
// Per-block fp32 partials [blocks][9 * 64 * 64] are summed in a fixed order by
// wgrad3_reduce_kernel (deterministic, no atomics) and added into the (arena)
// gradient -- the same contract as gemm_tn's float-atomic accumulate.
#include <hip/hip_runtime.h>

#include "common.h"
#include "gk_kernels.h"
#include "mfma_util.h"

namespace gk {
namespace {

constexpr int kW3Waves = 9;
constexpr int kW3Threads = 64 * kW3Waves;
constexpr int kW3MaxRows = 480;   // staged output pixels per band (padded)
constexpr int kW3TileF = 9 * 64 * 64;

struct W3Geo {
  int N, H, W, C, K;
  int WP;        // W + 2
  int R;         // output rows per band
  int Mp;        // staged (padded) output pixels per band, multiple of 32
  int XR;        // staged X rows per band
  int nb;        // bands per image
  int pairs;     // (C / 64) * (K / 64)
  int bpp;       // blocks per pair
};

// 16-byte chunk ck of staged row r sits at chunk ck ^ tr_swz<128>(r)
__device__ __forceinline__ int w3_off(int r, int ck) { return r * 128 + ((ck ^ tr_swz<128>(r)) << 4); }

__global__ void __launch_bounds__(kW3Threads)
wgrad3_kernel(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ x, float* __restrict__ part, W3Geo g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* dyb = smem;                        // [Mp][128 B]
  char* xb = smem + g.Mp * 128;            // [XR][128 B]
  const int lane = threadIdx.x & 63, tap = threadIdx.x >> 6;
  const int kh = tap / 3, kw = tap - kh * 3;
  const int fr = lane & 15, fq = lane >> 4;
  const int pair = blockIdx.x / g.bpp, bsub = blockIdx.x - pair * g.bpp;
  const int ci = pair % (g.C / 64), co = pair / (g.C / 64);
  const int64_t total = (int64_t)g.N * g.nb;
  const int64_t b0 = total * bsub / g.bpp, b1 = total * (bsub + 1) / g.bpp;

  // transposed-fragment addresses of step 0 (a step adds 32 rows = 4096 bytes;
  // the swizzle repeats every 16 rows): A = dY rows q0 + 8g + 0..7 of column
  // 16 nt + li, B = X rows q0 + tap offset + 8g + 0..7 of column 16 kt + li
  const int toff = kh * g.WP + kw;
  uint32_t aa[4][2], ba[4][2];
  {
    const int gq = lane >> 4, li = lane & 15, q4 = li >> 2, pp = li & 3;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int col = t * 16 + 4 * pp;
      const int ra = 8 * gq + q4, rb = ra + 4;
      aa[t][0] = (uint32_t)(uintptr_t)(GK_LDS char*)(dyb + ra * 128 + ((((col >> 3) ^ tr_swz<128>(ra)) << 4) | ((col & 7) << 1)));
      aa[t][1] = (uint32_t)(uintptr_t)(GK_LDS char*)(dyb + rb * 128 + ((((col >> 3) ^ tr_swz<128>(rb)) << 4) | ((col & 7) << 1)));
      const int xa = toff + ra, xbr = toff + rb;
      ba[t][0] = (uint32_t)(uintptr_t)(GK_LDS char*)(xb + xa * 128 + ((((col >> 3) ^ tr_swz<128>(xa)) << 4) | ((col & 7) << 1)));
      ba[t][1] = (uint32_t)(uintptr_t)(GK_LDS char*)(xb + xbr * 128 + ((((col >> 3) ^ tr_swz<128>(xbr)) << 4) | ((col & 7) << 1)));
    }
  }
  f32x4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int64_t bi = b0; bi < b1; ++bi) {
    const int n = (int)(bi / g.nb);
    const int r0 = (int)(bi - (int64_t)n * g.nb) * g.R;
    __syncthreads();   // the previous band's fragments are read
    // dY band: staged row q = (r, w') -> dY[n, r0 + r, w' - 1, 64 co ..] (zero on pads / past the band)
    for (int base = 0; base < g.Mp * 8; base += 8 * kW3Threads) {
      uint4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = base + u * kW3Threads + (int)threadIdx.x;
        const int q = i >> 3, ck = i & 7;
        const int r = q / g.WP, wq = q - r * g.WP;
        const bool ok = i < g.Mp * 8 && r < g.R && r0 + r < g.H && wq >= 1 && wq <= g.W;
        const uint16_t* src = ok ? dy + (((int64_t)n * g.H + r0 + r) * g.W + wq - 1) * g.K + co * 64 + ck * 8 : dy;
        v[u] = *reinterpret_cast<const uint4*>(src);
        if (!ok) v[u] = make_uint4(0u, 0u, 0u, 0u);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = base + u * kW3Threads + (int)threadIdx.x;
        if (i < g.Mp * 8) *reinterpret_cast<uint4*>(dyb + w3_off(i >> 3, i & 7)) = v[u];
      }
    }
    // X band: staged row e >= 1 -> input (r0 - 1 + (e-1) / WP, (e-1) % WP - 1), zero outside
    for (int base = 0; base < g.XR * 8; base += 8 * kW3Threads) {
      uint4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = base + u * kW3Threads + (int)threadIdx.x;
        const int e = i >> 3, ck = i & 7;
        const int ei = e - 1;
        const int ii = ei / g.WP, jj = ei - ii * g.WP;
        const int ih = r0 - 1 + ii, iw = jj - 1;
        const bool ok = i < g.XR * 8 && e >= 1 && ii < g.R + 2 && (unsigned)ih < (unsigned)g.H &&
                        (unsigned)iw < (unsigned)g.W;
        const uint16_t* src = ok ? x + (((int64_t)n * g.H + ih) * g.W + iw) * g.C + ci * 64 + ck * 8 : x;
        v[u] = *reinterpret_cast<const uint4*>(src);
        if (!ok) v[u] = make_uint4(0u, 0u, 0u, 0u);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = base + u * kW3Threads + (int)threadIdx.x;
        if (i < g.XR * 8) *reinterpret_cast<uint4*>(xb + w3_off(i >> 3, i & 7)) = v[u];
      }
    }
    __syncthreads();
#pragma unroll 2
    for (int q0 = 0; q0 < g.Mp; q0 += 32) {
      const uint32_t step = (uint32_t)q0 * 128u;
      bf16x8 av[4], bv[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((GK_LDS bf16x4*)(uintptr_t)(aa[t][0] + step));
        const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((GK_LDS bf16x4*)(uintptr_t)(aa[t][1] + step));
        av[t] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        const bf16x4 xl = __builtin_amdgcn_ds_read_tr16_b64_v4i16((GK_LDS bf16x4*)(uintptr_t)(ba[t][0] + step));
        const bf16x4 xh = __builtin_amdgcn_ds_read_tr16_b64_v4i16((GK_LDS bf16x4*)(uintptr_t)(ba[t][1] + step));
        bv[t] = bf16x8{xl[0], xl[1], xl[2], xl[3], xh[0], xh[1], xh[2], xh[3]};
      }
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
          acc[nt][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[nt], bv[kt], acc[nt][kt], 0, 0, 0);
    }
  }
  // lane holds D[cout 16 nt + 4 fq + r][cin 16 kt + fr] of tap (kh, kw)
  float* out = part + (int64_t)blockIdx.x * kW3TileF + tap * 4096;
#pragma unroll
  for (int nt = 0; nt < 4; ++nt)
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) out[(nt * 16 + 4 * fq + r) * 64 + kt * 16 + fr] = acc[nt][kt][r];
}

// out[k][c][kh][kw] (element strides) += sum over the pair's blocks of part[b][tap][k % 64][c % 64]
__global__ void __launch_bounds__(256) wgrad3_reduce_kernel(const float* __restrict__ part, W3Geo g,
                                                            float* __restrict__ out, int64_t s0, int64_t s1,
                                                            int64_t s2, int64_t s3) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t tot = (int64_t)g.pairs * kW3TileF;
  if (i >= tot) return;
  const int pair = (int)(i / kW3TileF), rem = (int)(i - (int64_t)pair * kW3TileF);
  const int tap = rem >> 12, kk = (rem >> 6) & 63, cc = rem & 63;
  const int ci = pair % (g.C / 64), co = pair / (g.C / 64);
  const float* p = part + ((int64_t)pair * g.bpp) * kW3TileF + rem;
  float s = 0.f;
  for (int b = 0; b < g.bpp; ++b) s += p[(int64_t)b * kW3TileF];
  const int k = co * 64 + kk, c = ci * 64 + cc, kh = tap / 3, kw = tap - kh * 3;
  out[k * s0 + c * s1 + kh * s2 + kw * s3] += s;
}

W3Geo w3_geo(int N, int H, int W, int C, int K) {
  W3Geo g;
  g.N = N;
  g.H = H;
  g.W = W;
  g.C = C;
  g.K = K;
  g.WP = W + 2;
  int R = kW3MaxRows / g.WP;
  if (R > H) R = H;
  if (R < 1) R = 1;
  g.R = R;
  g.Mp = (R * g.WP + 31) / 32 * 32;
  g.XR = g.Mp + 2 * g.WP + 3;
  g.nb = (H + R - 1) / R;
  g.pairs = (C / 64) * (K / 64);
  const int64_t total = (int64_t)N * g.nb;
  int64_t bpp = (512 + g.pairs - 1) / g.pairs;
  if (bpp > total) bpp = total;
  if (bpp < 1) bpp = 1;
  g.bpp = (int)bpp;
  return g;
}

int w3_lds(const W3Geo& g) { return (g.Mp + g.XR) * 128; }

}  // namespace

bool wgrad3_supported(int H, int W, int C, int K) {
  if (C % 64 || K % 64 || H < 1 || W < 1 || W + 2 > kW3MaxRows) return false;
  return w3_lds(w3_geo(1, H, W, C, K)) <= 160 * 1024;
}

int64_t wgrad3_ws_floats(int N, int H, int W, int C, int K) {
  const W3Geo g = w3_geo(N, H, W, C, K);
  return (int64_t)g.pairs * g.bpp * kW3TileF;
}

void wgrad3_acc(const void* dy, const void* x, int N, int H, int W, int C, int K, float* part, float* out, int64_t s0,
                int64_t s1, int64_t s2, int64_t s3, hipStream_t stream) {
  const W3Geo g = w3_geo(N, H, W, C, K);
  static bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad3_kernel),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
  (void)attr;
  hipLaunchKernelGGL(wgrad3_kernel, dim3(g.pairs * g.bpp), dim3(kW3Threads), w3_lds(g), stream,
                     static_cast<const uint16_t*>(dy), static_cast<const uint16_t*>(x), part, g);
  const int64_t tot = (int64_t)g.pairs * kW3TileF;
  hipLaunchKernelGGL(wgrad3_reduce_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, stream, part, g, out, s0,
                     s1, s2, s3);
}

}  // namespace gk
