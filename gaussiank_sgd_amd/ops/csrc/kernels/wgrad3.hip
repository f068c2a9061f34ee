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
constexpr int kW3Rows = 256;      // staged (padded) output pixels per band: target
constexpr int kW3U = 4;           // 32-pixel steps per immediate-offset group
constexpr int kW3TileF = 9 * 64 * 64;

struct W3Geo {
  int N, H, W, C, K;
  int WP;        // W + 2
  int R;         // output rows per band
  int Mp;        // staged (padded) output pixels per band, multiple of 32 * kW3U
  int XR;        // staged X rows per band
  int ninst;     // 1-KiB LDS-DMA pieces per band image
  int bufb;      // bytes per LDS buffer (ninst KiB)
  int nb;        // bands per image
  int pairs;     // (C / 64) * (K / 64)
  int bpp;       // blocks per pair
  float rcp_wp;  // 1 / WP
  const uint16_t* zero;   // >= 64 zero bf16 (LDS-DMA source of padding rows)
};

// a / d for a < 2^22 via the float reciprocal (one correction step)
__device__ __forceinline__ int w3_div(int a, int d, float rcp) {
  int q = (int)((float)a * rcp);
  const int r = a - q * d;
  if (r < 0) --q;
  else if (r >= d) ++q;
  return q;
}

// Stage band (n, r0) of pair (ci, co) into the LDS buffer at `buf` with 16-byte
// LDS-DMA: piece p of 64 lanes fills chunk positions 64 p + lane, i.e. row
// 8 p + lane / 8, position lane % 8, which holds logical chunk
// position ^ tr_swz<128>(row) -- the swizzle lives on the source address.
// Rows [0, Mp): dY (padded pixel q = r * WP + w'); rows [Mp, Mp + XR): X with
// one leading zero row; pads and rows past the band read the zero buffer.
// A wave's pieces are 9 apart (72 rows), so each lane walks its (row / WP,
// row % WP) incrementally -- one division per region, not per piece -- and
// addresses are 32-bit offsets from the band image's (wave-uniform) base.
__device__ __forceinline__ void w3_issue(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ x,
                                        const W3Geo& g, int n, int r0, int ci, int co, char* buf, int wave,
                                        int lane) {
  const uint16_t* dimg = dy + (int64_t)n * g.H * g.W * g.K + co * 64;
  const uint16_t* ximg = x + (int64_t)n * g.H * g.W * g.C + ci * 64;
  const int l3 = lane >> 3, l7 = lane & 7;
  const int step_q = (8 * kW3Waves) / g.WP, step_r = (8 * kW3Waves) - step_q * g.WP;
  int region = -1, qr = 0, qc = 0;
  for (int p = wave; p < g.ninst; p += kW3Waves) {
    const int row = p * 8 + l3;
    const int ck = l7 ^ (2 * (((l3 >> 1) & 1) | ((p & 1) << 1)));   // tr_swz<128>(row)
    const uint16_t* src = g.zero + ck * 8;
    if (p * 8 < g.Mp) {                     // wave-uniform: Mp is a multiple of 128
      if (region != 0) {
        region = 0;
        qr = w3_div(row, g.WP, g.rcp_wp);
        qc = row - qr * g.WP;
      }
      if (qr < g.R && r0 + qr < g.H && qc >= 1 && qc <= g.W)
        src = dimg + (uint32_t)(((r0 + qr) * g.W + qc - 1) * g.K) + ck * 8;
    } else if (p * 8 < g.Mp + g.XR) {
      if (region != 1) {                    // X row e = row - Mp; e - 1 = ii * WP + jj
        region = 1;
        const int t = row - g.Mp - 1 + g.WP;  // >= WP - 1 >= 0
        qr = w3_div(t, g.WP, g.rcp_wp);
        qc = t - qr * g.WP;
        --qr;
      }
      const int ih = r0 - 1 + qr, iw = qc - 1;
      if (qr >= 0 && qr < g.R + 2 && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W)
        src = ximg + (uint32_t)((ih * g.W + iw) * g.C) + ck * 8;
    }
    glds16(src, (GK_LDS char*)(buf + p * 1024));
    qr += step_q;
    qc += step_r;
    if (qc >= g.WP) {
      qc -= g.WP;
      ++qr;
    }
  }
}

// transposed LDS read at a precomputed address + immediate byte offset
template <int OFF>
__device__ __forceinline__ bf16x4 w3_tr(uint32_t a) {
  bf16x4 v;
  if (OFF == 0) asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(a));
  else asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(v) : "v"(a), "i"(OFF));
  return v;
}

// s_waitcnt lgkmcnt(N) tied to two fragments (the asm reads are invisible to
// the compiler's wait-count pass; the tie keeps dependent MFMAs below the wait)
template <int N>
__device__ __forceinline__ void w3_wait(bf16x8& a, bf16x8& b) {
  asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(a), "+v"(b) : "n"(N));
}

// One 32-pixel step: 16 transposed reads issued as (A_t, B_t) pairs, then the
// 16 MFMAs in the order the pairs land -- the wait before pair t's MFMAs leaves
// the later pairs' reads in flight, so the LDS latency hides behind MFMAs.
template <int S>
__device__ __forceinline__ void w3_step(const uint32_t (&aa)[4][2], const uint32_t (&ba)[4][2], uint32_t base,
                                        f32x4 (&acc)[4][4]) {
  constexpr int OFF = S * 4096;   // 32 staged rows of 128 B per step
  bf16x8 av[4], bv[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const bf16x4 lo = w3_tr<OFF>(aa[t][0] + base), hi = w3_tr<OFF>(aa[t][1] + base);
    const bf16x4 xl = w3_tr<OFF>(ba[t][0] + base), xh = w3_tr<OFF>(ba[t][1] + base);
    av[t] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    bv[t] = bf16x8{xl[0], xl[1], xl[2], xl[3], xh[0], xh[1], xh[2], xh[3]};
  }
  w3_wait<12>(av[0], bv[0]);
  acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[0], bv[0], acc[0][0], 0, 0, 0);
  __builtin_amdgcn_sched_barrier(0);   // keep each MFMA group between its wait and the next
  w3_wait<8>(av[1], bv[1]);
  acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[0], bv[1], acc[0][1], 0, 0, 0);
  acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[1], bv[0], acc[1][0], 0, 0, 0);
  acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[1], bv[1], acc[1][1], 0, 0, 0);
  __builtin_amdgcn_sched_barrier(0);
  w3_wait<4>(av[2], bv[2]);
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    acc[t][2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[t], bv[2], acc[t][2], 0, 0, 0);
    acc[2][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[2], bv[t], acc[2][t], 0, 0, 0);
  }
  acc[2][2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[2], bv[2], acc[2][2], 0, 0, 0);
  __builtin_amdgcn_sched_barrier(0);
  w3_wait<0>(av[3], bv[3]);
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    acc[t][3] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[t], bv[3], acc[t][3], 0, 0, 0);
    acc[3][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[3], bv[t], acc[3][t], 0, 0, 0);
  }
  acc[3][3] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[3], bv[3], acc[3][3], 0, 0, 0);
}

__global__ void __launch_bounds__(kW3Threads)
wgrad3_kernel(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ x, float* __restrict__ part, W3Geo g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, tap = threadIdx.x >> 6;
  const int kh = tap / 3, kw = tap - kh * 3;
  const int fr = lane & 15, fq = lane >> 4;
  const int pair = blockIdx.x / g.bpp, bsub = blockIdx.x - pair * g.bpp;
  const int ci = pair % (g.C / 64), co = pair / (g.C / 64);
  const int64_t total = (int64_t)g.N * g.nb;
  const int64_t b0 = total * bsub / g.bpp, b1 = total * (bsub + 1) / g.bpp;

  // fragment addresses of step 0 in buffer 0 (a step adds 32 rows = 4096 B;
  // the swizzle repeats every 16 rows): A = dY rows 8g + 0..7 of column
  // 16 t + li, B = X rows (tap offset) + 8g + 0..7
  const int toff = g.Mp + kh * g.WP + kw;
  uint32_t aa[4][2], ba[4][2];
  {
    const uint32_t lbase = (uint32_t)(uintptr_t)(GK_LDS char*)smem;
    const int gq = lane >> 4, li = lane & 15, q4 = li >> 2, pp = li & 3;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int col = t * 16 + 4 * pp;
      const int ra = 8 * gq + q4, rb = ra + 4, xa = toff + ra, xr = toff + rb;
      aa[t][0] = lbase + ra * 128 + ((((col >> 3) ^ tr_swz<128>(ra)) << 4) | ((col & 7) << 1));
      aa[t][1] = lbase + rb * 128 + ((((col >> 3) ^ tr_swz<128>(rb)) << 4) | ((col & 7) << 1));
      ba[t][0] = lbase + xa * 128 + ((((col >> 3) ^ tr_swz<128>(xa)) << 4) | ((col & 7) << 1));
      ba[t][1] = lbase + xr * 128 + ((((col >> 3) ^ tr_swz<128>(xr)) << 4) | ((col & 7) << 1));
    }
  }
  f32x4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  int cur = 0;
  if (b0 < b1) {
    const int n = (int)(b0 / g.nb);
    w3_issue(dy, x, g, n, (int)(b0 - (int64_t)n * g.nb) * g.R, ci, co, smem, tap, lane);
  }
  for (int64_t bi = b0; bi < b1; ++bi) {
    // this band's pieces (issued one band ago) have landed for every wave; the
    // other buffer's reads (previous band) are done -> restage it for the next band
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (bi + 1 < b1) {
      const int n = (int)((bi + 1) / g.nb);
      w3_issue(dy, x, g, n, (int)((bi + 1) - (int64_t)n * g.nb) * g.R, ci, co, smem + (cur ^ 1) * g.bufb, tap, lane);
    }
    const uint32_t boff = (uint32_t)(cur * g.bufb);
    for (int q0 = 0; q0 < g.Mp; q0 += 32 * kW3U) {
      const uint32_t base = boff + (uint32_t)q0 * 128u;
      w3_step<0>(aa, ba, base, acc);
      w3_step<1>(aa, ba, base, acc);
      w3_step<2>(aa, ba, base, acc);
      w3_step<3>(aa, ba, base, acc);
    }
    cur ^= 1;
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
  int R = kW3Rows / g.WP;
  if (R > H) R = H;
  if (R < 1) R = 1;
  g.R = R;
  g.Mp = (R * g.WP + 32 * kW3U - 1) / (32 * kW3U) * (32 * kW3U);
  g.XR = g.Mp + 2 * g.WP + 3;
  g.ninst = ((g.Mp + g.XR) * 8 + 63) / 64;
  g.bufb = g.ninst * 1024;
  g.nb = (H + R - 1) / R;
  g.pairs = (C / 64) * (K / 64);
  const int64_t total = (int64_t)N * g.nb;
  int64_t bpp = (256 + g.pairs - 1) / g.pairs;
  if (bpp > total) bpp = total;
  if (bpp < 1) bpp = 1;
  g.bpp = (int)bpp;
  g.rcp_wp = 1.0f / (float)g.WP;
  g.zero = nullptr;
  return g;
}

int w3_lds(const W3Geo& g) { return 2 * g.bufb; }

}  // namespace

bool wgrad3_supported(int H, int W, int C, int K) {
  if (C % 64 || K % 64 || H < 1 || W < 1 || W + 2 > kW3Rows) return false;
  return w3_lds(w3_geo(1, H, W, C, K)) <= 160 * 1024;
}

int64_t wgrad3_ws_floats(int N, int H, int W, int C, int K) {
  const W3Geo g = w3_geo(N, H, W, C, K);
  return (int64_t)g.pairs * g.bpp * kW3TileF;
}

void wgrad3_acc(const void* dy, const void* x, const void* zero, int N, int H, int W, int C, int K, float* part,
                float* out, int64_t s0, int64_t s1, int64_t s2, int64_t s3, hipStream_t stream) {
  W3Geo g = w3_geo(N, H, W, C, K);
  g.zero = static_cast<const uint16_t*>(zero);
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
