// MFMA GEMMs for 1x1 convolutions on channels-last (NHWC) activations, gfx950.
//
// A stride-1 1x1 convolution over NHWC data is a plain GEMM over the
// M = N*H*W pixel rows:
//   forward      Y[M, Cout] = X[M, Cin]  . W[Cout, Cin]^T          (gemm_nt)
//   grad-input  dX[M, Cin]  = dY[M, Cout] . Wt[Cin, Cout]^T        (gemm_nt, Wt = W^T)
//   grad-weight dW[Cout, Cin] += dY[M, Cout]^T . X[M, Cin]         (gemm_tn, split over M)
// MIOpen/hipBLASLt run these ResNet-50 shapes at 20-65 % of their HBM
// roofline and the tall-skinny grad-weight reduction at ~10 %
// (profiles/r01_resnet50_conv_roofline_bs512.txt), so they get their own
// kernels here.
//
// gemm_nt: 64*WM*WN threads, each wave owns a 64x64 output tile made of 4x4
//   v_mfma_f32_16x16x32_bf16 tiles.  Operands are K-contiguous, staged
//   global -> LDS with 16-byte global_load_lds (LDS-DMA) into 128-byte rows
//   (one 64-deep K slice) whose 16-byte chunks are XOR-swizzled by
//   (row >> 1) & 7, which makes every ds_read_b128 fragment read bank-conflict
//   free.  The MFMA is issued "swapped" (weight rows as the A operand, pixel
//   rows as B), so each lane ends with 4 consecutive output channels of one
//   pixel and writes them as one 8-byte store.  The grid is persistent over
//   M tiles and the two LDS stages are pipelined across tile boundaries, so
//   the next tile's loads are in flight during the current tile's MFMAs and
//   stores (the K = 64 layers have a single K step per tile).
// gemm_tn: reduction over the pixel dimension M; both operands are
//   M-major, so fragments are read with ds_read_b64_tr_b16 (the gfx950 LDS
//   transpose read: 4 rows x 16 columns of 16-bit data delivered column-wise).
//   Each block reduces a contiguous slice of M for one output tile and adds
//   its fp32 partial into the (gradient-arena) output with float atomics.
#include "gemm_kern.h"

namespace gk {

static int nt_unit_b16(bool gather, GK_NT_UNIT_ARGS) {
  return gather ? nt_b16_gat(GK_NT_UNIT_PASS) : nt_b16_row(GK_NT_UNIT_PASS);
}

// fp32 operands: cfg digit 100000 selects the bf16x6 products (gemm_kern.h X6)
static int nt_unit_f32(bool gather, GK_NT_UNIT_ARGS) {
  const int fam = (cfg / 100000) % 10;
  if (fam == 2 || fam == 3) {
    // bf16x6 with register staging: row GEMMs and stride / padding implicit
    // GEMMs (C a multiple of 32) without a lazy operand, split-K or remap;
    // family 3: B pre-split (geo.b3, the binding's split3_rows)
    if (lza || geo.KZ > 1 || geo.RH || (fam == 3) != (geo.b3 != nullptr)) return -2;
    if (gather) {
      // 32-bit element offsets into x (gemm_kern.h x62 gather)
      const int64_t nimg = M / ((int64_t)geo.OH * geo.OW);
      if (geo.C % 32 != 0 || nimg * geo.H * geo.W * geo.C >= ((int64_t)1 << 31)) return -2;
      return nt_x62_gat(static_cast<const float*>(A), static_cast<const float*>(B), static_cast<float*>(C), M, N, K,
                        cfg % 100000, max_blocks, geo, stats, stats_ld, stats_rows, bb, stream);
    }
    return nt_x62_row(static_cast<const float*>(A), lda, static_cast<const float*>(B), ldb, static_cast<float*>(C),
                      ldc, M, N, K, cfg % 100000, max_blocks, geo.bias, stats, stats_ld, stats_rows, bb, geo.b3, stream);
  }
  const bool x6 = (cfg / 100000) % 10 == 1;
  cfg %= 100000;
  if (x6) return gather ? nt_x6_gat(GK_NT_UNIT_PASS) : nt_x6_row(GK_NT_UNIT_PASS);
  return gather ? nt_f32_gat(GK_NT_UNIT_PASS) : nt_f32_row(GK_NT_UNIT_PASS);
}

// fp32 grad-weight: cfg digit 100000 selects the bf16x6 products
// (digit 200000: register-staged bf16x6, plain row form only; -2 = refused)
static int tn_unit_f32x(bool gather, const float* G, int64_t ldg, const float* X, int64_t ldx, float* W, int64_t ldw,
                        int64_t M, int N, int K, int cfg, int splits, const ConvGeo& geo, const LazyArgs* lza,
                        hipStream_t stream) {
  const int fam = (cfg / 100000) % 10;
  if (fam == 3) return -2;   // pre-split B: forward / grad-input kernels only
  if (fam == 2) {
    if (gather || lza) return -2;
    tn_x62_row(G, ldg, X, ldx, W, ldw, M, N, K, cfg % 100000, splits, stream);
  } else if (fam == 1) {
    tn_unit_x6(gather, G, ldg, X, ldx, W, ldw, M, N, K, cfg % 100000, splits, geo, lza, stream);
  } else {
    tn_unit_f32(gather, G, ldg, X, ldx, W, ldw, M, N, K, cfg % 100000, splits, geo, lza, stream);
  }
  return 0;
}

// fp32 [R, S] (row stride ld) -> three bf16 planes [R][S / 32][3][32] (the B
// operand layout of the register-staged bf16x6 kernels, cfg family 3): one
// thread splits 8 consecutive elements (split3x8) and writes 3 x 16 bytes
__global__ __launch_bounds__(256) void split3_rows_kernel(const float* __restrict__ src, int64_t ld,
                                                          uint16_t* __restrict__ dst, int64_t R, int S) {
  const int64_t g8 = S / 8;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= R * g8) return;
  const int64_t r = t / g8;
  const int g = (int)(t - r * g8);
  const float* p = src + r * ld + 8 * g;
  bf16x8 h, m, l;
  split3x8(*reinterpret_cast<const f32x4*>(p), *reinterpret_cast<const f32x4*>(p + 4), h, m, l);
  uint16_t* d = dst + (r * (S / 32) + g / 4) * 96 + (g % 4) * 8;
  *reinterpret_cast<bf16x8*>(d) = h;
  *reinterpret_cast<bf16x8*>(d + 32) = m;
  *reinterpret_cast<bf16x8*>(d + 64) = l;
}

void split3_rows(const float* src, int64_t ld, void* dst, int64_t R, int S, hipStream_t stream) {
  const int64_t n = R * (S / 8);
  if (n <= 0) return;
  hipLaunchKernelGGL(split3_rows_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, src, ld,
                     static_cast<uint16_t*>(dst), R, S);
}

bool gemm_supported(int64_t N, int64_t K) { return N >= 64 && K >= 64 && N % 64 == 0 && K % 64 == 0; }


// Split-K epilogue: C = sum of the KZ fp32 planes (+ bias), with the epilogue
// of the fused kernel -- BatchNorm statistics partials of the output, or the
// BN-backward dz = mask ? dx + dy2 : 0 with sum(dz), sum(dz * h) -- one
// partial row per block ([gy][N] layout of bn_finalize_kernel).  Block: 64
// column quads x 4 row lanes over a contiguous row range.
__global__ __launch_bounds__(256) void nt_splitk_reduce_kernel(const float* __restrict__ ws, int S, int64_t M, int N,
                                                               float* __restrict__ C, int64_t ldc,
                                                               const float* __restrict__ bias,
                                                               float* __restrict__ stats, int64_t stats_ld,
                                                               int64_t rows_per_block, BnBwd bb) {
  const int q = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int n = (blockIdx.y * 64 + q) * 4;
  const bool colok = n < N;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = r0 + rows_per_block < M ? r0 + rows_per_block : M;
  const int64_t plane = M * (int64_t)N;
  const float* hp = static_cast<const float*>(bb.h);
  const float* d2p = static_cast<const float*>(bb.dy2);
  f32x4 b = f32x4{0.f, 0.f, 0.f, 0.f};
  if (bias && colok) b = *reinterpret_cast<const f32x4*>(bias + n);
  float ps[4] = {0.f, 0.f, 0.f, 0.f}, pq[4] = {0.f, 0.f, 0.f, 0.f};
  if (colok) {
    for (int64_t m = r0 + rl; m < r1; m += 4) {
      const float* src = ws + m * N + n;
      f32x4 v = *reinterpret_cast<const f32x4*>(src);
      for (int z = 1; z < S; ++z) v += *reinterpret_cast<const f32x4*>(src + z * plane);
      v += b;
      if (hp) {
        const f32x4 hv = *reinterpret_cast<const f32x4*>(hp + m * ldc + n);
        const f32x4 d2 = d2p ? *reinterpret_cast<const f32x4*>(d2p + m * ldc + n) : f32x4{0.f, 0.f, 0.f, 0.f};
        const uint32_t bits = bb.mask ? (uint32_t)bb.mask[m * (N >> 2) + (n >> 2)] : 0xfu;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float dz = (bits >> r) & 1u ? v[r] + d2[r] : 0.f;
          v[r] = dz;
          ps[r] += dz;
          pq[r] = fmaf(dz, hv[r], pq[r]);
        }
      } else if (stats) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          ps[r] += v[r];
          pq[r] = fmaf(v[r], v[r], pq[r]);
        }
      }
      *reinterpret_cast<f32x4*>(C + m * ldc + n) = v;
    }
  }
  if (!stats) return;
  __shared__ float red[2][4][256];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    red[0][rl][q * 4 + r] = ps[r];
    red[1][rl][q * 4 + r] = pq[r];
  }
  __syncthreads();
  const int c = threadIdx.x;   // 256 columns of this block
  const int nc = blockIdx.y * 256 + c;
  if (nc < N) {
    const float sa = (red[0][0][c] + red[0][1][c]) + (red[0][2][c] + red[0][3][c]);
    const float sb = (red[1][0][c] + red[1][1][c]) + (red[1][2][c] + red[1][3][c]);
    stats[(int64_t)blockIdx.x * N + nc] = sa;
    stats[stats_ld + (int64_t)blockIdx.x * N + nc] = sb;
  }
}

int splitk_reduce(const float* ws, int S, int64_t M, int N, float* C, int64_t ldc, const float* bias, float* stats,
                  int stats_rows, const BnBwdArgs* bn, hipStream_t stream) {
  const BnBwd bb = bn ? BnBwd{bn->h, bn->dy2, bn->mask} : BnBwd{};
  const int ny = (N + 255) / 256;
  int64_t gx = 1024 / ny;
  const int64_t rmax = (M + 3) / 4;
  if (gx > rmax) gx = rmax;
  if (stats && gx > stats_rows) gx = stats_rows;
  if (gx < 1) gx = 1;
  const int64_t rpb = (M + gx - 1) / gx;
  gx = (M + rpb - 1) / rpb;
  hipLaunchKernelGGL(nt_splitk_reduce_kernel, dim3((unsigned)gx, (unsigned)ny), dim3(256), 0, stream, ws, S, M, N, C,
                     ldc, bias, stats, (int64_t)stats_rows * N, rpb, bb);
  return (int)gx;
}

int gemm_nt(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int64_t M, int N, int K,
            bool f32, int cfg, int max_blocks, float* stats, int stats_rows, const float* bias, const BnBwdArgs* bn,
            const LazyArgs* lazy, hipStream_t stream, float* splitk_ws, const void* b3) {
  ConvGeo g{};
  g.bias = bias;
  g.b3 = static_cast<const uint16_t*>(b3);
  const BnBwd bb = bn ? BnBwd{bn->h, bn->dy2, bn->mask} : BnBwd{};
  const int64_t sld = (int64_t)stats_rows * N;
  const int S = (cfg / 10000) % 10;
  const int x6 = cfg / 100000 * 100000;   // bf16x6 digit, kept for the split-K planes
  if (S > 1) {
    // split-K (fp32 row GEMM, host-checked: K % (64 S) == 0, no lazy operand):
    // KZ plain partial planes into splitk_ws [S][M][N], then the reduce epilogue
    if (!f32 || lazy || splitk_ws == nullptr || K % (64 * S) != 0) return -1;
    ConvGeo gz{};
    gz.KZ = S;
    const int r = nt_unit_f32(false, A, lda, B, ldb, splitk_ws, N, M, N, K / S, x6 + cfg % 10000, max_blocks, gz,
                                            nullptr, 0, 0, BnBwd{}, nullptr, stream);
    if (r < 0) return r;
    return splitk_reduce(splitk_ws, S, M, N, static_cast<float*>(C), ldc, bias, stats, stats_rows, bn, stream);
  }
  return f32 ? nt_unit_f32(false, A, lda, B, ldb, C, ldc, M, N, K, cfg, max_blocks, g, stats, sld, stats_rows, bb, lazy, stream)
             : nt_unit_b16(false, A, lda, B, ldb, C, ldc, M, N, K, cfg, max_blocks, g, stats, sld, stats_rows, bb, nullptr, stream);
}

int conv_nt(const void* X, const void* zero, int H, int W, int C, int OH, int OW, int S, int P, int KH, int KW,
            const void* B, void* Y, int64_t M, int N, bool f32, int cfg, int max_blocks, float* stats, int stats_rows,
            const float* bias, const BnBwdArgs* bn, const LazyArgs* lazy, hipStream_t stream, float* splitk_ws, const void* b3) {
  ConvGeo g{zero, H, W, C, OH, OW, S, P, KW, bias};
  g.b3 = static_cast<const uint16_t*>(b3);
  const int K = KH * KW * C;
  const int SK = (cfg / 10000) % 10;
  const int x6 = cfg / 100000 * 100000;
  if (SK > 1) {
    // split-K over the (tap, channel) slices: plain partial planes, then the reduce epilogue
    const int nks = K / 32;   // fp32 K slices
    if (!f32 || lazy || splitk_ws == nullptr || nks % SK != 0 || C % 32 != 0) return -1;
    ConvGeo gz{zero, H, W, C, OH, OW, S, P, KW, nullptr};
    gz.KZ = SK;
    const int r = nt_unit_f32(true, X, C, B, K, splitk_ws, N, M, N, K / SK, x6 + cfg % 10000, max_blocks, gz,
                                           nullptr, 0, 0, BnBwd{}, nullptr, stream);
    if (r < 0) return r;
    return splitk_reduce(splitk_ws, SK, M, N, static_cast<float*>(Y), N, bias, stats, stats_rows, bn, stream);
  }
  const BnBwd bb = bn ? BnBwd{bn->h, bn->dy2, bn->mask} : BnBwd{};
  const int64_t sld = (int64_t)stats_rows * N;
  return f32 ? nt_unit_f32(true, X, C, B, K, Y, N, M, N, K, cfg, max_blocks, g, stats, sld, stats_rows, bb, lazy, stream)
             : nt_unit_b16(true, X, C, B, K, Y, N, M, N, K, cfg, max_blocks, g, stats, sld, stats_rows, bb, nullptr, stream);
}

int conv_nt_remap(const void* X, int64_t ldx, const void* zero, int H, int W, int C, int OH, int OW, int KH, int KW,
                  const void* B, void* Y, int64_t M, int N, int RH, int RW, int RA, int RB, int RZ, bool f32, int cfg,
                  int max_blocks, const LazyArgs* lazy, hipStream_t stream) {
  ConvGeo g{zero, H, W, C, OH, OW, 1, 0, KW, nullptr, RH, RW, RA, RB, RZ};
  const int K = KH * KW * C;
  if (KH * KW == 1) {   // one tap at the class pixel itself: the plain row GEMM
    return f32 ? nt_unit_f32(false, X, ldx, B, K, Y, N, M, N, K, cfg, max_blocks, g, nullptr, 0, 0, BnBwd{}, lazy, stream)
               : nt_unit_b16(false, X, ldx, B, K, Y, N, M, N, K, cfg, max_blocks, g, nullptr, 0, 0, BnBwd{}, nullptr, stream);
  }
  return f32 ? nt_unit_f32(true, X, C, B, K, Y, N, M, N, K, cfg, max_blocks, g, nullptr, 0, 0, BnBwd{}, lazy, stream)
             : nt_unit_b16(true, X, C, B, K, Y, N, M, N, K, cfg, max_blocks, g, nullptr, 0, 0, BnBwd{}, nullptr, stream);
}

int gemm_tn_acc(const void* G, int64_t ldg, const void* X, int64_t ldx, float* W, int64_t ldw, int64_t M, int N,
                 int K, bool f32, int cfg, int splits, const LazyArgs* lazy, hipStream_t stream) {
  if (f32)
    return tn_unit_f32x(false, static_cast<const float*>(G), ldg, static_cast<const float*>(X), ldx, W, ldw, M, N, K, cfg,
                           splits, ConvGeo{}, lazy, stream);
  tn_unit_b16(false, G, ldg, X, ldx, W, ldw, M, N, K, cfg, splits, ConvGeo{}, stream);
  return 0;
}

int conv_tn_acc(const void* G, const void* X, const void* zero, int H, int W_, int C, int OH, int OW, int S, int P,
                 int KH, int KW, float* Wout, int64_t M, int N, bool f32, int cfg, int splits, const LazyArgs* lazy,
                 hipStream_t stream) {
  ConvGeo g{zero, H, W_, C, OH, OW, S, P, KW, nullptr};
  const int K = KH * KW * C;
  if (f32)
    return tn_unit_f32x(true, static_cast<const float*>(G), N, static_cast<const float*>(X), C, Wout, K, M, N, K, cfg,
                          splits, g, lazy, stream);
  tn_unit_b16(true, G, N, X, C, Wout, K, M, N, K, cfg, splits, g, stream);
  return 0;
}

}  // namespace gk
