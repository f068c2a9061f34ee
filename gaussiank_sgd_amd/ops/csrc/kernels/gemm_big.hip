// Large-tile bf16 GEMM for the transformer linears (BERT-base: M = 16384 rows,
// K and N in {768, 2304, 3072}):  C[M, N] = A[M, K] . B[N, K]^T (+ bias), bf16
// operands, fp32 accumulation, bf16 out.
//
// gemm.hip's gemm_nt is built for convolution shapes (K of 64..512, 64x64 wave
// tiles, persistent over M); on these K >= 768 linears hipBLASLt's 256x256
// macro tiles beat it by 15-35% (autotune dump, round 3).  This kernel is the
// large-tile design: a 2x2-wave block owns a (2 TM) x (2 TN) output tile, each
// wave TM x TN (128 x 128: 16 v_mfma_f32_32x32x16_bf16 accumulators, 256 fp32
// registers -- accumulation VGPRs, one wave per SIMD), so every 16-byte LDS
// fragment feeds TN/32 (or TM/32) MFMAs and the LDS read traffic is half that of
// 64x64 wave tiles.  K advances in 64-wide slices (one 128-byte row per staged
// row) through two LDS stages filled by LDS-DMA (global_load_lds, 16 B per
// lane) one slice ahead; the 16-byte chunks of a row are XOR-swizzled by
// (row >> 1) & 7 (the gemm.hip swizzle: a 16-lane pass of ds_read_b128 over
// rows r..r+15 at one chunk covers all 64 banks).  The weights are the MFMA A
// operand, the activations B, so a lane ends with 4 consecutive output
// channels of one row per register group: 8-byte stores.  Blocks are
// remapped so the N tiles of one M row of tiles run on one XCD (shared A rows
// in its L2).
#include <hip/hip_runtime.h>

#include "common.h"
#include "gk_kernels.h"
#include "mfma_util.h"

namespace gk {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int bswz(int r) { return (r >> 1) & 7; }

template <int TM, int TN>
struct BigCfg {
  static constexpr int WM = 2, WN = 2;
  static constexpr int THREADS = 64 * WM * WN;
  static constexpr int BM = WM * TM, BN = WN * TN;
  static constexpr int STAGE = (BM + BN) * 128;   // bytes: one 64-wide K slice of the A and B rows
  static constexpr int LDS = 2 * STAGE;
  static constexpr int INSTS = STAGE / 1024;       // 1-KiB LDS-DMA instructions per stage (8 rows each)
  static_assert(INSTS % (WM * WN) == 0, "stage split");
  static constexpr int LPW = INSTS / (WM * WN);
  static constexpr int MT = TM / 32, NT = TN / 32;
};

template <int TM, int TN>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1)))
gemm_big_nt_kernel(const uint16_t* __restrict__ A, int64_t lda, const uint16_t* __restrict__ B, int64_t ldb,
                   uint16_t* __restrict__ C, int64_t ldc, int M, int N, int K, const float* __restrict__ bias) {
  using Cfg = BigCfg<TM, TN>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave / Cfg::WN, wn = wave % Cfg::WN;
  const int ntiles = N / Cfg::BN;
  const int nb = (M / Cfg::BM) * ntiles;
  // consecutive logical tiles (one M row of tiles) on one XCD: hardware block b runs on XCD b % 8
  const int b = blockIdx.x;
  const int logical = (nb & 7) == 0 ? (b & 7) * (nb >> 3) + (b >> 3) : b;
  const int m0 = (logical / ntiles) * Cfg::BM, n0 = (logical % ntiles) * Cfg::BN;
  const int nk = K / 64;

  // stage K slice ks into LDS buffer s: lane (row-in-8 = lane >> 3, chunk
  // position lane & 7) fetches the logical chunk that position holds
  auto stage = [&](int ks, int s) __attribute__((always_inline)) {
    GK_LDS char* base = (GK_LDS char*)smem + s * Cfg::STAGE;
#pragma unroll
    for (int i = 0; i < Cfg::LPW; ++i) {
      const int inst = wave * Cfg::LPW + i;
      const int row = inst * 8 + (lane >> 3);
      const int lch = (lane & 7) ^ bswz(row);
      const uint16_t* src = row < Cfg::BM ? A + (int64_t)(m0 + row) * lda + ks * 64 + lch * 8
                                          : B + (int64_t)(n0 + row - Cfg::BM) * ldb + ks * 64 + lch * 8;
      glds16(src, base + inst * 1024);
    }
  };

  f32x16 acc[Cfg::MT][Cfg::NT];
#pragma unroll
  for (int i = 0; i < Cfg::MT; ++i)
#pragma unroll
    for (int j = 0; j < Cfg::NT; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int r = lane & 31, h = lane >> 5;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int ks = 0; ks < nk; ++ks) {
    if (ks + 1 < nk) stage(ks + 1, (ks + 1) & 1);
    const char* S = smem + (ks & 1) * Cfg::STAGE;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int c = kk * 2 + h;   // logical 16-byte chunk: k = 16 kk + 8 h .. +7
      bf16x8 wa[Cfg::NT], xb[Cfg::MT];
#pragma unroll
      for (int j = 0; j < Cfg::NT; ++j) {
        const int row = Cfg::BM + wn * TN + j * 32 + r;
        wa[j] = *reinterpret_cast<const bf16x8*>(S + row * 128 + ((c ^ bswz(row)) << 4));
      }
#pragma unroll
      for (int i = 0; i < Cfg::MT; ++i) {
        const int row = wm * TM + i * 32 + r;
        xb[i] = *reinterpret_cast<const bf16x8*>(S + row * 128 + ((c ^ bswz(row)) << 4));
      }
#pragma unroll
      for (int i = 0; i < Cfg::MT; ++i)
#pragma unroll
        for (int j = 0; j < Cfg::NT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[j], xb[i], acc[i][j], 0, 0, 0);
    }
    // the next slice's LDS-DMA landed and every wave is done with this buffer
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // D[n][m]: lane holds m = col (lane & 31), n = (reg & 3) + 8 (reg >> 2) + 4 h
#pragma unroll
  for (int j = 0; j < Cfg::NT; ++j) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int n = n0 + wn * TN + j * 32 + 8 * g + 4 * h;
      float bv[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) bv[e] = bias ? bias[n + e] : 0.f;
#pragma unroll
      for (int i = 0; i < Cfg::MT; ++i) {
        const int m = m0 + wm * TM + i * 32 + r;
        const f32x16 a = acc[i][j];
        uint2 v;
        v.x = pack_bf16x2(a[4 * g + 0] + bv[0], a[4 * g + 1] + bv[1]);
        v.y = pack_bf16x2(a[4 * g + 2] + bv[2], a[4 * g + 3] + bv[3]);
        *reinterpret_cast<uint2*>(C + (int64_t)m * ldc + n) = v;
      }
    }
  }
}

template <int TM, int TN>
void launch_big(const uint16_t* A, int64_t lda, const uint16_t* B, int64_t ldb, uint16_t* C, int64_t ldc, int M,
                int N, int K, const float* bias, hipStream_t stream) {
  using Cfg = BigCfg<TM, TN>;
  static bool attr = [] {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_big_nt_kernel<TM, TN>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, Cfg::LDS) == hipSuccess;
  }();
  (void)attr;
  const int nb = (M / Cfg::BM) * (N / Cfg::BN);
  hipLaunchKernelGGL((gemm_big_nt_kernel<TM, TN>), dim3((unsigned)nb), dim3(Cfg::THREADS), Cfg::LDS, stream, A, lda, B,
                     ldb, C, ldc, M, N, K, bias);
}

}  // namespace

// cfg 0: 256 x 256 block tiles (128 x 128 per wave); 1: 128 x 256 (64 x 128);
// 2: 256 x 128 (128 x 64).  Returns false (nothing launched) when the shape
// does not divide into the tile.
bool gemm_big_supported(int64_t M, int64_t N, int64_t K, int cfg) {
  const int bm = cfg == 1 ? 128 : 256, bn = cfg == 2 ? 128 : 256;
  return M > 0 && M % bm == 0 && N % bn == 0 && K % 64 == 0 && K >= 64 && M < (int64_t(1) << 31);
}

bool gemm_big_nt(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int64_t M, int N, int K,
                 int cfg, const float* bias, hipStream_t stream) {
  if (!gemm_big_supported(M, N, K, cfg)) return false;
  const auto* a = static_cast<const uint16_t*>(A);
  const auto* b = static_cast<const uint16_t*>(B);
  auto* c = static_cast<uint16_t*>(C);
  switch (cfg) {
    case 1: launch_big<64, 128>(a, lda, b, ldb, c, ldc, (int)M, N, K, bias, stream); break;
    case 2: launch_big<128, 64>(a, lda, b, ldb, c, ldc, (int)M, N, K, bias, stream); break;
    default: launch_big<128, 128>(a, lda, b, ldb, c, ldc, (int)M, N, K, bias, stream); break;
  }
  return true;
}

}  // namespace gk
