// Kernel templates of the hand-written MFMA GEMMs (gemm.hip: public entry
// points; gemm_inst.hip: one instantiation unit per operand type / row-vs-
// gather form, compiled in parallel -- see ops/build.py GEMM_UNITS).
//
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
#pragma once

#ifndef GK_XCD_REMAP
#define GK_XCD_REMAP 1   // XCD-aware block order of gemm_nt (0: identity, A/B builds)
#endif
#ifndef GK_X6_SCHED
#define GK_X6_SCHED 1   // software-pipelined bf16x6 loop (0: the first form, A/B builds)
#endif
#ifndef GK_X6_EXP
#define GK_X6_EXP 0   // bf16x6 kernel experiments (variant builds only)
#endif
#include <hip/hip_runtime.h>

#include <type_traits>

#include "common.h"
#include "gk_kernels.h"
#include "mfma_util.h"
namespace gk {

// Implicit-GEMM convolution: row m of the A operand is output pixel
// (n, oh, ow) and K slice k0 (64 channels) is tap (kh, kw) of input channels
// c0..c0+63 (K = KH*KW*C, tap-major, matching a channels-last [Cout][KH][KW][C]
// weight).  Out-of-image taps read a zero row (padding) -- LDS-DMA cannot write
// zeros itself.
constexpr int kMaxTaps = 4;   // gemm_nt gather: at most 4 taps per kernel dimension

struct ConvGeo {
  const void* zero;       // >= 128 zero bytes (one K slice row of either element type)
  int H, W, C, OH, OW, S, P, KW;
  const float* bias;      // optional per-output-channel bias (gemm_nt / conv_nt epilogue)
  // gemm_nt output row remap (stride-2 grad-input parity classes): RH > 0 stores
  // row m = (n, oh, ow) of the OH x OW class grid at image row
  // (n * RH + 2 oh + RA) * RW + 2 ow + RB of the RH x RW output; RZ also writes
  // zeros to the three other parity positions (1x1 stride-2: those get no tap)
  int RH, RW, RA, RB, RZ;
  // gemm_nt split-K (row GEMMs only): KZ > 1 launches KZ planes along z, plane z
  // multiplies K slices [z K, (z + 1) K) of A and B into its own fp32 output
  // plane C + z M ldc (plain epilogue); nt_splitk_reduce_kernel sums the planes
  int KZ;
  // bf16x6 register-staged kernels, cfg family 3: the B operand already split
  // into three bf16 planes, [N][K / 32][3][32] (split3_rows); nullptr otherwise
  const uint16_t* b3;
};

// BatchNorm-backward epilogue (grad-input GEMM of the convolution that consumes
// a fused BN + ReLU [+ residual] output): instead of the plain gradient dy the
// kernel stores dz = relu_mask ? bf16(dy) + dy2 : 0 (dy2: the BN output's second
// consumer's gradient, ResNet shortcut) and reduces per-channel partials
// sum(dz) and sum(dz * h) (h: the BN input) into `stats`, which is what the BN
// backward's separate reduction pass would read dy, dy2, h and the mask for.
// The operands are loaded per output row in the epilogue (transient registers:
// the main loop's register budget is unchanged).
struct BnBwd {
  const void* h;          // BN input [M, N] (same ld and element type as C); nullptr: plain epilogue
  const void* dy2;        // optional second gradient [M, N]
  const uint8_t* mask;    // optional 1-bit ReLU mask, one byte per 16-byte vector: (m, n / V) at
                          // m * (N / V) + n / V, V = 8 (bf16) or 4 (fp32) -- bn_act.hip's layout
};

// Lazy BatchNorm-backward operand (fp32): the A operand (NT) / G operand (TN)
// is the gradient of a BN input, dx = k1 ((dz - k2) - (x - mu) k4), which is
// never materialised -- the kernel stages dz AND x tiles and applies the
// per-channel affine map after its LDS reads (bn_act.hip bn_bwd_finalize_lazy
// makes coef[c] = {k1, k2, mu, k4}).  Padding taps load the rows padz = k2 and
// padx = mu, so they contribute exactly 0.  The BN's apply pass (read dz and
// x, write dx) disappears; the two consumers (grad-input and grad-weight of
// the producing convolution) read dz and x instead of dx.
struct LazyA {
  const void* x;          // BN input, same layout / strides as the dz operand
  const float* coef;      // [C] x {k1, k2, mu, k4}
  const void* padz;       // [C] padding row of dz (k2)
  const void* padx;       // [C] padding row of x (mu)
  int C;                  // channels of dz (coefficient table length)
};

// per-unit dispatchers (gemm_inst.hip, one object per GK_GEMM_UNIT)
#define GK_NT_UNIT_ARGS                                                                                      \
  const void *A, int64_t lda, const void *B, int64_t ldb, void *C, int64_t ldc, int64_t M, int N, int K, int cfg, \
      int max_blocks, const ConvGeo &geo, float *stats, int64_t stats_ld, int stats_rows, const BnBwd &bb,      \
      const LazyArgs *lza, hipStream_t stream
#define GK_NT_UNIT_PASS A, lda, B, ldb, C, ldc, M, N, K, cfg, max_blocks, geo, stats, stats_ld, stats_rows, bb, lza, stream
int nt_b16_row(GK_NT_UNIT_ARGS);   // unit 0
int nt_b16_gat(GK_NT_UNIT_ARGS);   // unit 1
int nt_f32_row(GK_NT_UNIT_ARGS);   // unit 2
int nt_f32_gat(GK_NT_UNIT_ARGS);   // unit 3
int nt_x6_row(GK_NT_UNIT_ARGS);    // unit 5: fp32 operands, bf16x6 products
int nt_x6_gat(GK_NT_UNIT_ARGS);    // unit 6
// unit 8: fp32 row GEMMs, bf16x6 with register staging (gemm_nt_x62_kernel)
int nt_x62_row(const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc, int64_t M, int N, int K,
               int cfg, int max_blocks, const float* bias, float* stats, int64_t stats_ld, int stats_rows,
               const BnBwd& bb, const uint16_t* b3, hipStream_t stream);
// unit 10: implicit-GEMM convolutions, bf16x6 with register staging
int nt_x62_gat(const float* A, const float* B, float* C, int64_t M, int N, int K, int cfg, int max_blocks,
               const ConvGeo& geo, float* stats, int64_t stats_ld, int stats_rows, const BnBwd& bb,
               hipStream_t stream);
// unit 9: fp32 row grad-weight GEMMs, bf16x6 with register staging (gemm_tn_x62_kernel)
void tn_x62_row(const float* G, int64_t ldg, const float* X, int64_t ldx, float* W, int64_t ldw, int64_t M, int N,
                int K, int cfg, int splits, hipStream_t stream);
// unit 7: fp32 grad-weight (TN) GEMMs with bf16x6 products
void tn_unit_x6(bool gather, const float* G, int64_t ldg, const float* X, int64_t ldx, float* W, int64_t ldw,
                int64_t M, int N, int K, int cfg, int splits, const ConvGeo& geo, const LazyArgs* lza,
                hipStream_t stream);
// unit 4: grad-weight (TN) GEMMs, both operand types and forms
void tn_unit_b16(bool gather, const void* G, int64_t ldg, const void* X, int64_t ldx, float* W, int64_t ldw, int64_t M,
                 int N, int K, int cfg, int splits, const ConvGeo& geo, hipStream_t stream);
void tn_unit_f32(bool gather, const float* G, int64_t ldg, const float* X, int64_t ldx, float* W, int64_t ldw,
                 int64_t M, int N, int K, int cfg, int splits, const ConvGeo& geo, const LazyArgs* lza,
                 hipStream_t stream);

namespace {

__device__ __forceinline__ int swz(int r) { return (r >> 1) & 7; }

// XCD-aware block order.  The hardware deals workgroups round-robin over the 8
// XCDs (linear id L -> XCD L % 8; relied on for speed only, never for
// correctness) and every XCD has its own L2.  With the identity order each XCD
// gets 1/8 of every row and column of the (x = M start, y = N tile) grid, so
// every XCD streams every A tile and every weight panel from HBM.  Instead XCD
// k runs the contiguous logical range [k G/8, (k+1) G/8): x fastest when there
// are >= 8 N tiles (an XCD keeps gy/8 weight panels in its L2 and its blocks
// read each A tile once per XCD), y fastest otherwise (every panel, a slice of
// the M tiles).  A bijection whenever 8 divides the grid; identity otherwise.
__device__ __forceinline__ void xcd_remap2(int& bx, int& by) {
  const int gx = (int)gridDim.x, gy = (int)gridDim.y, G = gx * gy;
  bx = (int)blockIdx.x;
  by = (int)blockIdx.y;
  if (!GK_XCD_REMAP || (G & 7) != 0 || G < 16) return;
  const int L = bx + by * gx;
  const int q = (L & 7) * (G >> 3) + (L >> 3);
  if (gy >= 8) {
    bx = q % gx;
    by = q / gx;
  } else {
    by = q % gy;
    bx = q / gy;
  }
}

// The same for the grad-weight grids (x = N tile, y = K tile, z = M split):
// XCD k runs a contiguous range of the x-fastest logical order, i.e. whole
// M splits, so the G and X rows of a split are fetched by one XCD instead of
// by every XCD holding one of its (x, y) tiles.
__device__ __forceinline__ void xcd_remap3(int& bx, int& by, int& bz) {
  const int gx = (int)gridDim.x, gy = (int)gridDim.y, gz = (int)gridDim.z, G = gx * gy * gz;
  bx = (int)blockIdx.x;
  by = (int)blockIdx.y;
  bz = (int)blockIdx.z;
  if (!GK_XCD_REMAP || (G & 7) != 0 || G < 16) return;
  const int L = bx + (by + bz * gy) * gx;
  const int q = (L & 7) * (G >> 3) + (L >> 3);
  bx = q % gx;
  by = (q / gx) % gy;
  bz = q / (gx * gy);
}

// s_waitcnt vmcnt(n) for a wave-uniform runtime n: waits until at most n of
// this wave's vector-memory operations (loads, stores, LDS-DMA; they retire
// in issue order) are still in flight.
template <int N>
__device__ __forceinline__ void vmcnt_le() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

__device__ __forceinline__ void wait_vmcnt(int n) {
#define GK_VMW(k) \
  case k: vmcnt_le<k>(); break;
  switch (n) {
    GK_VMW(0) GK_VMW(1) GK_VMW(2) GK_VMW(3) GK_VMW(4) GK_VMW(5) GK_VMW(6) GK_VMW(7) GK_VMW(8) GK_VMW(9)
    GK_VMW(10) GK_VMW(11) GK_VMW(12) GK_VMW(13) GK_VMW(14) GK_VMW(15) GK_VMW(16) GK_VMW(17) GK_VMW(18)
    GK_VMW(19) GK_VMW(20) GK_VMW(21) GK_VMW(22) GK_VMW(23) GK_VMW(24) GK_VMW(25) GK_VMW(26) GK_VMW(27)
    GK_VMW(28) GK_VMW(29) GK_VMW(30) GK_VMW(31) GK_VMW(32) GK_VMW(33) GK_VMW(34) GK_VMW(35) GK_VMW(36)
    GK_VMW(37) GK_VMW(38) GK_VMW(39) GK_VMW(40) GK_VMW(41) GK_VMW(42) GK_VMW(43) GK_VMW(44) GK_VMW(45)
    GK_VMW(46) GK_VMW(47) GK_VMW(48) GK_VMW(49) GK_VMW(50) GK_VMW(51) GK_VMW(52) GK_VMW(53) GK_VMW(54)
    GK_VMW(55) GK_VMW(56) GK_VMW(57) GK_VMW(58) GK_VMW(59) GK_VMW(60) GK_VMW(61) GK_VMW(62) GK_VMW(63)
    default: vmcnt_le<0>(); break;
  }
#undef GK_VMW
}

// wait_vmcnt with the loop's steady-state count as a compile-time fast path:
// the generic switch compiles to a compare-and-branch chain (~15 scalar
// instructions per K step); the steady state is one compare.
template <int COMMON>
__device__ __forceinline__ void wait_vmcnt_fast(int n) {
  if (n == COMMON) vmcnt_le<COMMON>();
  else wait_vmcnt(n);
}

// --------------------------------------------------------------------------
// gemm_nt
// --------------------------------------------------------------------------
// BRES: the block's whole weight panel [BN x K] stays resident in LDS (it is
// the same for every M tile of the persistent loop); only A is streamed.
// NS: LDS stages; NS = 3 keeps two K slices in flight behind the one being
// multiplied.
// MSB: 16-row MFMA subtiles per wave along M (4: 64x64 wave tile, 8: 128x64 --
// fewer LDS reads per MFMA for the compute-bound shapes; bf16 only).
// T: element type, uint16_t (bf16 bits) or float.  A K slice is always one
// 128-byte LDS row per staged row -- 64 bf16 or 32 fp32 -- so staging,
// swizzle and fragment addressing are shared; a 16-byte fragment feeds one
// v_mfma_f32_16x16x32_bf16 (bf16) or four v_mfma_f32_16x16x4_f32 (fp32, exact
// fp32 products and sums: the reference's precision, no bf16 splitting).
template <typename T>
struct Elem {
  static constexpr bool F32 = sizeof(T) == 4;
  static constexpr int EPC = 16 / (int)sizeof(T);   // elements per 16-byte chunk
  static constexpr int KS = 8 * EPC;                // K elements per 128-byte slice row
  // 16-byte epilogue stores per 16-row subtile per wave (64 output columns)
  static constexpr int ST_PER_SUB = F32 ? 4 : 2;
};

template <int WM, int WN, bool BRES, int MSB = 4, typename T = uint16_t, bool LZ = false>
struct NtCfg {
  static constexpr int NW = WM * WN;
  static constexpr int THREADS = 64 * NW;
  static constexpr int WTM = 16 * MSB;            // wave tile rows
  static constexpr int BM = WTM * WM;
  static constexpr int BN = 64 * WN;
  static constexpr int ASTAGE = BM * 128;         // bytes: BM rows x one K slice
  static constexpr int NACOPY = LZ ? 2 : 1;       // lazy BN operand: dz and x tiles
  static constexpr int ASTAGES = NACOPY * ASTAGE;
  static constexpr int BSTAGE = BN * 128;
  static constexpr int STAGE = BRES ? ASTAGES : ASTAGES + BSTAGE;
  static constexpr int INSTS = STAGE / 1024;      // 1-KiB LDS-DMA instructions per stage
  static_assert(INSTS % NW == 0, "stage split");
  static constexpr int LPW = INSTS / NW;          // LDS-DMA instructions per wave per stage
  static_assert((BM / 8) % NW == 0, "A rows split evenly over the waves");
  static constexpr int LPWA = BRES ? LPW : NACOPY * (BM / 8) / NW;   // of which A-row instructions (j < LPWA)
  static constexpr int NST = Elem<T>::ST_PER_SUB * MSB;     // 16-byte epilogue stores per wave per tile
  static_assert(NST <= 63, "wait_vmcnt range (vmcnt is 6 bits)");
  static constexpr bool NS3_OK = LPW + 2 * NST <= 63;       // three stages: 1 stage + 2 tiles of stores in flight
  static constexpr bool NS4_OK = 2 * LPW + 3 * NST <= 63;   // four stages: 2 stages + 3 tiles of stores in flight
  // LDS: [lazy coefficient table][resident weight panel][stages]
  __host__ __device__ static int coef_bytes(int C) { return LZ ? ((C * 16 + 1023) / 1024) * 1024 : 0; }
  static int lds_bytes(int K, int ns, int C = 0) {
    return ns * STAGE + (BRES ? BN * K * (int)sizeof(T) : 0) + coef_bytes(C);
  }
};

template <int WM, int WN, bool BRES, int NS, bool GATHER, int MSB = 4, bool BNB = false, typename T = uint16_t,
          bool LZ = false, bool X6 = false>
__global__ void __launch_bounds__(64 * WM * WN) __attribute__((amdgpu_waves_per_eu(WM * WN >= 8 ? 1 : 2)))
gemm_nt_kernel(const T* __restrict__ A, int64_t lda, const T* __restrict__ B, int64_t ldb,
               T* __restrict__ C, int64_t ldc, int64_t M, int K, ConvGeo geo, float* __restrict__ stats,
               int64_t stats_ld, BnBwd bb, LazyA lz) {
  // stats != nullptr: per-block BatchNorm partials of the (dtype-rounded)
  // output, psum at stats[bx * N + n], psq at stats[stats_ld + ...]
  // (the [gy][C] layout bn_finalize_kernel reduces).  With bb.h (BN-backward
  // epilogue, MSB == 4 tiles only) the partials are sum(dz), sum(dz*h); the
  // finalize centres the second with the mean.
  using Cfg = NtCfg<WM, WN, BRES, MSB, T, LZ>;
  using E = Elem<T>;
  constexpr bool F32 = E::F32;
  static_assert(!LZ || F32, "lazy BN operand: fp32 kernels");
  static_assert(!X6 || F32, "bf16x6 products: fp32 operands");
  constexpr int EPC = E::EPC;
  constexpr int KS = E::KS;
  static_assert(!BNB || MSB == 4 || F32, "bf16 BN-backward epilogue: 64x64 wave tiles");
  static_assert(!F32 || MSB == 4 || MSB == 2 || (X6 && MSB == 8), "fp32: 64x64 or 32x64 wave tiles (bf16x6: 128x64)");
  static_assert(NS == 2 || (NS == 3 && Cfg::NS3_OK) || (NS == 4 && Cfg::NS4_OK), "wait_vmcnt range (vmcnt is 6 bits)");
  constexpr bool bnb = BNB;
  static_assert(NS >= 2 && NS <= 4, "stages");
  constexpr int LPW = Cfg::LPW;
  // split-K plane (ConvGeo::KZ): K is the per-plane depth; a gathered A starts
  // at the plane's first (tap, channel) slice instead of a column offset
  int kz_kh = 0, kz_kw = 0, kz_c0 = 0;
  if constexpr (!LZ) {
    if (gridDim.z > 1) {
      const int64_t z = blockIdx.z;
      if constexpr (GATHER) {
        const int per = geo.C / E::KS;   // K slices per tap
        const int s0 = (int)z * (K / E::KS);
        const int tap = s0 / per;
        kz_c0 = (s0 - tap * per) * E::KS;
        kz_kh = tap / geo.KW;
        kz_kw = tap - kz_kh * geo.KW;
      } else {
        A += z * K;
      }
      B += z * K;
      C += z * M * ldc;
    }
  }
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int bx, by;   // logical block coordinates (XCD-aware order)
  xcd_remap2(bx, by);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform: LDS-DMA M0 and fragment bases in SGPRs
  const int wm = wave / WN, wn = wave % WN;
  const int n0 = by * Cfg::BN;
  const int64_t mtiles = (M + Cfg::BM - 1) / Cfg::BM;
  const int nk = K / KS;
  // this block's work: M tiles bx, +gridDim.x, ...; each has nk K slices
  const int64_t my_tiles = bx < mtiles ? (mtiles - 1 - bx) / gridDim.x + 1 : 0;
  const int T_ = (int)(my_tiles * nk);
  const int Ntot = gridDim.y * Cfg::BN;
  if (T_ == 0) {
    if (stats)
      for (int c = threadIdx.x; c < Cfg::BN; c += Cfg::THREADS) {
        stats[(int64_t)bx * Ntot + n0 + c] = 0.f;
        stats[stats_ld + (int64_t)bx * Ntot + n0 + c] = 0.f;
      }
    return;
  }
  const int coefb = Cfg::coef_bytes(lz.C);
  char* panel = smem + coefb;
  char* stage_base = panel + (BRES ? Cfg::BN * K * (int)sizeof(T) : 0);
  if (LZ) {
    // lazy BN coefficients -> LDS (read back per fragment); drained before any
    // stage is issued, so the pipeline's vmcnt bookkeeping is untouched
    float4* ct = reinterpret_cast<float4*>(smem);
    const float4* cg = reinterpret_cast<const float4*>(lz.coef);
    for (int c = threadIdx.x; c < lz.C; c += Cfg::THREADS) ct[c] = cg[c];
    __syncthreads();
  }

  if (BRES) {  // weight panel: slice ks at panel + ks*BSTAGE, rows swizzled as the streamed tiles
    const int per = Cfg::BN / 8;
    for (int i = wave; i < nk * per; i += Cfg::NW) {
      const int ks = i / per, ri = i % per;
      const int r = ri * 8 + (lane >> 3);
      const int c = (lane & 7) ^ swz(r);
      glds16(B + (int64_t)(n0 + r) * ldb + ks * KS + c * EPC, (GK_LDS char*)panel + ks * Cfg::BSTAGE + ri * 1024);
    }
  }

  // ---- staging cursor: every per-lane address is set up once per M tile (A
  // rows) or once per kernel (B rows); a K step only adds the slice offset.
  // Instruction j of this wave fills staged rows i*8 .. i*8+7, i = wave + j*NW:
  // A rows while i*8 < BM, B rows after (streamed panel only).
  const T* ptr[LPW];          // A: row (or gathered pixel) base + chunk; B: row base + chunk
  // gather: bit kh of okh / bit kw of okw set when tap row kh / column kw of
  // this lane's output pixel lies inside the image (set once per M tile; a K
  // step tests two bits instead of recomputing and comparing the position)
  uint32_t okh[LPW], okw[LPW];
  const T* zrow[LPW];         // gather: this lane's chunk of the zero row (padding taps)
  // lazy operand: instructions i in [BM/8, 2 BM/8) stage the x tile; its
  // rows are the dz rows at a fixed element offset (same layout)
  const int64_t xoff = LZ ? static_cast<const T*>(lz.x) - A : 0;
#pragma unroll
  for (int j = 0; j < LPW; ++j) {
    const int i = wave + j * Cfg::NW;
    const int r = i * 8 + (lane >> 3);
    const int c = (lane & 7) ^ swz(r);
    const bool isx = LZ && i >= Cfg::BM / 8 && j < Cfg::LPWA;
    ptr[j] = j < Cfg::LPWA ? nullptr : B + (int64_t)(n0 + r - Cfg::NACOPY * Cfg::BM) * ldb + c * EPC;
    okh[j] = okw[j] = 0u;
    zrow[j] = !GATHER ? nullptr
              : LZ ? static_cast<const T*>(isx ? lz.padx : lz.padz) + c * EPC
                   : static_cast<const T*>(geo.zero) + c * EPC;
  }
  auto set_rows = [&](int64_t mt) {
    const int64_t m0 = mt * Cfg::BM;
#pragma unroll
    for (int j = 0; j < LPW; ++j) {
      const int i = wave + j * Cfg::NW;
      if (j < Cfg::LPWA) {
        const int ia = (LZ && i >= Cfg::BM / 8) ? i - Cfg::BM / 8 : i;   // row group within its A copy
        const int64_t xo = (LZ && i >= Cfg::BM / 8) ? xoff : 0;
        const int r = ia * 8 + (lane >> 3);
        const int c = (lane & 7) ^ swz(r);
        int64_t gr = m0 + r;
        gr = gr < M ? gr : M - 1;
        if (GATHER) {
          const uint32_t ohw = (uint32_t)(geo.OH * geo.OW);
          const uint32_t mu = (uint32_t)gr;
          const uint32_t n = mu / ohw, rem = mu - n * ohw;
          const uint32_t oh = rem / (uint32_t)geo.OW, ow = rem - oh * (uint32_t)geo.OW;
          const int ih0 = (int)oh * geo.S - geo.P;
          const int iw0 = (int)ow * geo.S - geo.P;
          uint32_t bh = 0u, bw = 0u;
#pragma unroll
          for (int q = 0; q < kMaxTaps; ++q) {   // host: KH, KW <= kMaxTaps
            bh |= (uint32_t)((unsigned)(ih0 + q) < (unsigned)geo.H) << q;
            bw |= (uint32_t)((unsigned)(iw0 + q) < (unsigned)geo.W) << q;
          }
          okh[j] = bh;
          okw[j] = bw;
          ptr[j] = A + xo + (((int64_t)n * geo.H + ih0) * geo.W + iw0) * geo.C + c * EPC;
        } else {
          ptr[j] = A + xo + gr * lda + c * EPC;
        }
      }
    }
  };
  int64_t s_mt = bx;    // tile of the next stage to issue
  int s_ks = 0;                 // its K slice
  int s_kh = kz_kh, s_kw = kz_kw, s_c0 = kz_c0;   // gather: tap and channel offset of that slice
  int s_t = 0;
  int s_buf = 0;                // LDS stage of the next issue (s_t % NS)
  set_rows(s_mt);
  // A stage is issued in three parts so the main loop can spread its LDS-DMA
  // instructions over the MFMA stream (stage_issue(j) between MFMA groups)
  // instead of issuing them back to back after the barrier, where their issue
  // cost (~60-180 cycles each among MFMAs, MI355X_MICROARCH.md LDS-DMA row)
  // left the matrix pipe idle at one wave per SIMD.
  GK_LDS char* st_base = nullptr;   // snapshot of the stage being issued
  int st_k0 = 0, st_kh = 0, st_kw = 0, st_c0 = 0;
  int64_t st_toff = 0;
  auto stage_prep = [&]() {
    st_base = (GK_LDS char*)stage_base + s_buf * Cfg::STAGE;
    st_k0 = s_ks * KS;
    st_toff = GATHER ? (int64_t)(s_kh * geo.W + s_kw) * geo.C + s_c0 : 0;   // wave-uniform
    st_kh = s_kh; st_kw = s_kw; st_c0 = s_c0;
  };
  auto stage_issue = [&](int j) {   // j: compile-time after unrolling
    const int i = wave + j * Cfg::NW;
    const T* src;
    if (j < Cfg::LPWA) {
      if (GATHER) {
        const bool ok = ((okh[j] >> st_kh) & (okw[j] >> st_kw) & 1u) != 0u;
        src = ok ? ptr[j] + st_toff : zrow[j] + (LZ ? st_c0 : 0);   // lazy: per-channel padding rows
      } else {
        src = ptr[j] + st_k0;
      }
    } else {
      src = ptr[j] + st_k0;
    }
    glds16(src, st_base + i * 1024);
  };
  auto stage_advance = [&]() {
    ++s_t;
    s_buf = s_buf + 1 == NS ? 0 : s_buf + 1;
    if (GATHER) {
      s_c0 += KS;
      if (s_c0 == geo.C) {
        s_c0 = 0;
        if (++s_kw == geo.KW) { s_kw = 0; ++s_kh; }
      }
    }
    if (++s_ks == nk) {
      s_ks = 0;
      s_kh = kz_kh; s_kw = kz_kw; s_c0 = kz_c0;
      s_mt += gridDim.x;
      if (s_t < T_) set_rows(s_mt);
    }
  };
  auto stage = [&]() {
    stage_prep();
#pragma unroll
    for (int j = 0; j < LPW; ++j) stage_issue(j);
    stage_advance();
  };

  f32x4 acc[MSB][4];
#pragma unroll
  for (int a = 0; a < MSB; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  stage();
  if (NS >= 3 && T_ > 1) stage();
  if (NS == 4 && T_ > 2) stage();
  const int fr = lane & 15, fq = lane >> 4;
  // stores issued by the last two steps (0 when none, or when a partial tile
  // drained its stores with vmcnt(0) right away)
  int st1 = 0, st2 = 0, st3 = 0;
  int ks = 0;
  int buf = 0;
  float ssum[4][4], ssq[4][4];   // BN partials: [ns][r] of this lane's column, summed over its rows
  float bia[4][4];               // bias of this lane's columns
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      ssum[a][b] = ssq[a][b] = 0.f;
      bia[a][b] = geo.bias ? geo.bias[n0 + wn * 64 + a * 16 + fq * 4 + b] : 0.f;
    }
  // bf16 BN-backward epilogue: in the store layout every lane owns 8 consecutive
  // channels per column pair pr (the same channels for every tile): offset
  // cofs within the pair's 32 columns
  const int cofs = (fq & 1) ? 16 + 4 * (fq - 1) : 4 * fq;
  // fp32 BN-backward epilogue operands (h, dy2, mask byte per 16-byte chunk)
  // of a 16-row subtile row ms.  The first PMS rows of a tile are loaded at
  // the start of its last K slice, so their latency hides under that slice's
  // MFMAs instead of stalling the epilogue; row ms + PMS is loaded into the
  // slot row ms frees while row ms is written.  (These loads are consumed
  // inside the same iteration, so the stage / store vmcnt accounting below is
  // unchanged.)
  // (32x64 wave tiles only: the 64x64 ones have no registers for it -- one
  // prefetched row already pushed them into 15-190 VGPRs of spills)
  constexpr bool PRE = F32 && BNB && MSB == 2;
  constexpr int PMS = PRE ? 2 : 1;
  f32x4 pre_h[PMS][4], pre_d[PMS][4];
  uint32_t pre_b[PMS][4];
  auto bn_row_load = [&](int64_t mbase_, int ms, f32x4* hh, f32x4* dd, uint32_t* bits) {
    const int64_t m = mbase_ + wm * Cfg::WTM + ms * 16 + fr;
#pragma unroll
    for (int ns = 0; ns < 4; ++ns) {
      hh[ns] = dd[ns] = f32x4{0.f, 0.f, 0.f, 0.f};
      bits[ns] = 0u;
    }
    if (m < M) {
#pragma unroll
      for (int ns = 0; ns < 4; ++ns) {
        const int n = n0 + wn * 64 + ns * 16 + fq * 4;
        hh[ns] = *reinterpret_cast<const f32x4*>(static_cast<const float*>(bb.h) + m * ldc + n);
        if (bb.dy2) dd[ns] = *reinterpret_cast<const f32x4*>(static_cast<const float*>(bb.dy2) + m * ldc + n);
        bits[ns] = bb.mask ? (uint32_t)bb.mask[m * (Ntot >> 2) + (n >> 2)] : 0xfu;
      }
    }
  };
  int64_t mt = bx;
  for (int t = 0; t < T_; ++t) {
    // ops issued after stage(t), in order: NS=2: stores(t-1);
    // NS=3: stores(t-2), stage(t+1), stores(t-1).  Retire stage(t) only.
    // after stage(t): stores(t-NS+1..t-1) and the stages t+1 .. t+NS-2 issued since
    if (NS == 2) wait_vmcnt_fast<0>(st1);
    else if (NS == 3) wait_vmcnt_fast<LPW>(st2 + (t + 1 < T_ ? LPW : 0) + st1);
    else wait_vmcnt_fast<2 * LPW>(st3 + st2 + st1 + ((t + 1 < T_) + (t + 2 < T_)) * LPW);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    const bool pf = s_t < T_;   // a stage to issue during this slice's MFMAs (wave-uniform)
    // fp32 spreads the next stage's LDS-DMA over the MFMA groups (16 fp32 MFMAs
    // per group hide each piece's issue cost); bf16 (4 MFMAs per group) issues
    // the whole stage right after the barrier -- measured on the ResNet-50
    // bs512 step: spreading cost bf16 ~1.4 ms (41.0 -> 42.4 ms); fp32 128.3 ms
    // with the previous tuning choices (128.1 before), 127.0 ms after a retune
    constexpr bool SPREAD = F32;
    if (pf) stage_prep();
    if constexpr (PRE) {
      if (ks == nk - 1) {
#pragma unroll
        for (int r = 0; r < PMS; ++r) bn_row_load(mt * Cfg::BM, r, pre_h[r], pre_d[r], pre_b[r]);
      }
    }
    if (!SPREAD && pf) {
#pragma unroll
      for (int q = 0; q < LPW; ++q) stage_issue(q);
    }
    const char* As = stage_base + buf * Cfg::STAGE;
    buf = buf + 1 == NS ? 0 : buf + 1;
    const char* Bs = BRES ? panel + ks * Cfg::BSTAGE : As + Cfg::ASTAGES;
    // lazy operand: channel of element 0 of this slice (K = taps x C, tap-major)
    const int cbase = LZ ? (ks * KS) % lz.C : 0;
    // MFMA groups per K slice: one per (half kk, 16-row subtile ms) -- fp32
    // 16 MFMAs (4 contraction slots x 4 subtiles), bf16 4; LDS-DMA piece q of
    // the next stage is issued after group (q * NG) / LPW
    constexpr int NG = 2 * MSB;
    auto issue_group = [&](int gi) {
      if constexpr (SPREAD) {
        if (pf) {
#pragma unroll
          for (int q = 0; q < LPW; ++q)
            if ((q * NG) / LPW == gi) stage_issue(q);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    // Fragments: the 4 B fragments of a half are read one half ahead (both
    // halves' in flight at the slice start), the A fragment of subtile ms one
    // subtile ahead -- LDS latency hides under the previous group's MFMAs and
    // only ~40 (fp32) / ~24 (bf16) VGPRs of operands are live.
    // fp32: lane (fr, fq) holds K elements 16 kk + 4 fq + 0..3 of its row; MFMA
    // j contracts element j of every lane group (the same K permutation on
    // both operands, so the sum is the GEMM's).
    using Frag = typename std::conditional<F32, f32x4, bf16x8>::type;
    auto ldA = [&](int kk, int s) -> Frag {
      const int c = kk * 4 + fq;
      const int ra = wm * Cfg::WTM + s * 16 + fr;
      Frag v = *reinterpret_cast<const Frag*>(As + ra * 128 + ((c ^ swz(ra)) << 4));
      if constexpr (LZ) {
        // dx = k1 ((dz - k2) - (x - mu) k4) for channels cbase + 4c .. +3
        const float4* ct = reinterpret_cast<const float4*>(smem) + cbase + 4 * c;
        const f32x4 xv = *reinterpret_cast<const f32x4*>(As + Cfg::ASTAGE + ra * 128 + ((c ^ swz(ra)) << 4));
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float4 cf = ct[e];
          v[e] = cf.x * ((v[e] - cf.y) - (xv[e] - cf.z) * cf.w);
        }
      }
      return v;
    };
    // B fragments of both halves up front, except for the 128x64 bf16 wave
    // tiles (MSB 8: 128 accumulator VGPRs), which read each half's at its start
    constexpr int NBB = (F32 || MSB == 4) ? 2 : 1;
    Frag bv[NBB][4];
    auto ldB = [&](int kk, Frag* b) {
      const int c = kk * 4 + fq;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int rb = wn * 64 + s * 16 + fr;
        b[s] = *reinterpret_cast<const Frag*>(Bs + rb * 128 + ((c ^ swz(rb)) << 4));
      }
    };
    if constexpr (!F32) {
      // bf16: each half's A and B fragments read at its start, then its MFMAs
      // (the round-3 schedule; streaming A one subtile ahead measured slower here)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        Frag av[MSB], bh[4];
#pragma unroll
        for (int s2 = 0; s2 < MSB; ++s2) av[s2] = ldA(kk, s2);
        ldB(kk, bh);
#pragma unroll
        for (int ms = 0; ms < MSB; ++ms)
#pragma unroll
          for (int ns = 0; ns < 4; ++ns)
            acc[ms][ns] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh[ns], av[ms], acc[ms][ns], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int kk = 0; kk < NBB; ++kk) ldB(kk, bv[kk]);
      if constexpr (X6) {
        // fp32-accurate products on the bf16 matrix cores: every fp32 operand
        // is split exactly into bf16 parts x = hi + mid + lo (split3x8) and the
        // six part products of order <= 2 -- all but mid*lo, lo*mid, lo*lo,
        // each < 2^-24 |a b| -- are accumulated in fp32.  Lane (fr, fq) holds
        // K elements 4 fq + 0..3 (half 0) and 16 + 4 fq + 0..3 (half 1) of its
        // row, the same permutation on both operands.  One K slice = one
        // 16x16x32 bf16 step: 6 x 16 cycles against 8 x 32 for the fp32 MFMA.
        bf16x8 bh[4], bm[4], bl[4];
#if GK_X6_SCHED
        // Software-pipelined: the B splits of ns = 1..3 are interleaved with the
        // MFMAs of subtile row 0, the A split of subtile row ms + 1 with the
        // MFMAs of row ms (sched_group_barrier: 1 MFMA, then a few VALU) -- a
        // wave issues in order, so VALU placed after a run of MFMAs would wait
        // for the matrix pipe instead of filling its 16-cycle shadow.
        split3x8(bv[0][0], bv[1][0], bh[0], bm[0], bl[0]);
        bf16x8 ah, am, al;
        {
          const Frag a0 = ldA(0, 0), a1 = ldA(1, 0);
          split3x8(a0, a1, ah, am, al);
        }
#pragma unroll
        for (int ms = 0; ms < MSB; ++ms) {
          Frag n0, n1;
          if (ms + 1 < MSB) {
            n0 = ldA(0, ms + 1);
            n1 = ldA(1, ms + 1);
          }
          bf16x8 nh, nm, nl;
#pragma unroll
          for (int ns = 0; ns < 4; ++ns) {
            if (ms == 0 && ns + 1 < 4) split3x8(bv[0][ns + 1], bv[1][ns + 1], bh[ns + 1], bm[ns + 1], bl[ns + 1]);
            if (ns == 1 && ms + 1 < MSB) split3x8(n0, n1, nh, nm, nl);
            f32x4 c = acc[ms][ns];
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bl[ns], ah, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh[ns], al, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bm[ns], am, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bm[ns], ah, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh[ns], am, c, 0, 0, 0);
            acc[ms][ns] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh[ns], ah, c, 0, 0, 0);
          }
          // schedule of this region: the next row's fragment reads first, then
          // the 24 MFMAs each followed by up to V VALU (ms 0: three B splits +
          // one A split, ~150 VALU; later rows: one A split, ~40)
          constexpr int V = 6;
          __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);   // DS reads
          if (ms == 0) {
#pragma unroll
            for (int q = 0; q < 24; ++q) {
              __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
              __builtin_amdgcn_sched_group_barrier(0x002, V, 0);   // VALU
            }
          } else {
#pragma unroll
            for (int q = 0; q < 24; ++q) {
              __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
              __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
            }
          }
          if (ms + 1 < MSB) {
            ah = nh;
            am = nm;
            al = nl;
          }
          issue_group(2 * ms);
          issue_group(2 * ms + 1);
        }
#else
#pragma unroll
        for (int ns = 0; ns < 4; ++ns) {
#if GK_X6_EXP == 1
          bh[ns] = __builtin_bit_cast(bf16x8, f32x4{bv[0][ns][0], bv[0][ns][1], bv[1][ns][0], bv[1][ns][1]});
          bm[ns] = __builtin_bit_cast(bf16x8, f32x4{bv[0][ns][2], bv[0][ns][3], bv[1][ns][2], bv[1][ns][3]});
          bl[ns] = bh[ns];
#else
          split3x8(bv[0][ns], bv[1][ns], bh[ns], bm[ns], bl[ns]);
#endif
        }
        Frag a0n = ldA(0, 0), a1n = ldA(1, 0);
#pragma unroll
        for (int ms = 0; ms < MSB; ++ms) {
          bf16x8 ah, am, al;
#if GK_X6_EXP == 1   // experiment: bit-slice instead of the exact split (VALU cost probe)
          ah = __builtin_bit_cast(bf16x8, f32x4{a0n[0], a0n[1], a1n[0], a1n[1]});
          am = __builtin_bit_cast(bf16x8, f32x4{a0n[2], a0n[3], a1n[2], a1n[3]});
          al = ah;
#else
          split3x8(a0n, a1n, ah, am, al);
#endif
          if (ms + 1 < MSB) {
            a0n = ldA(0, ms + 1);
            a1n = ldA(1, ms + 1);
          }
#pragma unroll
          for (int ns = 0; ns < 4; ++ns) {
            f32x4 c = acc[ms][ns];
#if GK_X6_EXP != 2   // experiment 2: one product only (data-movement probe)
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bl[ns], ah, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh[ns], al, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bm[ns], am, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bm[ns], ah, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh[ns], am, c, 0, 0, 0);
#endif
            acc[ms][ns] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh[ns], ah, c, 0, 0, 0);
          }
          issue_group(2 * ms);
          issue_group(2 * ms + 1);
        }
#endif
      } else {
      Frag an = ldA(0, 0);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int sb = NBB == 2 ? kk : 0;
        if (NBB == 1 && kk == 1) ldB(1, bv[0]);
#pragma unroll
        for (int ms = 0; ms < MSB; ++ms) {
          const Frag a = an;
          if (ms + 1 < MSB) an = ldA(kk, ms + 1);
          else if (kk == 0) an = ldA(1, 0);
          if constexpr (F32) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
              for (int ns = 0; ns < 4; ++ns)
                acc[ms][ns] = __builtin_amdgcn_mfma_f32_16x16x4f32(bv[sb][ns][j], a[j], acc[ms][ns], 0, 0, 0);
          } else {
#pragma unroll
            for (int ns = 0; ns < 4; ++ns)
              acc[ms][ns] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bv[sb][ns], a, acc[ms][ns], 0, 0, 0);
          }
          issue_group(kk * MSB + ms);
        }
      }
      }
    }
    if (pf) stage_advance();
    st3 = st2;
    st2 = st1;
    st1 = 0;
    if (++ks == nk) {
      ks = 0;
      // lane holds C[m = fr][n = 4*fq + r] of every 16x16 subtile.
      const int64_t mbase = mt * Cfg::BM;
      mt += gridDim.x;
      const bool full = mbase + Cfg::BM <= M;
      const bool odd = fq & 1;
#pragma unroll
      for (int ms = 0; ms < MSB; ++ms) {
        const int64_t m = mbase + wm * Cfg::WTM + ms * 16 + fr;
        const bool live = full || m < M;
        int64_t orow = m;     // output row (remapped for stride-2 grad-input classes)
        int zr = 0, zc = 0;   // RZ: sibling row / column inside the image
        if (geo.RH) {
          const uint32_t ohw = (uint32_t)(geo.OH * geo.OW);
          const uint32_t mu = (uint32_t)(m < M ? m : M - 1);
          const uint32_t ni = mu / ohw, rem = mu - ni * ohw;
          const uint32_t oh = rem / (uint32_t)geo.OW, ow = rem - oh * (uint32_t)geo.OW;
          orow = ((int64_t)ni * geo.RH + 2 * oh + geo.RA) * geo.RW + 2 * ow + geo.RB;
          zr = (int)(2 * oh + 1) < geo.RH;
          zc = (int)(2 * ow + 1) < geo.RW;
        }
        if constexpr (F32) {
          // fp32: lane owns 4 consecutive channels of every subtile -- one
          // 16-byte store per subtile, no shuffle.  BN-backward operands of the
          // row's four subtiles: prefetch slots (32x64 wave tiles) or loaded
          // here, all four before the first use.
          f32x4 ehv[4], ed2[4];
          uint32_t ebits[4];
          if constexpr (PRE) {
            const int slot = ms % PMS;
#pragma unroll
            for (int ns = 0; ns < 4; ++ns) {
              ehv[ns] = pre_h[slot][ns];
              ed2[ns] = pre_d[slot][ns];
              ebits[ns] = pre_b[slot][ns];
            }
            if (ms + PMS < MSB) bn_row_load(mbase, ms + PMS, pre_h[slot], pre_d[slot], pre_b[slot]);
          } else if (bnb) {
#pragma unroll
            for (int ns = 0; ns < 4; ++ns) {
              ehv[ns] = ed2[ns] = f32x4{0.f, 0.f, 0.f, 0.f};
              ebits[ns] = 0u;
            }
            if (live) {
#pragma unroll
              for (int ns = 0; ns < 4; ++ns) {
                const int n = n0 + wn * 64 + ns * 16 + fq * 4;
                ehv[ns] = *reinterpret_cast<const f32x4*>(static_cast<const float*>(bb.h) + m * ldc + n);
                if (bb.dy2) ed2[ns] = *reinterpret_cast<const f32x4*>(static_cast<const float*>(bb.dy2) + m * ldc + n);
                ebits[ns] = bb.mask ? (uint32_t)bb.mask[m * (Ntot >> 2) + (n >> 2)] : 0xfu;
              }
            }
          }
#pragma unroll
          for (int ns = 0; ns < 4; ++ns) {
            const int n = n0 + wn * 64 + ns * 16 + fq * 4;
            f32x4 v = acc[ms][ns];
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] += bia[ns][r];
            if (bnb) {
              // dz = mask ? dy + dy2 : 0; partials sum(dz), sum(dz * h)
              const f32x4 hv = ehv[ns], d2 = ed2[ns];
              const uint32_t bits = ebits[ns];
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const float dz = (bits >> r) & 1u ? v[r] + d2[r] : 0.f;
                v[r] = dz;
                ssum[ns][r] += dz;
                ssq[ns][r] = fmaf(dz, hv[r], ssq[ns][r]);
              }
            } else if (stats && live) {
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                ssum[ns][r] += v[r];
                ssq[ns][r] = fmaf(v[r], v[r], ssq[ns][r]);
              }
            }
            if (live) {
              *reinterpret_cast<f32x4*>(C + orow * ldc + n) = v;
              if (geo.RZ) {
                const f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
                if (zc) *reinterpret_cast<f32x4*>(C + (orow + 1) * ldc + n) = z;
                if (zr) *reinterpret_cast<f32x4*>(C + (orow + geo.RW) * ldc + n) = z;
                if (zr && zc) *reinterpret_cast<f32x4*>(C + (orow + geo.RW + 1) * ldc + n) = z;
              }
            }
          }
        } else {
          // bf16: lanes fq and fq^1 swap halves of the subtile pair (2p, 2p+1) so
          // each lane owns 8 consecutive channels: one 16-byte store per lane per pair.
          uint4 eh[2], ed[2];   // BN-backward operands of this row: h, dy2 and the mask byte per pair
          uint32_t em[2];
          if (bnb) {
#pragma unroll
            for (int pr = 0; pr < 2; ++pr) {
              const int n = n0 + wn * 64 + pr * 32 + cofs;
              eh[pr] = ed[pr] = make_uint4(0u, 0u, 0u, 0u);
              em[pr] = 0u;
              if (live) {
                eh[pr] = *reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(bb.h) + m * ldc + n);
                if (bb.dy2) ed[pr] = *reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(bb.dy2) + m * ldc + n);
                em[pr] = bb.mask ? (uint32_t)bb.mask[m * (Ntot >> 3) + (n >> 3)] : 0xffu;
              }
            }
          }
#pragma unroll
          for (int pr = 0; pr < 2; ++pr) {
            const f32x4 va = acc[ms][2 * pr], vb = acc[ms][2 * pr + 1];
            const float* ba = bia[2 * pr];
            const float* bb2 = bia[2 * pr + 1];
            const uint32_t a0 = pack_bf16x2(va[0] + ba[0], va[1] + ba[1]), a1 = pack_bf16x2(va[2] + ba[2], va[3] + ba[3]);
            const uint32_t b0 = pack_bf16x2(vb[0] + bb2[0], vb[1] + bb2[1]), b1 = pack_bf16x2(vb[2] + bb2[2], vb[3] + bb2[3]);
            if (stats && !bnb && live) {   // statistics of the values as stored (bf16)
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
            uint4 v = odd ? make_uint4(r0, r1, b0, b1) : make_uint4(a0, a1, r0, r1);
            const int n = n0 + wn * 64 + pr * 32 + cofs;
            if (bnb) {
              const uint32_t dv[4] = {v.x, v.y, v.z, v.w};
              const uint4 e2 = ed[pr], eh4 = eh[pr];
              const uint32_t d2[4] = {e2.x, e2.y, e2.z, e2.w};
              const uint32_t hh[4] = {eh4.x, eh4.y, eh4.z, eh4.w};
              const uint32_t bits = em[pr];
              uint32_t o[4];
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                float lo = __uint_as_float(dv[i] << 16) + __uint_as_float(d2[i] << 16);
                float hi = __uint_as_float(dv[i] & 0xffff0000u) + __uint_as_float(d2[i] & 0xffff0000u);
                lo = (bits >> (2 * i)) & 1u ? lo : 0.f;
                hi = (bits >> (2 * i + 1)) & 1u ? hi : 0.f;
                o[i] = pack_bf16x2(lo, hi);
                const float hl = __uint_as_float(hh[i] << 16);
                const float hu = __uint_as_float(hh[i] & 0xffff0000u);
                const int a = 2 * pr + (i >> 1), b = (i & 1) * 2;
                ssum[a][b] += lo;
                ssq[a][b] = fmaf(lo, hl, ssq[a][b]);
                ssum[a][b + 1] += hi;
                ssq[a][b + 1] = fmaf(hi, hu, ssq[a][b + 1]);
              }
              v = make_uint4(o[0], o[1], o[2], o[3]);
            }
            if (live) {
              *reinterpret_cast<uint4*>(C + orow * ldc + n) = v;
              if (geo.RZ) {
                const uint4 z = make_uint4(0u, 0u, 0u, 0u);
                if (zc) *reinterpret_cast<uint4*>(C + (orow + 1) * ldc + n) = z;
                if (zr) *reinterpret_cast<uint4*>(C + (orow + geo.RW) * ldc + n) = z;
                if (zr && zc) *reinterpret_cast<uint4*>(C + (orow + geo.RW + 1) * ldc + n) = z;
              }
            }
          }
        }
#pragma unroll
        for (int ns = 0; ns < 4; ++ns) acc[ms][ns] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      if (full && !geo.RZ) st1 = Cfg::NST;
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // skipped / extra stores: keep the counts exact
    }
  }
  if (stats) {
    // sum over the 16 rows (lanes fr) of each lane group, then over the WM
    // waves sharing a column range, through LDS (every stage is consumed)
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
    float* red = reinterpret_cast<float*>(smem);   // [2][WM][BN]
    if (fr == 0) {
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          // forward and fp32: [subtile a][row b] of 4fq..; bf16 BN-backward:
          // store-layout channel cofs + 4 * (a & 1) + b of column pair a / 2
          const int col = (bnb && !F32) ? wn * 64 + (a >> 1) * 32 + cofs + (a & 1) * 4 + b
                                        : wn * 64 + a * 16 + fq * 4 + b;
          red[wm * Cfg::BN + col] = ssum[a][b];
          red[(WM + wm) * Cfg::BN + col] = ssq[a][b];
        }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < Cfg::BN; c += Cfg::THREADS) {
      float sa = 0.f, sb = 0.f;
#pragma unroll
      for (int w2 = 0; w2 < WM; ++w2) {
        sa += red[w2 * Cfg::BN + c];
        sb += red[(WM + w2) * Cfg::BN + c];
      }
      stats[(int64_t)bx * Ntot + n0 + c] = sa;
      stats[stats_ld + (int64_t)bx * Ntot + n0 + c] = sb;
    }
  }
}

template <int WM, int WN, bool BRES, int NS, bool GATHER, int MSB = 4, bool BNB = false, typename T = uint16_t,
          bool LZ = false, bool X6 = false>
int launch_nt(const T* A, int64_t lda, const T* B, int64_t ldb, T* C, int64_t ldc, int64_t M,
              int N, int K, int max_blocks, const ConvGeo& geo, float* stats, int64_t stats_ld, int stats_rows,
              const BnBwd& bb, const LazyA& lz, hipStream_t stream) {
  using Cfg = NtCfg<WM, WN, BRES, MSB, T, LZ>;
  const int ntiles = N / Cfg::BN;
  const int64_t mtiles = (M + Cfg::BM - 1) / Cfg::BM;
  const int lds = Cfg::lds_bytes(K, NS, lz.C);
  const int per_cu = (160 * 1024) / lds > 0 ? (160 * 1024) / lds : 1;
  const int kz = (!LZ && geo.KZ > 1) ? geo.KZ : 1;
  int64_t gx = ((int64_t)256 * per_cu + ntiles * kz - 1) / (ntiles * kz);
  if (max_blocks > 0) gx = max_blocks;
  if (gx < 1) gx = 1;
  if (gx > mtiles) gx = mtiles;
  if (stats && gx > stats_rows) gx = stats_rows;   // one partial row per block
  dim3 grid((unsigned)gx, (unsigned)ntiles, (unsigned)kz);
  static bool attr = [] {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_nt_kernel<WM, WN, BRES, NS, GATHER, MSB, BNB, T, LZ, X6>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
  }();
  (void)attr;
  hipLaunchKernelGGL((gemm_nt_kernel<WM, WN, BRES, NS, GATHER, MSB, BNB, T, LZ, X6>), grid, dim3(Cfg::THREADS), lds, stream,
                     A, lda, B, ldb, C, ldc, M, K, geo, stats, stats_ld, bb, lz);
  return (int)gx;
}

template <int WM, int WN, bool GATHER, int MSB = 4, bool BNB = false, typename T = uint16_t, bool LZ = false,
          bool X6 = false>
int launch_nt_any(const T* A, int64_t lda, const T* B, int64_t ldb, T* C, int64_t ldc,
                  int64_t M, int N, int K, int max_blocks, int bres, int ns, const ConvGeo& geo, float* stats,
                  int64_t stats_ld, int stats_rows, const BnBwd& bb, const LazyA& lz, hipStream_t stream) {
  using CR = NtCfg<WM, WN, true, MSB, T, LZ>;
  using CS = NtCfg<WM, WN, false, MSB, T, LZ>;
  const int cc = lz.C;
  // keep the weight panel resident when it fits next to the two A stages
  if (bres < 0) bres = (64 * WN) * K * (int)sizeof(T) <= 64 * 1024;
  if (bres && CR::lds_bytes(K, 2, cc) > 160 * 1024) bres = 0;
  constexpr int L = 160 * 1024;
#define GK_NT(BR, S) \
  launch_nt<WM, WN, BR, S, GATHER, MSB, BNB, T, LZ, X6>(A, lda, B, ldb, C, ldc, M, N, K, max_blocks, geo, stats, stats_ld, stats_rows, bb, lz, stream)
  if constexpr (CR::NS4_OK)
    if (ns == 4 && bres && CR::lds_bytes(K, 4, cc) <= L) return GK_NT(true, 4);
  if constexpr (CS::NS4_OK)
    if (ns == 4 && !bres && CS::lds_bytes(K, 4, cc) <= L) return GK_NT(false, 4);
  if (bres) {
    if constexpr (CR::NS3_OK)
      if (ns != 2 && CR::lds_bytes(K, 3, cc) <= L) return GK_NT(true, 3);
    return GK_NT(true, 2);
  }
  if constexpr (CS::NS3_OK)
    if (ns != 2 && CS::lds_bytes(K, 3, cc) <= L) return GK_NT(false, 3);
  if (CS::lds_bytes(K, 2, cc) > L) return -1;   // does not fit (lazy coefficient table too large)
  return GK_NT(false, 2);
#undef GK_NT
}

// --------------------------------------------------------------------------
// gemm_tn: W[N, K] += G[M, N]^T . X[M, K]
// --------------------------------------------------------------------------
// WS waves split the 64*WS pixel rows of a stage for the same output tile;
// their partial sums are combined through LDS before the atomics.
// MSN: 64-row groups of the wave tile along N (1: 64x64 per wave, 2: 128x64 --
// 25% fewer LDS reads per MFMA and twice the work per staged G row)
template <int WN, int WK, int WS, int NS_, int MSN = 1>
struct TnCfg {
  static constexpr int NW = WN * WK * WS;
  static constexpr int THREADS = 64 * NW;
  static constexpr int WTN = 64 * MSN;               // wave tile rows (G columns)
  static constexpr int BN = WTN * WN;                // output rows (G columns)
  static constexpr int BK = 64 * WK;                 // output cols (X columns)
  static constexpr int ROWS = 64 * WS;               // pixel rows per stage
  static constexpr int GROW = BN * 2;                // bytes per staged G row
  static constexpr int XROW = BK * 2;
  static constexpr int GBYTES = ROWS * GROW;
  static constexpr int STAGE = ROWS * (GROW + XROW);
  static constexpr int NS = NS_;                     // LDS stages (3: two slices in flight)
  static constexpr int LDS = NS * STAGE;
  static constexpr int GINSTS = GBYTES / 1024;
  static constexpr int INSTS = STAGE / 1024;
  static_assert(INSTS % NW == 0, "stage split");
  static constexpr int LPW = INSTS / NW;
  static_assert(LPW <= 63, "wait_vmcnt range");
  static_assert(GINSTS % NW == 0, "G rows split evenly over the waves");
  static constexpr int LPWG = GINSTS / NW;           // G-row instructions per wave (j < LPWG)
  static_assert((WS - 1) * WN * WK * MSN * 16384 <= LDS, "reduction scratch");
};

// a / d for small a (< 2^22): float reciprocal, one correction step
__device__ __forceinline__ uint32_t udiv_small(uint32_t a, uint32_t d, float rcp) {
  uint32_t q = (uint32_t)((float)a * rcp);
  const int32_t r = (int32_t)(a - q * d);
  if (r < 0) --q;
  else if (r >= (int32_t)d) ++q;
  return q;
}

// Transposed fragment: lane l (group g = l>>4, li = l&15) gets rows
// r0 + 8g + 0..7 of column c0 + li of the swizzled [rows][RB] bf16 image, as
// the 8 k-elements of a 16x16x32 MFMA operand.  c0 is a multiple of 16.
// The transposed LDS read is issued as inline asm (mfma_util.h ds_read_tr):
// with the builtin, the compiler's wait-count pass cannot tell the read apart
// from the LDS-DMA writes of the NEXT stage issued just before it and inserts
// `s_waitcnt vmcnt(0)` -- which serialises the whole global->LDS pipeline
// (each stage would wait for the loads it has just started).  The asm reads
// carry no such dependence; tr_sync() below waits for them (lgkmcnt) and ties
// the fragments to that wait so no MFMA can be scheduled before it.
template <int RB>
__device__ __forceinline__ bf16x8 tr_frag(const char* tile, int r0, int c0, int lane) {
  const int g = lane >> 4, li = lane & 15;
  const int q = li >> 2, p = li & 3;
  const int col = c0 + 4 * p;
  const int ra = r0 + 8 * g + q, rb = ra + 4;
  const char* a0 = tile + ra * RB + ((((col >> 3) ^ tr_swz<RB>(ra)) << 4) | ((col & 7) << 1));
  const char* a1 = tile + rb * RB + ((((col >> 3) ^ tr_swz<RB>(rb)) << 4) | ((col & 7) << 1));
  bf16x4 lo = ds_read_tr(a0);
  bf16x4 hi = ds_read_tr(a1);
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// the two halves of a transposed fragment at precomputed LDS addresses, k-step
// kk adding the immediate kk * KSTEP bytes
template <int KSTEP>
__device__ __forceinline__ bf16x8 tr_pair(uint32_t a0, uint32_t a1, int kk) {
  bf16x4 lo, hi;
  if (kk == 0) {
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(a0));
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(hi) : "v"(a1));
  } else {
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(lo) : "v"(a0), "i"(KSTEP));
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(hi) : "v"(a1), "i"(KSTEP));
  }
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// lgkmcnt(0) tied to the fragments of one k-step
template <int MSN>
__device__ __forceinline__ void tr_sync(bf16x8* a, bf16x8* b) {
  if (MSN == 1) {
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]));
  } else {
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]),
                   "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]));
  }
}

template <int WN, int WK, int WS, int NS, bool GATHER, int MSN = 1>
__global__ void __launch_bounds__(64 * WN * WK * WS) __attribute__((amdgpu_waves_per_eu(MSN > 1 ? 1 : 2)))
gemm_tn_kernel(const uint16_t* __restrict__ G, int64_t ldg, const uint16_t* __restrict__ X, int64_t ldx,
               float* __restrict__ W, int64_t ldw, int64_t M, int64_t rows_per_split, ConvGeo geo) {
  using Cfg = TnCfg<WN, WK, WS, NS, MSN>;
  constexpr int NF = 4 * MSN;                        // G fragments (16 rows each) per wave
  constexpr int LPW = Cfg::LPW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wk = wave % WK, wn = (wave / WK) % WN, ws = wave / (WK * WN);
  int bx, by, bz;   // logical block coordinates (XCD-aware order)
  xcd_remap3(bx, by, bz);
  const int n0 = bx * Cfg::BN;
  const int c0 = by * Cfg::BK;
  const int64_t mbeg = (int64_t)bz * rows_per_split;
  int64_t mend = mbeg + rows_per_split;
  if (mend > M) mend = M;
  if (mbeg >= mend) return;
  const int T = (int)((mend - mbeg + Cfg::ROWS - 1) / Cfg::ROWS);

  // Per-lane staging state, set up once and advanced by ROWS pixel rows per
  // stage (no per-stage divisions or 64-bit multiplies): G / plain-X
  // instructions keep a row pointer; gathered X instructions keep the output
  // pixel (n, oh, ow) and their tap (dkh, dkw).
  const uint16_t* rptr[LPW];     // current row pointer (G / plain X)
  const uint16_t* rlast[LPW];    // row M-1 (clamp target past the end)
  int64_t row[LPW];              // current pixel row index
  int pn[LPW], poh[LPW], pow_[LPW], dkh[LPW], dkw[LPW], ccol[LPW];
#pragma unroll
  for (int j = 0; j < LPW; ++j) {
    const int i = wave + j * Cfg::NW;
    int srow, colo;
    bool gath = false;
    dkh[j] = dkw[j] = 0;
    if (j < Cfg::LPWG) {
      constexpr int CPR = Cfg::GROW / 16;
      const int e = i * 64 + lane;
      srow = e / CPR;
      colo = n0 + ((e % CPR) ^ tr_swz<Cfg::GROW>(srow)) * 8;
      rptr[j] = G + (mbeg + srow) * ldg + colo;
      rlast[j] = G + (M - 1) * ldg + colo;
    } else {
      constexpr int CPR = Cfg::XROW / 16;
      const int e = (i - Cfg::GINSTS) * 64 + lane;
      srow = e / CPR;
      const int ch = (e % CPR) ^ tr_swz<Cfg::XROW>(srow);
      if (GATHER) {
        const int k0 = c0 + (ch >> 3) * 64;          // 64-channel slice of one tap
        const int tap = k0 / geo.C;
        dkh[j] = tap / geo.KW;
        dkw[j] = tap - dkh[j] * geo.KW;
        colo = (k0 - tap * geo.C) + (ch & 7) * 8;
        gath = true;
      } else {
        colo = c0 + ch * 8;
      }
      rptr[j] = X + (mbeg + srow) * ldx + colo;
      rlast[j] = X + (M - 1) * ldx + colo;
    }
    row[j] = mbeg + srow;
    ccol[j] = colo;
    pn[j] = poh[j] = pow_[j] = 0;
    if (GATHER && gath) {
      const int64_t m = mbeg + srow;
      const int64_t ohw = (int64_t)geo.OH * geo.OW;
      pn[j] = (int)(m / ohw);
      const int rem = (int)(m - (int64_t)pn[j] * ohw);
      poh[j] = rem / geo.OW;
      pow_[j] = rem - poh[j] * geo.OW;
    }
  }
  const int adv_q = Cfg::ROWS / (GATHER ? geo.OW : 1), adv_r = Cfg::ROWS - adv_q * (GATHER ? geo.OW : 1);
  const int64_t gstep = (int64_t)Cfg::ROWS * ldg, xstep = (int64_t)Cfg::ROWS * ldx;

  auto stage = [&](int t) {
    GK_LDS char* base = (GK_LDS char*)smem + (t % NS) * Cfg::STAGE;
#pragma unroll
    for (int j = 0; j < LPW; ++j) {
      const int i = wave + j * Cfg::NW;
      const bool in = row[j] < M;
      const uint16_t* src;
      if (j < Cfg::LPWG) {
        src = in ? rptr[j] : rlast[j];
        rptr[j] += gstep;
      } else if (GATHER) {
        const int ih = poh[j] * geo.S - geo.P + dkh[j], iw = pow_[j] * geo.S - geo.P + dkw[j];
        const bool ok = in && (unsigned)ih < (unsigned)geo.H && (unsigned)iw < (unsigned)geo.W;
        const uint32_t off = (((uint32_t)pn[j] * (uint32_t)geo.H + (uint32_t)ih) * (uint32_t)geo.W + (uint32_t)iw) *
                                 (uint32_t)geo.C + (uint32_t)ccol[j];
        src = ok ? X + off : static_cast<const uint16_t*>(geo.zero) + (ccol[j] & 63);
        // advance the pixel by ROWS
        pow_[j] += adv_r;
        poh[j] += adv_q;
        if (pow_[j] >= geo.OW) { pow_[j] -= geo.OW; ++poh[j]; }
        while (poh[j] >= geo.OH) { poh[j] -= geo.OH; ++pn[j]; }
      } else {
        src = in ? rptr[j] : rlast[j];
        rptr[j] += xstep;
      }
      row[j] += Cfg::ROWS;
      glds16(src, base + i * 1024);
    }
  };

  f32x4 acc[NF][4];
#pragma unroll
  for (int a = 0; a < NF; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Per-lane LDS byte offsets of the 16 transposed reads of a k-step, set up
  // once: the swizzle depends on row bits 0, 1 and 3 only, so the second
  // k-step (rows + 32) is the same addresses + 32 rows -- an immediate offset
  // -- and a new stage only adds its (uniform) base: 16 adds per stage instead
  // of the full address arithmetic per read.
  uint32_t goff[NF][2], xoff[4][2];
  {
    const int g = lane >> 4, li = lane & 15;
    const int q = li >> 2, p = li & 3;
    const int ra = ws * 64 + 8 * g + q, rb = ra + 4;
#pragma unroll
    for (int s2 = 0; s2 < NF; ++s2) {
      const int gc = wn * Cfg::WTN + s2 * 16 + 4 * p;
      goff[s2][0] = ra * Cfg::GROW + ((((gc >> 3) ^ tr_swz<Cfg::GROW>(ra)) << 4) | ((gc & 7) << 1));
      goff[s2][1] = rb * Cfg::GROW + ((((gc >> 3) ^ tr_swz<Cfg::GROW>(rb)) << 4) | ((gc & 7) << 1));
    }
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
      const int xc = wk * 64 + s2 * 16 + 4 * p;
      xoff[s2][0] = Cfg::GBYTES + ra * Cfg::XROW + ((((xc >> 3) ^ tr_swz<Cfg::XROW>(ra)) << 4) | ((xc & 7) << 1));
      xoff[s2][1] = Cfg::GBYTES + rb * Cfg::XROW + ((((xc >> 3) ^ tr_swz<Cfg::XROW>(rb)) << 4) | ((xc & 7) << 1));
    }
  }
  const uint32_t lds0 = (uint32_t)(uintptr_t)(GK_LDS char*)smem;

  stage(0);
  if (NS == 3 && T > 1) stage(1);
  for (int t = 0; t < T; ++t) {
    // retire slice t (with NS = 3, slice t+1 stays in flight)
    if (NS == 3) wait_vmcnt_fast<LPW>(t + 1 < T ? LPW : 0);
    else wait_vmcnt(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (t + NS - 1 < T) stage(t + NS - 1);
    const uint32_t sb = lds0 + (uint32_t)((t % NS) * Cfg::STAGE);
    uint32_t ga[NF][2], xa[4][2];
#pragma unroll
    for (int s2 = 0; s2 < NF; ++s2)
#pragma unroll
      for (int h = 0; h < 2; ++h) ga[s2][h] = sb + goff[s2][h];
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2)
#pragma unroll
      for (int h = 0; h < 2; ++h) xa[s2][h] = sb + xoff[s2][h];
    const int64_t m0 = mbeg + (int64_t)t * Cfg::ROWS + ws * 64;
    const bool tail = m0 + 64 > mend;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 gv[NF], xv[4];
#pragma unroll
      for (int s2 = 0; s2 < NF; ++s2) gv[s2] = tr_pair<32 * Cfg::GROW>(ga[s2][0], ga[s2][1], kk);
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) xv[s2] = tr_pair<32 * Cfg::XROW>(xa[s2][0], xa[s2][1], kk);
      tr_sync<MSN>(gv, xv);
      if (tail) {  // rows past this split's end contribute nothing
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int64_t m = m0 + kk * 32 + 8 * (lane >> 4) + j;
          if (m >= mend) {
#pragma unroll
            for (int s2 = 0; s2 < NF; ++s2) gv[s2][j] = 0;
          }
        }
      }
#pragma unroll
      for (int ns = 0; ns < NF; ++ns)
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
          acc[ns][ks] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(gv[ns], xv[ks], acc[ns][ks], 0, 0, 0);
    }
  }
  if (WS > 1) {   // combine the WS partial tiles through LDS
    __syncthreads();
    f32x4* red = reinterpret_cast<f32x4*>(smem);
    const int slot = wn * WK + wk;
    if (ws > 0) {
#pragma unroll
      for (int ns = 0; ns < NF; ++ns)
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
          red[(((ws - 1) * WN * WK + slot) * 4 * NF + ns * 4 + ks) * 64 + lane] = acc[ns][ks];
    }
    __syncthreads();
    if (ws == 0) {
#pragma unroll
      for (int w2 = 1; w2 < WS; ++w2)
#pragma unroll
        for (int ns = 0; ns < NF; ++ns)
#pragma unroll
          for (int ks = 0; ks < 4; ++ks) {
            const f32x4 v = red[(((w2 - 1) * WN * WK + slot) * 4 * NF + ns * 4 + ks) * 64 + lane];
            acc[ns][ks] += v;
          }
    }
  }
  if (ws != 0) return;
  // D[i = n][j = c]: lane holds column c = .. + (lane&15), rows n = .. + 4*(lane>>4) + r
  const int fr = lane & 15, fq = lane >> 4;
#pragma unroll
  for (int ns = 0; ns < NF; ++ns)
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int c = c0 + wk * 64 + ks * 16 + fr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wn * Cfg::WTN + ns * 16 + fq * 4 + r;
        atomicAdd(W + (int64_t)n * ldw + c, acc[ns][ks][r]);
      }
    }
}

template <int WN, int WK, int WS, int NS, bool GATHER, int MSN = 1>
void launch_tn(const uint16_t* G, int64_t ldg, const uint16_t* X, int64_t ldx, float* W, int64_t ldw, int64_t M,
               int N, int K, int splits, const ConvGeo& geo, hipStream_t stream) {
  using Cfg = TnCfg<WN, WK, WS, NS, MSN>;
  const int tiles = (N / Cfg::BN) * (K / Cfg::BK);
  if (splits <= 0) {
    // Whole rounds of the chip: one 8-wave block per CU at 2 waves / SIMD
    // (the 16-wave tile: one per CU too), two rounds -- a 2.1-round grid
    // would leave the third round almost empty (a 33% tail).
    static const int cus = [] {
      int d = 0, n = 0;
      hipGetDevice(&d);
      return hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, d) == hipSuccess && n > 0 ? n : 256;
    }();
    const int64_t bpc = Cfg::NW >= 8 ? 1 : 8 / Cfg::NW;
    const int64_t slots = (int64_t)cus * bpc;
    // splits < 0: -splits quarter rounds (a grad-weight on the side stream that
    // should leave CUs to the critical path); 0: two rounds
    const int64_t quarters = splits == 0 ? 8 : -(int64_t)splits;
    splits = (int)(quarters * slots / (4 * (int64_t)tiles));
    if (splits < 1) splits = 1;
  }
  int64_t rows = (M + splits - 1) / splits;
  rows = (rows + Cfg::ROWS - 1) / Cfg::ROWS * Cfg::ROWS;
  if (rows < 4 * Cfg::ROWS) rows = 4 * Cfg::ROWS;
  const int64_t nsplit = (M + rows - 1) / rows;
  dim3 grid((unsigned)(N / Cfg::BN), (unsigned)(K / Cfg::BK), (unsigned)nsplit);
  static bool attr = [] {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_tn_kernel<WN, WK, WS, NS, GATHER, MSN>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, Cfg::LDS) == hipSuccess;
  }();
  (void)attr;
  hipLaunchKernelGGL((gemm_tn_kernel<WN, WK, WS, NS, GATHER, MSN>), grid, dim3(Cfg::THREADS), Cfg::LDS, stream, G, ldg, X, ldx, W, ldw,
                     M, rows, geo);
}

// --------------------------------------------------------------------------
// gemm_tn, fp32 operands: W[N, K] += G[M, N]^T . X[M, K] on v_mfma_f32_16x16x4_f32
// --------------------------------------------------------------------------
// Both operands are M-major (pixel rows), the contraction runs over M, so an
// MFMA operand wants one column of 4 consecutive staged rows per lane.  fp32
// has no transposed LDS read; fp32 MFMA is 16x slower than bf16 per FLOP, so
// 4 ds_read_b32 per 4 MFMAs (128 cycles) cost nothing that matters: lane
// (i = l % 16, g = l / 16) reads rows kb + 4g + j (j = 0..3) of column i and
// MFMA j contracts rows {kb + j, kb + 4 + j, kb + 8 + j, kb + 12 + j} -- the
// same row permutation on both operands.  The 16-byte chunk index of a staged
// row is XOR-ed with bit 2 of the row, which puts the two half-waves of every
// ds_read_b32 (rows 4 apart) on disjoint banks.  Rows past this block's split
// (and padding taps) load from a zero vector, so the tail needs no masking.
// Each wave owns a 64x64 output tile; WN x WK waves per block, ROWS = 32
// pixel rows (two 16-row k-groups, 128 MFMAs per wave) per LDS stage.
__device__ __attribute__((aligned(16))) float g_tn_zero[32];

template <int WN, int WK, int NS_, bool LZ = false>
struct TnF32Cfg {
  static constexpr int NW = WN * WK;
  static constexpr int THREADS = 64 * NW;
  static constexpr int BN = 64 * WN;
  static constexpr int BK = 64 * WK;
  static constexpr int ROWS = 32;
  static constexpr int GROW = BN * 4;
  static constexpr int XROW = BK * 4;
  static constexpr int NGCOPY = LZ ? 2 : 1;        // lazy BN operand: dz and x tiles of G
  static constexpr int GBYTES = ROWS * GROW;       // one G copy
  static constexpr int GBYTES_ALL = NGCOPY * GBYTES;
  static constexpr int STAGE = ROWS * (NGCOPY * GROW + XROW);
  static constexpr int NS = NS_;
  static constexpr int LDS = NS * STAGE;
  static constexpr int GINSTS1 = GBYTES / 1024;
  static constexpr int GINSTS = GBYTES_ALL / 1024;
  static constexpr int INSTS = STAGE / 1024;
  static_assert(INSTS % NW == 0 && GINSTS % NW == 0, "stage split");
  static constexpr int LPW = INSTS / NW;
  static constexpr int LPWG = GINSTS / NW;
  static_assert(LPW <= 63, "wait_vmcnt range");
};

__device__ __forceinline__ int swz4(int r) { return r & 4; }

template <int WN, int WK, int NS, bool GATHER, bool LZ = false, bool X6 = false>
__global__ void __launch_bounds__(64 * WN * WK) __attribute__((amdgpu_waves_per_eu(1)))
gemm_tn_f32_kernel(const float* __restrict__ G, int64_t ldg, const float* __restrict__ X, int64_t ldx,
                   float* __restrict__ W, int64_t ldw, int64_t M, int64_t rows_per_split, ConvGeo geo, LazyA lz) {
  using Cfg = TnF32Cfg<WN, WK, NS, LZ>;
  constexpr int LPW = Cfg::LPW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wk = wave % WK, wn = wave / WK;
  int bx, by, bz;   // logical block coordinates (XCD-aware order)
  xcd_remap3(bx, by, bz);
  const int n0 = bx * Cfg::BN;
  const int c0 = by * Cfg::BK;
  const int64_t mbeg = (int64_t)bz * rows_per_split;
  int64_t mend = mbeg + rows_per_split;
  if (mend > M) mend = M;
  if (mbeg >= mend) return;
  const int T = (int)((mend - mbeg + Cfg::ROWS - 1) / Cfg::ROWS);

  // per-lane staging state (set once, advanced by ROWS rows per stage)
  const float* rptr[LPW];
  int64_t row[LPW];
  int pn[LPW], poh[LPW], pow_[LPW], dkh[LPW], dkw[LPW], ccol[LPW];
#pragma unroll
  for (int j = 0; j < LPW; ++j) {
    const int i = wave + j * Cfg::NW;
    int srow, colo;
    bool gath = false;
    dkh[j] = dkw[j] = 0;
    if (j < Cfg::LPWG) {
      constexpr int CPR = Cfg::GROW / 16;
      const bool isx = LZ && i >= Cfg::GINSTS1;    // lazy: second G copy = the BN input x
      const int e = (isx ? i - Cfg::GINSTS1 : i) * 64 + lane;
      srow = e / CPR;
      colo = n0 + ((e % CPR) ^ swz4(srow)) * 4;
      rptr[j] = (isx ? static_cast<const float*>(lz.x) : G) + (mbeg + srow) * ldg + colo;
    } else {
      constexpr int CPR = Cfg::XROW / 16;
      const int e = (i - Cfg::GINSTS) * 64 + lane;
      srow = e / CPR;
      const int kcol = c0 + ((e % CPR) ^ swz4(srow)) * 4;
      if (GATHER) {
        const int tap = kcol / geo.C;
        dkh[j] = tap / geo.KW;
        dkw[j] = tap - dkh[j] * geo.KW;
        colo = kcol - tap * geo.C;
        gath = true;
      } else {
        colo = kcol;
      }
      rptr[j] = X + (mbeg + srow) * ldx + colo;
    }
    row[j] = mbeg + srow;
    ccol[j] = colo;
    pn[j] = poh[j] = pow_[j] = 0;
    if (GATHER && gath) {
      const int64_t m = mbeg + srow;
      const int64_t ohw = (int64_t)geo.OH * geo.OW;
      pn[j] = (int)(m / ohw);
      const int rem = (int)(m - (int64_t)pn[j] * ohw);
      poh[j] = rem / geo.OW;
      pow_[j] = rem - poh[j] * geo.OW;
    }
  }
  const int adv_q = Cfg::ROWS / (GATHER ? geo.OW : 1), adv_r = Cfg::ROWS - adv_q * (GATHER ? geo.OW : 1);
  const int64_t gstep = (int64_t)Cfg::ROWS * ldg, xstep = (int64_t)Cfg::ROWS * ldx;

  auto stage = [&](int t) {
    GK_LDS char* base = (GK_LDS char*)smem + (t % NS) * Cfg::STAGE;
#pragma unroll
    for (int j = 0; j < LPW; ++j) {
      const int i = wave + j * Cfg::NW;
      const bool in = row[j] < mend;
      const float* src;
      if (j < Cfg::LPWG) {
        src = in ? rptr[j] : g_tn_zero;
        rptr[j] += gstep;
      } else if (GATHER) {
        const int ih = poh[j] * geo.S - geo.P + dkh[j], iw = pow_[j] * geo.S - geo.P + dkw[j];
        const bool ok = in && (unsigned)ih < (unsigned)geo.H && (unsigned)iw < (unsigned)geo.W;
        const uint32_t off = (((uint32_t)pn[j] * (uint32_t)geo.H + (uint32_t)ih) * (uint32_t)geo.W + (uint32_t)iw) *
                                 (uint32_t)geo.C + (uint32_t)ccol[j];
        src = ok ? X + off : g_tn_zero;
        pow_[j] += adv_r;
        poh[j] += adv_q;
        if (pow_[j] >= geo.OW) { pow_[j] -= geo.OW; ++poh[j]; }
        while (poh[j] >= geo.OH) { poh[j] -= geo.OH; ++pn[j]; }
      } else {
        src = in ? rptr[j] : g_tn_zero;
        rptr[j] += xstep;
      }
      row[j] += Cfg::ROWS;
      glds16(src, base + i * 1024);
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  // per-lane byte offsets of row 4g (+ j + 16 kg: immediates) of this lane's
  // column in each 16-column fragment
  const int fi = lane & 15, fg = lane >> 4;
  int goff[4], xoff[4];
#pragma unroll
  for (int s2 = 0; s2 < 4; ++s2) {
    const int gc = wn * 64 + s2 * 16 + fi;
    const int xc = wk * 64 + s2 * 16 + fi;
    const int r = 4 * fg;
    goff[s2] = r * Cfg::GROW + ((((gc >> 2) ^ swz4(r)) << 4) | ((gc & 3) << 2));
    xoff[s2] = Cfg::GBYTES_ALL + r * Cfg::XROW + ((((xc >> 2) ^ swz4(r)) << 4) | ((xc & 3) << 2));
  }
  // lazy operand: coefficients of this lane's four G columns (fixed for the block)
  float4 cf[4];
#pragma unroll
  for (int s2 = 0; s2 < 4; ++s2)
    cf[s2] = LZ ? reinterpret_cast<const float4*>(lz.coef)[n0 + wn * 64 + s2 * 16 + fi] : make_float4(0.f, 0.f, 0.f, 0.f);

  stage(0);
  if (NS >= 3 && T > 1) stage(1);
  for (int t = 0; t < T; ++t) {
    if (NS == 3) wait_vmcnt_fast<LPW>(t + 1 < T ? LPW : 0);
    else wait_vmcnt(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (t + NS - 1 < T) stage(t + NS - 1);
    const char* sb = smem + (t % NS) * Cfg::STAGE;
    const int64_t mst = mbeg + (int64_t)t * Cfg::ROWS;   // first row of this stage
    const bool tail = LZ && mst + Cfg::ROWS > mend;      // lazy: rows past the split must give 0, not k1(-k2 + mu k4)
    // fragments of k-group kg: [j][s2] (32 values); the next group's reads are
    // issued before this group's 64 MFMAs so only one LDS latency per stage shows
    float gv[2][4][4], xv[2][4][4];
    auto load = [&](int kg, float (&g)[4][4], float (&x)[4][4]) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int rr = kg * 16 + j;   // row offset of MFMA j's k-slot 0
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) {
          g[j][s2] = *reinterpret_cast<const float*>(sb + goff[s2] + rr * Cfg::GROW);
          x[j][s2] = *reinterpret_cast<const float*>(sb + xoff[s2] + rr * Cfg::XROW);
        }
        if constexpr (LZ) {
          const bool live = !tail || mst + rr + 4 * fg < mend;
#pragma unroll
          for (int s2 = 0; s2 < 4; ++s2) {
            const float xz = *reinterpret_cast<const float*>(sb + Cfg::GBYTES + goff[s2] + rr * Cfg::GROW);
            const float d = cf[s2].x * ((g[j][s2] - cf[s2].y) - (xz - cf[s2].z) * cf[s2].w);
            g[j][s2] = live ? d : 0.f;
          }
        }
      }
    };
    if constexpr (X6) {
      // bf16x6 products (gemm_nt_kernel X6): the lane's 8 rows {16 kg + 4 fg + j}
      // of a column form one 16x16x32 bf16 operand (the same row permutation on
      // G and X), split exactly into hi + mid + lo parts
      load(0, gv[0], xv[0]);
      load(1, gv[1], xv[1]);
      bf16x8 gh[4], gm[4], gl[4];
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2)
        split3x8(f32x4{gv[0][0][s2], gv[0][1][s2], gv[0][2][s2], gv[0][3][s2]},
                 f32x4{gv[1][0][s2], gv[1][1][s2], gv[1][2][s2], gv[1][3][s2]}, gh[s2], gm[s2], gl[s2]);
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        bf16x8 xh, xm, xl;
        split3x8(f32x4{xv[0][0][ks], xv[0][1][ks], xv[0][2][ks], xv[0][3][ks]},
                 f32x4{xv[1][0][ks], xv[1][1][ks], xv[1][2][ks], xv[1][3][ks]}, xh, xm, xl);
#pragma unroll
        for (int ns = 0; ns < 4; ++ns) {
          f32x4 c = acc[ns][ks];
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(gl[ns], xh, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(gh[ns], xl, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(gm[ns], xm, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(gm[ns], xh, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(gh[ns], xm, c, 0, 0, 0);
          acc[ns][ks] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(gh[ns], xh, c, 0, 0, 0);
        }
      }
      continue;
    }
    load(0, gv[0], xv[0]);
#pragma unroll
    for (int kg = 0; kg < Cfg::ROWS / 16; ++kg) {
      if (kg + 1 < Cfg::ROWS / 16) load(kg + 1, gv[(kg + 1) & 1], xv[(kg + 1) & 1]);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int ns = 0; ns < 4; ++ns)
#pragma unroll
          for (int ks = 0; ks < 4; ++ks)
            acc[ns][ks] = __builtin_amdgcn_mfma_f32_16x16x4f32(gv[kg & 1][j][ns], xv[kg & 1][j][ks], acc[ns][ks], 0, 0, 0);
    }
  }
  // D[i = n][j = c]: lane holds column c = .. + (lane & 15), rows n = .. + 4 (lane >> 4) + r
#pragma unroll
  for (int ns = 0; ns < 4; ++ns)
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int c = c0 + wk * 64 + ks * 16 + fi;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wn * 64 + ns * 16 + fg * 4 + r;
        atomicAdd(W + (int64_t)n * ldw + c, acc[ns][ks][r]);
      }
    }
}

template <int WN, int WK, int NS, bool GATHER, bool LZ = false, bool X6 = false>
void launch_tn_f32(const float* G, int64_t ldg, const float* X, int64_t ldx, float* W, int64_t ldw, int64_t M, int N,
                   int K, int splits, const ConvGeo& geo, const LazyA& lz, hipStream_t stream) {
  using Cfg = TnF32Cfg<WN, WK, NS, LZ>;
  const int tiles = (N / Cfg::BN) * (K / Cfg::BK);
  if (splits <= 0) {
    // two rounds of the chip's block slots (LDS-limited blocks per CU)
    static const int cus = [] {
      int d = 0, n = 0;
      hipGetDevice(&d);
      return hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, d) == hipSuccess && n > 0 ? n : 256;
    }();
    int bpc = (160 * 1024) / Cfg::LDS;
    const int by_waves = 16 / Cfg::NW;
    if (bpc > by_waves) bpc = by_waves;
    if (bpc < 1) bpc = 1;
    // splits < 0: -splits quarter rounds (see launch_tn); 0: two rounds
    const int64_t quarters = splits == 0 ? 8 : -(int64_t)splits;
    splits = (int)(quarters * (int64_t)cus * bpc / (4 * (int64_t)tiles));
    if (splits < 1) splits = 1;
  }
  int64_t rows = (M + splits - 1) / splits;
  rows = (rows + Cfg::ROWS - 1) / Cfg::ROWS * Cfg::ROWS;
  if (rows < 4 * Cfg::ROWS) rows = 4 * Cfg::ROWS;
  const int64_t nsplit = (M + rows - 1) / rows;
  dim3 grid((unsigned)(N / Cfg::BN), (unsigned)(K / Cfg::BK), (unsigned)nsplit);
  static bool attr = [] {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_tn_f32_kernel<WN, WK, NS, GATHER, LZ, X6>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, Cfg::LDS) == hipSuccess;
  }();
  (void)attr;
  hipLaunchKernelGGL((gemm_tn_f32_kernel<WN, WK, NS, GATHER, LZ, X6>), grid, dim3(Cfg::THREADS), Cfg::LDS, stream, G, ldg,
                     X, ldx, W, ldw, M, rows, geo, lz);
}

template <bool GATHER, bool X6 = false>
void tn_f32_dispatch(const float* G, int64_t ldg, const float* X, int64_t ldx, float* W, int64_t ldw, int64_t M, int N,
                     int K, int cfg, int splits, const ConvGeo& geo, const LazyArgs* lza, hipStream_t stream) {
  // cfg = tile + 10 * stages (0/2: three, 1: two).  tiles (WN, WK), 64x64 per wave:
  // 1 (1,1)  2 (2,1)  3 (1,2)  4 (2,2)  5 (4,1)  6 (1,4)  7 (4,2)  8 (2,4)  9 (4,4, two stages)
  const bool ns3 = (cfg / 10) % 10 != 1;
  cfg %= 10;
  if (cfg <= 0) cfg = (N % 128 == 0 && K % 128 == 0) ? 4 : (N % 128 == 0 ? 2 : (K % 128 == 0 ? 3 : 1));
  static const int cfg_bn[10] = {64, 64, 128, 64, 128, 256, 64, 256, 128, 256};
  static const int cfg_bk[10] = {64, 64, 64, 128, 128, 64, 256, 128, 256, 256};
  if (N % cfg_bn[cfg] != 0 || K % cfg_bk[cfg] != 0) cfg = 1;
  const LazyA lz = lza ? LazyA{lza->x, lza->coef, lza->padz, lza->padx, lza->C} : LazyA{};
#define GK_TNF(WN_, WK_)                                                                                      \
  do {                                                                                                        \
    if (lza) {                                                                                                \
      if (ns3 && TnF32Cfg<WN_, WK_, 3, true>::LDS <= 160 * 1024)                                              \
        launch_tn_f32<WN_, WK_, 3, GATHER, true, X6>(G, ldg, X, ldx, W, ldw, M, N, K, splits, geo, lz, stream);   \
      else                                                                                                    \
        launch_tn_f32<WN_, WK_, 2, GATHER, true, X6>(G, ldg, X, ldx, W, ldw, M, N, K, splits, geo, lz, stream);   \
    } else if (ns3 && TnF32Cfg<WN_, WK_, 3>::LDS <= 160 * 1024)                                               \
      launch_tn_f32<WN_, WK_, 3, GATHER, false, X6>(G, ldg, X, ldx, W, ldw, M, N, K, splits, geo, lz, stream);           \
    else                                                                                                      \
      launch_tn_f32<WN_, WK_, 2, GATHER, false, X6>(G, ldg, X, ldx, W, ldw, M, N, K, splits, geo, lz, stream);           \
  } while (0)
  switch (cfg) {
    case 2: GK_TNF(2, 1); break;
    case 3: GK_TNF(1, 2); break;
    case 4: GK_TNF(2, 2); break;
    case 5: GK_TNF(4, 1); break;
    case 6: GK_TNF(1, 4); break;
    case 7: GK_TNF(4, 2); break;
    case 8: GK_TNF(2, 4); break;
    case 9:
      if (lza) {
        GK_TNF(2, 4);   // the lazy 256x256 tile does not fit in LDS
      } else if (ns3 && TnF32Cfg<4, 4, 3>::LDS <= 160 * 1024) {
        launch_tn_f32<4, 4, 3, GATHER, false, X6>(G, ldg, X, ldx, W, ldw, M, N, K, splits, geo, lz, stream);
      } else {
        launch_tn_f32<4, 4, 2, GATHER, false, X6>(G, ldg, X, ldx, W, ldw, M, N, K, splits, geo, lz, stream);
      }
      break;
    default: GK_TNF(1, 1); break;
  }
#undef GK_TNF
}

// --------------------------------------------------------------------------
// gemm_nt, bf16x6 with register staging ("x62"): C[M, N] = A[M, K] B[N, K]^T,
// fp32 operands, row GEMMs only
// --------------------------------------------------------------------------
// The X6 form of gemm_nt_kernel stages fp32 tiles by LDS-DMA and every wave
// splits the fragments it reads, so each element is split once per wave that
// reads it (twice on a 2x2 wave grid) and every 1 KiB of fp32 costs one
// LDS-DMA issue (~60-185 cycles among MFMAs, MI355X_MICROARCH.md).  Here
// each thread loads 8 consecutive K elements of a row pair-wise into
// registers (global_load_dwordx4), splits them ONCE (split3x8) and writes the
// three bf16 planes to LDS; the MFMA loop reads bf16 fragments directly.  The
// next slice's loads are in flight during the current slice's MFMAs and its
// split + LDS writes are issued in the middle of them (two LDS stages of
// 3 x (BM + BN) x 64 bytes, one barrier per 32-deep K slice).  Persistent over
// M tiles like gemm_nt_kernel; XCD-aware block order; epilogue: bias, the
// BatchNorm statistics partials or the BN-backward dz (fp32 layouts of
// gemm_nt_kernel).
template <int WM, int WN>
struct X62Cfg {
  static constexpr int NW = WM * WN;
  static constexpr int THREADS = 64 * NW;
  static constexpr int BM = 64 * WM;
  static constexpr int BN = 64 * WN;
  static constexpr int PA = BM * 64;                 // bytes of one A plane (BM rows x 32 bf16)
  static constexpr int PB = BN * 64;
  static constexpr int STAGE = 3 * (PA + PB);
  static constexpr int LDS = 2 * STAGE;
  static constexpr int PRA = BM * 4 / THREADS;       // 8-element row pieces of A per thread per slice
  static constexpr int PRB = BN * 4 / THREADS;
  static_assert(PRA >= 1 && PRB >= 1 && (BM * 4) % THREADS == 0 && (BN * 4) % THREADS == 0, "pieces per thread");
  static_assert(LDS <= 160 * 1024, "LDS");
};

// 16-byte chunk q of a 64-byte plane row r lives at chunk q ^ x62_swz(r).  A
// ds_read_b128 is serviced in four 16-lane groups ({0-3,12-15,20-27},
// {4-11,16-19,28-31} and the same +32, MI355X_MICROARCH.md LDS table); a
// fragment read puts lane (fr, fq) on row base + fr, chunk fq.  XOR-ing the
// chunk with 2 * bit 3 of the row gives every group 16 distinct 16-byte bank
// slots (searched exhaustively; (r >> 2) & 3, which is conflict-free for
// contiguous 16-lane groups, measured 36% conflict cycles here).  The split
// writes (ds_write_b128, 8-lane groups on two adjacent rows) stay
// conflict-free under any per-row permutation.
__device__ __forceinline__ int x62_swz(int r) { return ((r >> 3) & 1) << 1; }

template <int WM, int WN, bool BNB, int NPF = 1, bool GATHER = false, bool P3 = false>
__global__ void __launch_bounds__(64 * WM * WN) __attribute__((amdgpu_waves_per_eu(1)))
gemm_nt_x62_kernel(const float* __restrict__ A, int64_t lda, const float* __restrict__ B, int64_t ldb,
                   float* __restrict__ C, int64_t ldc, int64_t M, int K, const float* __restrict__ bias,
                   float* __restrict__ stats, int64_t stats_ld, BnBwd bb, ConvGeo geo) {
  // GATHER: implicit-GEMM convolution over channels-last A = x [N, H, W, C]
  // (gemm_nt_kernel's ConvGeo, C a multiple of 32): row m is output pixel
  // (n, oh, ow), K slice ks is tap (kh, kw) of channels c0 .. c0 + 31; a tap
  // outside the image loads geo.zero
  using Cfg = X62Cfg<WM, WN>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int bx, by;
  xcd_remap2(bx, by);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int fr = lane & 15, fq = lane >> 4;
  const int n0 = by * Cfg::BN;
  const int Ntot = (int)gridDim.y * Cfg::BN;
  const int64_t mtiles = (M + Cfg::BM - 1) / Cfg::BM;
  const int nk = K / 32;
  const int64_t my_tiles = bx < mtiles ? (mtiles - 1 - bx) / gridDim.x + 1 : 0;
  const int T_ = (int)(my_tiles * nk);
  if (T_ == 0) {
    if (stats)
      for (int c = tid; c < Cfg::BN; c += Cfg::THREADS) {
        stats[(int64_t)bx * Ntot + n0 + c] = 0.f;
        stats[stats_ld + (int64_t)bx * Ntot + n0 + c] = 0.f;
      }
    return;
  }

  // ---- register staging: piece p of A is row cid >> 2, K elements 8 (cid & 3) .. +7
  // of the slice (cid = tid + THREADS p); same for B (rows of the weight panel)
  // NPF register sets: the loads of slice s go to set s % NPF (NPF = 2: two
  // slices in flight ahead of the one being multiplied)
  // P3: B arrives pre-split (geo.b3, [N][K/32][3][32] bf16): a B piece is three
  // 16-byte loads written to the planes as they are -- no split VALU for B
  f32x4 ra[NPF][Cfg::PRA][2], rb[NPF][P3 ? 1 : Cfg::PRB][2];
  u32x4 rb3[NPF][P3 ? Cfg::PRB : 1][3];
  const uint16_t* lpb3[P3 ? Cfg::PRB : 1];
  // load cursor: per-piece pointers to the next slice's 8 floats, advanced by
  // 32 floats per slice; the 64-bit row arithmetic runs only at an M-tile
  // change (a wave-uniform branch), not for every slice
  int64_t l_mt = bx;
  int l_ks = 0;
  const float* lpa[GATHER ? 1 : Cfg::PRA];
  const float* lpb[Cfg::PRB];
  // gather: tap / channel offset of the next slice (wave-uniform) and, per
  // piece, its output pixel's in-image taps (bits kh of okhw, bits 8 + kw) and
  // its 32-bit element offset into x (the host refuses x of >= 2^31 elements):
  // two registers per piece instead of four -- the 4x2-wave gather tiles
  // spilled with 64-bit pointers and separate tap masks
  int l_kh = 0, l_kw = 0, l_c0 = 0;
  uint32_t okhw[GATHER ? Cfg::PRA : 1];
  int32_t aoff[GATHER ? Cfg::PRA : 1];
  auto set_a_rows = [&]() __attribute__((always_inline)) {
    const int64_t m0 = l_mt * Cfg::BM;
#pragma unroll
    for (int p = 0; p < Cfg::PRA; ++p) {
      const int cid = tid + Cfg::THREADS * p;
      int64_t gr = m0 + (cid >> 2);
      gr = gr < M ? gr : M - 1;   // tail rows: computed, never stored
      if constexpr (GATHER) {
        const uint32_t ohw = (uint32_t)(geo.OH * geo.OW);
        const uint32_t mu = (uint32_t)gr;
        const uint32_t n = mu / ohw, rem = mu - n * ohw;
        const uint32_t oh = rem / (uint32_t)geo.OW, ow = rem - oh * (uint32_t)geo.OW;
        const int ih0 = (int)oh * geo.S - geo.P, iw0 = (int)ow * geo.S - geo.P;
        uint32_t bh = 0u, bw = 0u;
#pragma unroll
        for (int t = 0; t < kMaxTaps; ++t) {
          bh |= (uint32_t)((unsigned)(ih0 + t) < (unsigned)geo.H) << t;
          bw |= (uint32_t)((unsigned)(iw0 + t) < (unsigned)geo.W) << t;
        }
        okhw[p] = bh | (bw << 8);
        aoff[p] = (((int)n * geo.H + ih0) * geo.W + iw0) * geo.C + (cid & 3) * 8;
      } else {
        lpa[p] = A + gr * lda + (cid & 3) * 8;
      }
    }
  };
  set_a_rows();
#pragma unroll
  for (int p = 0; p < Cfg::PRB; ++p) {
    const int cid = tid + Cfg::THREADS * p;
    if constexpr (P3) lpb3[p] = geo.b3 + (int64_t)(n0 + (cid >> 2)) * (3 * K) + (cid & 3) * 8;
    else lpb[p] = B + (int64_t)(n0 + (cid >> 2)) * ldb + (cid & 3) * 8;
  }
  const float* zrow = static_cast<const float*>(geo.zero);
  auto issue_loads = [&](auto SET) __attribute__((always_inline)) {
    constexpr int q = decltype(SET)::value;
    const int64_t toff = GATHER ? (int64_t)(l_kh * geo.W + l_kw) * geo.C + l_c0 : 0;   // wave-uniform
#pragma unroll
    for (int p = 0; p < Cfg::PRA; ++p) {
      const float* src;
      if constexpr (GATHER) {
        const bool ok = ((okhw[p] >> l_kh) & (okhw[p] >> (8 + l_kw)) & 1u) != 0u;
        src = ok ? A + ((int64_t)aoff[p] + toff) : zrow;
      } else {
        src = lpa[p];
        lpa[p] += 32;
      }
      ra[q][p][0] = *reinterpret_cast<const f32x4*>(src);
      ra[q][p][1] = *reinterpret_cast<const f32x4*>(src + 4);
    }
#pragma unroll
    for (int p = 0; p < Cfg::PRB; ++p) {
      if constexpr (P3) {
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) rb3[q][p][pl] = *reinterpret_cast<const u32x4*>(lpb3[p] + pl * 32);
        lpb3[p] += 96;
      } else {
        rb[q][p][0] = *reinterpret_cast<const f32x4*>(lpb[p]);
        rb[q][p][1] = *reinterpret_cast<const f32x4*>(lpb[p] + 4);
        lpb[p] += 32;
      }
    }
    if constexpr (GATHER) {
      l_c0 += 32;
      if (l_c0 == geo.C) {
        l_c0 = 0;
        if (++l_kw == geo.KW) {
          l_kw = 0;
          ++l_kh;
        }
      }
    }
    if (++l_ks == nk) {
      l_ks = 0;
      l_kh = l_kw = l_c0 = 0;
      l_mt += gridDim.x;
      set_a_rows();
#pragma unroll
      for (int p = 0; p < Cfg::PRB; ++p) {
        if constexpr (P3) lpb3[p] -= 3 * K;
        else lpb[p] -= K;
      }
    }
  };
  // piece pc of the slice (A pieces 0 .. PRA-1, then B pieces), or all of them (pc < 0)
  auto split_write = [&](int buf, auto SET, int pc = -1) __attribute__((always_inline)) {
    constexpr int q = decltype(SET)::value;
    char* st = smem + buf * Cfg::STAGE;
#pragma unroll
    for (int p = 0; p < Cfg::PRA; ++p) {
      if (pc >= 0 && pc != p) continue;
      const int cid = tid + Cfg::THREADS * p;
      const int r = cid >> 2;
      bf16x8 h, m, l;
      split3x8(ra[q][p][0], ra[q][p][1], h, m, l);
      const int off = r * 64 + (((cid & 3) ^ x62_swz(r)) << 4);
      *reinterpret_cast<bf16x8*>(st + off) = h;
      *reinterpret_cast<bf16x8*>(st + Cfg::PA + off) = m;
      *reinterpret_cast<bf16x8*>(st + 2 * Cfg::PA + off) = l;
    }
    char* sb = st + 3 * Cfg::PA;
#pragma unroll
    for (int p = 0; p < Cfg::PRB; ++p) {
      if (pc >= 0 && pc != Cfg::PRA + p) continue;
      const int cid = tid + Cfg::THREADS * p;
      const int r = cid >> 2;
      const int off = r * 64 + (((cid & 3) ^ x62_swz(r)) << 4);
      if constexpr (P3) {
        *reinterpret_cast<u32x4*>(sb + off) = rb3[q][p][0];
        *reinterpret_cast<u32x4*>(sb + Cfg::PB + off) = rb3[q][p][1];
        *reinterpret_cast<u32x4*>(sb + 2 * Cfg::PB + off) = rb3[q][p][2];
      } else {
        bf16x8 h, m, l;
        split3x8(rb[q][p][0], rb[q][p][1], h, m, l);
        *reinterpret_cast<bf16x8*>(sb + off) = h;
        *reinterpret_cast<bf16x8*>(sb + Cfg::PB + off) = m;
        *reinterpret_cast<bf16x8*>(sb + 2 * Cfg::PB + off) = l;
      }
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  // (BN-backward epilogue: no bias -- the binding makes them exclusive -- so
  // no 16 bias registers beside its operand loads)
  float ssum[4][4], ssq[4][4], bia[BNB ? 1 : 4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      ssum[a][b] = ssq[a][b] = 0.f;
      if constexpr (!BNB) bia[a][b] = bias ? bias[n0 + wn * 64 + a * 16 + fq * 4 + b] : 0.f;
    }

  auto epilogue = [&](int64_t mt) __attribute__((always_inline)) {
    const int64_t mbase = mt * Cfg::BM;
    // BN-backward operands two fragments at a time (all four beside the
    // accumulators and the staged next slice spill at 256 VGPRs)
    constexpr int EH = BNB ? 1 : 4;
#pragma unroll
    for (int ms = 0; ms < 4; ++ms) {
      const int64_t m = mbase + wm * 64 + ms * 16 + fr;
      const bool live = m < M;
#pragma unroll
      for (int nh = 0; nh < 4; nh += EH) {
      f32x4 ehv[EH], ed2[EH];
      uint32_t ebits[EH];
      if constexpr (BNB) {
#pragma unroll
        for (int e = 0; e < EH; ++e) {
          ehv[e] = ed2[e] = f32x4{0.f, 0.f, 0.f, 0.f};
          ebits[e] = 0u;
        }
        if (live) {
#pragma unroll
          for (int e = 0; e < EH; ++e) {
            const int n = n0 + wn * 64 + (nh + e) * 16 + fq * 4;
            ehv[e] = *reinterpret_cast<const f32x4*>(static_cast<const float*>(bb.h) + m * ldc + n);
            if (bb.dy2) ed2[e] = *reinterpret_cast<const f32x4*>(static_cast<const float*>(bb.dy2) + m * ldc + n);
            ebits[e] = bb.mask ? (uint32_t)bb.mask[m * (Ntot >> 2) + (n >> 2)] : 0xfu;
          }
        }
      }
#pragma unroll
      for (int e = 0; e < EH; ++e) {
        const int ns = nh + e;
        const int n = n0 + wn * 64 + ns * 16 + fq * 4;
        f32x4 v = acc[ms][ns];
        acc[ms][ns] = f32x4{0.f, 0.f, 0.f, 0.f};
        if constexpr (!BNB) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] += bia[ns][r];
        }
        if constexpr (BNB) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float dz = (ebits[e] >> r) & 1u ? v[r] + ed2[e][r] : 0.f;
            v[r] = dz;
            ssum[ns][r] += dz;
            ssq[ns][r] = fmaf(dz, ehv[e][r], ssq[ns][r]);
          }
        } else {
          if (stats && live) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              ssum[ns][r] += v[r];
              ssq[ns][r] = fmaf(v[r], v[r], ssq[ns][r]);
            }
          }
        }
        if (live) *reinterpret_cast<f32x4*>(C + m * ldc + n) = v;
      }
      }
    }
  };

  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, (NPF > 1 ? 1 : 0)>;
  // prologue: slice 0 into LDS stage 0, slices 1 .. NPF in flight
  issue_loads(I0{});
  split_write(0, I0{});
  if (T_ > 1) issue_loads(I1{});
  if (NPF > 1 && T_ > 2) issue_loads(I0{});
  __syncthreads();
  int ks = 0;
  int64_t mt = bx;
  // one K slice t (register set of slice t + 1: (t + 1) % NPF, compile-time through PAR = t % 2)
  auto slice = [&](int t, auto PAR) __attribute__((always_inline)) {
    constexpr int par = decltype(PAR)::value;
    using SN = std::integral_constant<int, (NPF > 1 ? (par ^ 1) : 0)>;   // set holding slice t + 1
    const int cur = par;
    const char* st = smem + cur * Cfg::STAGE;
    const char* pa = st;
    const char* pb = st + 3 * Cfg::PA;
    auto frag = [&](const char* plane, int row) __attribute__((always_inline)) -> bf16x8 {
      return *reinterpret_cast<const bf16x8*>(plane + row * 64 + ((fq ^ x62_swz(row)) << 4));
    };
    bf16x8 bh[4], bm[4], bl[4];
#pragma unroll
    for (int ns = 0; ns < 4; ++ns) {
      const int row = wn * 64 + ns * 16 + fr;
      bh[ns] = frag(pb, row);
      bm[ns] = frag(pb + Cfg::PB, row);
      bl[ns] = frag(pb + 2 * Cfg::PB, row);
    }
    // The next slice's split pieces, plane writes and loads go between this
    // slice's MFMA groups (program order fixed by sched_barrier: a wave issues
    // in order, so VALU after a long MFMA run would wait for the matrix pipe
    // instead of filling the 8 of every 16 cycles an MFMA leaves free).
    constexpr int NPC = Cfg::PRA + Cfg::PRB;   // split pieces per thread per slice
#pragma unroll
    for (int ms = 0; ms < 4; ++ms) {
      const int row = wm * 64 + ms * 16 + fr;
      const bf16x8 ah = frag(pa, row), am = frag(pa + Cfg::PA, row), al = frag(pa + 2 * Cfg::PA, row);
#pragma unroll
      for (int ns = 0; ns < 4; ++ns) {
        f32x4 c = acc[ms][ns];
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bl[ns], ah, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh[ns], al, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bm[ns], am, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bm[ns], ah, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh[ns], am, c, 0, 0, 0);
        acc[ms][ns] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh[ns], ah, c, 0, 0, 0);
        // step g = 4 ms + ns (16 steps): pieces on steps 1 .. NPC, the loads
        // on step NPC + 1 (all past the block's last slice too: the cursor
        // walks on over clamped, valid rows; the writes go to the stage nobody
        // reads again -- no branch, nothing for the scheduler to cluster around)
        const int gstep = 4 * ms + ns;
        if (gstep >= 1 && gstep <= NPC) split_write(cur ^ 1, SN{}, gstep - 1);
        if (gstep == NPC + 1) issue_loads(SN{});
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if (++ks == nk) {
      ks = 0;
      epilogue(mt);
      mt += gridDim.x;
    }
    __syncthreads();
  };
  for (int t = 0; t < T_; t += 2) {
    slice(t, I0{});
    if (t + 1 < T_) slice(t + 1, std::integral_constant<int, 1>{});
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
    float* red = reinterpret_cast<float*>(smem);   // [2][WM][BN]; every stage is consumed
    if (fr == 0) {
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int col = wn * 64 + a * 16 + fq * 4 + b;
          red[wm * Cfg::BN + col] = ssum[a][b];
          red[(WM + wm) * Cfg::BN + col] = ssq[a][b];
        }
    }
    __syncthreads();
    for (int c = tid; c < Cfg::BN; c += Cfg::THREADS) {
      float sa = 0.f, sb = 0.f;
#pragma unroll
      for (int w2 = 0; w2 < WM; ++w2) {
        sa += red[w2 * Cfg::BN + c];
        sb += red[(WM + w2) * Cfg::BN + c];
      }
      stats[(int64_t)bx * Ntot + n0 + c] = sa;
      stats[stats_ld + (int64_t)bx * Ntot + n0 + c] = sb;
    }
  }
}

template <int WM, int WN, bool BNB, int NPF, bool GATHER, bool P3 = false>
int launch_nt_x62(const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc, int64_t M, int N,
                  int K, int max_blocks, const float* bias, float* stats, int64_t stats_ld, int stats_rows,
                  const BnBwd& bb, const ConvGeo& geo, hipStream_t stream) {
  using Cfg = X62Cfg<WM, WN>;
  const int ntiles = N / Cfg::BN;
  const int64_t mtiles = (M + Cfg::BM - 1) / Cfg::BM;
  const int per_cu = (160 * 1024) / Cfg::LDS > 0 ? (160 * 1024) / Cfg::LDS : 1;
  int64_t gx = ((int64_t)256 * per_cu + ntiles - 1) / ntiles;
  if (max_blocks > 0) gx = max_blocks;
  if (gx < 1) gx = 1;
  if (gx > mtiles) gx = mtiles;
  if (stats && gx > stats_rows) gx = stats_rows;   // one partial row per block
  static bool attr = [] {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_nt_x62_kernel<WM, WN, BNB, NPF, GATHER, P3>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
  }();
  (void)attr;
  hipLaunchKernelGGL((gemm_nt_x62_kernel<WM, WN, BNB, NPF, GATHER, P3>), dim3((unsigned)gx, (unsigned)ntiles), dim3(Cfg::THREADS),
                     Cfg::LDS, stream, A, lda, B, ldb, C, ldc, M, K, bias, stats, stats_ld, bb, geo);
  return (int)gx;
}

// cfg % 10: tile (WM, WN) of 64x64 wave tiles: 1 (2,2) 128x128, 2 (2,4) 128x256, 3 (4,2) 256x128,
// 4 (1,4) 64x256, 5 (4,1) 256x64, 6 (1,2) 64x128, 7 (2,1) 128x64
template <bool GATHER>
int nt_x62_dispatch(const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc, int64_t M,
                    int N, int K, int cfg, int max_blocks, const float* bias, float* stats, int64_t stats_ld,
                    int stats_rows, const BnBwd& bb, const ConvGeo& geo, hipStream_t stream) {
  static const int cfg_bn[8] = {128, 128, 256, 128, 256, 64, 128, 64};
  cfg %= 10;
  if (cfg < 1 || cfg > 7 || N % cfg_bn[cfg] != 0) cfg = N % 128 == 0 ? 1 : 7;
  if (N % cfg_bn[cfg] != 0) cfg = 5;
#define GK_X62N(WM_, WN_, P3_)                                                                                      \
  return bb.h ? launch_nt_x62<WM_, WN_, true, 1, GATHER, P3_>(A, lda, B, ldb, C, ldc, M, N, K, max_blocks, bias, stats, \
                                                              stats_ld, stats_rows, bb, geo, stream)                  \
              : launch_nt_x62<WM_, WN_, false, 1, GATHER, P3_>(A, lda, B, ldb, C, ldc, M, N, K, max_blocks, bias,     \
                                                               stats, stats_ld, stats_rows, bb, geo, stream)
  // (two register sets in flight, cfg digit 10, measured slower everywhere: no longer instantiated)
#define GK_X62(WM_, WN_)                  \
  do {                                    \
    if (geo.b3) GK_X62N(WM_, WN_, true);  \
    GK_X62N(WM_, WN_, false);             \
  } while (0)
  switch (cfg) {
    case 2: GK_X62(2, 4);
    case 3: GK_X62(4, 2);
    case 4: GK_X62(1, 4);
    case 5: GK_X62(4, 1);
    case 6: GK_X62(1, 2);
    case 7: GK_X62(2, 1);
    default: GK_X62(2, 2);
  }
#undef GK_X62
#undef GK_X62N
}

// --------------------------------------------------------------------------
// gemm_tn, bf16x6 with register staging ("x62"): W[N, K] += G[M, N]^T X[M, K]
// --------------------------------------------------------------------------
// The grad-weight counterpart of gemm_nt_x62_kernel (row form: 1x1 stride-1
// convolutions, linear layers).  The contraction runs over the pixel rows M,
// so a bf16 MFMA operand wants 8 consecutive ROWS of one column per lane: a
// staging thread loads 8 rows x 4 columns (eight 16-byte loads, each wave
// instruction one contiguous row segment), splits every column's 8 rows once
// (split3x8) and writes them as one 16-byte chunk of that column's 64-byte
// plane row -- the transpose happens in registers, the LDS image is the NT
// kernel's ([column][32 rows] per plane, same conflict-free swizzle).  Each
// block reduces a contiguous slice of M for one output tile and adds its fp32
// partial into W with float atomics, like gemm_tn_f32_kernel.
template <int WN, int WK>
struct TnX62Cfg {
  static constexpr int NW = WN * WK;
  static constexpr int THREADS = 64 * NW;
  static constexpr int BN = 64 * WN;
  static constexpr int BK = 64 * WK;
  static constexpr int PG = BN * 64;                  // bytes of one G plane (BN columns x 32 rows)
  static constexpr int PX = BK * 64;
  static constexpr int STAGE = 3 * (PG + PX);
  static constexpr int LDS = 2 * STAGE;
  static constexpr int PIECES = BN + BK;              // 8 rows x 4 columns each: BN / 4 x 4 for G, BK / 4 x 4 for X
  static constexpr int PPT = (PIECES + THREADS - 1) / THREADS;
  static constexpr int ROWS = 32;
  static_assert(LDS <= 160 * 1024, "LDS");
};

template <int WN, int WK>
__global__ void __launch_bounds__(64 * WN * WK) __attribute__((amdgpu_waves_per_eu(1)))
gemm_tn_x62_kernel(const float* __restrict__ G, int64_t ldg, const float* __restrict__ X, int64_t ldx,
                   float* __restrict__ W, int64_t ldw, int64_t M, int64_t rows_per_split) {
  using Cfg = TnX62Cfg<WN, WK>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int bx, by, bz;
  xcd_remap3(bx, by, bz);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wk = wave % WK, wn = wave / WK;
  const int fr = lane & 15, fq = lane >> 4;
  const int n0 = bx * Cfg::BN;
  const int c0 = by * Cfg::BK;
  const int64_t mbeg = (int64_t)bz * rows_per_split;
  int64_t mend = mbeg + rows_per_split;
  if (mend > M) mend = M;
  if (mbeg >= mend) return;
  const int T_ = (int)((mend - mbeg + Cfg::ROWS - 1) / Cfg::ROWS);

  // piece pid: G pieces first (column chunk pid % (BN/4), row group pid / (BN/4)), then X
  f32x4 rv[Cfg::PPT][8];
  int64_t l_row = mbeg;   // first row of the next slice to load
  auto issue_loads = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < Cfg::PPT; ++j) {
      const int pid = tid + Cfg::THREADS * j;
      if (pid >= Cfg::PIECES) break;   // wave-uniform (PIECES is a multiple of 64)
      const bool isg = pid < Cfg::BN;
      const int q = isg ? pid : pid - Cfg::BN;
      const int nchunk = (isg ? Cfg::BN : Cfg::BK) / 4;
      const int cc = q % nchunk, rg = q / nchunk;
      const float* base = isg ? G + n0 + 4 * cc : X + c0 + 4 * cc;
      const int64_t ld = isg ? ldg : ldx;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int64_t r = l_row + 8 * rg + i;
        const int64_t rc = r < mend ? r : mend - 1;
        const f32x4 v = *reinterpret_cast<const f32x4*>(base + rc * ld);
        rv[j][i] = r < mend ? v : f32x4{0.f, 0.f, 0.f, 0.f};   // rows past the split contribute 0
      }
    }
    l_row += Cfg::ROWS;
  };
  auto split_write = [&](int buf, int jj) __attribute__((always_inline)) {
    char* st = smem + buf * Cfg::STAGE;
#pragma unroll
    for (int j = 0; j < Cfg::PPT; ++j) {
      if (jj >= 0 && j != jj) continue;
      const int pid = tid + Cfg::THREADS * j;
      if (pid >= Cfg::PIECES) break;
      const bool isg = pid < Cfg::BN;
      const int q = isg ? pid : pid - Cfg::BN;
      const int nchunk = (isg ? Cfg::BN : Cfg::BK) / 4;
      const int cc = q % nchunk, rg = q / nchunk;
      char* pl = isg ? st : st + 3 * Cfg::PG;
      const int psz = isg ? Cfg::PG : Cfg::PX;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        bf16x8 h, m, l;
        split3x8(f32x4{rv[j][0][c], rv[j][1][c], rv[j][2][c], rv[j][3][c]},
                 f32x4{rv[j][4][c], rv[j][5][c], rv[j][6][c], rv[j][7][c]}, h, m, l);
        const int col = 4 * cc + c;
        const int off = col * 64 + ((rg ^ x62_swz(col)) << 4);
        *reinterpret_cast<bf16x8*>(pl + off) = h;
        *reinterpret_cast<bf16x8*>(pl + psz + off) = m;
        *reinterpret_cast<bf16x8*>(pl + 2 * psz + off) = l;
      }
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  issue_loads();
  split_write(0, -1);
  issue_loads();
  __syncthreads();
  auto slice = [&](int t, auto PAR) __attribute__((always_inline)) {
    constexpr int cur = decltype(PAR)::value;
    const char* st = smem + cur * Cfg::STAGE;
    const char* pg = st;
    const char* px = st + 3 * Cfg::PG;
    auto frag = [&](const char* plane, int col) __attribute__((always_inline)) -> bf16x8 {
      return *reinterpret_cast<const bf16x8*>(plane + col * 64 + ((fq ^ x62_swz(col)) << 4));
    };
    bf16x8 gh[4], gm[4], gl[4];
#pragma unroll
    for (int ns = 0; ns < 4; ++ns) {
      const int col = wn * 64 + ns * 16 + fr;
      gh[ns] = frag(pg, col);
      gm[ns] = frag(pg + Cfg::PG, col);
      gl[ns] = frag(pg + 2 * Cfg::PG, col);
    }
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int col = wk * 64 + ks * 16 + fr;
      const bf16x8 xh = frag(px, col), xm = frag(px + Cfg::PX, col), xl = frag(px + 2 * Cfg::PX, col);
#pragma unroll
      for (int ns = 0; ns < 4; ++ns) {
        f32x4 c = acc[ns][ks];
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(gl[ns], xh, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(gh[ns], xl, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(gm[ns], xm, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(gm[ns], xh, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(gh[ns], xm, c, 0, 0, 0);
        acc[ns][ks] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(gh[ns], xh, c, 0, 0, 0);
        // next slice's pieces between the MFMA groups (branch-free: past the
        // split's end the loads read clamped rows and zero them; the writes go
        // to the stage nobody reads again)
        const int gstep = 4 * ks + ns;
        if (gstep >= 1 && gstep <= Cfg::PPT) split_write(cur ^ 1, gstep - 1);
        if (gstep == Cfg::PPT + 1) issue_loads();
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    __syncthreads();
  };
  for (int t = 0; t < T_; t += 2) {
    slice(t, std::integral_constant<int, 0>{});
    if (t + 1 < T_) slice(t + 1, std::integral_constant<int, 1>{});
  }
  // D[i = n][j = k]: lane holds column k = .. + fr, rows n = .. + 4 fq + r
#pragma unroll
  for (int ns = 0; ns < 4; ++ns)
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int c = c0 + wk * 64 + ks * 16 + fr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wn * 64 + ns * 16 + fq * 4 + r;
        atomicAdd(W + (int64_t)n * ldw + c, acc[ns][ks][r]);
      }
    }
}

template <int WN, int WK>
void launch_tn_x62(const float* G, int64_t ldg, const float* X, int64_t ldx, float* W, int64_t ldw, int64_t M, int N,
                   int K, int splits, hipStream_t stream) {
  using Cfg = TnX62Cfg<WN, WK>;
  const int tiles = (N / Cfg::BN) * (K / Cfg::BK);
  if (splits <= 0) {
    static const int cus = [] {
      int d = 0, n = 0;
      (void)hipGetDevice(&d);
      return hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, d) == hipSuccess && n > 0 ? n : 256;
    }();
    const int bpc = (160 * 1024) / Cfg::LDS > 0 ? (160 * 1024) / Cfg::LDS : 1;
    splits = (int)(2 * (int64_t)cus * bpc / tiles);
    if (splits < 1) splits = 1;
  }
  int64_t rows = (M + splits - 1) / splits;
  rows = (rows + Cfg::ROWS - 1) / Cfg::ROWS * Cfg::ROWS;
  if (rows < 4 * Cfg::ROWS) rows = 4 * Cfg::ROWS;
  const int64_t nsplit = (M + rows - 1) / rows;
  static bool attr = [] {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_tn_x62_kernel<WN, WK>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
  }();
  (void)attr;
  hipLaunchKernelGGL((gemm_tn_x62_kernel<WN, WK>), dim3((unsigned)(N / Cfg::BN), (unsigned)(K / Cfg::BK), (unsigned)nsplit),
                     dim3(Cfg::THREADS), Cfg::LDS, stream, G, ldg, X, ldx, W, ldw, M, rows);
}

// cfg % 10: tile (WN, WK) of 64x64 wave tiles: 1 (1,1) 64x64  2 (2,1) 128x64  3 (1,2) 64x128  4 (2,2) 128x128
// 5 (4,1) 256x64  6 (1,4) 64x256  7 (4,2) 256x128  8 (2,4) 128x256
inline void tn_x62_dispatch(const float* G, int64_t ldg, const float* X, int64_t ldx, float* W, int64_t ldw, int64_t M,
                            int N, int K, int cfg, int splits, hipStream_t stream) {
  static const int cfg_bn[9] = {64, 64, 128, 64, 128, 256, 64, 256, 128};
  static const int cfg_bk[9] = {64, 64, 64, 128, 128, 64, 256, 128, 256};
  cfg %= 10;
  if (cfg < 1 || cfg > 8 || N % cfg_bn[cfg] != 0 || K % cfg_bk[cfg] != 0) cfg = 1;
  switch (cfg) {
    case 2: launch_tn_x62<2, 1>(G, ldg, X, ldx, W, ldw, M, N, K, splits, stream); break;
    case 3: launch_tn_x62<1, 2>(G, ldg, X, ldx, W, ldw, M, N, K, splits, stream); break;
    case 4: launch_tn_x62<2, 2>(G, ldg, X, ldx, W, ldw, M, N, K, splits, stream); break;
    case 5: launch_tn_x62<4, 1>(G, ldg, X, ldx, W, ldw, M, N, K, splits, stream); break;
    case 6: launch_tn_x62<1, 4>(G, ldg, X, ldx, W, ldw, M, N, K, splits, stream); break;
    case 7: launch_tn_x62<4, 2>(G, ldg, X, ldx, W, ldw, M, N, K, splits, stream); break;
    case 8: launch_tn_x62<2, 4>(G, ldg, X, ldx, W, ldw, M, N, K, splits, stream); break;
    default: launch_tn_x62<1, 1>(G, ldg, X, ldx, W, ldw, M, N, K, splits, stream); break;
  }
}

template <bool GATHER, typename T, bool X6 = false>
int nt_dispatch(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int64_t M, int N,
                int K, int cfg, int max_blocks, const ConvGeo& geo, float* stats, int64_t stats_ld, int stats_rows,
                const BnBwd& bb, const LazyArgs* lza, hipStream_t stream) {
  // cfg = tile + 10 * panel (1: resident, 2: streamed) + 100 * stages (0: three, 1: two, 2: four; a
  // four-stage request falls back to three where the counts or the LDS do not fit)
  // + 1000 * family (fp32 only; 1: 32x64 wave tiles -- twice the waves of the 64x64 tiles for the
  // small-M layers of small batches, where the 64x64 grid leaves SIMDs idle)
  const int bres = (cfg / 10) % 10 == 0 ? -1 : ((cfg / 10) % 10 == 1 ? 1 : 0);
  const int ns = (cfg / 100) % 10 == 1 ? 2 : ((cfg / 100) % 10 == 2 ? 4 : 3);
  const int fam = (cfg / 1000) % 10;
  cfg %= 10;
  auto a = static_cast<const T*>(A);
  auto b = static_cast<const T*>(B);
  auto c = static_cast<T*>(C);
  const int cfg_req = cfg;   // the 32x64 family checks its own tile widths
  if (cfg <= 0) cfg = N % 256 == 0 ? 3 : (N % 128 == 0 ? 2 : 1);
  // tiles (BM x BN, waves): 1 256x64 (4)  2 256x128 (8)  3 128x256 (8)  4 128x128 (4)
  //                         5 256x256 (8, 128x64 per wave)  6 256x128 (4, 128x64)  7 128x256 (4, 128x64)
  // fp32 runs 64x64 wave tiles only (5-7 map to the 64x64 tile of the same block width)
  static const int cfg_bn[8] = {64, 64, 128, 256, 128, 256, 128, 256};
  if (cfg > 7 || N % cfg_bn[cfg] != 0) cfg = 1;   // the tile must divide N (B rows are not clamped)
  const LazyA lz = lza ? LazyA{lza->x, lza->coef, lza->padz, lza->padx, lza->C} : LazyA{};
#define GK_NTA(WM_, WN_, MSB_, BNB_, LZ_) \
  return launch_nt_any<WM_, WN_, GATHER, MSB_, BNB_, T, LZ_, X6>(a, lda, b, ldb, c, ldc, M, N, K, max_blocks, bres, ns, geo, stats, stats_ld, stats_rows, bb, lz, stream)
  if constexpr (sizeof(T) == 4) {
    if (lza) {   // lazy BN-backward A operand (fp32)
      if (bb.h) {
        switch (cfg) {
          case 2: GK_NTA(4, 2, 4, true, true);
          case 3: case 5: case 7: GK_NTA(2, 4, 4, true, true);
          case 4: case 6: GK_NTA(2, 2, 4, true, true);
          default: GK_NTA(4, 1, 4, true, true);
        }
      }
      switch (cfg) {
        case 2: GK_NTA(4, 2, 4, false, true);
        case 3: case 5: case 7: GK_NTA(2, 4, 4, false, true);
        case 4: case 6: GK_NTA(2, 2, 4, false, true);
        default: GK_NTA(4, 1, 4, false, true);
      }
    }
  }
  if constexpr (sizeof(T) == 4) {
    if (fam == 1 && !lza) {
      // 32x64 wave tiles: 1 128x64 (4 waves)  2 64x128 (4)  3 64x64 (2)  4 32x256 (4)  5 128x128 (8)
      //                   6 64x256 (8)  7 32x128 (2)
      static const int bn32[8] = {64, 64, 128, 64, 256, 128, 256, 128};
      cfg = cfg_req;
      if (cfg <= 0 || cfg > 7 || N % bn32[cfg] != 0) cfg = 1;
      if (bb.h) {
        switch (cfg) {
          case 2: GK_NTA(2, 2, 2, true, false);
          case 3: GK_NTA(2, 1, 2, true, false);
          case 4: GK_NTA(1, 4, 2, true, false);
          case 5: GK_NTA(4, 2, 2, true, false);
          case 6: GK_NTA(2, 4, 2, true, false);
          case 7: GK_NTA(1, 2, 2, true, false);
          default: GK_NTA(4, 1, 2, true, false);
        }
      }
      switch (cfg) {
        case 2: GK_NTA(2, 2, 2, false, false);
        case 3: GK_NTA(2, 1, 2, false, false);
        case 4: GK_NTA(1, 4, 2, false, false);
        case 5: GK_NTA(4, 2, 2, false, false);
        case 6: GK_NTA(2, 4, 2, false, false);
        case 7: GK_NTA(1, 2, 2, false, false);
        default: GK_NTA(4, 1, 2, false, false);
      }
    }
  }
  if (bb.h) {   // BN-backward epilogue: 64x64 wave tiles only
    switch (cfg) {
      case 2: GK_NTA(4, 2, 4, true, false);
      case 3: case 5: case 7: GK_NTA(2, 4, 4, true, false);
      case 4: case 6: GK_NTA(2, 2, 4, true, false);
      default: GK_NTA(4, 1, 4, true, false);
    }
  }
  if constexpr (sizeof(T) == 4) {
    if constexpr (X6) {   // bf16x6: 128x64 wave tiles (fewer operand splits and LDS reads per product)
      switch (cfg) {
        case 5: GK_NTA(2, 4, 8, false, false);
        case 6: GK_NTA(2, 2, 8, false, false);
        case 7: GK_NTA(1, 4, 8, false, false);
        default: break;
      }
    }
    switch (cfg) {
      case 2: GK_NTA(4, 2, 4, false, false);
      case 3: case 5: GK_NTA(2, 4, 4, false, false);
      case 7: GK_NTA(1, 4, 4, false, false);
      case 4: case 6: GK_NTA(2, 2, 4, false, false);
      default: GK_NTA(4, 1, 4, false, false);
    }
  } else {
    switch (cfg) {
      case 2: GK_NTA(4, 2, 4, false, false);
      case 3: GK_NTA(2, 4, 4, false, false);
      case 4: GK_NTA(2, 2, 4, false, false);
      case 5: GK_NTA(2, 4, 8, false, false);
      case 6: GK_NTA(2, 2, 8, false, false);
      case 7: GK_NTA(1, 4, 8, false, false);
      default: GK_NTA(4, 1, 4, false, false);
    }
  }
#undef GK_NTA
}

template <int WN, int WK, int WS, bool GATHER, int MSN = 1>
void launch_tn_any(const uint16_t* G, int64_t ldg, const uint16_t* X, int64_t ldx, float* W, int64_t ldw, int64_t M,
                   int N, int K, int splits, int ns, const ConvGeo& geo, hipStream_t stream) {
  if (ns == 3 && TnCfg<WN, WK, WS, 3, MSN>::LDS <= 160 * 1024)
    launch_tn<WN, WK, WS, 3, GATHER, MSN>(G, ldg, X, ldx, W, ldw, M, N, K, splits, geo, stream);
  else launch_tn<WN, WK, WS, 2, GATHER, MSN>(G, ldg, X, ldx, W, ldw, M, N, K, splits, geo, stream);
}

template <bool GATHER>
void tn_dispatch(const void* G, int64_t ldg, const void* X, int64_t ldx, float* W, int64_t ldw, int64_t M, int N,
                 int K, int cfg, int splits, const ConvGeo& geo, hipStream_t stream) {
  // cfg = tile digit + 10 * (1: two stages, 2: three) + 100 * tile group.
  // tile = cfg % 10 + 10 * (cfg / 100), (WN, WK, WS), 64x64 per wave:
  // 1 (1,1,4)  2 (2,1,2)  3 (1,2,2)  4 (2,2,1)  5 (4,1,1)  6 (1,4,1)  7 (2,2,2)  8 (1,1,2)
  // 9 (4,2,1) 256x128  11 (2,4,1) 128x256  12 (4,4,1) 256x256 (16 waves): the large output
  // tiles halve the LDS-DMA / L2 traffic per MFMA of the compute-bound (long-K) grad-weights
  // 128x64 per wave (MSN 2, one wave per SIMD to fit 340-460 VGPRs) measured 1.3-3x slower than
  // the 64x64 tiles on every BERT / ResNet-50 grad-weight shape (profiles/r02_tn_probe.json), so
  // no tile instantiates it; the template parameter stays for future occupancy experiments.
  const int ns = (cfg / 10) % 10 == 2 ? 3 : 2;
  cfg = cfg % 10 + 10 * ((cfg / 100) % 10);
  auto g = static_cast<const uint16_t*>(G);
  auto x = static_cast<const uint16_t*>(X);
  if (cfg <= 0) {
    const bool n2 = N % 128 == 0, k2 = K % 128 == 0;
    cfg = n2 && k2 ? 7 : (n2 ? 2 : (k2 ? 3 : 1));
  }
  static const int cfg_bn[13] = {64, 64, 128, 64, 128, 256, 64, 128, 64, 256, 64, 128, 256};
  static const int cfg_bk[13] = {64, 64, 64, 128, 128, 64, 256, 128, 64, 128, 64, 256, 256};
  if (cfg > 12 || cfg == 10 || N % cfg_bn[cfg] != 0 || K % cfg_bk[cfg] != 0) cfg = 1;   // tiles must divide N and K
  switch (cfg) {
    case 9: launch_tn_any<4, 2, 1, GATHER>(g, ldg, x, ldx, W, ldw, M, N, K, splits, ns, geo, stream); break;
    case 11: launch_tn_any<2, 4, 1, GATHER>(g, ldg, x, ldx, W, ldw, M, N, K, splits, ns, geo, stream); break;
    case 12: launch_tn_any<4, 4, 1, GATHER>(g, ldg, x, ldx, W, ldw, M, N, K, splits, ns, geo, stream); break;
    case 2: launch_tn_any<2, 1, 2, GATHER>(g, ldg, x, ldx, W, ldw, M, N, K, splits, ns, geo, stream); break;
    case 3: launch_tn_any<1, 2, 2, GATHER>(g, ldg, x, ldx, W, ldw, M, N, K, splits, ns, geo, stream); break;
    case 4: launch_tn_any<2, 2, 1, GATHER>(g, ldg, x, ldx, W, ldw, M, N, K, splits, ns, geo, stream); break;
    case 5: launch_tn_any<4, 1, 1, GATHER>(g, ldg, x, ldx, W, ldw, M, N, K, splits, ns, geo, stream); break;
    case 6: launch_tn_any<1, 4, 1, GATHER>(g, ldg, x, ldx, W, ldw, M, N, K, splits, ns, geo, stream); break;
    case 7: launch_tn_any<2, 2, 2, GATHER>(g, ldg, x, ldx, W, ldw, M, N, K, splits, ns, geo, stream); break;
    case 8: launch_tn_any<1, 1, 2, GATHER>(g, ldg, x, ldx, W, ldw, M, N, K, splits, ns, geo, stream); break;
    default: launch_tn_any<1, 1, 4, GATHER>(g, ldg, x, ldx, W, ldw, M, N, K, splits, ns, geo, stream); break;
  }
}


}  // namespace
}  // namespace gk
