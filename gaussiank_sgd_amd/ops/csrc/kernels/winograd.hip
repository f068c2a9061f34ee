// Winograd F(2x2, 3x3) convolution in fp32 on v_mfma_f32_16x16x4_f32 (gfx950).
//
// Why: at the reference's precision (fp32, settings.py:28) the 3x3 stride-1
// convolutions of a ResNet are bound by the fp32 MFMA rate (64 FLOP/clk/SIMD,
// 1/16 of bf16), not by memory.  F(2x2, 3x3) computes each 2x2 output tile
// from a 4x4 input patch with 16 element-wise products per (tile, Cin, Cout)
// instead of 36: 2.25x fewer MFMA FLOPs.  The transforms are exact-weight
// additions (+-1 for the data, 1/2 for the filter), so the result is a
// rearranged fp32 sum of the same products with a few extra roundings --
// same precision class as the direct convolution (tests vs fp64).
//
//   V[xi][t][c]  = (B^T d_t,c B)[xi]            input transform (in-kernel)
//   U[xi][c][k]  = (G g_k,c G^T)[xi]            filter transform (wino_wt)
//   M[xi][t][k]  = sum_c V[xi][t][c] U[xi][c][k]   16 GEMMs on MFMA
//   Y_t,k        = A^T M[.][t][k] A             output transform (epilogue)
//
// Grad-input of the same convolution is the forward convolution of dY with the
// flipped, transposed filter: the same kernel with U built from W'[c][kh][kw][k]
// = W[k][2-kh][2-kw][c] (wino_wt flip = 1).
//
// (GK_WINO_PROBE_* macros: timing-only A/B builds of bench/wino_probe.hip that
// drop the loads / LDS stores / epilogue stores / barriers; never defined in
// the extension build.)
//
// Kernel layout.  512 threads = 8 waves (two per SIMD); a block owns 64 tiles
// x 64 output channels for ALL 16 xi, each wave 32 tiles x 16 channels x 16 xi
// (128 fp32 accumulators per lane).  Keeping every xi of a (tile, channel) in
// one lane makes the output transform a register-only epilogue.
// Input channels stream in stages of 8: per stage every thread loads one
// tile's 4x4 patch for one channel (16 loads, zero padding in registers),
// transforms it and writes 16 V values; U arrives pre-chunked
// ([Cin/8][16][Cout][8]) so a block's stage slice is 16 contiguous 2-KiB rows.
// Two LDS stages (64 KiB each): the next stage's global loads are issued
// before this stage's 128 MFMAs per wave and land in LDS after them (one
// barrier per stage), pipelined across tile-block boundaries of the
// persistent loop.  Operand reads are ds_read_b64: lane (i, q) reads channels
// 2q, 2q+1 of row i and MFMA j contracts channels {2q + j} -- the same
// permutation on both operands.  The MFMA is issued with U as the A operand
// so a lane ends with 4 consecutive output channels of one tile: 16-byte
// stores.  (One wave per SIMD with 32x32 wave tiles -- 256 accumulators per
// lane -- spills even with all 512 VGPR + AGPR registers.)
//
// Grid: (tile blocks, Cout / 64) persistent along tiles with the x extent a
// multiple of 8, so all Cout blocks of a tile block run on one XCD (blocks
// are dealt round-robin to the 8 XCDs) and share the input patches in its L2.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "common.h"
#include "gk_kernels.h"
#include "mfma_util.h"

namespace gk {
namespace {

constexpr int WBT = 64;                 // tiles per block
constexpr int WBK = 64;                 // output channels per block
constexpr int WCK = 8;                  // input channels per stage
constexpr int WVS = 16 * WBT * WCK;     // floats of one V stage
constexpr int WUS = 16 * WBK * WCK;     // floats of one U stage
constexpr int WSTAGE = WVS + WUS;       // 16384 floats = 64 KiB
constexpr int WLDS = 2 * WSTAGE * 4;    // bytes
// xi slot at which the forward kernel waits for the next stage's patches and
// transforms them; its 16 LDS writes then go out 16 / (16 - slot) per slot.
// Measured on the bs512 shapes (r4c18-r4c21, bench/wino_probe.hip): one burst
// at slot 8 (the round-3 form) 563-665 us, spread from slot 8 1-2% faster,
// from slot 12 2-3% faster; staggering the two waves of a SIMD over different
// slots (a wave-uniform branch per slot) was slower than either, and so was
// deferring xi = 15's MFMAs across the stage barrier (+1-2%, r4c22).
#ifndef GK_WINO_XFORM
#define GK_WINO_XFORM 12
#endif
constexpr int kWinoXform = GK_WINO_XFORM;
static_assert(kWinoXform == 8 || kWinoXform == 12 || kWinoXform == 14 || kWinoXform == 15, "16 - slot divides 16");

struct WinoGeo {
  int H, W, Ci, Co, TH, TW, ntiles;
  uint32_t xbytes;   // bytes of the input tensor (< 2^31: buffer-descriptor range check)
  uint32_t ybytes;   // bytes of the output tensor (< 2^31; BN-backward operands have its shape)
  int64_t yplane;    // split over the input channels (grid z > 1): floats between output planes
};

struct WBnb {                // BN-backward epilogue operands (gemm.hip BnBwd, fp32)
  const float* h;            // BN input [M, Co]; nullptr: plain epilogue
  const float* dy2;          // optional second gradient [M, Co]
  const uint8_t* mask;       // optional ReLU mask, one byte per 4 channels (bit r: channel 4j + r)
};

// LDS bank swizzle of the forward kernel's operand rows (8 floats = four
// 8-byte slots per row): slot q of row r lives at q ^ wsw(r).  An MFMA operand
// read has 16 lanes on rows r..r+15 at one slot; without the swizzle rows 4
// apart share banks (4-way conflicts, measured 0.59 conflict cycles per LDS
// cycle); with it the 16 rows cover all 32 banks.  U is stored pre-swizzled
// by the filter transform, so its LDS-DMA copy lands swizzled.
__host__ __device__ __forceinline__ int wsw(int r) { return (r >> 2) & 3; }

// filter transform: one thread per (co, ci) of the convolution being run;
// u = [Ci/8][16][Co][8] (slots swizzled by wsw(co))
__global__ void __launch_bounds__(256) wino_wt_kernel(const float* __restrict__ w, float* __restrict__ u, int Co, int Ci,
                                                      int flip) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (int64_t)Co * Ci) return;
  const int co = (int)(idx / Ci), ci = (int)(idx - (int64_t)co * Ci);
  float g[3][3];
#pragma unroll
  for (int kh = 0; kh < 3; ++kh)
#pragma unroll
    for (int kw = 0; kw < 3; ++kw)
      g[kh][kw] = flip ? w[((int64_t)ci * 9 + (2 - kh) * 3 + (2 - kw)) * Co + co]    // W[k = ci][.][.][c = co]
                       : w[((int64_t)co * 9 + kh * 3 + kw) * Ci + ci];               // W[co][kh][kw][ci]
  float t[4][3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    t[0][j] = g[0][j];
    t[1][j] = 0.5f * (g[0][j] + g[1][j] + g[2][j]);
    t[2][j] = 0.5f * (g[0][j] - g[1][j] + g[2][j]);
    t[3][j] = g[2][j];
  }
  // 8-byte slot (ci & 7) >> 1 of row co stored at slot ^ wsw(co) (see wsw)
  float* dst = u + ((int64_t)(ci >> 3) * 16 * Co + co) * 8 + ((((ci & 7) >> 1) ^ wsw(co)) << 1) + (ci & 1);
  const int64_t xs = (int64_t)Co * 8;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    dst[(4 * i + 0) * xs] = t[i][0];
    dst[(4 * i + 1) * xs] = 0.5f * (t[i][0] + t[i][1] + t[i][2]);
    dst[(4 * i + 2) * xs] = 0.5f * (t[i][0] - t[i][1] + t[i][2]);
    dst[(4 * i + 3) * xs] = t[i][2];
  }
}

template <bool STATS, bool BNB>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2)))
wino_f23_kernel(const float* __restrict__ x, const float* __restrict__ u, float* __restrict__ y, WinoGeo g,
                float* __restrict__ stats, int64_t stats_ld, WBnb bb) {
  extern __shared__ __attribute__((aligned(16))) float wlds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wt = wave >> 2, wk = wave & 3;
  const int fi = lane & 15, fq = lane >> 4;
  const int k0 = blockIdx.y * WBK;
  const int ntb = (g.ntiles + WBT - 1) / WBT;
  // split over the input channels (small batches: too few tile blocks to fill
  // the chip): plane z accumulates stages [sb, sb + nst) into its own output
  // plane (plain epilogue); splitk_reduce sums the planes with the epilogue
  const int nst = g.Ci / WCK / (int)gridDim.z;
  const int sb = (int)blockIdx.z * nst;
  if (!STATS && !BNB && gridDim.z > 1) y += (int64_t)blockIdx.z * g.yplane;
  const int my_tb = (int)blockIdx.x < ntb ? (ntb - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  const int total = my_tb * nst;
  const int THW = g.TH * g.TW;
  // loader role: tile ltile of the block's 64, channel lc of the stage's 8
  const int ltile = tid >> 3, lc = tid & 7;

  f32x4 acc[16][2];     // [xi][tile subtile]
#pragma unroll
  for (int xi = 0; xi < 16; ++xi)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[xi][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  float ssum[4], ssq[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) ssum[r] = ssq[r] = 0.f;

  // x through a buffer descriptor: a patch pixel outside the image gets the
  // byte offset 0x80000000 (past num_records), which the hardware range check
  // turns into a zero load -- no branches, no per-load address arithmetic
  // (the stage's channel offset is the scalar soffset).
  uint32_t voff[16];
  auto set_tile = [&](int tb) __attribute__((always_inline)) {
    const int tt = tb * WBT + ltile;
    const bool tv = tt < g.ntiles;
    const int ttc = tv ? tt : 0;
    const int n = ttc / THW, r = ttc - n * THW, th = r / g.TW, tw = r - th * g.TW;
    const int ih0 = 2 * th - 1, iw0 = 2 * tw - 1;
    // modulo-2^32 byte offset of pixel (ih0, iw0) (may wrap for ih0 = -1; valid taps land in range)
    const uint32_t base = (uint32_t)((((int64_t)n * g.H + ih0) * g.W + iw0) * g.Ci + lc) * 4u;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool v = tv && (unsigned)(ih0 + i) < (unsigned)g.H && (unsigned)(iw0 + j) < (unsigned)g.W;
        voff[4 * i + j] = v ? base + (uint32_t)((i * g.W + j) * g.Ci) * 4u : 0x80000000u;
      }
  };

  float dv[1][16];
  // Issued as inline asm: the compiler's wait-count pass, unable to order the
  // ring's loads against the LDS-DMA and epilogue stores across the loop
  // back-edge, would wait vmcnt(0) before the transform (draining the
  // stage-(s + 2) prefetch it just issued).  The transform waits itself
  // (vwait, tied to the registers).
  // the descriptor as four readfirstlane'd words: provably uniform, so the
  // "s" asm operand gets SGPRs
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const uint64_t xa = (uint64_t)(uintptr_t)x;
  const u32x4 xrs = u32x4{(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)xa),
                          (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(xa >> 32)),
                          (uint32_t)__builtin_amdgcn_readfirstlane((int)g.xbytes), 0x00020000u};
  auto gload_v = [&](int s, int r) __attribute__((always_inline)) {
    const int so = __builtin_amdgcn_readfirstlane((sb + s) * WCK * 4);
#pragma unroll
    for (int p = 0; p < 16; ++p) {
#ifdef GK_WINO_PROBE_NOLOAD
      dv[r][p] = (float)(voff[p] & 7);
#else
      asm volatile("buffer_load_dword %0, %1, %2, %3 offen" : "=v"(dv[r][p]) : "v"(voff[p]), "s"(xrs), "s"(so));
#endif
    }
  };
  // at most N vector-memory ops outstanding; the ring's registers tied to the wait
  auto vwait = [&](auto NC, int r) __attribute__((always_inline)) {
    constexpr int N = decltype(NC)::value;
    float* d = dv[r];
    asm volatile("s_waitcnt vmcnt(%16)"
                 : "+v"(d[0]), "+v"(d[1]), "+v"(d[2]), "+v"(d[3]), "+v"(d[4]), "+v"(d[5]), "+v"(d[6]), "+v"(d[7]),
                   "+v"(d[8]), "+v"(d[9]), "+v"(d[10]), "+v"(d[11]), "+v"(d[12]), "+v"(d[13]), "+v"(d[14]), "+v"(d[15])
                 : "n"(N)
                 : "memory");
  };
  // U's 32 KiB slice of stage s into LDS buffer b by LDS-DMA, 4 x 1 KiB per wave
  auto gload_u = [&](int s, int b) __attribute__((always_inline)) {
#ifndef GK_WINO_PROBE_NOLOAD
    GK_LDS char* ub = (GK_LDS char*)wlds + (b * WSTAGE + WVS) * 4;
    const float* us = u + ((int64_t)(sb + s) * 16 * g.Co + k0) * 8;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = wave * 4 + i, xi = q >> 1, half = q & 1;
      glds16(us + (int64_t)xi * g.Co * 8 + half * 256 + lane * 4, ub + q * 1024);
    }
#endif
  };
  // input transform B^T d B of the landed patch into vt[xi] (registers); its 16
  // LDS writes are issued two per xi slot of the next compute() (lwrite), so
  // they interleave with the operand reads instead of queueing ahead of them
  // in one burst (measured: the burst form stalls the MFMAs behind the LDS
  // queue, r4c18 ablation)
  float vt[16];
  auto ltrans = [&](int r) __attribute__((always_inline)) {
    const float* d = dv[r];
    float t[16];
#pragma unroll
    for (int j = 0; j < 4; ++j) {   // B^T d
      t[0 + j] = d[0 + j] - d[8 + j];
      t[4 + j] = d[4 + j] + d[8 + j];
      t[8 + j] = d[8 + j] - d[4 + j];
      t[12 + j] = d[4 + j] - d[12 + j];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {   // (.) B
      vt[4 * i + 0] = t[4 * i + 0] - t[4 * i + 2];
      vt[4 * i + 1] = t[4 * i + 1] + t[4 * i + 2];
      vt[4 * i + 2] = t[4 * i + 2] - t[4 * i + 1];
      vt[4 * i + 3] = t[4 * i + 1] - t[4 * i + 3];
    }
  };
  const int lcol = ((((lc >> 1) ^ wsw(ltile)) << 1) | (lc & 1));
  // LDS writes of vt[q0 .. q0 + NQ) into buffer b
  auto lwrite = [&](int b, int q0, int nq) __attribute__((always_inline)) {
    float* V = wlds + b * WSTAGE;
#pragma unroll
    for (int q = q0; q < q0 + nq; ++q) V[(q * WBT + ltile) * WCK + lcol] = vt[q];
  };
  auto lstore = [&](int b, int r) __attribute__((always_inline)) {
    ltrans(r);
    lwrite(b, 0, 16);
  };
  // All 16 xi of LDS buffer b, the operands of xi + 1 read (into the other
  // register set) before the MFMAs of xi are issued, so the LDS latency hides
  // behind them; mid(xi) runs before the MFMAs of each xi (from xi = 8: the next stage's
  // transform: its VALU and LDS writes issue while MFMAs are in flight).
  // Offsets are lane constants plus compile-time xi strides: the reads are
  // one base register and immediate offsets.
  const int rcol = (fq ^ wsw(fi)) << 1;   // swizzled slot of this lane's operand rows (rows = 16-multiple + fi)
  const int aoff = (wk * 16 + fi) * WCK + rcol;
  const int boff = (wt * 32 + fi) * WCK + rcol;
  f32x2 fa[2], fb[2][2];   // operand register double buffer
  auto mfma_xi = [&](int xi, int sl) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int ts = 0; ts < 2; ++ts)
        acc[xi][ts] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[sl][j], fb[sl][ts][j], acc[xi][ts], 0, 0, 0);
  };
  auto compute = [&](int b, auto mid) __attribute__((always_inline)) {
    const float* V = wlds + b * WSTAGE;
    const float* U = V + WVS;
    auto rd = [&](int xi, int sl) __attribute__((always_inline)) {
      fa[sl] = *reinterpret_cast<const f32x2*>(U + xi * (WBK * WCK) + aoff);
      fb[sl][0] = *reinterpret_cast<const f32x2*>(V + xi * (WBT * WCK) + boff);
      fb[sl][1] = *reinterpret_cast<const f32x2*>(V + xi * (WBT * WCK) + boff + 16 * WCK);
    };
    rd(0, 0);
#pragma unroll
    for (int xi = 0; xi < 16; ++xi) {
      const int sl = xi & 1;
      if (xi + 1 < 16) rd(xi + 1, sl ^ 1);
      mid(xi);
      __builtin_amdgcn_sched_barrier(0);   // keep the reads of xi + 1 ahead of the MFMAs of xi
      mfma_xi(xi, sl);
    }
  };
  // BN-backward epilogue operands through buffer descriptors (an invalid
  // pixel's offset is past the range and loads zero): all loads of a 16-tile
  // subtile's four pixels are issued before any is used, one exposed latency
  // per subtile instead of one per pixel
  const auto hr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(bb.h), (short)0, (int)g.ybytes, 0x00020000);
  const auto dr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(bb.dy2), (short)0, bb.dy2 ? (int)g.ybytes : 0,
                                                    0x00020000);
  const auto mr = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(bb.mask), (short)0,
                                                    bb.mask ? (int)(g.ybytes / 16) : 0, 0x00020000);
  auto epilogue = [&](int tb) __attribute__((always_inline)) {
#pragma unroll
    for (int ts = 0; ts < 2; ++ts) {
      const int tt = tb * WBT + wt * 32 + ts * 16 + fi;
      const bool tv = tt < g.ntiles;
      const int ttc = tv ? tt : 0;
      const int n = ttc / THW, rr = ttc - n * THW, th = rr / g.TW, tw = rr - th * g.TW;
      const int kk = k0 + wk * 16 + 4 * fq;
      bool pv[4];
      int64_t row[4];
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const int oh = 2 * th + (p >> 1), ow = 2 * tw + (p & 1);
        pv[p] = tv && oh < g.H && ow < g.W;
        row[p] = ((int64_t)n * g.H + oh) * g.W + ow;
      }
      f32x4 hv[4], d2[4];
      uint32_t bits[4];
      // BN operands of pixels [p0, p0 + 2): two pixels per batch keeps the
      // epilogue inside the register budget of the pipelined main loop
      auto bnload = [&](int p0) __attribute__((always_inline)) {
#pragma unroll
        for (int p = p0; p < p0 + 2; ++p) {
          const uint32_t off = pv[p] ? (uint32_t)(row[p] * g.Co + kk) * 4u : 0x80000000u;
          hv[p] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(hr, (int)off, 0, 0));
          d2[p] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(dr, (int)off, 0, 0));
          const uint32_t moff = pv[p] ? (uint32_t)(row[p] * (g.Co >> 2) + (kk >> 2)) : 0x80000000u;
          bits[p] = bb.mask ? (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(mr, (int)moff, 0, 0) : 0xfu;
        }
      };
      if constexpr (BNB) bnload(0);
      f32x4 o[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {   // A^T M A
        float s0[4], s1[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          s0[j] = acc[j][ts][r] + acc[4 + j][ts][r] + acc[8 + j][ts][r];
          s1[j] = acc[4 + j][ts][r] - acc[8 + j][ts][r] - acc[12 + j][ts][r];
        }
        o[0][r] = s0[0] + s0[1] + s0[2];
        o[1][r] = s0[1] - s0[2] - s0[3];
        o[2][r] = s1[0] + s1[1] + s1[2];
        o[3][r] = s1[1] - s1[2] - s1[3];
      }
#pragma unroll
      for (int xi = 0; xi < 16; ++xi) acc[xi][ts] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        if constexpr (BNB) {
          if (p == 2) bnload(2);
        }
        f32x4 v = o[p];
        if constexpr (BNB) {
          // invalid pixels: bits = 0 -> dz = 0, no contribution
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float dz = (bits[p] >> r) & 1u ? v[r] + d2[p][r] : 0.f;
            v[r] = dz;
            ssum[r] += dz;
            ssq[r] = fmaf(dz, hv[p][r], ssq[r]);
          }
        } else if constexpr (STATS) {
          const float m = pv[p] ? 1.f : 0.f;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            ssum[r] = fmaf(m, v[r], ssum[r]);
            ssq[r] = fmaf(m * v[r], v[r], ssq[r]);
          }
        }
#ifdef GK_WINO_PROBE_NOEPI
        if (g.H < 0)
#endif
        if (pv[p]) *reinterpret_cast<f32x4*>(y + row[p] * g.Co + kk) = v;
      }
    }
  };

  if (total > 0) {
    int tb = blockIdx.x, s = 0;   // compute cursor (tile block, stage)
    int lb = blockIdx.x, ls = 0;  // load cursor, one stage ahead
    auto adv = [&](int& t, int& st) __attribute__((always_inline)) {
      if (++st == nst) {
        st = 0;
        t += gridDim.x;
      }
    };
    set_tile(lb);
    gload_u(0, 0);
    gload_v(0, 0);
    vwait(std::integral_constant<int, 0>{}, 0);   // everything, U's LDS-DMA included
    lstore(0, 0);
    __syncthreads();
    // One stage of patches in flight: stage it + 1's loads are issued at the
    // top of iteration it (after its U LDS-DMA) and transformed in the middle
    // of the iteration's MFMAs.  (Two stages in flight measured the same and
    // cost 16 registers the BN epilogues spill without.)
    int it = 0;
    auto step = [&](auto CUR) __attribute__((always_inline)) {
      constexpr int cur = decltype(CUR)::value, nxt = cur ^ 1;
      const bool more = it + 1 < total;
      if (more) {
        adv(lb, ls);
        if (ls == 0) set_tile(lb);
        gload_u(ls, nxt);
        gload_v(ls, 0);
      }
      compute(cur, [&](int xi) __attribute__((always_inline)) {
        constexpr int X0 = kWinoXform, PER = 16 / (16 - X0);
        if (more && xi >= X0) {
          if (xi == X0) {
            vwait(std::integral_constant<int, 0>{}, 0);   // the patch loads are the youngest ops
            ltrans(0);
          }
#ifndef GK_WINO_PROBE_NOLSTORE
          // BN-backward epilogue variant: one burst (the spread form's live
          // transform registers push its epilogue into spills)
          if constexpr (BNB) {
            if (xi == X0) lwrite(nxt, 0, 16);
          } else {
            lwrite(nxt, PER * (xi - X0), PER);
          }
#endif
        }
      });
      if (s == nst - 1) epilogue(tb);
      // Barrier without __syncthreads()' release fence (the epilogue's global
      // stores need no ordering here): U's LDS-DMA and this wave's LDS writes
      // are done.  One asm statement with a memory clobber so no LDS access
      // moves across it.
#ifndef GK_WINO_PROBE_NOBAR
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
#else
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
#endif
      adv(tb, s);
      ++it;
    };
    while (it < total) {
      step(std::integral_constant<int, 0>{});
      if (it < total) step(std::integral_constant<int, 1>{});
    }
  }

  if constexpr (STATS || BNB) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) {
        ssum[r] += __shfl_xor(ssum[r], off, 64);
        ssq[r] += __shfl_xor(ssq[r], off, 64);
      }
    __syncthreads();
    float* red = wlds;   // [sum | sq][wt][64]
    if (fi == 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int col = wk * 16 + 4 * fq + r;
        red[wt * WBK + col] = ssum[r];
        red[(2 + wt) * WBK + col] = ssq[r];
      }
    }
    __syncthreads();
    if (tid < WBK) {
      stats[(int64_t)blockIdx.x * g.Co + k0 + tid] = red[tid] + red[WBK + tid];
      stats[stats_ld + (int64_t)blockIdx.x * g.Co + k0 + tid] = red[2 * WBK + tid] + red[3 * WBK + tid];
    }
  }
}

template <bool STATS, bool BNB>
int launch_wino(const float* x, const float* u, float* y, const WinoGeo& g, int max_blocks, float* stats,
                int stats_rows, const WBnb& bb, hipStream_t stream, int splits = 1) {
  const int ntb = (g.ntiles + WBT - 1) / WBT;
  const int nkb = g.Co / WBK;
  // persistent along tiles, about one block per CU (128 KiB of LDS), x extent a multiple of 8
  // (with z planes too: block id x + gx (y + ny z) keeps a tile block's planes on one XCD)
  int gx = max_blocks > 0 ? max_blocks : ((256 + nkb * splits - 1) / (nkb * splits) + 7) / 8 * 8;
  if (gx > ntb) gx = ntb;
  if ((STATS || BNB) && gx > stats_rows) gx = stats_rows;   // one partial row per block
  if (gx < 1) gx = 1;
  static bool attr = [] {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&wino_f23_kernel<STATS, BNB>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, WLDS) == hipSuccess;
  }();
  (void)attr;
  hipLaunchKernelGGL((wino_f23_kernel<STATS, BNB>), dim3((unsigned)gx, (unsigned)nkb, (unsigned)splits), dim3(512), WLDS,
                     stream, x, u, y, g, stats, (int64_t)stats_rows * g.Co, bb);
  return gx;
}

// --------------------------------------------------------------------------
// Grad-weight.  Differentiating the forward tile formula w.r.t. the filter:
//   dU[xi][c][k] = sum_t V[xi][t][c] dM[xi][t][k],  dM_t = A dY_t A^T (4x4)
//   dW[k][c]     = G^T dU[.][c][k] G                (3x3)
// -- 16 GEMMs reduced over the tiles (2.25x fewer MFMA FLOPs than the 9-tap
// direct grad-weight).  Block = 64 input x 64 output channels x all 16 xi for
// one contiguous range of tiles (a split); 8 waves, each 32 c x 16 k x 16 xi
// (128 accumulators per lane; lane ends with 4 consecutive c of one k).
// Stages of 8 tiles: thread (tile, channel) loads the tile's 4x4 input patch
// of channel c (16 loads, 64 lanes = 256 contiguous bytes per pixel) and its
// 2x2 dY block of channel k, transforms the patch and writes V rows
// [xi][channel][tile] (row stride 10 floats: 2-way write conflicts, aligned
// 8-byte operand reads) and the dY block raw ([tile][k][2x2], one 16-byte
// write); the MFMA's dM operand is formed in registers from it (two raw
// blocks per lane per stage: one add per xi), which halved the LDS writes
// (grad-weight 7-8% faster than the transformed-dM layout, r4c24).  Two
// stages of 48 KiB.  Each
// block writes its dU partial (plain stores, no atomics: deterministic); the
// finalize kernel sums the splits, applies G^T . G and adds into the fp32
// gradient (channels-last [K][3][3][C]).  Blocks are remapped so the Cout /
// Cin blocks of one split sit on one XCD and share its patches in L2.
constexpr int WGT = 8;                      // tiles per stage
constexpr int WGRS = 10;                    // LDS row stride (floats)
constexpr int WGHALF = 16 * 64 * WGRS;      // floats of one V stage
constexpr int WGD = WGT * 64 * 4;           // floats of one raw dY stage: [tile][k][2x2]
constexpr int WGSTAGE = WGHALF + WGD;       // V + raw dY
constexpr int WGLDS = 2 * WGSTAGE * 4;      // 98304 bytes

__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2)))
wino_wgrad_kernel(const float* __restrict__ x, const float* __restrict__ dy, float* __restrict__ part, WinoGeo g,
                  int splits, int tps) {
  // g.Ci = C (input channels), g.Co = K (output channels)
  extern __shared__ __attribute__((aligned(16))) float wlds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wave >> 2, wk = wave & 3;
  const int fi = lane & 15, fq = lane >> 4;
  const int ncb = g.Ci / 64, nkb = g.Co / 64;
  const int nb = ncb * nkb * splits;
  // XCD-aware remap (nb % 8 == 0): hardware block b runs on XCD b % 8
  const int bid = blockIdx.x;
  const int logical = (bid & 7) * (nb >> 3) + (bid >> 3);
  const int split = logical / (ncb * nkb), rem = logical - split * ncb * nkb;
  const int c0 = (rem / nkb) * 64, k0 = (rem % nkb) * 64;
  const int t_begin = split * tps;
  int t_end = t_begin + tps;
  if (t_end > g.ntiles) t_end = g.ntiles;
  const int nst = t_end > t_begin ? (t_end - t_begin + WGT - 1) / WGT : 0;
  const int THW = g.TH * g.TW;
  const int lt = tid >> 6, lch = tid & 63;   // loader: tile lt of the stage, channel lch

  f32x4 acc[16][2];   // [xi][c subtile]
#pragma unroll
  for (int xi = 0; xi < 16; ++xi)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[xi][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  // x and dy through buffer descriptors (out-of-image taps: offset past the
  // range, loaded as zero); the loader's tile advances by 8 per stage, its
  // (n, th, tw) is stepped incrementally (no per-stage division)
  const auto xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x), (short)0, (int)g.xbytes, 0x00020000);
  const auto gr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(dy), (short)0,
                                                    (int)(g.xbytes / g.Ci * g.Co), 0x00020000);
  int ct = t_begin + lt, cn = 0, cth = 0, ctw = 0;
  {
    const int t0 = ct < g.ntiles ? ct : 0;
    cn = t0 / THW;
    const int r = t0 - cn * THW;
    cth = r / g.TW;
    ctw = r - cth * g.TW;
  }
  float dv[16], gv[4];
  auto gload = [&](int st) __attribute__((always_inline)) {
    const bool tv = ct < t_end;
    const int ih0 = 2 * cth - 1, iw0 = 2 * ctw - 1;
    const uint32_t xb = (uint32_t)((((int64_t)cn * g.H + ih0) * g.W + iw0) * g.Ci + c0 + lch) * 4u;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool v = tv && (unsigned)(ih0 + i) < (unsigned)g.H && (unsigned)(iw0 + j) < (unsigned)g.W;
        const uint32_t o = v ? xb + (uint32_t)((i * g.W + j) * g.Ci) * 4u : 0x80000000u;
#ifdef GK_WINO_PROBE_NOLOAD
        dv[4 * i + j] = (float)(o & 7);
#else
        dv[4 * i + j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, (int)o, 0, 0));
#endif
      }
    const uint32_t gb = (uint32_t)((((int64_t)cn * g.H + 2 * cth) * g.W + 2 * ctw) * g.Co + k0 + lch) * 4u;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const bool v = tv && 2 * cth + a < g.H && 2 * ctw + b < g.W;
        const uint32_t o = v ? gb + (uint32_t)((a * g.W + b) * g.Co) * 4u : 0x80000000u;
#ifdef GK_WINO_PROBE_NOLOAD
        gv[2 * a + b] = (float)(o & 7);
#else
        gv[2 * a + b] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(gr, (int)o, 0, 0));
#endif
      }
    // next stage's tile: +WGT
    ct += WGT;
    ctw += WGT;
    while (ctw >= g.TW) {
      ctw -= g.TW;
      if (++cth == g.TH) {
        cth = 0;
        ++cn;
      }
    }
    (void)st;
  };
  // input transform of the landed patch into registers (tv); its 16 LDS
  // writes and the raw dY block's one go out together at xi = 8 of the next
  // compute() (spreading them over the xi slots measured slower, r4c19)
  float tv[16];
  auto ltrans_v = [&]() __attribute__((always_inline)) {
    float t[16];
#pragma unroll
    for (int j = 0; j < 4; ++j) {   // B^T d
      t[0 + j] = dv[0 + j] - dv[8 + j];
      t[4 + j] = dv[4 + j] + dv[8 + j];
      t[8 + j] = dv[8 + j] - dv[4 + j];
      t[12 + j] = dv[4 + j] - dv[12 + j];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {   // (.) B
      tv[4 * i + 0] = t[4 * i + 0] - t[4 * i + 2];
      tv[4 * i + 1] = t[4 * i + 1] + t[4 * i + 2];
      tv[4 * i + 2] = t[4 * i + 2] - t[4 * i + 1];
      tv[4 * i + 3] = t[4 * i + 1] - t[4 * i + 3];
    }
  };
  // LDS writes of V rows [q0, q0 + nq) into buffer buf (2-way bank conflicts:
  // rows 32 apart share banks at the 10-word stride; storing the rows with bit
  // 5 set tile-swapped -- conflict-free, the wc = 1 waves swapping their dM
  // pair to match -- measured 7% slower, r4c33)
  auto lwrite_v = [&](int buf, int q0, int nq) __attribute__((always_inline)) {
    float* V = wlds + buf * WGSTAGE;
#pragma unroll
    for (int q = q0; q < q0 + nq; ++q) V[(q * 64 + lch) * WGRS + lt] = tv[q];
  };
  // the raw 2x2 dY block of (tile lt, channel k = lch): one 16-byte write
  // ([tile][k][4]: consecutive lanes, consecutive 16 bytes); dM = A dY A^T is
  // formed in the consumer's registers (compute), which replaces the 16
  // transformed dM rows per thread of the round-3 layout -- half of this
  // kernel's LDS writes, and the 16 dM operand reads per stage
  auto lwrite_d = [&](int buf) __attribute__((always_inline)) {
    float* D = wlds + buf * WGSTAGE + WGHALF;
    *reinterpret_cast<f32x4*>(D + (lt * 64 + lch) * 4) = f32x4{gv[0], gv[1], gv[2], gv[3]};
  };
  // all 16 xi of buffer buf, the operands of xi + 1 read before the MFMAs of
  // xi (forward kernel's scheme); mid(xi) before the MFMAs of each xi
  auto compute = [&](int buf, auto mid) __attribute__((always_inline)) {
    const float* V = wlds + buf * WGSTAGE;
    const float* D = V + WGHALF;
    // this lane's B operand rows: dM[xi][k = wk*16 + fi][tiles 2fq, 2fq + 1]
    // from the two raw dY blocks.  Row transform once per stage (m = A dY:
    // rows p, p + q, p - q, -q of each column); dM[4i + c] is then one add /
    // negate of m[i][0], m[i][1] per xi (A's column combination).
    float m[2][4][2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const f32x4 r = *reinterpret_cast<const f32x4*>(D + ((2 * fq + j) * 64 + wk * 16 + fi) * 4);
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const float p = r[b], q = r[2 + b];
        m[j][0][b] = p;
        m[j][1][b] = p + q;
        m[j][2][b] = p - q;
        m[j][3][b] = -q;
      }
    }
    auto dm = [&](int j, int xi) __attribute__((always_inline)) {
      const float p = m[j][xi >> 2][0], q = m[j][xi >> 2][1];
      const int c = xi & 3;
      return c == 0 ? p : c == 1 ? p + q : c == 2 ? p - q : -q;
    };
    f32x2 fa[2][2], fb[2];
    auto rd = [&](int xi, int sl) __attribute__((always_inline)) {
#pragma unroll
      for (int cs = 0; cs < 2; ++cs)
        fa[sl][cs] = *reinterpret_cast<const f32x2*>(V + ((xi * 64) + wc * 32 + cs * 16 + fi) * WGRS + 2 * fq);
      fb[sl] = f32x2{dm(0, xi), dm(1, xi)};
    };
    rd(0, 0);
#pragma unroll
    for (int xi = 0; xi < 16; ++xi) {
      const int sl = xi & 1;
      if (xi + 1 < 16) rd(xi + 1, sl ^ 1);
      mid(xi);
      __builtin_amdgcn_sched_barrier(0);   // keep the reads of xi + 1 ahead of the MFMAs of xi
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int cs = 0; cs < 2; ++cs)
          acc[xi][cs] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[sl][cs][j], fb[sl][j], acc[xi][cs], 0, 0, 0);
    }
  };

  if (nst > 0) {
    gload(0);
    ltrans_v();
    lwrite_v(0, 0, 16);
    lwrite_d(0);
    __syncthreads();
    for (int st = 0; st < nst; ++st) {
      const bool more = st + 1 < nst;
      if (more) gload(st + 1);
      compute(st & 1, [&](int xi) __attribute__((always_inline)) {
        // one burst at xi = 8: the 16 V rows and the raw dY block (spreading
        // the V writes over the xi slots measured 3-4% slower, r4c19 / r4c24)
        if (more && xi == 8) {
          ltrans_v();
#ifndef GK_WINO_PROBE_NOLSTORE
          lwrite_v((st + 1) & 1, 0, 16);
          lwrite_d((st + 1) & 1);
#endif
        }
      });
#ifndef GK_WINO_PROBE_NOBAR
      __syncthreads();
#endif
    }
  }
  // dU partial of this split: part[split][xi][k][c], 4 consecutive c per lane
  const int k = k0 + wk * 16 + fi;
#pragma unroll
  for (int xi = 0; xi < 16; ++xi)
#pragma unroll
    for (int cs = 0; cs < 2; ++cs) {
      const int c = c0 + wc * 32 + cs * 16 + 4 * fq;
      *reinterpret_cast<f32x4*>(part + (((int64_t)split * 16 + xi) * g.Co + k) * g.Ci + c) = acc[xi][cs];
    }
}

// out[k][kh][kw][c] += G^T (sum_s part[s][.][k][c]) G.  A block handles
// kWfKC consecutive (k, c) pairs with kWfP threads each: thread (pair, q)
// sums splits q, q + kWfP, ... (a wave reads 32 consecutive pairs' rows: 128-
// byte segments), the kWfP partial sums meet in LDS in a fixed order
// (deterministic).  One thread per pair walking every split was latency-bound
// at the small-channel layers: 256 splits x 16 loads per thread, 42 us per
// call at bs512 (4,096 threads for the 64 x 64 layer).
constexpr int kWfKC = 32, kWfP = 8;
__global__ void __launch_bounds__(256) wino_wgrad_finalize_kernel(const float* __restrict__ part, float* __restrict__ out,
                                                                  int K, int C, int splits) {
  static_assert(kWfKC * kWfP == 256, "block shape");
  const int pr = threadIdx.x % kWfKC, q = threadIdx.x / kWfKC;
  const int64_t idx = (int64_t)blockIdx.x * kWfKC + pr;
  const bool valid = idx < (int64_t)K * C;
  const int64_t kc = valid ? idx : 0;
  const int k = (int)(kc / C), c = (int)(kc - (int64_t)k * C);
  float du[16];
#pragma unroll
  for (int xi = 0; xi < 16; ++xi) du[xi] = 0.f;
  if (valid) {
    for (int sp = q; sp < splits; sp += kWfP) {
      const float* p = part + ((int64_t)sp * 16 * K + k) * C + c;
#pragma unroll
      for (int xi = 0; xi < 16; ++xi) du[xi] += p[(int64_t)xi * K * C];
    }
  }
  __shared__ float red[kWfP][16][kWfKC];
#pragma unroll
  for (int xi = 0; xi < 16; ++xi) red[q][xi][pr] = du[xi];
  __syncthreads();
  if (q != 0 || !valid) return;
#pragma unroll
  for (int xi = 0; xi < 16; ++xi) {
    float a = red[0][xi][pr];
#pragma unroll
    for (int j = 1; j < kWfP; ++j) a += red[j][xi][pr];
    du[xi] = a;
  }
  float t[3][4];   // G^T dU
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float a = du[j], b = du[4 + j], c2 = du[8 + j], d = du[12 + j];
    t[0][j] = a + 0.5f * (b + c2);
    t[1][j] = 0.5f * (b - c2);
    t[2][j] = 0.5f * (b + c2) + d;
  }
  float* o = out + (int64_t)k * 9 * C + c;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    o[(3 * i + 0) * C] += t[i][0] + 0.5f * (t[i][1] + t[i][2]);
    o[(3 * i + 1) * C] += 0.5f * (t[i][1] - t[i][2]);
    o[(3 * i + 2) * C] += 0.5f * (t[i][1] + t[i][2]) + t[i][3];
  }
}

}  // namespace

void wino_weights(const float* w, float* u, int Co, int Ci, int flip, hipStream_t stream) {
  const int64_t n = (int64_t)Co * Ci;
  hipLaunchKernelGGL(wino_wt_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, w, u, Co, Ci, flip);
}

int wino_conv(const float* x, const float* u, float* y, int N, int H, int W, int Ci, int Co, int max_blocks,
              float* stats, int stats_rows, const BnBwdArgs* bn, hipStream_t stream, int splits, float* split_ws) {
  WinoGeo g{H, W, Ci, Co, (H + 1) / 2, (W + 1) / 2, 0, 0, 0, 0};
  g.ntiles = N * g.TH * g.TW;
  g.xbytes = (uint32_t)((int64_t)N * H * W * Ci * 4);
  g.ybytes = (uint32_t)((int64_t)N * H * W * Co * 4);
  if (splits > 1) {
    // input-channel split: plain partial planes into split_ws [splits][N H W][Co],
    // then one reduce pass with the statistics / BN-backward epilogue
    if (split_ws == nullptr || Ci % (WCK * splits) != 0) return -1;
    g.yplane = (int64_t)N * H * W * Co;
    launch_wino<false, false>(x, u, split_ws, g, max_blocks, nullptr, 0, WBnb{}, stream, splits);
    return splitk_reduce(split_ws, splits, (int64_t)N * H * W, Co, y, Co, nullptr, stats, stats_rows, bn, stream);
  }
  const WBnb bb = bn ? WBnb{static_cast<const float*>(bn->h), static_cast<const float*>(bn->dy2), bn->mask} : WBnb{};
  if (bn) return launch_wino<false, true>(x, u, y, g, max_blocks, stats, stats_rows, bb, stream);
  if (stats) return launch_wino<true, false>(x, u, y, g, max_blocks, stats, stats_rows, bb, stream);
  return launch_wino<false, false>(x, u, y, g, max_blocks, nullptr, 0, bb, stream);
}

int wino_wgrad_splits(int N, int H, int W, int C, int K, int splits) {
  const int ntiles = N * ((H + 1) / 2) * ((W + 1) / 2);
  const int cells = (C / 64) * (K / 64);
  if (splits <= 0) splits = (256 + cells - 1) / cells;     // about one block per CU
  splits = (splits + 7) / 8 * 8;                            // XCD remap: block count % 8 == 0
  const int maxs = (ntiles + WGT - 1) / WGT;
  if (splits > maxs) splits = (maxs + 7) / 8 * 8;
  return splits;
}

void wino_wgrad(const float* x, const float* dy, float* part, float* out, int N, int H, int W, int C, int K,
                int splits, hipStream_t stream) {
  WinoGeo g{H, W, C, K, (H + 1) / 2, (W + 1) / 2, 0, 0, 0, 0};
  g.ntiles = N * g.TH * g.TW;
  g.xbytes = (uint32_t)((int64_t)N * H * W * C * 4);
  splits = wino_wgrad_splits(N, H, W, C, K, splits);
  int tps = (g.ntiles + splits - 1) / splits;
  tps = (tps + WGT - 1) / WGT * WGT;
  const int nb = (C / 64) * (K / 64) * splits;
  static bool attr = [] {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&wino_wgrad_kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, WGLDS) == hipSuccess;
  }();
  (void)attr;
  hipLaunchKernelGGL(wino_wgrad_kernel, dim3((unsigned)nb), dim3(512), WGLDS, stream, x, dy, part, g, splits, tps);
  const int64_t n = (int64_t)K * C;
  hipLaunchKernelGGL(wino_wgrad_finalize_kernel, dim3((unsigned)((n + kWfKC - 1) / kWfKC)), dim3(256), 0, stream, part,
                     out, K, C, splits);
}

}  // namespace gk
