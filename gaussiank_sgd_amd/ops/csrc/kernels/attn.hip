// Fused multi-head self-attention for gfx950 (head dim 64): flash-style
// forward and backward for the BERT encoder (models/bert.py).  Not part of the
// reference (its BERT-free model zoo is models/*.py in the reference tree);
// this replaces torch's SDPA + the head split/merge copies around it.
//
// I/O layouts (bf16), no permute copies anywhere:
//   qkv  [B, T, 3, heads, 64]  the QKV projection output as produced
//   out  [B, T, heads, 64]     = the attention-output linear's input
//   dqkv [B, T, 3, heads, 64]  = the QKV projection's output gradient
//   lse  [B, heads, T] fp32    log2-domain row normaliser: P = exp2(c*s - lse)
//   with s = q.k and c = log2(e) / sqrt(64).
//
// MFMA conventions (v_mfma_f32_16x16x32_bf16, lane = 16*g + li):
//   operand A[i][k] and B[k][j]: the lane holds index li and k = 8g .. 8g+7;
//   result D[i][j]: the lane holds D[4g + r][li], r = 0..3.
// The forward (and the dQ kernel) compute S^T = K Q^T, so a lane owns ONE
// query (li) and keys 4g + r of every 16-key tile.  Two adjacent 16-key result
// tiles are then exactly the 8 k-slots of the B operand of O^T = V^T P^T
// (keys {4g + r} and {16 + 4g + r}); V^T is read with ds_read_b64_tr_b16 from
// those same key rows.  Softmax is lane-local up to the row max, which needs
// lanes li, li^16, li^32, li^48 only; the row sum is reduced once at the end.
// The dK/dV kernel keeps 32 keys per wave resident and computes S = Q K^T
// (query on 4g + r), so P and dS are directly the B operands of
// dV^T = dO^T P and dK^T = Q^T dS.
//
// Every [64 rows][64] bf16 LDS tile uses one XOR swizzle of its 16-byte chunks
// (aswz below) that is conflict-free for both the 16-row ds_read_b128 operand
// reads and the 8-row transposed reads, so Q / K tiles serve both.
//
// Dropout: keep(query, key) = hash(seed, (bh*T + q)*T + k) >= p * 65536, the
// same function in all three kernels (and attn_dropout_mask, for tests); the
// mask is regenerated, never stored.
#include "common.h"
#include "gk_kernels.h"
#include "mfma_util.h"

namespace gk {
namespace {

constexpr int kHD = 64;                 // head dim
constexpr int kKT = 64;                 // rows per LDS tile (keys, or queries in the dK/dV kernel)
constexpr int kTileB = kKT * kHD * 2;   // 8 KiB
constexpr int kAW = 4;                  // waves per workgroup, 32 rows each
constexpr int kRows = 32 * kAW;         // rows per workgroup

// chunk swizzle of a [rows][128 B] tile: 16 consecutive rows read at one chunk
// hit 16 distinct 16-byte bank slots, and 8 aligned rows x a chunk pair (the
// transposed read of one half-wave) too
__device__ __forceinline__ int aswz(int r) { return (((r >> 1) & 3) << 1) | ((r >> 3) & 1); }
__device__ __forceinline__ int aoff(int r, int c) { return r * 128 + ((c ^ aswz(r)) << 4); }

__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }

__device__ __forceinline__ bool drop_keep(uint32_t seed, uint32_t idx, uint32_t thr) {
  return (hash_u32(idx, seed) >> 16) >= thr;
}

__device__ __forceinline__ uint32_t lds_addr(const void* p) { return (uint32_t)(uintptr_t)(GK_LDS const char*)p; }

// rows r0 .. r0+63 (64 bf16 columns each) of two matrices into two swizzled
// LDS tiles at dst and dst + 8 KiB (16-byte LDS-DMA, one 1-KiB piece per
// wave-instruction)
__device__ __forceinline__ void stage_pair(const uint16_t* a, int64_t lda, const uint16_t* b, int64_t ldb, int r0,
                                           GK_LDS char* dst, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 16 / kAW; ++i) {
    const int piece = wave * (16 / kAW) + i;
    const int r = (piece & 7) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ aswz(r);
    const uint16_t* src = piece < 8 ? a + (int64_t)(r0 + r) * lda : b + (int64_t)(r0 + r) * ldb;
    glds16(src + c * 8, dst + piece * 1024);
  }
}

// transposed operand fragment: rows R .. R+3 (lo) and R+16 .. R+19 (hi) of a
// tile, the lane's column; addr = lane address of the lo read, OFF a byte
// immediate (row block / tile)
template <int OFF>
__device__ __forceinline__ bf16x8 tr_frag16(uint32_t addr) {
  bf16x4 lo, hi;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(lo) : "v"(addr), "i"(OFF));
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(hi) : "v"(addr), "i"(OFF + 2048));
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

__device__ __forceinline__ void lgkm_sync4(bf16x8* f) {
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]));
}

// lane address of the transposed read for output block dt (16 columns):
// row 4g + (li >> 2), columns 16 dt + 4 (li & 3) .. + 3
__device__ __forceinline__ uint32_t tr_lane_off(int lane, int dt) {
  const int li = lane & 15, g = lane >> 4;
  const int row = 4 * g + (li >> 2), p = li & 3;
  return (uint32_t)(aoff(row, 2 * dt + (p >> 1)) + (p & 1) * 8);
}

// 8 k-slots of a B operand from two 16-row result tiles (rows 4g+r of each)
__device__ __forceinline__ bf16x8 pack_pair(const f32x4& a, const f32x4& b) {
  const uint32_t w[4] = {pack_bf16x2(a[0], a[1]), pack_bf16x2(a[2], a[3]), pack_bf16x2(b[0], b[1]),
                         pack_bf16x2(b[2], b[3])};
  return __builtin_bit_cast(bf16x8, w);
}

__device__ __forceinline__ f32x4 mfma(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void store4(uint16_t* p, const f32x4& v, float s) {
  *reinterpret_cast<uint2*>(p) = make_uint2(pack_bf16x2(v[0] * s, v[1] * s), pack_bf16x2(v[2] * s, v[3] * s));
}

struct AttnArgs {
  const uint16_t* qkv;
  const uint16_t* out;
  const uint16_t* dout;
  uint16_t* o;        // forward output
  uint16_t* dqkv;
  float* lse;
  float* delta;
  int T, H;
  float sc;           // log2(e) / sqrt(64)
  float qscale;       // 1 / sqrt(64)
  float dscale;       // 1 / (1 - p_effective)
  uint32_t thr;       // drop threshold on 16 hash bits
  uint32_t seed;
};

// ---------------------------------------------------------------------------
// forward: one workgroup = 4 waves x 32 queries of one (batch, head); K/V
// tiles of 64 keys double-buffered in LDS
// ---------------------------------------------------------------------------
template <bool DROP>
__global__ void __launch_bounds__(64 * kAW) attn_fwd_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(1024))) char smem[4 * kTileB];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, li = lane & 15, g = lane >> 4;
  const int T = a.T, H = a.H;
  const int nqb = T / kRows;
  const int bh = blockIdx.x / nqb, qb = blockIdx.x - bh * nqb;
  const int b = bh / H, h = bh - b * H;
  const int64_t ld = 3LL * H * kHD;
  const uint16_t* base = a.qkv + (int64_t)b * T * ld;
  const uint16_t* kp = base + (int64_t)(H + h) * kHD;
  const uint16_t* vp = base + (int64_t)(2 * H + h) * kHD;
  const int q0 = qb * kRows + wave * 32;
  GK_LDS char* lds = (GK_LDS char*)smem;
  stage_pair(kp, ld, vp, ld, 0, lds, wave, lane);

  bf16x8 qf[2][2];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      qf[qt][ks] = *reinterpret_cast<const bf16x8*>(base + h * kHD + (int64_t)(q0 + 16 * qt + li) * ld + 32 * ks + 8 * g);

  f32x4 o[2][4];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[qt][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m[2] = {-1e30f, -1e30f}, l[2] = {0.f, 0.f};
  uint32_t hrow[2];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) hrow[qt] = ((uint32_t)bh * T + q0 + 16 * qt + li) * (uint32_t)T + 4 * g;
  uint32_t toff[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) toff[dt] = tr_lane_off(lane, dt);
  const uint32_t lbase = lds_addr(smem);

  const int nt = T / kKT;
  for (int t = 0; t < nt; ++t) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (t + 1 < nt) stage_pair(kp, ld, vp, ld, (t + 1) * kKT, lds + ((t + 1) & 1) * 2 * kTileB, wave, lane);
    const char* Ks = smem + (t & 1) * 2 * kTileB;

    f32x4 s[2][4];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) s[qt][kt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(Ks + aoff(16 * kt + li, 4 * ks + g));
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) s[qt][kt] = mfma(kf, qf[qt][ks], s[qt][kt]);
      }

#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      float mx = s[qt][0][0];
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) mx = fmaxf(mx, s[qt][kt][r]);
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mn = fmaxf(m[qt], mx * a.sc);
      const float al = fexp2(m[qt] - mn);
      m[qt] = mn;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) o[qt][dt] *= al;
      float ls = 0.f;
      const uint32_t hb = hrow[qt] + t * kKT;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float p = fexp2(fmaf(s[qt][kt][r], a.sc, -mn));
          ls += p;
          if (DROP && !drop_keep(a.seed, hb + 16 * kt + r, a.thr)) p = 0.f;
          s[qt][kt][r] = p;
        }
      l[qt] = l[qt] * al + ls;
    }

    const uint32_t vb = lbase + (t & 1) * 2 * kTileB + kTileB;
    bf16x8 pf[2][2];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      pf[qt][0] = pack_pair(s[qt][0], s[qt][1]);
      pf[qt][1] = pack_pair(s[qt][2], s[qt][3]);
    }
    bf16x8 vf[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) vf[dt] = tr_frag16<0>(vb + toff[dt]);
    lgkm_sync4(vf);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) o[qt][dt] = mfma(vf[dt], pf[qt][0], o[qt][dt]);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) vf[dt] = tr_frag16<4096>(vb + toff[dt]);
    lgkm_sync4(vf);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) o[qt][dt] = mfma(vf[dt], pf[qt][1], o[qt][dt]);
  }

#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    float lt = l[qt];
    lt += __shfl_xor(lt, 16, 64);
    lt += __shfl_xor(lt, 32, 64);
    const int q = q0 + 16 * qt + li;
    if (g == 0) a.lse[(int64_t)bh * T + q] = m[qt] + __log2f(lt);
    const float inv = a.dscale / lt;
    uint16_t* op = a.o + ((int64_t)b * T + q) * (H * kHD) + h * kHD + 4 * g;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) store4(op + 16 * dt, o[qt][dt], inv);
  }
}

// ---------------------------------------------------------------------------
// backward, dQ (+ delta = rowsum(dO * O)): the forward's structure; per key
// tile S^T = K Q^T, dZ^T = V dO^T, dS^T = P^T (dP^T - delta), dQ^T += K^T dS^T
// ---------------------------------------------------------------------------
template <bool DROP>
__global__ void __launch_bounds__(64 * kAW) attn_bwd_dq_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(1024))) char smem[4 * kTileB];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, li = lane & 15, g = lane >> 4;
  const int T = a.T, H = a.H;
  const int nqb = T / kRows;
  const int bh = blockIdx.x / nqb, qb = blockIdx.x - bh * nqb;
  const int b = bh / H, h = bh - b * H;
  const int64_t ld = 3LL * H * kHD, ldo = (int64_t)H * kHD;
  const uint16_t* base = a.qkv + (int64_t)b * T * ld;
  const uint16_t* kp = base + (int64_t)(H + h) * kHD;
  const uint16_t* vp = base + (int64_t)(2 * H + h) * kHD;
  const int q0 = qb * kRows + wave * 32;
  GK_LDS char* lds = (GK_LDS char*)smem;
  stage_pair(kp, ld, vp, ld, 0, lds, wave, lane);

  bf16x8 qf[2][2], df[2][2];
  float lse2[2], del[2];
  uint32_t hrow[2];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int q = q0 + 16 * qt + li;
    const int64_t orow = ((int64_t)b * T + q) * ldo + h * kHD;
    float dsum = 0.f;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      qf[qt][ks] = *reinterpret_cast<const bf16x8*>(base + h * kHD + (int64_t)q * ld + 32 * ks + 8 * g);
      df[qt][ks] = *reinterpret_cast<const bf16x8*>(a.dout + orow + 32 * ks + 8 * g);
      const bf16x8 ov = *reinterpret_cast<const bf16x8*>(a.out + orow + 32 * ks + 8 * g);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        dsum = fmaf(__uint_as_float((uint32_t)(uint16_t)df[qt][ks][j] << 16),
                    __uint_as_float((uint32_t)(uint16_t)ov[j] << 16), dsum);
    }
    dsum += __shfl_xor(dsum, 16, 64);
    dsum += __shfl_xor(dsum, 32, 64);
    del[qt] = dsum;
    if (g == 0) a.delta[(int64_t)bh * T + q] = dsum;
    lse2[qt] = a.lse[(int64_t)bh * T + q];
    hrow[qt] = ((uint32_t)bh * T + q) * (uint32_t)T + 4 * g;
  }

  f32x4 dq[2][4];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dq[qt][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  uint32_t toff[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) toff[dt] = tr_lane_off(lane, dt);
  const uint32_t lbase = lds_addr(smem);

  const int nt = T / kKT;
  for (int t = 0; t < nt; ++t) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (t + 1 < nt) stage_pair(kp, ld, vp, ld, (t + 1) * kKT, lds + ((t + 1) & 1) * 2 * kTileB, wave, lane);
    const char* Ks = smem + (t & 1) * 2 * kTileB;
    const char* Vs = Ks + kTileB;

    f32x4 s[2][4], dz[2][4];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) s[qt][kt] = dz[qt][kt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(Ks + aoff(16 * kt + li, 4 * ks + g));
        const bf16x8 vf = *reinterpret_cast<const bf16x8*>(Vs + aoff(16 * kt + li, 4 * ks + g));
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) {
          s[qt][kt] = mfma(kf, qf[qt][ks], s[qt][kt]);
          dz[qt][kt] = mfma(vf, df[qt][ks], dz[qt][kt]);
        }
      }

#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const uint32_t hb = hrow[qt] + t * kKT;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = fexp2(fmaf(s[qt][kt][r], a.sc, -lse2[qt]));
          float dp = dz[qt][kt][r];
          if (DROP) dp = drop_keep(a.seed, hb + 16 * kt + r, a.thr) ? dp * a.dscale : 0.f;
          s[qt][kt][r] = p * (dp - del[qt]);
        }
    }

    const uint32_t kb = lbase + (t & 1) * 2 * kTileB;
    bf16x8 pf[2][2];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      pf[qt][0] = pack_pair(s[qt][0], s[qt][1]);
      pf[qt][1] = pack_pair(s[qt][2], s[qt][3]);
    }
    bf16x8 kf[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) kf[dt] = tr_frag16<0>(kb + toff[dt]);
    lgkm_sync4(kf);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) dq[qt][dt] = mfma(kf[dt], pf[qt][0], dq[qt][dt]);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) kf[dt] = tr_frag16<4096>(kb + toff[dt]);
    lgkm_sync4(kf);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) dq[qt][dt] = mfma(kf[dt], pf[qt][1], dq[qt][dt]);
  }

#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int q = q0 + 16 * qt + li;
    uint16_t* dp = a.dqkv + ((int64_t)b * T + q) * ld + h * kHD + 4 * g;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) store4(dp + 16 * dt, dq[qt][dt], a.qscale);
  }
}

// ---------------------------------------------------------------------------
// backward, dK / dV: one workgroup = 4 waves x 32 keys; K and V of the wave's
// keys stay in registers while query tiles of 64 (Q, dO, lse, delta) stream
// through LDS.  Per 32-query half: S = Q K^T, dZ = dO V^T (query on 4g + r),
// P, dS elementwise, dV^T += dO^T P, dK^T += Q^T dS.
// ---------------------------------------------------------------------------
constexpr int kKvBuf = 2 * kTileB + 512;   // Q tile, dO tile, lse[64], delta[64]

template <bool DROP>
__global__ void __launch_bounds__(64 * kAW) attn_bwd_kv_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(1024))) char smem[2 * kKvBuf];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, li = lane & 15, g = lane >> 4;
  const int T = a.T, H = a.H;
  const int nkb = T / kRows;
  const int bh = blockIdx.x / nkb, kb = blockIdx.x - bh * nkb;
  const int b = bh / H, h = bh - b * H;
  const int64_t ld = 3LL * H * kHD, ldo = (int64_t)H * kHD;
  const uint16_t* base = a.qkv + (int64_t)b * T * ld;
  const uint16_t* qp = base + (int64_t)h * kHD;
  const uint16_t* dop = a.dout + (int64_t)b * T * ldo + (int64_t)h * kHD;
  const float* lsep = a.lse + (int64_t)bh * T;
  const float* delp = a.delta + (int64_t)bh * T;
  const int k0 = kb * kRows + wave * 32;
  GK_LDS char* lds = (GK_LDS char*)smem;

  auto stage = [&](int t, int buf) {
    GK_LDS char* dst = lds + buf * kKvBuf;
    stage_pair(qp, ld, dop, ldo, t * kKT, dst, wave, lane);
    if (wave < 2) __builtin_amdgcn_global_load_lds((wave ? delp : lsep) + t * kKT + lane, dst + 2 * kTileB + wave * 256, 4, 0, 0);
  };
  stage(0, 0);

  bf16x8 kf[2][2], vf[2][2];
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int64_t row = (int64_t)(k0 + 16 * kt + li) * ld + 32 * ks + 8 * g;
      kf[kt][ks] = *reinterpret_cast<const bf16x8*>(base + (int64_t)(H + h) * kHD + row);
      vf[kt][ks] = *reinterpret_cast<const bf16x8*>(base + (int64_t)(2 * H + h) * kHD + row);
    }
  f32x4 dv[2][4], dk[2][4];
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dv[kt][dt] = dk[kt][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  uint32_t toff[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) toff[dt] = tr_lane_off(lane, dt);
  const uint32_t lbase = lds_addr(smem);
  // hash index of (query 4g + r of a tile, this lane's key) before the query offset
  const uint32_t hkey = (uint32_t)bh * T * (uint32_t)T + k0 + li;

  const int nt = T / kKT;
  for (int t = 0; t < nt; ++t) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (t + 1 < nt) stage(t + 1, (t + 1) & 1);
    const char* Qs = smem + (t & 1) * kKvBuf;
    const char* Ds = Qs + kTileB;
    const float* Ls = reinterpret_cast<const float*>(Qs + 2 * kTileB);
    const uint32_t qb = lbase + (t & 1) * kKvBuf;

#pragma unroll
    for (int half = 0; half < 2; ++half) {
      f32x4 s[2][2], dz[2][2];   // [qt][kt]
#pragma unroll
      for (int qt = 0; qt < 2; ++qt)
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) s[qt][kt] = dz[qt][kt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) {
          const int row = 32 * half + 16 * qt + li;
          const bf16x8 qa = *reinterpret_cast<const bf16x8*>(Qs + aoff(row, 4 * ks + g));
          const bf16x8 da = *reinterpret_cast<const bf16x8*>(Ds + aoff(row, 4 * ks + g));
#pragma unroll
          for (int kt = 0; kt < 2; ++kt) {
            s[qt][kt] = mfma(qa, kf[kt][ks], s[qt][kt]);
            dz[qt][kt] = mfma(da, vf[kt][ks], dz[qt][kt]);
          }
        }
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        const int qr = 32 * half + 16 * qt + 4 * g;   // tile row of r = 0
        const f32x4 lse4 = *reinterpret_cast<const f32x4*>(Ls + qr);
        const f32x4 del4 = *reinterpret_cast<const f32x4*>(Ls + 64 + qr);
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float p = fexp2(fmaf(s[qt][kt][r], a.sc, -lse4[r]));
            float z = p, dp = dz[qt][kt][r];
            if (DROP) {
              const bool k = drop_keep(a.seed, hkey + (uint32_t)(t * kKT + qr + r) * (uint32_t)T + 16 * kt, a.thr);
              z = k ? p * a.dscale : 0.f;
              dp = k ? dp * a.dscale : 0.f;
            }
            s[qt][kt][r] = z;
            dz[qt][kt][r] = p * (dp - del4[r]);
          }
      }
      bf16x8 zf[2], sf[2];
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        zf[kt] = pack_pair(s[0][kt], s[1][kt]);
        sf[kt] = pack_pair(dz[0][kt], dz[1][kt]);
      }
      bf16x8 tf[4];
      // dO^T fragments (dO tile, rows 32 half + 4g + ..)
      if (half == 0) {
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) tf[dt] = tr_frag16<kTileB>(qb + toff[dt]);
      } else {
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) tf[dt] = tr_frag16<kTileB + 4096>(qb + toff[dt]);
      }
      lgkm_sync4(tf);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) dv[kt][dt] = mfma(tf[dt], zf[kt], dv[kt][dt]);
      if (half == 0) {
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) tf[dt] = tr_frag16<0>(qb + toff[dt]);
      } else {
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) tf[dt] = tr_frag16<4096>(qb + toff[dt]);
      }
      lgkm_sync4(tf);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) dk[kt][dt] = mfma(tf[dt], sf[kt], dk[kt][dt]);
    }
  }

#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    const int key = k0 + 16 * kt + li;
    uint16_t* row = a.dqkv + ((int64_t)b * T + key) * ld + 4 * g;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      store4(row + (int64_t)(H + h) * kHD + 16 * dt, dk[kt][dt], a.qscale);
      store4(row + (int64_t)(2 * H + h) * kHD + 16 * dt, dv[kt][dt], 1.f);
    }
  }
}

__global__ void attn_dropout_mask_kernel(uint8_t* __restrict__ mask, int64_t n, uint32_t seed, uint32_t thr) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) mask[i] = drop_keep(seed, (uint32_t)i, thr) ? 1 : 0;
}

AttnArgs make_args(int T, int H, float p, uint32_t seed) {
  AttnArgs a{};
  a.T = T;
  a.H = H;
  a.qscale = 0.125f;                       // 1 / sqrt(64)
  a.sc = 1.4426950408889634f * 0.125f;     // log2(e) / sqrt(64)
  uint32_t thr = p > 0.f ? (uint32_t)lrintf(p * 65536.f) : 0u;
  if (thr > 65535u) thr = 65535u;
  a.thr = thr;
  a.dscale = thr ? 65536.f / (float)(65536u - thr) : 1.f;
  a.seed = seed;
  return a;
}

}  // namespace

bool attn_supported(int T, int D) { return D == kHD && T >= kRows && T % kRows == 0; }

void attn_fwd(const void* qkv, void* out, float* lse, int B, int T, int H, float p, uint32_t seed,
              hipStream_t stream) {
  AttnArgs a = make_args(T, H, p, seed);
  a.qkv = static_cast<const uint16_t*>(qkv);
  a.o = static_cast<uint16_t*>(out);
  a.lse = lse;
  const dim3 grid((unsigned)(B * H * (T / kRows)));
  if (a.thr) hipLaunchKernelGGL(attn_fwd_kernel<true>, grid, dim3(64 * kAW), 0, stream, a);
  else hipLaunchKernelGGL(attn_fwd_kernel<false>, grid, dim3(64 * kAW), 0, stream, a);
}

void attn_bwd(const void* qkv, const void* out, const void* dout, const float* lse, float* delta, void* dqkv, int B,
              int T, int H, float p, uint32_t seed, hipStream_t stream) {
  AttnArgs a = make_args(T, H, p, seed);
  a.qkv = static_cast<const uint16_t*>(qkv);
  a.out = static_cast<const uint16_t*>(out);
  a.dout = static_cast<const uint16_t*>(dout);
  a.lse = const_cast<float*>(lse);
  a.delta = delta;
  a.dqkv = static_cast<uint16_t*>(dqkv);
  const dim3 grid((unsigned)(B * H * (T / kRows)));
  if (a.thr) {
    hipLaunchKernelGGL(attn_bwd_dq_kernel<true>, grid, dim3(64 * kAW), 0, stream, a);
    hipLaunchKernelGGL(attn_bwd_kv_kernel<true>, grid, dim3(64 * kAW), 0, stream, a);
  } else {
    hipLaunchKernelGGL(attn_bwd_dq_kernel<false>, grid, dim3(64 * kAW), 0, stream, a);
    hipLaunchKernelGGL(attn_bwd_kv_kernel<false>, grid, dim3(64 * kAW), 0, stream, a);
  }
}

void attn_dropout_mask(uint8_t* mask, int B, int H, int T, float p, uint32_t seed, hipStream_t stream) {
  const AttnArgs a = make_args(T, H, p, seed);
  const int64_t n = (int64_t)B * H * T * T;
  hipLaunchKernelGGL(attn_dropout_mask_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, mask, n,
                     seed, a.thr);
}

}  // namespace gk
