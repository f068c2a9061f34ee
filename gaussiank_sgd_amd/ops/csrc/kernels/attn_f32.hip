// Fused multi-head self-attention in fp32 (head dim 64) for gfx950: the
// flash-style forward and two-kernel backward of attn.hip, at the
// reference's precision (fp32 operands, v_mfma_f32_16x16x4_f32: exact fp32
// products, fp32 accumulation).  Replaces torch's SDPA on the fp32 BERT path
// (BASELINE config 5; the reference trains in fp32, settings.py:28), which
// materialises every [T x T] score / probability matrix in HBM.
//
// I/O layouts (fp32), as attn.hip: qkv / dqkv [B, T, 3, heads, 64], out / dout
// [B, T, heads, 64], lse [B, heads, T] (log2 domain), delta [B, heads, T].
// Dropout: the same pair hashes as attn.hip (keep(query, key) = half (key & 1)
// of hash(seed, (bh*T + q)*T/2 + key/2) >= round(p * 65536)), so
// ops/attention.dropout_mask describes both precisions.
//
// MFMA v_mfma_f32_16x16x4_f32, lane = 16 g + li: operand A[i][k] -> lane
// (i = li, k = g), B[k][j] -> lane (k = g, j = li), D[i][j] -> lane holds
// D[4g + r][li], r = 0..3.  A contraction over 16 consecutive elements is
// issued as 4 MFMAs over a fixed permutation: lane group g holds elements
// 4g .. 4g+3 as one float4 and MFMA j contracts element j of every group (the
// same permutation on both operands, so the sum is exact and the ds_read_b128
// feeds four MFMAs).
//
// Scores are computed transposed, S^T = K Q^T (forward, dQ kernel): a lane owns
// ONE query (li) and keys 4g + r of every 16-key tile; those are exactly the
// B-operand slots of O^T = V^T P^T when MFMA j contracts keys {4g + j}, so P
// never leaves the registers.  The V (or K) operand of that product is read as
// one fp32 per lane (ds_read_b32) from the same LDS tile.  The dK/dV kernel
// keeps 32 keys per wave resident and computes S = Q K^T (query on 4g + r).
//
// Every [64 rows][64] fp32 LDS tile (256-byte rows) stores 16-byte chunk c of
// row r at chunk c ^ (r & 15): conflict-free for the 16-row ds_read_b128
// operand reads (lane groups {0-3,12-15,20-27}, ...) and for the ds_read_b32
// reads of rows 4g + j (g = 0 and 1 land in disjoint bank halves).  Tiles are
// staged by LDS-DMA (global_load_lds 16 B per lane; the swizzle is applied to
// the source address), two stages deep.
#include "common.h"
#include "gk_kernels.h"
#include "mfma_util.h"

namespace gk {
namespace {

constexpr int kHD = 64;                     // head dim
constexpr int kKT = 64;                     // rows per LDS tile
constexpr int kFTile = kKT * kHD * 4;       // 16 KiB
constexpr int kWaves = 4;                   // 32 rows per wave
constexpr int kRows = 32 * kWaves;          // rows per workgroup
constexpr float kLazy = 8.f;                // forward: rescale when a row max grows by more than this (log2)

__device__ __forceinline__ uint32_t foff(int r, int c) { return (uint32_t)(r * 256 + ((c ^ (r & 15)) << 4)); }
// byte offset of element (r, col) (ds_read_b32)
__device__ __forceinline__ uint32_t foff1(int r, int col) { return foff(r, col >> 2) + ((col & 3) << 2); }

__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ f32x4 splat4(float v) { return f32x4{v, v, v, v}; }
__device__ __forceinline__ f32x4 mfma4(float a, float b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
// 16-element contraction: acc += sum_j a[j] * b[j] over the permuted K slots
__device__ __forceinline__ f32x4 mfma16(const f32x4& a, const f32x4& b, f32x4 c) {
  c = mfma4(a[0], b[0], c);
  c = mfma4(a[1], b[1], c);
  c = mfma4(a[2], b[2], c);
  return mfma4(a[3], b[3], c);
}

__device__ __forceinline__ int xcd_block() {
  const int n = gridDim.x, b = blockIdx.x;
  if (n % 8) return b;
  return (b & 7) * (n >> 3) + (b >> 3);
}

struct AttnF32Args {
  const float* qkv;
  const float* out;
  const float* dout;
  float* o;
  float* dqkv;
  float* lse;
  float* delta;
  int T, H;
  float sc;        // log2(e) / sqrt(64)
  float qscale;    // 1 / sqrt(64)
  float dscale;    // 1 / (1 - p_effective)
  uint32_t thr;    // drop threshold on 16 hash bits
  uint32_t seed;
  const uint32_t* seed_dev;
};

__device__ __forceinline__ uint32_t eff_seed(const AttnF32Args& a) {
  if (a.seed_dev == nullptr) return a.seed;
  return hash_u32(__builtin_amdgcn_readfirstlane(*a.seed_dev), a.seed);
}

// this wave's 4 LDS-DMA pieces (1 KiB = 4 rows each) of a [64][64] fp32 tile
// whose row 0 is at src (row stride ld floats): pieces 4 wave .. 4 wave + 3
struct TileDma {
  const float* p[4];
  __device__ __forceinline__ void init(const float* src, int64_t ld, int wave, int lane) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int piece = wave * 4 + i;
      const int r = piece * 4 + (lane >> 4);
      const int c = (lane & 15) ^ (r & 15);
      p[i] = src + (int64_t)r * ld + c * 4;
    }
  }
  __device__ __forceinline__ void issue(int64_t off, GK_LDS char* tile, int wave) const {
#pragma unroll
    for (int i = 0; i < 4; ++i) glds16(p[i] + off, tile + (wave * 4 + i) * 1024);
  }
};

__device__ __forceinline__ f32x4 ld4(const char* lds, uint32_t off) {
  return *reinterpret_cast<const f32x4*>(lds + off);
}
__device__ __forceinline__ float ld1(const char* lds, uint32_t off) { return *reinterpret_cast<const float*>(lds + off); }

// ---------------------------------------------------------------------------
// forward: 4 waves x 32 queries of one (batch, head); K / V tiles of 64 keys
// ---------------------------------------------------------------------------
template <bool DROP>
__global__ void __launch_bounds__(64 * kWaves, 2) attn_f32_fwd_kernel(AttnF32Args a) {
  extern __shared__ __attribute__((aligned(1024))) char smem[];   // 2 stages x (K, V)
  const uint32_t seed = DROP ? eff_seed(a) : 0u;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int li = lane & 15, g = lane >> 4;
  const int T = a.T, H = a.H;
  const int nqb = T / kRows;
  const int blk = xcd_block();
  const int bh = blk / nqb, qb = blk - bh * nqb;
  const int b = bh / H, h = bh - b * H;
  const int64_t ld = 3LL * H * kHD;
  const float* base = a.qkv + (int64_t)b * T * ld;
  const int q0 = qb * kRows + wave * 32;
  GK_LDS char* lds = (GK_LDS char*)smem;
  TileDma dk, dv;
  dk.init(base + (int64_t)(H + h) * kHD, ld, wave, lane);
  dv.init(base + (int64_t)(2 * H + h) * kHD, ld, wave, lane);
  const int64_t tstep = kKT * ld;
  const int nt = T / kKT;

  dk.issue(0, lds, wave);
  dv.issue(0, lds + kFTile, wave);
  f32x4 qf[2][4];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int c = 0; c < 4; ++c)
      qf[qt][c] = *reinterpret_cast<const f32x4*>(base + h * kHD + (int64_t)(q0 + 16 * qt + li) * ld + 16 * c + 4 * g) *
                  a.sc;

  f32x4 o[2][4];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[qt][dt] = splat4(0.f);
  float m[2] = {0.f, 0.f}, l[2] = {0.f, 0.f};
  uint32_t hrow[2];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) hrow[qt] = ((uint32_t)bh * T + q0 + 16 * qt + li) * (uint32_t)(T >> 1) + 2 * g;

  for (int t = 0; t < nt; ++t) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's pieces of tile t
    __builtin_amdgcn_s_barrier();                        // everyone's pieces; tile t - 1 consumed
    __builtin_amdgcn_sched_barrier(0);
    const char* Ks = smem + (t & 1) * 2 * kFTile;
    const char* Vs = Ks + kFTile;
    if (t + 1 < nt) {
      GK_LDS char* nx = lds + ((t + 1) & 1) * 2 * kFTile;
      dk.issue((t + 1) * tstep, nx, wave);
      dv.issue((t + 1) * tstep, nx + kFTile, wave);
    }

    // S^T - m (log2 units)
    f32x4 s[2][4];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) s[qt][kt] = splat4(-m[qt]);
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        const f32x4 kv = ld4(Ks, foff(16 * kt + li, 4 * c + g));
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) s[qt][kt] = mfma16(kv, qf[qt][c], s[qt][kt]);
      }

#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      float mx = fmaxf(fmaxf(s[qt][0][0], s[qt][0][1]), fmaxf(s[qt][0][2], s[qt][0][3]));
#pragma unroll
      for (int kt = 1; kt < 4; ++kt)
        mx = fmaxf(mx, fmaxf(fmaxf(s[qt][kt][0], s[qt][kt][1]), fmaxf(s[qt][kt][2], s[qt][kt][3])));
      if (t == 0 || __ballot(mx > kLazy) != 0) {
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        const float d = t == 0 ? mx : fmaxf(mx, 0.f);
        m[qt] += d;
        const float al = fexp2(-d);
        l[qt] *= al;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) o[qt][dt] *= al;
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) s[qt][kt] -= splat4(d);
      }
      float ls = 0.f;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        uint32_t hh[2];
        if (DROP) {
          const uint32_t pi = hrow[qt] + t * (kKT / 2) + 8 * kt;
          hh[0] = hash_u32(pi, seed);
          hh[1] = hash_u32(pi + 1, seed);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float p = fexp2(s[qt][kt][r]);
          ls += p;
          if (DROP) {
            const uint32_t u = (r & 1) ? hh[r >> 1] >> 16 : hh[r >> 1] & 0xffffu;
            p = u >= a.thr ? p : 0.f;
          }
          s[qt][kt][r] = p;
        }
      }
      l[qt] += ls;
    }

    // O^T += V^T P^T: MFMA j contracts keys 16 kt + 4g + j
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float vv[4];
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) vv[dt] = ld1(Vs, foff1(16 * kt + 4 * g + j, 16 * dt + li));
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
          for (int qt = 0; qt < 2; ++qt) o[qt][dt] = mfma4(vv[dt], s[qt][kt][j], o[qt][dt]);
      }
  }

#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    float lt = l[qt];
    lt += __shfl_xor(lt, 16, 64);
    lt += __shfl_xor(lt, 32, 64);
    const int q = q0 + 16 * qt + li;
    if (g == 0) a.lse[(int64_t)bh * T + q] = m[qt] + __log2f(lt);
    const float inv = a.dscale / lt;
    float* op = a.o + ((int64_t)b * T + q) * (H * kHD) + h * kHD + 4 * g;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) *reinterpret_cast<f32x4*>(op + 16 * dt) = o[qt][dt] * inv;
  }
}

// ---------------------------------------------------------------------------
// backward, dQ (+ delta = rowsum(dO * O)): per key tile S^T = c K Q^T - lse,
// dZ^T = V dO^T - delta', dS^T = P^T (dP^T - delta), dQ^T += K^T dS^T
// ---------------------------------------------------------------------------
template <bool DROP>
__global__ void __launch_bounds__(64 * kWaves, 2) attn_f32_bwd_dq_kernel(AttnF32Args a) {
  extern __shared__ __attribute__((aligned(1024))) char smem[];   // 2 stages x (K, V)
  const uint32_t seed = DROP ? eff_seed(a) : 0u;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int li = lane & 15, g = lane >> 4;
  const int T = a.T, H = a.H;
  const int nqb = T / kRows;
  const int blk = xcd_block();
  const int bh = blk / nqb, qb = blk - bh * nqb;
  const int b = bh / H, h = bh - b * H;
  const int64_t ld = 3LL * H * kHD, ldo = (int64_t)H * kHD;
  const float* base = a.qkv + (int64_t)b * T * ld;
  const int q0 = qb * kRows + wave * 32;
  GK_LDS char* lds = (GK_LDS char*)smem;
  TileDma dk, dv;
  dk.init(base + (int64_t)(H + h) * kHD, ld, wave, lane);
  dv.init(base + (int64_t)(2 * H + h) * kHD, ld, wave, lane);
  const int64_t tstep = kKT * ld;
  const int nt = T / kKT;

  dk.issue(0, lds, wave);
  dv.issue(0, lds + kFTile, wave);
  f32x4 qf[2][4], df[2][4];
  float nlse[2], del[2], ndel[2];
  uint32_t hrow[2];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int q = q0 + 16 * qt + li;
    const int64_t orow = ((int64_t)b * T + q) * ldo + h * kHD;
    float dsum = 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      qf[qt][c] = *reinterpret_cast<const f32x4*>(base + h * kHD + (int64_t)q * ld + 16 * c + 4 * g) * a.sc;
      df[qt][c] = *reinterpret_cast<const f32x4*>(a.dout + orow + 16 * c + 4 * g);
      const f32x4 ov = *reinterpret_cast<const f32x4*>(a.out + orow + 16 * c + 4 * g);
#pragma unroll
      for (int e = 0; e < 4; ++e) dsum = fmaf(df[qt][c][e], ov[e], dsum);
    }
    dsum += __shfl_xor(dsum, 16, 64);
    dsum += __shfl_xor(dsum, 32, 64);
    del[qt] = dsum;
    ndel[qt] = DROP ? -dsum / a.dscale : -dsum;
    nlse[qt] = -a.lse[(int64_t)bh * T + q];
    if (g == 0) a.delta[(int64_t)bh * T + q] = dsum;
    hrow[qt] = ((uint32_t)bh * T + q) * (uint32_t)(T >> 1) + 2 * g;
  }

  f32x4 dq[2][4];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dq[qt][dt] = splat4(0.f);

  for (int t = 0; t < nt; ++t) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    const char* Ks = smem + (t & 1) * 2 * kFTile;
    const char* Vs = Ks + kFTile;
    if (t + 1 < nt) {
      GK_LDS char* nx = lds + ((t + 1) & 1) * 2 * kFTile;
      dk.issue((t + 1) * tstep, nx, wave);
      dv.issue((t + 1) * tstep, nx + kFTile, wave);
    }

    f32x4 s[2][4], dz[2][4];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        s[qt][kt] = splat4(nlse[qt]);
        dz[qt][kt] = splat4(ndel[qt]);
      }
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const f32x4 kv = ld4(Ks, foff(16 * kt + li, 4 * c + g));
        const f32x4 vv = ld4(Vs, foff(16 * kt + li, 4 * c + g));
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) {
          s[qt][kt] = mfma16(kv, qf[qt][c], s[qt][kt]);
          dz[qt][kt] = mfma16(vv, df[qt][c], dz[qt][kt]);
        }
      }
      __builtin_amdgcn_sched_barrier(0);   // one key tile's operand reads in flight at a time (VGPRs)
    }

#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        uint32_t hh[2];
        if (DROP) {
          const uint32_t pi = hrow[qt] + t * (kKT / 2) + 8 * kt;
          hh[0] = hash_u32(pi, seed);
          hh[1] = hash_u32(pi + 1, seed);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = fexp2(s[qt][kt][r]);
          float dd = dz[qt][kt][r];   // dP - delta (no dropout)
          if (DROP) {
            const uint32_t u = (r & 1) ? hh[r >> 1] >> 16 : hh[r >> 1] & 0xffffu;
            dd = u >= a.thr ? dd * a.dscale : -del[qt];
          }
          s[qt][kt][r] = p * dd;
        }
      }

    // dQ^T += K^T dS^T: MFMA j contracts keys 16 kt + 4g + j
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float kk[4];
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) kk[dt] = ld1(Ks, foff1(16 * kt + 4 * g + j, 16 * dt + li));
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
          for (int qt = 0; qt < 2; ++qt) dq[qt][dt] = mfma4(kk[dt], s[qt][kt][j], dq[qt][dt]);
        __builtin_amdgcn_sched_barrier(0);
      }
  }

#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int q = q0 + 16 * qt + li;
    float* dp = a.dqkv + ((int64_t)b * T + q) * ld + h * kHD + 4 * g;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) *reinterpret_cast<f32x4*>(dp + 16 * dt) = dq[qt][dt] * a.qscale;
  }
}

// ---------------------------------------------------------------------------
// backward, dK / dV: 4 waves x 32 keys; K (pre-scaled) and V of the wave's
// keys stay in registers while query tiles of 64 (Q, dO, lse, delta) stream
// through LDS.  Per 16-query tile: S = c Q K^T - lse, dZ = dO V^T - delta'
// (query on 4g + r), P, dS; dV^T += dO^T P, dK^T += Q^T dS.
// ---------------------------------------------------------------------------
constexpr int kKvStage = 2 * kFTile + 512;   // Q tile, dO tile, lse[64], delta[64]

template <bool DROP>
__global__ void __launch_bounds__(64 * kWaves, 2) attn_f32_bwd_kv_kernel(AttnF32Args a) {
  extern __shared__ __attribute__((aligned(1024))) char smem[];   // 2 x kKvStage
  const uint32_t seed = DROP ? eff_seed(a) : 0u;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int li = lane & 15, g = lane >> 4;
  const int T = a.T, H = a.H;
  const int nkb = T / kRows;
  const int blk = xcd_block();
  const int bh = blk / nkb, kb = blk - bh * nkb;
  const int b = bh / H, h = bh - b * H;
  const int64_t ld = 3LL * H * kHD, ldo = (int64_t)H * kHD;
  const float* base = a.qkv + (int64_t)b * T * ld;
  const float* lsep = a.lse + (int64_t)bh * T;
  const float* delp = a.delta + (int64_t)bh * T;
  const int k0 = kb * kRows + wave * 32;
  GK_LDS char* lds = (GK_LDS char*)smem;
  TileDma dq, dd;
  dq.init(base + (int64_t)h * kHD, ld, wave, lane);
  dd.init(a.dout + (int64_t)b * T * ldo + (int64_t)h * kHD, ldo, wave, lane);
  auto stage = [&](int t, int buf) {
    GK_LDS char* dst = lds + buf * kKvStage;
    dq.issue((int64_t)t * kKT * ld, dst, wave);
    dd.issue((int64_t)t * kKT * ldo, dst + kFTile, wave);
    if (wave < 2)
      __builtin_amdgcn_global_load_lds((wave ? delp : lsep) + t * kKT + lane, dst + 2 * kFTile + wave * 256, 4, 0, 0);
  };
  const int nt = T / kKT;

  stage(0, 0);
  f32x4 kf[2][4], vf[2][4];
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int64_t row = (int64_t)(k0 + 16 * kt + li) * ld + 16 * c + 4 * g;
      kf[kt][c] = *reinterpret_cast<const f32x4*>(base + (int64_t)(H + h) * kHD + row) * a.sc;
      vf[kt][c] = *reinterpret_cast<const f32x4*>(base + (int64_t)(2 * H + h) * kHD + row);
    }
  f32x4 dvv[2][4], dkk[2][4];
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dvv[kt][dt] = dkk[kt][dt] = splat4(0.f);
  // dropout: pair hash of (query, key >> 1); key & 1 = li & 1 picks the half
  const uint32_t hbase = (uint32_t)bh * T * (uint32_t)(T >> 1);
  const uint32_t hsh = 16u * (uint32_t)(li & 1);

  for (int t = 0; t < nt; ++t) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    const char* Qs = smem + (t & 1) * kKvStage;
    const char* Ds = Qs + kFTile;
    const float* Ls = reinterpret_cast<const float*>(Qs + 2 * kFTile);
    if (t + 1 < nt) stage(t + 1, (t + 1) & 1);

#pragma unroll 1
    for (int qt = 0; qt < 4; ++qt) {   // not unrolled: one 16-query tile's operands live at a time
      const int qr = 16 * qt + 4 * g;   // tile row of r = 0
      const f32x4 nl = -*reinterpret_cast<const f32x4*>(Ls + qr);
      const f32x4 del4 = *reinterpret_cast<const f32x4*>(Ls + 64 + qr);
      const f32x4 nd = DROP ? -del4 * (1.f / a.dscale) : -del4;
      f32x4 s[2], dz[2];
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        s[kt] = nl;
        dz[kt] = nd;
      }
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const f32x4 qv = ld4(Qs, foff(16 * qt + li, 4 * c + g));
        const f32x4 ov = ld4(Ds, foff(16 * qt + li, 4 * c + g));
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          s[kt] = mfma16(qv, kf[kt][c], s[kt]);
          dz[kt] = mfma16(ov, vf[kt][c], dz[kt]);
        }
      }
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = fexp2(s[kt][r]);
          float z = p, d2 = dz[kt][r];   // dP - delta (no dropout)
          if (DROP) {
            const uint32_t qg = (uint32_t)(t * kKT + qr + r);
            const uint32_t hv = hash_u32(hbase + qg * (uint32_t)(T >> 1) + (uint32_t)((k0 + 16 * kt + li) >> 1), seed);
            const bool keep = __builtin_amdgcn_ubfe(hv, hsh, 16) >= a.thr;
            z = keep ? p * a.dscale : 0.f;
            d2 = keep ? d2 * a.dscale : -del4[r];
          }
          s[kt][r] = z;
          dz[kt][r] = p * d2;
        }
      }
      // dV^T += dO^T P, dK^T += Q^T dS: MFMA j contracts queries 16 qt + 4g + j
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float ov[4], qv[4];
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          ov[dt] = ld1(Ds, foff1(16 * qt + 4 * g + j, 16 * dt + li));
          qv[dt] = ld1(Qs, foff1(16 * qt + 4 * g + j, 16 * dt + li));
        }
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
          for (int kt = 0; kt < 2; ++kt) {
            dvv[kt][dt] = mfma4(ov[dt], s[kt][j], dvv[kt][dt]);
            dkk[kt][dt] = mfma4(qv[dt], dz[kt][j], dkk[kt][dt]);
          }
      }
    }
  }

#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    const int key = k0 + 16 * kt + li;
    float* row = a.dqkv + ((int64_t)b * T + key) * ld + 4 * g;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      *reinterpret_cast<f32x4*>(row + (int64_t)(H + h) * kHD + 16 * dt) = dkk[kt][dt] * a.qscale;
      *reinterpret_cast<f32x4*>(row + (int64_t)(2 * H + h) * kHD + 16 * dt) = dvv[kt][dt];
    }
  }
}

AttnF32Args make_args(int T, int H, float p, uint32_t seed, const uint32_t* seed_dev) {
  AttnF32Args a{};
  a.seed_dev = seed_dev;
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

template <typename K>
void launch(K kern, int nblocks, int lds, const AttnF32Args& a, hipStream_t stream) {
  hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  hipLaunchKernelGGL(kern, dim3((unsigned)nblocks), dim3(64 * kWaves), lds, stream, a);
}

}  // namespace

bool attn_f32_supported(int T, int D) { return D == kHD && T >= kRows && T % kRows == 0; }

void attn_f32_fwd(const float* qkv, float* out, float* lse, int B, int T, int H, float p, uint32_t seed,
                  const uint32_t* seed_dev, hipStream_t stream) {
  AttnF32Args a = make_args(T, H, p, seed, seed_dev);
  a.qkv = qkv;
  a.o = out;
  a.lse = lse;
  const int nb = B * H * (T / kRows);
  if (a.thr) launch(attn_f32_fwd_kernel<true>, nb, 4 * kFTile, a, stream);
  else launch(attn_f32_fwd_kernel<false>, nb, 4 * kFTile, a, stream);
}

void attn_f32_bwd(const float* qkv, const float* out, const float* dout, const float* lse, float* delta, float* dqkv,
                  int B, int T, int H, float p, uint32_t seed, const uint32_t* seed_dev, hipStream_t stream) {
  AttnF32Args a = make_args(T, H, p, seed, seed_dev);
  a.qkv = qkv;
  a.out = out;
  a.dout = dout;
  a.lse = const_cast<float*>(lse);
  a.delta = delta;
  a.dqkv = dqkv;
  const int nb = B * H * (T / kRows);
  if (a.thr) {
    launch(attn_f32_bwd_dq_kernel<true>, nb, 4 * kFTile, a, stream);
    launch(attn_f32_bwd_kv_kernel<true>, nb, 2 * kKvStage, a, stream);
  } else {
    launch(attn_f32_bwd_dq_kernel<false>, nb, 4 * kFTile, a, stream);
    launch(attn_f32_bwd_kv_kernel<false>, nb, 2 * kKvStage, a, stream);
  }
}

}  // namespace gk
