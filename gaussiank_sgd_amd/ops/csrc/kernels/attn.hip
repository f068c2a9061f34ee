// Fused multi-head self-attention for gfx950 (head dim 64): flash-style
// forward and backward for the BERT encoder (models/bert.py).  Not part of the
// reference (its model zoo has no transformer); this replaces torch's SDPA and
// the head split / merge copies around it.
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
// those same key rows.  The dK/dV kernel keeps 32 keys per wave resident and
// computes S = Q K^T (query on 4g + r), so P and dS are directly the B
// operands of dV^T = dO^T P and dK^T = Q^T dS.
//
// The kernels are VALU-bound before they are MFMA-bound (d = 64: 4 MFMAs per
// 16x16 score tile), so the per-score vector work is cut to the bone:
//  - the resident operand (Q in the forward / dQ kernel, K in the dK/dV
//    kernel) is pre-scaled by c once, and the row constants are the MFMA's
//    initial accumulator: S = c q.k - m (forward), c q.k - lse and
//    dZ - delta (backward), so p = exp2(S) needs no per-score arithmetic;
//  - the forward rescales its running max lazily: only when some row's tile
//    max exceeds the current m by 8 (log2 units, so p <= 256) does the wave
//    take the textbook update (cross-lane row max, O and l rescale).  The
//    first tile always takes it, so m starts at the first tile's row max;
//  - one 32-bit hash per PAIR of keys gives both dropout uniforms (16 bits
//    each); the dK/dV kernel (keys on lanes) splits the pair's hashes between
//    neighbour lanes and swaps them with a DPP quad permute.
//
// Every [64 rows][64] bf16 LDS tile uses one XOR swizzle of its 16-byte chunks
// (aswz) that is conflict-free both for the 16-row ds_read_b128 operand reads
// and for the 8-row transposed reads, so Q / K tiles serve both.
//
// Dropout: keep(query, key) = half (key & 1) of hash(seed, (bh*T + q)*T/2 +
// key/2) >= round(p * 65536), in all three kernels and attn_dropout_mask (for
// tests); the mask is regenerated, never stored.
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
constexpr int kPieces = 16 / kAW;       // 1-KiB LDS-DMA pieces per wave per tile pair
constexpr float kLazy = 8.f;            // forward: rescale when a row max grows by more than this (log2)
constexpr int kStages = 3;              // LDS ring: tiles t+1 and t+2 in flight while t is consumed

// chunk swizzle of a [rows][128 B] tile (chunk c of row r at c ^ aswz(r)):
// conflict-free for the ds_read_b128 operand reads (16 consecutive rows at one
// chunk, serviced in the lane groups {0-3,12-15,20-27}, {4-11,16-19,28-31}, ..)
// and for the transposed reads (8 aligned rows x a chunk pair per half-wave);
// found by exhaustive search over XOR maps of the row bits (the plain
// (r >> 1) & 7 map leaves both reads 2-way)
__device__ __forceinline__ int aswz(int r) { return (((r >> 2) & 1) << 1) | (((r >> 1) & 1) << 2); }
__device__ __forceinline__ int aoff(int r, int c) { return r * 128 + ((c ^ aswz(r)) << 4); }

__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }

// Workgroups are dispatched round-robin over the 8 XCDs (each with its own
// L2): give every XCD a contiguous range of logical blocks, so the row blocks
// of one (batch, head) -- which all stream the same K / V (or Q / dO) -- run
// on one XCD and share its L2 instead of fetching them once per XCD.
__device__ __forceinline__ int xcd_block() {
  const int n = gridDim.x, b = blockIdx.x;
  if (n % 8) return b;
  return (b & 7) * (n >> 3) + (b >> 3);
}

// wait until the LDS-DMA of the current tile has landed: only the next
// tile's N pieces (issued after it) may still be in flight
template <int N>
__device__ __forceinline__ void wait_tile(bool last) {
  if (last) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ int ring_next(int b) { return b + 1 == kStages ? 0 : b + 1; }

__device__ __forceinline__ uint32_t lds_addr(const void* p) { return (uint32_t)(uintptr_t)(GK_LDS const char*)p; }

// dropout uniforms of keys (2j, 2j + 1) of one (bh, query)
__device__ __forceinline__ uint32_t pair_hash(uint32_t seed, uint32_t pidx) { return hash_u32(pidx, seed); }

// this wave's LDS-DMA sources for two [rows][64] matrices staged as tiles
// (a: pieces 0..7, b: 8..15) -- row r0 is added per tile
struct DmaSrc {
  const uint16_t* p[kPieces];
  __device__ __forceinline__ void init(const uint16_t* a, int64_t lda, const uint16_t* b, int64_t ldb, int wave,
                                       int lane) {
#pragma unroll
    for (int i = 0; i < kPieces; ++i) {
      const int piece = wave * kPieces + i;
      const int r = (piece & 7) * 8 + (lane >> 3);
      const int c = (lane & 7) ^ aswz(r);
      p[i] = (piece < 8 ? a + (int64_t)r * lda : b + (int64_t)r * ldb) + c * 8;
    }
  }
  // rows r0 .. r0+63 into the tile pair at dst (a at dst, b at dst + 8 KiB)
  __device__ __forceinline__ void issue(int64_t offa, int64_t offb, GK_LDS char* dst, int wave) const {
#pragma unroll
    for (int i = 0; i < kPieces; ++i) {
      const int piece = wave * kPieces + i;
      glds16(p[i] + (piece < 8 ? offa : offb), dst + piece * 1024);
    }
  }
};

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

__device__ __forceinline__ float bf2f(short v) { return __uint_as_float((uint32_t)(uint16_t)v << 16); }

// x * s rounded back to bf16 (the pre-scaled resident operand)
__device__ __forceinline__ bf16x8 scale_bf16x8(const bf16x8& x, float s) {
  const uint32_t w[4] = {pack_bf16x2(bf2f(x[0]) * s, bf2f(x[1]) * s), pack_bf16x2(bf2f(x[2]) * s, bf2f(x[3]) * s),
                         pack_bf16x2(bf2f(x[4]) * s, bf2f(x[5]) * s), pack_bf16x2(bf2f(x[6]) * s, bf2f(x[7]) * s)};
  return __builtin_bit_cast(bf16x8, w);
}

__device__ __forceinline__ f32x4 splat4(float v) { return f32x4{v, v, v, v}; }

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
  // optional replay word (graph capture): the effective seed mixes it in, so
  // a replayed step draws a fresh mask while forward and backward of one
  // replay read the same word
  const uint32_t* seed_dev;
};

__device__ __forceinline__ uint32_t eff_seed(const AttnArgs& a) {
  if (a.seed_dev == nullptr) return a.seed;
  return hash_u32(__builtin_amdgcn_readfirstlane(*a.seed_dev), a.seed);
}

// ---------------------------------------------------------------------------
// forward: one workgroup = 4 waves x 32 queries of one (batch, head); K/V
// tiles of 64 keys in a 3-deep LDS ring
// ---------------------------------------------------------------------------
template <bool DROP>
__global__ void __launch_bounds__(64 * kAW, 2) attn_fwd_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(1024))) char smem[kStages * 2 * kTileB];
  const uint32_t seed = DROP ? eff_seed(a) : 0u;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, li = lane & 15, g = lane >> 4;
  const int T = a.T, H = a.H;
  const int nqb = T / kRows;
  const int blk = xcd_block();
  const int bh = blk / nqb, qb = blk - bh * nqb;
  const int b = bh / H, h = bh - b * H;
  const int64_t ld = 3LL * H * kHD;
  const uint16_t* base = a.qkv + (int64_t)b * T * ld;
  const int q0 = qb * kRows + wave * 32;
  GK_LDS char* lds = (GK_LDS char*)smem;
  DmaSrc dma;
  dma.init(base + (int64_t)(H + h) * kHD, ld, base + (int64_t)(2 * H + h) * kHD, ld, wave, lane);
  const int64_t tstep = kKT * ld;
  const int nt = T / kKT;

  bf16x8 qf[2][2];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      qf[qt][ks] = *reinterpret_cast<const bf16x8*>(base + h * kHD + (int64_t)(q0 + 16 * qt + li) * ld + 32 * ks + 8 * g);
  dma.issue(0, 0, lds, wave);
  if (nt > 1) dma.issue(tstep, tstep, lds + 2 * kTileB, wave);
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) qf[qt][ks] = scale_bf16x8(qf[qt][ks], a.sc);

  f32x4 o[2][4];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[qt][dt] = splat4(0.f);
  float m[2] = {0.f, 0.f}, l[2] = {0.f, 0.f};
  uint32_t hrow[2];   // pair-hash index of key 4g of tile 0
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) hrow[qt] = ((uint32_t)bh * T + q0 + 16 * qt + li) * (uint32_t)(T >> 1) + 2 * g;
  uint32_t toff[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) toff[dt] = tr_lane_off(lane, dt);
  const uint32_t lbase = lds_addr(smem);

  int cur = 0, pre = 2;   // ring slots of tile t and of tile t + 2
  for (int t = 0; t < nt; ++t) {
    wait_tile<kPieces>(t + 1 >= nt);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (t + 2 < nt) dma.issue((t + 2) * tstep, (t + 2) * tstep, lds + pre * 2 * kTileB, wave);
    const char* Ks = smem + cur * 2 * kTileB;

    // S^T - m (log2 units), the running max as the initial accumulator
    f32x4 s[2][4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      const bf16x8 k0 = *reinterpret_cast<const bf16x8*>(Ks + aoff(16 * kt + li, g));
      const bf16x8 k1 = *reinterpret_cast<const bf16x8*>(Ks + aoff(16 * kt + li, 4 + g));
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) s[qt][kt] = mfma(k1, qf[qt][1], mfma(k0, qf[qt][0], splat4(-m[qt])));
    }

#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      float mx = fmaxf(fmaxf(s[qt][0][0], s[qt][0][1]), fmaxf(s[qt][0][2], s[qt][0][3]));
#pragma unroll
      for (int kt = 1; kt < 4; ++kt)
        mx = fmaxf(mx, fmaxf(fmaxf(s[qt][kt][0], s[qt][kt][1]), fmaxf(s[qt][kt][2], s[qt][kt][3])));
      if (t == 0 || __ballot(mx > kLazy) != 0) {   // wave-uniform, rare after the first tile
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
          hh[0] = pair_hash(seed, pi);
          hh[1] = pair_hash(seed, pi + 1);
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

    const uint32_t vb = lbase + cur * 2 * kTileB + kTileB;
    cur = ring_next(cur);
    pre = ring_next(pre);
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
// tile S^T = c K Q^T - lse, dZ^T = V dO^T - delta', dS^T = P^T (dP^T - delta),
// dQ^T += K^T dS^T
// ---------------------------------------------------------------------------
template <bool DROP>
__global__ void __launch_bounds__(64 * kAW, 2) attn_bwd_dq_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(1024))) char smem[kStages * 2 * kTileB];
  const uint32_t seed = DROP ? eff_seed(a) : 0u;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, li = lane & 15, g = lane >> 4;
  const int T = a.T, H = a.H;
  const int nqb = T / kRows;
  const int blk = xcd_block();
  const int bh = blk / nqb, qb = blk - bh * nqb;
  const int b = bh / H, h = bh - b * H;
  const int64_t ld = 3LL * H * kHD, ldo = (int64_t)H * kHD;
  const uint16_t* base = a.qkv + (int64_t)b * T * ld;
  const int q0 = qb * kRows + wave * 32;
  GK_LDS char* lds = (GK_LDS char*)smem;
  DmaSrc dma;
  dma.init(base + (int64_t)(H + h) * kHD, ld, base + (int64_t)(2 * H + h) * kHD, ld, wave, lane);
  const int64_t tstep = kKT * ld;
  const int nt = T / kKT;

  bf16x8 qf[2][2], df[2][2], of[2][2];
  float nlse[2], del[2], ndel[2];
  uint32_t hrow[2];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int q = q0 + 16 * qt + li;
    const int64_t orow = ((int64_t)b * T + q) * ldo + h * kHD;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      qf[qt][ks] = *reinterpret_cast<const bf16x8*>(base + h * kHD + (int64_t)q * ld + 32 * ks + 8 * g);
      df[qt][ks] = *reinterpret_cast<const bf16x8*>(a.dout + orow + 32 * ks + 8 * g);
      of[qt][ks] = *reinterpret_cast<const bf16x8*>(a.out + orow + 32 * ks + 8 * g);
    }
    nlse[qt] = -a.lse[(int64_t)bh * T + q];
  }
  dma.issue(0, 0, lds, wave);
  if (nt > 1) dma.issue(tstep, tstep, lds + 2 * kTileB, wave);
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int q = q0 + 16 * qt + li;
    float dsum = 0.f;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      qf[qt][ks] = scale_bf16x8(qf[qt][ks], a.sc);
#pragma unroll
      for (int j = 0; j < 8; ++j) dsum = fmaf(bf2f(df[qt][ks][j]), bf2f(of[qt][ks][j]), dsum);
    }
    dsum += __shfl_xor(dsum, 16, 64);
    dsum += __shfl_xor(dsum, 32, 64);
    del[qt] = dsum;
    ndel[qt] = DROP ? -dsum / a.dscale : -dsum;
    if (g == 0) a.delta[(int64_t)bh * T + q] = dsum;
    hrow[qt] = ((uint32_t)bh * T + q) * (uint32_t)(T >> 1) + 2 * g;
  }

  f32x4 dq[2][4];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dq[qt][dt] = splat4(0.f);
  uint32_t toff[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) toff[dt] = tr_lane_off(lane, dt);
  const uint32_t lbase = lds_addr(smem);

  int cur = 0, pre = 2;   // ring slots of tile t and of tile t + 2
  for (int t = 0; t < nt; ++t) {
    // the delta stores follow tile 1's pieces: drain everything on the first tile
    wait_tile<kPieces>(t == 0 || t + 1 >= nt);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (t + 2 < nt) dma.issue((t + 2) * tstep, (t + 2) * tstep, lds + pre * 2 * kTileB, wave);
    const char* Ks = smem + cur * 2 * kTileB;
    const char* Vs = Ks + kTileB;

    f32x4 s[2][4], dz[2][4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      const bf16x8 k0 = *reinterpret_cast<const bf16x8*>(Ks + aoff(16 * kt + li, g));
      const bf16x8 k1 = *reinterpret_cast<const bf16x8*>(Ks + aoff(16 * kt + li, 4 + g));
      const bf16x8 v0 = *reinterpret_cast<const bf16x8*>(Vs + aoff(16 * kt + li, g));
      const bf16x8 v1 = *reinterpret_cast<const bf16x8*>(Vs + aoff(16 * kt + li, 4 + g));
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        s[qt][kt] = mfma(k1, qf[qt][1], mfma(k0, qf[qt][0], splat4(nlse[qt])));
        dz[qt][kt] = mfma(v1, df[qt][1], mfma(v0, df[qt][0], splat4(ndel[qt])));
      }
    }

#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        uint32_t hh[2];
        if (DROP) {
          const uint32_t pi = hrow[qt] + t * (kKT / 2) + 8 * kt;
          hh[0] = pair_hash(seed, pi);
          hh[1] = pair_hash(seed, pi + 1);
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

    const uint32_t kb = lbase + cur * 2 * kTileB;
    cur = ring_next(cur);
    pre = ring_next(pre);
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
// backward, dK / dV: one workgroup = 4 waves x 32 keys; K (pre-scaled) and V
// of the wave's keys stay in registers while query tiles of 64 (Q, dO, lse,
// delta) stream through LDS.  Per 32-query half: S = c Q K^T - lse,
// dZ = dO V^T - delta' (query on 4g + r), P, dS elementwise,
// dV^T += dO^T P, dK^T += Q^T dS.
// ---------------------------------------------------------------------------
constexpr int kKvBuf = 2 * kTileB + 512;   // Q tile, dO tile, lse[64], delta[64]

template <bool DROP>
__global__ void __launch_bounds__(64 * kAW, 2) attn_bwd_kv_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(1024))) char smem[kStages * kKvBuf];
  const uint32_t seed = DROP ? eff_seed(a) : 0u;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, li = lane & 15, g = lane >> 4;
  const int T = a.T, H = a.H;
  const int nkb = T / kRows;
  const int blk = xcd_block();
  const int bh = blk / nkb, kb = blk - bh * nkb;
  const int b = bh / H, h = bh - b * H;
  const int64_t ld = 3LL * H * kHD, ldo = (int64_t)H * kHD;
  const uint16_t* base = a.qkv + (int64_t)b * T * ld;
  const float* lsep = a.lse + (int64_t)bh * T;
  const float* delp = a.delta + (int64_t)bh * T;
  const int k0 = kb * kRows + wave * 32;
  GK_LDS char* lds = (GK_LDS char*)smem;
  DmaSrc dma;
  dma.init(base + (int64_t)h * kHD, ld, a.dout + (int64_t)b * T * ldo + (int64_t)h * kHD, ldo, wave, lane);

  auto stage = [&](int t, int buf) {
    GK_LDS char* dst = lds + buf * kKvBuf;
    dma.issue((int64_t)t * kKT * ld, (int64_t)t * kKT * ldo, dst, wave);
    if (wave < 2)
      __builtin_amdgcn_global_load_lds((wave ? delp : lsep) + t * kKT + lane, dst + 2 * kTileB + wave * 256, 4, 0, 0);
  };
  const int nt = T / kKT;

  bf16x8 kf[2][2], vf[2][2];
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int64_t row = (int64_t)(k0 + 16 * kt + li) * ld + 32 * ks + 8 * g;
      kf[kt][ks] = *reinterpret_cast<const bf16x8*>(base + (int64_t)(H + h) * kHD + row);
      vf[kt][ks] = *reinterpret_cast<const bf16x8*>(base + (int64_t)(2 * H + h) * kHD + row);
    }
  stage(0, 0);
  if (nt > 1) stage(1, 1);
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) kf[kt][ks] = scale_bf16x8(kf[kt][ks], a.sc);
  f32x4 dv[2][4], dk[2][4];
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dv[kt][dt] = dk[kt][dt] = splat4(0.f);
  uint32_t toff[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) toff[dt] = tr_lane_off(lane, dt);
  const uint32_t lbase = lds_addr(smem);
  // dropout: this lane hashes queries 2 (li & 1) + {0, 1} of every 4 for its
  // key pair, the neighbour lane the other two (DPP swap); key & 1 picks the half
  const uint32_t hkey = (uint32_t)bh * T * (uint32_t)(T >> 1) + ((k0 + li) >> 1);
  const uint32_t hsh = 16u * (uint32_t)(li & 1);
  const int rown = 2 * (li & 1);

  int cur = 0, pre = 2;   // ring slots of tile t and of tile t + 2
  for (int t = 0; t < nt; ++t) {
    if (wave < 2) wait_tile<kPieces + 1>(t + 1 >= nt);   // waves 0 / 1 also stage lse / delta
    else wait_tile<kPieces>(t + 1 >= nt);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (t + 2 < nt) stage(t + 2, pre);
    const char* Qs = smem + cur * kKvBuf;
    const char* Ds = Qs + kTileB;
    const float* Ls = reinterpret_cast<const float*>(Qs + 2 * kTileB);
    const uint32_t qb = lbase + cur * kKvBuf;
    cur = ring_next(cur);
    pre = ring_next(pre);

#pragma unroll
    for (int half = 0; half < 2; ++half) {
      f32x4 s[2][2], dz[2][2];   // [qt][kt]
      f32x4 del4[2];
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        const int qr = 32 * half + 16 * qt + 4 * g;   // tile row of r = 0
        const f32x4 nl = -*reinterpret_cast<const f32x4*>(Ls + qr);
        del4[qt] = *reinterpret_cast<const f32x4*>(Ls + 64 + qr);
        const f32x4 nd = DROP ? -del4[qt] * (1.f / a.dscale) : -del4[qt];
        const int row = 32 * half + 16 * qt + li;
        const bf16x8 qa0 = *reinterpret_cast<const bf16x8*>(Qs + aoff(row, g));
        const bf16x8 qa1 = *reinterpret_cast<const bf16x8*>(Qs + aoff(row, 4 + g));
        const bf16x8 da0 = *reinterpret_cast<const bf16x8*>(Ds + aoff(row, g));
        const bf16x8 da1 = *reinterpret_cast<const bf16x8*>(Ds + aoff(row, 4 + g));
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          s[qt][kt] = mfma(qa1, kf[kt][1], mfma(qa0, kf[kt][0], nl));
          dz[qt][kt] = mfma(da1, vf[kt][1], mfma(da0, vf[kt][0], nd));
        }
      }
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        const int qr = 32 * half + 16 * qt + 4 * g;
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          uint32_t hq[4];
          if (DROP) {
            const uint32_t pi = hkey + (uint32_t)(t * kKT + qr + rown) * (uint32_t)(T >> 1) + 8 * kt;
            const uint32_t m0 = pair_hash(seed, pi), m1 = pair_hash(seed, pi + (uint32_t)(T >> 1));
            const uint32_t o0 = (uint32_t)__builtin_amdgcn_mov_dpp((int)m0, 0xB1, 0xF, 0xF, false);
            const uint32_t o1 = (uint32_t)__builtin_amdgcn_mov_dpp((int)m1, 0xB1, 0xF, 0xF, false);
            const bool odd = li & 1;
            hq[0] = odd ? o0 : m0;
            hq[1] = odd ? o1 : m1;
            hq[2] = odd ? m0 : o0;
            hq[3] = odd ? m1 : o1;
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float p = fexp2(s[qt][kt][r]);
            float z = p, dd = dz[qt][kt][r];   // dP - delta (no dropout)
            if (DROP) {
              const bool k = __builtin_amdgcn_ubfe(hq[r], hsh, 16) >= a.thr;
              z = k ? p * a.dscale : 0.f;
              dd = k ? dd * a.dscale : -del4[qt][r];
            }
            s[qt][kt][r] = z;
            dz[qt][kt][r] = p * dd;
          }
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

// keep mask [B*H][T][T] as bytes, from the same pair hashes
__global__ void attn_dropout_mask_kernel(uint8_t* __restrict__ mask, int64_t npairs, AttnArgs a, uint32_t thr) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t seed = eff_seed(a);
  if (i < npairs) {
    const uint32_t hv = pair_hash(seed, (uint32_t)i);
    mask[2 * i] = (hv & 0xffffu) >= thr ? 1 : 0;
    mask[2 * i + 1] = (hv >> 16) >= thr ? 1 : 0;
  }
}

AttnArgs make_args(int T, int H, float p, uint32_t seed, const uint32_t* seed_dev) {
  AttnArgs a{};
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

}  // namespace

bool attn_supported(int T, int D) { return D == kHD && T >= kRows && T % kRows == 0; }

void attn_fwd(const void* qkv, void* out, float* lse, int B, int T, int H, float p, uint32_t seed,
              const uint32_t* seed_dev, hipStream_t stream) {
  AttnArgs a = make_args(T, H, p, seed, seed_dev);
  a.qkv = static_cast<const uint16_t*>(qkv);
  a.o = static_cast<uint16_t*>(out);
  a.lse = lse;
  const dim3 grid((unsigned)(B * H * (T / kRows)));
  if (a.thr) hipLaunchKernelGGL(attn_fwd_kernel<true>, grid, dim3(64 * kAW), 0, stream, a);
  else hipLaunchKernelGGL(attn_fwd_kernel<false>, grid, dim3(64 * kAW), 0, stream, a);
}

void attn_bwd(const void* qkv, const void* out, const void* dout, const float* lse, float* delta, void* dqkv, int B,
              int T, int H, float p, uint32_t seed, const uint32_t* seed_dev, hipStream_t stream) {
  AttnArgs a = make_args(T, H, p, seed, seed_dev);
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

void attn_dropout_mask(uint8_t* mask, int B, int H, int T, float p, uint32_t seed, const uint32_t* seed_dev,
                       hipStream_t stream) {
  const AttnArgs a = make_args(T, H, p, seed, seed_dev);
  const int64_t npairs = (int64_t)B * H * T * T / 2;
  hipLaunchKernelGGL(attn_dropout_mask_kernel, dim3((unsigned)((npairs + 255) / 256)), dim3(256), 0, stream, mask,
                     npairs, a, a.thr);
}

}  // namespace gk
