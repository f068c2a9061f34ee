// Fused batch-norm (training) + residual add + ReLU for channels-last (NHWC)
// activations on gfx950.
//
// ResNet-style blocks spend ~1/3 of a training step in MIOpen's NHWC batch
// norm plus separate ReLU / residual-add passes (profiles/r01_*).  Here one
// BN layer is:
//   forward : stats (grid)  -> per-block per-channel sum / sum^2 (fp32)
//             finalize      -> mean, invstd, scale, shift, running stats
//             apply (grid)  -> y = act(x*scale + shift [+ residual])
//   backward: reduce (grid) -> sum dz, sum dz*xhat   (dz = dy * relu mask)
//             finalize      -> dgamma, dbeta
//             apply (grid)  -> dx = scale*(dz - dbeta/M - xhat*dgamma/M),
//                              dresidual = dz
// so the ReLU mask, the residual gradient and the normalisation share the
// same streaming passes.  The forward writes the ReLU mask as 1 bit per
// element (1 byte per 16-byte vector); the backward reads it instead of y,
// cutting the backward's read traffic by a third.  Activations are viewed as [M = N*H*W, C]; each
// thread owns 16 contiguous bytes of channels (8 bf16 / 4 fp32) and walks
// rows, so every wave reads whole 1-KiB contiguous runs.  Statistics are
// accumulated in fp32 per thread and combined in fp64.
#include <hip/hip_runtime.h>

#include <atomic>

#include "common.h"
#include "gk_kernels.h"

namespace gk {
namespace {

constexpr size_t kFinStateFlagsOffset = 16;   // per-layer state: [u64 ticket | pad | u32 flags[ngroups]]

__device__ __forceinline__ float bf16_to_f32(uint16_t h) { return __uint_as_float(((uint32_t)h) << 16); }
__device__ __forceinline__ uint16_t f32_to_bf16(float f);
__device__ __forceinline__ float round_to_bf16(float f) { return bf16_to_f32(f32_to_bf16(f)); }
__device__ __forceinline__ void store_elem(float* p, float v) { *p = v; }
__device__ __forceinline__ void store_elem(uint16_t* p, float v) { *p = f32_to_bf16(v); }

__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x7fffffu)) return (uint16_t)((u >> 16) | 0x40);  // NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

// Streaming 16-byte accesses of the BN passes.  The activations (up to 1.6 GB
// per tensor at ResNet-50 bs512 fp32) are touched once per pass and do not fit
// the 4 MB L2 / 256 MB MALL, so loads and stores are non-temporal.  Measured
// (bench/bn_probe.py, every ResNet-50 bs512 BN shape and pass summed,
// profiles/r03_bn_nontemporal.txt): fp32 14.24 -> 13.63 ms, bf16 7.67 -> 7.32
// ms (stores only: 13.93 / 7.30).  -DGK_BN_NT_LD=0 / -DGK_BN_NT_ST=0 restore
// plain accesses (ops/build.py GKSGD_VARIANT A/B builds).
#ifndef GK_BN_NT_LD
#define GK_BN_NT_LD 1
#endif
#ifndef GK_BN_NT_ST
#define GK_BN_NT_ST 1
#endif
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld16(const uint4* p) {
  if (GK_BN_NT_LD) {
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    return make_uint4(v[0], v[1], v[2], v[3]);
  }
  return *p;
}
__device__ __forceinline__ void st16(uint4* p, uint4 v) {
  if (GK_BN_NT_ST) __builtin_nontemporal_store(u32x4{v.x, v.y, v.z, v.w}, reinterpret_cast<u32x4*>(p));
  else *p = v;
}

// 16-byte vector of VEC elements of T, converted to/from fp32.
template <typename T>
struct Vec;

template <>
struct Vec<uint16_t> {  // bf16
  static constexpr int N = 8;
  __device__ static void load(const uint16_t* p, float* v) {
    const uint4 u = ld16(reinterpret_cast<const uint4*>(p));
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(w[i] << 16);
      v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
  __device__ static void store(uint16_t* p, const float* v) {
    // v_cvt_pk_bf16_f32: round-to-nearest-even, NaN stays NaN (same values as f32_to_bf16)
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      w[i] = __builtin_bit_cast(uint32_t, __builtin_convertvector(
                 (float __attribute__((ext_vector_type(2)))){v[2 * i], v[2 * i + 1]}, __bf16 __attribute__((ext_vector_type(2)))));
    st16(reinterpret_cast<uint4*>(p), make_uint4(w[0], w[1], w[2], w[3]));
  }
};

template <>
struct Vec<float> {
  static constexpr int N = 4;
  __device__ static void load(const float* p, float* v) {
    const uint4 u = ld16(reinterpret_cast<const uint4*>(p));
    v[0] = __uint_as_float(u.x); v[1] = __uint_as_float(u.y); v[2] = __uint_as_float(u.z); v[3] = __uint_as_float(u.w);
  }
  __device__ static void store(float* p, const float* v) {
    st16(reinterpret_cast<uint4*>(p), make_uint4(__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]),
                                                 __float_as_uint(v[3])));
  }
};

// Streaming row loop of the BN passes: a thread walks rows r, r + rl, ... < r1
// of its 16-byte channel vector; U rows are loaded before any is used.
// Measured (bench/bn_probe.py, profiles/r02_bn_probe_unroll.txt): U = 4 and
// 2048-4096 workgroups are SLOWER than U = 1 at 1024 workgroups on every
// ResNet-50 shape (block-output backward 1151 -> 1285 us at 56x56x256), so the
// passes run U = 1; all of them sit at 4.5-5.8 TB/s either way.
template <int U, typename Row, typename L, typename F>
__device__ __forceinline__ void stream_rows(int64_t r, int64_t r1, int rl, L&& load, F&& use) {
  for (; r + (int64_t)(U - 1) * rl < r1; r += (int64_t)U * rl) {
    Row v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) load(v[u], r + (int64_t)u * rl);
#pragma unroll
    for (int u = 0; u < U; ++u) use(v[u], r + (int64_t)u * rl);
  }
  for (; r < r1; r += rl) {
    Row v;
    load(v, r);
    use(v, r);
  }
}

// rows in flight per thread in the streaming passes (stream_rows)
#ifndef GK_BN_UNROLL
#define GK_BN_UNROLL 1
#endif
constexpr int kBnUnroll = GK_BN_UNROLL;

struct Geo {
  int tpr;      // threads across the channel tile
  int rl;       // row lanes per block
  int ct;       // channels per tile
  int gx;       // channel tiles
  int gy;       // row chunks
  int64_t rows_per_block;
};

template <typename T>
Geo make_geo(int64_t M, int C, int target_blocks) {
  constexpr int V = Vec<T>::N;
  Geo g;
  int cv = C / V;
  g.tpr = cv < 64 ? cv : 64;
  while (cv % g.tpr) --g.tpr;  // tpr divides C/V
  g.ct = g.tpr * V;
  g.rl = kBlock / g.tpr;
  g.gx = C / g.ct;
  int64_t gy = (target_blocks + g.gx - 1) / g.gx;
  const int64_t max_gy = (M + g.rl - 1) / g.rl;
  if (gy > max_gy) gy = max_gy;
  if (gy < 1) gy = 1;
  g.gy = (int)gy;
  g.rows_per_block = (M + g.gy - 1) / g.gy;
  return g;
}

// ---------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------
template <typename T, int U = kBnUnroll>
__global__ __launch_bounds__(kBlock) void bn_stats_kernel(const T* __restrict__ x, int64_t M, int C, Geo g,
                                                          float* __restrict__ psum, float* __restrict__ psq) {
  constexpr int V = Vec<T>::N;
  const int tc = threadIdx.x % g.tpr;
  const int lane_r = threadIdx.x / g.tpr;
  const int c0 = blockIdx.x * g.ct + tc * V;
  const int64_t r0 = (int64_t)blockIdx.y * g.rows_per_block;
  int64_t r1 = r0 + g.rows_per_block;
  if (r1 > M) r1 = M;
  float s[V], q[V];
#pragma unroll
  for (int i = 0; i < V; ++i) s[i] = q[i] = 0.f;
  struct Row { float v[V]; };
  stream_rows<U, Row>(
      lane_r < g.rl ? r0 + lane_r : r1, r1, g.rl, [&](Row& w, int64_t r) { Vec<T>::load(x + r * C + c0, w.v); },
      [&](const Row& w, int64_t) {
#pragma unroll
        for (int i = 0; i < V; ++i) {
          s[i] += w.v[i];
          q[i] = fmaf(w.v[i], w.v[i], q[i]);
        }
      });
  __shared__ float sh[2][kBlock * 8];
#pragma unroll
  for (int i = 0; i < V; ++i) {
    sh[0][threadIdx.x * V + i] = s[i];
    sh[1][threadIdx.x * V + i] = q[i];
  }
  __syncthreads();
  // reduce over row lanes: thread t < ct handles channel (tile-local) t
  for (int cl = threadIdx.x; cl < g.ct; cl += kBlock) {
    const int t = cl / V, i = cl % V;
    float a = 0.f, b = 0.f;
    for (int l = 0; l < g.rl; ++l) {
      a += sh[0][(l * g.tpr + t) * V + i];
      b += sh[1][(l * g.tpr + t) * V + i];
    }
    const int c = blockIdx.x * g.ct + cl;
    psum[(int64_t)blockIdx.y * C + c] = a;
    psq[(int64_t)blockIdx.y * C + c] = b;
  }
}

// Per-channel reduction of the [gy][C] partials: a workgroup owns kFinC
// channels; its 256 threads split the gy rows kFinParts ways and keep 8 loads
// in flight per thread (the partials are L2-resident; an un-pipelined loop is
// latency-bound), then combine the partial sums in fp64 through LDS.
constexpr int kFinC = 16;
constexpr int kFinParts = kBlock / kFinC;

__device__ __forceinline__ void reduce_partials2(const float* __restrict__ pa, const float* __restrict__ pb, int gy,
                                                 int C, double* out_a, double* out_b, bool* owner, int* c_out,
                                                 int grp) {
  __shared__ double sh[2][kFinParts][kFinC];
  const int cl = threadIdx.x % kFinC;
  const int part = threadIdx.x / kFinC;
  const int c = grp * kFinC + cl;
  double a = 0.0, b = 0.0;
  if (c < C) {
    int j = part;
    for (; j + 7 * kFinParts < gy; j += 8 * kFinParts) {
      float va[8], vb[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        va[u] = pa[(int64_t)(j + u * kFinParts) * C + c];
        vb[u] = pb[(int64_t)(j + u * kFinParts) * C + c];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        a += va[u];
        b += vb[u];
      }
    }
    for (; j < gy; j += kFinParts) {
      a += pa[(int64_t)j * C + c];
      b += pb[(int64_t)j * C + c];
    }
  }
  sh[0][part][cl] = a;
  sh[1][part][cl] = b;
  __syncthreads();
  *owner = part == 0 && c < C;
  *c_out = c;
  if (part == 0) {
    double sa = 0.0, sb = 0.0;
#pragma unroll
    for (int p = 0; p < kFinParts; ++p) {
      sa += sh[0][p][cl];
      sb += sh[1][p][cl];
    }
    *out_a = sa;
    *out_b = sb;
  }
}

// Device-coherent (agent-scope, `sc1`) accesses of the in-launch finalize
// hand-off below: they bypass the per-XCD L2s, so no L2 write-back /
// invalidate fence is needed (MI355X_MICROARCH.md, inter-workgroup
// visibility: all-`sc1` stores and loads, drained stores, one flag per
// producing workgroup).
template <typename T>
__device__ __forceinline__ void st_dev(T* p, T v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
template <typename T>
__device__ __forceinline__ T ld_dev(const T* p) {
  return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// pipelined `sc1` loads (an agent-scope atomic load waits for each one)
__device__ __forceinline__ float ld_coh_f32(const float* base, int idx) {
  const auto r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, 0x7fffffff, 0x00020000);
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, idx * 4, 0, 16 /* SC1 */));
}
template <bool COH>
__device__ __forceinline__ void put(float* p, float v) {
  if (COH) st_dev(p, v);
  else *p = v;
}

struct FwdFin {   // forward finalize: partials -> mean, invstd, scale, shift, running stats
  const float* psum;
  const float* psq;
  int gy;
  const float* w;
  const float* b;
  float eps, momentum;
  float* run_mean;
  float* run_var;
  float* save_mean;
  float* save_invstd;
  float* scale;
  float* shift;
  int64_t* nbt;
};

// channel group `grp` (kFinC channels) of the forward finalize; COH: the
// outputs are read back inside the same launch (in-launch finalize)
template <bool COH>
__device__ __forceinline__ void fwd_fin_group(const FwdFin& f, int64_t M, int C, int grp) {
  double s = 0.0, q = 0.0;
  bool owner;
  int c;
  reduce_partials2(f.psum, f.psq, f.gy, C, &s, &q, &owner, &c, grp);
  if (f.nbt && grp == 0 && threadIdx.x == 0) *f.nbt += 1;  // BatchNorm num_batches_tracked
  if (!owner) return;
  const double mean = s / (double)M;
  double var = q / (double)M - mean * mean;
  if (var < 0.0) var = 0.0;
  const float invstd = (float)(1.0 / sqrt(var + (double)f.eps));
  const float gam = f.w ? f.w[c] : 1.f;
  const float bet = f.b ? f.b[c] : 0.f;
  f.save_mean[c] = (float)mean;
  f.save_invstd[c] = invstd;
  put<COH>(f.scale + c, gam * invstd);
  put<COH>(f.shift + c, bet - (float)mean * gam * invstd);
  if (f.run_mean) {
    const double unbiased = M > 1 ? var * (double)M / (double)(M - 1) : var;
    f.run_mean[c] = (1.f - f.momentum) * f.run_mean[c] + f.momentum * (float)mean;
    f.run_var[c] = (1.f - f.momentum) * f.run_var[c] + f.momentum * (float)unbiased;
  }
}

__global__ __launch_bounds__(kBlock) void bn_finalize_kernel(const float* __restrict__ psum,
                                                             const float* __restrict__ psq, int gy, int64_t M, int C,
                                                             const float* __restrict__ w, const float* __restrict__ b,
                                                             float eps, float momentum, float* __restrict__ run_mean,
                                                             float* __restrict__ run_var, float* __restrict__ save_mean,
                                                             float* __restrict__ save_invstd, float* __restrict__ scale,
                                                             float* __restrict__ shift, int64_t* __restrict__ nbt) {
  const FwdFin f{psum, psq, gy, w, b, eps, momentum, run_mean, run_var, save_mean, save_invstd, scale, shift, nbt};
  fwd_fin_group<false>(f, M, C, blockIdx.x);
}

// In-launch finalize (the separate 1-row finalize launch folded into the
// apply pass that consumes it): every workgroup draws a ticket; tickets
// 0 .. ngroups-1 run the finalize of one kFinC-channel group and publish a
// flag = epoch (all outputs stored `sc1` and drained first); every workgroup
// then waits for the flags of the groups its channel tile covers and reads
// the finalized values with `sc1` loads.  A leader waits only after its own
// flag is out and a waiter only for groups whose leaders drew their ticket
// -- i.e. are running -- so no workgroup waits on one that is not resident.
// The ticket counter is reset by the holder of the last ticket; the flags
// are per-layer persistent (ops/bn.py) and `epoch` is unique per launch
// (host counter), so they need no reset.  Not used under graph capture
// (the epoch would be frozen into the replays).
struct FinSync {
  unsigned long long* ticket;
  uint32_t* flags;
  uint32_t epoch;
  uint32_t nblocks;
  int ngroups;
};

template <typename F>
__device__ __forceinline__ void fin_prologue(const FinSync& fs, int g0, int g1, F&& finalize_group) {
  __shared__ uint32_t s_ticket;
  if (threadIdx.x == 0) {
    const unsigned long long t = __hip_atomic_fetch_add(fs.ticket, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == (unsigned long long)fs.nblocks - 1ull) st_dev(fs.ticket, 0ull);   // every ticket of this launch is out
    s_ticket = (uint32_t)t;
  }
  __syncthreads();
  const uint32_t t = s_ticket;
  if (t < (uint32_t)fs.ngroups) {
    finalize_group((int)t);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this thread's sc1 stores completed
    __syncthreads();
    if (threadIdx.x == 0) st_dev(fs.flags + t, fs.epoch);
  }
  const int gi = g0 + (int)threadIdx.x;
  if (gi < g1) {
    uint32_t spins = 0;
    while (ld_dev(fs.flags + gi) != fs.epoch && ++spins < (1u << 24)) __builtin_amdgcn_s_sleep(1);
  }
  __syncthreads();
}

// RBN: the residual is itself a batch-normalised tensor whose apply pass was
// deferred to here (ResNet downsample shortcut, ops/bn.py _BNDeferFn):
// res = r * rscale + rshift is formed on load, so the shortcut BN output is
// never written and read back (one streaming pass less per downsample block).
template <typename T, bool RELU, bool RES, bool FIN = false, int U = kBnUnroll, bool RBN = false>
__global__ __launch_bounds__(kBlock) void bn_apply_kernel(const T* __restrict__ x, const T* __restrict__ res,
                                                          T* __restrict__ y, uint8_t* __restrict__ mask, int64_t M,
                                                          int C, Geo g, const float* __restrict__ scale,
                                                          const float* __restrict__ shift, FinSync fs = FinSync{},
                                                          FwdFin ff = FwdFin{}, const float* __restrict__ rscale = nullptr,
                                                          const float* __restrict__ rshift = nullptr) {
  constexpr int V = Vec<T>::N;
  const int tc = threadIdx.x % g.tpr;
  const int lane_r = threadIdx.x / g.tpr;
  const int c0 = blockIdx.x * g.ct + tc * V;
  float sc[V], sf[V];
  if (FIN) {
    fin_prologue(fs, (blockIdx.x * g.ct) / kFinC, ((blockIdx.x + 1) * g.ct + kFinC - 1) / kFinC,
                 [&](int grp) { fwd_fin_group<true>(ff, M, C, grp); });
#pragma unroll
    for (int i = 0; i < V; ++i) { sc[i] = ld_coh_f32(scale, c0 + i); sf[i] = ld_coh_f32(shift, c0 + i); }
  } else {
#pragma unroll
    for (int i = 0; i < V; ++i) { sc[i] = scale[c0 + i]; sf[i] = shift[c0 + i]; }
  }
  float rsc[RBN ? V : 1], rsf[RBN ? V : 1];
  if constexpr (RBN) {
#pragma unroll
    for (int i = 0; i < V; ++i) { rsc[i] = rscale[c0 + i]; rsf[i] = rshift[c0 + i]; }
  }
  const int64_t r0 = (int64_t)blockIdx.y * g.rows_per_block;
  int64_t r1 = r0 + g.rows_per_block;
  if (r1 > M) r1 = M;
  struct Row { float v[V], rv[RES ? V : 1]; };
  stream_rows<U, Row>(
      lane_r < g.rl ? r0 + lane_r : r1, r1, g.rl,
      [&](Row& w, int64_t r) {
        Vec<T>::load(x + r * C + c0, w.v);
        if (RES) Vec<T>::load(res + r * C + c0, w.rv);
      },
      [&](const Row& w, int64_t r) {
        float o[V];
        uint32_t bits = 0;
#pragma unroll
        for (int i = 0; i < V; ++i) {
          float t = fmaf(w.v[i], sc[i], sf[i]);
          if constexpr (RBN) t += fmaf(w.rv[i], rsc[i], rsf[i]);
          else if (RES) t += w.rv[i];
          if (RELU) {
            bits |= (t > 0.f ? 1u : 0u) << i;
            t = fmaxf(t, 0.f);
          }
          o[i] = t;
        }
        Vec<T>::store(y + r * C + c0, o);
        if (RELU) mask[r * (C / V) + c0 / V] = (uint8_t)bits;
      });
}

__device__ __forceinline__ float round_bf16(float f) { return __uint_as_float((uint32_t)f32_to_bf16(f) << 16); }

// Fused BN apply + ReLU + max-pool (the ResNet stem): one thread per 16-byte
// channel vector of one OUTPUT pixel walks its k x k window, normalises each
// input on the fly and keeps the max of the (dtype-rounded) pre-ReLU values.
// max(relu(z)) == relu(max(z)), so the ReLU needs no mask of its own: the
// window position of the max is stored as one byte per output element
// (0xff when the max is <= 0, i.e. the ReLU blocks the gradient).  The
// full-resolution BN output is never written.  Window scan order and the
// strict '>' (first max wins, NaN propagates) match at::max_pool2d.
// KK > 0: compile-time k x k window whose KK*KK loads are all issued before
// any is used (out-of-image taps read the always-valid window centre and are
// skipped); the runtime loop waits for each tap's load in turn.
template <typename T, int KK = 0>
__global__ __launch_bounds__(kBlock) void bn_relu_pool_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                              uint8_t* __restrict__ amax, int64_t P, int C, PoolGeo pg,
                                                              const float* __restrict__ scale,
                                                              const float* __restrict__ shift) {
  constexpr int V = Vec<T>::N;
  const int cv = C / V;
  const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (t >= P * cv) return;
  const int64_t op = t / cv;
  const int c0 = (int)(t - op * cv) * V;
  const int64_t ohw = (int64_t)pg.OH * pg.OW;
  const int64_t n = op / ohw;
  const int rem = (int)(op - n * ohw);
  const int oh = rem / pg.OW, ow = rem - (rem / pg.OW) * pg.OW;
  float sc[V], sf[V], m[V];
  uint32_t idx[V];
#pragma unroll
  for (int i = 0; i < V; ++i) {
    sc[i] = scale[c0 + i];
    sf[i] = shift[c0 + i];
    m[i] = -INFINITY;
    idx[i] = 0xffu;
  }
  if constexpr (KK > 0) {
    const int hc = oh * pg.s - pg.p + KK / 2, wc = ow * pg.s - pg.p + KK / 2;   // centre (requires p == KK / 2)
    float v[KK * KK][V];
    bool ok[KK * KK];
#pragma unroll
    for (int q = 0; q < KK * KK; ++q) {
      const int ih = hc - KK / 2 + q / KK, iw = wc - KK / 2 + q % KK;
      ok[q] = ih >= 0 && ih < pg.H && iw >= 0 && iw < pg.W;
      Vec<T>::load(x + ((n * pg.H + (ok[q] ? ih : hc)) * pg.W + (ok[q] ? iw : wc)) * C + c0, v[q]);
    }
#pragma unroll
    for (int q = 0; q < KK * KK; ++q) {
      if (!ok[q]) continue;
#pragma unroll
      for (int i = 0; i < V; ++i) {
        float z = fmaf(v[q][i], sc[i], sf[i]);
        if (sizeof(T) == 2) z = round_bf16(z);
        if (z > m[i] || z != z) {
          m[i] = z;
          idx[i] = (uint32_t)q;
        }
      }
    }
  } else {
    for (int kh = 0; kh < pg.k; ++kh) {
      const int ih = oh * pg.s - pg.p + kh;
      if (ih < 0 || ih >= pg.H) continue;
      for (int kw = 0; kw < pg.k; ++kw) {
        const int iw = ow * pg.s - pg.p + kw;
        if (iw < 0 || iw >= pg.W) continue;
        float v[V];
        Vec<T>::load(x + ((n * pg.H + ih) * pg.W + iw) * C + c0, v);
        const uint32_t pos = (uint32_t)(kh * pg.k + kw);
#pragma unroll
        for (int i = 0; i < V; ++i) {
          float z = fmaf(v[i], sc[i], sf[i]);
          if (sizeof(T) == 2) z = round_bf16(z);
          if (z > m[i] || z != z) {
            m[i] = z;
            idx[i] = pos;
          }
        }
      }
    }
  }
  float o[V];
  uint32_t packed[2] = {0u, 0u};
#pragma unroll
  for (int i = 0; i < V; ++i) {
    o[i] = m[i] > 0.f ? m[i] : (m[i] != m[i] ? m[i] : 0.f);
    const uint32_t b = m[i] > 0.f ? idx[i] : 0xffu;
    packed[i / 4] |= b << (8 * (i % 4));
  }
  Vec<T>::store(y + op * C + c0, o);
  if (V == 8)
    *reinterpret_cast<uint2*>(amax + op * C + c0) = make_uint2(packed[0], packed[1]);
  else
    *reinterpret_cast<uint32_t*>(amax + op * C + c0) = packed[0];
}

// ---------------------------------------------------------------------------
// backward
//
// The upstream gradient dz of the BN output is produced by a "source":
//   DyPlain: dy (optionally gated by the forward's 1-bit ReLU mask);
//   DyPool : gathered from the max-pool output gradient -- input pixel (h, w)
//            receives dy_pool[oh, ow] from every window whose stored argmax is
//            (h, w); the full-resolution pool gradient is never materialised.
// ---------------------------------------------------------------------------
//   TWIN   : the BN output was consumed twice (ResNet: next block's conv1 and
//            its residual / downsample path); the two gradients dy + dy2 are
//            summed on load instead of by a separate add kernel.
template <typename T, bool RELU, bool TWIN>
struct DyPlain {
  const T* dy;
  const T* dy2;
  const uint8_t* mask;
  __device__ __forceinline__ void load(int64_t r, int C, int c0, float* d) const {
    constexpr int V = Vec<T>::N;
    Vec<T>::load(dy + r * C + c0, d);
    if (TWIN) {
      float e[V];
      Vec<T>::load(dy2 + r * C + c0, e);
#pragma unroll
      for (int i = 0; i < V; ++i) d[i] += e[i];
    }
    if (RELU) {
      const uint32_t bits = (uint32_t)mask[r * (C / V) + c0 / V];
#pragma unroll
      for (int i = 0; i < V; ++i) d[i] = ((bits >> i) & 1u) ? d[i] : 0.f;
    }
  }
};

// WM = 2: at most 2 windows per dimension cover an input pixel (k <= 2s, e.g.
// the 3x3/s2 stem pool): the <= 4 candidate windows are fixed, so all their
// argmax bytes and gradient vectors are loaded up front (independent loads in
// flight) and matched afterwards.  WM = 0: generic k, s (runtime loops).
template <typename T, bool TWIN, int WM>
struct DyPool {
  const T* dy;          // [N, OH, OW, C]
  const T* dy2;         // optional second consumer's gradient, same shape
  const uint8_t* amax;  // [N, OH, OW, C]
  PoolGeo pg;

  __device__ __forceinline__ void load_amax(int64_t o, uint32_t* a) const {
    constexpr int V = Vec<T>::N;
    if (V == 8) {
      const uint2 u = *reinterpret_cast<const uint2*>(amax + o);
      a[0] = u.x;
      a[1] = u.y;
    } else {
      a[0] = *reinterpret_cast<const uint32_t*>(amax + o);
      a[1] = 0xffffffffu;
    }
  }
  __device__ __forceinline__ void load_g(int64_t o, float* g) const {
    constexpr int V = Vec<T>::N;
    Vec<T>::load(dy + o, g);
    if (TWIN) {
      float e[V];
      Vec<T>::load(dy2 + o, e);
#pragma unroll
      for (int i = 0; i < V; ++i) g[i] += e[i];
    }
  }

  __device__ __forceinline__ void load(int64_t r, int C, int c0, float* d) const {
    constexpr int V = Vec<T>::N;
#pragma unroll
    for (int i = 0; i < V; ++i) d[i] = 0.f;
    const uint32_t hw = (uint32_t)(pg.H * pg.W);
    const uint32_t ru = (uint32_t)r;  // M < 2^32 (host check)
    const uint32_t n = ru / hw;
    const int rem = (int)(ru - n * hw);
    const int ih = rem / pg.W, iw = rem - (rem / pg.W) * pg.W;
    const int ah = ih + pg.p, aw = iw + pg.p;
    int oh0 = ah - pg.k + 1;
    oh0 = oh0 <= 0 ? 0 : (oh0 + pg.s - 1) / pg.s;
    int oh1 = ah / pg.s;
    if (oh1 > pg.OH - 1) oh1 = pg.OH - 1;
    int ow0 = aw - pg.k + 1;
    ow0 = ow0 <= 0 ? 0 : (ow0 + pg.s - 1) / pg.s;
    int ow1 = aw / pg.s;
    if (ow1 > pg.OW - 1) ow1 = pg.OW - 1;
    const int64_t nbase = (int64_t)n * pg.OH;
    if (WM == 2) {
      uint32_t a[4][2];
      float g[4][V];
      uint32_t pos[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int oh = oh1 - 1 + (j >> 1), ow = ow1 - 1 + (j & 1);
        const bool valid = oh >= oh0 && ow >= ow0;
        pos[j] = (uint32_t)((ah - oh * pg.s) * pg.k + (aw - ow * pg.s));
        a[j][0] = a[j][1] = 0xffffffffu;
#pragma unroll
        for (int i = 0; i < V; ++i) g[j][i] = 0.f;
        if (valid) {
          const int64_t o = ((nbase + oh) * pg.OW + ow) * C + c0;
          load_amax(o, a[j]);
          load_g(o, g[j]);
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < V; ++i)
          if (((a[j][i / 4] >> (8 * (i % 4))) & 0xffu) == pos[j]) d[i] += g[j][i];
      return;
    }
    for (int oh = oh0; oh <= oh1; ++oh) {
      for (int ow = ow0; ow <= ow1; ++ow) {
        const uint32_t p = (uint32_t)((ah - oh * pg.s) * pg.k + (aw - ow * pg.s));
        const int64_t o = ((nbase + oh) * pg.OW + ow) * C + c0;
        uint32_t a[2];
        load_amax(o, a);
        bool any = false;
#pragma unroll
        for (int i = 0; i < V; ++i) any |= ((a[i / 4] >> (8 * (i % 4))) & 0xffu) == p;
        if (!any) continue;
        float g[V];
        load_g(o, g);
#pragma unroll
        for (int i = 0; i < V; ++i)
          if (((a[i / 4] >> (8 * (i % 4))) & 0xffu) == p) d[i] += g[i];
      }
    }
  }
};

// WDZ: also store dz (the gated, twin-summed gradient -- the residual branch's
// gradient) so the apply pass reads one tensor instead of dy, dy2 and the mask.
template <typename T, typename Src, bool WDZ = false, int U = kBnUnroll>
__global__ __launch_bounds__(kBlock) void bn_bwd_reduce_kernel(Src src, const T* __restrict__ x, int64_t M, int C, Geo g,
                                                               const float* __restrict__ mean,
                                                               const float* __restrict__ invstd,
                                                               float* __restrict__ pdb, float* __restrict__ pdg,
                                                               T* __restrict__ dzo = nullptr) {
  constexpr int V = Vec<T>::N;
  const int tc = threadIdx.x % g.tpr;
  const int lane_r = threadIdx.x / g.tpr;
  const int c0 = blockIdx.x * g.ct + tc * V;
  float mu[V], is[V], sb[V], sg[V];
#pragma unroll
  for (int i = 0; i < V; ++i) { mu[i] = mean[c0 + i]; is[i] = invstd[c0 + i]; sb[i] = sg[i] = 0.f; }
  const int64_t r0 = (int64_t)blockIdx.y * g.rows_per_block;
  int64_t r1 = r0 + g.rows_per_block;
  if (r1 > M) r1 = M;
  struct Row { float d[V], xv[V]; };
  stream_rows<U, Row>(
      lane_r < g.rl ? r0 + lane_r : r1, r1, g.rl,
      [&](Row& w, int64_t r) {
        src.load(r, C, c0, w.d);
        Vec<T>::load(x + r * C + c0, w.xv);
      },
      [&](const Row& w, int64_t r) {
        if (WDZ) Vec<T>::store(dzo + r * C + c0, w.d);
#pragma unroll
        for (int i = 0; i < V; ++i) {
          const float dz = w.d[i];
          sb[i] += dz;
          sg[i] = fmaf(dz, (w.xv[i] - mu[i]) * is[i], sg[i]);
        }
      });
  __shared__ float sh[2][kBlock * 8];
#pragma unroll
  for (int i = 0; i < V; ++i) {
    sh[0][threadIdx.x * V + i] = sb[i];
    sh[1][threadIdx.x * V + i] = sg[i];
  }
  __syncthreads();
  for (int cl = threadIdx.x; cl < g.ct; cl += kBlock) {
    const int t = cl / V, i = cl % V;
    float a = 0.f, b = 0.f;
    for (int l = 0; l < g.rl; ++l) {
      a += sh[0][(l * g.tpr + t) * V + i];
      b += sh[1][(l * g.tpr + t) * V + i];
    }
    const int c = blockIdx.x * g.ct + cl;
    pdb[(int64_t)blockIdx.y * C + c] = a;
    pdg[(int64_t)blockIdx.y * C + c] = b;
  }
}

struct BwdFin {   // backward finalize: partials -> dbeta, dgamma (+ arena accumulation)
  const float* pdb;
  const float* pdg;
  int gy;
  float* dbeta;
  float* dgamma;
  float* gb_acc;
  float* gw_acc;
  const float* cmean;     // non-null: the dgamma partials are sum(dz * x) (GEMM epilogue)
  const float* cinvstd;
};

template <bool COH>
__device__ __forceinline__ void bwd_fin_group(const BwdFin& f, int C, int grp) {
  double a = 0.0, b = 0.0;
  bool owner;
  int c;
  reduce_partials2(f.pdb, f.pdg, f.gy, C, &a, &b, &owner, &c, grp);
  if (!owner) return;
  // partials of sum(dz * x) from a GEMM epilogue: sum(dz * xhat) = invstd * (sum(dz x) - mean sum(dz))
  if (f.cmean) b = (double)f.cinvstd[c] * (b - (double)f.cmean[c] * a);
  put<COH>(f.dbeta + c, (float)a);
  put<COH>(f.dgamma + c, (float)b);
  // direct-to-arena parameter gradients (AccumulateGrad semantics)
  if (f.gb_acc) f.gb_acc[c] += (float)a;
  if (f.gw_acc) f.gw_acc[c] += (float)b;
}

__global__ __launch_bounds__(kBlock) void bn_bwd_finalize_kernel(const float* __restrict__ pdb,
                                                                 const float* __restrict__ pdg, int gy, int C,
                                                                 float* __restrict__ dbeta, float* __restrict__ dgamma,
                                                                 float* __restrict__ gb_acc,
                                                                 float* __restrict__ gw_acc,
                                                                 const float* __restrict__ cmean = nullptr,
                                                                 const float* __restrict__ cinvstd = nullptr) {
  const BwdFin f{pdb, pdg, gy, dbeta, dgamma, gb_acc, gw_acc, cmean, cinvstd};
  bwd_fin_group<false>(f, C, blockIdx.x);
}

// Lazy backward apply (the consumer kernels compute dx themselves): finalize as
// above and emit, per channel, the coefficients of
//   dx = k1 * ((dz - k2) - (x - mu) * k4),  k1 = gamma invstd, k2 = mean(dz),
//   k4 = invstd^2 mean(dz (x - mu)) ... = invstd * mean(dz * xhat)
// as coef[c] = {k1, k2, mu, k4}, plus the two padding rows padz = k2 and
// padx = mu in the activation dtype: a padding tap that loads them yields
// exactly dx = 0 (gemm.hip LazyA / LazyG).  center: the dgamma partials are
// sum(dz * x) (GEMM epilogue) rather than sum(dz * xhat) (reduce pass).
template <typename T>
__global__ __launch_bounds__(kBlock) void bn_bwd_finalize_lazy_kernel(
    const float* __restrict__ pdb, const float* __restrict__ pdg, int gy, int C, int64_t M, int center,
    const float* __restrict__ w, const float* __restrict__ mean, const float* __restrict__ invstd,
    float* __restrict__ dbeta, float* __restrict__ dgamma, float* __restrict__ gb_acc, float* __restrict__ gw_acc,
    float4* __restrict__ coef, T* __restrict__ padz, T* __restrict__ padx) {
  double a = 0.0, b = 0.0;
  bool owner;
  int c;
  reduce_partials2(pdb, pdg, gy, C, &a, &b, &owner, &c, blockIdx.x);
  if (!owner) return;
  const float is = invstd[c];
  if (center) b = (double)is * (b - (double)mean[c] * a);
  dbeta[c] = (float)a;
  dgamma[c] = (float)b;
  if (gb_acc) gb_acc[c] += (float)a;
  if (gw_acc) gw_acc[c] += (float)b;
  const float invM = 1.f / (float)M;
  const float gam = w ? w[c] : 1.f;
  const float k1 = gam * is;
  const float k2 = (float)a * invM;
  const float k4 = is * ((float)b * invM);
  float mu = mean[c];
  float k2r = k2;
  if (sizeof(T) == 2) {   // bf16 padding rows: the transform subtracts the same rounded values
    k2r = round_to_bf16(k2);
    mu = round_to_bf16(mu);
  }
  coef[c] = make_float4(k1, k2r, mu, k4);
  store_elem(padz + c, k2r);
  store_elem(padx + c, mu);
}

// DUAL: a second BN whose output gradient is the same dz (the deferred
// ResNet shortcut BN, ops/bn.py _BNDeferFn: out = relu(bn3(x) + bn_ds(x2)))
// gets its dx2 in the same pass -- dz is read once for both.
template <typename T>
struct BwdDual {
  const T* x;
  T* dx;
  const float* w;
  const float* mean;
  const float* invstd;
  const float* dbeta;
  const float* dgamma;
};

template <typename T, typename Src, bool DRES, bool FIN = false, int U = kBnUnroll, bool DUAL = false>
__global__ __launch_bounds__(kBlock) void bn_bwd_apply_kernel(Src src, const T* __restrict__ x, T* __restrict__ dx,
                                                              T* __restrict__ dres, int64_t M, int C, Geo g,
                                                              const float* __restrict__ w,
                                                              const float* __restrict__ mean,
                                                              const float* __restrict__ invstd,
                                                              const float* __restrict__ dbeta,
                                                              const float* __restrict__ dgamma,
                                                              FinSync fs = FinSync{}, BwdFin bf = BwdFin{},
                                                              BwdDual<T> d2 = BwdDual<T>{}) {
  constexpr int V = Vec<T>::N;
  const int tc = threadIdx.x % g.tpr;
  const int lane_r = threadIdx.x / g.tpr;
  const int c0 = blockIdx.x * g.ct + tc * V;
  const float invM = 1.f / (float)M;
  if (FIN)
    fin_prologue(fs, (blockIdx.x * g.ct) / kFinC, ((blockIdx.x + 1) * g.ct + kFinC - 1) / kFinC,
                 [&](int grp) { bwd_fin_group<true>(bf, C, grp); });
  float mu[V], is[V], k1[V], k2[V], k3[V];
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int c = c0 + i;
    mu[i] = mean[c];
    is[i] = invstd[c];
    const float gam = w ? w[c] : 1.f;
    k1[i] = gam * is[i];                                              // scale
    k2[i] = (FIN ? ld_coh_f32(dbeta, c) : dbeta[c]) * invM;          // mean of dz
    k3[i] = (FIN ? ld_coh_f32(dgamma, c) : dgamma[c]) * invM;        // mean of dz * xhat
  }
  constexpr int V2 = DUAL ? V : 1;
  float mu2[V2], is2[V2], q1[V2], q2[V2], q3[V2];
  if constexpr (DUAL) {
#pragma unroll
    for (int i = 0; i < V; ++i) {
      const int c = c0 + i;
      mu2[i] = d2.mean[c];
      is2[i] = d2.invstd[c];
      q1[i] = (d2.w ? d2.w[c] : 1.f) * is2[i];
      q2[i] = d2.dbeta[c] * invM;
      q3[i] = d2.dgamma[c] * invM;
    }
  }
  const int64_t r0 = (int64_t)blockIdx.y * g.rows_per_block;
  int64_t r1 = r0 + g.rows_per_block;
  if (r1 > M) r1 = M;
  struct Row { float d[V], xv[V], x2[V2]; };
  stream_rows<U, Row>(
      lane_r < g.rl ? r0 + lane_r : r1, r1, g.rl,
      [&](Row& w, int64_t r) {
        src.load(r, C, c0, w.d);
        Vec<T>::load(x + r * C + c0, w.xv);
        if constexpr (DUAL) Vec<T>::load(d2.x + r * C + c0, w.x2);
      },
      [&](const Row& w, int64_t r) {
        float o[V];
#pragma unroll
        for (int i = 0; i < V; ++i) {
          const float xh = (w.xv[i] - mu[i]) * is[i];
          o[i] = k1[i] * (w.d[i] - k2[i] - xh * k3[i]);
        }
        Vec<T>::store(dx + r * C + c0, o);
        if (DRES) Vec<T>::store(dres + r * C + c0, w.d);
        if constexpr (DUAL) {
          float o2[V];
#pragma unroll
          for (int i = 0; i < V; ++i) {
            const float xh = (w.x2[i] - mu2[i]) * is2[i];
            o2[i] = q1[i] * (w.d[i] - q2[i] - xh * q3[i]);
          }
          Vec<T>::store(d2.dx + r * C + c0, o2);
        }
      });
}

// Tile-ordered pool backward (k <= 2s, s == 2: the 3x3/s2 stem pool).  The
// input plane is partitioned into s x s tiles, tile (th, tw) owning input rows
// th*s-p .. th*s-p+s-1 (and the same for columns); exactly the windows
// oh in {th-1, th} x ow in {tw-1, tw} can reach a tile, so one thread loads
// those <= 4 argmax/gradient vectors ONCE and produces dz for all s*s pixels
// it owns (4x fewer gathers than the per-pixel DyPool path, no division per
// pixel).  APPLY=false: per-block partial sums of dz and dz*xhat (same
// [gy][C] partial layout as bn_bwd_reduce_kernel, finished by
// bn_bwd_finalize_kernel); APPLY=true: dx = scale*(dz - mean(dz) - xhat*mean(dz*xhat)).
template <typename T, bool TWIN, bool APPLY>
__global__ __launch_bounds__(kBlock) void bn_pool_tile_kernel(const T* __restrict__ dy, const T* __restrict__ dy2,
                                                              const uint8_t* __restrict__ amax,
                                                              const T* __restrict__ x, T* __restrict__ dx,
                                                              int64_t ntiles, int C, PoolGeo pg, int TH, int TW, Geo g,
                                                              int64_t M, const float* __restrict__ w,
                                                              const float* __restrict__ mean,
                                                              const float* __restrict__ invstd,
                                                              const float* __restrict__ dbeta,
                                                              const float* __restrict__ dgamma,
                                                              float* __restrict__ pdb, float* __restrict__ pdg) {
  constexpr int V = Vec<T>::N;
  constexpr int S = 2;
  const int tc = threadIdx.x % g.tpr;
  const int lane_r = threadIdx.x / g.tpr;
  const int c0 = blockIdx.x * g.ct + tc * V;
  const float invM = 1.f / (float)M;
  float mu[V], is[V], k1[V], k2[V], k3[V], sb[V], sg[V];
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int c = c0 + i;
    mu[i] = mean[c];
    is[i] = invstd[c];
    sb[i] = sg[i] = 0.f;
    if (APPLY) {
      k1[i] = (w ? w[c] : 1.f) * is[i];
      k2[i] = dbeta[c] * invM;
      k3[i] = dgamma[c] * invM;
    }
  }
  const int64_t r0 = (int64_t)blockIdx.y * g.rows_per_block;
  int64_t r1 = r0 + g.rows_per_block;
  if (r1 > ntiles) r1 = ntiles;
  const int tplane = TH * TW;
  for (int64_t t = (lane_r < g.rl ? r0 + lane_r : r1); t < r1; t += g.rl) {
    const int64_t n = t / tplane;
    const int rem = (int)(t - n * tplane);
    const int th = rem / TW, tw = rem - (rem / TW) * TW;
    // the s*s input pixels of the tile (issued first: independent of the windows;
    // out-of-image pixels read the tile's first in-image pixel and are skipped)
    float xv[S * S][V];
    bool okq[S * S];
    int64_t xo[S * S];
    {
      const int ihb = th * S - pg.p, iwb = tw * S - pg.p;
      const int ihs = ihb < 0 ? 0 : (ihb < pg.H ? ihb : pg.H - 1);   // an in-image pixel (clamped)
      const int iws = iwb < 0 ? 0 : (iwb < pg.W ? iwb : pg.W - 1);
#pragma unroll
      for (int q = 0; q < S * S; ++q) {
        const int ih = ihb + q / S, iw = iwb + q % S;
        okq[q] = ih >= 0 && ih < pg.H && iw >= 0 && iw < pg.W;
        xo[q] = ((n * pg.H + (okq[q] ? ih : ihs)) * pg.W + (okq[q] ? iw : iws)) * C + c0;
        Vec<T>::load(x + xo[q], xv[q]);
      }
    }
    // the <= 4 windows that reach this tile
    uint32_t a[4][2];
    float gv[4][V];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int oh = th - 1 + (j >> 1), ow = tw - 1 + (j & 1);
      a[j][0] = a[j][1] = 0xffffffffu;
#pragma unroll
      for (int i = 0; i < V; ++i) gv[j][i] = 0.f;
      if (oh >= 0 && oh < pg.OH && ow >= 0 && ow < pg.OW) {
        const int64_t o = ((n * pg.OH + oh) * pg.OW + ow) * C + c0;
        if (V == 8) {
          const uint2 u = *reinterpret_cast<const uint2*>(amax + o);
          a[j][0] = u.x;
          a[j][1] = u.y;
        } else {
          a[j][0] = *reinterpret_cast<const uint32_t*>(amax + o);
        }
        Vec<T>::load(dy + o, gv[j]);
        if (TWIN) {
          float e[V];
          Vec<T>::load(dy2 + o, e);
#pragma unroll
          for (int i = 0; i < V; ++i) gv[j][i] += e[i];
        }
      }
    }
#pragma unroll
    for (int q = 0; q < S * S; ++q) {
      const int ih = th * S - pg.p + (q / S), iw = tw * S - pg.p + (q % S);
      if (!okq[q]) continue;
      float d[V];
#pragma unroll
      for (int i = 0; i < V; ++i) d[i] = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int kh = ih - ((th - 1 + (j >> 1)) * S - pg.p);
        const int kw = iw - ((tw - 1 + (j & 1)) * S - pg.p);
        if (kh < 0 || kh >= pg.k || kw < 0 || kw >= pg.k) continue;
        const uint32_t pos = (uint32_t)(kh * pg.k + kw);
#pragma unroll
        for (int i = 0; i < V; ++i)
          if (((a[j][i / 4] >> (8 * (i % 4))) & 0xffu) == pos) d[i] += gv[j][i];
      }
      if (APPLY) {
        float o[V];
#pragma unroll
        for (int i = 0; i < V; ++i) o[i] = k1[i] * (d[i] - k2[i] - (xv[q][i] - mu[i]) * is[i] * k3[i]);
        Vec<T>::store(dx + xo[q], o);
      } else {
#pragma unroll
        for (int i = 0; i < V; ++i) {
          sb[i] += d[i];
          sg[i] = fmaf(d[i], (xv[q][i] - mu[i]) * is[i], sg[i]);
        }
      }
    }
  }
  if (APPLY) return;
  __shared__ float sh[2][kBlock * 8];
#pragma unroll
  for (int i = 0; i < V; ++i) {
    sh[0][threadIdx.x * V + i] = sb[i];
    sh[1][threadIdx.x * V + i] = sg[i];
  }
  __syncthreads();
  for (int cl = threadIdx.x; cl < g.ct; cl += kBlock) {
    const int tt = cl / V, i = cl % V;
    float s0 = 0.f, s1 = 0.f;
    for (int l = 0; l < g.rl; ++l) {
      s0 += sh[0][(l * g.tpr + tt) * V + i];
      s1 += sh[1][(l * g.tpr + tt) * V + i];
    }
    const int c = blockIdx.x * g.ct + cl;
    pdb[(int64_t)blockIdx.y * C + c] = s0;
    pdg[(int64_t)blockIdx.y * C + c] = s1;
  }
}

constexpr int kPoolTargetBlocks = 4096;
// blocks per streaming pass (<= kPoolTargetBlocks: the workspace is sized for that)
int g_bn_blocks = 1024;
#define kTargetBlocks g_bn_blocks

// In-launch finalize for one launch of grid g, or a FinSync with ticket ==
// nullptr (separate finalize launch): needs the per-layer state, no stream
// capture (the epoch argument would be frozen into the replays), and at least
// one workgroup per finalize group.
FinSync make_fin(void* state, const Geo& g, int C, hipStream_t s) {
  static std::atomic<uint32_t> epoch{0};
  FinSync fs{};
  if (state == nullptr) return fs;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return fs;
  const int ngroups = (C + kFinC - 1) / kFinC;
  const int64_t nb = (int64_t)g.gx * g.gy;
  if (nb < ngroups || nb > 0x7fffffff) return fs;
  uint32_t e = epoch.fetch_add(1) + 1;
  if (e == 0) e = epoch.fetch_add(1) + 1;   // 0 is the flags' initial value
  fs.ticket = reinterpret_cast<unsigned long long*>(state);
  fs.flags = reinterpret_cast<uint32_t*>(static_cast<char*>(state) + kFinStateFlagsOffset);
  fs.epoch = e;
  fs.nblocks = (uint32_t)nb;
  fs.ngroups = ngroups;
  return fs;
}

}  // namespace

size_t bn_fin_state_bytes(int C) { return kFinStateFlagsOffset + sizeof(uint32_t) * (size_t)((C + kFinC - 1) / kFinC); }

size_t bn_workspace_floats(int64_t M, int C, int elem_bytes) {
  // sized for the larger (pool-backward) grid so one workspace fits every pass
  const Geo g =
      elem_bytes == 2 ? make_geo<uint16_t>(M, C, kPoolTargetBlocks) : make_geo<float>(M, C, kPoolTargetBlocks);
  return (size_t)2 * g.gy * C;
}

void bn_set_blocks(int blocks) { g_bn_blocks = blocks < 64 ? 64 : blocks > kPoolTargetBlocks ? kPoolTargetBlocks : blocks; }

bool bn_supported(int C, int elem_bytes) {
  const int V = elem_bytes == 2 ? 8 : 4;
  return C % V == 0 && C >= V;
}

template <typename T>
void bn_stats_t(const T* x, int64_t M, int C, const float* w, const float* b, float eps, float momentum,
                float* run_mean, float* run_var, float* save_mean, float* save_invstd, float* scale, float* shift,
                float* ws, int64_t* nbt, hipStream_t s) {
  const Geo g = make_geo<T>(M, C, kTargetBlocks);
  float* psum = ws;
  float* psq = ws + (int64_t)g.gy * C;
  hipLaunchKernelGGL(bn_stats_kernel<T>, dim3(g.gx, g.gy), dim3(kBlock), 0, s, x, M, C, g, psum, psq);
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + kFinC - 1) / kFinC), dim3(kBlock), 0, s, psum, psq, g.gy, M, C,
                     w, b, eps, momentum, run_mean, run_var, save_mean, save_invstd, scale, shift, nbt);
}

template <typename T>
void launch_apply(const T* x, const T* res, T* y, uint8_t* mask, int64_t M, int C, const Geo& g, float* scale,
                  float* shift, int relu, const FinSync& fs, const FwdFin& ff, hipStream_t s,
                  const float* rscale = nullptr, const float* rshift = nullptr) {
  if (res && rscale) {
    // deferred residual BN (its scale / shift finalized by an earlier launch)
    if (relu)
      hipLaunchKernelGGL((bn_apply_kernel<T, true, true, false, kBnUnroll, true>), dim3(g.gx, g.gy), dim3(kBlock), 0, s,
                         x, res, y, mask, M, C, g, scale, shift, fs, ff, rscale, rshift);
    else
      hipLaunchKernelGGL((bn_apply_kernel<T, false, true, false, kBnUnroll, true>), dim3(g.gx, g.gy), dim3(kBlock), 0,
                         s, x, res, y, mask, M, C, g, scale, shift, fs, ff, rscale, rshift);
    return;
  }
#define GK_APPLY(R, D, F)                                                                                           \
  hipLaunchKernelGGL((bn_apply_kernel<T, R, D, F>), dim3(g.gx, g.gy), dim3(kBlock), 0, s, x, res, y, mask, M, C, g, \
                     scale, shift, fs, ff, nullptr, nullptr)
#define GK_APPLY2(R, D) if (fs.ticket) GK_APPLY(R, D, true); else GK_APPLY(R, D, false);
  if (relu && res) { GK_APPLY2(true, true) }
  else if (relu) { GK_APPLY2(true, false) }
  else if (res) { GK_APPLY2(false, true) }
  else { GK_APPLY2(false, false) }
#undef GK_APPLY2
#undef GK_APPLY
}

template <typename T>
void bn_forward_t(const T* x, const T* res, T* y, uint8_t* mask, int64_t M, int C, const float* w, const float* b, float eps,
                  float momentum, float* run_mean, float* run_var, float* save_mean, float* save_invstd,
                  float* scale, float* shift, float* ws, int relu, int64_t* nbt, void* fin_state, hipStream_t s,
                  const float* rscale = nullptr, const float* rshift = nullptr) {
  const Geo g = make_geo<T>(M, C, kTargetBlocks);
  if (rscale) fin_state = nullptr;   // the deferred-residual apply has no in-launch finalize form
  const FinSync fs = make_fin(fin_state, g, C, s);
  const FwdFin ff{ws, ws + (int64_t)g.gy * C, g.gy, w, b, eps, momentum, run_mean, run_var, save_mean, save_invstd,
                  scale, shift, nbt};
  if (fs.ticket) {
    hipLaunchKernelGGL(bn_stats_kernel<T>, dim3(g.gx, g.gy), dim3(kBlock), 0, s, x, M, C, g, ws, ws + (int64_t)g.gy * C);
  } else {
    bn_stats_t<T>(x, M, C, w, b, eps, momentum, run_mean, run_var, save_mean, save_invstd, scale, shift, ws, nbt, s);
  }
  launch_apply<T>(x, res, y, mask, M, C, g, scale, shift, relu, fs, ff, s, rscale, rshift);
}

// finalize (separate launch unless fs carries the in-launch state) + apply
template <typename T, typename Src, bool DRES>
void launch_bwd_apply(Src src, const T* x, T* dx, T* dres, int64_t M, int C, const Geo& g, const float* w,
                      const float* mean, const float* invstd, const BwdFin& bf, const FinSync& fs, hipStream_t s) {
  if (fs.ticket) {
    hipLaunchKernelGGL((bn_bwd_apply_kernel<T, Src, DRES, true>), dim3(g.gx, g.gy), dim3(kBlock), 0, s, src, x, dx,
                       dres, M, C, g, w, mean, invstd, bf.dbeta, bf.dgamma, fs, bf);
    return;
  }
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + kFinC - 1) / kFinC), dim3(kBlock), 0, s, bf.pdb, bf.pdg, bf.gy,
                     C, bf.dbeta, bf.dgamma, bf.gb_acc, bf.gw_acc, bf.cmean, bf.cinvstd);
  hipLaunchKernelGGL((bn_bwd_apply_kernel<T, Src, DRES, false>), dim3(g.gx, g.gy), dim3(kBlock), 0, s, src, x, dx,
                     dres, M, C, g, w, mean, invstd, bf.dbeta, bf.dgamma, FinSync{}, BwdFin{});
}

template <typename T, typename Src>
void bn_backward_src(Src src, const T* x, T* dx, T* dres, int64_t M, int C, const float* w, const float* mean,
                     const float* invstd, float* dgamma, float* dbeta, float* ws, float* gw_acc, float* gb_acc,
                     void* fin_state, hipStream_t s, int target_blocks = kTargetBlocks) {
  const Geo g = make_geo<T>(M, C, target_blocks);
  float* pdb = ws;
  float* pdg = ws + (int64_t)g.gy * C;
  hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, Src>), dim3(g.gx, g.gy), dim3(kBlock), 0, s, src, x, M, C, g, mean,
                     invstd, pdb, pdg);
  const FinSync fs = make_fin(fin_state, g, C, s);
  const BwdFin bf{pdb, pdg, g.gy, dbeta, dgamma, gb_acc, gw_acc, nullptr, nullptr};
  if (dres) launch_bwd_apply<T, Src, true>(src, x, dx, dres, M, C, g, w, mean, invstd, bf, fs, s);
  else launch_bwd_apply<T, Src, false>(src, x, dx, dres, M, C, g, w, mean, invstd, bf, fs, s);
}

template <typename T>
void bn_backward_t(const T* dy, const T* dy2, const uint8_t* mask, const T* x, T* dx, T* dres, int64_t M, int C,
                   const float* w, const float* mean, const float* invstd, float* dgamma, float* dbeta, float* ws,
                   int relu, float* gw_acc, float* gb_acc, void* fin_state, hipStream_t s) {
  if (dy2 && dres) {
    // twin + residual (ResNet block output): the reduce pass writes dz = dres
    // and the apply pass reads it back (one tensor instead of dy, dy2, mask)
    const Geo g = make_geo<T>(M, C, kTargetBlocks);
    float* pdb = ws;
    float* pdg = ws + (int64_t)g.gy * C;
#define GK_RED(R)                                                                                                  \
  hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, DyPlain<T, R, true>, true>), dim3(g.gx, g.gy), dim3(kBlock), 0, s,     \
                     DyPlain<T, R, true>{dy, dy2, mask}, x, M, C, g, mean, invstd, pdb, pdg, dres)
    if (relu) GK_RED(true);
    else GK_RED(false);
#undef GK_RED
    const FinSync fs = make_fin(fin_state, g, C, s);
    const BwdFin bf{pdb, pdg, g.gy, dbeta, dgamma, gb_acc, gw_acc, nullptr, nullptr};
    launch_bwd_apply<T, DyPlain<T, false, false>, false>(DyPlain<T, false, false>{dres, nullptr, nullptr}, x, dx,
                                                         (T*)nullptr, M, C, g, w, mean, invstd, bf, fs, s);
    return;
  }
#define GK_BWD(R, TW)                                                                                              \
  bn_backward_src<T>(DyPlain<T, R, TW>{dy, dy2, mask}, x, dx, dres, M, C, w, mean, invstd, dgamma, dbeta, ws, gw_acc, \
                     gb_acc, fin_state, s)
  if (relu && dy2) GK_BWD(true, true);
  else if (relu) GK_BWD(true, false);
  else if (dy2) GK_BWD(false, true);
  else GK_BWD(false, false);
#undef GK_BWD
}

size_t bn_mask_bytes(int64_t M, int C, int elem_bytes) { return (size_t)M * (size_t)(C / (elem_bytes == 2 ? 8 : 4)); }

void bn_stats_partials(const void* x, int64_t M, int C, int elem_bytes, float* ws, hipStream_t s) {
  if (elem_bytes == 2) {
    const Geo g = make_geo<uint16_t>(M, C, kTargetBlocks);
    hipLaunchKernelGGL(bn_stats_kernel<uint16_t>, dim3(g.gx, g.gy), dim3(kBlock), 0, s, static_cast<const uint16_t*>(x), M,
                       C, g, ws, ws + (int64_t)g.gy * C);
  } else {
    const Geo g = make_geo<float>(M, C, kTargetBlocks);
    hipLaunchKernelGGL(bn_stats_kernel<float>, dim3(g.gx, g.gy), dim3(kBlock), 0, s, static_cast<const float*>(x), M, C,
                       g, ws, ws + (int64_t)g.gy * C);
  }
}

void bn_act_forward(const void* x, const void* res, void* y, uint8_t* mask, int64_t M, int C, int elem_bytes,
                    const float* w, const float* b, float eps, float momentum, float* run_mean, float* run_var,
                    float* save_mean, float* save_invstd, float* scale, float* shift, float* ws, int relu,
                    int64_t* nbt, hipStream_t s, void* fin_state, const float* rscale, const float* rshift) {
  if (elem_bytes == 2)
    bn_forward_t<uint16_t>((const uint16_t*)x, (const uint16_t*)res, (uint16_t*)y, mask, M, C, w, b, eps, momentum,
                           run_mean, run_var, save_mean, save_invstd, scale, shift, ws, relu, nbt, fin_state, s,
                           rscale, rshift);
  else
    bn_forward_t<float>((const float*)x, (const float*)res, (float*)y, mask, M, C, w, b, eps, momentum, run_mean,
                        run_var, save_mean, save_invstd, scale, shift, ws, relu, nbt, fin_state, s, rscale, rshift);
}

// Statistics (or the producer's partials) + finalize only: the BN whose apply
// pass is deferred into its consumer (bn_apply_kernel RBN).
void bn_act_finalize(const void* x, int64_t M, int C, int elem_bytes, const float* psum, const float* psq, int gy,
                     const float* w, const float* b, float eps, float momentum, float* run_mean, float* run_var,
                     float* save_mean, float* save_invstd, float* scale, float* shift, float* ws, int64_t* nbt,
                     hipStream_t s) {
  if (!psum) {
    if (elem_bytes == 2)
      bn_stats_t<uint16_t>((const uint16_t*)x, M, C, w, b, eps, momentum, run_mean, run_var, save_mean, save_invstd,
                           scale, shift, ws, nbt, s);
    else
      bn_stats_t<float>((const float*)x, M, C, w, b, eps, momentum, run_mean, run_var, save_mean, save_invstd, scale,
                        shift, ws, nbt, s);
    return;
  }
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + kFinC - 1) / kFinC), dim3(kBlock), 0, s, psum, psq, gy, M, C, w, b,
                     eps, momentum, run_mean, run_var, save_mean, save_invstd, scale, shift, nbt);
}

template <typename T>
void bn_forward_pre_t(const T* x, const T* res, T* y, uint8_t* mask, int64_t M, int C, const float* psum,
                      const float* psq, int gy, const float* w, const float* b, float eps, float momentum,
                      float* run_mean, float* run_var, float* save_mean, float* save_invstd, float* scale, float* shift,
                      int relu, int64_t* nbt, void* fin_state, hipStream_t s, const float* rscale = nullptr,
                      const float* rshift = nullptr) {
  const Geo g = make_geo<T>(M, C, kTargetBlocks);
  if (rscale) fin_state = nullptr;
  const FinSync fs = make_fin(fin_state, g, C, s);
  const FwdFin ff{psum, psq, gy, w, b, eps, momentum, run_mean, run_var, save_mean, save_invstd, scale, shift, nbt};
  if (!fs.ticket)
    hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + kFinC - 1) / kFinC), dim3(kBlock), 0, s, psum, psq, gy, M, C, w,
                       b, eps, momentum, run_mean, run_var, save_mean, save_invstd, scale, shift, nbt);
  launch_apply<T>(x, res, y, mask, M, C, g, scale, shift, relu, fs, ff, s, rscale, rshift);
}

void bn_act_forward_pre(const void* x, const void* res, void* y, uint8_t* mask, int64_t M, int C, int elem_bytes,
                        const float* psum, const float* psq, int gy, const float* w, const float* b, float eps, float momentum,
                        float* run_mean, float* run_var, float* save_mean, float* save_invstd, float* scale,
                        float* shift, int relu, int64_t* nbt, hipStream_t s, void* fin_state, const float* rscale,
                        const float* rshift) {
  if (elem_bytes == 2)
    bn_forward_pre_t<uint16_t>((const uint16_t*)x, (const uint16_t*)res, (uint16_t*)y, mask, M, C, psum, psq, gy, w,
                               b, eps, momentum, run_mean, run_var, save_mean, save_invstd, scale, shift, relu, nbt,
                               fin_state, s, rscale, rshift);
  else
    bn_forward_pre_t<float>((const float*)x, (const float*)res, (float*)y, mask, M, C, psum, psq, gy, w, b, eps,
                            momentum, run_mean, run_var, save_mean, save_invstd, scale, shift, relu, nbt, fin_state, s,
                            rscale, rshift);
}

void bn_act_backward(const void* dy, const void* dy2, const uint8_t* mask, const void* x, void* dx, void* dres,
                     int64_t M, int C, int elem_bytes, const float* w, const float* mean, const float* invstd,
                     float* dgamma, float* dbeta, float* ws, int relu, float* gw_acc, float* gb_acc, hipStream_t s,
                     void* fin_state) {
  if (elem_bytes == 2)
    bn_backward_t<uint16_t>((const uint16_t*)dy, (const uint16_t*)dy2, mask, (const uint16_t*)x, (uint16_t*)dx,
                            (uint16_t*)dres, M, C, w, mean, invstd, dgamma, dbeta, ws, relu, gw_acc, gb_acc, fin_state,
                            s);
  else
    bn_backward_t<float>((const float*)dy, (const float*)dy2, mask, (const float*)x, (float*)dx, (float*)dres, M, C, w,
                         mean, invstd, dgamma, dbeta, ws, relu, gw_acc, gb_acc, fin_state, s);
}

// dz (already gated and twin-summed) and its partials sum(dz), sum(dz*(x-mean))
// [2][gy][C] from the consuming convolution's grad-input epilogue (gemm.hip
// BnBwd): no reduction pass, only finalize + apply.
template <typename T>
void bn_bwd_apply_pre_t(const T* dz, const T* x, T* dx, int64_t M, int C, const float* w, const float* mean,
                        const float* invstd, float* dgamma, float* dbeta, const float* pdb, const float* pdg, int gy,
                        float* gw_acc, float* gb_acc, void* fin_state, hipStream_t s) {
  const Geo g = make_geo<T>(M, C, kTargetBlocks);
  const FinSync fs = make_fin(fin_state, g, C, s);
  const BwdFin bf{pdb, pdg, gy, dbeta, dgamma, gb_acc, gw_acc, mean, invstd};
  launch_bwd_apply<T, DyPlain<T, false, false>, false>(DyPlain<T, false, false>{dz, nullptr, nullptr}, x, dx,
                                                       (T*)nullptr, M, C, g, w, mean, invstd, bf, fs, s);
}

void bn_bwd_finalize_lazy(const float* pdb, const float* pdg, int gy, int64_t M, int C, int elem_bytes, int center,
                          const float* w, const float* mean, const float* invstd, float* dgamma, float* dbeta,
                          float* gw_acc, float* gb_acc, float* coef, void* padz, void* padx, hipStream_t s) {
  const dim3 grid((C + kFinC - 1) / kFinC);
  if (elem_bytes == 2)
    hipLaunchKernelGGL(bn_bwd_finalize_lazy_kernel<uint16_t>, grid, dim3(kBlock), 0, s, pdb, pdg, gy, C, M, center, w,
                       mean, invstd, dbeta, dgamma, gb_acc, gw_acc, reinterpret_cast<float4*>(coef),
                       static_cast<uint16_t*>(padz), static_cast<uint16_t*>(padx));
  else
    hipLaunchKernelGGL(bn_bwd_finalize_lazy_kernel<float>, grid, dim3(kBlock), 0, s, pdb, pdg, gy, C, M, center, w,
                       mean, invstd, dbeta, dgamma, gb_acc, gw_acc, reinterpret_cast<float4*>(coef),
                       static_cast<float*>(padz), static_cast<float*>(padx));
}

// Full (unlinked) backward without the apply pass: the reduce pass writes dz
// (ReLU-masked, twin-summed dy) and the partials; the finalize emits the lazy
// coefficients.  dz doubles as the residual gradient.
template <typename T>
void bn_backward_lazy_t(const T* dy, const T* dy2, const uint8_t* mask, const T* x, T* dz, int64_t M, int C,
                        const float* w, const float* mean, const float* invstd, float* dgamma, float* dbeta, float* ws,
                        int relu, float* gw_acc, float* gb_acc, float* coef, void* padz, void* padx, hipStream_t s) {
  const Geo g = make_geo<T>(M, C, kTargetBlocks);
  float* pdb = ws;
  float* pdg = ws + (int64_t)g.gy * C;
#define GK_RED(R, TW)                                                                                              \
  hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, DyPlain<T, R, TW>, true>), dim3(g.gx, g.gy), dim3(kBlock), 0, s,      \
                     DyPlain<T, R, TW>{dy, dy2, mask}, x, M, C, g, mean, invstd, pdb, pdg, dz)
  if (relu && dy2) GK_RED(true, true);
  else if (relu) GK_RED(true, false);
  else if (dy2) GK_RED(false, true);
  else GK_RED(false, false);
#undef GK_RED
  bn_bwd_finalize_lazy(pdb, pdg, g.gy, M, C, sizeof(T), 0, w, mean, invstd, dgamma, dbeta, gw_acc, gb_acc, coef,
                       padz, padx, s);
}

void bn_act_backward_lazy(const void* dy, const void* dy2, const uint8_t* mask, const void* x, void* dz, int64_t M,
                          int C, int elem_bytes, const float* w, const float* mean, const float* invstd,
                          float* dgamma, float* dbeta, float* ws, int relu, float* gw_acc, float* gb_acc, float* coef,
                          void* padz, void* padx, hipStream_t s) {
  if (elem_bytes == 2)
    bn_backward_lazy_t<uint16_t>((const uint16_t*)dy, (const uint16_t*)dy2, mask, (const uint16_t*)x, (uint16_t*)dz,
                                 M, C, w, mean, invstd, dgamma, dbeta, ws, relu, gw_acc, gb_acc, coef, padz, padx, s);
  else
    bn_backward_lazy_t<float>((const float*)dy, (const float*)dy2, mask, (const float*)x, (float*)dz, M, C, w, mean,
                              invstd, dgamma, dbeta, ws, relu, gw_acc, gb_acc, coef, padz, padx, s);
}

// Materialise a lazy dx (a consumer that cannot take the lazy operand):
// dx = k1 * ((dz - k2) - (x - mu) * k4) from the coefficient table.
template <typename T>
__global__ __launch_bounds__(kBlock) void bn_lazy_apply_kernel(const T* __restrict__ dz, const T* __restrict__ x,
                                                               T* __restrict__ dx, int64_t M, int C, Geo g,
                                                               const float4* __restrict__ coef) {
  constexpr int V = Vec<T>::N;
  const int tc = threadIdx.x % g.tpr;
  const int lane_r = threadIdx.x / g.tpr;
  const int c0 = blockIdx.x * g.ct + tc * V;
  float4 cf[V];
#pragma unroll
  for (int i = 0; i < V; ++i) cf[i] = coef[c0 + i];
  const int64_t r0 = (int64_t)blockIdx.y * g.rows_per_block;
  int64_t r1 = r0 + g.rows_per_block;
  if (r1 > M) r1 = M;
  for (int64_t r = lane_r < g.rl ? r0 + lane_r : r1; r < r1; r += g.rl) {
    float d[V], xv[V], o[V];
    Vec<T>::load(dz + r * C + c0, d);
    Vec<T>::load(x + r * C + c0, xv);
#pragma unroll
    for (int i = 0; i < V; ++i) o[i] = cf[i].x * ((d[i] - cf[i].y) - (xv[i] - cf[i].z) * cf[i].w);
    Vec<T>::store(dx + r * C + c0, o);
  }
}

void bn_lazy_apply(const void* dz, const void* x, void* dx, int64_t M, int C, int elem_bytes, const float* coef,
                   hipStream_t s) {
  if (elem_bytes == 2) {
    const Geo g = make_geo<uint16_t>(M, C, kTargetBlocks);
    hipLaunchKernelGGL(bn_lazy_apply_kernel<uint16_t>, dim3(g.gx, g.gy), dim3(kBlock), 0, s, (const uint16_t*)dz,
                       (const uint16_t*)x, (uint16_t*)dx, M, C, g, reinterpret_cast<const float4*>(coef));
  } else {
    const Geo g = make_geo<float>(M, C, kTargetBlocks);
    hipLaunchKernelGGL(bn_lazy_apply_kernel<float>, dim3(g.gx, g.gy), dim3(kBlock), 0, s, (const float*)dz,
                       (const float*)x, (float*)dx, M, C, g, reinterpret_cast<const float4*>(coef));
  }
}

// Linked backward (dz + partials from the consumer's GEMM epilogue) of a BN
// whose residual was a deferred BN of x2 (bn_apply_kernel RBN): the second
// BN's reduce pass over (dz, x2) and both finalizes, then ONE apply pass
// writing dx and dx2 (dz read once).
template <typename T>
void bn_bwd_pre_dual_t(const T* dz, const T* x, T* dx, int64_t M, int C, const float* w, const float* mean,
                       const float* invstd, float* dgamma, float* dbeta, const float* pdb, const float* pdg, int gy,
                       float* gw_acc, float* gb_acc, const T* x2, T* dx2, const float* w2, const float* mean2,
                       const float* invstd2, float* dgamma2, float* dbeta2, float* ws2, float* gw2_acc,
                       float* gb2_acc, hipStream_t s) {
  const Geo g = make_geo<T>(M, C, kTargetBlocks);
  float* pdb2 = ws2;
  float* pdg2 = ws2 + (int64_t)g.gy * C;
  using Src = DyPlain<T, false, false>;
  const Src src{dz, nullptr, nullptr};
  hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, Src>), dim3(g.gx, g.gy), dim3(kBlock), 0, s, src, x2, M, C, g, mean2,
                     invstd2, pdb2, pdg2, (T*)nullptr);
  const dim3 fg((C + kFinC - 1) / kFinC);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, fg, dim3(kBlock), 0, s, pdb2, pdg2, g.gy, C, dbeta2, dgamma2, gb2_acc,
                     gw2_acc, nullptr, nullptr);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, fg, dim3(kBlock), 0, s, pdb, pdg, gy, C, dbeta, dgamma, gb_acc, gw_acc,
                     mean, invstd);
  const BwdDual<T> d2{x2, dx2, w2, mean2, invstd2, dbeta2, dgamma2};
  hipLaunchKernelGGL((bn_bwd_apply_kernel<T, Src, false, false, kBnUnroll, true>), dim3(g.gx, g.gy), dim3(kBlock), 0,
                     s, src, x, dx, (T*)nullptr, M, C, g, w, mean, invstd, dbeta, dgamma, FinSync{}, BwdFin{}, d2);
}

void bn_act_backward_pre_dual(const void* dz, const void* x, void* dx, int64_t M, int C, int elem_bytes,
                              const float* w, const float* mean, const float* invstd, float* dgamma, float* dbeta,
                              const float* pdb, const float* pdg, int gy, float* gw_acc, float* gb_acc, const void* x2,
                              void* dx2, const float* w2, const float* mean2, const float* invstd2, float* dgamma2,
                              float* dbeta2, float* ws2, float* gw2_acc, float* gb2_acc, hipStream_t s) {
  if (elem_bytes == 2)
    bn_bwd_pre_dual_t<uint16_t>((const uint16_t*)dz, (const uint16_t*)x, (uint16_t*)dx, M, C, w, mean, invstd, dgamma,
                                dbeta, pdb, pdg, gy, gw_acc, gb_acc, (const uint16_t*)x2, (uint16_t*)dx2, w2, mean2,
                                invstd2, dgamma2, dbeta2, ws2, gw2_acc, gb2_acc, s);
  else
    bn_bwd_pre_dual_t<float>((const float*)dz, (const float*)x, (float*)dx, M, C, w, mean, invstd, dgamma, dbeta, pdb,
                             pdg, gy, gw_acc, gb_acc, (const float*)x2, (float*)dx2, w2, mean2, invstd2, dgamma2,
                             dbeta2, ws2, gw2_acc, gb2_acc, s);
}

void bn_act_backward_pre(const void* dz, const void* x, void* dx, int64_t M, int C, int elem_bytes, const float* w,
                         const float* mean, const float* invstd, float* dgamma, float* dbeta, const float* pdb,
                         const float* pdg, int gy, float* gw_acc, float* gb_acc, hipStream_t s, void* fin_state) {
  if (elem_bytes == 2)
    bn_bwd_apply_pre_t<uint16_t>((const uint16_t*)dz, (const uint16_t*)x, (uint16_t*)dx, M, C, w, mean, invstd, dgamma,
                                 dbeta, pdb, pdg, gy, gw_acc, gb_acc, fin_state, s);
  else
    bn_bwd_apply_pre_t<float>((const float*)dz, (const float*)x, (float*)dx, M, C, w, mean, invstd, dgamma, dbeta, pdb,
                              pdg, gy, gw_acc, gb_acc, fin_state, s);
}

// ---------------------------------------------------------------------------
// BN + ReLU + max-pool
// ---------------------------------------------------------------------------
void bn_relu_pool_forward(const void* x, void* y, uint8_t* amax, int64_t N, int C, PoolGeo pg, int elem_bytes,
                          const float* w, const float* b, float eps, float momentum, float* run_mean, float* run_var,
                          float* save_mean, float* save_invstd, float* scale, float* shift, float* ws, int64_t* nbt,
                          hipStream_t s) {
  const int64_t M = N * pg.H * pg.W;
  const int64_t P = N * pg.OH * pg.OW;
  const int V = elem_bytes == 2 ? 8 : 4;
  const int64_t threads = P * (C / V);
  const dim3 grid((unsigned)((threads + kBlock - 1) / kBlock));
  if (elem_bytes == 2) {
    bn_stats_t<uint16_t>((const uint16_t*)x, M, C, w, b, eps, momentum, run_mean, run_var, save_mean, save_invstd,
                         scale, shift, ws, nbt, s);
    if (pg.k == 3 && pg.p == 1)
      hipLaunchKernelGGL((bn_relu_pool_kernel<uint16_t, 3>), grid, dim3(kBlock), 0, s, (const uint16_t*)x, (uint16_t*)y,
                         amax, P, C, pg, scale, shift);
    else
      hipLaunchKernelGGL(bn_relu_pool_kernel<uint16_t>, grid, dim3(kBlock), 0, s, (const uint16_t*)x, (uint16_t*)y, amax,
                         P, C, pg, scale, shift);
  } else {
    bn_stats_t<float>((const float*)x, M, C, w, b, eps, momentum, run_mean, run_var, save_mean, save_invstd, scale,
                       shift, ws, nbt, s);
    if (pg.k == 3 && pg.p == 1)   // all 9 window loads in flight
      hipLaunchKernelGGL((bn_relu_pool_kernel<float, 3>), grid, dim3(kBlock), 0, s, (const float*)x, (float*)y, amax, P,
                         C, pg, scale, shift);
    else
      hipLaunchKernelGGL(bn_relu_pool_kernel<float>, grid, dim3(kBlock), 0, s, (const float*)x, (float*)y, amax, P, C,
                         pg, scale, shift);
  }
}

// statistics pre-reduced by the producing convolution (stem.hip / stem_f32.hip
// epilogues): finalize + the fused BN / ReLU / max-pool pass only
void bn_relu_pool_forward_pre(const void* x, void* y, uint8_t* amax, int64_t N, int C, PoolGeo pg, int elem_bytes,
                              const float* psum, const float* psq, int gy, const float* w, const float* b, float eps,
                              float momentum, float* run_mean, float* run_var, float* save_mean, float* save_invstd,
                              float* scale, float* shift, int64_t* nbt, hipStream_t s) {
  const int64_t M = N * pg.H * pg.W;
  const int64_t P = N * pg.OH * pg.OW;
  const int64_t threads = P * (C / (elem_bytes == 2 ? 8 : 4));
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + kFinC - 1) / kFinC), dim3(kBlock), 0, s, psum, psq, gy, M, C, w, b,
                     eps, momentum, run_mean, run_var, save_mean, save_invstd, scale, shift, nbt);
  const dim3 grid((unsigned)((threads + kBlock - 1) / kBlock));
  if (elem_bytes == 4 && pg.k == 3 && pg.p == 1)
    hipLaunchKernelGGL((bn_relu_pool_kernel<float, 3>), grid, dim3(kBlock), 0, s, (const float*)x, (float*)y, amax, P, C,
                       pg, scale, shift);
  else if (elem_bytes == 4)
    hipLaunchKernelGGL(bn_relu_pool_kernel<float>, grid, dim3(kBlock), 0, s, (const float*)x, (float*)y, amax, P, C, pg,
                       scale, shift);
  else if (pg.k == 3 && pg.p == 1)
    hipLaunchKernelGGL((bn_relu_pool_kernel<uint16_t, 3>), grid, dim3(kBlock), 0, s, (const uint16_t*)x, (uint16_t*)y,
                       amax, P, C, pg, scale, shift);
  else
    hipLaunchKernelGGL(bn_relu_pool_kernel<uint16_t>, grid, dim3(kBlock), 0, s, (const uint16_t*)x, (uint16_t*)y, amax,
                       P, C, pg, scale, shift);
}

template <typename T, bool TWIN>
void bn_pool_backward_tw(const T* dy, const T* dy2, const uint8_t* amax, const T* x, T* dx, int64_t M, int C,
                         PoolGeo pg, const float* w, const float* mean, const float* invstd, float* dgamma,
                         float* dbeta, float* ws, float* gw_acc, float* gb_acc, hipStream_t s) {
  if (pg.s == 2 && pg.k <= 4) {  // every window reaching tile th has oh in {th-1, th}
    // tile-ordered fast path (3x3/s2 stem pool)
    const int TH = (pg.H + pg.p + pg.s - 1) / pg.s, TW = (pg.W + pg.p + pg.s - 1) / pg.s;
    const int64_t N = M / ((int64_t)pg.H * pg.W);
    const int64_t ntiles = N * TH * TW;
    const Geo g = make_geo<T>(ntiles, C, kPoolTargetBlocks);
    float* pdb = ws;
    float* pdg = ws + (int64_t)g.gy * C;
    hipLaunchKernelGGL((bn_pool_tile_kernel<T, TWIN, false>), dim3(g.gx, g.gy), dim3(kBlock), 0, s, dy, dy2, amax, x,
                       (T*)nullptr, ntiles, C, pg, TH, TW, g, M, w, mean, invstd, (const float*)nullptr,
                       (const float*)nullptr, pdb, pdg);
    hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + kFinC - 1) / kFinC), dim3(kBlock), 0, s, pdb, pdg, g.gy, C,
                       dbeta, dgamma, gb_acc, gw_acc);
    hipLaunchKernelGGL((bn_pool_tile_kernel<T, TWIN, true>), dim3(g.gx, g.gy), dim3(kBlock), 0, s, dy, dy2, amax, x,
                       dx, ntiles, C, pg, TH, TW, g, M, w, mean, invstd, dbeta, dgamma, (float*)nullptr,
                       (float*)nullptr);
    return;
  }
  // generic k, s: per-pixel gather (latency-bound: more workgroups than the plain BN passes)
  if ((pg.k + pg.s - 1) / pg.s <= 2)
    bn_backward_src<T>(DyPool<T, TWIN, 2>{dy, dy2, amax, pg}, x, dx, (T*)nullptr, M, C, w, mean, invstd, dgamma,
                       dbeta, ws, gw_acc, gb_acc, nullptr, s, kPoolTargetBlocks);
  else
    bn_backward_src<T>(DyPool<T, TWIN, 0>{dy, dy2, amax, pg}, x, dx, (T*)nullptr, M, C, w, mean, invstd, dgamma,
                       dbeta, ws, gw_acc, gb_acc, nullptr, s, kPoolTargetBlocks);
}

template <typename T>
void bn_pool_backward_t(const T* dy, const T* dy2, const uint8_t* amax, const T* x, T* dx, int64_t M, int C, PoolGeo pg,
                        const float* w, const float* mean, const float* invstd, float* dgamma, float* dbeta, float* ws,
                        float* gw_acc, float* gb_acc, hipStream_t s) {
  if (dy2)
    bn_pool_backward_tw<T, true>(dy, dy2, amax, x, dx, M, C, pg, w, mean, invstd, dgamma, dbeta, ws, gw_acc, gb_acc, s);
  else
    bn_pool_backward_tw<T, false>(dy, dy2, amax, x, dx, M, C, pg, w, mean, invstd, dgamma, dbeta, ws, gw_acc, gb_acc,
                                  s);
}

void bn_relu_pool_backward(const void* dy, const void* dy2, const uint8_t* amax, const void* x, void* dx, int64_t N,
                           int C, PoolGeo pg, int elem_bytes, const float* w, const float* mean, const float* invstd,
                           float* dgamma, float* dbeta, float* ws, float* gw_acc, float* gb_acc, hipStream_t s) {
  const int64_t M = N * pg.H * pg.W;
  if (elem_bytes == 2)
    bn_pool_backward_t<uint16_t>((const uint16_t*)dy, (const uint16_t*)dy2, amax, (const uint16_t*)x, (uint16_t*)dx, M,
                                 C, pg, w, mean, invstd, dgamma, dbeta, ws, gw_acc, gb_acc, s);
  else
    bn_pool_backward_t<float>((const float*)dy, (const float*)dy2, amax, (const float*)x, (float*)dx, M, C, pg, w, mean,
                              invstd, dgamma, dbeta, ws, gw_acc, gb_acc, s);
}

}  // namespace gk
