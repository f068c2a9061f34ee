// Fused sparsification pipeline for gfx950.
//
// One compress() call turns a gradient bucket into a packed sparse record
// with no host synchronisation:
//
//   stats   (grid)   acc = g (+ r); r <- acc; g <- 0; per-block sum, sum^2,
//                    sum|x|, max|x|                          [K1+K2, fused]
//   radix   (grid)   3 histogram passes (11/11/10 key bits) for exact top-k,
//                    random-k (hash keys) and DGC            [K6, K8]
//   finalize(1 WG)   reduce statistics, build the candidate-threshold ladder
//                    of the selected mode (or the radix key)  [K3]
//   count   (grid)   per-block counts of |x| > t_j for ALL candidates in one
//                    pass, counters in registers             [K4]
//   decide  (1 WG)   replay the reference's refinement decision tree on the
//                    totals, exclusive scan of per-block counts -> offsets
//   select  (grid)   ballot/popcount block scan, writes ascending indices +
//                    values into the record, zeroes sent entries of r [K5]
//
// The 1-workgroup steps run as their own launches or (handoff = lastblock) in
// the LAST block of the preceding grid pass (last_block(): device-coherent
// partials + a two-level arrival counter, no spin).  With launch hand-offs,
// threshold modes fold the decide and the conditional exact fallback (three
// radix passes, key resolve, second count / decide) into ONE launch,
// decide_fb_kernel, whose grid barriers run only when the fallback fires:
// stats, finalize, count, decide_fb, select -- 5 launches per call (r5c39:
// 125.6 us kernel span on the 25.6 M bucket, from 142.0 us with the decide and
// four early-exit launches).
//
// Reference semantics reproduced (compression.py):
//   gaussian  :358-389  threshold mu + |ppf(ratio/2)| * sigma, <=3 loops
//   gaussian2 :405-435  same, <=5 loops, no residual add
//   redsync   :623-691, redsynctrim :694-738, dgcsampling :555-620
// Deviation (documented in SURVEY 2.3/7.4): the record holds at most k_cap
// entries.  When the reference rule's threshold passes more than k_cap
// entries, decide re-selects by magnitude: the tightest-fitting evaluated
// candidate (the largest count in [2k/3, k_cap] -- a higher threshold, so a
// subset of the largest |x|), or, when no candidate lands there, the exact
// radix key at k_cap (top-k_cap, conditional passes).  The record therefore always
// holds the largest entries; everything unsent stays in the residual, and the
// header's `total` keeps the reference rule's count.
#include <cstdlib>
#include <cstring>

#include "common.h"
#include "gk_kernels.h"

namespace gk {
namespace {

constexpr int kTileElems = kBlock * 16;  // 4 float4 per thread per tile
constexpr int kKeyAbs = 0, kKeyHash = 1, kKeySample = 2;
// calibrated Gaussian-k ladder size: the ladder re-centres every call, so 8
// candidates (the count pass tests each element against every candidate) keep
// the count pass as cheap as the reference ladder's 6
constexpr int kCalCand = 8;
constexpr int kHistSet = kRadixBins0 + kRadixBins1 + kRadixBins2;
// stats->finalize, count->decide, radix2->fallback key, cond count->decide,
// fused-fallback grid barrier, fused-fallback exit
constexpr int kSyncCounters = 6;
// Each arrival counter is two-level: kSyncSub sub-counters (block b counts in
// at sub b % kSyncSub) and one top counter the last arrival of every sub
// counts in at.  Agent-scope atomics on ONE address serialise (~19 ns each,
// 1024 blocks finishing together queue ~20 us behind the last block);
// sub-counters kSyncStride words apart land in different memory channels and
// proceed in parallel: 32 + 32 serial adds instead of 1024.
constexpr int kSyncSub = 32, kSyncStride = 1024;
constexpr int kSyncWords = (kSyncSub + 1) * kSyncStride;   // words per counter

struct Ws {
  double* partials;   // kMaxStatsBlocks * 4
  uint32_t* blockcnt; // kMaxCountBlocks * kMaxCand
  int64_t* offsets;   // kMaxCountBlocks
  int64_t* eqtake;    // kMaxCountBlocks
  int64_t* blocksel;  // kMaxCountBlocks
  uint32_t* hist;     // 2 * kHistSet (set 0: exact/hash, set 1: DGC sample)
  uint32_t* sync;     // kSyncCounters two-level arrival counters of kSyncWords (last-block hand-off), zero between kernels
};

__host__ __device__ inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Partials handed from every block to a last-block reduction go through
// device-coherent (agent-scope) accesses: they bypass the per-XCD L2s, so no
// L2 write-back / invalidate fence is needed around the hand-off.
template <typename T>
__device__ __forceinline__ void st_dev(T* p, T v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
template <typename T>
__device__ __forceinline__ T ld_dev(const T* p) {
  return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Bulk device-coherent reads for the single-workgroup hand-offs (finalize /
// decide / fallback key).  The compiler follows every agent-scope atomic load
// with s_waitcnt vmcnt(0), so a loop of ld_dev() is a chain of serial
// round trips past the XCD's L2 (64 in a row for the decide's block counts:
// most of the count pass's 41 us against select's 25 us over the same data).
// A raw buffer load with the sc1 cache policy is the instruction the atomic
// load becomes, but an ordinary load to the compiler: issued back to back,
// one wait before the first use.  base: wave-uniform array base.
constexpr int kCpolSc1 = 16;   // SC1 (LLVM CPol::SC1)
template <typename T>
__device__ __forceinline__ T ld_coh(const T* base, int idx) {
  static_assert(sizeof(T) == 4 || sizeof(T) == 8, "32- or 64-bit element");
  const auto r = __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(base), (short)0, 0x7fffffff, 0x00020000);
  if constexpr (sizeof(T) == 4) {
    return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b32(r, idx * 4, 0, kCpolSc1));
  } else {
    return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b64(r, idx * 8, 0, kCpolSc1));
  }
}

__host__ __device__ inline Ws carve(void* base) {
  char* p = reinterpret_cast<char*>(base);
  Ws w;
  size_t o = 0;
  w.partials = reinterpret_cast<double*>(p + o); o = align_up(o + sizeof(double) * kMaxStatsBlocks * 4, 256);
  w.blockcnt = reinterpret_cast<uint32_t*>(p + o); o = align_up(o + sizeof(uint32_t) * kMaxCountBlocks * kMaxCand, 256);
  w.offsets = reinterpret_cast<int64_t*>(p + o); o = align_up(o + sizeof(int64_t) * kMaxCountBlocks, 256);
  w.eqtake = reinterpret_cast<int64_t*>(p + o); o = align_up(o + sizeof(int64_t) * kMaxCountBlocks, 256);
  w.blocksel = reinterpret_cast<int64_t*>(p + o); o = align_up(o + sizeof(int64_t) * kMaxCountBlocks, 256);
  w.hist = reinterpret_cast<uint32_t*>(p + o); o = align_up(o + sizeof(uint32_t) * 2 * kHistSet, 256);
  w.sync = reinterpret_cast<uint32_t*>(p + o);
  return w;
}

size_t ws_bytes() {
  size_t o = 0;
  o = align_up(o + sizeof(double) * kMaxStatsBlocks * 4, 256);
  o = align_up(o + sizeof(uint32_t) * kMaxCountBlocks * kMaxCand, 256);
  o = align_up(o + sizeof(int64_t) * kMaxCountBlocks, 256) * 1;
  o = align_up(o + sizeof(int64_t) * kMaxCountBlocks, 256);
  o = align_up(o + sizeof(int64_t) * kMaxCountBlocks, 256);
  o = align_up(o + sizeof(uint32_t) * 2 * kHistSet, 256);
  o += sizeof(uint32_t) * (kSyncCounters * kSyncWords + 2 * 64);   // + fused-fallback flag / generation words
  return align_up(o, 256);
}

// --------------------------------------------------------------------------
// block scans
// --------------------------------------------------------------------------
__device__ __forceinline__ uint64_t wave_incl_scan_u64(uint64_t v) {
  const int l = lane_id();
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    uint64_t o = __shfl_up(v, off, 64);
    if (l >= off) v += o;
  }
  return v;
}

// Exclusive scan over the 256 threads of the block, in thread order.
__device__ __forceinline__ uint64_t block_excl_scan_u64(uint64_t v, uint64_t* sh /*>=4*/, uint64_t* total) {
  const uint64_t inc = wave_incl_scan_u64(v);
  __syncthreads();
  if (lane_id() == 63) sh[wave_id()] = inc;
  __syncthreads();
  uint64_t before = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kWavesPerBlock; ++w) {
    const uint64_t s = sh[w];
    if (w < wave_id()) before += s;
    tot += s;
  }
  *total = tot;
  return before + inc - v;
}

// Exclusive scan of a u32 over the 256 threads of the block, in thread order
// (half the shuffles of the u64 form; for counts bounded by the bucket size).
__device__ __forceinline__ uint32_t block_excl_scan_u32(uint32_t v, uint32_t* sh /*>=4*/, uint32_t* total) {
  uint32_t inc = v;
  const int l = lane_id();
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t o = __shfl_up(inc, off, 64);
    if (l >= off) inc += o;
  }
  __syncthreads();
  if (l == 63) sh[wave_id()] = inc;
  __syncthreads();
  uint32_t before = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kWavesPerBlock; ++w) {
    const uint32_t s = sh[w];
    if (w < wave_id()) before += s;
    tot += s;
  }
  *total = tot;
  return before + inc - v;
}

// Block totals of N (<= 16) per-thread u32 counters through one LDS
// transpose: every thread stores its N values, then thread t sums the 16
// values t % 16 + 16 i of counter t / 16 and the 16 partials of a
// counter (16 consecutive lanes) meet in four shuffle steps -- instead of N
// dependent six-step shuffle chains (wave_sum per counter: 16 x 6 ds_bpermute
// on the decide / count tails).  out[j] (LDS) holds counter j's total on
// return; sh holds N * kBlock words.
template <int N>
__device__ __forceinline__ void block_totals_u32(const uint32_t (&v)[N], uint32_t* sh, uint32_t* out) {
  static_assert(N >= 1 && N <= kBlock / 16, "one 16-thread group per counter");
#pragma unroll
  for (int j = 0; j < N; ++j) sh[j * kBlock + threadIdx.x] = v[j];
  __syncthreads();
  const int j = threadIdx.x >> 4, part = threadIdx.x & 15;
  uint32_t a = 0u;
  if (j < N) {
    // elements part, part + 16, ...: the 16 lanes of a group read 16
    // consecutive words per step (no bank conflicts)
    const uint32_t* p = sh + j * kBlock + part;
#pragma unroll
    for (int i = 0; i < 16; ++i) a += p[16 * i];
  }
#pragma unroll
  for (int off = 8; off > 0; off >>= 1) a += __shfl_xor(a, off, 16);
  if (j < N && part == 0) out[j] = a;
  __syncthreads();
}

// Find the digit holding the kr-th largest key (1-based) in a histogram of
// nbins (multiple of 256, <= 256 kRadixPer).  Result broadcast to every thread.
constexpr int kRadixPer = (kRadixBins0 > kRadixBins1 ? kRadixBins0 : kRadixBins1) / kBlock;
static_assert(kRadixBins2 <= kRadixBins0 && kRadixPer <= 8, "radix bins per thread");
__device__ void radix_find(const uint32_t* hist, int nbins, int64_t kr, uint64_t* sh, int* digit_out,
                           int64_t* kr_out) {
  const int per = nbins / kBlock;   // <= kRadixPer
  const int t = threadIdx.x;
  const int hi = nbins - t * per;
  uint32_t hv[kRadixPer];           // this thread's bins, all loads in flight at once
#pragma unroll
  for (int q = 0; q < kRadixPer; ++q) hv[q] = q < per ? ld_coh(hist, hi - 1 - q) : 0u;
  uint64_t ls = 0;
#pragma unroll
  for (int q = 0; q < kRadixPer; ++q) ls += hv[q];
  uint64_t tot;
  const uint64_t before = block_excl_scan_u64(ls, sh, &tot);
  __shared__ int s_digit;
  __shared__ int64_t s_kr;
  if (t == 0) { s_digit = 0; s_kr = kr; }
  __syncthreads();
  if ((int64_t)before < kr && kr <= (int64_t)(before + ls)) {
    int64_t cum = (int64_t)before;
#pragma unroll
    for (int q = 0; q < kRadixPer; ++q) {
      if (q >= per) break;
      const int d = hi - 1 - q;
      const int64_t h = hv[q];
      if (cum + h >= kr) { s_digit = d; s_kr = kr - cum; break; }
      cum += h;
    }
  }
  __syncthreads();
  *digit_out = s_digit;
  *kr_out = s_kr;
  __syncthreads();
}

__device__ __forceinline__ uint32_t bound_from_threshold(float t) {
  // elements with |x| > t  <=>  abs_key(x) >= bound   (non-NaN x)
  if (!(t >= 0.0f)) {
    if (t < 0.0f) return 0u;          // every element selected
    return 0x7fc00001u;               // NaN threshold: nothing selected
  }
  return (__float_as_uint(t) & 0x7fffffffu) + 1u;
}

// Hash keys rank a uniformly random subset (random-k: the k LARGEST keys are
// taken).  Arena padding slots (valid bit 0) get key 0 and are never picked
// while enough real elements exist.
template <int KEYKIND>
__device__ __forceinline__ uint32_t key_of(int64_t i, float x, uint32_t seed, const uint32_t* valid) {
  if (KEYKIND == kKeyHash) {
    if (valid != nullptr && !((valid[i >> 5] >> (i & 31)) & 1u)) return 0u;
    uint32_t h = hash_u32((uint32_t)i, seed);
    return h == 0xffffffffu ? 0xfffffffeu : (h == 0u ? 1u : h);
  }
  return abs_key(x);
}

template <bool VEC>
__device__ __forceinline__ void load4(const float* __restrict__ p, int64_t e, int64_t n, float v[4]) {
  if (VEC) {
    if (e < n) {
      const float4 f = *reinterpret_cast<const float4*>(p + e);
      v[0] = f.x; v[1] = f.y; v[2] = f.z; v[3] = f.w;
    } else {
      v[0] = v[1] = v[2] = v[3] = 0.f;
    }
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = (e + q < n) ? p[e + q] : 0.f;
  }
}

// --------------------------------------------------------------------------
// Last-block hand-off: every block publishes its partials, then counts itself
// in; the block that arrives last runs the 1-workgroup reduction (finalize /
// decide / fallback key) in place of a separate launch.  No block waits on
// another (no spin), so there is no co-residency requirement.  The counter
// is reset by the last block, ready for the next kernel that uses it.
// --------------------------------------------------------------------------
// The partials are written with st_dev (device-coherent) and read with
// ld_dev; each writer waits for its stores to complete before the block
// counts itself in, so the last block reads every block's values.  (An
// agent-scope release / acquire fence would instead write back / invalidate
// the whole L2 of the XCD -- per block, that costs more than the launch it
// saves: the stats pass leaves every block's slice of r dirty in L2.)
//
// Hardware assumption (gfx950, ROCm 7.2), stated because the C++ memory model
// alone does not give this hand-off a happens-before edge (relaxed RMW): it is
// the first row of the measured-valid table of MI355X_MICROARCH.md
// "Workgroup dispatch, XCD placement & inter-workgroup visibility" --
//   * every handed-off byte is stored `sc1` (st_dev / agent-scope atomics: the
//     per-block partials, block counts and histogram adds) and loaded `sc1`
//     (ld_dev) -- 4- or 8-byte accesses, hipMalloc'd workspace;
//   * every storing wave runs `s_waitcnt vmcnt(0)` after its stores and the
//     workgroup barrier precedes the ONE lane's agent-scope add to ONE
//     unsharded counter;
//   * the workgroup whose add came last (told by the value returned) loads
//     only after its add returned, its other waves after a barrier.
// The asm waitcnt and the barriers also keep the compiler from moving the
// atomic loads / stores across the add.  tests/test_kernels_gpu.py
// (test_last_block_handoff_stress) replays the hand-offs at the largest grid
// sizes, back to back, and checks every header and record against the host.
// Two levels (kSyncSub): the last arrival at a sub-counter resets it and
// counts in at the top counter; the last arrival there is the last block.
// Every add is issued after the adding lane's earlier adds returned, so the
// order above carries over: a block's stores completed -> its sub add -> the
// sub's last add -> the top add -> the last block's loads.
// (one lane) count block `bid` of `G` in at a two-level counter; true for the
// last arrival.  The resets complete (vmcnt) before the next add, so a counter
// reused right after (the fused fallback's grid barriers) never loses an add
// to a late reset store.
__device__ __forceinline__ bool arrive(uint32_t* counter, uint32_t G, uint32_t bid) {
  const uint32_t nsub = G < (uint32_t)kSyncSub ? G : (uint32_t)kSyncSub;
  const uint32_t j = bid % nsub;
  const uint32_t expect = (G - j + nsub - 1) / nsub;   // blocks b with b % nsub == j
  uint32_t* sub = counter + j * kSyncStride;
  const uint32_t prev = __hip_atomic_fetch_add(sub, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  bool last = false;
  if (prev == expect - 1) {
    st_dev(sub, 0u);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint32_t* top = counter + kSyncSub * kSyncStride;
    const uint32_t p2 = __hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = p2 == nsub - 1;
    if (last) {
      st_dev(top, 0u);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  return last;
}

__device__ __forceinline__ bool last_block(uint32_t* counter) {
  __shared__ uint32_t s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this thread's st_dev / atomics completed
  __syncthreads();
  if (threadIdx.x == 0) s_last = arrive(counter, gridDim.x, blockIdx.x) ? 1u : 0u;
  __syncthreads();
  return s_last != 0u;
}

// Live candidates of a mode's threshold ladder: the ONE definition both the
// finalize step (which fills ctrl->bound[0 .. n)) and the host's choice of the
// count kernel's compile-time candidate bound NC (count_cands) read, so a
// ladder cannot grow on one side only (a count pass with NC below the live
// count would report zero for the candidates past NC).
// Gaussian-k: the reference's refinement walk (tri(loops) nodes t0 * 1.5^b *
// 0.5^a) plus, for loops <= 3, kGaussExt overflow-extension thresholds
// above the walk's top node (t_top * 1.25^j, slots kGaussWalk ..): when every
// walk node passes more than k_cap entries (heavy-tailed gradients: the walk
// stops at 2.25 t0 with the count still above 4k/3), the decide step picks the
// extension node with the largest count in [2k/3, k_cap] -- a magnitude-
// correct selection from the same count pass -- instead of running the three
// radix passes of the exact top-k_cap fallback.  The extension is tested only
// for the rare elements above its lowest threshold (count_kernel NX).
constexpr int kGaussWalk = 6, kGaussExt = kMaxCand - kGaussWalk;
constexpr double kGaussExtRatio = 1.25;
__host__ __device__ constexpr int gauss_walk(int loops) {
  return (loops < 1 ? 1 : loops) * ((loops < 1 ? 1 : loops) + 1) / 2 < kMaxCand
             ? (loops < 1 ? 1 : loops) * ((loops < 1 ? 1 : loops) + 1) / 2
             : kMaxCand;
}
__host__ __device__ constexpr bool gauss_ext(int loops) { return gauss_walk(loops) <= kGaussWalk; }
__host__ __device__ constexpr int ladder_cands(int mode, int loops) {
  return mode == kModeGaussian ? (gauss_ext(loops) ? kGaussWalk + kGaussExt : gauss_walk(loops))
         : mode == kModeRedSync ? 7
         : mode == kModeGaussianCal ? kCalCand
         : mode == kModeThreshold ? 1
         : (mode == kModeTopK || mode == kModeRandomK) ? 2
         : mode == kModeDGC ? 3
         : kMaxCand;   // RedSyncTrim: the whole descending-ratio ladder
}
constexpr int kFallbackCands = 2;   // conditional exact-key pass: key > K, key >= K
static_assert(ladder_cands(kModeGaussian, 5) == 15 && ladder_cands(kModeGaussian, 3) == kMaxCand &&
              gauss_walk(3) == kGaussWalk && kGaussExt > 0, "gaussian ladder");
static_assert(ladder_cands(kModeRedSync, 3) <= kMaxCand && kCalCand <= kMaxCand, "ladder sizes");

struct FinArgs {   // finalize_body arguments (stats -> finalize hand-off)
  GkCtrl* ctrl;
  int64_t n;
  int mode, loops;
  double z, fixed_thr;
  int64_t k;
  float* stats_out;
  uint32_t* counter;
};

struct DecArgs {   // decide_body arguments (count -> decide hand-off)
  int in_kernel;     // 1: decide in the count pass's last block; 0: a separate decide_kernel launch
  GkCtrl* ctrl;
  int mode, loops;
  int64_t k, k_cap;
  int64_t* offsets;
  int64_t* eqtake;
  int64_t* blocksel;
  int32_t* hdr;
  uint32_t* hist_reset;
  uint32_t* counter;
};

template <bool BATCH = false>
__device__ __forceinline__ void finalize_body(GkCtrl* __restrict__ ctrl, const double* __restrict__ partials, int nparts, int64_t n,
                              int mode, int loops, double z, double fixed_thr, int64_t k, const uint32_t* hist_exact,
                              const uint32_t* hist_sample, float* stats_out);
__device__ __forceinline__ void decide_body(GkCtrl* __restrict__ gctrl, const uint32_t* __restrict__ blockcnt, int G, int mode,
                            int loops, int64_t k, int64_t k_cap, int64_t* __restrict__ offsets,
                            int64_t* __restrict__ eqtake, int64_t* __restrict__ blocksel, int32_t* __restrict__ hdr,
                            int cond, uint32_t* __restrict__ hist_reset);
__device__ __forceinline__ void cal_fallback_body(GkCtrl* __restrict__ ctrl, const uint32_t* hist_exact, int64_t k);

// --------------------------------------------------------------------------
// K1+K2: residual add + moments (FIN: + finalize in the last block)
// --------------------------------------------------------------------------
// (8 waves per SIMD: the rarely-run finalize call must not set the register
// budget of this streaming kernel)
template <bool VEC, bool EC, bool WRITE_R, bool ZERO_G, bool FIN>
__global__ __launch_bounds__(kBlock, 8) void stats_kernel(float* __restrict__ g, float* __restrict__ r, int64_t n,
                                                       double* __restrict__ partials, FinArgs fa) {
  float s = 0.f, ss = 0.f, sa = 0.f, mx = 0.f;
  const int64_t tid = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  if (VEC) {
    const int64_t n4 = n >> 2;
    float4* g4 = reinterpret_cast<float4*>(g);
    float4* r4 = reinterpret_cast<float4*>(r);
    for (int64_t i = tid; i < n4; i += stride) {
      float4 a = g4[i];
      if (EC) {
        const float4 rv = r4[i];
        a.x += rv.x; a.y += rv.y; a.z += rv.z; a.w += rv.w;
      }
      if (WRITE_R) r4[i] = a;
      if (ZERO_G) g4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      s += (a.x + a.y) + (a.z + a.w);
      ss += (a.x * a.x + a.y * a.y) + (a.z * a.z + a.w * a.w);
      const float ax = fabsf(a.x), ay = fabsf(a.y), az = fabsf(a.z), aw = fabsf(a.w);
      sa += (ax + ay) + (az + aw);
      mx = fmaxf(mx, fmaxf(fmaxf(ax, ay), fmaxf(az, aw)));
    }
  } else {
    for (int64_t i = tid; i < n; i += stride) {
      float a = g[i];
      if (EC) a += r[i];
      if (WRITE_R) r[i] = a;
      if (ZERO_G) g[i] = 0.f;
      s += a;
      ss += a * a;
      sa += fabsf(a);
      mx = fmaxf(mx, fabsf(a));
    }
  }
  __shared__ double sh[kWavesPerBlock];
  __shared__ float shf[kWavesPerBlock];
  const double bs = block_sum((double)s, sh);
  const double bss = block_sum((double)ss, sh);
  const double bsa = block_sum((double)sa, sh);
  const float bmx = block_max(mx, shf);
  if (threadIdx.x == 0) {
    st_dev(&partials[blockIdx.x * 4 + 0], bs);
    st_dev(&partials[blockIdx.x * 4 + 1], bss);
    st_dev(&partials[blockIdx.x * 4 + 2], bsa);
    st_dev(&partials[blockIdx.x * 4 + 3], (double)bmx);
  }
  if (FIN && last_block(fa.counter))
    finalize_body(fa.ctrl, partials, (int)gridDim.x, fa.n, fa.mode, fa.loops, fa.z, fa.fixed_thr, fa.k, nullptr,
                  nullptr, fa.stats_out);
}

// DGC momentum correction fused into K1+K2: one pass reads u, g, w, r and
// writes u, r, g:  u = mu*u + (g + wd*w);  acc = u (+ r);  r = acc;  g = 0,
// with the moments of acc.  Replaces momentum_correct (u, g, w -> u, g) plus
// stats (g, r -> r, g): 9 -> 7 arena streams.  Per-chunk hyper-parameters
// (param groups); chunks are 64-element aligned, so every access is a float4.
struct McHyper {
  float mu[8];
  float wd[8];
};

template <bool EC, bool FIN>
__global__ __launch_bounds__(kBlock, 8) void mc_stats_kernel(float* __restrict__ g, float* __restrict__ r,
                                                          float* __restrict__ u, const float* __restrict__ w,
                                                          const Chunk* __restrict__ chunks, int nchunks,
                                                          int64_t base, McHyper hp, double* __restrict__ partials,
                                                          FinArgs fa) {
  float s = 0.f, ss = 0.f, sa = 0.f, mx = 0.f;
  for (int ci = blockIdx.x; ci < nchunks; ci += gridDim.x) {
    const Chunk c = chunks[ci];
    const float mu = hp.mu[c.group], wd = hp.wd[c.group];
    const int64_t off = c.start - base;
    float4* g4 = reinterpret_cast<float4*>(g + off);
    float4* r4 = reinterpret_cast<float4*>(r + off);
    float4* u4 = reinterpret_cast<float4*>(u + off);
    const float4* w4 = reinterpret_cast<const float4*>(w + off);
    const int n4 = c.len >> 2;
    for (int i = threadIdx.x; i < n4; i += kBlock) {
      float4 uv = u4[i];
      const float4 gv = g4[i];
      const float4 wv = w4[i];
      uv.x = fmaf(mu, uv.x, fmaf(wd, wv.x, gv.x));
      uv.y = fmaf(mu, uv.y, fmaf(wd, wv.y, gv.y));
      uv.z = fmaf(mu, uv.z, fmaf(wd, wv.z, gv.z));
      uv.w = fmaf(mu, uv.w, fmaf(wd, wv.w, gv.w));
      u4[i] = uv;
      float4 a = uv;
      if (EC) {
        const float4 rv = r4[i];
        a.x += rv.x; a.y += rv.y; a.z += rv.z; a.w += rv.w;
      }
      r4[i] = a;
      g4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      s += (a.x + a.y) + (a.z + a.w);
      ss += (a.x * a.x + a.y * a.y) + (a.z * a.z + a.w * a.w);
      const float ax = fabsf(a.x), ay = fabsf(a.y), az = fabsf(a.z), aw = fabsf(a.w);
      sa += (ax + ay) + (az + aw);
      mx = fmaxf(mx, fmaxf(fmaxf(ax, ay), fmaxf(az, aw)));
    }
  }
  __shared__ double sh[kWavesPerBlock];
  __shared__ float shf[kWavesPerBlock];
  const double bs = block_sum((double)s, sh);
  const double bss = block_sum((double)ss, sh);
  const double bsa = block_sum((double)sa, sh);
  const float bmx = block_max(mx, shf);
  if (threadIdx.x == 0) {
    st_dev(&partials[blockIdx.x * 4 + 0], bs);
    st_dev(&partials[blockIdx.x * 4 + 1], bss);
    st_dev(&partials[blockIdx.x * 4 + 2], bsa);
    st_dev(&partials[blockIdx.x * 4 + 3], (double)bmx);
  }
  if (FIN && last_block(fa.counter))
    finalize_body(fa.ctrl, partials, (int)gridDim.x, fa.n, fa.mode, fa.loops, fa.z, fa.fixed_thr, fa.k, nullptr,
                  nullptr, fa.stats_out);
}

// --------------------------------------------------------------------------
// radix histogram passes
// --------------------------------------------------------------------------
template <int PASS>
__device__ __forceinline__ uint32_t radix_digit(uint32_t key) {
  if (PASS == 0) return key >> 21;
  if (PASS == 1) return (key >> 10) & 0x7ffu;
  return key & 0x3ffu;
}

// One histogram pass over the grid-stride slice of block `bid` of `nblk`
// (radix_hist_kernel, and the fused conditional fallback of decide_fb_kernel).
// sh: kWavesPerBlock x (the pass's bins) words of LDS, one copy per wave.
constexpr int kRadixShWords = kWavesPerBlock * (kRadixBins0 > kRadixBins1 ? kRadixBins0 : kRadixBins1);
template <int PASS, int KEYKIND, bool VEC>
__device__ __forceinline__ void radix_hist_body(const float* __restrict__ x, int64_t n, uint32_t seed,
                                                uint32_t sample_thr, int64_t k, uint32_t* hist_set,
                                                const uint32_t* __restrict__ valid, int bid, int nblk,
                                                uint32_t* sh) {
  constexpr int NB = PASS == 0 ? kRadixBins0 : (PASS == 1 ? kRadixBins1 : kRadixBins2);
  static_assert(kWavesPerBlock * NB <= kRadixShWords, "radix LDS");
  __shared__ uint64_t sh_scan[kWavesPerBlock];
  uint32_t* hist0 = hist_set;
  uint32_t* hist1 = hist_set + kRadixBins0;
  uint32_t* hist2 = hist1 + kRadixBins1;
  uint32_t prefix = 0;
  if (PASS >= 1) {
    // eligible total (DGC sample size) and k_eff
    uint64_t loc = 0;
    {
      uint32_t hv[kRadixBins0 / kBlock];   // all loads in flight before the adds
#pragma unroll
      for (int q = 0; q < kRadixBins0 / kBlock; ++q) hv[q] = ld_coh(hist0, threadIdx.x + q * kBlock);
#pragma unroll
      for (int q = 0; q < kRadixBins0 / kBlock; ++q) loc += hv[q];
    }
    uint64_t tot;
    (void)block_excl_scan_u64(loc, sh_scan, &tot);
    int64_t kr = k < (int64_t)tot ? k : (int64_t)tot;
    if (kr < 1) kr = 1;
    int d0; int64_t kr1;
    radix_find(hist0, kRadixBins0, kr, sh_scan, &d0, &kr1);
    prefix = (uint32_t)d0;
    if (PASS == 2) {
      int d1; int64_t kr2;
      radix_find(hist1, kRadixBins1, kr1, sh_scan, &d1, &kr2);
      prefix = (prefix << 11) | (uint32_t)d1;
    }
  }
  for (int i = threadIdx.x; i < kWavesPerBlock * NB; i += kBlock) sh[i] = 0u;
  __syncthreads();
  uint32_t* my = sh + wave_id() * NB;
  const int64_t tid = (int64_t)bid * kBlock + threadIdx.x;
  const int64_t stride = (int64_t)nblk * kBlock;
  const int64_t n4 = (n + 3) >> 2;
  for (int64_t i4 = tid; i4 < n4; i4 += stride) {
    const int64_t e = i4 << 2;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    if (KEYKIND != kKeyHash) load4<VEC>(x, e, n, v);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t idx = e + q;
      if (idx >= n) continue;
      uint32_t key;
      if (KEYKIND == kKeySample) {
        if (hash_u32((uint32_t)idx, seed) >= sample_thr) continue;
        key = abs_key(v[q]) + 1u;
      } else {
        key = key_of<KEYKIND>(idx, v[q], seed, valid);
      }
      bool elig = true;
      if (PASS == 1) elig = (key >> 21) == prefix;
      if (PASS == 2) elig = (key >> 10) == prefix;
      if (elig) atomicAdd(&my[radix_digit<PASS>(key)], 1u);
    }
  }
  __syncthreads();
  uint32_t* out = PASS == 0 ? hist0 : (PASS == 1 ? hist1 : hist2);
  for (int b = threadIdx.x; b < NB; b += kBlock) {
    const uint32_t c = sh[b] + sh[NB + b] + sh[2 * NB + b] + sh[3 * NB + b];
    if (c) atomicAdd(&out[b], c);
  }
  __syncthreads();   // the LDS copies are reused by the next pass (fused fallback)
}

template <int PASS, int KEYKIND, bool VEC, bool FB = false>
__global__ __launch_bounds__(kBlock) void radix_hist_kernel(const float* __restrict__ x, int64_t n, uint32_t seed,
                                                            uint32_t sample_thr, int64_t k, uint32_t* hist_set,
                                                            const uint32_t* __restrict__ valid,
                                                            GkCtrl* __restrict__ cond,
                                                            const uint32_t* __restrict__ seed_dev,
                                                            uint32_t* __restrict__ fb_counter = nullptr) {
  if (cond != nullptr && cond->fallback == 0) return;   // conditional pass (calibrated mode), grid-uniform
  if (seed_dev != nullptr) seed = __builtin_amdgcn_readfirstlane(*seed_dev);
  constexpr int NB = PASS == 0 ? kRadixBins0 : (PASS == 1 ? kRadixBins1 : kRadixBins2);
  __shared__ uint32_t sh_hist[kWavesPerBlock * NB];
  radix_hist_body<PASS, KEYKIND, VEC>(x, n, seed, sample_thr, k, hist_set, valid, (int)blockIdx.x, (int)gridDim.x,
                                      sh_hist);
  // conditional chain: the last block of pass 2 resolves the fallback key
  if (FB && PASS == 2 && last_block(fb_counter)) cal_fallback_body(cond, hist_set, k);
}

// Derive the final key (k-th largest) and the tie quota from three hists.
__device__ void radix_resolve(const uint32_t* hist_set, int64_t k, uint64_t* sh, uint32_t* key_out,
                              int64_t* kremain_out, int64_t* keff_out) {
  const uint32_t* hist0 = hist_set;
  const uint32_t* hist1 = hist_set + kRadixBins0;
  const uint32_t* hist2 = hist1 + kRadixBins1;
  uint64_t loc = 0;
  {
      uint32_t hv[kRadixBins0 / kBlock];   // all loads in flight before the adds
#pragma unroll
      for (int q = 0; q < kRadixBins0 / kBlock; ++q) hv[q] = ld_coh(hist0, threadIdx.x + q * kBlock);
#pragma unroll
      for (int q = 0; q < kRadixBins0 / kBlock; ++q) loc += hv[q];
    }
  uint64_t tot;
  (void)block_excl_scan_u64(loc, sh, &tot);
  int64_t keff = k < (int64_t)tot ? k : (int64_t)tot;
  int64_t kr = keff < 1 ? 1 : keff;
  int d0, d1, d2;
  int64_t kr1, kr2, kr3;
  radix_find(hist0, kRadixBins0, kr, sh, &d0, &kr1);
  radix_find(hist1, kRadixBins1, kr1, sh, &d1, &kr2);
  radix_find(hist2, kRadixBins2, kr2, sh, &d2, &kr3);
  *key_out = ((uint32_t)d0 << 21) | ((uint32_t)d1 << 10) | (uint32_t)d2;
  *kremain_out = kr3;
  *keff_out = keff;
}

// --------------------------------------------------------------------------
// finalize: statistics + candidate ladder (1 workgroup)
// --------------------------------------------------------------------------
template <bool BATCH>
__device__ __forceinline__ void finalize_body(GkCtrl* __restrict__ ctrl, const double* __restrict__ partials, int nparts, int64_t n,
                              int mode, int loops, double z, double fixed_thr, int64_t k, const uint32_t* hist_exact,
                              const uint32_t* hist_sample, float* stats_out) {
  __shared__ double sh[kWavesPerBlock];
  __shared__ float shf[kWavesPerBlock];
  __shared__ uint64_t sh_scan[kWavesPerBlock];
  double s = 0, ss = 0, sa = 0;
  float mx = 0.f;
  if (BATCH) {
    // finalize_kernel (its own launch, full register file): every partial row
    // of this thread in flight at once, one round trip
    constexpr int kRows = kMaxStatsBlocks / kBlock;
    double v[kRows][4];
#pragma unroll
    for (int i = 0; i < kRows; ++i) {
      const int b = threadIdx.x + i * kBlock;
#pragma unroll
      for (int c = 0; c < 4; ++c) v[i][c] = b < nparts ? ld_coh(partials, b * 4 + c) : 0.0;
    }
#pragma unroll
    for (int i = 0; i < kRows; ++i) {
      s += v[i][0];
      ss += v[i][1];
      sa += v[i][2];
      mx = fmaxf(mx, (float)v[i][3]);
    }
  } else {
    // in the stats pass's last block: a partial row's four loads in flight
    // before the adds (two rows per step spill at the 64-VGPR budget)
    for (int b = threadIdx.x; b < nparts; b += kBlock) {
      double v[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) v[c] = ld_coh(partials, b * 4 + c);
      s += v[0];
      ss += v[1];
      sa += v[2];
      mx = fmaxf(mx, (float)v[3]);
    }
  }
  if (BATCH) {
    // the three sums and the max through one LDS transpose (thread t reduces
    // 16 values of quantity t / 16; 16-lane groups meet in four shuffle
    // steps) instead of three block_sum + block_max shuffle chains
    __shared__ __attribute__((aligned(16))) double sh_q[4 * kBlock];
    __shared__ double s_q[4];
    sh_q[threadIdx.x] = s;
    sh_q[kBlock + threadIdx.x] = ss;
    sh_q[2 * kBlock + threadIdx.x] = sa;
    sh_q[3 * kBlock + threadIdx.x] = (double)mx;
    __syncthreads();
    const int qi = threadIdx.x >> 4, part = threadIdx.x & 15;
    double a = 0.0;
    if (qi < 4) {
      const double* p = sh_q + qi * kBlock + part;   // elements part + 16 i: conflict-free
      double t[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) t[i] = p[16 * i];
      a = t[0];
#pragma unroll
      for (int i = 1; i < 16; ++i) a = qi == 3 ? fmax(a, t[i]) : a + t[i];
    }
#pragma unroll
    for (int off = 8; off > 0; off >>= 1) {
      const double o = __shfl_xor(a, off, 16);
      a = qi == 3 ? fmax(a, o) : a + o;
    }
    if (qi < 4 && part == 0) s_q[qi] = a;
    __syncthreads();
    s = s_q[0];
    ss = s_q[1];
    sa = s_q[2];
    mx = (float)s_q[3];
  } else {
    s = block_sum(s, sh);
    ss = block_sum(ss, sh);
    sa = block_sum(sa, sh);
    mx = block_max(mx, shf);
  }

  uint32_t rkey[2] = {0u, 0u};
  int64_t rkrem[2] = {0, 0}, rkeff[2] = {0, 0};
  if (mode == kModeTopK || mode == kModeRandomK || mode == kModeDGC)
    radix_resolve(hist_exact, k, sh_scan, &rkey[1], &rkrem[1], &rkeff[1]);
  if (mode == kModeDGC) radix_resolve(hist_sample, k, sh_scan, &rkey[0], &rkrem[0], &rkeff[0]);

  if (threadIdx.x != 0) return;
  const double nd = (double)n;
  const double mean = s / nd;
  const double var = (ss - s * s / nd) / (nd - 1.0);
  const double stdev = sqrt(var > 0.0 ? var : 0.0);
  const double meanabs = sa / nd;
  ctrl->raw[0] = s; ctrl->raw[1] = ss; ctrl->raw[2] = sa; ctrl->raw[3] = (double)mx;
  ctrl->mean = mean; ctrl->stdev = stdev; ctrl->meanabs = meanabs; ctrl->maxabs = (double)mx;
  if (stats_out) {
    stats_out[0] = (float)mean; stats_out[1] = (float)stdev; stats_out[2] = (float)meanabs; stats_out[3] = mx;
  }
  for (int j = 0; j < kMaxCand; ++j) { ctrl->bound[j] = 0xffffffffu; ctrl->cand_thr[j] = 0.0; }
  int nc = 0;
  if (mode == kModeGaussian) {
    // candidates t0 * 1.5^b * 0.5^a for a + b <= loops - 1, index tri(a+b) + b
    const double t0 = mean + z * stdev;
    for (int sdeg = 0; sdeg < loops; ++sdeg) {
      for (int b = 0; b <= sdeg; ++b) {
        const int a = sdeg - b;
        double t = t0;
        for (int q = 0; q < b; ++q) t *= 1.5;
        for (int q = 0; q < a; ++q) t *= 0.5;
        if (nc < kMaxCand) {
          ctrl->bound[nc] = bound_from_threshold((float)t);
          ctrl->cand_thr[nc] = t;
        }
        ++nc;
      }
    }
    if (gauss_ext(loops)) {
      // overflow extension (see ladder_cands); slots nc .. kGaussWalk stay dead
      double t = t0;
      for (int q = 0; q < (loops < 1 ? 1 : loops) - 1; ++q) t *= 1.5;
      for (int j = 0; j < kGaussExt; ++j) {
        t *= kGaussExtRatio;
        ctrl->bound[kGaussWalk + j] = bound_from_threshold((float)t);
        ctrl->cand_thr[kGaussWalk + j] = t;
      }
    }
  } else if (mode == kModeRedSync || mode == kModeRedSyncTrim) {
    const float mean_val = (float)meanabs;
    const float max_val = mx;
    const float diff = __fsub_rn(max_val, mean_val);
    if (mode == kModeRedSync) {
      // heap-ordered binary-search tree of ratios, depth 3 (r - l halves 1 -> 0.125)
      double lo[7], hi[7];
      lo[0] = 0.0; hi[0] = 1.0;
      for (int i = 0; i < 7; ++i) {
        const double mid = lo[i] + (hi[i] - lo[i]) / 2;
        const float t = __fadd_rn(mean_val, __fmul_rn((float)mid, diff));
        ctrl->bound[i] = bound_from_threshold(t);
        ctrl->cand_thr[i] = (double)t;
        if (2 * i + 2 < 7) {
          lo[2 * i + 1] = lo[i]; hi[2 * i + 1] = mid;   // nnz < k/2: r = mid
          lo[2 * i + 2] = mid;   hi[2 * i + 2] = hi[i]; // otherwise: l = mid
        }
      }
      nc = 7;
    } else {
      double ratio = 1.0 - 0.2;
      for (int j = 0; j < kMaxCand; ++j) {
        const float t = __fadd_rn(mean_val, __fmul_rn((float)ratio, diff));
        ctrl->bound[j] = bound_from_threshold(t);
        ctrl->cand_thr[j] = (double)t;
        ratio = ratio - 0.2;
      }
      nc = kMaxCand;
    }
  } else if (mode == kModeGaussianCal) {
    // kCalCand thresholds t_c * exp(step * (j - 3.5)), ascending in j.  The centre
    // t_c = cal_c * sigma and the spacing persist per bucket (decide_kernel
    // re-centres on the best candidate and adapts the spacing to the local
    // slope of the count curve); first call / new k: the Gaussian estimate.
    if (ctrl->cal_k != k || !(ctrl->cal_c > 0.0) || !(ctrl->cal_step > 0.0)) {
      const double t0 = mean + z * stdev;
      ctrl->cal_c = stdev > 0.0 && t0 > 0.0 ? t0 / stdev : (z > 0.0 ? z : 1.0);
      ctrl->cal_step = 0.105;   // ~ln(1.11): neighbours ~1.3x apart in count on a Gaussian at 3.3 sigma
      ctrl->cal_k = k;
    }
    const double tc = ctrl->cal_c * stdev;
    for (int j = 0; j < kCalCand; ++j) {
      const double t = tc * exp(ctrl->cal_step * ((double)j - 0.5 * (kCalCand - 1)));
      ctrl->bound[j] = bound_from_threshold((float)t);
      ctrl->cand_thr[j] = t;
    }
    nc = kCalCand;
  } else if (mode == kModeThreshold) {
    ctrl->bound[0] = bound_from_threshold((float)fixed_thr);
    ctrl->cand_thr[0] = fixed_thr;
    nc = 1;
  } else if (mode == kModeTopK || mode == kModeRandomK) {
    ctrl->bound[0] = rkey[1] + 1u;  // key > K
    ctrl->bound[1] = rkey[1];       // key >= K
    ctrl->cand_thr[0] = (double)__uint_as_float(rkey[1] & 0x7fffffffu);
    nc = 2;
  } else if (mode == kModeDGC) {
    // sampled keys are abs_key + 1: |x| > thr  <=>  abs_key >= Ks
    ctrl->bound[0] = rkey[0];
    ctrl->bound[1] = rkey[1] + 1u;
    ctrl->bound[2] = rkey[1];
    ctrl->cand_thr[0] = rkey[0] ? (double)__uint_as_float(rkey[0] - 1u) : 0.0;
    ctrl->cand_thr[1] = (double)__uint_as_float(rkey[1] & 0x7fffffffu);
    nc = 3;
  }
  (void)nc;
  ctrl->ncand = ladder_cands(mode, loops);   // == the ladder filled above (shared with count_cands)
  ctrl->radix_key[0] = rkey[0]; ctrl->radix_key[1] = rkey[1];
  ctrl->radix_kremain[0] = rkrem[0]; ctrl->radix_kremain[1] = rkrem[1];
  ctrl->k_eff = rkeff[1];
  ctrl->fallback = 0;
  ctrl->ref_total = -1;
}

__global__ __launch_bounds__(kBlock) void finalize_kernel(GkCtrl* __restrict__ ctrl, const double* __restrict__ partials,
                                                          int nparts, int64_t n, int mode, int loops, double z,
                                                          double fixed_thr, int64_t k, const uint32_t* hist_exact,
                                                          const uint32_t* hist_sample, float* stats_out) {
  finalize_body<true>(ctrl, partials, nparts, n, mode, loops, z, fixed_thr, k, hist_exact, hist_sample, stats_out);
}

// Calibrated mode with no candidate in [2k/3, 4k/3] (k = k_eff), or a
// threshold mode whose every candidate overflows k_cap (k = k_cap): resolve
// the exact radix key (k-th largest |x|) from the conditional histogram
// passes; the second count /
// decide / select then run exactly as in top-k mode.
__device__ __forceinline__ void cal_fallback_body(GkCtrl* __restrict__ ctrl, const uint32_t* hist_exact, int64_t k) {
  if (ctrl->fallback == 0) return;
  __shared__ uint64_t sh_scan[kWavesPerBlock];
  uint32_t key;
  int64_t krem, keff;
  radix_resolve(hist_exact, k, sh_scan, &key, &krem, &keff);
  if (threadIdx.x != 0) return;
  for (int j = 0; j < kMaxCand; ++j) ctrl->bound[j] = 0xffffffffu;
  ctrl->bound[0] = key + 1u;  // key > K
  ctrl->bound[1] = key;       // key >= K
  ctrl->ncand = kFallbackCands;
  ctrl->radix_key[1] = key;
  ctrl->radix_kremain[1] = krem;
  ctrl->k_eff = keff;
  ctrl->cand_thr[0] = (double)__uint_as_float(key & 0x7fffffffu);
}

// --------------------------------------------------------------------------
// K4: one-pass multi-threshold count (counters in registers)
// --------------------------------------------------------------------------
// Block `bid`'s tile chunk: per-candidate counts -> blockcnt row bid (and the
// lane-max sketch).  The candidate bounds are read device-coherent (the fused
// fallback writes them inside the same grid).
template <int KEYKIND, bool VEC, int NC, int NX>
__device__ __forceinline__ void count_body(const float* __restrict__ x, int64_t n, uint32_t seed,
                                           const GkCtrl* __restrict__ ctrl, int64_t chunk_tiles,
                                           uint32_t* __restrict__ blockcnt, const uint32_t* __restrict__ valid,
                                           int bid) {
  // Per-lane counters, summed over the wave once per block.  |x| keys are
  // < 2^31, so [key < b] is the sign bit of key - b (b <= 2^31): one v_sub +
  // one v_lshr_add per (element, candidate), independent chains, and
  // count(key >= b) = in-range elements - count(key < b).  (A compare +
  // carry-in add -- v_cmp + v_addc -- chains every candidate through VCC with
  // a wait state per pair: 45 us for the 6-candidate Gaussian ladder on a
  // 25.6 M bucket, ~5 us per candidate; round 3's ballots on the scalar unit
  // were 40 us.)  Hash / sample keys span 32 bits and keep the compare.  NC
  // (>= the live candidate count, chosen by the host from the mode) is a
  // compile-time bound: no per-test branch; dead candidates carry bound
  // 0xffffffff and count nothing.
  constexpr bool SIGN = KEYKIND == kKeyAbs;
  uint32_t bnd[NC];
#pragma unroll
  for (int j = 0; j < NC; ++j) bnd[j] = __builtin_amdgcn_readfirstlane(ld_coh(ctrl->bound, j));
  uint32_t cnt[NC];   // SIGN: elements below bound j; else: elements at or above it
#pragma unroll
  for (int j = 0; j < NC; ++j) cnt[j] = 0u;
  uint32_t nin = 0u;  // SIGN: in-range elements of this lane
  // NX ascending extension candidates (bound[NC ..]): tested only when one of
  // a float4's elements is above the lowest of them (a branch that is almost
  // never taken for a Gaussian-k overflow ladder)
  constexpr int NXA = NX > 0 ? NX : 1;
  uint32_t xb[NXA], xc[NXA];
#pragma unroll
  for (int j = 0; j < NXA; ++j) {
    xb[j] = NX > 0 ? __builtin_amdgcn_readfirstlane(ld_coh(ctrl->bound, NC + j)) : 0xffffffffu;
    xc[j] = 0u;
  }
  auto test_ext = [&](uint32_t key, bool in) {
#pragma unroll
    for (int j = 0; j < NXA; ++j) xc[j] += (in && key >= xb[j]) ? 1u : 0u;
  };
  auto test = [&](uint32_t key, bool in) {
    if constexpr (SIGN) {
      nin += in ? 1u : 0u;
#pragma unroll
      for (int j = 0; j < NC; ++j) cnt[j] += in ? (key - bnd[j]) >> 31 : 0u;
    } else {
#pragma unroll
      for (int j = 0; j < NC; ++j) cnt[j] += (in && key >= bnd[j]) ? 1u : 0u;
    }
    if (NX > 0 && in && key >= xb[0]) test_ext(key, true);
  };
  const int64_t ntiles = (n + kTileElems - 1) / kTileElems;
  const int64_t t0 = (int64_t)bid * chunk_tiles;
  const int64_t t1 = t0 + chunk_tiles < ntiles ? t0 + chunk_tiles : ntiles;
  int64_t tile = t0;
  if (VEC && KEYKIND != kKeyHash) {
    // full tiles, two tiles of loads in flight: buffers a / b alternate
    // without register copies (a copy of a load's destination would wait for
    // it), so testing tile t waits for its own four float4 only
    // (vmcnt(4): tile t + 1's are still in flight).  One tile ahead measured
    // 47 us on the 25.6 M bucket (2.2 TB/s): the wait at each tile boundary
    // drained the only outstanding loads.
    const int64_t nfull = n / kTileElems;
    const int64_t tf = t1 < nfull ? t1 : nfull;
    if (tile < tf) {
      const float4* p = reinterpret_cast<const float4*>(x) + threadIdx.x;
      float4 ba[4], bb[4];
      auto ld = [&](int64_t t, float4* b) {
#pragma unroll
        for (int j4 = 0; j4 < 4; ++j4) b[j4] = p[t * (kTileElems / 4) + j4 * kBlock];
      };
      auto run = [&](const float4* b) {
#pragma unroll
        for (int j4 = 0; j4 < 4; ++j4) {
          const uint32_t k4[4] = {abs_key(b[j4].x), abs_key(b[j4].y), abs_key(b[j4].z), abs_key(b[j4].w)};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            if constexpr (SIGN) {
#pragma unroll
              for (int j = 0; j < NC; ++j) cnt[j] += (k4[q] - bnd[j]) >> 31;
            } else {
#pragma unroll
              for (int j = 0; j < NC; ++j) cnt[j] += k4[q] >= bnd[j] ? 1u : 0u;
            }
          }
          if constexpr (NX > 0) {   // one guard per float4
            const uint32_t m = max(max(k4[0], k4[1]), max(k4[2], k4[3]));
            if (m >= xb[0]) {
#pragma unroll
              for (int q = 0; q < 4; ++q) test_ext(k4[q], true);
            }
          }
        }
        nin += 16u;
      };
      ld(tile, ba);
      if (tile + 1 < tf) ld(tile + 1, bb);
      for (; tile < tf; tile += 2) {
        run(ba);
        if (tile + 2 < tf) ld(tile + 2, ba);
        if (tile + 1 < tf) {
          run(bb);
          if (tile + 3 < tf) ld(tile + 3, bb);
        }
      }
      tile = tf;
    }
  }
  for (; tile < t1; ++tile) {
    const int64_t base = tile * kTileElems;
    uint32_t key[16];
    uint32_t inb = 0xffffu;         // in-range bits of this thread's 16 elements
    if (base + kTileElems <= n) {   // full tile (block-uniform): no bounds tests
#pragma unroll
      for (int j4 = 0; j4 < 4; ++j4) {
        const int64_t e = base + j4 * (kBlock * 4) + threadIdx.x * 4;
        float v[4] = {0.f, 0.f, 0.f, 0.f};
        if (KEYKIND != kKeyHash) {
          if (VEC) {
            const float4 f = *reinterpret_cast<const float4*>(x + e);
            v[0] = f.x; v[1] = f.y; v[2] = f.z; v[3] = f.w;
          } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = x[e + q];
          }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) key[j4 * 4 + q] = key_of<KEYKIND>(e + q, v[q], seed, valid);
      }
    } else {
#pragma unroll
      for (int j4 = 0; j4 < 4; ++j4) {
        const int64_t e = base + j4 * (kBlock * 4) + threadIdx.x * 4;
        float v[4] = {0.f, 0.f, 0.f, 0.f};
        if (KEYKIND != kKeyHash) load4<VEC>(x, e, n, v);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const bool in = e + q < n;
          key[j4 * 4 + q] = in ? key_of<KEYKIND>(e + q, v[q], seed, valid) : 0u;
          if (!in) inb &= ~(1u << (j4 * 4 + q));
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) test(key[q], (inb >> q) & 1u);
  }
  if constexpr (SIGN) {
#pragma unroll
    for (int j = 0; j < NC; ++j) cnt[j] = bnd[j] == 0xffffffffu ? 0u : nin - cnt[j];
  }
  // per-lane counts -> block totals (one LDS transpose per block)
  static_assert(NC + NX <= kMaxCand, "candidate slots");
  uint32_t all[NC + NX];
#pragma unroll
  for (int j = 0; j < NC; ++j) all[j] = cnt[j];
#pragma unroll
  for (int j = 0; j < NX; ++j) all[NC + j] = xc[j];
  __shared__ __attribute__((aligned(16))) uint32_t sh[(NC + NX) * kBlock];
  __shared__ uint32_t s_bt[kMaxCand];
  block_totals_u32<NC + NX>(all, sh, s_bt);
  if (threadIdx.x < kMaxCand) {
    const int j = threadIdx.x;
    st_dev(&blockcnt[bid * kMaxCand + j], j < NC + NX ? s_bt[j] : 0u);
  }
}

template <int KEYKIND, bool VEC, int NC, int NX = 0, bool DEC = true>
__global__ __launch_bounds__(kBlock) void count_kernel(const float* __restrict__ x, int64_t n, uint32_t seed,
                                                       GkCtrl* __restrict__ ctrl, int64_t chunk_tiles,
                                                       uint32_t* __restrict__ blockcnt,
                                                       const uint32_t* __restrict__ valid, int cond,
                                                       const uint32_t* __restrict__ seed_dev, DecArgs da) {
  if (cond && ctrl->fallback == 0) return;
  if (seed_dev != nullptr) seed = __builtin_amdgcn_readfirstlane(*seed_dev);
  count_body<KEYKIND, VEC, NC, NX>(x, n, seed, ctrl, chunk_tiles, blockcnt, valid, (int)blockIdx.x);
  if constexpr (DEC) {   // decide on the totals in the last block (else: decide_kernel after this grid)
    if (last_block(da.counter))
      decide_body(ctrl, blockcnt, (int)gridDim.x, da.mode, da.loops, da.k, da.k_cap, da.offsets, da.eqtake,
                  da.blocksel, da.hdr, cond, da.hist_reset);
  }
}

// the decide as its own 1-workgroup launch (hand-off by kernel boundary)
__global__ __launch_bounds__(kBlock) void decide_kernel(const uint32_t* __restrict__ blockcnt, int G, int cond,
                                                        DecArgs da) {
  decide_body(da.ctrl, blockcnt, G, da.mode, da.loops, da.k, da.k_cap, da.offsets, da.eqtake, da.blocksel, da.hdr,
              cond, da.hist_reset);
}

// --------------------------------------------------------------------------
// decide: replay the reference decision tree, offsets per block (1 WG)
// --------------------------------------------------------------------------
__device__ __forceinline__ void decide_body(GkCtrl* __restrict__ gctrl, const uint32_t* __restrict__ blockcnt, int G, int mode,
                            int loops, int64_t k, int64_t k_cap, int64_t* __restrict__ offsets,
                            int64_t* __restrict__ eqtake, int64_t* __restrict__ blocksel, int32_t* __restrict__ hdr,
                            int cond, uint32_t* __restrict__ hist_reset) {
  __shared__ uint64_t sh_scan[kWavesPerBlock];
  __shared__ int s_chosen, s_gt, s_ge, s_stop;
  __shared__ int64_t s_quota, s_ref_total;
  __shared__ float s_thr;
  __shared__ __attribute__((aligned(16))) GkCtrl s_ctrl;
  // ONE batch of loads, then no global read: the control block into an LDS
  // snapshot (one dword per thread; every ctrl read below is an LDS read and
  // the fields the decision writes go back to global after it) and this
  // thread's kPer block rows of counts into registers (totals AND offsets).
  // Loaded one dependent round trip at a time this step took 16 us on the
  // 892-block count grid (its own launch, r4c12), ~2/3 of it waiting.
  constexpr int kCw = (int)(sizeof(GkCtrl) / 4);
  static_assert(sizeof(GkCtrl) % 4 == 0 && kCw <= kBlock, "ctrl snapshot: one dword per thread");
  constexpr int kPer = kMaxCountBlocks / kBlock;   // each thread owns kPer consecutive blocks
  const uint32_t cw = threadIdx.x < kCw ? ld_coh(reinterpret_cast<const uint32_t*>(gctrl), (int)threadIdx.x) : 0u;
  uint32_t row[kPer][kMaxCand];
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    const int b = threadIdx.x * kPer + q;
#pragma unroll
    for (int j = 0; j < kMaxCand; ++j) row[q][j] = b < G ? ld_coh(blockcnt, b * kMaxCand + j) : 0u;
  }
  if (threadIdx.x < kCw) reinterpret_cast<uint32_t*>(&s_ctrl)[threadIdx.x] = cw;
  __syncthreads();
  // read-only snapshot: everything the decision changes goes through `dec`
  // and is written back to gctrl below (a write to the snapshot, which would
  // be silently dropped, does not compile)
  const GkCtrl* ctrl = &s_ctrl;
  if (cond) {
    if (ctrl->fallback == 0) return;
    mode = kModeTopK;   // second decide of a fallback: exact top-k (or top-k_cap) on the radix key
  }
  const int nc = ctrl->ncand;
  // totals per candidate (u32: a candidate's count is at most the bucket
  // size, < 2^31 elements) through one LDS transpose
  uint32_t loc[kMaxCand];
#pragma unroll
  for (int j = 0; j < kMaxCand; ++j) {
    loc[j] = 0u;
#pragma unroll
    for (int q = 0; q < kPer; ++q) loc[j] += row[q][j];
  }
  __shared__ __attribute__((aligned(16))) uint32_t sh_t[kMaxCand * kBlock];
  __shared__ uint32_t s_tot32[kMaxCand];
  block_totals_u32<kMaxCand>(loc, sh_t, s_tot32);
  // per-candidate totals in LDS: the decision indexes them dynamically (a
  // private array would live in scratch)
  __shared__ int64_t s_tot[kMaxCand];
  if (threadIdx.x < kMaxCand) s_tot[threadIdx.x] = (int64_t)s_tot32[threadIdx.x];
  __syncthreads();
  if (threadIdx.x == 0) {
    s_stop = 0;
    struct {
      double cal_c, cal_step;
      int32_t fallback;
      int64_t ref_total;
    } dec = {ctrl->cal_c, ctrl->cal_step, ctrl->fallback, ctrl->ref_total};
    const int64_t* tot = s_tot;
    int chosen = 0, gt = 0, ge = -1;
    int64_t quota = 0;
    const double kd = (double)k;
    if (mode == kModeGaussian) {
      int a = 0, b = 0;
      for (int loop = 0; loop < loops; ++loop) {
        const int64_t c = tot[(a + b) * (a + b + 1) / 2 + b];
        if (loop == loops - 1) break;
        if ((double)c < 2.0 * kd / 3.0) ++a;
        else if ((double)c > 4.0 * kd / 3.0) ++b;
        else break;
      }
      chosen = (a + b) * (a + b + 1) / 2 + b;
    } else if (mode == kModeRedSync) {
      int node = 0;
      for (int depth = 0; depth < 3; ++depth) {
        const int64_t c = tot[node];
        if (c > k && 2 * k > c) break;
        if (depth == 2) break;
        node = ((double)c < kd / 2.0) ? 2 * node + 1 : 2 * node + 2;
      }
      chosen = node;
    } else if (mode == kModeRedSyncTrim) {
      chosen = nc - 1;
      for (int j = 0; j < nc; ++j) if (tot[j] >= k) { chosen = j; break; }
    } else if (mode == kModeGaussianCal) {
      // counts are non-increasing in j.  Pick the count closest to k (log
      // distance) among those in [2k/3, 4k/3]; re-centre the ladder on the
      // closest candidate overall and adapt its spacing so that neighbours
      // two steps apart differ ~1.7x in count (a candidate then always lands
      // in the 2x-wide window).
      int best = -1, closest = 0;
      double bestd = 1e300, closed = 1e300;
      for (int j = 0; j < nc; ++j) {
        const double c = (double)tot[j];
        const double d = fabs(log((c > 0.0 ? c : 0.5) / kd));
        if (d < closed) { closed = d; closest = j; }
        if (c >= 2.0 * kd / 3.0 && c <= 4.0 * kd / 3.0 && d < bestd) { bestd = d; best = j; }
      }
      const int jc = best >= 0 ? best : closest;
      double step = dec.cal_step;
      if (best < 0 && (jc == 0 || jc == nc - 1)) {
        step = step * 2.0;                                  // target beyond the ladder: widen
      } else if (jc > 0 && jc < nc - 1 && tot[jc + 1] > 0) {
        const double R = (double)tot[jc - 1] / (double)tot[jc + 1];
        if (R > 1.0001) {
          double f = log(1.7) / log(R);
          f = f < 0.5 ? 0.5 : (f > 2.0 ? 2.0 : f);
          step = step * f;
        } else {
          step = step * 2.0;
        }
      }
      step = step < 0.002 ? 0.002 : (step > 1.0 ? 1.0 : step);
      const double sd = ctrl->stdev;
      if (sd > 0.0 && ctrl->cand_thr[jc] > 0.0) dec.cal_c = ctrl->cand_thr[jc] / sd;
      dec.cal_step = step;
      chosen = jc;
      if (best < 0) {
        s_stop = 1;
        dec.fallback = 1;
      }
    } else if (mode == kModeThreshold) {
      chosen = 0;
    } else if (mode == kModeTopK || mode == kModeRandomK) {
      chosen = 0; gt = 0; ge = 1; quota = ctrl->radix_kremain[1];
    } else if (mode == kModeDGC) {
      if ((double)tot[0] > 4.0 * kd / 3.0) { chosen = 1; gt = 1; ge = 2; quota = ctrl->radix_kremain[1]; }
      else chosen = 0;
    }
    // magnitude-correct overflow: the threshold choice passes more than k_cap
    // entries -> the evaluated candidate with the largest count in
    // [2k/3, k_cap] (a higher threshold: the largest entries), else the exact
    // key at k_cap
    if (!cond && ge < 0 && !s_stop && tot[chosen] > k_cap) {
      dec.ref_total = tot[chosen];
      int alt = -1;
      int64_t bc = -1;
      for (int j = 0; j < nc; ++j)
        if (tot[j] <= k_cap && 3 * tot[j] >= 2 * k && tot[j] > bc) { bc = tot[j]; alt = j; }
      if (alt >= 0) {
        chosen = alt;
      } else {
        s_stop = 1;
        dec.fallback = 2;
      }
    }
    if (ge < 0) gt = chosen;
    s_chosen = cond ? (dec.fallback == 2 ? kOverflowExact : kCalFallback) : chosen;
    s_gt = gt; s_ge = ge; s_quota = quota;
    s_thr = (float)ctrl->cand_thr[chosen];
    s_ref_total = dec.ref_total;
    // the decision's fields to the control block (read by the select /
    // conditional passes and the next call)
    gctrl->cal_c = dec.cal_c;
    gctrl->cal_step = dec.cal_step;
    gctrl->fallback = dec.fallback;
    gctrl->ref_total = dec.ref_total;
    gctrl->chosen = s_chosen;
    gctrl->sel_bound = ctrl->bound[gt];
    gctrl->eq_key = ge >= 0 ? ctrl->bound[ge] : 0xffffffffu;
    gctrl->eq_quota = ge >= 0 ? quota : 0;
    gctrl->thr = s_thr;
  }
  __syncthreads();
  if (s_stop) {
    // fallback to the exact key: clear the exact-key histograms for the
    // conditional radix passes; offsets and header come from the second
    // (conditional) count / decide
    if (hist_reset != nullptr)   // (the fused fallback clears them device-coherent itself)
      for (int i = threadIdx.x; i < kHistSet; i += kBlock) hist_reset[i] = 0u;
    return;
  }
  const int gt = s_gt, ge = s_ge;
  const int64_t quota = s_quota;
  int64_t gtc[kPer], eqc[kPer];
  uint32_t eq_loc = 0u;
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    // row[q][gt], row[q][ge] by uniform selects (no dynamic register index);
    // rows past G were loaded as zeros
    uint32_t vg = 0u, ve = 0u;
#pragma unroll
    for (int j = 0; j < kMaxCand; ++j) {
      vg = j == gt ? row[q][j] : vg;
      ve = j == ge ? row[q][j] : ve;
    }
    gtc[q] = vg;
    eqc[q] = ge >= 0 ? (int64_t)ve - (int64_t)vg : 0;
    eq_loc += (uint32_t)eqc[q];
  }
  // the equal-key quota scan only when the decision has an exact-key slot
  // (block-uniform: ge comes from LDS)
  uint32_t eq_before = 0u;
  if (ge >= 0) {
    uint32_t eq_tot;
    eq_before = block_excl_scan_u32(eq_loc, reinterpret_cast<uint32_t*>(sh_scan), &eq_tot);
  }
  int64_t take[kPer];
  uint32_t sel_loc = 0u;
  int64_t eqb = (int64_t)eq_before;
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    int64_t rem = quota - eqb;
    if (rem < 0) rem = 0;
    take[q] = eqc[q] < rem ? eqc[q] : rem;
    eqb += eqc[q];
    sel_loc += (uint32_t)(gtc[q] + take[q]);
  }
  uint32_t sel_tot32;
  uint64_t sel_before = block_excl_scan_u32(sel_loc, reinterpret_cast<uint32_t*>(sh_scan), &sel_tot32);
  const uint64_t sel_tot = sel_tot32;
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    const int b = threadIdx.x * kPer + q;
    if (b < G) {
      offsets[b] = (int64_t)sel_before;
      eqtake[b] = take[q];
      blocksel[b] = gtc[q] + take[q];
    }
    sel_before += gtc[q] + take[q];
  }
  if (threadIdx.x == 0) {
    const int64_t total = (int64_t)sel_tot;
    const int64_t sent = total < k_cap ? total : k_cap;
    gctrl->total = total;
    gctrl->sent = sent;
    const int64_t rt = s_ref_total >= 0 ? s_ref_total : total;
    hdr[0] = (int32_t)sent;
    hdr[1] = (int32_t)(rt > 0x7fffffff ? 0x7fffffff : rt);
    hdr[2] = s_chosen;
    hdr[3] = __float_as_int(s_thr);
  }
}

// --------------------------------------------------------------------------
// Fused decide + conditional exact fallback (threshold modes): ONE launch in
// place of decide_kernel and the four early-exit launches of the fallback
// chain (radix passes 0-2, conditional count), which cost ~4.7 us each even
// when they exit at once (r5c34: 19 us of a 142 us pipeline).  Block 0 runs
// the decision and publishes its fallback flag; every other block polls it.
// No fallback (the common case): every block exits.  Fallback: the grid runs
// the three histogram passes, the key resolve, the conditional count over
// the count pass's block chunks and the second decide, separated by grid
// barriers.  The grid is HALF of what is co-resident on an idle device
// (host: occupancy x CUs / 2, <= 512 blocks), so two such grids -- two ranks
// sharing one GPU in the multi-rank rehearsals -- are resident together.
// Used for the calls with launch hand-offs only: a bucket compressed while
// the backward still runs (handoff = lastblock) keeps the launch chain, whose
// blocks do not hold CU slots while GEMM blocks they share the device with
// drain (and whose extra launches are hidden under the backward anyway).
// Every spin is bounded (s_sleep, 2^24 polls).
// --------------------------------------------------------------------------
struct FbArgs {
  uint32_t* flag;       // 0 until block 0 decided, then 1 + ctrl->fallback; cleared by the last block out
  uint32_t* gen;        // grid-barrier generation
  uint32_t* bar;        // grid-barrier arrival counter (two-level)
  uint32_t* exit_ctr;   // exit arrival counter (two-level)
  GkCtrl* ctrl;         // sync_timeouts
  uint32_t* hist;       // exact-key histogram set
  uint32_t* blockcnt;
  const float* x;
  int64_t n, kfb, chunk_tiles;
  int G;                // count-pass blocks (the select grid)
};

// MI355X_MICROARCH.md "inter-workgroup visibility": every storing wave waits
// for its stores, barrier, lane 0 releases (agent; the explicit wait after
// the fence, which ROCm 7.2 can drop), counts in; the last arrival bumps the
// generation, the others poll it relaxed; then ONE agent acquire + wait and a
// barrier before any load of another block's bytes.
// an expired bounded spin: counted (sticky) in the control block, so a grid
// that was not co-resident shows up instead of passing silently
__device__ __forceinline__ void sync_timeout(const FbArgs& f) {
  __hip_atomic_fetch_add(&f.ctrl->sync_timeouts, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void grid_sync(const FbArgs& f) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t g0 = ld_dev(f.gen);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // generation read before this block counts in
    if (arrive(f.bar, gridDim.x, blockIdx.x)) {
      st_dev(f.gen, g0 + 1u);
    } else {
      uint32_t spins = 0;
      while (ld_dev(f.gen) == g0 && ++spins < (1u << 24)) __builtin_amdgcn_s_sleep(2);
      if (spins >= (1u << 24)) sync_timeout(f);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

// DECIDED: the count pass already decided in its last block (kernel boundary
// in between), block 0 only reads the flag.
template <bool VEC, bool DECIDED>
__global__ __launch_bounds__(kBlock) void decide_fb_kernel(DecArgs da, FbArgs f) {
  GkCtrl* ctrl = da.ctrl;
  const int bid = blockIdx.x, nblk = gridDim.x;
  __shared__ uint32_t s_fb;
  {
    if (bid == 0) {
      if constexpr (!DECIDED)
        decide_body(ctrl, f.blockcnt, f.G, da.mode, da.loops, da.k, da.k_cap, da.offsets, da.eqtake, da.blocksel,
                    da.hdr, 0, nullptr);
      __syncthreads();
      if (threadIdx.x == 0) s_fb = (uint32_t)ctrl->fallback;   // this lane wrote it in decide_body
      __syncthreads();
      if (s_fb != 0u)
        for (int i = threadIdx.x; i < kHistSet; i += kBlock) st_dev(&f.hist[i], 0u);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) st_dev(f.flag, 1u + s_fb);
    } else {
      if (threadIdx.x == 0) {
        uint32_t v, spins = 0;
        while ((v = ld_dev(f.flag)) == 0u && ++spins < (1u << 24)) __builtin_amdgcn_s_sleep(2);
        if (v == 0u) sync_timeout(f);
        s_fb = v == 0u ? 0u : v - 1u;
      }
      __syncthreads();
    }
  }
  if (s_fb != 0u) {
    __shared__ uint32_t sh_rad[kRadixShWords];   // one LDS histogram buffer for the three passes
    radix_hist_body<0, kKeyAbs, VEC>(f.x, f.n, 0u, 0u, f.kfb, f.hist, nullptr, bid, nblk, sh_rad);
    grid_sync(f);
    radix_hist_body<1, kKeyAbs, VEC>(f.x, f.n, 0u, 0u, f.kfb, f.hist, nullptr, bid, nblk, sh_rad);
    grid_sync(f);
    radix_hist_body<2, kKeyAbs, VEC>(f.x, f.n, 0u, 0u, f.kfb, f.hist, nullptr, bid, nblk, sh_rad);
    grid_sync(f);
    if (bid == 0) cal_fallback_body(ctrl, f.hist, f.kfb);
    grid_sync(f);
    for (int vb = bid; vb < f.G; vb += nblk)
      count_body<kKeyAbs, VEC, kFallbackCands, 0>(f.x, f.n, 0u, ctrl, f.chunk_tiles, f.blockcnt, nullptr, vb);
    grid_sync(f);
    if (bid == 0)
      decide_body(ctrl, f.blockcnt, f.G, da.mode, da.loops, da.k, da.k_cap, da.offsets, da.eqtake, da.blocksel,
                  da.hdr, 1, nullptr);
  }
  // the last block out clears the flag for the next call
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0 && arrive(f.exit_ctr, nblk, bid)) st_dev(f.flag, 0u);
}

// --------------------------------------------------------------------------
// K5: select + compact (ascending indices) + residual write-back
// --------------------------------------------------------------------------
template <int KEYKIND, bool VEC>
__global__ __launch_bounds__(kBlock) void select_kernel(float* __restrict__ r, int64_t n, uint32_t seed,
                                                        const GkCtrl* __restrict__ ctrl, int64_t chunk_tiles,
                                                        const int64_t* __restrict__ offsets,
                                                        const int64_t* __restrict__ eqtake,
                                                        const int64_t* __restrict__ blocksel, int64_t k_cap,
                                                        int32_t* __restrict__ out_idx, float* __restrict__ out_val,
                                                        const uint32_t* __restrict__ valid, float* __restrict__ u,
                                                        const uint32_t* __restrict__ seed_dev) {
  const int64_t my_sel = blocksel[blockIdx.x];
  if (seed_dev != nullptr) seed = __builtin_amdgcn_readfirstlane(*seed_dev);
  int64_t running = offsets[blockIdx.x];
  if (my_sel == 0 || running >= k_cap) return;  // block-uniform
  const uint32_t bound = __builtin_amdgcn_readfirstlane(ctrl->sel_bound);
  const uint32_t eqkey = __builtin_amdgcn_readfirstlane(ctrl->eq_key);
  const int64_t my_eq = eqtake[blockIdx.x];
  int64_t eq_running = 0;
  __shared__ uint32_t sh_tot[4][kWavesPerBlock];
  __shared__ uint32_t sh_eq[4][kWavesPerBlock];
  const int64_t ntiles = (n + kTileElems - 1) / kTileElems;
  const int64_t t0 = (int64_t)blockIdx.x * chunk_tiles;
  const int64_t t1 = t0 + chunk_tiles < ntiles ? t0 + chunk_tiles : ntiles;
  const int w = wave_id();
  // two tiles of loads in flight: buffers va / vb alternate without register
  // copies (a copy of a load's destination waits for it), so the barriers of
  // tile t wait for tile t's loads only
  float va[4][4], vb[4][4];
  auto ldt = [&](int64_t t, float (*b)[4]) {
#pragma unroll
    for (int j4 = 0; j4 < 4; ++j4) load4<VEC>(r, t * kTileElems + j4 * (kBlock * 4) + threadIdx.x * 4, n, b[j4]);
  };
  auto body = [&](int64_t tile, float (*v)[4]) {
    const int64_t base = tile * kTileElems;
    uint32_t selm[4], eqm[4];
#pragma unroll
    for (int j4 = 0; j4 < 4; ++j4) {
      const int64_t e = base + j4 * (kBlock * 4) + threadIdx.x * 4;
      selm[j4] = 0; eqm[j4] = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const bool inb = e + q < n;
        const uint32_t key = inb ? key_of<KEYKIND>(e + q, v[j4][q], seed, valid) : 0u;
        if (inb && key >= bound) selm[j4] |= 1u << q;
        if (inb && my_eq > 0 && key == eqkey) eqm[j4] |= 1u << q;
      }
    }
    // ties (radix modes): take the first `my_eq` key==eqkey elements of this block
    if (my_eq > 0) {
      uint32_t pre[4];
#pragma unroll
      for (int j4 = 0; j4 < 4; ++j4) {
        uint32_t tot;
        pre[j4] = wave_excl_prefix_small<3>(__popc(eqm[j4]), &tot);
        if (lane_id() == 0) sh_eq[j4][w] = tot;
      }
      __syncthreads();
      int64_t acc = eq_running;
#pragma unroll
      for (int j4 = 0; j4 < 4; ++j4) {
        int64_t before = acc;
        for (int ww = 0; ww < kWavesPerBlock; ++ww) {
          if (ww < w) before += sh_eq[j4][ww];
          acc += sh_eq[j4][ww];
        }
        int64_t rank = before + pre[j4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (eqm[j4] & (1u << q)) {
            if (rank < my_eq) selm[j4] |= 1u << q;
            ++rank;
          }
        }
      }
      eq_running = acc;
      __syncthreads();
    }
    uint32_t pre[4];
#pragma unroll
    for (int j4 = 0; j4 < 4; ++j4) {
      uint32_t tot;
      pre[j4] = wave_excl_prefix_small<3>(__popc(selm[j4]), &tot);
      if (lane_id() == 0) sh_tot[j4][w] = tot;
    }
    __syncthreads();
    int64_t acc = running;
#pragma unroll
    for (int j4 = 0; j4 < 4; ++j4) {
      int64_t before = acc;
      for (int ww = 0; ww < kWavesPerBlock; ++ww) {
        if (ww < w) before += sh_tot[j4][ww];
        acc += sh_tot[j4][ww];
      }
      if (selm[j4]) {
        int64_t pos = before + pre[j4];
        const int64_t e = base + j4 * (kBlock * 4) + threadIdx.x * 4;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (selm[j4] & (1u << q)) {
            if (pos < k_cap) {
              out_idx[pos] = (int32_t)(e + q);
              out_val[pos] = v[j4][q];
              r[e + q] = 0.f;
              if (u != nullptr) u[e + q] = 0.f;   // momentum factor masking (DGC)
            }
            ++pos;
          }
        }
      }
    }
    running = acc;
    __syncthreads();
  };
  if (t0 < t1) ldt(t0, va);
  if (t0 + 1 < t1) ldt(t0 + 1, vb);
  for (int64_t tile = t0; tile < t1 && running < k_cap; tile += 2) {
    body(tile, va);
    if (tile + 2 < t1) ldt(tile + 2, va);
    if (tile + 1 < t1 && running < k_cap) {
      body(tile + 1, vb);
      if (tile + 3 < t1) ldt(tile + 3, vb);
    }
  }
}

// live candidates of a count pass (finalize_kernel / cal_fallback_kernel ladders)
int count_cands(const CompressArgs& a, int cond) { return cond ? kFallbackCands : ladder_cands(a.mode, a.loops); }

// Single-workgroup hand-offs: by last-block arrival counter inside the
// producing grid, or by a separate 1-workgroup launch after it.  The counter
// costs one agent-scope atomic per block on ONE address, and the atomics
// serialise (~19 ns each, measured: count pass on a 4 M bucket, 1024 blocks
// of one tile each, 32 us against select's 5.5 us over the same data); a
// launch costs ~5 us.  Default: launches (GKSGD_HANDOFF=lastblock restores
// the in-grid hand-off).  The conditional fallback chain keeps the in-grid
// form: it must cost nothing extra when it does not fire.
bool handoff_by_launch_env() {
  const char* e = getenv("GKSGD_HANDOFF");
  return !(e != nullptr && strcmp(e, "lastblock") == 0);
}

bool handoff_by_launch(const CompressArgs& a) { return a.handoff < 0 ? handoff_by_launch_env() : a.handoff == 0; }

DecArgs make_dec(const CompressArgs& a, const Ws& w, GkCtrl* ctrl, int cond) {
  DecArgs da;
  da.in_kernel = (cond || !handoff_by_launch(a)) ? 1 : 0;
  da.ctrl = ctrl; da.mode = a.mode; da.loops = a.loops; da.k = a.k; da.k_cap = a.k_cap;
  da.offsets = w.offsets; da.eqtake = w.eqtake; da.blocksel = w.blocksel; da.hdr = a.record;
  da.hist_reset = w.hist; da.counter = w.sync + (cond ? 3 : 1) * kSyncWords;
  return da;
}

// defer_decide: a launch-hand-off decide is left to decide_fb_kernel
template <int KEYKIND>
void launch_count(const CompressArgs& a, const Ws& w, bool vec, int G, int64_t chunk_tiles, GkCtrl* ctrl, int cond,
                  hipStream_t s, bool defer_decide = false) {
  const int nc = count_cands(a, cond);
  const DecArgs da = make_dec(a, w, ctrl, cond);
#define GK_COUNT3(NC, NX, DEC)                                                                                    \
  if (vec)                                                                                                        \
    hipLaunchKernelGGL((count_kernel<KEYKIND, true, NC, NX, DEC>), dim3(G), dim3(kBlock), 0, s, a.r, a.n, a.seed,  \
                       ctrl, chunk_tiles, w.blockcnt, a.valid, cond, a.seed_dev, da);                             \
  else                                                                                                            \
    hipLaunchKernelGGL((count_kernel<KEYKIND, false, NC, NX, DEC>), dim3(G), dim3(kBlock), 0, s, a.r, a.n, a.seed, \
                       ctrl, chunk_tiles, w.blockcnt, a.valid, cond, a.seed_dev, da);
#define GK_COUNT2(NC, NX) if (da.in_kernel) { GK_COUNT3(NC, NX, true) } else { GK_COUNT3(NC, NX, false) }
#define GK_COUNT(NC) GK_COUNT2(NC, 0)
  if constexpr (KEYKIND == kKeyHash) {
    GK_COUNT(2)
  } else {
    if (!cond && a.mode == kModeGaussian && gauss_ext(a.loops)) { GK_COUNT2(kGaussWalk, kGaussExt) }
    else if (nc <= 2) { GK_COUNT(2) }
    else if (nc <= 3) { GK_COUNT(3) }
    else if (nc <= 6) { GK_COUNT(6) }
    else if (nc <= 8) { GK_COUNT(8) }
    else { GK_COUNT(kMaxCand) }
  }
#undef GK_COUNT
#undef GK_COUNT2
#undef GK_COUNT3
  if (!da.in_kernel && !defer_decide)
    hipLaunchKernelGGL(decide_kernel, dim3(1), dim3(kBlock), 0, s, w.blockcnt, G, cond, da);
}

// fused decide + fallback: GKSGD_FB_FUSED=0 restores the separate launches
bool fb_fused_env() {
  const char* e = getenv("GKSGD_FB_FUSED");
  return !(e != nullptr && strcmp(e, "0") == 0);
}

// GKSGD_STEP_INGRID=1 (opt-in, measured slower): launch hand-offs with the
// 1-workgroup steps in-grid -- the finalize in the stats pass's last block, the
// decide in the count pass's last block, the fused fallback launch only
// reading the decision.  25.6 M bucket, same box (r5c54): stats + finalize
// 72.8 us in-grid vs 62.6 + 7.9 as launches, count + decide_fb 33.0 + 4.7 vs
// 21.6 + 14.4; kernel span 131.8 vs 130.0 us, wall 134.2 / 136.1 vs 137.1 /
// 139.6 us (two fewer launches) -- within noise either way: the last block's
// wait for the arrivals and its serial reduction cost about the kernel
// boundary they replace, so the default keeps the unchanged launch chain.
bool step_ingrid_env() {
  const char* e = getenv("GKSGD_STEP_INGRID");
  return e != nullptr && strcmp(e, "1") == 0;
}

// half the co-resident grid of decide_fb_kernel on an idle device (<= 512);
// 0: unavailable
template <bool VEC>
int fb_grid() {
  static int g = -1;
  if (g < 0) {
    int dev = 0, cus = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, decide_fb_kernel<VEC, false>, kBlock, 0) != hipSuccess)
      per = 0;
    const int64_t v = (int64_t)per * cus / 2;
    g = v < 1 ? 0 : (v > 512 ? 512 : (int)v);
  }
  return g;
}

// decide + the conditional exact fallback as one launch (launch hand-offs
// only); false: not available, nothing launched
bool launch_decide_fb(const CompressArgs& a, const Ws& w, bool vec, int G, int64_t chunk_tiles, GkCtrl* ctrl,
                      int64_t kfb, hipStream_t s, bool decided) {
  const DecArgs da = make_dec(a, w, ctrl, 0);
  const int Gf = vec ? fb_grid<true>() : fb_grid<false>();
  if (Gf < 1) return false;
  FbArgs f;
  f.flag = w.sync + kSyncCounters * kSyncWords;
  f.gen = f.flag + 64;
  f.bar = w.sync + 4 * kSyncWords;
  f.exit_ctr = w.sync + 5 * kSyncWords;
  f.ctrl = ctrl; f.hist = w.hist; f.blockcnt = w.blockcnt; f.x = a.r; f.n = a.n; f.kfb = kfb; f.chunk_tiles = chunk_tiles; f.G = G;
  if (decided) {
    if (vec) hipLaunchKernelGGL((decide_fb_kernel<true, true>), dim3(Gf), dim3(kBlock), 0, s, da, f);
    else hipLaunchKernelGGL((decide_fb_kernel<false, true>), dim3(Gf), dim3(kBlock), 0, s, da, f);
  } else {
    if (vec) hipLaunchKernelGGL((decide_fb_kernel<true, false>), dim3(Gf), dim3(kBlock), 0, s, da, f);
    else hipLaunchKernelGGL((decide_fb_kernel<false, false>), dim3(Gf), dim3(kBlock), 0, s, da, f);
  }
  return true;
}

template <int KEYKIND>
void launch_select(const CompressArgs& a, const Ws& w, bool vec, int G, int64_t chunk_tiles, GkCtrl* ctrl,
                   int32_t* out_idx, float* out_val, hipStream_t s) {
  if (vec)
    hipLaunchKernelGGL((select_kernel<KEYKIND, true>), dim3(G), dim3(kBlock), 0, s, a.r, a.n, a.seed, ctrl,
                       chunk_tiles, w.offsets, w.eqtake, w.blocksel, a.k_cap, out_idx, out_val, a.valid, a.u,
                       a.seed_dev);
  else
    hipLaunchKernelGGL((select_kernel<KEYKIND, false>), dim3(G), dim3(kBlock), 0, s, a.r, a.n, a.seed, ctrl,
                       chunk_tiles, w.offsets, w.eqtake, w.blocksel, a.k_cap, out_idx, out_val, a.valid, a.u,
                       a.seed_dev);
}

// fb_counter != nullptr: conditional fallback chain (cond != nullptr), pass 2
// resolves the fallback key in its last block
template <int KEYKIND>
void launch_radix(const float* x, int64_t n, uint32_t seed, uint32_t sample_thr, int64_t k, uint32_t* set, bool vec,
                  const uint32_t* valid, GkCtrl* cond, const uint32_t* seed_dev, hipStream_t s,
                  uint32_t* fb_counter = nullptr) {
  const int64_t n4 = (n + 3) / 4;
  int Gh = (int)ceil_div(n4, (int64_t)kBlock * 8);
  if (Gh < 1) Gh = 1;
  if (Gh > 512) Gh = 512;
  // (the conditional fallback chain keeps the full grid: it fires on every
  // step of the momentum-corrected bs32 ResNet-50 run -- 64 workgroups made
  // each of its passes 4x slower there, r5c2)
#define GK_RADIX_PASS(P)                                                                                         \
  if (vec)                                                                                                       \
    hipLaunchKernelGGL((radix_hist_kernel<P, KEYKIND, true>), dim3(Gh), dim3(kBlock), 0, s, x, n, seed, sample_thr, \
                       k, set, valid, cond, seed_dev);                                                           \
  else                                                                                                           \
    hipLaunchKernelGGL((radix_hist_kernel<P, KEYKIND, false>), dim3(Gh), dim3(kBlock), 0, s, x, n, seed,          \
                       sample_thr, k, set, valid, cond, seed_dev);
  GK_RADIX_PASS(0)
  GK_RADIX_PASS(1)
  if (fb_counter != nullptr) {
    if (vec)
      hipLaunchKernelGGL((radix_hist_kernel<2, KEYKIND, true, true>), dim3(Gh), dim3(kBlock), 0, s, x, n, seed,
                         sample_thr, k, set, valid, cond, seed_dev, fb_counter);
    else
      hipLaunchKernelGGL((radix_hist_kernel<2, KEYKIND, false, true>), dim3(Gh), dim3(kBlock), 0, s, x, n, seed,
                         sample_thr, k, set, valid, cond, seed_dev, fb_counter);
  } else {
    GK_RADIX_PASS(2)
  }
#undef GK_RADIX_PASS
}

}  // namespace

size_t compress_workspace_bytes(int64_t /*n*/) { return ws_bytes(); }

void compress(const CompressArgs& a, hipStream_t s) {
  const Ws w = carve(a.ws);
  GkCtrl* ctrl = reinterpret_cast<GkCtrl*>(a.ctrl);
  int32_t* out_idx = a.record + 4;
  float* out_val = reinterpret_cast<float*>(a.record + 4 + a.k_cap);
  if (a.n <= 0) {
    hipMemsetAsync(a.record, 0, sizeof(int32_t) * 4, s);
    return;
  }
  const bool vec_gr = ((reinterpret_cast<uintptr_t>(a.g) | reinterpret_cast<uintptr_t>(a.r)) & 15) == 0 && (a.n % 4) == 0;
  const bool vec_r = (reinterpret_cast<uintptr_t>(a.r) & 15) == 0 && (a.n % 4) == 0;

  // 1. stats (+ residual add, residual write, gradient zeroing; + DGC momentum
  //    correction when a chunk table is given); threshold modes finalize in
  //    the last stats block (radix modes need the histograms first)
  const bool radix_mode = a.mode == kModeTopK || a.mode == kModeRandomK || a.mode == kModeDGC;
  const bool by_launch = handoff_by_launch(a);
  const bool fb_fused = fb_fused_env() && by_launch;
  // finalize in the stats pass's last block: in-grid hand-offs, or launch
  // hand-offs with the fused fallback and the in-grid steps
  const bool step_in = fb_fused && step_ingrid_env();
  const bool fin_in = !radix_mode && (!by_launch || step_in);
  const int64_t keff = a.k < a.n ? a.k : a.n;
  const int64_t n_stats = a.n_stats > 0 ? a.n_stats : a.n;
  FinArgs fa;
  fa.ctrl = ctrl; fa.n = n_stats; fa.mode = a.mode; fa.loops = a.loops; fa.z = a.z; fa.fixed_thr = a.fixed_thr;
  fa.k = keff; fa.stats_out = a.stats_out; fa.counter = w.sync;
  int Gs;
  if (a.u != nullptr && a.chunks != nullptr) {
    Gs = a.chunk_count < kMaxStatsBlocks ? a.chunk_count : kMaxStatsBlocks;
    if (Gs < 1) Gs = 1;
    McHyper hp;
    for (int i = 0; i < 8; ++i) { hp.mu[i] = a.mc_mu[i]; hp.wd[i] = a.mc_wd[i]; }
    const Chunk* ch = a.chunks + a.chunk_begin;
#define GK_MC(EC, FIN)                                                                                            \
  hipLaunchKernelGGL((mc_stats_kernel<EC, FIN>), dim3(Gs), dim3(kBlock), 0, s, a.g, a.r, a.u, a.w, ch,             \
                     a.chunk_count, a.chunk_base, hp, w.partials, fa);
    if (a.ec) { if (!fin_in) { GK_MC(true, false) } else { GK_MC(true, true) } }
    else { if (!fin_in) { GK_MC(false, false) } else { GK_MC(false, true) } }
#undef GK_MC
  } else {
    Gs = (int)ceil_div(a.n, (int64_t)kBlock * 16);
    if (Gs < 1) Gs = 1;
    if (Gs > kMaxStatsBlocks) Gs = kMaxStatsBlocks;
#define GK_STATS2(VEC, EC, ZG, FIN)                                                                               \
  hipLaunchKernelGGL((stats_kernel<VEC, EC, true, ZG, FIN>), dim3(Gs), dim3(kBlock), 0, s, a.g, a.r, a.n,          \
                     w.partials, fa);
#define GK_STATS(VEC, EC, ZG)                                                                                     \
  if (!fin_in) { GK_STATS2(VEC, EC, ZG, false) } else { GK_STATS2(VEC, EC, ZG, true) }
    if (vec_gr) {
      if (a.ec) { if (a.zero_g) { GK_STATS(true, true, true) } else { GK_STATS(true, true, false) } }
      else { if (a.zero_g) { GK_STATS(true, false, true) } else { GK_STATS(true, false, false) } }
    } else {
      if (a.ec) { if (a.zero_g) { GK_STATS(false, true, true) } else { GK_STATS(false, true, false) } }
      else { if (a.zero_g) { GK_STATS(false, false, true) } else { GK_STATS(false, false, false) } }
    }
#undef GK_STATS
#undef GK_STATS2
  }

  // 2. radix histograms (exact / hash / sample)
  uint32_t* hist_exact = w.hist;
  uint32_t* hist_sample = w.hist + kHistSet;
  if (radix_mode) {
    hipMemsetAsync(w.hist, 0, sizeof(uint32_t) * 2 * kHistSet, s);
    if (a.mode == kModeRandomK)
      launch_radix<kKeyHash>(a.r, a.n, a.seed, 0u, keff, hist_exact, vec_r, a.valid, nullptr, a.seed_dev, s);
    else
      launch_radix<kKeyAbs>(a.r, a.n, a.seed, 0u, keff, hist_exact, vec_r, nullptr, nullptr, a.seed_dev, s);
    if (a.mode == kModeDGC) {
      double p = a.sample_p * 4294967296.0;
      uint32_t thr = p >= 4294967295.0 ? 0xffffffffu : (uint32_t)p;
      launch_radix<kKeySample>(a.r, a.n, a.seed, thr, a.k, hist_sample, vec_r, nullptr, nullptr, a.seed_dev, s);
    }
  }

  // 3. finalize (radix modes, or every mode with launch hand-offs)
  if (!fin_in)
    hipLaunchKernelGGL(finalize_kernel, dim3(1), dim3(kBlock), 0, s, ctrl, w.partials, Gs, n_stats, a.mode, a.loops,
                       a.z, a.fixed_thr, keff, hist_exact, hist_sample, a.stats_out);

  // 4-6. count (+ decide in its last block), select
  const int64_t ntiles = ceil_div(a.n, (int64_t)kTileElems);
  int G = (int)(ntiles < kMaxCountBlocks ? ntiles : kMaxCountBlocks);
  const int64_t chunk_tiles = ceil_div(ntiles, (int64_t)G);
  G = (int)ceil_div(ntiles, chunk_tiles);
  if (a.mode == kModeRandomK) {
    launch_count<kKeyHash>(a, w, vec_r, G, chunk_tiles, ctrl, 0, s);
    launch_select<kKeyHash>(a, w, vec_r, G, chunk_tiles, ctrl, out_idx, out_val, s);
  } else {
    if (a.mode == kModeTopK) {
      launch_count<kKeyAbs>(a, w, vec_r, G, chunk_tiles, ctrl, 0, s);
    } else {
      // conditional exact fallback: calibrated mode without a candidate in
      // [2k/3, 4k/3] (top-k), or a threshold mode whose every candidate
      // overflows k_cap (top-k_cap) -- one fused launch (decide_fb_kernel), or
      // a chain of kernels that exit at once unless the decide set ctrl->fallback
      const int64_t kfb = a.mode == kModeGaussianCal ? keff : (a.k_cap < a.n ? a.k_cap : a.n);
      const bool fused = fb_fused;
      // step_in: the count pass decides in its last block, decide_fb reads it
      CompressArgs ac = a;
      if (step_in) ac.handoff = 1;
      launch_count<kKeyAbs>(ac, w, vec_r, G, chunk_tiles, ctrl, 0, s, fused && !step_in);
      if (!fused || !launch_decide_fb(a, w, vec_r, G, chunk_tiles, ctrl, kfb, s, step_in)) {
        if (fused && !step_in)   // the deferred decide, after all
          hipLaunchKernelGGL(decide_kernel, dim3(1), dim3(kBlock), 0, s, w.blockcnt, G, 0, make_dec(a, w, ctrl, 0));
        launch_radix<kKeyAbs>(a.r, a.n, a.seed, 0u, kfb, hist_exact, vec_r, nullptr, ctrl, a.seed_dev, s,
                              w.sync + 2 * kSyncWords);
        launch_count<kKeyAbs>(a, w, vec_r, G, chunk_tiles, ctrl, 1, s);
      }
    }
    launch_select<kKeyAbs>(a, w, vec_r, G, chunk_tiles, ctrl, out_idx, out_val, s);
  }
}

void tensor_stats(const float* x, int64_t n, void* ctrl, void* ws, hipStream_t s) {
  const Ws w = carve(ws);
  int Gs = (int)ceil_div(n, (int64_t)kBlock * 16);
  if (Gs < 1) Gs = 1;
  if (Gs > kMaxStatsBlocks) Gs = kMaxStatsBlocks;
  float* xx = const_cast<float*>(x);
  const bool vec = (reinterpret_cast<uintptr_t>(x) & 15) == 0 && (n % 4) == 0;
  if (vec)
    hipLaunchKernelGGL((stats_kernel<true, false, false, false, false>), dim3(Gs), dim3(kBlock), 0, s, xx, xx, n,
                       w.partials, FinArgs{});
  else
    hipLaunchKernelGGL((stats_kernel<false, false, false, false, false>), dim3(Gs), dim3(kBlock), 0, s, xx, xx, n,
                       w.partials, FinArgs{});
  hipLaunchKernelGGL(finalize_kernel, dim3(1), dim3(kBlock), 0, s, reinterpret_cast<GkCtrl*>(ctrl), w.partials, Gs, n,
                     (int)kModeThreshold, 1, 0.0, 0.0, (int64_t)1, w.hist, w.hist, (float*)nullptr);
}

}  // namespace gk
