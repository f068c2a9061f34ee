// Batched per-step weight re-layouts: every Winograd filter transform and
// every grad-input weight transpose of a model step in ONE launch.
//
// The convolution kernels read their weights in kernel-specific layouts --
// Winograd F(2x2, 3x3) filter tiles u = [Ci/8][16][Co][8] (forward and the
// flipped grad-input filter), the transposed [C][K] weight of a 1x1 grad-input
// GEMM, the per-tap transposed weight of a non-Winograd 3x3 grad-input -- and
// the weights change every step, so each layout is rebuilt every step.  Built
// per call that is one small launch per layer and direction: 26 Winograd
// filter transforms (7.3 us each) and 37 transposing copies (5.8 us each) per
// ResNet-50 step at the reference's batch of 32 -- 3% of a 13 ms step
// (profiles/r04_resnet50_bs32_fp32_kernel_stats.csv), almost all of it
// launch and drain time.  ops/weight_prep.py registers the re-layouts a model
// uses once and replays them here at the start of every step: one grid, a
// descriptor table in LDS, each workgroup one unit of one descriptor (256
// filter pairs of a Winograd transform, or one 64 x 64 tile of a transpose,
// staged through LDS so both the reads and the writes are coalesced).
#include <hip/hip_runtime.h>

#include "common.h"
#include "gk_kernels.h"
#include "wino_x6_common.h"

namespace gk {
namespace {

constexpr int kTile = 64;
constexpr int kMaxDescs = 512;

// Winograd F(2x2, 3x3) filter transform of one (co, ci) pair: G g G^T with
// G = [1 0 0; 1/2 1/2 1/2; 1/2 -1/2 1/2; 0 0 1], into the swizzled u layout
// of winograd.hip (wino_wt_kernel: same arithmetic, same slots).
__device__ __forceinline__ int wsw(int r) { return (r >> 2) & 3; }

// Work item idx -> (co, ci) with 8 consecutive input channels innermost, then
// the output channel: a wave covers 8 co x 8 ci, so each of its 16 stores
// writes one contiguous 256-byte run of u ([Ci/8][16][Co][8]) and its 9 loads
// read 8 runs of 32 bytes for either filter orientation (Ci % 8 == 0).
__device__ __forceinline__ void wino_pair(const float* __restrict__ w, float* __restrict__ u, int Co, int Ci, int flip,
                                          int64_t idx) {
  const int64_t rest = idx >> 3;
  const int co = (int)(rest % Co), ci = (int)(rest / Co) * 8 + (int)(idx & 7);
  float g[3][3];
#pragma unroll
  for (int kh = 0; kh < 3; ++kh)
#pragma unroll
    for (int kw = 0; kw < 3; ++kw)
      g[kh][kw] = flip ? w[((int64_t)ci * 9 + (2 - kh) * 3 + (2 - kw)) * Co + co]
                       : w[((int64_t)co * 9 + kh * 3 + kw) * Ci + ci];
  float t[4][3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    t[0][j] = g[0][j];
    t[1][j] = 0.5f * (g[0][j] + g[1][j] + g[2][j]);
    t[2][j] = 0.5f * (g[0][j] - g[1][j] + g[2][j]);
    t[3][j] = g[2][j];
  }
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

// out[s * ld_out + r] = in[r * ld_in + s] for one 64 x 64 tile (r, s) of an
// R x S matrix, through LDS (+1 column of padding: conflict-free columns).
template <typename T>
__device__ __forceinline__ void transpose_tile(const T* __restrict__ in, T* __restrict__ out, int64_t ld_in,
                                               int64_t ld_out, int R, int S, int r0, int s0, T (*sh)[kTile + 1]) {
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;   // 64 x 4 threads
#pragma unroll
  for (int i = 0; i < kTile / 4; ++i) {
    const int r = r0 + ty + 4 * i, s = s0 + tx;
    if (r < R && s < S) sh[ty + 4 * i][tx] = in[(int64_t)r * ld_in + s];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < kTile / 4; ++i) {
    const int s = s0 + ty + 4 * i, r = r0 + tx;
    if (r < R && s < S) out[(int64_t)s * ld_out + r] = sh[tx][ty + 4 * i];
  }
}

__global__ void __launch_bounds__(kBlock) weight_prep_kernel(const PrepDesc* __restrict__ descs, int ndesc) {
  __shared__ PrepDesc sd[kMaxDescs];
  __shared__ int s_d;
  for (int i = threadIdx.x; i < ndesc; i += kBlock) sd[i] = descs[i];
  __syncthreads();
  const int64_t b = blockIdx.x;
  if (threadIdx.x == 0) {
    // last descriptor whose first block is <= b (block_begin ascending)
    int lo = 0, hi = ndesc - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (sd[mid].block_begin <= b) lo = mid;
      else hi = mid - 1;
    }
    s_d = lo;
  }
  __syncthreads();
  const PrepDesc& d = sd[s_d];
  const int64_t unit = b - d.block_begin;
  if (d.kind == kPrepWinoX6 || d.kind == kPrepWinoX6Flip) {
    // bf16x6 Winograd filter planes (wino_x6.hip): consecutive threads, consecutive rows co
    const int64_t idx = unit * kBlock + threadIdx.x;
    if (idx < (int64_t)d.R * d.S)
      wino_x6_pair(static_cast<const float*>(d.src), static_cast<uint16_t*>(d.dst), d.R, d.S,
                   d.kind == kPrepWinoX6Flip, (int)(idx % d.R), (int)(idx / d.R));
    return;
  }
  if (d.kind == kPrepWino || d.kind == kPrepWinoFlip) {
    const int64_t idx = unit * kBlock + threadIdx.x;
    if (idx < (int64_t)d.R * d.S)
      wino_pair(static_cast<const float*>(d.src), static_cast<float*>(d.dst), d.R, d.S, d.kind == kPrepWinoFlip, idx);
    return;
  }
  const int r0 = (int)(unit / d.tiles_s) * kTile, s0 = (int)(unit % d.tiles_s) * kTile;
  if (d.kind == kPrepT32) {
    __shared__ float sh32[kTile][kTile + 1];
    transpose_tile<float>(static_cast<const float*>(d.src), static_cast<float*>(d.dst), d.ld_in, d.ld_out, d.R, d.S,
                          r0, s0, sh32);
  } else {
    __shared__ uint16_t sh16[kTile][kTile + 1];
    transpose_tile<uint16_t>(static_cast<const uint16_t*>(d.src), static_cast<uint16_t*>(d.dst), d.ld_in, d.ld_out,
                             d.R, d.S, r0, s0, sh16);
  }
}

}  // namespace

int64_t weight_prep_blocks(int kind, int R, int S) {
  if (kind == kPrepWino || kind == kPrepWinoFlip || kind == kPrepWinoX6 || kind == kPrepWinoX6Flip)
    return ((int64_t)R * S + kBlock - 1) / kBlock;
  return (int64_t)((R + kTile - 1) / kTile) * ((S + kTile - 1) / kTile);
}

int weight_prep_max_descs() { return kMaxDescs; }

void weight_prep(const PrepDesc* descs, int ndesc, int64_t total_blocks, hipStream_t stream) {
  if (ndesc <= 0 || total_blocks <= 0) return;
  hipLaunchKernelGGL(weight_prep_kernel, dim3((unsigned)total_blocks), dim3(kBlock), 0, stream, descs, ndesc);
}

}  // namespace gk
