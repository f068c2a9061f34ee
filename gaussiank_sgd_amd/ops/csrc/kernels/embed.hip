// Fused BERT input embedding: x[m] = word[ids[m]] + pos[m % T] + type[tt[m]]
// (fp32 tables and output, rows of H = 4k floats) and its backward.
//
// PyTorch runs this as three gathers + two adds forward and, backward, three
// sort-based embedding_dense_backward passes (rocprim radix sort, segment
// offsets, sum_and_scatter: ~0.8 ms of a 21 ms BERT-base bs32 x 512 step,
// profiles/r02_bert_*).  Here:
//   forward : one pass, one float4 per thread of each output row;
//   backward: word rows from a stable sort of the ids (torch.sort): run
//             bounds per id, frequent ids (> 64 tokens; [MASK] is 2560 of
//             16384 tokens in the synthetic MLM batch) split into 16-token
//             chunks summed by a wave each, then one wave per vocabulary row writes the whole
//             dense [V, H] gradient row in ascending token order (zeros for
//             absent ids) -- deterministic, no zero fill, no fp32 atomics into
//             a 94 MB table that misses L2 (the atomic version: 375 us;
//             an unsplit [MASK] row: 3 ms),
//             position rows summed over the batch (one thread per (t, h4)
//             walks the B rows: deterministic, written not accumulated),
//             type rows summed per block in fixed order into [blocks][NT][H]
//             partials and finalized in block order (deterministic).
// Reference model: the BERT MLM config of SURVEY.md (configs/bert.conf);
// the reference repo has no BERT code of its own (parity unpinned).
#include <hip/hip_runtime.h>

#include "common.h"
#include "gk_kernels.h"

namespace gk {
namespace {

constexpr int kEmbTypes = 2;   // token types (BERT: segment A / B)

__global__ __launch_bounds__(kBlock) void emb_fwd_kernel(const int64_t* __restrict__ ids,
                                                         const int64_t* __restrict__ tt, const float* __restrict__ Ww,
                                                         const float* __restrict__ Wp, const float* __restrict__ Wt,
                                                         float* __restrict__ out, int64_t M, int T, int H4) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= M * H4) return;
  const int64_t m = i / H4;
  const int h = (int)(i - m * H4);
  const int64_t w = ids[m];
  const int t = (int)(m % T);
  const int64_t ty = tt ? tt[m] : 0;
  const float4 a = reinterpret_cast<const float4*>(Ww + w * (int64_t)H4 * 4)[h];
  const float4 b = reinterpret_cast<const float4*>(Wp + (int64_t)t * H4 * 4)[h];
  const float4 c = reinterpret_cast<const float4*>(Wt + ty * (int64_t)H4 * 4)[h];
  // (word + pos) + type: the order of the reference composition
  reinterpret_cast<float4*>(out)[i] = make_float4(a.x + b.x + c.x, a.y + b.y + c.y, a.z + b.z + c.z, a.w + b.w + c.w);
}

// dWp[t] = sum_b dx[b * T + t] for t < T; rows T..P-1 are zero
__global__ __launch_bounds__(kBlock) void emb_pos_bwd_kernel(const float* __restrict__ dx, float* __restrict__ dWp,
                                                             int B, int T, int P, int H4) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= (int64_t)P * H4) return;
  const int t = (int)(i / H4);
  const int h = (int)(i - (int64_t)t * H4);
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (t < T) {
    for (int b = 0; b < B; ++b) {
      const float4 g = reinterpret_cast<const float4*>(dx)[((int64_t)b * T + t) * H4 + h];
      s.x += g.x; s.y += g.y; s.z += g.z; s.w += g.w;
    }
  }
  reinterpret_cast<float4*>(dWp)[i] = s;
}

// type partials: block (bx, by) sums rows by*rows_per .. of column group bx
// per token type into part[by][type][H]
__global__ __launch_bounds__(kBlock) void emb_type_partial_kernel(const int64_t* __restrict__ tt,
                                                                  const float* __restrict__ dx,
                                                                  float* __restrict__ part, int64_t M, int H4,
                                                                  int64_t rows_per) {
  // threads: kBlock / 64 row lanes x 64 column float4 groups (H4 <= 64 * gridDim.x)
  const int hc = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rl = threadIdx.x >> 6;   // 0..3
  const int64_t r0 = (int64_t)blockIdx.y * rows_per;
  int64_t r1 = r0 + rows_per;
  if (r1 > M) r1 = M;
  float4 s[kEmbTypes];
#pragma unroll
  for (int k = 0; k < kEmbTypes; ++k) s[k] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (hc < H4) {
    for (int64_t m = r0 + rl; m < r1; m += kBlock / 64) {
      const float4 g = reinterpret_cast<const float4*>(dx)[m * H4 + hc];
      const int ty = tt ? (int)tt[m] : 0;
#pragma unroll
      for (int k = 0; k < kEmbTypes; ++k)
        if (ty == k) { s[k].x += g.x; s[k].y += g.y; s[k].z += g.z; s[k].w += g.w; }
    }
  }
  __shared__ float4 sh[kBlock / 64][kEmbTypes][64];
#pragma unroll
  for (int k = 0; k < kEmbTypes; ++k) sh[rl][k][threadIdx.x & 63] = s[k];
  __syncthreads();
  if (rl == 0 && hc < H4) {
#pragma unroll
    for (int k = 0; k < kEmbTypes; ++k) {
      float4 a = sh[0][k][threadIdx.x];
      for (int l = 1; l < kBlock / 64; ++l) {
        const float4 b = sh[l][k][threadIdx.x];
        a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
      }
      reinterpret_cast<float4*>(part)[((int64_t)blockIdx.y * kEmbTypes + k) * H4 + hc] = a;
    }
  }
}

// one wave per output float4 (type k, column h): lanes take parts p = lane,
// lane + 64, ... in order, then a fixed-order butterfly (deterministic)
__global__ __launch_bounds__(kBlock) void emb_type_final_kernel(const float* __restrict__ part, float* __restrict__ dWt,
                                                                int nparts, int NT, int H4) {
  const int i = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);   // over NT * H4
  const int lane = threadIdx.x & 63;
  if (i >= NT * H4) return;
  const int k = i / H4, h = i - k * H4;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (k < kEmbTypes) {
    for (int p = lane; p < nparts; p += 64) {
      const float4 b = reinterpret_cast<const float4*>(part)[((int64_t)p * kEmbTypes + k) * H4 + h];
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
  }
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) {
    a.x += __shfl_xor(a.x, d, 64);
    a.y += __shfl_xor(a.y, d, 64);
    a.z += __shfl_xor(a.z, d, 64);
    a.w += __shfl_xor(a.w, d, 64);
  }
  if (lane == 0) reinterpret_cast<float4*>(dWt)[i] = a;
}

constexpr int kEmbTypeParts = 256;

constexpr int kEmbLight = 64;   // ids with more tokens in a step are summed in chunks
constexpr int kEmbChunk = 16;   // tokens per chunk wave (2560 [MASK] tokens: 160 waves)
static_assert(kEmbLight <= 64 && kEmbChunk <= 64, "one token position per lane");

// ---- word-table backward over the stable id sort (sid = sorted ids, order =
// their token positions, ascending within one id): run bounds per id, heavy
// ids (> 64 tokens) split into 64-token chunks summed by one wave each, then
// one wave per vocabulary row writes the row from its tokens (light) or its
// chunk partials (heavy) in ascending order -- deterministic, no fp32 atomics.
__global__ __launch_bounds__(kBlock) void emb_bounds_kernel(const int64_t* __restrict__ sid, int* __restrict__ rstart,
                                                            int* __restrict__ rend, int64_t M) {
  const int64_t s = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (s >= M) return;
  const int64_t v = sid[s];
  if (s == 0 || sid[s - 1] != v) rstart[v] = (int)s;
  if (s == M - 1 || sid[s + 1] != v) rend[v] = (int)s;
}

__global__ __launch_bounds__(kBlock) void emb_chunks_kernel(const int* __restrict__ rstart,
                                                            const int* __restrict__ rend, int* __restrict__ cbase,
                                                            int* __restrict__ chunk_row, int* __restrict__ counter,
                                                            int V) {
  const int v = blockIdx.x * kBlock + threadIdx.x;
  if (v >= V) return;
  const int n = rend[v] - rstart[v] + 1;
  if (n <= kEmbLight) return;
  const int nc = (n + kEmbChunk - 1) / kEmbChunk;
  const int base = atomicAdd(counter, nc);   // slot order varies; chunk contents and per-row order do not
  cbase[v] = base;
  for (int c = 0; c < nc; ++c) chunk_row[base + c] = v;
}

template <int Q>
__device__ __forceinline__ void emb_add_row(float4* acc, const float* __restrict__ dx, int64_t m, int H4, int lane) {
  const float4* src = reinterpret_cast<const float4*>(dx) + m * H4;
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const int h = lane + 64 * q;
    if (h < H4) {
      const float4 g = src[h];
      acc[q].x += g.x; acc[q].y += g.y; acc[q].z += g.z; acc[q].w += g.w;
    }
  }
}

// acc += rows row(0), row(1), ..., row(n-1) of src (H4 float4 each) in that
// order, four rows' loads in flight at a time (the adds stay in order)
template <typename RowOf>
__device__ __forceinline__ void emb_sum_rows(float4* acc, const float* __restrict__ src, int n, RowOf row, int H4,
                                             int lane) {
  const float4* s4 = reinterpret_cast<const float4*>(src);
  int i = 0;
  for (; i + 4 <= n; i += 4) {
    float4 g[4][4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t r = row(i + u);
#pragma unroll
      for (int q = 0; q < 4; ++q) g[u][q] = lane + 64 * q < H4 ? s4[r * H4 + lane + 64 * q] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        acc[q].x += g[u][q].x; acc[q].y += g[u][q].y; acc[q].z += g[u][q].z; acc[q].w += g[u][q].w;
      }
  }
  for (; i < n; ++i) emb_add_row<4>(acc, src, row(i), H4, lane);
}

// one wave per heavy chunk slot w < *counter: partial[w] = sum of its <= kEmbChunk tokens
__global__ __launch_bounds__(kBlock) void emb_heavy_kernel(const int64_t* __restrict__ order,
                                                           const int* __restrict__ rstart, const int* __restrict__ rend,
                                                           const int* __restrict__ cbase,
                                                           const int* __restrict__ chunk_row,
                                                           const int* __restrict__ counter,
                                                           const float* __restrict__ dx, float* __restrict__ partial,
                                                           int maxc, int H4) {
  const int w = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (w >= maxc || w >= *counter) return;
  const int v = chunk_row[w];
  const int c = w - cbase[v];
  const int s0 = rstart[v] + kEmbChunk * c;
  int s1 = s0 + kEmbChunk;
  if (s1 > rend[v] + 1) s1 = rend[v] + 1;
  float4 acc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) acc[q] = make_float4(0.f, 0.f, 0.f, 0.f);
  // the chunk's token positions, one per lane, broadcast by shuffles
  const int64_t mine = s0 + lane < s1 ? order[s0 + lane] : 0;
  emb_sum_rows(acc, dx, s1 - s0, [&](int i) { return (int64_t)__shfl((long long)mine, i, 64); }, H4, lane);
  float4* dst = reinterpret_cast<float4*>(partial) + (int64_t)w * H4;
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (lane + 64 * q < H4) dst[lane + 64 * q] = acc[q];
}

// one wave per vocabulary row (4 rows per block): every row of dWw written
__global__ __launch_bounds__(kBlock) void emb_word_gather_kernel(const int64_t* __restrict__ order,
                                                                 const int* __restrict__ rstart,
                                                                 const int* __restrict__ rend,
                                                                 const int* __restrict__ cbase,
                                                                 const float* __restrict__ dx,
                                                                 const float* __restrict__ partial,
                                                                 float* __restrict__ dWw, int V, int H4) {
  const int v = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (v >= V) return;
  const int s0 = rstart[v], n = rend[v] - s0 + 1;
  float4 acc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) acc[q] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (n <= kEmbLight) {
    const int64_t mine = lane < n ? order[s0 + lane] : 0;   // n <= kEmbLight = 64: one position per lane
    emb_sum_rows(acc, dx, n, [&](int i) { return (int64_t)__shfl((long long)mine, i, 64); }, H4, lane);
  } else {
    const int base = cbase[v], nc = (n + kEmbChunk - 1) / kEmbChunk;
    emb_sum_rows(acc, partial, nc, [&](int i) { return (int64_t)(base + i); }, H4, lane);
  }
  float4* dst = reinterpret_cast<float4*>(dWw) + (int64_t)v * H4;
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (lane + 64 * q < H4) dst[lane + 64 * q] = acc[q];
}

}  // namespace

int emb_type_parts() { return kEmbTypeParts; }
bool emb_supported(int H, int NT) { return H % 4 == 0 && H / 4 <= 256 && NT <= kEmbTypes; }
// heavy ids (n > kEmbLight tokens): ceil(n / kEmbChunk) <= 2n / kEmbChunk chunks each
int64_t emb_word_maxc(int64_t M) { return 2 * M / kEmbChunk + 1; }
int64_t emb_word_ws_ints(int64_t V, int64_t M) { return 3 * V + 1 + emb_word_maxc(M); }

void emb_forward(const int64_t* ids, const int64_t* tt, const float* Ww, const float* Wp, const float* Wt, float* out,
                 int64_t M, int T, int H, hipStream_t s) {
  const int H4 = H / 4;
  const int64_t n = M * H4;
  hipLaunchKernelGGL(emb_fwd_kernel, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, ids, tt, Ww, Wp,
                     Wt, out, M, T, H4);
}

void emb_backward(const int64_t* ids, const int64_t* tt, const float* dx, float* dWw, float* dWp, float* dWt,
                  float* part, const int64_t* sid, const int64_t* order, int* wws, float* wpart, int64_t V,
                  int64_t M, int B, int T, int P, int NT, int H, hipStream_t s) {
  (void)ids;
  const int H4 = H / 4;
  if (dWw && sid) {   // stable-sort buckets + gathers: every row of dWw written (no zero fill)
    int* rstart = wws;
    int* rend = wws + V;
    int* cbase = wws + 2 * V;
    int* counter = wws + 3 * V;
    int* chunk_row = counter + 1;
    const int maxc = (int)emb_word_maxc(M);
    hipMemsetAsync(rstart, 0, sizeof(int) * V, s);
    hipMemsetAsync(rend, 0xff, sizeof(int) * V, s);   // -1: absent (n = 0)
    hipMemsetAsync(counter, 0, sizeof(int), s);
    hipLaunchKernelGGL(emb_bounds_kernel, dim3((unsigned)((M + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, sid, rstart,
                       rend, M);
    hipLaunchKernelGGL(emb_chunks_kernel, dim3((unsigned)((V + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, rstart, rend,
                       cbase, chunk_row, counter, (int)V);
    hipLaunchKernelGGL(emb_heavy_kernel, dim3((unsigned)((maxc + kBlock / 64 - 1) / (kBlock / 64))), dim3(kBlock), 0, s,
                       order, rstart, rend, cbase, chunk_row, counter, dx, wpart, maxc, H4);
    hipLaunchKernelGGL(emb_word_gather_kernel, dim3((unsigned)((V + kBlock / 64 - 1) / (kBlock / 64))), dim3(kBlock), 0,
                       s, order, rstart, rend, cbase, dx, wpart, dWw, (int)V, H4);
  }
  if (dWp)
    hipLaunchKernelGGL(emb_pos_bwd_kernel, dim3((unsigned)(((int64_t)P * H4 + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                       s, dx, dWp, B, T, P, H4);
  if (dWt) {
    const int64_t rows_per = (M + kEmbTypeParts - 1) / kEmbTypeParts;
    const int nparts = (int)((M + rows_per - 1) / rows_per);
    hipLaunchKernelGGL(emb_type_partial_kernel, dim3((unsigned)((H4 + 63) / 64), (unsigned)nparts), dim3(kBlock), 0, s,
                       tt, dx, part, M, H4, rows_per);
    hipLaunchKernelGGL(emb_type_final_kernel, dim3((unsigned)((NT * H4 + kBlock / 64 - 1) / (kBlock / 64))),
                       dim3(kBlock), 0, s, part, dWt, nparts, NT, H4);
  }
}

}  // namespace gk
