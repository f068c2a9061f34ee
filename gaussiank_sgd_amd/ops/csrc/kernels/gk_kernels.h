// Host-side launcher API of the gfx950 kernel library.
//
// Every launcher is asynchronous on the given stream, performs no host
// synchronisation and no allocation (workspaces are passed in), so any
// sequence of them can be captured into a hipGraph.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace gk {

// ---------------------------------------------------------------------------
// Threshold-selection modes of the fused compressor pipeline.
// ---------------------------------------------------------------------------
enum Mode : int {
  kModeGaussian = 0,      // mu + z*sigma, <= `loops` x0.5/x1.5 refinements (compression.py:358-389,405-435)
  kModeRedSync = 1,       // binary search of mean|x| + r(max|x|-mean|x|) (compression.py:623-691)
  kModeRedSyncTrim = 2,   // r = 0.8, 0.6, ... until nnz >= k (compression.py:694-738)
  kModeTopK = 3,          // exact top-k by radix select on |x|
  kModeRandomK = 4,       // k smallest hashes: a uniformly random k-subset
  kModeThreshold = 5,     // fixed threshold |x| > t
  kModeDGC = 6,           // 1% sample threshold, exact top-k when > 4k/3 (compression.py:555-620)
  kModeGaussianCal = 7,   // calibrated Gaussian-k: 8-candidate ladder (kCalCand) around a per-bucket
                          // adaptive centre, closest count to k in [2k/3, 4k/3], exact radix top-k otherwise
};

// Fallback markers written to the record header's `chosen` word: the
// calibrated mode found no candidate in range and used the exact radix key
// (top-k); a threshold mode's choice exceeded k_cap and no evaluated
// candidate fitted, so the exact radix key at k_cap was used (top-k_cap).
constexpr int kCalFallback = 16;
constexpr int kOverflowExact = 17;

constexpr int kMaxCand = 16;
constexpr int kRecHdr = 4;   // packed record header words: sent, total, chosen, thr
constexpr int kMaxCountBlocks = 1024;
constexpr int kMaxStatsBlocks = 2048;
constexpr int kRadixBins0 = 2048;  // key bits [31:21]
constexpr int kRadixBins1 = 2048;  // key bits [20:10]
constexpr int kRadixBins2 = 1024;  // key bits [9:0]

// Device-resident control block of one compression call.  Lives in a
// caller-provided buffer of sizeof(GkCtrl) bytes.
struct GkCtrl {
  double raw[4];        // sum, sumsq, sum|x|, max|x|
  double mean, stdev, meanabs, maxabs;
  uint32_t bound[kMaxCand];   // candidate j selects key >= bound[j]
  int32_t ncand;
  int32_t chosen;
  uint32_t sel_bound;   // select key >= sel_bound ...
  uint32_t eq_key;      // ... or key == eq_key within eq_quota (radix ties)
  int64_t eq_quota;
  int64_t total;        // true number selected
  int64_t sent;         // min(total, k_cap)
  int64_t k_eff;
  float thr;            // chosen threshold (|x| units) for logging
  int32_t pad0;
  uint32_t radix_key[2];      // [0] sampled (DGC), [1] exact
  int64_t radix_kremain[2];
  double cand_thr[kMaxCand];  // candidate thresholds in |x| units (logging/tests)
  // calibrated Gaussian-k state, persistent across calls on one bucket
  double cal_c;         // ladder centre / sigma
  double cal_step;      // log spacing of the ladder
  int64_t cal_k;        // k the state was calibrated for (re-initialised when k changes)
  int32_t fallback;     // this call fell back to the exact radix key (1: top-k, 2: top-k_cap)
  // sticky count of bounded spins that expired in decide_fb_kernel (a grid
  // that was not co-resident: that call's selection is not trustworthy);
  // never reset by the kernels, read by ops.ctrl_fields / bench.py
  uint32_t sync_timeouts;
  // entries above the reference rule's threshold when that exceeded k_cap and
  // the selection moved to a tighter candidate / the exact key (header word
  // `total`); -1 when the reference choice fitted
  int64_t ref_total;
};

static_assert(offsetof(GkCtrl, sync_timeouts) == 364, "ops/__init__.py CTRL_SYNC_TIMEOUTS_U32 = 364 / 4");

struct Chunk;

struct CompressArgs {
  float* g = nullptr;          // raw gradient bucket; zeroed when zero_g
  float* r = nullptr;          // residual in; (g + r) then new residual out
  int64_t n = 0;
  int64_t n_stats = 0;          // elements used to normalise statistics (<=0: n)
  int mode = kModeGaussian;
  int ec = 1;                  // add residual before selection
  int zero_g = 1;
  int loops = 3;               // gaussian refinement iterations
  double z = 0.0;              // gaussian |z| multiplier
  double fixed_thr = 0.0;      // kModeThreshold
  double sample_p = 0.01;      // kModeDGC
  int64_t k = 1;
  int64_t k_cap = 1;
  uint32_t seed = 0;
  const uint32_t* seed_dev = nullptr;   // optional: seed read from device memory (graph replays)
  void* ctrl = nullptr;        // GkCtrl
  void* ws = nullptr;          // gk_compress_workspace_bytes(n)
  int32_t* record = nullptr;   // [4 + 2*k_cap] int32: hdr | idx | val(fp32 bits)
  float* stats_out = nullptr;  // optional [4] copy of mean, std, meanabs, maxabs (fp32)
  // optional validity bitmask over the n elements (bit i = 1: real element,
  // 0: arena padding); hash-key modes (random-k) never pick invalid slots
  const uint32_t* valid = nullptr;
  // optional DGC momentum correction fused into the statistics pass:
  //   u = mu * u + g + wd * w;  acc = u (+ r);  ...  and u[idx] = 0 for every
  // sent index (momentum factor masking) in the select pass.  The chunk table
  // rows [chunk_begin, chunk_begin + chunk_count) tile this bucket; their
  // `start` is an arena offset, `chunk_base` the bucket's arena offset.
  float* u = nullptr;
  const float* w = nullptr;
  const Chunk* chunks = nullptr;
  int chunk_begin = 0, chunk_count = 0;
  int64_t chunk_base = 0;
  float mc_mu[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  float mc_wd[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  // single-workgroup hand-offs (finalize / decide): -1 = GKSGD_HANDOFF
  // (default: separate 1-workgroup launches), 0 = launches, 1 = in the last
  // block of the producing grid (no new dispatch: the bucket compressions
  // that overlap the backward pass, where a 1-workgroup launch waits behind
  // the GEMM blocks filling the chip)
  int handoff = -1;
};

size_t compress_workspace_bytes(int64_t n);
void compress(const CompressArgs& a, hipStream_t stream);

// Stand-alone statistics (no residual) for tests / the bucket planner.
void tensor_stats(const float* x, int64_t n, void* ctrl, void* ws, hipStream_t stream);

// ---------------------------------------------------------------------------
// Sparse aggregation: dst[idx] += val * scale for every rank's record.
// records: [P][4 + 2*k_cap] int32.  Atomic (default) or per-rank ordered.
// ---------------------------------------------------------------------------
void scatter_add_records(float* dst, int64_t n, const int32_t* records, int P, int64_t k_cap,
                         float scale, int deterministic, hipStream_t stream);
// Sparse SGD apply straight from the records (DGC momentum correction: the
// global update is plain SGD on the aggregate):  w[i] -= lr * (sum_r val_r[i]) * scale
// for every index in any record, sums in rank order; w_bf16 (optional) is
// refreshed at the same indices; lr_mult (optional device scalar) multiplies lr.
void apply_records_sgd(float* w, uint16_t* w_bf16, int64_t n, const int32_t* records, int P, int64_t k_cap,
                       float scale, float lr, const float* lr_mult, hipStream_t stream);
// 16-byte digest of a flat fp32 arena (replica consistency checks):
// out[0] = fp64 sum (bits), out[1] = order-independent 64-bit hash of the bits.
void arena_digest(const float* x, int64_t n, uint64_t* out, uint64_t* ws, hipStream_t stream);
void fill_zero(float* dst, int64_t n, hipStream_t stream);

// ---------------------------------------------------------------------------
// Sign-bucket mean compressor (BucketCompressor, compression.py:227-312).
// ---------------------------------------------------------------------------
size_t sign_bucket_workspace_bytes(int64_t n);
// means_out[2] = {mean(x>=0), mean(x<0)}; x -= mean per bucket; mask[i]=x>=0
void sign_bucket_compress(float* x, int64_t n, uint8_t* mask, float* means_out, void* ws,
                          hipStream_t stream);
void sign_bucket_decompress(float* x, int64_t n, const uint8_t* mask, const float* means,
                            hipStream_t stream);

// ---------------------------------------------------------------------------
// Fused optimizers over a chunk table (multi-tensor apply over flat arenas).
// ---------------------------------------------------------------------------
struct Chunk {
  int64_t start;      // element offset in the arenas
  int32_t len;        // elements (<= kChunkElems)
  int16_t group;      // param-group id (hyper-parameters)
  int16_t seg;        // tensor id (LARS trust ratios)
};
constexpr int kChunkElems = 16384;
constexpr int kMaxGroups = 8;

struct SgdGroup {
  float lr, momentum, dampening, weight_decay;
  int nesterov;
  int first_step;     // momentum buffer not yet initialised -> buf = d
  float pad0, pad1;
};
struct SgdArgs {
  float* w = nullptr;
  float* m = nullptr;        // may be null when no group uses momentum
  float* g = nullptr;
  const Chunk* chunks = nullptr;
  int nchunks = 0;
  SgdGroup groups[kMaxGroups];
  int ngroups = 0;
  int zero_grad = 1;
  const float* grad_scale = nullptr;  // optional device scalar (clip coefficient)
  uint16_t* w_bf16 = nullptr;         // optional bf16 shadow of w written in the same pass
  const float* lr_mult = nullptr;     // optional device scalar multiplying every group's lr (graph replay)
};
void fused_sgd(const SgdArgs& a, hipStream_t stream);

// DGC momentum correction over a chunk range: u = mu*u + g + wd*w; g = u.
struct McArgs {
  float* u = nullptr;
  float* g = nullptr;
  const float* w = nullptr;
  const Chunk* chunks = nullptr;
  int nchunks = 0;
  float momentum[kMaxGroups];
  float weight_decay[kMaxGroups];
};
void momentum_correct(const McArgs& a, hipStream_t stream);
// momentum factor masking: u[idx] = 0 for the indices of one packed record
void mask_records(float* u, const int32_t* record, int64_t k_cap, hipStream_t stream);

// dst[i] += float(src[i]) for a bf16 (src_bytes 2) or fp32 (4) gradient: the
// fused "cast + AccumulateGrad" of a parameter gradient into its fp32 arena slot.
void accum_grad(float* dst, const void* src, int64_t n, int src_bytes, hipStream_t stream);
// dst = bf16(src) (shadow refresh)
void cast_bf16(uint16_t* dst, const float* src, int64_t n, hipStream_t stream);

// Per-segment sum of squares: out[2*seg] += sum w^2, out[2*seg+1] += sum g^2.
void segmented_sumsq(const float* w, const float* g, const Chunk* chunks, int nchunks, double* out,
                     hipStream_t stream);

struct LarsArgs {
  float* w = nullptr;
  float* m = nullptr;        // 'acceleration' buffer (initialised to ones, lars.py:116-118)
  const float* g = nullptr;
  const Chunk* chunks = nullptr;
  int nchunks = 0;
  const double* seg_sumsq = nullptr;  // from segmented_sumsq
  float lr[kMaxGroups], momentum[kMaxGroups], weight_decay[kMaxGroups], eeta[kMaxGroups],
      epsilon[kMaxGroups];
  int ngroups = 0;
};
void fused_lars(const LarsArgs& a, hipStream_t stream);

// Global-norm gradient clipping without a host sync: computes
// coef = min(1, max_norm / (||g|| + 1e-6)) into coef_out and scales g.
void clip_grad_norm(float* g, int64_t n, float max_norm, double* ws, float* coef_out,
                    float* norm_out, hipStream_t stream);

// ---------------------------------------------------------------------------
// Fused batch norm (training) + residual add + ReLU, channels-last [M, C].
// elem_bytes: 2 (bf16) or 4 (fp32).  ws: bn_workspace_floats() floats.
// ---------------------------------------------------------------------------
size_t bn_workspace_floats(int64_t M, int C, int elem_bytes);
// fin_state (optional, bn_fin_state_bytes(C), zero-initialised once, kept per
// layer): the finalize of the statistics runs inside the apply pass that
// consumes it (bn_act.hip FinSync) instead of as a separate launch; ignored
// under stream capture.
size_t bn_fin_state_bytes(int C);
bool bn_supported(int C, int elem_bytes);
// workgroups per streaming BN pass (default 1024, clamped to [64, 4096]; bench/bn_probe.py)
void bn_set_blocks(int blocks);
size_t bn_mask_bytes(int64_t M, int C, int elem_bytes);
// the statistics pass of bn_act_forward alone (per-block sum / sum-of-squares
// partials into ws): what a convolution without the statistics epilogue costs
// the BN that consumes it (the autotuner times MIOpen candidates with it)
void bn_stats_partials(const void* x, int64_t M, int C, int elem_bytes, float* ws, hipStream_t s);
void bn_act_forward(const void* x, const void* res, void* y, uint8_t* mask, int64_t M, int C, int elem_bytes,
                    const float* w, const float* b, float eps, float momentum, float* run_mean, float* run_var,
                    float* save_mean, float* save_invstd, float* scale, float* shift, float* ws, int relu,
                    int64_t* nbt, hipStream_t stream, void* fin_state = nullptr, const float* rscale = nullptr,
                    const float* rshift = nullptr);
// rscale / rshift (optional, with res): the residual is a batch-normalised
// tensor whose apply was deferred here -- res * rscale + rshift is added.
// bn_act_finalize: the statistics (psum == nullptr: the stats pass over x;
// else the producer's [gy][C] partials) and the finalize of a BN whose apply
// pass is deferred into its consumer; no apply.
void bn_act_finalize(const void* x, int64_t M, int C, int elem_bytes, const float* psum, const float* psq, int gy,
                     const float* w, const float* b, float eps, float momentum, float* run_mean, float* run_var,
                     float* save_mean, float* save_invstd, float* scale, float* shift, float* ws, int64_t* nbt,
                     hipStream_t stream);
// dy2 (optional): a second upstream gradient of the same output, summed on load.
// bn_act_forward with the batch statistics already reduced to per-row
// partials (psum / psq: [gy][C] each), e.g. by the producing
// convolution's epilogue (gemm_nt / conv_nt `stats`).
void bn_act_forward_pre(const void* x, const void* res, void* y, uint8_t* mask, int64_t M, int C, int elem_bytes,
                        const float* psum, const float* psq, int gy, const float* w, const float* b, float eps, float momentum,
                        float* run_mean, float* run_var, float* save_mean, float* save_invstd, float* scale,
                        float* shift, int relu, int64_t* nbt, hipStream_t stream, void* fin_state = nullptr,
                        const float* rscale = nullptr, const float* rshift = nullptr);
// dz and its [2][gy][C] partials sum(dz), sum(dz * x) come from a grad-input
// GEMM's BatchNorm-backward epilogue (BnBwdArgs below); finalize (centring
// with the mean) + apply only.  bf16 (elem_bytes 2) or fp32 (4).
// Lazy BN backward (no apply pass): dx = k1 * ((dz - k2) - (x - mu) * k4) is
// computed by the consumer GEMMs (gemm.hip LazyA / LazyG) from dz, x and
// coef[C] = {k1, k2, mu, k4}; padz / padx ([C], activation dtype) are the
// padding rows that make a padded tap contribute exactly 0.
//   bn_bwd_finalize_lazy: from [2][gy][C] partials (center: sum(dz*x) form)
//   bn_act_backward_lazy: full path, the reduce pass writes dz
//   bn_lazy_apply       : materialise dx (for a consumer without the lazy path)
void bn_bwd_finalize_lazy(const float* pdb, const float* pdg, int gy, int64_t M, int C, int elem_bytes, int center,
                          const float* w, const float* mean, const float* invstd, float* dgamma, float* dbeta,
                          float* gw_acc, float* gb_acc, float* coef, void* padz, void* padx, hipStream_t stream);
void bn_act_backward_lazy(const void* dy, const void* dy2, const uint8_t* mask, const void* x, void* dz, int64_t M,
                          int C, int elem_bytes, const float* w, const float* mean, const float* invstd,
                          float* dgamma, float* dbeta, float* ws, int relu, float* gw_acc, float* gb_acc, float* coef,
                          void* padz, void* padx, hipStream_t stream);
void bn_lazy_apply(const void* dz, const void* x, void* dx, int64_t M, int C, int elem_bytes, const float* coef,
                   hipStream_t stream);
// bn_act_backward_pre of a BN whose residual was the deferred BN of x2
// (bn_act_forward rscale / rshift): also that BN's reduce (over dz, x2) and
// finalize, and its dx2 written by the same apply pass; ws2 >= bn_workspace_floats.
void bn_act_backward_pre_dual(const void* dz, const void* x, void* dx, int64_t M, int C, int elem_bytes,
                              const float* w, const float* mean, const float* invstd, float* dgamma, float* dbeta,
                              const float* pdb, const float* pdg, int gy, float* gw_acc, float* gb_acc, const void* x2,
                              void* dx2, const float* w2, const float* mean2, const float* invstd2, float* dgamma2,
                              float* dbeta2, float* ws2, float* gw2_acc, float* gb2_acc, hipStream_t stream);
void bn_act_backward_pre(const void* dz, const void* x, void* dx, int64_t M, int C, int elem_bytes, const float* w,
                         const float* mean, const float* invstd, float* dgamma, float* dbeta, const float* pdb,
                         const float* pdg, int gy, float* gw_acc, float* gb_acc, hipStream_t stream,
                         void* fin_state = nullptr);
void bn_act_backward(const void* dy, const void* dy2, const uint8_t* mask, const void* x, void* dx, void* dres,
                     int64_t M, int C, int elem_bytes, const float* w, const float* mean, const float* invstd,
                     float* dgamma, float* dbeta, float* ws, int relu, float* gw_acc, float* gb_acc,
                     hipStream_t stream, void* fin_state = nullptr);

// BN (training) + ReLU + k x k / stride s / pad p max-pool, channels-last
// [N, H, W, C] -> [N, OH, OW, C].  amax: one byte per OUTPUT element (window
// position of the max, 0xff when the ReLU blocks the gradient).  The backward
// gathers the pool gradient straight into the BN backward passes.
// Requires N*H*W < 2^32.
struct PoolGeo {
  int H, W, OH, OW, k, s, p;
};
void bn_relu_pool_forward_pre(const void* x, void* y, uint8_t* amax, int64_t N, int C, PoolGeo pg, int elem_bytes,
                              const float* psum,
                              const float* psq, int gy, const float* w, const float* b, float eps, float momentum,
                              float* run_mean, float* run_var, float* save_mean, float* save_invstd, float* scale,
                              float* shift, int64_t* nbt, hipStream_t stream);
void bn_relu_pool_forward(const void* x, void* y, uint8_t* amax, int64_t N, int C, PoolGeo pg, int elem_bytes,
                          const float* w, const float* b, float eps, float momentum, float* run_mean, float* run_var,
                          float* save_mean, float* save_invstd, float* scale, float* shift, float* ws, int64_t* nbt,
                          hipStream_t stream);
void bn_relu_pool_backward(const void* dy, const void* dy2, const uint8_t* amax, const void* x, void* dx, int64_t N,
                           int C, PoolGeo pg, int elem_bytes, const float* w, const float* mean, const float* invstd,
                           float* dgamma, float* dbeta, float* ws, float* gw_acc, float* gb_acc, hipStream_t stream);

// ---------------------------------------------------------------------------
// MFMA GEMMs and implicit-GEMM convolutions over channels-last activations
// (gemm.hip).  Operands bf16 (v_mfma_f32_16x16x32_bf16) or, with f32 = true,
// fp32 (v_mfma_f32_16x16x4_f32: exact fp32 products, fp32 accumulation).
// N, K multiples of 64 (gemm_supported).
//   gemm_nt    : C[M, N] (operand dtype) = A[M, K] . B[N, K]^T
//   gemm_tn_acc: W[N, K] (fp32) += G[M, N]^T . X[M, K]   (float atomics)
// cfg <= 0 picks the tile shape from N (and K); max_blocks / splits <= 0
// pick the grid.
// ---------------------------------------------------------------------------
bool gemm_supported(int64_t N, int64_t K);
// BatchNorm-backward epilogue of a grad-input GEMM (bn != nullptr): C receives
// dz = mask ? dy + dy2 : 0 instead of dy (dy rounded to the operand dtype), and
// `stats` the per-workgroup partials sum(dz), sum(dz * h) -- feed them to
// bn_act_backward_pre.  h / dy2 share C's row stride and dtype; mask is the BN
// forward's 1-bit ReLU mask (bn_act.hip layout).
struct BnBwdArgs {
  const void* h;
  const void* dy2;
  const uint8_t* mask;
};
// Lazy BN-backward operand (fp32; bn_bwd_finalize_lazy): the A operand of
// gemm_nt / conv_nt / conv_nt_remap (or G of the grad-weight) is
// dx = k1 ((dz - k2) - (x - mu) k4) computed in-kernel from dz (the operand
// pointer) and x (same layout); returns -1 when the coefficient table does not
// fit next to the tiles in LDS.
struct LazyArgs {
  const void* x;
  const float* coef;   // [C][4]
  const void* padz;    // [C]
  const void* padx;    // [C]
  int C;
};
// stats (optional): [2][stats_rows][N] fp32 BatchNorm partials (sum, sum of
// squares of the stored output) per workgroup row; returns the grid's row count
// (the partial rows written, <= stats_rows) -- feed it to bn_act_forward_pre.
// bias (optional): fp32 [N] added in the epilogue (before rounding and statistics)
int gemm_nt(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int64_t M, int N, int K,
            bool f32, int cfg, int max_blocks, float* stats, int stats_rows, const float* bias, const BnBwdArgs* bn,
            const LazyArgs* lazy, hipStream_t stream, float* splitk_ws = nullptr, const void* b3 = nullptr);
// C[M, N] (row stride ldc) = sum of the S fp32 planes ws[S][M][N] (+ bias), with the
// BatchNorm statistics partials (stats != nullptr) or the BN-backward epilogue (bn);
// returns the number of partial rows written (<= stats_rows)
int splitk_reduce(const float* ws, int S, int64_t M, int N, float* C, int64_t ldc, const float* bias, float* stats,
                  int stats_rows, const BnBwdArgs* bn, hipStream_t stream);
int gemm_tn_acc(const void* G, int64_t ldg, const void* X, int64_t ldx, float* W, int64_t ldw, int64_t M, int N,
                 int K, bool f32, int cfg, int splits, const LazyArgs* lazy, hipStream_t stream);
// Implicit-GEMM KHxKW convolution (stride S, zero padding P) over NHWC:
//   conv_nt    : Y[M = N*OH*OW, Cout] = im2col(X) . Wt[Cout, KH*KW*C]^T
//   conv_tn_acc: Wout[Cout, KH*KW*C] += G[M, Cout]^T . im2col(X)
// Weights are channels-last ([Cout][KH][KW][C]); C % 64 == 0; `zero` points at
// >= 128 zero bytes (the padding row).
int conv_nt(const void* X, const void* zero, int H, int W, int C, int OH, int OW, int S, int P, int KH, int KW,
            const void* B, void* Y, int64_t M, int N, bool f32, int cfg, int max_blocks, float* stats, int stats_rows,
            const float* bias, const BnBwdArgs* bn, const LazyArgs* lazy, hipStream_t stream,
            float* splitk_ws = nullptr, const void* b3 = nullptr);
// fp32 [R, S] (row stride ld, S % 32 == 0) -> bf16 planes [R][S / 32][3][32]:
// the pre-split B operand of the bf16x6 register-staged kernels (cfg family 3)
void split3_rows(const float* src, int64_t ld, void* dst, int64_t R, int S, hipStream_t stream);
// One parity class (RA, RB) of a stride-2 convolution's grad-input as a stride-1,
// padding-0 KHxKW implicit GEMM over dY (H x W x C, the forward output) whose
// OH x OW output grid is stored at rows (n*RH + 2 oh + RA) * RW + 2 ow + RB of
// the RH x RW grad-input (RZ: zeros at the other three parities); KH = KW = 1
// runs the plain row GEMM over X = dY rows (row stride ldx).
int conv_nt_remap(const void* X, int64_t ldx, const void* zero, int H, int W, int C, int OH, int OW, int KH, int KW,
                  const void* B, void* Y, int64_t M, int N, int RH, int RW, int RA, int RB, int RZ, bool f32, int cfg,
                  int max_blocks, const LazyArgs* lazy, hipStream_t stream);
int conv_tn_acc(const void* G, const void* X, const void* zero, int H, int W, int C, int OH, int OW, int S, int P,
                 int KH, int KW, float* Wout, int64_t M, int N, bool f32, int cfg, int splits, const LazyArgs* lazy,
                 hipStream_t stream);
// Winograd F(2x2, 3x3) fp32 convolution, stride 1, padding 1 (winograd.hip).
//   wino_weights: filter transform of w ([Co][3][3][Ci] channels-last fp32;
//                 flip = 1: of the grad-input filter W'[c][kh][kw][k] =
//                 W[k][2-kh][2-kw][c], w then being the forward [K][3][3][C])
//                 into u = [Ci/8][16][Co][8]
//   wino_conv   : y[N, H, W, Co] = conv3x3(x[N, H, W, Ci]) from u; Ci % 8 == 0,
//                 Co % 64 == 0; optional BatchNorm statistics / BN-backward
//                 epilogue (as conv_nt); returns the partial rows written.
// fp32 ResNet stem (stem_f32.hip): x NHWC fp32 [N, 224, 224, 3], w [64][3][7][7]
// fp32 with element strides s0..s3, y NHWC fp32 [N, 112, 112, 64]; forward
// returns the BatchNorm partial rows written; grad-weight adds into out
// (strided like w) through per-block partials (stem_f32_wgrad_blocks(N) x 64 x 148).
bool stem_f32_supported(int H, int W);
int stem_f32_wgrad_blocks(int N);
// bf16x6 stem forward (fp32-accurate): wp3 = a workspace of stem_f32x6_wplanes()
// bf16 elements that receives the three split planes of w
int stem_f32x6_wplanes();
int stem_f32x6_forward(const float* x, int N, int H, int W, const float* w, int64_t s0, int64_t s1, int64_t s2,
                       int64_t s3, uint16_t* wp3, float* y, float* stats, int stats_rows, hipStream_t stream);
int stem_f32_forward(const float* x, int N, int H, int W, const float* w, int64_t s0, int64_t s1, int64_t s2,
                     int64_t s3, float* y, float* stats, int stats_rows, hipStream_t stream);
void stem_f32_wgrad(const float* x, const float* dy, int N, int H, int W, float* part, float* out, int64_t s0,
                    int64_t s1, int64_t s2, int64_t s3, bool x6, hipStream_t stream);
void wino_weights(const float* w, float* u, int Co, int Ci, int flip, hipStream_t stream);
// Batched per-step weight re-layouts (prep.hip): one launch over a table of
// descriptors (device memory, block_begin ascending).  kind kPrepWino /
// kPrepWinoFlip: Winograd filter transform (R = Co, S = Ci of the conv run,
// as wino_weights); kPrepT32 / kPrepT16: out[s * ld_out + r] = in[r * ld_in + s]
// for an R x S matrix of 4- / 2-byte elements (64 x 64 LDS tiles, tiles_s =
// ceil(S / 64)).
// kPrepWinoX6 / kPrepWinoX6Flip: the bf16x6 Winograd filter planes (wino_x6_weights).
enum PrepKind : int32_t { kPrepWino = 0, kPrepWinoFlip = 1, kPrepT32 = 2, kPrepT16 = 3, kPrepWinoX6 = 4,
                          kPrepWinoX6Flip = 5 };
struct PrepDesc {
  const void* src;
  void* dst;
  int64_t ld_in, ld_out;
  int64_t block_begin;
  int32_t kind, R, S, tiles_s;
};
static_assert(sizeof(PrepDesc) == 56, "PrepDesc layout is packed by ops/weight_prep.py");
int64_t weight_prep_blocks(int kind, int R, int S);
int weight_prep_max_descs();
void weight_prep(const PrepDesc* descs, int ndesc, int64_t total_blocks, hipStream_t stream);
int wino_conv(const float* x, const float* u, float* y, int N, int H, int W, int Ci, int Co, int max_blocks,
              float* stats, int stats_rows, const BnBwdArgs* bn, hipStream_t stream, int splits = 1,
              float* split_ws = nullptr);
// bf16x6 (fp32-accurate) Winograd (wino_x6.hip): u3 = the filter transform
// split into three bf16 planes, [Ci/32][16][3][Co][32] (wino_x6_weights, flip
// as wino_weights); wino_x6_conv as wino_conv with Ci % 32 == 0, Co % 32 == 0
// (returns -1 otherwise).
void wino_x6_weights(const float* w, uint16_t* u3, int Co, int Ci, int flip, hipStream_t stream);
int wino_x6_conv(const float* x, const uint16_t* u3, float* y, int N, int H, int W, int Ci, int Co, int max_blocks,
                 float* stats, int stats_rows, const BnBwdArgs* bn, hipStream_t stream);
//   wino_wgrad  : out[K][3][3][C] (fp32, channels-last) += dW of the 3x3 stride-1
//                 convolution x[N, H, W, C] -> dy[N, H, W, K] (C, K % 64 == 0);
//                 part: wino_wgrad_splits(...) * 16 * K * C fp32 workspace
//                 (per-split partials, summed in a fixed order: deterministic)
int wino_wgrad_splits(int N, int H, int W, int C, int K, int splits);
void wino_wgrad(const float* x, const float* dy, float* part, float* out, int N, int H, int W, int C, int K,
                int splits, hipStream_t stream);

// ---------------------------------------------------------------------------
// ImageNet-ResNet stem: 7x7 / stride 2 / pad 3 convolution, 3 -> 64 channels
// (stem.hip).  x: NHWC [N, H, W, 3] fp32 or bf16; y: NHWC bf16 [N, OH, OW, 64];
// weights packed once per step into bf16 [64][224] (k = kh*32 + kw*4 + c) by
// stem_pack_weight from [64][3][7][7] fp32 with element strides s0..s3.
// stem_forward: optional per-block BatchNorm partials (sum, sum of squares)
// [2][stats_rows][64]; returns the rows written.  stem_wgrad: out (fp32,
// strides s0..s3) += dW, via per-block partials part[stem_wgrad_blocks * 64 * 224]
// summed in a fixed order.
// ---------------------------------------------------------------------------
bool stem_supported(int H, int W);
void stem_pack_weight(const float* w, int64_t s0, int64_t s1, int64_t s2, int64_t s3, uint16_t* wp,
                      hipStream_t stream);
int stem_forward(const void* x, bool x_f32, int N, int H, int W, const uint16_t* wp, uint16_t* y, float* stats,
                 int stats_rows, hipStream_t stream);
int stem_wgrad_blocks(int N, int H, int W);
void stem_wgrad(const void* x, bool x_f32, int N, int H, int W, const uint16_t* dy, float* part, float* out,
                int64_t s0, int64_t s1, int64_t s2, int64_t s3, hipStream_t stream);

// ---------------------------------------------------------------------------
// 3x3 / stride-1 / pad-1 convolution grad-weight, tap-parallel (wgrad3.hip):
// dy [N, H, W, K], x [N, H, W, C] channels-last bf16; out (fp32 [K][C][3][3]
// with element strides s0..s3) += dW via per-block partials
// part[wgrad3_ws_floats] summed in a fixed order; zero: >= 64 zero bf16.
// ---------------------------------------------------------------------------
bool wgrad3_supported(int H, int W, int C, int K);
int64_t wgrad3_ws_floats(int N, int H, int W, int C, int K);
void wgrad3_acc(const void* dy, const void* x, const void* zero, int N, int H, int W, int C, int K, float* part,
                float* out, int64_t s0, int64_t s1, int64_t s2, int64_t s3, hipStream_t stream);

// ---------------------------------------------------------------------------
// Fused multi-head self-attention, head dim 64 (attn.hip).  qkv / dqkv:
// [B, T, 3, H, 64] bf16; out / dout: [B, T, H, 64] bf16; lse / delta: fp32
// [B, H, T].  Dropout p on the attention probabilities with a hash mask
// (seed); attn_dropout_mask materialises the same mask as [B, H, T, T] bytes.
// seed_dev (optional): a device word mixed into the seed at run time
// (hash(*seed_dev, seed)) -- a captured graph draws a new mask every replay.
// ---------------------------------------------------------------------------
bool attn_supported(int T, int D);
// fp32 variants (attn_f32.hip): same layouts, fp32 qkv / out / dout / dqkv
bool attn_f32_supported(int T, int D);
void attn_f32_fwd(const float* qkv, float* out, float* lse, int B, int T, int H, float p, uint32_t seed,
                  const uint32_t* seed_dev, hipStream_t stream);
void attn_f32_bwd(const float* qkv, const float* out, const float* dout, const float* lse, float* delta, float* dqkv,
                  int B, int T, int H, float p, uint32_t seed, const uint32_t* seed_dev, hipStream_t stream);
void attn_fwd(const void* qkv, void* out, float* lse, int B, int T, int H, float p, uint32_t seed,
              const uint32_t* seed_dev, hipStream_t stream);
void attn_bwd(const void* qkv, const void* out, const void* dout, const float* lse, float* delta, void* dqkv, int B,
              int T, int H, float p, uint32_t seed, const uint32_t* seed_dev, hipStream_t stream);
void attn_dropout_mask(uint8_t* mask, int B, int H, int T, float p, uint32_t seed, const uint32_t* seed_dev,
                       hipStream_t stream);

// ---------------------------------------------------------------------------
// Fused BERT input embedding (embed.hip): out[m] = Ww[ids[m]] + Wp[m % T] + Wt[tt[m]]
// (fp32 [*, H], H % 4 == 0; tt may be null = type 0).  Backward: dWw (zeroed by
// the caller) += scatter of dx rows (fp32 atomics), dWp = sum over the batch
// (written, rows >= T zero), dWt = per-type sums through part
// (emb_type_parts() * 2 * H floats); any of the three may be null.
int emb_type_parts();
bool emb_supported(int H, int NT);
void emb_forward(const int64_t* ids, const int64_t* tt, const float* Ww, const float* Wp, const float* Wt, float* out,
                 int64_t M, int T, int H, hipStream_t s);
// sid / order: the ids stably sorted and their token positions; with them
// (and wws: emb_word_ws_ints(V, M) ints, wpart: emb_word_maxc(M) * H floats)
// dWw is WRITTEN row by row, deterministically (dWw requires sid / order).
int64_t emb_word_maxc(int64_t M);
int64_t emb_word_ws_ints(int64_t V, int64_t M);
void emb_backward(const int64_t* ids, const int64_t* tt, const float* dx, float* dWw, float* dWp, float* dWt,
                  float* part, const int64_t* sid, const int64_t* order, int* wws, float* wpart, int64_t V,
                  int64_t M, int B, int T, int P, int NT, int H, hipStream_t s);

// Fused softmax cross-entropy over bf16 logit rows (xent.hip), V even:
// forward writes lse[R] and loss[R] (0 for label == ignore); backward writes
// bf16 dlogits = (softmax - onehot) * (*scale) (0 rows for ignored labels).
bool xent_supported(int V);
void xent_forward(const void* logits, const int64_t* labels, float* lse, float* loss, int64_t R, int V, int64_t ignore,
                  hipStream_t s);
void xent_backward(const void* logits, const int64_t* labels, const float* lse, const float* scale, void* grad,
                   int64_t R, int V, int64_t ignore, hipStream_t s);

// Fused residual add (+ dropout) + LayerNorm over rows of H bf16 (ln.hip).
// forward : h = x + dropout_p(a), y = LN(h) * gamma + beta; saves h (bf16),
//           mean, rstd (fp32 per row).  The dropout mask is a hash of
//           (seed, row, column) -- recomputed in the backward, never stored.
// backward: dx = dLN/dh (residual branch), da = dx * mask / (1 - p) (null da:
//           no second output), dgamma / dbeta (+)= column sums; ws needs
//           2 * add_ln_partial_rows(R) * H floats.
// ---------------------------------------------------------------------------
bool add_ln_supported(int H);
int64_t add_ln_partial_rows(int64_t R);
// seed_dev (optional): device word mixed into the dropout seed (graph replays)
void add_ln_forward(const void* a, const void* x, const float* gamma, const float* beta, void* y, void* hsave,
                    float* mean, float* rstd, int64_t R, int H, float eps, float p, uint32_t seed,
                    const uint32_t* seed_dev, hipStream_t stream, bool f32 = false);
void add_ln_backward(const void* dy, const void* hsave, const float* mean, const float* rstd, const float* gamma,
                     void* dx, void* da, float* dgamma, float* dbeta, int accumulate, float* ws, int64_t R, int H,
                     float p, uint32_t seed, const uint32_t* seed_dev, hipStream_t stream, bool f32 = false);

// ---------------------------------------------------------------------------
// Linear-layer column passes over bf16 [M, N] row-major gradients (linear.hip);
// N % 8 == 0, rows 16-byte aligned; db: fp32 [N], accumulated with float atomics.
//   colsum_acc_bf16     : db[n] += sum_m dy[m, n]                   (bias gradient)
//   gelu_bwd_colsum_bf16: dpre = dy * gelu'(pre) (erf GELU, bf16 RNE) and, when db
//                         is non-null, db[n] += sum_m dpre[m, n]
// ---------------------------------------------------------------------------
void colsum_acc_bf16(const uint16_t* dy, float* db, int64_t M, int N, hipStream_t stream);
void gelu_bwd_colsum_bf16(const uint16_t* dy, const uint16_t* pre, uint16_t* dpre, float* db, int64_t M, int N,
                          hipStream_t stream);
void colsum_acc_f32(const float* dy, float* db, int64_t M, int N, hipStream_t stream);
void gelu_bwd_colsum_f32(const float* dy, const float* pre, float* dpre, float* db, int64_t M, int N,
                         hipStream_t stream);

// ---------------------------------------------------------------------------
// LSTM (lstm.hip), PyTorch gate order i, f, g, o.  Hp = H rounded up to 64.
//   lstm_rec_gemm: P[s][m][n] = sum_{k in slice s} A[m][k] B[n][k] (fp32 K-slice
//                  partials, S slices; K % (64 S) == 0, N % 64 == 0)
//   lstm_cell_fwd: G = xg [B][4H] (bf16) + hg [B][4H] (bf16, may be null)
//                  + sum_s P[s] [B][4Hp] (may be null) -> c (fp32),
//                  h (bf16 [B][H]; also into h_pad [B][Hp] when non-null), gates (fp32)
//   lstm_cell_bwd: dh = dout + dh_rec (bf16, may be null) + sum_s P[s] [B][Hp] (may be null),
//                  dc_next (fp32, may be null) -> dG (bf16 [B][4H]; also into
//                  dG_pad [B][4Hp] when non-null), dc_prev (fp32)
// ---------------------------------------------------------------------------
void lstm_rec_gemm(const uint16_t* A, int64_t lda, const uint16_t* B, int64_t ldb, float* P, int M, int N, int K,
                   int S, hipStream_t stream);
void lstm_cell_fwd(const uint16_t* xg, const uint16_t* hg, const float* P, int S, const float* c_prev, float* c, uint16_t* h,
                   uint16_t* h_pad, float* gates, int B, int H, int Hp, hipStream_t stream);
void lstm_cell_bwd(const uint16_t* dout, const uint16_t* dh_rec, const float* P, int S, const float* dc_next, const float* gates,
                   const float* c, const float* c_prev, uint16_t* dG, uint16_t* dG_pad, float* dc_prev, int B, int H,
                   int Hp, hipStream_t stream);
// fp32 variants (the reference's precision): fp32 operands, same layouts
// bf16x6 (fp32-accurate) split-K step GEMM: A fp32 [M][K] (split in registers),
// B3 = three bf16 planes [3][N][K] (plane stride bplane elements) of the fp32 B
void lstm_rec_gemm_x6(const float* A, int64_t lda, const uint16_t* B3, int64_t ldb, int64_t bplane, float* P, int M,
                      int N, int K, int S, hipStream_t stream);
void lstm_rec_gemm_f32(const float* A, int64_t lda, const float* B, int64_t ldb, float* P, int M, int N, int K, int S,
                       hipStream_t stream);
void lstm_cell_fwd_f32(const float* xg, const float* hg, const float* P, int S, const float* c_prev, float* c, float* h,
                       float* h_pad, float* gates, int B, int H, int Hp, hipStream_t stream);
void lstm_cell_bwd_f32(const float* dout, const float* dh_rec, const float* P, int S, const float* dc_next,
                       const float* gates, const float* c, const float* c_prev, float* dG, float* dG_pad, float* dc_prev,
                       int B, int H, int Hp, hipStream_t stream);

}  // namespace gk
