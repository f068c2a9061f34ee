// One instantiation unit of the GEMM kernel templates (gemm_kern.h), selected
// by -DGK_GEMM_UNIT=<n>: the templates used to live in one translation unit
// that took ~7 minutes to compile; ops/build.py compiles the units in parallel.
#include "gemm_kern.h"

#ifndef GK_GEMM_UNIT
#error "compile with -DGK_GEMM_UNIT=<unit>"
#endif

namespace gk {

#if GK_GEMM_UNIT == 0
int nt_b16_row(GK_NT_UNIT_ARGS) { return nt_dispatch<false, uint16_t>(GK_NT_UNIT_PASS); }
#elif GK_GEMM_UNIT == 1
int nt_b16_gat(GK_NT_UNIT_ARGS) { return nt_dispatch<true, uint16_t>(GK_NT_UNIT_PASS); }
#elif GK_GEMM_UNIT == 2
int nt_f32_row(GK_NT_UNIT_ARGS) { return nt_dispatch<false, float>(GK_NT_UNIT_PASS); }
#elif GK_GEMM_UNIT == 3
int nt_f32_gat(GK_NT_UNIT_ARGS) { return nt_dispatch<true, float>(GK_NT_UNIT_PASS); }
#elif GK_GEMM_UNIT == 4
void tn_unit_b16(bool gather, const void* G, int64_t ldg, const void* X, int64_t ldx, float* W, int64_t ldw, int64_t M,
                 int N, int K, int cfg, int splits, const ConvGeo& geo, hipStream_t stream) {
  if (gather) tn_dispatch<true>(G, ldg, X, ldx, W, ldw, M, N, K, cfg, splits, geo, stream);
  else tn_dispatch<false>(G, ldg, X, ldx, W, ldw, M, N, K, cfg, splits, geo, stream);
}
void tn_unit_f32(bool gather, const float* G, int64_t ldg, const float* X, int64_t ldx, float* W, int64_t ldw,
                 int64_t M, int N, int K, int cfg, int splits, const ConvGeo& geo, const LazyArgs* lza,
                 hipStream_t stream) {
  if (gather) tn_f32_dispatch<true>(G, ldg, X, ldx, W, ldw, M, N, K, cfg, splits, geo, lza, stream);
  else tn_f32_dispatch<false>(G, ldg, X, ldx, W, ldw, M, N, K, cfg, splits, geo, lza, stream);
}
#elif GK_GEMM_UNIT == 5
int nt_x6_row(GK_NT_UNIT_ARGS) { return nt_dispatch<false, float, true>(GK_NT_UNIT_PASS); }
#elif GK_GEMM_UNIT == 6
int nt_x6_gat(GK_NT_UNIT_ARGS) { return nt_dispatch<true, float, true>(GK_NT_UNIT_PASS); }
#elif GK_GEMM_UNIT == 7
void tn_unit_x6(bool gather, const float* G, int64_t ldg, const float* X, int64_t ldx, float* W, int64_t ldw,
                int64_t M, int N, int K, int cfg, int splits, const ConvGeo& geo, const LazyArgs* lza,
                hipStream_t stream) {
  if (gather) tn_f32_dispatch<true, true>(G, ldg, X, ldx, W, ldw, M, N, K, cfg, splits, geo, lza, stream);
  else tn_f32_dispatch<false, true>(G, ldg, X, ldx, W, ldw, M, N, K, cfg, splits, geo, lza, stream);
}
#elif GK_GEMM_UNIT == 8
int nt_x62_row(const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc, int64_t M, int N, int K,
               int cfg, int max_blocks, const float* bias, float* stats, int64_t stats_ld, int stats_rows,
               const BnBwd& bb, const uint16_t* b3, hipStream_t stream) {
  ConvGeo g{};
  g.b3 = b3;
  return nt_x62_dispatch<false>(A, lda, B, ldb, C, ldc, M, N, K, cfg, max_blocks, bias, stats, stats_ld, stats_rows, bb,
                                g, stream);
}
#elif GK_GEMM_UNIT == 9
void tn_x62_row(const float* G, int64_t ldg, const float* X, int64_t ldx, float* W, int64_t ldw, int64_t M, int N,
                int K, int cfg, int splits, hipStream_t stream) {
  tn_x62_dispatch(G, ldg, X, ldx, W, ldw, M, N, K, cfg, splits, stream);
}
#elif GK_GEMM_UNIT == 10
int nt_x62_gat(const float* A, const float* B, float* C, int64_t M, int N, int K, int cfg, int max_blocks,
               const ConvGeo& geo, float* stats, int64_t stats_ld, int stats_rows, const BnBwd& bb,
               hipStream_t stream) {
  return nt_x62_dispatch<true>(A, geo.C, B, K, C, N, M, N, K, cfg, max_blocks, geo.bias, stats, stats_ld, stats_rows,
                               bb, geo, stream);
}
#else
#error "unknown GK_GEMM_UNIT"
#endif

}  // namespace gk
