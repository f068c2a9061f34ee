// Shared gfx950 MFMA / LDS helpers of the hand-written GEMM-shaped kernels
// (gemm.hip, stem.hip): operand vector types, packed bf16 rounding, 16-byte
// LDS-DMA and the transposed LDS read.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gk {
namespace {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
#define GK_LDS __attribute__((address_space(3)))

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

// two fp32 -> packed bf16x2, round-to-nearest-even (one v_cvt_pk_bf16_f32)
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{lo, hi}, bf16x2_t));
}

// Exact split of eight fp32 values (x0: elements 0-3, x1: 4-7) into bf16 parts
// x = hi + mid + lo, each part the round-to-nearest-even bf16 of the residual
// left by the previous ones: the residuals are exact in fp32 (|x - hi| <=
// 2^-8 |x|, |x - hi - mid| <= 2^-16 |x|), so the three parts hold all 24
// mantissa bits.  Products of parts are exact in fp32 (8 x 8 significant bits).
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void split3x8(const f32x4& x0, const f32x4& x1, bf16x8& hi, bf16x8& mid, bf16x8& lo) {
  u32x4 h, m, l;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const float a = p < 2 ? x0[2 * p] : x1[2 * p - 4];
    const float b = p < 2 ? x0[2 * p + 1] : x1[2 * p - 3];
    const uint32_t hp = pack_bf16x2(a, b);
    const float ra = a - __uint_as_float(hp << 16), rb = b - __uint_as_float(hp & 0xffff0000u);
    const uint32_t mp = pack_bf16x2(ra, rb);
    const float sa = ra - __uint_as_float(mp << 16), sb = rb - __uint_as_float(mp & 0xffff0000u);
    h[p] = hp;
    m[p] = mp;
    l[p] = pack_bf16x2(sa, sb);
  }
  hi = __builtin_bit_cast(bf16x8, h);
  mid = __builtin_bit_cast(bf16x8, m);
  lo = __builtin_bit_cast(bf16x8, l);
}

__device__ __forceinline__ void glds16(const void* src, GK_LDS void* dst) {
  __builtin_amdgcn_global_load_lds(src, dst, 16, 0, 0);
}

// LDS image of a [rows][RB bytes] tile for transposed reads: 16-byte chunk
// c of row r is stored at chunk c ^ tr_swz(r).  A ds_read_b64_tr_b16 half-wave
// touches rows {R..R+3, R+8..R+11} x 32 bytes; the XOR spreads those 16
// (row, chunk) pairs over 16 distinct 16-byte bank slots.
template <int RB>
__device__ __forceinline__ int tr_swz(int r) {
  if (RB == 128) return 2 * (((r >> 1) & 1) | (((r >> 3) & 1) << 1));
  return 2 * ((r & 3) | (((r >> 3) & 1) << 2));
}

// gfx950 transposed LDS read (4 rows x 16 columns of 16-bit data delivered
// column-wise), as inline asm: the builtin makes the compiler's wait-count
// pass treat it as dependent on in-flight LDS-DMA (see gemm.hip tr_pair).
__device__ __forceinline__ bf16x4 ds_read_tr(const char* p) {
  bf16x4 v;
  const uint32_t a = (uint32_t)(uintptr_t)(GK_LDS char*)p;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(a));
  return v;
}

}  // namespace
}  // namespace gk
