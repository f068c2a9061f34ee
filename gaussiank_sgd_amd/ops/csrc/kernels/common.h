// Shared device helpers for the gfx950 (CDNA4, wave64) kernel library.
//
// Everything here assumes a 64-lane wavefront: ballots are 64-bit, lane ids
// are threadIdx.x & 63 and block sizes are multiples of 64.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gk {

constexpr int kWave = 64;
constexpr int kBlock = 256;            // 4 waves per workgroup
constexpr int kWavesPerBlock = kBlock / kWave;

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }

__device__ __forceinline__ uint64_t lanemask_lt() {
  const int l = lane_id();
  return l == 0 ? 0ull : ((~0ull) >> (64 - l));
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    T o = __shfl_xor(v, off, 64);
    v = o > v ? o : v;
  }
  return v;
}

// Block-wide sum of a double, result valid in every thread.  `scratch` must
// hold kWavesPerBlock doubles.
__device__ __forceinline__ double block_sum(double v, double* scratch) {
  v = wave_sum(v);
  __syncthreads();
  if (lane_id() == 0) scratch[wave_id()] = v;
  __syncthreads();
  double r = 0.0;
#pragma unroll
  for (int w = 0; w < kWavesPerBlock; ++w) r += scratch[w];
  return r;
}

__device__ __forceinline__ float block_max(float v, float* scratch) {
  v = wave_max(v);
  __syncthreads();
  if (lane_id() == 0) scratch[wave_id()] = v;
  __syncthreads();
  float r = scratch[0];
#pragma unroll
  for (int w = 1; w < kWavesPerBlock; ++w) r = fmaxf(r, scratch[w]);
  return r;
}

// Exclusive prefix of a small non-negative per-lane count (< 2^NBITS) across
// the 64 lanes of a wave using NBITS ballots (no shuffles, no LDS).
template <int NBITS>
__device__ __forceinline__ uint32_t wave_excl_prefix_small(uint32_t c, uint32_t* total) {
  const uint64_t lt = lanemask_lt();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int b = 0; b < NBITS; ++b) {
    const uint64_t m = __ballot((c >> b) & 1u);
    pre += (uint32_t)__popcll(m & lt) << b;
    tot += (uint32_t)__popcll(m) << b;
  }
  *total = tot;
  return pre;
}

// |x| as an order-preserving uint32 key (sign bit cleared).
__device__ __forceinline__ uint32_t abs_key(float x) { return __float_as_uint(x) & 0x7fffffffu; }

// 32-bit integer mixer (murmur3 fmix32 over a Weyl-sequenced index).
__device__ __forceinline__ uint32_t hash_u32(uint32_t i, uint32_t seed) {
  uint32_t h = i * 0x9E3779B1u + seed * 0x85EBCA77u + 0x27d4eb2fu;
  h ^= h >> 16; h *= 0x85ebca6bu;
  h ^= h >> 13; h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}

__host__ __device__ __forceinline__ int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

}  // namespace gk
