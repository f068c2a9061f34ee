// Standalone timing probe of the Winograd kernels (ops/csrc/kernels/winograd.hip)
// on the ResNet-50 bs512 3x3 stride-1 shapes, for A/B builds with -D flags:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I gaussiank_sgd_amd/ops/csrc/kernels \
//         [-DGK_WINO_PROBE_...] bench/wino_probe.hip -o /tmp/wino_probe
// prints one JSON line per (op, shape): {"op", "C", "H", "us", "tflops_eff"}
// (tflops_eff = direct-convolution FLOPs / time: comparable with the
// implicit-GEMM kernels).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#include "winograd.hip"

// the split-K reduce lives in gemm.hip (not linked into this probe; splits are never requested here)
namespace gk {
int splitk_reduce(const float*, int, int64_t, int, float*, int64_t, const float*, float*, int, const BnBwdArgs*,
                  hipStream_t) {
  return -1;
}
}  // namespace gk

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void fill_kernel(float* p, int64_t n, uint32_t seed) {
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    p[i] = ((h & 0xffff) / 65536.0f - 0.5f);
  }
}

static float* dalloc(int64_t n, uint32_t seed) {
  float* p;
  CK(hipMalloc(&p, n * 4));
  hipLaunchKernelGGL(fill_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, p, n, seed);
  return p;
}

int main(int argc, char** argv) {
  const int N = argc > 1 ? atoi(argv[1]) : 512;
  const int iters = argc > 2 ? atoi(argv[2]) : 20;
  const char* tag = argc > 3 ? argv[3] : "base";
  const int only_c = argc > 4 ? atoi(argv[4]) : 0;     // run one channel count only (0: all)
  const int only_op = argc > 5 ? atoi(argv[5]) : -1;   // 0 fwd, 1 fwd_stats, 2 wgrad (-1: all)
  struct S { int C, H; } shapes[] = {{64, 56}, {128, 28}, {256, 14}, {512, 7}};
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (auto sh : shapes) {
    if (only_c && sh.C != only_c) continue;
    const int C = sh.C, K = sh.C, H = sh.H, W = sh.H;
    const int64_t nx = (int64_t)N * H * W * C;
    float* x = dalloc(nx, 1);
    float* y = dalloc((int64_t)N * H * W * K, 2);
    float* w = dalloc((int64_t)K * 9 * C, 3);
    float* u = dalloc((int64_t)16 * K * C, 4);
    float* out = dalloc((int64_t)K * 9 * C, 5);
    float* st = dalloc((int64_t)2 * 1280 * K, 6);
    const int splits = gk::wino_wgrad_splits(N, H, W, C, K, 0);
    float* part = dalloc((int64_t)splits * 16 * K * C, 7);
    const double flops = 2.0 * N * H * W * (double)C * K * 9;
    for (int op = 0; op < 3; ++op) {
      if (only_op >= 0 && op != only_op) continue;
      auto run = [&]() {
        if (op == 0) gk::wino_conv(x, u, y, N, H, W, C, K, 0, nullptr, 0, nullptr, 0);
        else if (op == 1) gk::wino_conv(x, u, y, N, H, W, C, K, 0, st, 1280, nullptr, 0);
        else gk::wino_wgrad(x, y, part, out, N, H, W, C, K, 0, 0);
      };
      run();
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(a));
      for (int i = 0; i < iters; ++i) run();
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, a, b));
      const double us = 1e3 * ms / iters;
      printf("{\"variant\": \"%s\", \"op\": \"%s\", \"C\": %d, \"H\": %d, \"us\": %.1f, \"tflops_eff\": %.1f}\n", tag,
             op == 0 ? "fwd" : op == 1 ? "fwd_stats" : "wgrad", C, H, us, flops / us * 1e-6);
      fflush(stdout);
    }
    CK(hipFree(x)); CK(hipFree(y)); CK(hipFree(w)); CK(hipFree(u)); CK(hipFree(out)); CK(hipFree(st)); CK(hipFree(part));
  }
  return 0;
}
