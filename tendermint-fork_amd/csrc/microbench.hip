// microbench.hip — integer-VALU peak probe used as the roofline denominator.
//
// the verify kernel is bound by 32x32->64 integer multiply-adds;
// "peak_mad_rate = measured v_mad_u64_u32 throughput from a gfx950
// microbenchmark".  Each lane runs 16 independent accumulation chains (enough
// ILP to hide the dependent latency) for `iters` iterations; the result is
// folded into one store so nothing is dead-code-eliminated.
#include <hip/hip_runtime.h>

#include "../../include/tmed25519.h"

namespace {

constexpr int kChains = 16;
constexpr int kUnroll = 8;

template <int KIND>
__global__ __launch_bounds__(256) void valu_probe(uint32_t iters, uint32_t seed, uint64_t *sink) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t a = seed ^ t, b = seed * 2654435761u + t;
  int64_t si[kChains];
  uint64_t su[kChains];
  uint32_t s32[kChains];
#pragma unroll
  for (int c = 0; c < kChains; c++) { si[c] = c + t; su[c] = c ^ t; s32[c] = c * t; }
  for (uint32_t i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < kUnroll; u++) {
#pragma unroll
      for (int c = 0; c < kChains; c++) {
        if (KIND == 0) si[c] = (int64_t)(int32_t)si[c] * (int64_t)(int32_t)b + si[c];
        if (KIND == 1) su[c] = (uint64_t)(uint32_t)su[c] * (uint64_t)b + su[c];
        if (KIND == 2) s32[c] = s32[c] + s32[c ^ 1];
        if (KIND == 3) s32[c] = s32[c] * s32[c ^ 1];
      }
    }
    asm volatile("" : "+v"(b));  // keep the operands live & opaque
  }
  uint64_t acc = 0;
#pragma unroll
  for (int c = 0; c < kChains; c++) acc += (uint64_t)si[c] + su[c] + s32[c];
  if (acc == 0x1234567890abcdefull) sink[0] = acc;
}

}  // namespace

extern "C" int tmed_valu_peak(tmed_ctx *ctx, int kind, double *gops) {
  (void)ctx;
  if (!gops || kind < 0 || kind > 3) return TMED_EINVAL;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return TMED_EHIP;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return TMED_EHIP;
  uint64_t *sink = nullptr;
  if (hipMalloc(&sink, 8) != hipSuccess) return TMED_ENOMEM;
  const uint32_t blocks = prop.multiProcessorCount * 8;  // 8 waves of 256 lanes per CU... 2048 threads/CU
  const uint32_t iters = 4096;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto launch = [&](uint32_t it) {
    switch (kind) {
      case 0: hipLaunchKernelGGL(valu_probe<0>, dim3(blocks), dim3(256), 0, 0, it, 7u, sink); break;
      case 1: hipLaunchKernelGGL(valu_probe<1>, dim3(blocks), dim3(256), 0, 0, it, 7u, sink); break;
      case 2: hipLaunchKernelGGL(valu_probe<2>, dim3(blocks), dim3(256), 0, 0, it, 7u, sink); break;
      default: hipLaunchKernelGGL(valu_probe<3>, dim3(blocks), dim3(256), 0, 0, it, 7u, sink); break;
    }
  };
  launch(64);  // warm
  hipEventRecord(e0, 0);
  launch(iters);
  hipEventRecord(e1, 0);
  hipError_t e = hipEventSynchronize(e1);
  float ms = 0.f;
  if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  hipFree(sink);
  if (e != hipSuccess) return TMED_EHIP;
  const double ops = (double)blocks * 256.0 * iters * kUnroll * kChains;
  *gops = ops / (ms * 1e-3) / 1e9;
  return TMED_OK;
}
