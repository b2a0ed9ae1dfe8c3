// fe_micro.hip — microbenchmarks of the field / point layer (tools only, not the product):
// instruction counts per op from the ISA and device time per op, for A/B of arithmetic variants.
#include <hip/hip_runtime.h>
#include "../../tendermint-fork_amd/csrc/ge25519.h"

using namespace tmed;

__device__ __forceinline__ void load_fe(fe &f, const int32_t *p, uint32_t i, uint32_t n) {
#pragma unroll
  for (int k = 0; k < 10; k++) f.v[k] = p[k * n + i];
}
__device__ __forceinline__ void store_fe(int32_t *p, const fe &f, uint32_t i, uint32_t n) {
#pragma unroll
  for (int k = 0; k < 10; k++) p[k * n + i] = f.v[k];
}

extern "C" __global__ __launch_bounds__(256, 2) void k_sq(int32_t *io, uint32_t n, int iters) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  fe x;
  load_fe(x, io, i, n);
#pragma unroll 1
  for (int t = 0; t < iters; t++) fe_sq(x, x);
  store_fe(io, x, i, n);
}

extern "C" __global__ __launch_bounds__(256, 2) void k_mul(int32_t *io, uint32_t n, int iters) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  fe x, y;
  load_fe(x, io, i, n);
  load_fe(y, io + 10 * n, i, n);
#pragma unroll 1
  for (int t = 0; t < iters; t++) fe_mul(x, x, y);
  store_fe(io, x, i, n);
}

extern "C" __global__ __launch_bounds__(256, 2) void k_dbl(int32_t *io, uint32_t n, int iters) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  ge_p2 q;
  load_fe(q.X, io, i, n);
  load_fe(q.Y, io + 10 * n, i, n);
  load_fe(q.Z, io + 20 * n, i, n);
  ge_p1p1 t;
#pragma unroll 1
  for (int k = 0; k < iters; k++) {
    ge_p2_dbl(t, q);
    ge_p1p1_to_p2(q, t);
  }
  store_fe(io, q.X, i, n);
  store_fe(io + 10 * n, q.Y, i, n);
  store_fe(io + 20 * n, q.Z, i, n);
}

// Two independent squaring chains per lane: if the time per squaring drops against k_sq, the
// single chain is dependency-latency bound; if not, it is issue bound.
extern "C" __global__ __launch_bounds__(256, 2) void k_sq2(int32_t *io, uint32_t n, int iters) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  fe x, y;
  load_fe(x, io, i, n);
  load_fe(y, io + 10 * n, i, n);
#pragma unroll 1
  for (int t = 0; t < iters; t++) {
    fe_sq(x, x);
    fe_sq(y, y);
  }
  store_fe(io, x, i, n);
  store_fe(io + 10 * n, y, i, n);
}

extern "C" __global__ __launch_bounds__(256, 2) void k_mul2(int32_t *io, uint32_t n, int iters) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  fe x, y, z;
  load_fe(x, io, i, n);
  load_fe(y, io + 10 * n, i, n);
  load_fe(z, io + 20 * n, i, n);
#pragma unroll 1
  for (int t = 0; t < iters; t++) {
    fe_mul(x, x, y);
    fe_mul(z, z, y);
  }
  store_fe(io, x, i, n);
  store_fe(io + 20 * n, z, i, n);
}

#ifdef FE_MICRO_MAIN
#include <stdio.h>
#include <stdlib.h>
// Time per op at full occupancy (2 waves/SIMD x 256 CUs), one lane per element.
int main() {
  const uint32_t n = 256 * 1024 * 2;  // 2 waves/SIMD on 256 CUs
  const int iters = 2000;
  int32_t *d;
  hipMalloc(&d, (size_t)n * 30 * 4);
  int32_t *h = (int32_t *)malloc((size_t)n * 30 * 4);
  for (size_t k = 0; k < (size_t)n * 30; k++) h[k] = (int32_t)((k * 2654435761u) & 0x1ffffff) - (1 << 24);
  hipMemcpy(d, h, (size_t)n * 30 * 4, hipMemcpyHostToDevice);
  struct { const char *name; void (*k)(int32_t *, uint32_t, int); double ops; } ks[] = {
      {"sq", k_sq, 1}, {"sq2", k_sq2, 2}, {"mul", k_mul, 1}, {"mul2", k_mul2, 2}, {"dbl", k_dbl, 1}};
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int wv = 1; wv <= 4; wv++)  // waves per SIMD resident (the kernels need few VGPRs)
  for (auto &k : ks) {
    const uint32_t nw = 65536u * wv;  // wv waves/SIMD: 256 CUs x 4 SIMDs x 64 lanes x wv
    if (k.k == k_dbl) continue;
    hipLaunchKernelGGL(k.k, dim3(nw / 256), dim3(256), 0, 0, d, nw, 10);
    hipEventRecord(a, 0);
    hipLaunchKernelGGL(k.k, dim3(nw / 256), dim3(256), 0, 0, d, nw, iters);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"lane_Gop_s\": %.2f}\n", k.name, wv, ms,
           (double)nw * iters * k.ops / (ms * 1e-3) / 1e9);
  }
  for (auto &k : ks) {
    hipLaunchKernelGGL(k.k, dim3(n / 256), dim3(256), 0, 0, d, n, 10);
    hipEventRecord(a, 0);
    hipLaunchKernelGGL(k.k, dim3(n / 256), dim3(256), 0, 0, d, n, iters);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double per = (double)ms * 1e6 / (iters * k.ops);  // ns per op per wave-slot round
    printf("{\"op\": \"%s\", \"ms\": %.3f, \"ns_per_op_all_lanes\": %.4f, \"Gop_s\": %.2f}\n", k.name, ms, per,
           (double)n * iters * k.ops / (ms * 1e-3) / 1e9);
  }
  // Lone wave (one 64-lane block): the latency regime of the C1 kernels' serial chains.
  for (auto &k : ks) {
    const int it1 = 2550;
    hipLaunchKernelGGL(k.k, dim3(1), dim3(64), 0, 0, d, 64, 10);
    hipEventRecord(a, 0);
    hipLaunchKernelGGL(k.k, dim3(1), dim3(64), 0, 0, d, 64, it1);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("{\"op\": \"%s\", \"lone_wave\": true, \"ns_per_op_per_chain\": %.2f}\n", k.name,
           (double)ms * 1e6 / it1 / k.ops);
  }
  return 0;
}
#endif
