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
