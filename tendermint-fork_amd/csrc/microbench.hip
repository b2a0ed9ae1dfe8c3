// microbench.hip — integer-VALU peak probes (roofline denominator and cost model).
//
// the verify kernel is bound by 32x32->64 integer multiply-adds;
// "peak_mad_rate = measured v_mad throughput from a gfx950 microbenchmark".
// Each lane runs 16 independent chains of ONE instruction (inline asm, so the
// compiler cannot fold or re-select it) for `iters` x 8 steps.  The same probe,
// run for the other instructions the field arithmetic emits, gives the per-
// instruction issue cost used in DESIGN.md's cost model.
#include <hip/hip_runtime.h>

#include "../../include/tmed25519.h"

namespace {

constexpr int kChains = 16;
constexpr int kUnroll = 8;

template <int KIND>
__device__ __forceinline__ void step(uint64_t &x, uint32_t b, uint64_t m) {
  uint32_t lo = (uint32_t)x;
  if constexpr (KIND == 0) asm volatile("v_mad_i64_i32 %0, vcc, %1, %2, %0" : "+v"(x) : "v"(lo), "v"(b) : "vcc");
  if constexpr (KIND == 1) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(x) : "v"(lo), "v"(b) : "vcc");
  if constexpr (KIND == 2) { asm volatile("v_add_u32 %0, %0, %1" : "+v"(lo) : "v"(b)); x = lo; }
  if constexpr (KIND == 3) { asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(lo) : "v"(b)); x = lo; }
  if constexpr (KIND == 4) asm volatile("v_ashrrev_i64 %0, 3, %0" : "+v"(x));
  if constexpr (KIND == 5) asm volatile("v_lshl_add_u64 %0, %0, 2, %0" : "+v"(x));
  if constexpr (KIND == 6) { asm volatile("v_lshl_add_u32 %0, %0, 4, %1" : "+v"(lo) : "v"(b)); x = lo; }
  if constexpr (KIND == 7) asm volatile("v_add_co_u32 %0, vcc, %0, %1\n\tv_addc_co_u32 %2, vcc, 0, %2, vcc"
                                        : "+v"(lo), "+v"(b), "+v"(lo) :: "vcc");
  // the carry chain's alternatives (a 64-bit shift against two 32-bit ops, masks, selects)
  if constexpr (KIND == 8) asm volatile("v_lshrrev_b64 %0, 3, %0" : "+v"(x));
  if constexpr (KIND == 9) { asm volatile("v_alignbit_b32 %0, %1, %0, 26" : "+v"(lo) : "v"(b)); x = lo; }
  if constexpr (KIND == 10) { asm volatile("v_and_b32 %0, %1, %0" : "+v"(lo) : "v"(b)); x = lo; }
  if constexpr (KIND == 11) { asm volatile("v_bfe_i32 %0, %0, 0, 26" : "+v"(lo)); x = lo; }
  if constexpr (KIND == 12) { asm volatile("v_and_or_b32 %0, %0, %1, %1" : "+v"(lo) : "v"(b)); x = lo; }
  if constexpr (KIND == 13) { asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(lo) : "v"(b)); x = lo; }
  if constexpr (KIND == 14) { asm volatile("v_ashrrev_i32 %0, 26, %0" : "+v"(lo)); x = lo; }
  // the select as the field code emits it: a lane mask in an SGPR pair written once by v_cmp
  if constexpr (KIND == 15) { asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(lo) : "v"(b), "s"(m)); x = lo; }
  // compare + select pairs (counted as 2), the mask in vcc / in an SGPR pair
  if constexpr (KIND == 16)
  {
    asm volatile("v_cmp_gt_u32 vcc, %0, %1\n\tv_cndmask_b32 %0, %0, %1, vcc" : "+v"(lo) : "v"(b) : "vcc");
    x = lo;
  }
  if constexpr (KIND == 17) {
    uint64_t k;
    asm volatile("v_cmp_gt_u32_e64 %1, %0, %2\n\tv_cndmask_b32_e64 %0, %0, %2, %1" : "+v"(lo), "=s"(k) : "v"(b));
    x = lo;
  }
  (void)m;
}

template <int KIND>
__global__ __launch_bounds__(256) void valu_probe(uint32_t iters, uint32_t seed, uint64_t *sink) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t b = seed * 2654435761u + t;
  uint64_t s[kChains];
  uint64_t m;  // a lane mask (half the lanes) for the select probes
  asm volatile("v_cmp_gt_u32_e64 %0, %1, %2" : "=s"(m) : "v"(t & 63u), "v"(32u));
#pragma unroll
  for (int c = 0; c < kChains; c++) s[c] = (uint64_t)(c + 1) * 0x9E3779B97F4A7C15ull ^ t;
  for (uint32_t i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < kUnroll; u++) {
#pragma unroll
      for (int c = 0; c < kChains; c++) step<KIND>(s[c], b, m);
    }
  }
  uint64_t acc = 0;
#pragma unroll
  for (int c = 0; c < kChains; c++) acc += s[c];
  if (acc == 0x1234567890abcdefull) sink[0] = acc;
}

template <int KIND>
void launch_probe(uint32_t blocks, uint32_t it, uint64_t *sink) {
  hipLaunchKernelGGL(valu_probe<KIND>, dim3(blocks), dim3(256), 0, 0, it, 7u, sink);
}

}  // namespace

// kind: 0 v_mad_i64_i32, 1 v_mad_u64_u32, 2 v_add_u32, 3 v_mul_lo_u32, 4 v_ashrrev_i64,
//       5 v_lshl_add_u64, 6 v_lshl_add_u32, 7 v_add_co_u32+v_addc_co_u32 (counted as 2),
//       8 v_lshrrev_b64, 9 v_alignbit_b32, 10 v_and_b32, 11 v_bfe_i32, 12 v_and_or_b32,
//       13 v_cndmask_b32 (vcc, never written), 14 v_ashrrev_i32, 15 v_cndmask_b32_e64 (SGPR mask),
//       16 v_cmp_gt_u32 + v_cndmask_b32 through vcc, 17 the same pair through an SGPR pair (both counted as 2)
extern "C" int tmed_valu_peak(tmed_ctx *ctx, int kind, double *gops) {
  (void)ctx;
  if (!gops || kind < 0 || kind > 17) return TMED_EINVAL;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return TMED_EHIP;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return TMED_EHIP;
  uint64_t *sink = nullptr;
  if (hipMalloc(&sink, 8) != hipSuccess) return TMED_ENOMEM;
  const uint32_t blocks = prop.multiProcessorCount * 8;  // 8 x 256 lanes per CU (8 waves/SIMD)
  const uint32_t iters = 2048;
  auto launch = [&](uint32_t it) {
    switch (kind) {
      case 0: launch_probe<0>(blocks, it, sink); break;
      case 1: launch_probe<1>(blocks, it, sink); break;
      case 2: launch_probe<2>(blocks, it, sink); break;
      case 3: launch_probe<3>(blocks, it, sink); break;
      case 4: launch_probe<4>(blocks, it, sink); break;
      case 5: launch_probe<5>(blocks, it, sink); break;
      case 6: launch_probe<6>(blocks, it, sink); break;
      case 7: launch_probe<7>(blocks, it, sink); break;
      case 8: launch_probe<8>(blocks, it, sink); break;
      case 9: launch_probe<9>(blocks, it, sink); break;
      case 10: launch_probe<10>(blocks, it, sink); break;
      case 11: launch_probe<11>(blocks, it, sink); break;
      case 12: launch_probe<12>(blocks, it, sink); break;
      case 13: launch_probe<13>(blocks, it, sink); break;
      case 14: launch_probe<14>(blocks, it, sink); break;
      case 15: launch_probe<15>(blocks, it, sink); break;
      case 16: launch_probe<16>(blocks, it, sink); break;
      default: launch_probe<17>(blocks, it, sink); break;
    }
  };
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  launch(64);  // warm
  (void)hipEventRecord(e0, 0);
  launch(iters);
  (void)hipEventRecord(e1, 0);
  hipError_t e = hipEventSynchronize(e1);
  float ms = 0.f;
  if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipFree(sink);
  if (e != hipSuccess) return TMED_EHIP;
  const double ops = (double)blocks * 256.0 * iters * kUnroll * kChains * (kind == 7 || kind >= 16 ? 2 : 1);
  *gops = ops / (ms * 1e-3) / 1e9;
  return TMED_OK;
}
