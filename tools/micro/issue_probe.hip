// issue_probe.hip — tools only: cycles per wave-instruction of the VALU instructions the field
// arithmetic emits, at 1, 2 and 8 waves per SIMD (the main kernel runs at 2).  Each lane runs
// 16 independent chains of ONE instruction (inline asm), so the figure is issue cost, not latency.
// Build: hipcc -O3 --offload-arch=gfx950 issue_probe.hip -o issue_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int kChains = 16;
constexpr int kUnroll = 8;

template <int KIND>
__device__ __forceinline__ void step(uint64_t &x, uint32_t &y, uint32_t b) {
  uint32_t lo = (uint32_t)x;
  if constexpr (KIND == 0) asm volatile("v_mad_i64_i32 %0, vcc, %1, %2, %0" : "+v"(x) : "v"(lo), "v"(b) : "vcc");
  if constexpr (KIND == 1) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(x) : "v"(lo), "v"(b) : "vcc");
  if constexpr (KIND == 2) asm volatile("v_add_u32 %0, %0, %1" : "+v"(y) : "v"(b));
  if constexpr (KIND == 3) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(y) : "v"(b));
  if constexpr (KIND == 4) asm volatile("v_ashrrev_i64 %0, 3, %0" : "+v"(x));
  if constexpr (KIND == 5) asm volatile("v_lshl_add_u64 %0, %0, 0, %0" : "+v"(x));
  if constexpr (KIND == 6) asm volatile("v_lshl_add_u32 %0, %0, 4, %1" : "+v"(y) : "v"(b));
  if constexpr (KIND == 7) asm volatile("v_and_b32 %0, %0, %1" : "+v"(y) : "v"(b));
  if constexpr (KIND == 8) asm volatile("v_alignbit_b32 %0, %0, %1, 26" : "+v"(y) : "v"(b));
  if constexpr (KIND == 9) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(y) : "v"(b));
  if constexpr (KIND == 10) asm volatile("v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "=v"(y) : "v"(b));
  if constexpr (KIND == 11) asm volatile("v_lshlrev_b32 %0, 1, %0" : "+v"(y));
  if constexpr (KIND == 12) asm volatile("v_mul_i32_i24 %0, %0, %1" : "+v"(y) : "v"(b));
  if constexpr (KIND == 13) asm volatile("v_bfe_i32 %0, %0, 0, 26" : "+v"(y));
  if constexpr (KIND == 14) asm volatile("v_sub_u32 %0, %1, %0" : "+v"(y) : "v"(b));
  if constexpr (KIND == 15) asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(y) : "v"(b));
}

template <int KIND>
__global__ __launch_bounds__(256) void probe(uint32_t iters, uint32_t seed, uint64_t *sink) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t b = seed * 2654435761u + t;
  uint64_t s[kChains];
  uint32_t y[kChains];
#pragma unroll
  for (int c = 0; c < kChains; c++) { s[c] = (uint64_t)(c + 1) * 0x9E3779B97F4A7C15ull ^ t; y[c] = (uint32_t)s[c]; }
  for (uint32_t i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < kUnroll; u++) {
#pragma unroll
      for (int c = 0; c < kChains; c++) step<KIND>(s[c], y[c], b);
    }
  }
  uint64_t acc = 0;
#pragma unroll
  for (int c = 0; c < kChains; c++) acc += s[c] + y[c];
  if (acc == 0x1234567890abcdefull) sink[0] = acc;
}

template <int KIND>
static float run(uint32_t blocks, uint32_t iters, uint64_t *sink) {
  hipLaunchKernelGGL(probe<KIND>, dim3(blocks), dim3(256), 0, 0, 4, 7u, sink);
  hipEvent_t a, e;
  hipEventCreate(&a);
  hipEventCreate(&e);
  hipEventRecord(a, 0);
  hipLaunchKernelGGL(probe<KIND>, dim3(blocks), dim3(256), 0, 0, iters, 7u, sink);
  hipEventRecord(e, 0);
  hipEventSynchronize(e);
  float ms = 0;
  hipEventElapsedTime(&ms, a, e);
  return ms;
}

static const char *kNames[] = {"v_mad_i64_i32", "v_mad_u64_u32", "v_add_u32", "v_mul_lo_u32", "v_ashrrev_i64",
                               "v_lshl_add_u64", "v_lshl_add_u32", "v_and_b32", "v_alignbit_b32", "v_add3_u32",
                               "v_mov_b32_dpp", "v_lshlrev_b32", "v_mul_i32_i24", "v_bfe_i32", "v_sub_u32",
                               "v_mad_u32_u24"};

template <int KIND>
static void one(int cus, double ghz, uint64_t *sink) {
  const uint32_t iters = 512;
  printf("{\"instr\": \"%s\"", kNames[KIND]);
  for (int wps : {1, 2, 8}) {
    const uint32_t blocks = cus * wps;  // 256-thread blocks = one wave per SIMD each
    const float ms = run<KIND>(blocks, iters, sink);
    const double wave_instrs_per_simd = (double)wps * iters * kUnroll * kChains;
    const double cycles = ms * 1e-3 * ghz * 1e9;
    printf(", \"cyc_per_instr_%dw\": %.3f", wps, cycles / wave_instrs_per_simd);
  }
  printf("}\n");
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  const double ghz = p.clockRate / 1e6;  // nominal max clock (kHz -> GHz): cycles are at this clock
  uint64_t *sink;
  hipMalloc(&sink, 8);
  printf("{\"cus\": %d, \"clock_ghz_nominal\": %.3f}\n", cus, ghz);
  one<0>(cus, ghz, sink); one<1>(cus, ghz, sink); one<2>(cus, ghz, sink); one<3>(cus, ghz, sink);
  one<4>(cus, ghz, sink); one<5>(cus, ghz, sink); one<6>(cus, ghz, sink); one<7>(cus, ghz, sink);
  one<8>(cus, ghz, sink); one<9>(cus, ghz, sink); one<10>(cus, ghz, sink); one<11>(cus, ghz, sink);
  one<12>(cus, ghz, sink); one<13>(cus, ghz, sink); one<14>(cus, ghz, sink); one<15>(cus, ghz, sink);
  return 0;
}
