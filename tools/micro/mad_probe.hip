// mad_probe.hip — tools only: issue cost of v_mad_i64_i32 with its carry-out in VCC vs in
// rotating SGPR pairs, and its dependent-chain latency (chains of D independent accumulators),
// at 1 and 2 waves per SIMD.  Cycles at the nominal clock, per wave-instruction per SIMD.
// Build: hipcc -O3 --offload-arch=gfx950 mad_probe.hip -o mad_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <int KIND, int D>
__device__ __forceinline__ void step(uint64_t (&x)[16], uint32_t b) {
#pragma unroll
  for (int c = 0; c < 16; c++) {
    uint64_t &v = x[c % D];
    const uint32_t lo = (uint32_t)(x[(c + 1) % D] >> 7);
    if constexpr (KIND == 0) asm volatile("v_mad_i64_i32 %0, vcc, %1, %2, %0" : "+v"(v) : "v"(lo), "v"(b) : "vcc");
    if constexpr (KIND == 1) {
      if (c % 4 == 0) asm volatile("v_mad_i64_i32 %0, s[40:41], %1, %2, %0" : "+v"(v) : "v"(lo), "v"(b) : "s40", "s41");
      if (c % 4 == 1) asm volatile("v_mad_i64_i32 %0, s[42:43], %1, %2, %0" : "+v"(v) : "v"(lo), "v"(b) : "s42", "s43");
      if (c % 4 == 2) asm volatile("v_mad_i64_i32 %0, s[44:45], %1, %2, %0" : "+v"(v) : "v"(lo), "v"(b) : "s44", "s45");
      if (c % 4 == 3) asm volatile("v_mad_i64_i32 %0, s[46:47], %1, %2, %0" : "+v"(v) : "v"(lo), "v"(b) : "s46", "s47");
    }
    if constexpr (KIND == 2) asm volatile("v_mad_i64_i32 %0, vcc, %1, %2, %0" : "+v"(v) : "v"(b), "v"(b) : "vcc");
  }
}

template <int KIND, int D>
__global__ __launch_bounds__(256) void probe(uint32_t iters, uint32_t seed, uint64_t *sink) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t b = seed * 2654435761u + t;
  uint64_t s[16];
#pragma unroll
  for (int c = 0; c < 16; c++) s[c] = (uint64_t)(c + 1) * 0x9E3779B97F4A7C15ull ^ t;
  for (uint32_t i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 8; u++) step<KIND, D>(s, b);
  }
  uint64_t acc = 0;
#pragma unroll
  for (int c = 0; c < 16; c++) acc += s[c];
  if (acc == 0x1234567890abcdefull) sink[0] = acc;
}

template <int KIND, int D>
static void one(const char *name, int cus, double ghz, uint64_t *sink) {
  const uint32_t iters = 512;
  printf("{\"probe\": \"%s\", \"chains\": %d", name, D);
  for (int wps : {1, 2}) {
    const uint32_t blocks = cus * wps;
    hipLaunchKernelGGL((probe<KIND, D>), dim3(blocks), dim3(256), 0, 0, 4, 7u, sink);
    hipEvent_t a, e;
    hipEventCreate(&a);
    hipEventCreate(&e);
    hipEventRecord(a, 0);
    hipLaunchKernelGGL((probe<KIND, D>), dim3(blocks), dim3(256), 0, 0, iters, 7u, sink);
    hipEventRecord(e, 0);
    hipEventSynchronize(e);
    float ms = 0;
    hipEventElapsedTime(&ms, a, e);
    const double instrs = (double)wps * iters * 8 * 16;
    printf(", \"cyc_per_instr_%dw\": %.3f", wps, ms * 1e-3 * ghz * 1e9 / instrs);
  }
  printf("}\n");
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  const double ghz = p.clockRate / 1e6;
  uint64_t *sink;
  hipMalloc(&sink, 8);
  one<0, 16>("mad_vcc", cus, ghz, sink);
  one<1, 16>("mad_sgpr_rot4", cus, ghz, sink);
  one<0, 1>("mad_vcc_dep", cus, ghz, sink);
  one<2, 1>("mad_acc_dep", cus, ghz, sink);
  one<2, 2>("mad_acc_dep", cus, ghz, sink);
  one<2, 3>("mad_acc_dep", cus, ghz, sink);
  one<2, 4>("mad_acc_dep", cus, ghz, sink);
  one<2, 8>("mad_acc_dep", cus, ghz, sink);
  one<2, 16>("mad_acc_dep", cus, ghz, sink);
  return 0;
}
