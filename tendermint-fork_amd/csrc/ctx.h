// ctx.h — tmed_ctx internals shared by the host-side translation units.
#pragma once
#include <hip/hip_runtime.h>

#include <mutex>
#include <unordered_map>

#include "../../include/tmed25519.h"
#include "kernels.h"

struct tmed_ctx;

namespace tmed {

struct DevBuf {
  void *p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = bytes + bytes / 4 + 256;
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

struct HostBuf {
  void *p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    size_t want = bytes + bytes / 4 + 256;
    hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
};

inline int map_err(hipError_t e) {
  if (e == hipSuccess) return TMED_OK;
  if (e == hipErrorOutOfMemory) return TMED_ENOMEM;
  return TMED_EHIP;
}

// A validator set's key material resident in HBM.
struct Keyset {
  size_t n = 0;
  uint8_t *d_pub = nullptr;   // n x 32 raw encodings (hashed into k)
  uint8_t *d_ok = nullptr;    // n: Point.SetBytes accepted the key
  int4 *d_comb = nullptr;     // n x kCombBytesPerKey: signed radix-256 comb of -A
};

int build_comb(tmed_ctx *c, const uint8_t *d_pubs, size_t n, int negate, uint8_t *d_ok, int4 *d_comb);
void free_keyset(Keyset &k);

}  // namespace tmed

struct tmed_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  float last_ms = 0.f;
  std::mutex mu;
  tmed::ge_niels *d_btab = nullptr;
  int4 *d_bcomb = nullptr;  // signed radix-256 comb of +B (shared)
  int4 *d_slab = nullptr;
  int4 *d_prep = nullptr;
  uint32_t slab_slots = 0;
  uint32_t chunk = 0;     // signatures per prep/main launch pair (0 = slab_slots); env TMED_CHUNK
  int main_waves = 2;     // register budget variant of the main kernel; env TMED_MAIN_WAVES
  tmed::DevBuf d_a, d_b, d_msg, d_off, d_out, d_c;
  tmed::HostBuf h_a, h_b, h_msg, h_off, h_out, h_c;
  std::unordered_map<uint64_t, tmed::Keyset> keysets;
  uint64_t next_keyset = 1;
};
