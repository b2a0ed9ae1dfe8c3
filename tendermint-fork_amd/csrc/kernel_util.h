// kernel_util.h — small device helpers shared by the kernel translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"

namespace tmed {

// nwords16 x 16 B of a 16-B aligned row into 32-bit words.
__device__ __forceinline__ void load_row_words(uint32_t *w, const uint8_t *p, int nwords16) {
  const uint4 *q = reinterpret_cast<const uint4 *>(p);
#pragma unroll
  for (int i = 0; i < 4; i++) {
    if (i < nwords16) {
      const uint4 v = q[i];
      w[4 * i + 0] = v.x; w[4 * i + 1] = v.y; w[4 * i + 2] = v.z; w[4 * i + 3] = v.w;
    }
  }
}

// Message i of a batch: packed (off[i]..off[i+1]) or fixed kVoteSlot slots (off = lengths).
struct MsgSrc {
  const uint8_t *msgs;
  const uint32_t *off;  // packed mode (len == nullptr): n + 1 offsets; slot mode: lengths
  bool slots;
  __device__ __forceinline__ void get(uint32_t i, const uint8_t *&p, uint32_t &len) const {
    if (slots) {
      p = msgs + (size_t)i * kVoteSlot;
      len = off[i];
    } else {
      const uint32_t o0 = off[i], o1 = off[i + 1];
      p = msgs + o0;
      len = o1 - o0;
    }
  }
};

}  // namespace tmed
