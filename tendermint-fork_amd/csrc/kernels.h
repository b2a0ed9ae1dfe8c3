// kernels.h — launch interface between the C-ABI layer and the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "ge25519.h"

namespace tmed {

constexpr uint32_t kThreadsPerBlock = 256;
// Variable-base table slab: lane slots (grid-stride loop bounds the grid to
// slab_slots / kThreadsPerBlock blocks).  9 entries x 160 B per slot.
constexpr uint32_t kSlabSlotBytes = 9 * 160;

hipError_t launch_verify(const uint8_t *pub, const uint8_t *sig, const uint8_t *msgs, const uint32_t *off,
                         uint32_t n, uint8_t *out, int4 *slab, uint32_t slab_stride, const ge_niels *btab,
                         hipStream_t stream);

hipError_t launch_sign(const uint8_t *seeds, const uint8_t *msgs, const uint32_t *off, uint32_t n, uint8_t *sig_out,
                       uint8_t *pub_out, int4 *slab, uint32_t slab_stride, const ge_niels *btab,
                       hipStream_t stream);

void host_build_btab(ge_niels out[9]);

}  // namespace tmed
