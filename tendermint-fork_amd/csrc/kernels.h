// kernels.h — launch interface between the C-ABI layer and the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "ge25519.h"

namespace tmed {

// Optional per-launch HIP-event timing of the verify pipeline (diagnostics / bench roofline):
// events are recorded on the launch stream before prep, between prep and main, after main.
struct KernelTimer {
  hipEvent_t ev[96];
  int n = 0;
  void mark(hipStream_t s) {
    if (n < 96) (void)hipEventRecord(ev[n++], s);
  }
};

constexpr uint32_t kThreadsPerBlock = 256;
// Variable-base table slab: lane slots (grid-stride loop bounds the grid to
// slab_slots / kThreadsPerBlock blocks).  9 entries x 160 B per slot.
constexpr uint32_t kSlabSlotBytes = 9 * 160;

hipError_t launch_verify(const uint8_t *pub, const uint8_t *sig, const uint8_t *msgs, const uint32_t *off,
                         uint32_t n, uint8_t *out, int4 *slab, uint32_t slab_stride, const ge_niels *btab,
                         int4 *prep, hipStream_t stream, uint32_t chunk = 0, int main_waves = 2,
                         bool msg_slots = false, KernelTimer *timer = nullptr);

hipError_t launch_sign(const uint8_t *seeds, const uint8_t *msgs, const uint32_t *off, uint32_t n, uint8_t *sig_out,
                       uint8_t *pub_out, int4 *slab, uint32_t slab_stride, const ge_niels *btab,
                       hipStream_t stream);

// Shared fixed-base table j*B, j = 0..128 (niels), staged in LDS by the kernels.
constexpr int kBTabSize = 129;
// prep hand-off bytes per signature slot (k, s, A.x, A.y, ok)
constexpr uint32_t kPrepSlotBytes = 160;
void host_build_btab(ge_niels out[129]);

// ---- fixed-base combs (key cache) -------------------------------
// Signed radix-256 comb of a point P: entry [w][j] = j * 256^w * P (niels, affine),
// w = 0..31, j = 0..128 (j = 0 is the identity), 128 B per entry (30 limbs + pad).
// [k]P = sum_w comb[w][d_w] with d_w = byte_w(k + 0x80...80) - 128 in [-128, 127]:
// 32 mixed additions and no doublings.
constexpr int kCombWindows = 32;
constexpr int kCombEntries = 129;
constexpr int kCombEntryInt4 = 8;  // 128 B
constexpr size_t kCombBytesPerKey = (size_t)kCombWindows * kCombEntries * kCombEntryInt4 * 16;

// bases[key][w] = 256^w * (negate ? -A : A) as p3 (40 limbs); ok[key] = decode accepted.
hipError_t launch_comb_bases(const uint8_t *pubs, uint32_t n, int negate, uint8_t *ok, int32_t *bases,
                             hipStream_t stream);
// comb[key] from bases[key] (n * 32 workgroups of 128 lanes).
hipError_t launch_comb_fill(const int32_t *bases, uint32_t n, int4 *comb, hipStream_t stream);
// Key-cached verification: key index per signature into a keyset.
hipError_t launch_verify_keyset(const uint32_t *val_idx, const uint8_t *key_pub, const uint8_t *key_ok,
                                const int4 *acomb, const int4 *bcomb, const uint8_t *sig, const uint8_t *msgs,
                                const uint32_t *off, uint32_t n, uint8_t *out, int4 *prep, uint32_t stride,
                                hipStream_t stream, bool msg_slots = false);

// f1: on-device CanonicalVote assembly.  Templates are kVoteTmplBytes records
// ([pre_len, bid_len, cid_len, 0] + bytes); message i is written to out + i * kVoteSlot
// and its length to out_len[i].  With msg_slots = true the verify launchers read
// messages that way (off = lengths).
constexpr uint32_t kVoteTmplBytes = 256;
constexpr uint32_t kVoteSlot = 256;
hipError_t launch_assemble_votes(const uint8_t *tmpl, const uint32_t *tmpl_idx, const uint8_t *flags,
                                 const int64_t *ts_sec, const int32_t *ts_nanos, uint32_t n, uint8_t *out,
                                 uint32_t *out_len, hipStream_t stream);

}  // namespace tmed
