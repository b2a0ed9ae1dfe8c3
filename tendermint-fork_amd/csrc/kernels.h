// kernels.h — launch interface between the C-ABI layer and the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "ge25519.h"
#include "signbytes.h"

namespace tmed {

// Optional per-launch HIP-event timing of the verify pipeline (diagnostics / bench roofline):
// events are recorded on the launch stream before prep, between prep and main, after main.
// mark(s, kind) records an event that ENDS a kernel of that kind (0 prep, 1 main, 2 finish;
// -1 = start mark); interval i (ev[i-1] -> ev[i]) is charged to kind[i].
struct KernelTimer {
  static constexpr int kMax = 160;
  hipEvent_t ev[kMax];
  int kind[kMax];
  int n = 0;
  void mark(hipStream_t s, int k) {
    if (n < kMax) { kind[n] = k; (void)hipEventRecord(ev[n++], s); }
  }
};

constexpr uint32_t kThreadsPerBlock = 256;
// Variable-base table slab: lane slots (grid-stride loop bounds the grid to
// slab_slots / kThreadsPerBlock blocks).
constexpr uint32_t kSlabSlotBytes = 8 * 128;  // cached j*P, j = 1..8, in fe_pack256 form (j = 0: one shared row)
// The half-size path (main variant 6, the default) keeps two per-lane tables (-A and
// -sign(d) R): its slab has two slot regions; the full-length fallback (variant 5) one.
inline uint32_t slab_tables(int main_waves) { return main_waves == 5 ? 1u : 2u; }

// Batched finish (verify_core.h finish_group): the main kernels hand projective R' over in
// fin ([q][slot], kFinInt4 int4 per signature, kFinCap slots); the finish kernel runs once per
// block of <= kFinCap signatures, with up to kFinGroupMax signatures per inversion.  fin_pre
// holds the prefix products ([3][kFinPreStride] int4).
constexpr uint32_t kFinCap = 1u << 20;
constexpr int kFinInt4 = 8;
constexpr uint32_t kFinGroupMax = 16;
constexpr uint32_t kFinPreStride = kFinCap + 64;
constexpr size_t kFinBytes = (size_t)kFinCap * kFinInt4 * 16;
constexpr size_t kFinPreBytes = (size_t)kFinPreStride * 3 * 16;

// The shared B tables of the generic main kernels: the radix-2^16 table of j*B (full-length
// fallback, variant 5) and the radix-2^16 comb of B (windows 0 and 8: the half-size default).
struct BTabs {
  const int4 *b16;
  const int4 *comb16;
  const int4 *b26 = nullptr;  // radix-2^26 B windows of the half-size main kernel (null: radix 2^16)
};
// j * B and j * 2^128 B for j = 0..2^25 (affine niels, 128-B rows): the two radix-2^26 tables of
// verify_main_hs_kernel<26>, 8.6 GB, built once per device (tmed_capi.hip b26_acquire).
constexpr uint32_t kB26Entries = (1u << 25) + 1;
constexpr size_t kB26Bytes = 2 * (size_t)kB26Entries * 128;
hipError_t launch_build_b26(const int4 *comb16, int4 *tab, hipStream_t stream);
// Signed radix-2^24 comb of +B for the key-cached throughput kernel: window w holds j * 2^(24w) B
// for j = 0..2^23 (11 windows, 11.8 GB, built once per device at the first key-set load:
// keyset.hip b24_acquire): eleven B additions per signature instead of sixteen.
constexpr int kB24Windows = 11;
constexpr uint32_t kB24Entries = (1u << 23) + 1;
constexpr size_t kB24Bytes = (size_t)kB24Windows * kB24Entries * 128;
hipError_t launch_build_b24(const int4 *comb16, int4 *tab, hipStream_t stream);
constexpr uint32_t kB16Entries = 32769;
constexpr size_t kB16Bytes = (size_t)kB16Entries * 128;
hipError_t launch_build_b16(int4 *tab, hipStream_t stream);
// Radix-2^16 comb of +B for the key-cached throughput kernel (16 x kB16Entries x 128 B).
constexpr size_t kBComb16Bytes = 16 * kB16Bytes;
void host_bcomb16_bases(int32_t out[16 * 40]);
hipError_t launch_build_bcomb16(const int32_t *d_bases, int4 *comb, hipStream_t stream);

hipError_t launch_verify(const uint8_t *pub, const uint8_t *sig, const uint8_t *msgs, const uint32_t *off,
                         uint32_t n, uint8_t *out, int4 *slab, uint32_t slab_stride, BTabs btab,
                         int4 *prep, int4 *fin, int4 *fin_pre, hipStream_t stream, uint32_t chunk = 0,
                         int main_waves = 6, bool msg_slots = false, KernelTimer *timer = nullptr,
                         bool zip215 = false);

// The generic prep alone (k, S checks, decode of A) for signatures [base, base + count) into prep
// slots 0..count-1 (the ZIP-215 batch mode's first phase).
hipError_t launch_verify_prep(const uint8_t *pub, const uint8_t *sig, const uint8_t *msgs, const uint32_t *off,
                              bool msg_slots, uint32_t base, uint32_t count, int4 *prep, uint32_t stride,
                              hipStream_t stream);
// ZIP-215 (opt-in) batch verification of device-resident tuples (zip215.hip); ctx-level.
constexpr uint32_t kZipMax = 1u << 20;  // signatures per batch equation (one MSM)

// RFC 8032 signer (synthetic commits) on the shared comb of B.
hipError_t launch_sign(const uint8_t *seeds, const uint8_t *msgs, const uint32_t *off, uint32_t n, uint8_t *sig_out,
                       uint8_t *pub_out, const int4 *bcomb, hipStream_t stream);

// prep hand-off bytes per signature slot: 10 int4 (k, s, A, ok) + 16 int4 (the half-size hand-off,
// placed in window-count order: kernels.hip verify_prep_r_kernel).  The allocation carries
// kPrepTailBytes more for the two placement counters of the half-size path.
constexpr uint32_t kPrepSlotBytes = 416;
constexpr uint32_t kPrepTailBytes = 256;

// ---- fixed-base combs (key cache) -------------------------------
// Signed radix-256 comb of a point P: entry [w][j] = j * 256^w * P (niels, affine),
// w = 0..31, j = 0..128 (j = 0 is the identity), 128 B per entry (30 limbs + pad).
// [k]P = sum_w comb[w][d_w] with d_w = byte_w(k + 0x80...80) - 128 in [-128, 127]:
// 32 mixed additions and no doublings.
constexpr int kCombWindows = 32;
constexpr int kCombEntries = 129;
constexpr int kCombEntryInt4 = 8;  // 128 B
constexpr size_t kCombBytesPerKey = (size_t)kCombWindows * kCombEntries * kCombEntryInt4 * 16;
// A key set's combs live in chunks of kKeyChunkKeys keys, each chunk its own allocation, so a set
// grows by adding chunks: the keys already built never move, nothing is copied or freed (a pool
// of 20k keys is ~130 GB, and freeing a large allocation costs ~1.5 s per 68 GB on the box).  Key
// v's rows are in chunk v >> kKeyChunkBits at key offset v & (kKeyChunkKeys - 1); the kernels take
// a device table of chunk bases (keyset.hip: the radix-256 comb's table, then the radix-2^12's).
constexpr int kKeyChunkBits = 9;                                  // 512 keys: 270 MB radix-256, 2.96 GB radix-2^12
constexpr uint32_t kKeyChunkKeys = 1u << kKeyChunkBits;
constexpr uint32_t kKeyChunksMax = (1u << 24) >> kKeyChunkBits;  // key indexes are < 2^24

// bases[key][w] = 256^w * (negate ? -A : A) as p3 (40 limbs); ok[key] = decode accepted.
hipError_t launch_comb_bases(const uint8_t *pubs, uint32_t n, int negate, uint8_t *ok, int32_t *bases,
                             hipStream_t stream);
// comb[key] from bases[key] (n * 32 workgroups of 128 lanes).
hipError_t launch_comb_fill(const int32_t *bases, uint32_t n, int4 *comb, hipStream_t stream);
// Signed radix-2^B comb of -A for the key-cached throughput kernel (B = kCombABits, 12 by default):
// entry [w][j] = j * 2^(Bw) * (-A).  W = floor(253 / B) windows; digit m < W - 1 is bits
// [Bm, Bm + B) + bit (Bm - 1) - 2^B * bit (Bm + B - 1), in [-2^(B-1), 2^(B-1)] (no carry chain);
// the top digit (m = W - 1) is every bit from B(W - 1) up + bit (B(W - 1) - 1), unsigned: k < L
// puts it in [0, 2^(252 - B(W - 1)) + 1] (B = 12: bits 240..252, [0, 4097]), so window W - 1 holds
// j = 0 .. kCombATopEntries - 1 (whole 128-entry fill groups).  B = 12: 21 rows per signature
// (radix 2^11: 23, radix 2^10: 26, radix 256: 32), 5.8 MB per key (58 GB for 10k keys), built at a
// key set's first throughput batch.  TMED_COMBA_BITS picks B in 10..12.
#ifndef TMED_COMBA_BITS
#define TMED_COMBA_BITS 12
#endif
constexpr int kCombABits = TMED_COMBA_BITS;
constexpr int kCombAWindows = 253 / kCombABits;                             // 21 (B = 12), 23 (11), 25 (10)
constexpr int kCombATopField = 253 - kCombABits * (kCombAWindows - 1);      // 13 (B = 12)
constexpr uint32_t kCombAEntries = (1u << (kCombABits - 1)) + 1;            // 2049: j = 0..2048
constexpr uint32_t kCombATopMax = (1u << (kCombATopField - 1)) + 1;         // 4097 (k < L)
constexpr uint32_t kCombATopGroups = (kCombATopMax + 127) / 128;            // 33
constexpr uint32_t kCombATopEntries = kCombATopGroups * 128 + 1;            // 4225
static_assert(kCombABits >= 10 && kCombABits <= 12 && kCombATopField >= kCombABits, "comb radix");
constexpr size_t kCombARowsPerKey = (size_t)(kCombAWindows - 1) * kCombAEntries + kCombATopEntries;
constexpr size_t kCombABytesPerKey = kCombARowsPerKey * kCombEntryInt4 * 16;
// row of entry j of window w within a key's comb
constexpr size_t comba_row(int w, uint32_t j) { return (size_t)w * kCombAEntries + j; }
// comba[key] of -A_key (bases: scratch of n * kCombAWindows * 40 int32).
hipError_t launch_build_comba(const uint8_t *pubs, uint32_t n, int32_t *bases, int4 *comba, hipStream_t stream);
// Key-cached verification: key index per signature into a keyset of nkeys keys (an index
// >= nkeys rejects that signature); acomb / acomba: the key set's chunk tables (kKeyChunk*).  perm (nullable, n entries of scratch) + order_scratch
// (key_order_scratch_words): the main and finish kernels visit each chunk's signatures in
// key-grouped order (launch_key_order per chunk); decisions still land at out[i].
hipError_t launch_verify_keyset(const uint32_t *val_idx, uint32_t nkeys, const uint8_t *key_pub, const uint8_t *key_ok,
                                const int4 *const *acomb, const int4 *bcomb, const uint8_t *sig, const uint8_t *msgs,
                                const uint32_t *off, uint32_t n, uint8_t *out, int4 *prep, uint32_t stride,
                                int4 *fin, int4 *fin_pre, hipStream_t stream, bool msg_slots = false,
                                KernelTimer *timer = nullptr, uint32_t *perm = nullptr,
                                uint32_t *order_scratch = nullptr, const int4 *bcomb24 = nullptr,
                                const int4 *const *acomba = nullptr);
// Key-grouped visiting order of a key-cached batch (counting sort of val_idx by groups of
// consecutive keys, indices >= nkeys last): perm[0..n) = signature indices grouped by key.
// scratch: key_order_scratch_words(n, nkeys) u32.  The comb rows of the lanes in flight then
// come from few keys (TLB / L2 locality across a multi-GB key set).
constexpr uint32_t kKeyOrderMaxKeys = 1u << 24;
uint32_t key_order_scratch_words(uint32_t n, uint32_t nkeys);
// perm[j] = index_base + i for the signatures i of val_idx[0..n) in key-grouped order.
hipError_t launch_key_order(const uint32_t *val_idx, uint32_t n, uint32_t nkeys, uint32_t *scratch, uint32_t *perm,
                            uint32_t index_base, hipStream_t stream);

// Window-count statistics of the last half-size chunk in the prep hand-off (count lanes):
// d_hist[0..64] per-lane W, d_hist[65..129] per-wave maximum W.
// Tests (tmed_test_stream_delay): one wave that sleeps about `us` microseconds on `stream` before
// the work queued after it, so a consumer on another stream that does not wait for that work
// reads it unfinished.  us = 0: nothing is launched.
hipError_t launch_test_delay(hipStream_t stream, uint32_t us);
hipError_t launch_window_stats(const int4 *prep, uint32_t stride, uint32_t count, uint32_t *d_hist,
                               hipStream_t stream);

// Latency mode for small key-cached batches (n <= kLatMax): 8 lanes per signature for the
// comb sum, strict decode of R on other lanes instead of the inversion; two launches.
// fin as above; dec: kLatDecInt4 x n int4 (fits the fin_pre buffer for n <= kLatMax).
constexpr uint32_t kLatMax = 1u << 16;
struct VoteAsm;
// va (vote slots only): every lane of a signature's group assembles the vote's sign-bytes into
// its slot first (identical bytes; no separate assemble_votes launch in front).
hipError_t launch_verify_keyset_lat(const uint32_t *val_idx, uint32_t nkeys, const uint8_t *key_pub, const uint8_t *key_ok,
                                    const int4 *const *acomb, const int4 *bcomb, const uint8_t *sig, const uint8_t *msgs,
                                    const uint32_t *off, uint32_t n, uint8_t *out, int4 *fin, int4 *dec,
                                    hipStream_t stream, bool msg_slots = false, const VoteAsm *va = nullptr);

// Latency mode of the generic path (latency.hip; n <= kGLatMax): decode / hash roles, then
// 8 lanes per signature (two quads, 4-way point formulas).  hand: kGLatHandBytes of scratch.
constexpr uint32_t kGLatMax = 1u << 16;
constexpr size_t kGLatHandBytes = (size_t)kGLatMax * (6 * 2 + 7) * 16;
// Per-vote inputs of the device sign-bytes assembly (votes_dev.h; device or pinned-host pointers).
struct VoteAsm {
  const uint8_t *tmpl;
  const uint32_t *tmpl_idx;
  const uint8_t *flags;
  const int64_t *ts_sec;
  const int32_t *ts_nanos;
};

// va (vote slots only): the hash lanes assemble their vote's sign-bytes into its slot of msgs
// first (no separate assemble_votes launch in front of the latency kernels).
hipError_t launch_verify_glat(const uint8_t *pub, const uint8_t *sig, const uint8_t *msgs, const uint32_t *off,
                              uint32_t n, uint8_t *out, const int4 *comb16, int4 *hand, hipStream_t stream,
                              bool msg_slots = false, KernelTimer *timer = nullptr, const VoteAsm *va = nullptr);

// f1: on-device CanonicalVote assembly.  Templates are kVoteTmplBytes records
// ([pre_len, bid_len, cid_len, 0] + bytes); message i is written to out + i * kVoteSlot
// and its length to out_len[i].  With msg_slots = true the verify launchers read
// messages that way (off = lengths).
// (kVoteTmplBytes, kVoteSlot: signbytes.h, shared with the host seam)
hipError_t launch_assemble_votes(const uint8_t *tmpl, const uint32_t *tmpl_idx, const uint8_t *flags,
                                 const int64_t *ts_sec, const int32_t *ts_nanos, uint32_t n, uint8_t *out,
                                 uint32_t *out_len, hipStream_t stream);

}  // namespace tmed
