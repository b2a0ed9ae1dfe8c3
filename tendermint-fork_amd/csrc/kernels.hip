// kernels.hip — gfx950 kernels: batch ed25519 verify and RFC 8032 sign.
//
// One signature per lane (64 per wave) on the throughput paths.  The work per signature
// is ~2.2e5 32x32->64 integer multiply-adds, entirely VALU; the
// algorithmic HBM traffic is ~214 B per verify, so the kernels are bound by integer-VALU
// issue, not by memory and not by MFMA (which has no 32x32->64 integer path).
//
// Memory layout
//   pub   n x 32 B, sig n x 64 B (16-B aligned rows -> dwordx4 loads)
//   msgs  concatenated bytes, off[n+1] u32 (or fixed 256-B vote slots)
//   slab  per-lane variable-base tables: 8 cached points x 128 B (fe_pack256), lane-major [slot][entry][chunk]
//   b16   32769 niels multiples of B in 128-B rows in HBM (4.2 MB; the full-length fallback, variant 5)
//   combs key-set combs [key][window][entry] and the shared combs of B (radix 256, radix 2^16)
#include "kernels.h"
#ifndef TMED_SLAB_PF
#define TMED_SLAB_PF 1  // per-lane table rows loaded ahead (verify_hs.h hs_straus): the -A row before
                        // the last doubling, the R row before the -A addition (0: right before use)
#endif
#include "verify_core.h"
#include "verify_hs.h"
#include "kernel_util.h"
#include "votes_dev.h"

namespace tmed {

// Per-lane table in the HBM slab, lane-major [slot][entry 1..8][chunk]: each lane's entry is one
// aligned 128-B line (the four coordinates in fe_pack256 form), so a divergent lookup reads
// exactly one line.  The slab does not fit L2/MALL at full occupancy; the 160-B int32 form
// read 2.25 lines per lookup, and its traffic cost ~10 % of the clock (profiles/r02/s4).
// Entry 0 (the identity, cached form (1, 1, 1, 0)) is not stored per lane: every lane reads this
// one row (an L2 hit), so the slab holds entries 1..8.
// (a plain __device__ variable: global address space like the slab, so the row select below stays a
// global pointer and the table loads are global_load — a select against a constant-address-space
// row made them flat_load, which also count in lgkmcnt: every s_waitcnt lgkmcnt(0) of the B-row
// prefetch then waited for the table rows in flight as well)
__device__ int4 kIdentityRow[8] = {{1, 0, 0, 0}, {0, 0, 0, 0}, {1, 0, 0, 0}, {0, 0, 0, 0},
                                          {1, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};

// Per-lane table rows go through the default cache policy: a non-temporal policy for the slab
// stores, the slab loads or the B rows was measured at -12 / -6 / -0.5 % on C2 (all three -26 %,
// profiles/r05/s2/): a lane re-reads its rows ~4 times and nt sends every re-read to HBM.
__device__ __forceinline__ void slab_st(int4 *p, int4 v) { *p = v; }
__device__ __forceinline__ int4 slab_ld(const int4 *p) { return *p; }

struct SlabTab {
  int4 *base;
  uint32_t slot;

  __device__ __forceinline__ const int4 *row(int j) const {
    return j == 0 ? kIdentityRow : base + ((size_t)slot * 8 + (j - 1)) * 8;
  }

  __device__ __forceinline__ void store(int j, const ge_cached &c) const {
    if (j == 0) return;
    int4 *r = base + ((size_t)slot * 8 + (j - 1)) * 8;
    const fe *fs[4] = {&c.YpX, &c.YmX, &c.Z, &c.T2d};
#pragma unroll
    for (int f = 0; f < 4; f++) {
      uint32_t w[8];
      fe_pack256(w, *fs[f]);
      slab_st(r + 2 * f, make_int4((int)w[0], (int)w[1], (int)w[2], (int)w[3]));
      slab_st(r + 2 * f + 1, make_int4((int)w[4], (int)w[5], (int)w[6], (int)w[7]));
    }
  }
  __device__ __forceinline__ void load(int j, ge_cached &c) const {
    fe *fs[4] = {&c.YpX, &c.YmX, &c.Z, &c.T2d};
    const int4 *r = row(j);
    int4 v[8];
#pragma unroll
    for (int q = 0; q < 8; q++) v[q] = r[q];
#pragma unroll
    for (int f = 0; f < 4; f++) {
      const uint32_t w[8] = {(uint32_t)v[2 * f].x, (uint32_t)v[2 * f].y, (uint32_t)v[2 * f].z,
                             (uint32_t)v[2 * f].w, (uint32_t)v[2 * f + 1].x, (uint32_t)v[2 * f + 1].y,
                             (uint32_t)v[2 * f + 1].z, (uint32_t)v[2 * f + 1].w};
      fe_unpack256(*fs[f], w);
    }
  }
#if TMED_SLAB_PF
  // prefetch issues the row's eight 16-B loads into registers (swap: Y+X and Y-X exchanged by
  // the load addresses — a negative digit's entry, ge_add_cached_pre); take unpacks them
  int4 pv[8];
  __device__ __forceinline__ void prefetch(int j, bool swap = false) {
    const int4 *r = row(j);
    const int sx = swap ? 2 : 0;
#pragma unroll
    for (int q = 0; q < 8; q++) pv[q] = slab_ld(r + (q < 4 ? (q ^ sx) : q));
  }
  __device__ __forceinline__ void take(ge_cached &c) const {
    fe *fs[4] = {&c.YpX, &c.YmX, &c.Z, &c.T2d};
#pragma unroll
    for (int f = 0; f < 4; f++) {
      const uint32_t w[8] = {(uint32_t)pv[2 * f].x, (uint32_t)pv[2 * f].y, (uint32_t)pv[2 * f].z,
                             (uint32_t)pv[2 * f].w, (uint32_t)pv[2 * f + 1].x, (uint32_t)pv[2 * f + 1].y,
                             (uint32_t)pv[2 * f + 1].z, (uint32_t)pv[2 * f + 1].w};
      fe_unpack256(*fs[f], w);
    }
  }
#else
  int pf = 0;
  bool sw = false;
  __device__ __forceinline__ void prefetch(int j, bool swap = false) { pf = j; sw = swap; }
  __device__ __forceinline__ void take(ge_cached &c) const {
    ge_cached t;
    load(pf, t);
    fe_select(c.YpX, t.YpX, t.YmX, sw);
    fe_select(c.YmX, t.YmX, t.YpX, sw);
    fe_copy(c.Z, t.Z);
    fe_copy(c.T2d, t.T2d);
  }
#endif
};

typedef __attribute__((address_space(1))) void global_void;
typedef __attribute__((address_space(3))) void lds_void;

// Radix-2^16 / 2^26 B table (double_scalarmult<16>, hs_straus): j*B, j = 0..32768 / 2^25, affine niels in 128-B rows
// (kCombEntryInt4 int4, 4.2 MB, L2/MALL-resident).  The entry of the next B window is fetched
// into LDS with global_load_lds_dwordx4 right after the current B addition, 16 doublings
// before it is needed; buf is this wave's [8][64] int4 region (lane l's piece q at q*64+l).
template <int BITS>
struct BPf {
  static constexpr int kBits = BITS;
  const int4 *tab;
  int4 *buf;
  uint32_t lane;
  __device__ __forceinline__ void prefetch(int j) const {
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the previous take's LDS reads are done
#pragma unroll
    for (int q = 0; q < 8; q++)
      __builtin_amdgcn_global_load_lds((global_void *)(tab + (size_t)j * 8 + q), (lds_void *)(buf + q * 64), 16, 0, 0);
  }
  __device__ __forceinline__ void take(ge_niels &e) const {
    fe *fs[3] = {&e.YpX, &e.YmX, &e.XY2d};
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const int4 v = buf[q * 64 + lane];
      const int32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int c = 0; c < 4; c++) {
        const int f = 4 * q + c;
        if (f < 30) fs[f / 10]->v[f % 10] = w[c];
      }
    }
  }
};

// Per-signature hand-off from the prep to the main kernel: k, s, A.x, A.y, ok
// (37 words padded to 10 x int4), stored [chunk q][slot] for coalescing.
constexpr int kPrepInt4 = 10;

__device__ __forceinline__ void prep_store(int4 *prep, uint32_t stride, uint32_t slot, const uint32_t k[8],
                                           const uint32_t s[8], const ge_p3 &A, bool ok) {
  int32_t w[40];
#pragma unroll
  for (int i = 0; i < 8; i++) { w[i] = (int32_t)k[i]; w[8 + i] = (int32_t)s[i]; }
#pragma unroll
  for (int i = 0; i < 10; i++) { w[16 + i] = A.X.v[i]; w[26 + i] = A.Y.v[i]; }
  w[36] = ok ? 1 : 0;
  w[37] = w[38] = w[39] = 0;
#pragma unroll
  for (int q = 0; q < kPrepInt4; q++)
    prep[(size_t)q * stride + slot] = make_int4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
}

// The key-cached hand-off: only what verify_keyset_main_kernel reads (k, s in int4 0..3, ok at
// word 36 = int4 9): 80 B per signature instead of the generic prep's 160 B.
__device__ __forceinline__ void prep_store_ks(int4 *prep, uint32_t stride, uint32_t slot, const uint32_t k[8],
                                              const uint32_t s[8], bool ok) {
  prep[slot] = make_int4((int)k[0], (int)k[1], (int)k[2], (int)k[3]);
  prep[(size_t)stride + slot] = make_int4((int)k[4], (int)k[5], (int)k[6], (int)k[7]);
  prep[(size_t)2 * stride + slot] = make_int4((int)s[0], (int)s[1], (int)s[2], (int)s[3]);
  prep[(size_t)3 * stride + slot] = make_int4((int)s[4], (int)s[5], (int)s[6], (int)s[7]);
  prep[(size_t)9 * stride + slot] = make_int4(ok ? 1 : 0, 0, 0, 0);
}

__device__ __forceinline__ bool prep_load(const int4 *prep, uint32_t stride, uint32_t slot, uint32_t k[8],
                                          uint32_t s[8], ge_p3 &A) {
  int32_t w[40];
#pragma unroll
  for (int q = 0; q < kPrepInt4; q++) {
    const int4 v = prep[(size_t)q * stride + slot];
    w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
  }
#pragma unroll
  for (int i = 0; i < 8; i++) { k[i] = (uint32_t)w[i]; s[i] = (uint32_t)w[8 + i]; }
#pragma unroll
  for (int i = 0; i < 10; i++) { A.X.v[i] = w[16 + i]; A.Y.v[i] = w[26 + i]; }
  fe_1(A.Z);
  fe_mul(A.T, A.X, A.Y);
  return w[36] != 0;
}

// Phase 1: SHA-512(R||A||M) mod L, S < L, A = Point.SetBytes(pub)  (one lane per signature
// of the chunk [base, base + count)).
// Threads per block of the generic throughput kernels (prep, prep_r, the half-size main): 256.
// (Blocks of 64 / 128 threads, whose wave slots come back sooner at a launch's end, were level /
// 4 % slower per C2 step: profiles/r05/s32/.)
constexpr uint32_t kHsBlock = kThreadsPerBlock;

#ifndef TMED_PREP_WAVES
#define TMED_PREP_WAVES 3  // 152 VGPRs, no spills (4 waves with a leaner decode: no faster, profiles/r03/prep_joint)
#endif
__global__ __launch_bounds__(kHsBlock, TMED_PREP_WAVES) void verify_prep_kernel(
    const uint8_t *__restrict__ pub, const uint8_t *__restrict__ sig, MsgSrc ms, uint32_t base, uint32_t count,
    int4 *__restrict__ prep, uint32_t stride, uint32_t *__restrict__ place) {
  const uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x;
  if (place && slot == 0) place[0] = place[1] = 0;  // the half-size placement counters (verify_prep_r_kernel)
  if (slot >= count) return;
  const uint32_t i = base + slot;
#ifndef TMED_PREP_SHA_FIRST
#define TMED_PREP_SHA_FIRST 1
#endif
#if TMED_PREP_SHA_FIRST
  // verify_prep's steps with the hash first and k, s handed over at once, so the decode of A
  // runs with only the key's words live (s keeps S when only A fails to decode: the verdict
  // is false either way and S < L after the S checks).
  uint32_t pw[8];
  bool sok;
  {
    uint32_t sw[16], k[8], h[16];
    load_row_words(pw, pub + 32 * (size_t)i, 2);
    load_row_words(sw, sig + 64 * (size_t)i, 4);
    const uint8_t *m;
    uint32_t mlen;
    ms.get(i, m, mlen);
    sok = (sw[15] & 0xE0000000u) == 0 && sc_is_canonical(sw + 8);
    sha512_stream(h, sw, pw, 64, m, mlen);
    sc_reduce512(k, h);
#pragma unroll
    for (int q = 0; q < 2; q++)
      prep[(size_t)q * stride + slot] = make_int4((int)k[4 * q], (int)k[4 * q + 1], (int)k[4 * q + 2], (int)k[4 * q + 3]);
#pragma unroll
    for (int q = 0; q < 2; q++) {
      const uint32_t *S = sw + 8 + 4 * q;
      prep[(size_t)(2 + q) * stride + slot] = sok ? make_int4((int)S[0], (int)S[1], (int)S[2], (int)S[3])
                                                  : make_int4(0, 0, 0, 0);
    }
  }
  ge_p3 A;
  const bool ok = ge_frombytes_go(A, pw) && sok;  // Point.SetBytes (identity on failure)
  int32_t w[24];
#pragma unroll
  for (int j = 0; j < 10; j++) { w[j] = A.X.v[j]; w[10 + j] = A.Y.v[j]; }
  w[20] = ok ? 1 : 0;
  w[21] = w[22] = w[23] = 0;
#pragma unroll
  for (int q = 0; q < 6; q++)  // words 16..39: A.x, A.y, ok
    prep[(size_t)(4 + q) * stride + slot] = make_int4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
#else
  uint32_t pw[8], sw[16], k[8], s[8];
  load_row_words(pw, pub + 32 * (size_t)i, 2);
  load_row_words(sw, sig + 64 * (size_t)i, 4);
  const uint8_t *m;
  uint32_t mlen;
  ms.get(i, m, mlen);
  ge_p3 A;
  const bool ok = verify_prep(pw, sw, m, mlen, k, s, A);
  prep_store(prep, stride, slot, k, s, A, ok);
#endif
}

// ---- f1: CanonicalVote sign-bytes assembled on the device ----------
// (votes_dev.h assemble_vote_into; this kernel serves the throughput and key-cached paths, the
// latency kernels assemble in their hash lanes.)  One wave per block: every lane assembles its
// vote in LDS (byte stores to LDS, beside its staged template), then the wave writes its 64
// consecutive 256-B slots as sixteen coalesced 1-KB rows.  Assembled straight into the global
// slots, each lane's ~114 byte stores went to 64 different lines per instruction: 0.29 ms per
// 853k-vote blocksync batch (profiles/r03/fin2/kernel_stats.csv).
constexpr uint32_t kAsmLanes = 64;
__global__ __launch_bounds__(kAsmLanes) void assemble_votes_kernel(VoteAsm va, uint32_t n, uint8_t *__restrict__ out,
                                                                  uint32_t *__restrict__ out_len) {
  __shared__ int4 tl[kAsmLanes][kVoteTmplBytes / 16];
  __shared__ int4 ob[kAsmLanes][kVoteSlot / 16];
  const uint32_t lane = threadIdx.x, i0 = blockIdx.x * kAsmLanes, i = i0 + lane;
  if (i < n) {
#pragma unroll
    for (int q = 0; q < (int)(kVoteSlot / 16); q++) ob[lane][q] = make_int4(0, 0, 0, 0);
    out_len[i] = assemble_vote_into(va, i, reinterpret_cast<uint8_t *>(ob[lane]), tl[lane]);
  }
  __syncthreads();
  const uint32_t nslots = n - i0 < kAsmLanes ? n - i0 : kAsmLanes;
  int4 *dst = reinterpret_cast<int4 *>(out + (size_t)i0 * kVoteSlot);
  const int4 *src = &ob[0][0];
#pragma unroll
  for (uint32_t q = 0; q < kVoteSlot / 16; q++) {
    const uint32_t c = q * kAsmLanes + lane;  // int4 index in the wave's 16-KB run of slots
    if (c / (kVoteSlot / 16) < nslots) dst[c] = src[c];
  }
}

// Projective R' of signature slot (X, Y, Z: 30 limbs + 2 pad = 8 int4), stored [q][slot].
__device__ __forceinline__ void fin_store(int4 *fin, uint32_t stride, uint32_t slot, const fe &X, const fe &Y,
                                          const fe &Z) {
  int32_t w[32];
#pragma unroll
  for (int i = 0; i < 10; i++) { w[i] = X.v[i]; w[10 + i] = Y.v[i]; w[20 + i] = Z.v[i]; }
  w[30] = w[31] = 0;
#pragma unroll
  for (int q = 0; q < kFinInt4; q++)
    fin[(size_t)q * stride + slot] = make_int4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
}

// Phase 2 of the full-length fallback (TMED_MAIN_WAVES=5): table of -A, Straus [k](-A) + [s]B
// (radix-2^16 B windows from the HBM table, each entry fetched into LDS 16 doublings ahead)
// -> projective R' (hand-off to the batched finish).
__global__ __launch_bounds__(kThreadsPerBlock, 2) void verify_main_kernel(
    uint32_t base, uint32_t count, const int4 *__restrict__ prep, uint32_t stride, int4 *__restrict__ slab,
    const int4 *__restrict__ b16, int4 *__restrict__ fin, uint32_t fin_base, uint8_t *__restrict__ out) {
  __shared__ int4 sb16[kThreadsPerBlock / 64][8 * 64];
  const uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x;
  if (slot >= count) return;
  const uint32_t i = base + slot;
  uint32_t k[8], s[8];
  ge_p3 A;
  const bool ok = prep_load(prep, stride, slot, k, s, A);
  ge_p2 R;
  BPf<16> bt{b16, sb16[threadIdx.x >> 6], threadIdx.x & 63u};
  SlabTab tab{slab, slot};
  verify_main_point(R, k, s, A, tab, bt);
  fin_store(fin, kFinCap, i - fin_base, R.X, R.Y, R.Z);
  out[i] = ok ? 1 : 0;
}

// ---- half-size path (verify_hs.h; main variant 6, the default) -----------------------
// verify_prep_kernel writes k, s, A, ok to the first prep region (10 int4 per slot); the
// R kernel writes the second region (kPrepHsInt4 int4 per position, [q][position]): recoded c
// (words 0-7), recoded |d| (8-12), recoded e (13-20), R.x (21-30), R.y (31-40), flags (41:
// bit 0 ok, bit 1 d < 0, bits 8.. window count W), the signature's slot (42), A.x (44-53),
// A.y (54-63) — everything the main kernel reads.
//
// Placement by window count: the main kernel runs every lane of a wave over the wave's largest
// W, and W is 32 or 33 for almost every signature (a few lanes 34+).  The R kernel therefore
// writes signatures with W > 32 from the front of the region and the others (W <= 32) from the back
// (one atomic per wave and group on place[0] / place[1], the lanes of a group at consecutive
// positions, so the stores stay coalesced): the waves of the W <= 32 part run 32 windows instead
// of the unsorted wave maximum (~33.3 on average, tmed_window_stats), ~2 % of the main kernel.
// The longer waves go first, so the launch's last round holds short ones (-0.3 % per C2 step
// against short first, 9 of 11 alternating rounds, profiles/r05/s33/).
constexpr int kPrepHsInt4 = 16;
constexpr int kHsWSmall = 32;
static_assert((kPrepInt4 + kPrepHsInt4) * 16 <= kPrepSlotBytes, "prep slot too small for the half-size hand-off");

#ifndef TMED_PREP_R_WAVES
#define TMED_PREP_R_WAVES 3  // 168 VGPRs, 6 spilled: -0.06 ms per 2^20 against 2 waves (the Euclid loop hides its memory waits)
#endif
__global__ __launch_bounds__(kHsBlock, TMED_PREP_R_WAVES) void verify_prep_r_kernel(
    const uint8_t *__restrict__ sig, uint32_t base, uint32_t count, const int4 *__restrict__ prep,
    int4 *__restrict__ prep2, uint32_t stride, uint32_t *__restrict__ place, int zip215) {
  const uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x;
  if (slot >= count) return;
  // R's decode first (the sqrt-ratio chain), then k and s from the hand-off for the lattice step:
  // nothing of the hand-off is live across the chain, so the kernel fits 3 waves/SIMD unspilled
  uint32_t Rw[8];
  load_row_words(Rw, sig + 64 * (size_t)(base + slot), 2);
  fe Rx, Ry;
  bool rok;
  if (zip215) {
    ge_p3 P;
    rok = ge_frombytes_go(P, Rw);
    fe_copy(Rx, P.X);
    fe_copy(Ry, P.Y);
  } else {
    rok = r_decode_strict(Rx, Ry, Rw);
  }
  if (!rok) { fe_0(Rx); fe_1(Ry); }
  int32_t w[64];
#pragma unroll
  for (int q = 0; q < 4; q++) {  // k (words 0-7), s (8-15)
    const int4 v = prep[(size_t)q * stride + slot];
    w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
  }
  uint32_t k[8], s[8], cr[8], dr[8], er[8];
#pragma unroll
  for (int j = 0; j < 8; j++) { k[j] = (uint32_t)w[j]; s[j] = (uint32_t)w[8 + j]; }
  bool dneg;
  int W, Wl;  // W: the tight window count (top digits 0..16, hs_straus), Wl the latency kernels' count
  hs_scalars(k, s, cr, dr, er, dneg, Wl, /*raw_e=*/true, &W);  // (hs_prep_r's two phases, in this order)
  const bool ok = prep[(size_t)9 * stride + slot].x != 0;  // word 36
#pragma unroll
  for (int j = 0; j < 8; j++) { w[j] = (int32_t)cr[j]; w[13 + j] = (int32_t)er[j]; }
#pragma unroll
  for (int j = 0; j < 5; j++) w[8 + j] = (int32_t)dr[j];
#pragma unroll
  for (int j = 0; j < 10; j++) { w[21 + j] = Rx.v[j]; w[31 + j] = Ry.v[j]; }
  w[41] = ((ok && rok) ? 1 : 0) | (dneg ? 2 : 0) | (W << 8);
  w[42] = (int32_t)slot;
  w[43] = 0;
#pragma unroll
  for (int q = 4; q < 9; q++) {  // A.x, A.y: words 16..35 of the first region
    const int4 v = prep[(size_t)q * stride + slot];
    w[28 + 4 * q] = v.x; w[29 + 4 * q] = v.y; w[30 + 4 * q] = v.z; w[31 + 4 * q] = v.w;
  }
  // position: W > kHsWSmall from the front, the rest from the back (count - 1 downwards), so the
  // main kernel's longest waves are dispatched first
  const bool front = W > kHsWSmall;
  const uint64_t act = __ballot(1), sm = __ballot(front);
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  uint32_t fs = 0, fl = 0;
  if (lane == (uint32_t)__builtin_ctzll(act)) {  // the wave's first active lane takes both ranges
    const uint32_t ns = (uint32_t)__builtin_popcountll(sm), nl = (uint32_t)__builtin_popcountll(act & ~sm);
    if (ns) fs = atomicAdd(&place[0], ns);
    if (nl) fl = atomicAdd(&place[1], nl);
  }
  const int leader = __builtin_ctzll(act);
  fs = (uint32_t)__shfl((int)fs, leader);
  fl = (uint32_t)__shfl((int)fl, leader);
  const uint32_t pos = front ? fs + (uint32_t)__builtin_popcountll(sm & below)
                             : count - 1u - (fl + (uint32_t)__builtin_popcountll(act & ~sm & below));
#pragma unroll
  for (int q = 0; q < kPrepHsInt4; q++)
    prep2[(size_t)q * stride + pos] = make_int4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
}

// Digits of the recoded c / |d| straight from the hand-off (one dword per eight windows).
// Lanes past count read all-zero digits (0x88888888): their hand-off positions hold a previous
// batch's recodings, whose top digit (hs_top_digit) could leave [-8, 8] at this wave's W and
// index past the lane's table rows.
struct HsDigitsDev {
  const int4 *p2;
  uint32_t stride, slot;
  bool active;
  __device__ __forceinline__ uint32_t word(int w) const {
    return active ? reinterpret_cast<const uint32_t *>(p2 + (size_t)(w >> 2) * stride + slot)[w & 3] : 0x88888888u;
  }
  __device__ __forceinline__ uint32_t cword(int w) const { return word(w); }
  __device__ __forceinline__ uint32_t dword(int w) const { return w < 5 ? word(8 + w) : 0x88888888u; }
};

// Phase 2: tables of -A and -sign(d) R in the slab (two lane-major regions), the 3-point
// Straus sum over the wave's largest window count, B digits from windows 0 and 8 of the
// radix-2^16 comb (each entry fetched into LDS 16 doublings ahead), identity test.  Every
// lane of the grid stays to the end (the wave maximum of W is a shuffle reduction); lanes
// past count run on the identity and store nothing.
#ifndef TMED_HS_WAVES
#define TMED_HS_WAVES 2  // waves per SIMD of the half-size main kernel (248 VGPRs at 2)
#endif
// BB: radix of the B windows — 26 (the default: btab, two 2^25-entry tables, ten B additions) or
// 16 (windows 0 and 8 of the 2^16 comb, sixteen; when the 8.6-GB tables are unavailable).  The
// hand-off carries e unrecoded (hs_prep_r raw_e); radix 16 recodes it here.
template <int BB>
__global__ __launch_bounds__(kHsBlock, TMED_HS_WAVES) void verify_main_hs_kernel(
    uint32_t base, uint32_t count, const int4 *__restrict__ prep, const int4 *__restrict__ prep2, uint32_t stride,
    int4 *__restrict__ slab, const int4 *__restrict__ btab, uint8_t *__restrict__ out, int zip215) {
  __shared__ int4 sbl[kHsBlock / 64][8 * 64];
#if TMED_B16_ONEBUF
  auto &sbh = sbl;
#else
  __shared__ int4 sbh[kHsBlock / 64][8 * 64];
#endif
  const uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x;  // position in the placed hand-off
  const bool active = slot < count;
  int32_t w[64];
#pragma unroll
  for (int q = 3; q < kPrepHsInt4; q++) {  // e, R, flags, the signature's slot, A (words 12..63)
    const int4 v = active ? prep2[(size_t)q * stride + slot] : make_int4(0, 0, 0, 0);
    w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
  }
  uint32_t er[8];
#pragma unroll
  for (int j = 0; j < 8; j++) er[j] = (uint32_t)w[13 + j];
  if (BB == 16) {
    uint32_t e[8];
#pragma unroll
    for (int j = 0; j < 8; j++) e[j] = er[j];
    sc_recode_b<16>(er, e);
  }
  fe Rx, Ry;
#pragma unroll
  for (int j = 0; j < 10; j++) { Rx.v[j] = w[21 + j]; Ry.v[j] = w[31 + j]; }
  ge_p3 A;
#pragma unroll
  for (int j = 0; j < 10; j++) { A.X.v[j] = w[44 + j]; A.Y.v[j] = w[54 + j]; }
  if (!active) { fe_1(A.Y); fe_1(Ry); }
  fe_1(A.Z);
  fe_mul(A.T, A.X, A.Y);
  const int flags = w[41];
  int W = active ? (flags >> 8) : 29;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int x = __shfl_xor(W, o);
    W = x > W ? x : W;
  }
  W = __builtin_amdgcn_readfirstlane(W);
  if (W < 29) W = 29;
  if (W > 64) W = 64;
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const HsDigitsDev ds{prep2, stride, slot, active};
  SlabTab ta{slab, slot};
  SlabTab tr{slab + (size_t)stride * 64, slot};
  // the high table: the second radix-2^26 table, or window 8 (j * 2^128 B) of the 2^16 comb
  const size_t hi = BB == 26 ? (size_t)kB26Entries * kCombEntryInt4 : (size_t)8 * kB16Entries * kCombEntryInt4;
  BPf<BB> bl{btab, sbl[wv], lane};
  BPf<BB> bh{btab + hi, sbh[wv], lane};
  const bool id = verify_main_hs(ds, (flags & 2) != 0, er, W, A, Rx, Ry, ta, tr, bl, bh, zip215 != 0);
  if (active) out[base + (uint32_t)w[42]] = ((flags & 1) && id) ? 1 : 0;
}

// Diagnostics (tmed_window_stats): the lattice step's window count W of every lane of the last
// half-size chunk (hand-off flags, bits 8..), as a per-lane histogram and a histogram of the
// wave maxima — the loop length each wave of verify_main_hs_kernel actually ran (W = 64: the
// (k, 1) fallback).  Same 64-slot waves as the main kernel.
__global__ __launch_bounds__(kThreadsPerBlock) void window_stats_kernel(const int4 *__restrict__ prep2, uint32_t stride,
                                                                       uint32_t count, uint32_t *__restrict__ lane_hist,
                                                                       uint32_t *__restrict__ wave_hist) {
  __shared__ uint32_t lh[65], wh[65];  // block-local histograms, one global atomic per bin per block
  for (uint32_t b = threadIdx.x; b < 65; b += blockDim.x) lh[b] = wh[b] = 0;
  __syncthreads();
  const uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x;
  const bool active = slot < count;
  int W = active ? (prep2[(size_t)10 * stride + slot].y >> 8) : 0;  // word 41
  if (W < 0 || W > 64) W = 64;
  if (active) atomicAdd(&lh[W], 1u);
  int m = W;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int x = __shfl_xor(m, o);
    m = x > m ? x : m;
  }
  if ((threadIdx.x & 63u) == 0 && slot < count) atomicAdd(&wh[m], 1u);
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < 65; b += blockDim.x) {
    if (lh[b]) atomicAdd(&lane_hist[b], lh[b]);
    if (wh[b]) atomicAdd(&wave_hist[b], wh[b]);
  }
}

// (s_sleep 127 is ~8k clocks, ~3.4 us at 2.4 GHz; a bounded loop, no memory access)
__global__ __launch_bounds__(64) void test_delay_kernel(uint32_t iters) {
  for (uint32_t i = 0; i < iters; i++) __builtin_amdgcn_s_sleep(127);
}

hipError_t launch_test_delay(hipStream_t stream, uint32_t us) {
  if (us == 0) return hipSuccess;
  hipLaunchKernelGGL(test_delay_kernel, dim3(1), dim3(64), 0, stream, (us < 100000u ? us : 100000u) / 3u + 1u);
  return hipGetLastError();
}

hipError_t launch_window_stats(const int4 *prep, uint32_t stride, uint32_t count, uint32_t *d_hist,
                               hipStream_t stream) {
  if (count == 0) return hipSuccess;
  hipError_t e = hipMemsetAsync(d_hist, 0, 2 * 65 * sizeof(uint32_t), stream);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(window_stats_kernel, dim3((count + kThreadsPerBlock - 1) / kThreadsPerBlock),
                     dim3(kThreadsPerBlock), 0, stream, prep + (size_t)kPrepInt4 * stride, stride, count, d_hist,
                     d_hist + 65);
  return hipGetLastError();
}

// Phase 3: batched finish.  Lane l owns slots l, l + L, l + 2L, ... (< m) of the block of m
// signatures starting at fin_base (coalesced [q][slot] loads); finish_group inverts their
// Z with one inversion and compares each canonical encoding with R.
struct FinDev {
  const int4 *fin;
  int4 *pre;
  const uint8_t *sig;
  uint8_t *out;
  uint32_t fin_base, lane, L, m;
  const uint32_t *perm;  // position -> signature index (key-grouped order), or null
  __device__ __forceinline__ int count() const { return lane < m ? (int)((m - lane + L - 1) / L) : 0; }
  __device__ __forceinline__ uint32_t slot(int j) const { return lane + (uint32_t)j * L; }
  __device__ __forceinline__ void load_z(int j, fe &z) const {
    int32_t w[12];  // words 20..31
#pragma unroll
    for (int q = 0; q < 3; q++) {
      const int4 v = fin[(size_t)(5 + q) * kFinCap + slot(j)];
      w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
    }
#pragma unroll
    for (int i = 0; i < 10; i++) z.v[i] = w[i];
  }
  __device__ __forceinline__ void load_xy(int j, fe &X, fe &Y) const {
    int32_t w[20];  // words 0..19
#pragma unroll
    for (int q = 0; q < 5; q++) {
      const int4 v = fin[(size_t)q * kFinCap + slot(j)];
      w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
    }
#pragma unroll
    for (int i = 0; i < 10; i++) { X.v[i] = w[i]; Y.v[i] = w[10 + i]; }
  }
  __device__ __forceinline__ void store_pre(int j, const fe &p) const {
    const size_t idx = (size_t)j * L + lane;
    pre[idx] = make_int4(p.v[0], p.v[1], p.v[2], p.v[3]);
    pre[kFinPreStride + idx] = make_int4(p.v[4], p.v[5], p.v[6], p.v[7]);
    pre[2 * (size_t)kFinPreStride + idx] = make_int4(p.v[8], p.v[9], 0, 0);
  }
  __device__ __forceinline__ void load_pre(int j, fe &p) const {
    const size_t idx = (size_t)j * L + lane;
    const int4 a = pre[idx], b = pre[kFinPreStride + idx], c = pre[2 * (size_t)kFinPreStride + idx];
    p.v[0] = a.x; p.v[1] = a.y; p.v[2] = a.z; p.v[3] = a.w;
    p.v[4] = b.x; p.v[5] = b.y; p.v[6] = b.z; p.v[7] = b.w;
    p.v[8] = c.x; p.v[9] = c.y;
  }
  __device__ __forceinline__ uint32_t sig_index(int j) const {
    const uint32_t p = fin_base + slot(j);
    return perm ? perm[p] : p;
  }
  __device__ __forceinline__ void load_r(int j, uint32_t Rw[8]) const {
    load_row_words(Rw, sig + 64 * (size_t)sig_index(j), 2);
  }
  __device__ __forceinline__ void result(int j, bool ok) const {
    uint8_t *o = out + sig_index(j);
    *o = (*o && ok) ? 1 : 0;
  }
};

__global__ __launch_bounds__(kThreadsPerBlock) void verify_finish_kernel(
    const int4 *__restrict__ fin, int4 *__restrict__ pre, const uint8_t *__restrict__ sig, uint8_t *__restrict__ out,
    uint32_t fin_base, uint32_t L, uint32_t m, const uint32_t *__restrict__ perm) {
  const uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x;
  if (lane >= L) return;
  FinDev a{fin, pre, sig, out, fin_base, lane, L, m, perm};
  finish_group(a);
}

// Finish launch for the m signatures at fin_base: group size G = ceil(m / 65536) clamped to
// [1, 16], so at most 65,536 lanes = one wave per SIMD: each lane pays one inversion per group,
// a latency-bound chain, and a SIMD holding two such waves runs them ~twice as long (a C4 batch of
// ~853k votes took 13 per group = 1,025 waves with the floor: C4 585 -> 591 M/s, profiles/r05/s17/).
hipError_t launch_finish(const int4 *fin, int4 *pre, const uint8_t *sig, uint8_t *out, uint32_t fin_base, uint32_t m,
                         hipStream_t stream, const uint32_t *perm = nullptr) {
  if (m == 0) return hipSuccess;
  constexpr uint32_t kLanes = 65536;  // one inversion per lane and group; 65,536 lanes fill every SIMD
  uint32_t G = (m + kLanes - 1) / kLanes;
  if (G < 1) G = 1;
  if (G > kFinGroupMax) G = kFinGroupMax;
  const uint32_t L = (m + G - 1) / G;
  hipLaunchKernelGGL(verify_finish_kernel, dim3((L + kThreadsPerBlock - 1) / kThreadsPerBlock),
                     dim3(kThreadsPerBlock), 0, stream, fin, pre, sig, out, fin_base, L, m, perm);
  return hipGetLastError();
}

struct GlobalComb;  // defined with the key-set kernels below
__device__ void comb_sign_one(uint32_t sg[16], uint32_t pb[8], const uint32_t seed[8], const uint8_t *m,
                              uint32_t mlen, const int4 *bcomb);

// RFC 8032 signer for synthetic commits: [a]B and [r]B from the shared comb of B.
__global__ __launch_bounds__(kThreadsPerBlock) void sign_kernel(
    const uint8_t *__restrict__ seeds, const uint8_t *__restrict__ msgs, const uint32_t *__restrict__ off,
    uint32_t n, uint8_t *__restrict__ sig_out, uint8_t *__restrict__ pub_out, const int4 *__restrict__ bcomb) {
  const uint32_t gtid = blockIdx.x * blockDim.x + threadIdx.x;
  for (uint32_t i = gtid; i < n; i += gridDim.x * blockDim.x) {
    uint32_t seed[8], sg[16], pb[8];
    load_row_words(seed, seeds + 32 * (size_t)i, 2);
    const uint32_t o0 = off[i], o1 = off[i + 1];
    comb_sign_one(sg, pb, seed, msgs + o0, o1 - o0, bcomb);
    uint4 *so = reinterpret_cast<uint4 *>(sig_out + 64 * (size_t)i);
#pragma unroll
    for (int q = 0; q < 4; q++) so[q] = make_uint4(sg[4 * q], sg[4 * q + 1], sg[4 * q + 2], sg[4 * q + 3]);
    uint4 *po = reinterpret_cast<uint4 *>(pub_out + 32 * (size_t)i);
#pragma unroll
    for (int q = 0; q < 2; q++) po[q] = make_uint4(pb[4 * q], pb[4 * q + 1], pb[4 * q + 2], pb[4 * q + 3]);
  }
}

uint32_t grid_for(size_t n, uint32_t max_blocks) {
  size_t b = (n + kThreadsPerBlock - 1) / kThreadsPerBlock;
  if (b > max_blocks) b = max_blocks;
  if (b == 0) b = 1;
  return (uint32_t)b;
}

hipError_t launch_verify(const uint8_t *pub, const uint8_t *sig, const uint8_t *msgs, const uint32_t *off,
                         uint32_t n, uint8_t *out, int4 *slab, uint32_t slab_stride, BTabs btab,
                         int4 *prep, int4 *fin, int4 *fin_pre, hipStream_t stream, uint32_t chunk, int main_waves,
                         bool msg_slots, KernelTimer *timer, bool zip215) {
  const MsgSrc ms{msgs, off, msg_slots};
  // Chunks of at most slab_stride signatures (the per-lane tables and the prep hand-off are
  // sized for one chunk; tmed_init keeps both multiples of kThreadsPerBlock, so every lane of
  // every launched block owns a slot below slab_stride).  The finish (variant 5 only) runs
  // once per kFinCap block.
  if (chunk == 0 || chunk > slab_stride) chunk = slab_stride;
  if (chunk % kThreadsPerBlock != 0 || slab_stride % kThreadsPerBlock != 0) return hipErrorInvalidValue;
  const bool hs = main_waves != 5 || zip215;  // the ZIP-215 rule runs on the half-size path only
  // placement counters of the half-size hand-off: the tail of the prep allocation (kPrepTailBytes)
  uint32_t *place = reinterpret_cast<uint32_t *>(reinterpret_cast<char *>(prep) + (size_t)slab_stride * kPrepSlotBytes);
  if (timer) timer->mark(stream, -1);
  for (uint32_t fbase = 0; fbase < n; fbase += kFinCap) {
    const uint32_t m = (n - fbase) < kFinCap ? (n - fbase) : kFinCap;
    for (uint32_t base = fbase; base < fbase + m; base += chunk) {
      const uint32_t count = (fbase + m - base) < chunk ? (fbase + m - base) : chunk;
      const uint32_t blocks = (count + kThreadsPerBlock - 1) / kThreadsPerBlock;
      const uint32_t hblocks = (count + kHsBlock - 1) / kHsBlock;

      hipLaunchKernelGGL(verify_prep_kernel, dim3(hblocks), dim3(kHsBlock), 0, stream, pub, sig, ms, base,
                         count, prep, slab_stride, hs ? place : nullptr);
      if (timer) timer->mark(stream, 0);
      if (hs) {  // default: half-size scalars (verify_hs.h): R decode + lattice, main; no finish
        int4 *prep2 = prep + (size_t)kPrepInt4 * slab_stride;
        hipLaunchKernelGGL(verify_prep_r_kernel, dim3(hblocks), dim3(kHsBlock), 0, stream, sig, base, count,
                           prep, prep2, slab_stride, place, zip215 ? 1 : 0);
        if (timer) timer->mark(stream, 0);
        if (btab.b26)
          hipLaunchKernelGGL(verify_main_hs_kernel<26>, dim3(hblocks), dim3(kHsBlock), 0, stream, base, count,
                             prep, prep2, slab_stride, slab, btab.b26, out, zip215 ? 1 : 0);
        else
          hipLaunchKernelGGL(verify_main_hs_kernel<16>, dim3(hblocks), dim3(kHsBlock), 0, stream, base, count,
                             prep, prep2, slab_stride, slab, btab.comb16, out, zip215 ? 1 : 0);
      } else {  // fallback 5: full-length Straus + batched finish
        hipLaunchKernelGGL(verify_main_kernel, dim3(blocks), dim3(kThreadsPerBlock), 0, stream, base, count, prep,
                           slab_stride, slab, btab.b16, fin, fbase, out);
      }
      if (timer) timer->mark(stream, 1);
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
    }
    hipError_t e = hs ? hipSuccess : launch_finish(fin, fin_pre, sig, out, fbase, m, stream);
    if (timer) timer->mark(stream, 2);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_verify_prep(const uint8_t *pub, const uint8_t *sig, const uint8_t *msgs, const uint32_t *off,
                              bool msg_slots, uint32_t base, uint32_t count, int4 *prep, uint32_t stride,
                              hipStream_t stream) {
  if (count == 0) return hipSuccess;
  if (count > stride) return hipErrorInvalidValue;
  const MsgSrc ms{msgs, off, msg_slots};
  hipLaunchKernelGGL(verify_prep_kernel, dim3((count + kHsBlock - 1) / kHsBlock),
                     dim3(kHsBlock), 0, stream, pub, sig, ms, base, count, prep, stride, nullptr);
  return hipGetLastError();
}

hipError_t launch_sign(const uint8_t *seeds, const uint8_t *msgs, const uint32_t *off, uint32_t n, uint8_t *sig_out,
                       uint8_t *pub_out, const int4 *bcomb, hipStream_t stream) {
  const uint32_t grid = grid_for(n, 4096);
  hipLaunchKernelGGL(sign_kernel, dim3(grid), dim3(kThreadsPerBlock), 0, stream, seeds, msgs, off, n, sig_out,
                     pub_out, bcomb);
  return hipGetLastError();
}

// j*B for j = 0..kB16Entries-1 into 128-B rows (one lane per entry; once per context).
__global__ __launch_bounds__(256) void b16_fill_kernel(int4 *__restrict__ tab) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= kB16Entries) return;
  ge_niels e;
  if (j == 0) {
    ge_niels_0(e);
  } else {
    ge_p3 B;
    ge_base_point(B);
    comb_entry(e, B, j, 16);
  }
  const fe *fs[3] = {&e.YpX, &e.YmX, &e.XY2d};
#pragma unroll
  for (int q = 0; q < 8; q++) {
    int32_t w[4];
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const int f = 4 * q + c;
      w[c] = f < 30 ? fs[f / 10]->v[f % 10] : 0;
    }
    tab[(size_t)j * 8 + q] = make_int4(w[0], w[1], w[2], w[3]);
  }
}

hipError_t launch_build_b16(int4 *tab, hipStream_t stream) {
  hipLaunchKernelGGL(b16_fill_kernel, dim3((kB16Entries + 255) / 256), dim3(256), 0, stream, tab);
  return hipGetLastError();
}

// ============================================================ fixed-base combs

__device__ __forceinline__ void p3_store(int32_t *dst, const ge_p3 &p) {
  const fe *fs[4] = {&p.X, &p.Y, &p.Z, &p.T};
#pragma unroll
  for (int f = 0; f < 40; f++) dst[f] = fs[f / 10]->v[f % 10];
}
__device__ __forceinline__ void p3_load(ge_p3 &p, const int32_t *src) {
  fe *fs[4] = {&p.X, &p.Y, &p.Z, &p.T};
#pragma unroll
  for (int f = 0; f < 40; f++) fs[f / 10]->v[f % 10] = src[f];
}

__global__ __launch_bounds__(64) void comb_bases_kernel(const uint8_t *__restrict__ pubs, uint32_t n, int negate,
                                                       uint8_t *__restrict__ ok_out, int32_t *__restrict__ bases) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t pw[8];
  load_row_words(pw, pubs + 32 * (size_t)i, 2);
  ge_p3 P;
  const bool ok = ge_frombytes_go(P, pw);
  ok_out[i] = ok ? 1 : 0;
  if (negate) { fe_neg(P.X, P.X); fe_neg(P.T, P.T); }
#pragma unroll 1
  for (int w = 0; w < kCombWindows; w++) {
    p3_store(bases + ((size_t)i * kCombWindows + w) * 40, P);
    ge_mul256(P);
  }
}

__device__ __forceinline__ void niels_store(int4 *dst, const ge_niels &e) {
  const fe *fs[3] = {&e.YpX, &e.YmX, &e.XY2d};
#pragma unroll
  for (int q = 0; q < kCombEntryInt4; q++) {
    int32_t w[4];
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const int f = 4 * q + c;
      w[c] = f < 30 ? fs[f / 10]->v[f % 10] : 0;
    }
    dst[q] = make_int4(w[0], w[1], w[2], w[3]);
  }
}
__device__ __forceinline__ void niels_load(ge_niels &e, const int4 *src) {
  fe *fs[3] = {&e.YpX, &e.YmX, &e.XY2d};
#pragma unroll
  for (int q = 0; q < kCombEntryInt4; q++) {
    const int4 v = src[q];
    const int32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const int f = 4 * q + c;
      if (f < 30) fs[f / 10]->v[f % 10] = w[c];
    }
  }
}

// Comb entries in runs of kCombARun consecutive j per lane: the run's first entry j0 * base by
// double-and-add over nbits bits of j0, the next ones by one cached addition each (8 M), the run's
// projective points parked in their own comb rows (X, Y, Z: 30 of the row's 32 words) and their
// prefix products of Z in LDS, ONE inversion per run (Montgomery's trick: 3 M per entry), then
// each row rewritten in affine niels form.  ~6k mads per entry against ~34k for a double-and-add
// and an inversion per entry (the round-5 radix-2^12 comb of 10k keys: 1.6 s of device time that
// way, 98 ms like this — profiles/r05/final/ and s14/ kernel_stats.csv).
constexpr uint32_t kCombARun = 8;
__device__ __forceinline__ void row_store_xyz(int4 *row, const ge_p3 &P) {
  const fe *fs[3] = {&P.X, &P.Y, &P.Z};
#pragma unroll
  for (int q = 0; q < kCombEntryInt4; q++) {
    int32_t w[4];
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const int f = 4 * q + c;
      w[c] = f < 30 ? fs[f / 10]->v[f % 10] : 0;
    }
    row[q] = make_int4(w[0], w[1], w[2], w[3]);
  }
}
__device__ __forceinline__ void row_load_xyz(const int4 *row, fe &X, fe &Y, fe &Z) {
  fe *fs[3] = {&X, &Y, &Z};
#pragma unroll
  for (int q = 0; q < kCombEntryInt4; q++) {
    const int4 v = row[q];
    const int32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const int f = 4 * q + c;
      if (f < 30) fs[f / 10]->v[f % 10] = w[c];
    }
  }
}
// rows[j] = j * base for j = j0 .. j0 + kCombARun - 1 (rows: the window's entry 0; base: p3 words;
// pre: this block's LDS, 64 lanes)
__device__ __forceinline__ void comb_fill_run(int4 *rows, const int32_t *base, uint32_t j0, int nbits,
                              fe (*pre)[64], uint32_t lane) {
  ge_p3 B, P;
  p3_load(B, base);
  ge_cached cB;
  ge_p3_to_cached(cB, B);
  {  // P = j0 * B, double-and-add over j0's bits
    ge_p3 sum;
    ge_p1p1 t;
    ge_p2 q;
    ge_p3_0(P);
#pragma unroll 1
    for (int b = nbits - 1; b >= 0; b--) {
      ge_p3_to_p2(q, P);
      ge_p2_dbl(t, q);
      ge_p1p1_to_p3(P, t);
      ge_add_cached(t, P, cB, false);
      ge_p1p1_to_p3(sum, t);
      const bool bit = (j0 >> b) & 1u;
      fe_select(P.X, P.X, sum.X, bit);
      fe_select(P.Y, P.Y, sum.Y, bit);
      fe_select(P.Z, P.Z, sum.Z, bit);
      fe_select(P.T, P.T, sum.T, bit);
    }
  }
  fe acc;
#pragma unroll 1
  for (uint32_t t = 0; t < kCombARun; t++) {
    if (t) {
      ge_p1p1 s;
      ge_add_cached(s, P, cB, false);
      ge_p1p1_to_p3(P, s);
      fe_mul(acc, acc, P.Z);
    } else {
      fe_copy(acc, P.Z);
    }
    row_store_xyz(rows + (size_t)(j0 + t) * kCombEntryInt4, P);
    pre[t][lane] = acc;
  }
  fe inv, d2;
  fe_invert_bgcd(inv, acc);
  fe_const_d2(d2);
#pragma unroll 1
  for (int t = (int)kCombARun - 1; t >= 0; t--) {
    int4 *r = rows + (size_t)(j0 + t) * kCombEntryInt4;
    fe X, Y, Z, zi, x, y, xy;
    row_load_xyz(r, X, Y, Z);
    if (t) {
      fe_mul(zi, inv, pre[t - 1][lane]);
      fe_mul(inv, inv, Z);
    } else {
      fe_copy(zi, inv);
    }
    fe_mul_x2(x, X, zi, y, Y, zi);
    ge_niels e;
    fe_add(e.YpX, y, x); fe_carry(e.YpX, e.YpX);
    fe_sub(e.YmX, y, x); fe_carry(e.YmX, e.YmX);
    fe_mul(xy, x, y);
    fe_mul(e.XY2d, xy, d2);
    niels_store(r, e);
  }
}
// the bit length of a run's largest start 1 + kCombARun (runs - 1)
constexpr int comb_start_bits(uint32_t runs) {
  int b = 0;
  for (uint32_t v = 1 + kCombARun * (runs - 1); v; v >>= 1) b++;
  return b;
}

// The radix-256 comb: 16 runs of 8 per (key, window) (j = 1..128), four windows per 64-lane block.
constexpr uint32_t kCombRuns = (kCombEntries - 1) / kCombARun;  // 16
static_assert((kCombEntries - 1) % kCombARun == 0 && 64 % kCombRuns == 0, "radix-256 comb runs");
__global__ __launch_bounds__(64) void comb_fill_kernel(const int32_t *__restrict__ bases, uint32_t n,
                                                       int4 *__restrict__ comb) {
  __shared__ fe pre[kCombARun][64];
  const uint32_t kw = blockIdx.x * (64 / kCombRuns) + threadIdx.x / kCombRuns;  // key * 32 + window
  const uint32_t run = threadIdx.x % kCombRuns;
  if (kw >= n * kCombWindows) return;
  int4 *rows = comb + (size_t)kw * kCombEntries * kCombEntryInt4;
  if (run == 0) {
    ge_niels id;
    ge_niels_0(id);
    niels_store(rows, id);
  }
  comb_fill_run(rows, bases + (size_t)kw * 40, 1u + kCombARun * run, comb_start_bits(kCombRuns), pre, threadIdx.x);
}

struct GlobalComb {
  static constexpr int kBits = 8;
  const int4 *base;  // 32 windows x 129 entries x 8 int4
  __device__ __forceinline__ void load(int w, int j, ge_niels &e) const {
    niels_load(e, base + ((size_t)w * kCombEntries + j) * kCombEntryInt4);
  }
};

// Radix-2^16 comb of +B for the key-cached throughput kernel: 16 windows x 32769 entries
// (j * 2^(16w) * B) x 8 int4 = 67 MB in HBM, built once per context.
struct GlobalComb16 {
  static constexpr int kBits = 16;
  const int4 *base;
  __device__ __forceinline__ void load(int w, int j, ge_niels &e) const {
    niels_load(e, base + ((size_t)w * kB16Entries + j) * kCombEntryInt4);
  }
};

// Lane (w, j) of the radix-2^16 B comb: j * bases[w] (bases[w] = 2^(16w) B, p3 words).
__global__ __launch_bounds__(256) void bcomb16_fill_kernel(const int32_t *__restrict__ bases, int4 *__restrict__ comb) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= 16u * kB16Entries) return;
  const uint32_t w = g / kB16Entries, j = g % kB16Entries;
  ge_niels e;
  if (j == 0) {
    ge_niels_0(e);
  } else {
    ge_p3 P;
    p3_load(P, bases + (size_t)w * 40);
    comb_entry(e, P, j, 16);
  }
  niels_store(comb + (size_t)g * kCombEntryInt4, e);
}

void host_bcomb16_bases(int32_t out[16 * 40]) {
  ge_p3 P;
  ge_base_point(P);
  for (int w = 0; w < 16; w++) {
    const fe *fs[4] = {&P.X, &P.Y, &P.Z, &P.T};
    for (int f = 0; f < 40; f++) out[w * 40 + f] = fs[f / 10]->v[f % 10];
    ge_mul256(P);
    ge_mul256(P);
  }
}

hipError_t launch_build_bcomb16(const int32_t *d_bases, int4 *comb, hipStream_t stream) {
  hipLaunchKernelGGL(bcomb16_fill_kernel, dim3((16u * kB16Entries + 255) / 256), dim3(256), 0, stream, d_bases, comb);
  return hipGetLastError();
}

// Entry (t, j) of the radix-2^26 B tables: j * 2^(128 t) B for j = 0..2^25 (t = 0, 1), from
// windows 8t and 8t + 1 of the radix-2^16 comb (j = d0 + 2^16 d1, d0 signed: two mixed
// additions), then affine niels with one inversion (per entry: ~15k mads, 2^26 entries, once
// per device).
__global__ __launch_bounds__(256) void b26_fill_kernel(const int4 *__restrict__ comb16, int4 *__restrict__ tab) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= 2u * kB26Entries) return;
  const uint32_t t = g / kB26Entries, j = g % kB26Entries;
  ge_niels e;
  if (j == 0) {
    ge_niels_0(e);
  } else {
    int d0 = (int)(j & 0xffffu);
    uint32_t d1 = j >> 16;
    if (d0 >= 32768) { d0 -= 65536; d1++; }
    const GlobalComb16 bc{comb16};
    ge_p3 P;
    ge_p1p1 q;
    ge_niels n;
    ge_p3_0(P);
    bc.load(8 * (int)t, d0 < 0 ? -d0 : d0, n);
    niels_apply_sign(n, d0 < 0);
    ge_madd_niels(q, P, n, false);
    ge_p1p1_to_p3(P, q);
    bc.load(8 * (int)t + 1, (int)d1, n);
    ge_madd_niels(q, P, n, false);
    ge_p1p1_to_p3(P, q);
    ge_p3_to_niels(e, P);
  }
  niels_store(tab + (size_t)g * kCombEntryInt4, e);
}

hipError_t launch_build_b26(const int4 *comb16, int4 *tab, hipStream_t stream) {
  hipLaunchKernelGGL(b26_fill_kernel, dim3((2u * kB26Entries + 255) / 256), dim3(256), 0, stream, comb16, tab);
  return hipGetLastError();
}

// Entry (w, j) of the radix-2^24 comb: j * 2^(24w) B for j = 0..2^23.  24w = 16v + r (r = 0 or 8):
// J = j 2^r < 2^31 as two signed 16-bit digits at windows v, v + 1 of the radix-2^16 comb (two mixed
// additions), then affine niels with one inversion.  Window 10 (bits 240..263) only ever needs
// j <= 2^16 (S < 2^256); its entries whose second digit would fall past the comb's last window are
// left as the identity.
__global__ __launch_bounds__(256) void b24_fill_kernel(const int4 *__restrict__ comb16, int4 *__restrict__ tab) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= (uint32_t)kB24Windows * kB24Entries) return;
  const uint32_t w = g / kB24Entries, j = g % kB24Entries;
  const uint32_t v = (24u * w) >> 4, r = (24u * w) & 15u;
  const uint32_t J = j << r;
  int d0 = (int)(J & 0xffffu);
  uint32_t d1 = J >> 16;
  if (d0 >= 32768) { d0 -= 65536; d1++; }
  ge_niels e;
  if (j == 0 || (v + 1 >= 16 && d1 != 0)) {
    ge_niels_0(e);
  } else {
    const GlobalComb16 bc{comb16};
    ge_p3 P;
    ge_p1p1 q;
    ge_niels n;
    ge_p3_0(P);
    bc.load((int)v, d0 < 0 ? -d0 : d0, n);
    niels_apply_sign(n, d0 < 0);
    ge_madd_niels(q, P, n, false);
    ge_p1p1_to_p3(P, q);
    if (d1) {
      bc.load((int)v + 1, (int)d1, n);
      ge_madd_niels(q, P, n, false);
      ge_p1p1_to_p3(P, q);
    }
    ge_p3_to_niels(e, P);
  }
  niels_store(tab + (size_t)g * kCombEntryInt4, e);
}

hipError_t launch_build_b24(const int4 *comb16, int4 *tab, hipStream_t stream) {
  const uint32_t n = (uint32_t)kB24Windows * kB24Entries;
  hipLaunchKernelGGL(b24_fill_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, comb16, tab);
  return hipGetLastError();
}

__device__ void comb_sign_one(uint32_t sg[16], uint32_t pb[8], const uint32_t seed[8], const uint8_t *m,
                              uint32_t mlen, const int4 *bcomb) {
  const GlobalComb bc{bcomb};
  sign_one_bm(sg, pb, seed, m, mlen, [&](uint32_t enc[8], const uint32_t s[8]) { comb_base_mult(enc, s, bc); });
}

#ifndef TMED_KS_PREP_WAVES
#define TMED_KS_PREP_WAVES 4  // 128 VGPRs, 4 spilled: keyed prep 0.347 -> 0.337 ms per 2^20 against 3 waves
                              // (130 VGPRs), three alternating runs each (profiles/r04/s22)
#endif
__global__ __launch_bounds__(kThreadsPerBlock, TMED_KS_PREP_WAVES) void verify_keyset_prep_kernel(
    const uint32_t *__restrict__ val_idx, uint32_t nkeys, const uint8_t *__restrict__ key_pub,
    const uint8_t *__restrict__ key_ok, const uint8_t *__restrict__ sig, MsgSrc ms, uint32_t base, uint32_t count,
    int4 *__restrict__ prep, uint32_t stride) {
  const uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x;
  if (slot >= count) return;
  const uint32_t i = base + slot;
  const uint32_t vi = val_idx[i];
  const bool vin = vi < nkeys;  // an index past the key set rejects the signature (row 0 is read)
  const uint32_t v = vin ? vi : 0u;
  uint32_t pw[8], sw[16], k[8], s[8];
  load_row_words(pw, key_pub + 32 * (size_t)v, 2);
  load_row_words(sw, sig + 64 * (size_t)i, 4);
  const uint8_t *m;
  uint32_t mlen;
  ms.get(i, m, mlen);
  const bool ok = verify_prep_comb(pw, vin && key_ok[v] != 0, sw, m, mlen, k, s, ms.slots);  // slots: hashed from dwordx4 loads (sha512_stream_slot)
  prep_store_ks(prep, stride, slot, k, s, ok);
}

// Key-cached Straus with the next comb row in flight (TMED_KS_PF): the 48 rows a signature
// reads (32 from its key's radix-256 comb, 16 from the shared radix-2^16 comb of B) are random
// 128-B lines of a multi-GB table, so a row loaded right before its addition leaves the wave
// parked on HBM latency for most of it (rocprof: 0.35 of the mad peak, round 2).  Here the row
// of addition t+1 is loaded into registers before addition t runs.  Schedule per 32-bit word q
// of the recodings: A(4q), A(4q+1), B(2q), A(4q+2), A(4q+3), B(2q+1) — the same sum as
// verify_main_comb_point<16>.  The first addition starts from the identity, so it is replaced
// by the niels -> extended conversion (1 M instead of 7 M), and the last one stops at
// projective (X, Y, Z) (3 M instead of 4 M for p1p1 -> p3).
#ifndef TMED_KS_PF
#define TMED_KS_PF 1
#endif
#ifndef TMED_KS_ROLL
#define TMED_KS_ROLL 0  // 1: one addition per loop iteration (A/B of the loop body's code size)
#endif
struct CombRowPf {
  int4 pv[8];
  bool neg;
  __device__ __forceinline__ void fetch(const int4 *row, bool n) {
#pragma unroll
    for (int q = 0; q < 8; q++) pv[q] = row[q];
    neg = n;
  }
  __device__ __forceinline__ void take(ge_niels &e) const {
    fe *fs[3] = {&e.YpX, &e.YmX, &e.XY2d};
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const int32_t w[4] = {pv[q].x, pv[q].y, pv[q].z, pv[q].w};
#pragma unroll
      for (int c = 0; c < 4; c++) {
        const int f = 4 * q + c;
        if (f < 30) fs[f / 10]->v[f % 10] = w[c];
      }
    }
    niels_apply_sign(e, neg);
  }
};

// (x, y) affine niels (y+x, y-x, 2dxy) -> extended (4x : 4y : 4 : 4xy): X = 2(a - b), Y = 2(a + b),
// T = (a - b)(a + b) with a = y+x, b = y-x.
__device__ __forceinline__ void ge_niels_to_p3(ge_p3 &r, const ge_niels &e) {
  fe d, s;
  fe_sub(d, e.YpX, e.YmX);
  fe_add(s, e.YpX, e.YmX);
  fe_mul(r.T, d, s);
  fe_add(r.X, d, d);
  fe_carry(r.X, r.X);  // the next addition's Y +- X must stay a 3-sum of carried values
  fe_add(r.Y, s, s);
  fe_carry(r.Y, r.Y);
  fe_0(r.Z);
  r.Z.v[0] = 4;
}

__device__ __forceinline__ const int4 *ks_arow(const int4 *ak, int w, uint32_t byte, bool &neg) {
  const int d = (int)byte - 128;
  neg = d < 0;
  return ak + ((size_t)w * kCombEntries + (uint32_t)(neg ? -d : d)) * kCombEntryInt4;
}
__device__ __forceinline__ const int4 *ks_brow(const int4 *bc, int wb, uint32_t half, bool &neg) {
  const int d = (int)half - 32768;
  neg = d < 0;
  return bc + ((size_t)wb * kB16Entries + (uint32_t)(neg ? -d : d)) * kCombEntryInt4;
}

// out (X : Y : Z) = [k](-A) + [s]B from the key's comb (ak) and the radix-2^16 comb of B (bc).
__device__ __forceinline__ void keyset_straus_pf(ge_p2 &out, const uint32_t k[8], const uint32_t s[8],
                                                 const int4 *ak, const int4 *bc) {
  uint32_t kr[8], sr[8];
  sc_recode256(kr, k);
  sc_recode_b<16>(sr, s);
  CombRowPf pf;
  bool ng;
  pf.fetch(ks_arow(ak, 0, kr[0] & 0xffu, ng), ng);
  ge_p3 acc;
  ge_p1p1 t;
  ge_niels e;
#if TMED_KS_ROLL
  // one addition per iteration (small loop body); the step's role comes from uniform branches
  uint32_t kc = kr[0], sc = sr[0];
#pragma unroll 1
  for (int tt = 0; tt < 48; tt++) {
    const int q = tt / 6, st = tt - 6 * (tt / 6);
    pf.take(e);
    const int nx = st + 1;
    if (nx == 6) {
#pragma unroll
      for (int m = 0; m < 7; m++) { kr[m] = kr[m + 1]; sr[m] = sr[m + 1]; }
      kc = kr[0];
      sc = sr[0];
    }
    const int4 *row;
    if (nx == 6) {
      row = ks_arow(ak, 4 * q + 4 < 32 ? 4 * q + 4 : 0, kc & 0xffu, ng);
    } else if (nx == 2 || nx == 5) {
      row = ks_brow(bc, 2 * q + (nx == 5), (sc >> (nx == 5 ? 16 : 0)) & 0xffffu, ng);
    } else {
      const int b = nx < 2 ? nx : nx - 1;
      row = ks_arow(ak, 4 * q + b, (kc >> (8 * b)) & 0xffu, ng);
    }
    if (tt < 47) pf.fetch(row, ng);
    if (tt == 0) {
      ge_niels_to_p3(acc, e);
    } else {
      ge_madd_niels(t, acc, e, false);
      if (tt == 47) ge_p1p1_to_p2(out, t);
      else ge_p1p1_to_p3(acc, t);
    }
  }
  return;
#endif
#pragma unroll 1
  for (int q = 0; q < 8; q++) {
    const uint32_t kc = kr[0], sc = sr[0];
#pragma unroll
    for (int m = 0; m < 7; m++) { kr[m] = kr[m + 1]; sr[m] = sr[m + 1]; }
#pragma unroll
    for (int st = 0; st < 6; st++) {
      pf.take(e);
      // the row of the next addition: A byte, A byte, B half, A, A, B, then the next word's A byte 0
      const int nx = st + 1;
      const int4 *row;
      if (nx == 6) {
        row = ks_arow(ak, 4 * q + 4 < 32 ? 4 * q + 4 : 0, kr[0] & 0xffu, ng);  // past the end: any row
      } else if (nx == 2 || nx == 5) {
        row = ks_brow(bc, 2 * q + (nx == 5), (sc >> (nx == 5 ? 16 : 0)) & 0xffffu, ng);
      } else {
        const int b = nx < 2 ? nx : nx - 1;  // byte of kc
        row = ks_arow(ak, 4 * q + b, (kc >> (8 * b)) & 0xffu, ng);
      }
      if (q < 7 || st < 5) pf.fetch(row, ng);
      if (st == 0 && q == 0) {
        ge_niels_to_p3(acc, e);
      } else {
        ge_madd_niels(t, acc, e, false);
        if (q == 7 && st == 5) {
          ge_p1p1_to_p2(out, t);
        } else {
          ge_p1p1_to_p3(acc, t);
        }
      }
    }
  }
}

// out (X : Y : Z) = [k](-A) + [s]B with the radix-2^24 comb of B: the key's 32 radix-256 rows, then
// eleven B rows, d_m = bits [24m, 24m + 24) of s + bit (24m - 1) - 2^24 bit (24m + 23), read off a
// copy of s shifted right by 24 bits per row (no carry chain); 43 mixed additions, the row of
// addition t + 1 loaded while addition t runs.
__device__ __forceinline__ const int4 *ks_b24row(const int4 *bc, int w, int d, bool &neg) {
  neg = d < 0;
  return bc + ((size_t)w * kB24Entries + (uint32_t)(neg ? -d : d)) * kCombEntryInt4;
}
__device__ __forceinline__ void keyset_straus_b24(ge_p2 &out, const uint32_t k[8], const uint32_t s[8],
                                                  const int4 *ak, const int4 *bc) {
  uint32_t kr[8], sw[8];
  sc_recode256(kr, k);
#pragma unroll
  for (int i = 0; i < 8; i++) sw[i] = s[i];
  CombRowPf pf;
  bool ng;
  pf.fetch(ks_arow(ak, 0, kr[0] & 0xffu, ng), ng);
  ge_p3 acc;
  ge_p1p1 t;
  ge_niels e;
  // the key's 32 rows, four per word of the recoding
#pragma unroll 1
  for (int q = 0; q < 8; q++) {
    const uint32_t kc = kr[0];
#pragma unroll
    for (int m = 0; m < 7; m++) kr[m] = kr[m + 1];
#pragma unroll
    for (int b = 0; b < 4; b++) {
      pf.take(e);
      if (b < 3) {
        pf.fetch(ks_arow(ak, 4 * q + b + 1, (kc >> (8 * (b + 1))) & 0xffu, ng), ng);
      } else if (q < 7) {
        pf.fetch(ks_arow(ak, 4 * q + 4, kr[0] & 0xffu, ng), ng);
      } else {  // the first B row: digit 0
        const uint32_t u = sw[0] & 0xffffffu;
        pf.fetch(ks_b24row(bc, 0, (int)u - (int)((u >> 23) << 24), ng), ng);
      }
      if (q == 0 && b == 0) {
        ge_niels_to_p3(acc, e);
      } else {
        ge_madd_niels(t, acc, e, false);
        ge_p1p1_to_p3(acc, t);
      }
    }
  }
  // the eleven B rows; row m + 1's digit is read off s shifted right by 24 (m + 1) bits
#pragma unroll 1
  for (int m = 0; m < kB24Windows; m++) {
    pf.take(e);
    if (m + 1 < kB24Windows) {
      const uint32_t below = (sw[0] >> 23) & 1u;  // bit 24(m + 1) - 1
#pragma unroll
      for (int i = 0; i < 7; i++) sw[i] = __builtin_amdgcn_alignbit(sw[i + 1], sw[i], 24);
      sw[7] >>= 24;
      const uint32_t u = sw[0] & 0xffffffu;
      pf.fetch(ks_b24row(bc, m + 1, (int)(u + below) - (int)((u >> 23) << 24), ng), ng);
    }
    ge_madd_niels(t, acc, e, false);
    if (m + 1 == kB24Windows) ge_p1p1_to_p2(out, t);
    else ge_p1p1_to_p3(acc, t);
  }
}

// The same sum with -A from its radix-2^B comb (kernels.h kCombA*, B = 12: 21 A rows), then the
// eleven B rows.  Digit m of k is read off k shifted right by Bm bits (bits [Bm, Bm + B) plus the
// bit below, minus 2^B times the top bit of the field; the top digit is every bit left, unsigned).
__device__ __forceinline__ const int4 *ks_arow(const int4 *ak, int w, int d, bool &neg) {
  neg = d < 0;
  return ak + comba_row(w, (uint32_t)(neg ? -d : d)) * kCombEntryInt4;
}
__device__ __forceinline__ void keyset_straus_ab24(ge_p2 &out, const uint32_t k[8], const uint32_t s[8],
                                                   const int4 *ak, const int4 *bc) {
  uint32_t kw[8], sw[8];
#pragma unroll
  for (int i = 0; i < 8; i++) { kw[i] = k[i]; sw[i] = s[i]; }
  CombRowPf pf;
  bool ng;
  constexpr uint32_t kMask = (1u << kCombABits) - 1u;
  {
    const uint32_t u = kw[0] & kMask;
    pf.fetch(ks_arow(ak, 0, (int)u - (int)((u >> (kCombABits - 1)) << kCombABits), ng), ng);
  }
  ge_p3 acc;
  ge_p1p1 t;
  ge_niels e;
#pragma unroll 1
  for (int m = 0; m < kCombAWindows; m++) {
    pf.take(e);
    if (m + 1 < kCombAWindows) {
      const uint32_t below = (kw[0] >> (kCombABits - 1)) & 1u;  // bit B(m + 1) - 1
#pragma unroll
      for (int i = 0; i < 7; i++) kw[i] = __builtin_amdgcn_alignbit(kw[i + 1], kw[i], kCombABits);
      kw[7] >>= kCombABits;
      // the top window's digit: every bit left (k < L: bits B(W-1)..252) + the bit below, unsigned
      const bool last = m + 2 == kCombAWindows;
      const uint32_t u = last ? kw[0] : kw[0] & kMask;
      const int top = last ? 0 : (int)((u >> (kCombABits - 1)) << kCombABits);
      pf.fetch(ks_arow(ak, m + 1, (int)(u + below) - top, ng), ng);
    } else {  // the first B row: digit 0
      const uint32_t u = sw[0] & 0xffffffu;
      pf.fetch(ks_b24row(bc, 0, (int)u - (int)((u >> 23) << 24), ng), ng);
    }
    if (m == 0) {
      ge_niels_to_p3(acc, e);
    } else {
      ge_madd_niels(t, acc, e, false);
      ge_p1p1_to_p3(acc, t);
    }
  }
#pragma unroll 1
  for (int m = 0; m < kB24Windows; m++) {
    pf.take(e);
    if (m + 1 < kB24Windows) {
      const uint32_t below = (sw[0] >> 23) & 1u;
#pragma unroll
      for (int i = 0; i < 7; i++) sw[i] = __builtin_amdgcn_alignbit(sw[i + 1], sw[i], 24);
      sw[7] >>= 24;
      const uint32_t u = sw[0] & 0xffffffu;
      pf.fetch(ks_b24row(bc, m + 1, (int)(u + below) - (int)((u >> 23) << 24), ng), ng);
    }
    ge_madd_niels(t, acc, e, false);
    if (m + 1 == kB24Windows) ge_p1p1_to_p2(out, t);
    else ge_p1p1_to_p3(acc, t);
  }
}

// First row of key v's comb in a chunked key set (kernels.h kKeyChunk*): one 8-B table load per
// signature in front of its first comb row.
__device__ __forceinline__ const int4 *key_rows(const int4 *const *__restrict__ tab, uint32_t v, size_t int4_per_key) {
  return tab[v >> kKeyChunkBits] + (size_t)(v & (kKeyChunkKeys - 1)) * int4_per_key;
}

template <int WAVES, bool B24 = false, bool ACOMB = false>
__global__ __launch_bounds__(kThreadsPerBlock, WAVES) void verify_keyset_main_kernel(
    const uint32_t *__restrict__ val_idx, uint32_t nkeys, const int4 *const *__restrict__ acomb,
    const int4 *__restrict__ bcomb, uint32_t base, uint32_t count, const int4 *__restrict__ prep, uint32_t stride,
    int4 *__restrict__ fin, uint32_t fin_base, uint8_t *__restrict__ out, const uint32_t *__restrict__ perm) {
  const uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x;
  if (slot >= count) return;
  // visiting position pos (key-grouped when perm is set: perm holds this chunk's signature
  // indices, so the prep hand-off of signature i is at slot i - base)
  const uint32_t pos = base + slot;
  const uint32_t i = perm ? perm[pos] : pos;
  const uint32_t ps = i - base;
  const uint32_t vi = val_idx[i];
  const uint32_t v = vi < nkeys ? vi : 0u;  // the prep kernel rejected an index past the key set
  uint32_t k[8], s[8];
  int32_t w[16];
#pragma unroll
  for (int q = 0; q < 4; q++) {  // k, s; ok at word 36
    const int4 x = prep[(size_t)q * stride + ps];
    w[4 * q] = x.x; w[4 * q + 1] = x.y; w[4 * q + 2] = x.z; w[4 * q + 3] = x.w;
  }
  const bool ok = prep[(size_t)9 * stride + ps].x != 0;
#pragma unroll
  for (int j = 0; j < 8; j++) { k[j] = (uint32_t)w[j]; s[j] = (uint32_t)w[8 + j]; }
#if TMED_KS_PF
  ge_p2 R;
  if (ACOMB) keyset_straus_ab24(R, k, s, key_rows(acomb, v, kCombARowsPerKey * kCombEntryInt4), bcomb);
  else if (B24) keyset_straus_b24(R, k, s, key_rows(acomb, v, (size_t)kCombWindows * kCombEntries * kCombEntryInt4), bcomb);
  else keyset_straus_pf(R, k, s, key_rows(acomb, v, (size_t)kCombWindows * kCombEntries * kCombEntryInt4), bcomb);
#else
  const GlobalComb ac{key_rows(acomb, v, (size_t)kCombWindows * kCombEntries * kCombEntryInt4)};
  const GlobalComb16 bc{bcomb};
  ge_p3 R;
  verify_main_comb_point(R, k, s, ac, bc);
#endif
  fin_store(fin, kFinCap, pos - fin_base, R.X, R.Y, R.Z);
  out[i] = ok ? 1 : 0;
}

// ---- key-grouped visiting order (launch_key_order) -------------------------------------
// A counting sort of one chunk's signatures by key group (G consecutive keys per bin, G a power
// of two chosen so that at most kKeyBins bins exist; indices past the key set form the last
// bin).  Random-address global atomics run far below the streaming rate on this part, so every
// tile of kKeyTile signatures counts in LDS and touches the global counters once per non-empty
// bin, 64 consecutive bins per wave instruction: (1) per-bin totals, (2) one block turns them
// into bin starts, (3) each tile reserves its range of every bin and places its signatures at
// LDS-atomic ranks inside it (the order inside a bin is irrelevant).
constexpr uint32_t kKeyBins = 4096, kKeyTile = 4096;

__device__ __forceinline__ uint32_t key_bin(uint32_t v, uint32_t nkeys, uint32_t shift) {
  return v < nkeys ? (v >> shift) : ((nkeys - 1) >> shift) + 1;
}

__global__ __launch_bounds__(256) void key_hist_kernel(const uint32_t *__restrict__ val_idx, uint32_t n,
                                                       uint32_t nkeys, uint32_t shift, uint32_t nbins,
                                                       uint32_t *__restrict__ total) {
  __shared__ uint32_t h[kKeyBins];
  for (uint32_t b = threadIdx.x; b < nbins; b += blockDim.x) h[b] = 0;
  __syncthreads();
  const uint32_t t0 = blockIdx.x * kKeyTile;
  for (uint32_t j = threadIdx.x; j < kKeyTile; j += blockDim.x) {
    const uint32_t i = t0 + j;
    if (i < n) atomicAdd(&h[key_bin(val_idx[i], nkeys, shift)], 1u);
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < nbins; b += blockDim.x)
    if (h[b]) atomicAdd(&total[b], h[b]);
}

// Exclusive prefix sum of cnt[0..m) in place, one 1024-lane block (m <= kKeyBins): lane t scans
// a contiguous run, the run totals are scanned in LDS, then the runs are rebased.
__global__ __launch_bounds__(1024) void key_scan_kernel(uint32_t *__restrict__ cnt, uint32_t m) {
  __shared__ uint32_t tot[1024];
  const uint32_t t = threadIdx.x;
  const uint32_t per = (m + 1023) / 1024, lo = t * per, hi = lo + per < m ? lo + per : m;
  uint32_t s = 0;
  for (uint32_t j = lo; j < hi; j++) s += cnt[j];
  tot[t] = s;
  __syncthreads();
  for (uint32_t o = 1; o < 1024; o <<= 1) {  // Hillis-Steele inclusive scan of the run totals
    const uint32_t x = t >= o ? tot[t - o] : 0u;
    __syncthreads();
    tot[t] += x;
    __syncthreads();
  }
  uint32_t acc = t ? tot[t - 1] : 0u;
  for (uint32_t j = lo; j < hi; j++) {
    const uint32_t c = cnt[j];
    cnt[j] = acc;
    acc += c;
  }
}

__global__ __launch_bounds__(256) void key_scatter_kernel(const uint32_t *__restrict__ val_idx, uint32_t n,
                                                          uint32_t nkeys, uint32_t shift, uint32_t nbins,
                                                          uint32_t *__restrict__ cursor, uint32_t index_base,
                                                          uint32_t *__restrict__ perm) {
  __shared__ uint32_t h[kKeyBins];
  for (uint32_t b = threadIdx.x; b < nbins; b += blockDim.x) h[b] = 0;
  __syncthreads();
  const uint32_t t0 = blockIdx.x * kKeyTile;
  for (uint32_t j = threadIdx.x; j < kKeyTile; j += blockDim.x) {
    const uint32_t i = t0 + j;
    if (i < n) atomicAdd(&h[key_bin(val_idx[i], nkeys, shift)], 1u);
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < nbins; b += blockDim.x)
    h[b] = h[b] ? atomicAdd(&cursor[b], h[b]) : 0u;  // this tile's range of bin b
  __syncthreads();
  for (uint32_t j = threadIdx.x; j < kKeyTile; j += blockDim.x) {
    const uint32_t i = t0 + j;
    if (i < n) perm[atomicAdd(&h[key_bin(val_idx[i], nkeys, shift)], 1u)] = index_base + i;
  }
}

static uint32_t key_shift(uint32_t nkeys) {
  uint32_t shift = 0;
  while (((nkeys - 1) >> shift) + 2 > kKeyBins) shift++;
  return shift;
}

uint32_t key_order_scratch_words(uint32_t n, uint32_t nkeys) {
  (void)n;
  return ((nkeys - 1) >> key_shift(nkeys)) + 2;
}

hipError_t launch_key_order(const uint32_t *val_idx, uint32_t n, uint32_t nkeys, uint32_t *scratch, uint32_t *perm,
                            uint32_t index_base, hipStream_t stream) {
  if (nkeys == 0 || nkeys > kKeyOrderMaxKeys) return hipErrorInvalidValue;
  if (n == 0) return hipSuccess;
  const uint32_t shift = key_shift(nkeys), nbins = ((nkeys - 1) >> shift) + 2;
  const uint32_t ntiles = (n + kKeyTile - 1) / kKeyTile;
  hipError_t e = hipMemsetAsync(scratch, 0, (size_t)nbins * 4, stream);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(key_hist_kernel, dim3(ntiles), dim3(256), 0, stream, val_idx, n, nkeys, shift, nbins, scratch);
  hipLaunchKernelGGL(key_scan_kernel, dim3(1), dim3(1024), 0, stream, scratch, nbins);
  hipLaunchKernelGGL(key_scatter_kernel, dim3(ntiles), dim3(256), 0, stream, val_idx, n, nkeys, shift, nbins, scratch,
                     index_base, perm);
  return hipGetLastError();
}

hipError_t launch_comb_bases(const uint8_t *pubs, uint32_t n, int negate, uint8_t *ok, int32_t *bases,
                             hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(comb_bases_kernel, dim3((n + 63) / 64), dim3(64), 0, stream, pubs, n, negate, ok, bases);
  return hipGetLastError();
}

hipError_t launch_comb_fill(const int32_t *bases, uint32_t n, int4 *comb, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(comb_fill_kernel, dim3((n * kCombWindows + 64 / kCombRuns - 1) / (64 / kCombRuns)), dim3(64), 0,
                     stream, bases, n, comb);
  return hipGetLastError();
}


// ---- radix-2^B comb of -A (kernels.h kCombA*) -------------------------------------------
__global__ __launch_bounds__(64) void comba_bases_kernel(const uint8_t *__restrict__ pubs, uint32_t n,
                                                        int32_t *__restrict__ bases) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t pw[8];
  load_row_words(pw, pubs + 32 * (size_t)i, 2);
  ge_p3 P;
  (void)ge_frombytes_go(P, pw);  // the identity when the key does not decode (key_ok rejects it)
  fe_neg(P.X, P.X);
  fe_neg(P.T, P.T);
#pragma unroll 1
  for (int w = 0; w < kCombAWindows; w++) {
    p3_store(bases + ((size_t)i * kCombAWindows + w) * 40, P);
    ge_mul256(P);  // x 2^B: B - 8 more doublings
    ge_p1p1 t;
    ge_p2 q;
    ge_p3_to_p2(q, P);
#pragma unroll 1
    for (int d = 0; d < kCombABits - 8; d++) {
      ge_p2_dbl(t, q);
      if (d + 1 < kCombABits - 8) ge_p1p1_to_p2(q, t);
    }
    ge_p1p1_to_p3(P, t);
  }
}

// The radix-2^B comb of -A: runs of 8 (comb_fill_run), 64 runs per block, each block within one
// (key, window).
constexpr uint32_t kCombARunsReg = (kCombAEntries - 1) / kCombARun;     // 256: j = 1..2048
constexpr uint32_t kCombARunsTop = (kCombATopEntries - 1) / kCombARun;  // 528: j = 1..4224
static_assert((kCombAEntries - 1) % kCombARun == 0 && (kCombATopEntries - 1) % kCombARun == 0, "runs");
constexpr uint32_t kCombABlocksReg = (kCombARunsReg + 63) / 64, kCombABlocksTop = (kCombARunsTop + 63) / 64;
constexpr uint32_t kCombABlocksPerKey = (kCombAWindows - 1) * kCombABlocksReg + kCombABlocksTop;
__global__ __launch_bounds__(64) void comba_fill_kernel(const int32_t *__restrict__ bases, int4 *__restrict__ comb) {
  __shared__ fe pre[kCombARun][64];
  const uint32_t key = blockIdx.x / kCombABlocksPerKey, g = blockIdx.x % kCombABlocksPerKey;
  const bool top = g >= (kCombAWindows - 1) * kCombABlocksReg;
  const uint32_t w = top ? kCombAWindows - 1 : g / kCombABlocksReg;
  const uint32_t run = (g - w * kCombABlocksReg) * 64u + threadIdx.x;
  int4 *rows = comb + ((size_t)key * kCombARowsPerKey + comba_row((int)w, 0)) * kCombEntryInt4;
  if (run == 0) {
    ge_niels id;
    ge_niels_0(id);
    niels_store(rows, id);
  }
  if (run >= (top ? kCombARunsTop : kCombARunsReg)) return;
  comb_fill_run(rows, bases + ((size_t)key * kCombAWindows + w) * 40, 1u + kCombARun * run,
                top ? comb_start_bits(kCombARunsTop) : comb_start_bits(kCombARunsReg), pre, threadIdx.x);
}

hipError_t launch_build_comba(const uint8_t *pubs, uint32_t n, int32_t *bases, int4 *comba, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(comba_bases_kernel, dim3((n + 63) / 64), dim3(64), 0, stream, pubs, n, bases);
  hipLaunchKernelGGL(comba_fill_kernel, dim3(n * kCombABlocksPerKey), dim3(64), 0, stream, bases, comba);
  return hipGetLastError();
}

// ---- latency mode (verify_core.h): small key-cached batches ------------------------------
// One launch, two roles by block (64-lane blocks; the R blocks come first so the longest
// chain is dispatched first):
//  * blocks [0, nR): lane i strictly decodes R of signature i -> (x_R, y_R, ok) in dec;
//  * blocks [nR, nR + nC): 8 lanes per signature; every lane of the group hashes (the same
//    SHA-512, so no divergence), lane r sums its 8 comb entries, three __shfl_down steps
//    add the partial sums, lane 0 writes R' (fin) and the prep verdict (out).
// verify_lat_finish_kernel then compares projectively.  dec layout: [q][i], q < 6 int4.
constexpr int kLatDecInt4 = 6;

__device__ __forceinline__ void shfl_down_fe(fe &o, const fe &f, int L) {
#pragma unroll
  for (int i = 0; i < 10; i++) o.v[i] = __shfl_down(f.v[i], (unsigned)L, kLatLanes);
}

// comb_partial (verify_core.h) with the next comb row in flight and the first row converted
// instead of added to the identity: lane rr's 8 rows are A(w), B(w) for w = rr, rr+8, rr+16, rr+24.
__device__ __forceinline__ const int4 *lat_row(const int4 *comb, int w, uint32_t byte, bool &neg) {
  const int d = (int)byte - 128;
  neg = d < 0;
  return comb + ((size_t)w * kCombEntries + (uint32_t)(neg ? -d : d)) * kCombEntryInt4;
}
__device__ __forceinline__ void comb_partial_pf(ge_p3 &acc, const uint32_t kr[8], const uint32_t sr[8], int rr,
                                                const int4 *ac, const int4 *bc) {
  const int sh = 8 * (rr & 3);
  CombRowPf pf;
  bool ng;
  pf.fetch(lat_row(ac, rr, ((rr & 4) ? kr[1] : kr[0]) >> sh & 0xffu, ng), ng);
  ge_p1p1 t;
  ge_niels e;
#pragma unroll
  for (int st = 0; st < 8; st++) {
    const int q = st >> 1;
    pf.take(e);
    if (st < 7) {  // the row of step st + 1
      const int nq = (st + 1) >> 1, w = rr + 8 * nq;
      const uint32_t word = (st + 1) & 1 ? ((rr & 4) ? sr[2 * nq + 1] : sr[2 * nq])
                                         : ((rr & 4) ? kr[2 * nq + 1] : kr[2 * nq]);
      pf.fetch(lat_row((st + 1) & 1 ? bc : ac, w, (word >> sh) & 0xffu, ng), ng);
    }
    (void)q;
    if (st == 0) {
      ge_niels_to_p3(acc, e);
    } else {
      ge_madd_niels(t, acc, e, false);
      ge_p1p1_to_p3(acc, t);
    }
  }
}

__global__ __launch_bounds__(64) void verify_keyset_lat_kernel(
    const uint32_t *__restrict__ val_idx, uint32_t nkeys, const uint8_t *__restrict__ key_pub,
    const uint8_t *__restrict__ key_ok,
    const int4 *const *__restrict__ acomb, const int4 *__restrict__ bcomb, const uint8_t *__restrict__ sig, MsgSrc ms,
    uint32_t m, uint32_t nR, int4 *__restrict__ fin, int4 *__restrict__ dec, uint8_t *__restrict__ out, VoteAsm va,
    int assemble) {
  __shared__ int4 tl[64][kVoteTmplBytes / 16];  // the comb lanes' vote templates (assemble_vote)
  if (blockIdx.x < nR) {
    const uint32_t i = blockIdx.x * 64 + threadIdx.x;
    if (i >= m) return;
    uint32_t Rw[8];
    load_row_words(Rw, sig + 64 * (size_t)i, 2);
    fe x, y;
    const bool ok = r_decode_strict(x, y, Rw);
    int32_t w[24];
#pragma unroll
    for (int j = 0; j < 10; j++) { w[j] = x.v[j]; w[10 + j] = y.v[j]; }
    w[20] = ok ? 1 : 0;
    w[21] = w[22] = w[23] = 0;
#pragma unroll
    for (int q = 0; q < kLatDecInt4; q++) dec[(size_t)q * m + i] = make_int4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
    return;
  }
  const uint32_t g = (blockIdx.x - nR) * (64 / kLatLanes) + (threadIdx.x / kLatLanes);
  const int r = (int)(threadIdx.x % kLatLanes);
  if (g >= m) return;  // whole 8-lane groups leave together: the shuffles stay inside live groups
  if (assemble) assemble_vote(va, g, const_cast<uint8_t *>(ms.msgs), const_cast<uint32_t *>(ms.off), tl[threadIdx.x]);
  const uint32_t vi = val_idx[g];
  const bool vin = vi < nkeys;  // an index past the key set rejects the signature (row 0 is read)
  const uint32_t v = vin ? vi : 0u;
  uint32_t pw[8], sw[16], k[8], s[8], kr[8], sr[8];
  load_row_words(pw, key_pub + 32 * (size_t)v, 2);
  load_row_words(sw, sig + 64 * (size_t)g, 4);
  const uint8_t *msg;
  uint32_t mlen;
  ms.get(g, msg, mlen);
  const bool ok = verify_prep_comb(pw, vin && key_ok[v] != 0, sw, msg, mlen, k, s);
  sc_recode256(kr, k);
  sc_recode256(sr, s);
  ge_p3 acc, o;
  comb_partial_pf(acc, kr, sr, r, key_rows(acomb, v, (size_t)kCombWindows * kCombEntries * kCombEntryInt4), bcomb);
#pragma unroll 1
  for (int L = 1; L < kLatLanes; L <<= 1) {
    shfl_down_fe(o.X, acc.X, L);
    shfl_down_fe(o.Y, acc.Y, L);
    shfl_down_fe(o.Z, acc.Z, L);
    shfl_down_fe(o.T, acc.T, L);
    ge_p3_add(acc, o);
  }
  if (r == 0) {
    fin_store(fin, kFinCap, g, acc.X, acc.Y, acc.Z);
    out[g] = ok ? 1 : 0;
  }
}

__global__ __launch_bounds__(kThreadsPerBlock) void verify_lat_finish_kernel(const int4 *__restrict__ fin,
                                                                            const int4 *__restrict__ dec, uint32_t m,
                                                                            uint8_t *__restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  int32_t w[32];
#pragma unroll
  for (int q = 0; q < kFinInt4; q++) {
    const int4 t = fin[(size_t)q * kFinCap + i];
    w[4 * q] = t.x; w[4 * q + 1] = t.y; w[4 * q + 2] = t.z; w[4 * q + 3] = t.w;
  }
  fe X, Y, Z, x, y;
#pragma unroll
  for (int j = 0; j < 10; j++) { X.v[j] = w[j]; Y.v[j] = w[10 + j]; Z.v[j] = w[20 + j]; }
#pragma unroll
  for (int q = 0; q < kLatDecInt4; q++) {
    const int4 t = dec[(size_t)q * m + i];
    w[4 * q] = t.x; w[4 * q + 1] = t.y; w[4 * q + 2] = t.z; w[4 * q + 3] = t.w;
  }
#pragma unroll
  for (int j = 0; j < 10; j++) { x.v[j] = w[j]; y.v[j] = w[10 + j]; }
  const bool ok = out[i] && w[20] && projective_matches(X, Y, Z, x, y);
  out[i] = ok ? 1 : 0;
}

hipError_t launch_verify_keyset_lat(const uint32_t *val_idx, uint32_t nkeys, const uint8_t *key_pub, const uint8_t *key_ok,
                                    const int4 *const *acomb, const int4 *bcomb, const uint8_t *sig, const uint8_t *msgs,
                                    const uint32_t *off, uint32_t n, uint8_t *out, int4 *fin, int4 *dec,
                                    hipStream_t stream, bool msg_slots, const VoteAsm *va) {
  if (n == 0) return hipSuccess;
  if (n > kLatMax) return hipErrorInvalidValue;  // fin / dec are sized for kLatMax signatures
  if (va && !msg_slots) return hipErrorInvalidValue;
  const MsgSrc ms{msgs, off, msg_slots};
  const uint32_t nR = (n + 63) / 64, nC = (n + 64 / kLatLanes - 1) / (64 / kLatLanes);
  hipLaunchKernelGGL(verify_keyset_lat_kernel, dim3(nR + nC), dim3(64), 0, stream, val_idx, nkeys, key_pub, key_ok, acomb,
                     bcomb, sig, ms, n, nR, fin, dec, out, va ? *va : VoteAsm{}, va ? 1 : 0);
  hipLaunchKernelGGL(verify_lat_finish_kernel, dim3((n + kThreadsPerBlock - 1) / kThreadsPerBlock),
                     dim3(kThreadsPerBlock), 0, stream, fin, dec, n, out);
  return hipGetLastError();
}

hipError_t launch_verify_keyset(const uint32_t *val_idx, uint32_t nkeys, const uint8_t *key_pub, const uint8_t *key_ok,
                                const int4 *const *acomb, const int4 *bcomb, const uint8_t *sig, const uint8_t *msgs,
                                const uint32_t *off, uint32_t n, uint8_t *out, int4 *prep, uint32_t stride,
                                int4 *fin, int4 *fin_pre, hipStream_t stream, bool msg_slots, KernelTimer *timer,
                                uint32_t *perm, uint32_t *order_scratch, const int4 *bcomb24,
                                const int4 *const *acomba) {
  const MsgSrc ms{msgs, off, msg_slots};
  if (stride > kFinCap) stride = kFinCap;
  if (timer) timer->mark(stream, -1);
  for (uint32_t fbase = 0; fbase < n; fbase += kFinCap) {
    const uint32_t m = (n - fbase) < kFinCap ? (n - fbase) : kFinCap;
    for (uint32_t base = fbase; base < fbase + m; base += stride) {
      const uint32_t count = (fbase + m - base) < stride ? (fbase + m - base) : stride;
      const uint32_t blocks = (count + kThreadsPerBlock - 1) / kThreadsPerBlock;
      if (perm) {  // key-grouped visiting order of this chunk (main + finish)
        hipError_t e = launch_key_order(val_idx + base, count, nkeys, order_scratch, perm + base, base, stream);
        if (e != hipSuccess) return e;
      }
      hipLaunchKernelGGL(verify_keyset_prep_kernel, dim3(blocks), dim3(kThreadsPerBlock), 0, stream, val_idx,
                         nkeys, key_pub, key_ok, sig, ms, base, count, prep, stride);
      if (timer) timer->mark(stream, 0);
      if (bcomb24 && acomba)
        hipLaunchKernelGGL((verify_keyset_main_kernel<2, true, true>), dim3(blocks), dim3(kThreadsPerBlock), 0, stream,
                           val_idx, nkeys, acomba, bcomb24, base, count, prep, stride, fin, fbase, out, perm);
      else if (bcomb24)
        hipLaunchKernelGGL((verify_keyset_main_kernel<2, true>), dim3(blocks), dim3(kThreadsPerBlock), 0, stream,
                           val_idx, nkeys, acomb, bcomb24, base, count, prep, stride, fin, fbase, out, perm);
      else
        hipLaunchKernelGGL(verify_keyset_main_kernel<2>, dim3(blocks), dim3(kThreadsPerBlock), 0, stream, val_idx,
                           nkeys, acomb, bcomb, base, count, prep, stride, fin, fbase, out, perm);
      if (timer) timer->mark(stream, 1);
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
    }
    hipError_t e = launch_finish(fin, fin_pre, sig, out, fbase, m, stream, perm);
    if (timer) timer->mark(stream, 2);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace tmed

namespace tmed {

hipError_t launch_assemble_votes(const uint8_t *tmpl, const uint32_t *tmpl_idx, const uint8_t *flags,
                                 const int64_t *ts_sec, const int32_t *ts_nanos, uint32_t n, uint8_t *out,
                                 uint32_t *out_len, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(assemble_votes_kernel, dim3((n + kAsmLanes - 1) / kAsmLanes), dim3(kAsmLanes), 0, stream,
                     VoteAsm{tmpl, tmpl_idx, flags, ts_sec, ts_nanos}, n, out, out_len);
  return hipGetLastError();
}

}  // namespace tmed
