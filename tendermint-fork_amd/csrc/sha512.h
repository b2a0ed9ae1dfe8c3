// sha512.h — SHA-512 for the verify/sign kernels (one message per lane).
//
// Replaces Go crypto/sha512 as used by crypto/ed25519.Verify to form
// k = SHA-512(R || A || M) (reference call site crypto/ed25519/ed25519.go:154),
// and by the RFC 8032 signer for synthetic commits (ed25519.go:57-60).
//
// The message is presented as a "virtual stream" of up to three segments:
// two 32-byte register-resident prefixes (R and A as LE words) and a byte
// string in global memory.  Blocks are assembled on the fly (no staging),
// 64-bit words are big-endian.  64-bit rotates lower to v_alignbit_b32 pairs.
#pragma once
#include "fe25519.h"

namespace tmed {

#if defined(__HIP_DEVICE_COMPILE__)
#define TMED_ROTR64(x, n) __builtin_rotateright64((x), (n))
#else
#define TMED_ROTR64(x, n) (((x) >> (n)) | ((x) << (64 - (n))))
#endif

#if defined(__HIPCC__)
__constant__ static const uint64_t kSha512K[80] = {
      0x428a2f98d728ae22ull, 0x7137449123ef65cdull, 0xb5c0fbcfec4d3b2full, 0xe9b5dba58189dbbcull,
      0x3956c25bf348b538ull, 0x59f111f1b605d019ull, 0x923f82a4af194f9bull, 0xab1c5ed5da6d8118ull,
      0xd807aa98a3030242ull, 0x12835b0145706fbeull, 0x243185be4ee4b28cull, 0x550c7dc3d5ffb4e2ull,
      0x72be5d74f27b896full, 0x80deb1fe3b1696b1ull, 0x9bdc06a725c71235ull, 0xc19bf174cf692694ull,
      0xe49b69c19ef14ad2ull, 0xefbe4786384f25e3ull, 0x0fc19dc68b8cd5b5ull, 0x240ca1cc77ac9c65ull,
      0x2de92c6f592b0275ull, 0x4a7484aa6ea6e483ull, 0x5cb0a9dcbd41fbd4ull, 0x76f988da831153b5ull,
      0x983e5152ee66dfabull, 0xa831c66d2db43210ull, 0xb00327c898fb213full, 0xbf597fc7beef0ee4ull,
      0xc6e00bf33da88fc2ull, 0xd5a79147930aa725ull, 0x06ca6351e003826full, 0x142929670a0e6e70ull,
      0x27b70a8546d22ffcull, 0x2e1b21385c26c926ull, 0x4d2c6dfc5ac42aedull, 0x53380d139d95b3dfull,
      0x650a73548baf63deull, 0x766a0abb3c77b2a8ull, 0x81c2c92e47edaee6ull, 0x92722c851482353bull,
      0xa2bfe8a14cf10364ull, 0xa81a664bbc423001ull, 0xc24b8b70d0f89791ull, 0xc76c51a30654be30ull,
      0xd192e819d6ef5218ull, 0xd69906245565a910ull, 0xf40e35855771202aull, 0x106aa07032bbd1b8ull,
      0x19a4c116b8d2d0c8ull, 0x1e376c085141ab53ull, 0x2748774cdf8eeb99ull, 0x34b0bcb5e19b48a8ull,
      0x391c0cb3c5c95a63ull, 0x4ed8aa4ae3418acbull, 0x5b9cca4f7763e373ull, 0x682e6ff3d6b2b8a3ull,
      0x748f82ee5defb2fcull, 0x78a5636f43172f60ull, 0x84c87814a1f0ab72ull, 0x8cc702081a6439ecull,
      0x90befffa23631e28ull, 0xa4506cebde82bde9ull, 0xbef9a3f7b2c67915ull, 0xc67178f2e372532bull,
      0xca273eceea26619cull, 0xd186b8c721c0c207ull, 0xeada7dd6cde0eb1eull, 0xf57d4f7fee6ed178ull,
      0x06f067aa72176fbaull, 0x0a637dc5a2c898a6ull, 0x113f9804bef90daeull, 0x1b710b35131c471bull,
      0x28db77f523047d84ull, 0x32caab7b40c72493ull, 0x3c9ebe0a15c9bebcull, 0x431d67c49c100d4cull,
      0x4cc5d4becb3e42b6ull, 0x597f299cfc657e2aull, 0x5fcb6fab3ad6faecull, 0x6c44198c4a475817ull};
#else
static const uint64_t kSha512K[80] = {
      0x428a2f98d728ae22ull, 0x7137449123ef65cdull, 0xb5c0fbcfec4d3b2full, 0xe9b5dba58189dbbcull,
      0x3956c25bf348b538ull, 0x59f111f1b605d019ull, 0x923f82a4af194f9bull, 0xab1c5ed5da6d8118ull,
      0xd807aa98a3030242ull, 0x12835b0145706fbeull, 0x243185be4ee4b28cull, 0x550c7dc3d5ffb4e2ull,
      0x72be5d74f27b896full, 0x80deb1fe3b1696b1ull, 0x9bdc06a725c71235ull, 0xc19bf174cf692694ull,
      0xe49b69c19ef14ad2ull, 0xefbe4786384f25e3ull, 0x0fc19dc68b8cd5b5ull, 0x240ca1cc77ac9c65ull,
      0x2de92c6f592b0275ull, 0x4a7484aa6ea6e483ull, 0x5cb0a9dcbd41fbd4ull, 0x76f988da831153b5ull,
      0x983e5152ee66dfabull, 0xa831c66d2db43210ull, 0xb00327c898fb213full, 0xbf597fc7beef0ee4ull,
      0xc6e00bf33da88fc2ull, 0xd5a79147930aa725ull, 0x06ca6351e003826full, 0x142929670a0e6e70ull,
      0x27b70a8546d22ffcull, 0x2e1b21385c26c926ull, 0x4d2c6dfc5ac42aedull, 0x53380d139d95b3dfull,
      0x650a73548baf63deull, 0x766a0abb3c77b2a8ull, 0x81c2c92e47edaee6ull, 0x92722c851482353bull,
      0xa2bfe8a14cf10364ull, 0xa81a664bbc423001ull, 0xc24b8b70d0f89791ull, 0xc76c51a30654be30ull,
      0xd192e819d6ef5218ull, 0xd69906245565a910ull, 0xf40e35855771202aull, 0x106aa07032bbd1b8ull,
      0x19a4c116b8d2d0c8ull, 0x1e376c085141ab53ull, 0x2748774cdf8eeb99ull, 0x34b0bcb5e19b48a8ull,
      0x391c0cb3c5c95a63ull, 0x4ed8aa4ae3418acbull, 0x5b9cca4f7763e373ull, 0x682e6ff3d6b2b8a3ull,
      0x748f82ee5defb2fcull, 0x78a5636f43172f60ull, 0x84c87814a1f0ab72ull, 0x8cc702081a6439ecull,
      0x90befffa23631e28ull, 0xa4506cebde82bde9ull, 0xbef9a3f7b2c67915ull, 0xc67178f2e372532bull,
      0xca273eceea26619cull, 0xd186b8c721c0c207ull, 0xeada7dd6cde0eb1eull, 0xf57d4f7fee6ed178ull,
      0x06f067aa72176fbaull, 0x0a637dc5a2c898a6ull, 0x113f9804bef90daeull, 0x1b710b35131c471bull,
      0x28db77f523047d84ull, 0x32caab7b40c72493ull, 0x3c9ebe0a15c9bebcull, 0x431d67c49c100d4cull,
      0x4cc5d4becb3e42b6ull, 0x597f299cfc657e2aull, 0x5fcb6fab3ad6faecull, 0x6c44198c4a475817ull};
#endif

TMED_HD uint64_t sha512_k(int i) {
#if defined(__HIP_DEVICE_COMPILE__)
  return kSha512K[i];  // i is wave-uniform: scalar load
#else
  return kSha512K[i];
#endif
}

TMED_HD void sha512_init(uint64_t st[8]) {
  st[0] = 0x6a09e667f3bcc908ull; st[1] = 0xbb67ae8584caa73bull;
  st[2] = 0x3c6ef372fe94f82bull; st[3] = 0xa54ff53a5f1d36f1ull;
  st[4] = 0x510e527fade682d1ull; st[5] = 0x9b05688c2b3e6c1full;
  st[6] = 0x1f83d9abfb41bd6bull; st[7] = 0x5be0cd19137e2179ull;
}

// The round functions on the device as 32-bit halves: a 64-bit rotate is two v_alignbit_b32
// (LLVM's lowering of rotr64 is a 64-bit shift, a 32-bit shift and an or: three instructions),
// three-way xors and Maj are one v_bitop3_b32 per half (gfx950; LUT 0x96 = a ^ b ^ c, 0xE8 =
// majority — both symmetric, so the operand order is immaterial).  Host builds use the plain
// 64-bit expressions below.
#ifndef TMED_SHA_BITOP3
#define TMED_SHA_BITOP3 1  // A/B knob: 0 = the plain 64-bit expressions on the device too
#endif
#if defined(__HIP_DEVICE_COMPILE__) && TMED_SHA_BITOP3
__device__ __forceinline__ uint32_t sha_xor3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ uint32_t sha_maj(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xe8" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
// (lo, hi) -> uint64 as a register pair (a shift / or lets LLVM split the value into two
// zero-extended 64-bit adds downstream)
typedef uint32_t sha_u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint64_t sha_pack(uint32_t lo, uint32_t hi) {
  const sha_u32x2 v = {lo, hi};
  return __builtin_bit_cast(uint64_t, v);
}
// rotr64(x, n) as (lo, hi) halves, n a compile-time constant in 1..63, n != 32
template <int N>
__device__ __forceinline__ void sha_rotr(uint32_t &lo, uint32_t &hi, uint32_t xl, uint32_t xh) {
  if (N < 32) {
    lo = __builtin_amdgcn_alignbit(xh, xl, N);
    hi = __builtin_amdgcn_alignbit(xl, xh, N);
  } else {
    lo = __builtin_amdgcn_alignbit(xl, xh, N - 32);
    hi = __builtin_amdgcn_alignbit(xh, xl, N - 32);
  }
}
// rotr(x, A) ^ rotr(x, B) ^ rotr(x, C)      (Sigma0 / Sigma1)
template <int A, int B, int C>
__device__ __forceinline__ uint64_t sha_Sig(uint64_t x) {
  const uint32_t xl = (uint32_t)x, xh = (uint32_t)(x >> 32);
  uint32_t l0, h0, l1, h1, l2, h2;
  sha_rotr<A>(l0, h0, xl, xh);
  sha_rotr<B>(l1, h1, xl, xh);
  sha_rotr<C>(l2, h2, xl, xh);
  return sha_pack(sha_xor3(l0, l1, l2), sha_xor3(h0, h1, h2));
}
// rotr(x, A) ^ rotr(x, B) ^ (x >> C)       (sigma0 / sigma1 of the message schedule, C < 32)
template <int A, int B, int C>
__device__ __forceinline__ uint64_t sha_sig(uint64_t x) {
  const uint32_t xl = (uint32_t)x, xh = (uint32_t)(x >> 32);
  uint32_t l0, h0, l1, h1;
  sha_rotr<A>(l0, h0, xl, xh);
  sha_rotr<B>(l1, h1, xl, xh);
  const uint32_t l2 = __builtin_amdgcn_alignbit(xh, xl, C), h2 = xh >> C;
  return sha_pack(sha_xor3(l0, l1, l2), sha_xor3(h0, h1, h2));
}
__device__ __forceinline__ uint64_t sha_Maj(uint64_t a, uint64_t b, uint64_t c) {
  return sha_pack(sha_maj((uint32_t)a, (uint32_t)b, (uint32_t)c),
                  sha_maj((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32)));
}
#define TMED_SHA_S0(a) sha_Sig<28, 34, 39>(a)
#define TMED_SHA_S1(e) sha_Sig<14, 18, 41>(e)
#define TMED_SHA_s0(w) sha_sig<1, 8, 7>(w)
#define TMED_SHA_s1(w) sha_sig<19, 61, 6>(w)
#define TMED_SHA_MAJ(a, b, c) sha_Maj(a, b, c)
#else
#define TMED_SHA_S0(a) (TMED_ROTR64(a, 28) ^ TMED_ROTR64(a, 34) ^ TMED_ROTR64(a, 39))
#define TMED_SHA_S1(e) (TMED_ROTR64(e, 14) ^ TMED_ROTR64(e, 18) ^ TMED_ROTR64(e, 41))
#define TMED_SHA_s0(w) (TMED_ROTR64(w, 1) ^ TMED_ROTR64(w, 8) ^ ((w) >> 7))
#define TMED_SHA_s1(w) (TMED_ROTR64(w, 19) ^ TMED_ROTR64(w, 61) ^ ((w) >> 6))
#define TMED_SHA_MAJ(a, b, c) (((a) & (b)) ^ ((c) & ((a) ^ (b))))
#endif

// One round on the working variables (the caller rotates their roles by renaming, below).
TMED_HD void sha512_round(const uint64_t a, const uint64_t b, const uint64_t c, uint64_t &d, const uint64_t e,
                          const uint64_t f, const uint64_t g, uint64_t &h, uint64_t kw) {
  const uint64_t S1 = TMED_SHA_S1(e);
  const uint64_t ch = (e & f) ^ (~e & g);
  const uint64_t t1 = h + S1 + ch + kw;
  const uint64_t S0 = TMED_SHA_S0(a);
  const uint64_t mj = TMED_SHA_MAJ(a, b, c);
  d += t1;           // the next round's e
  h = t1 + S0 + mj;  // the next round's a
}
TMED_HD void sha512_sched(uint64_t w[16], int j) {
  const uint64_t w15 = w[(j + 1) & 15], w2 = w[(j + 14) & 15];
  w[j] += TMED_SHA_s0(w15) + w[(j + 9) & 15] + TMED_SHA_s1(w2);
}
// Eight rounds with the roles of the working variables rotated by renaming (no register moves).
#define TMED_SHA_8ROUNDS(R, J, SCHED)                                                  \
  do {                                                                                 \
    if (SCHED) sha512_sched(w, (J) + 0);                                               \
    sha512_round(v0, v1, v2, v3, v4, v5, v6, v7, sha512_k((R) + (J) + 0) + w[(J) + 0]); \
    if (SCHED) sha512_sched(w, (J) + 1);                                               \
    sha512_round(v7, v0, v1, v2, v3, v4, v5, v6, sha512_k((R) + (J) + 1) + w[(J) + 1]); \
    if (SCHED) sha512_sched(w, (J) + 2);                                               \
    sha512_round(v6, v7, v0, v1, v2, v3, v4, v5, sha512_k((R) + (J) + 2) + w[(J) + 2]); \
    if (SCHED) sha512_sched(w, (J) + 3);                                               \
    sha512_round(v5, v6, v7, v0, v1, v2, v3, v4, sha512_k((R) + (J) + 3) + w[(J) + 3]); \
    if (SCHED) sha512_sched(w, (J) + 4);                                               \
    sha512_round(v4, v5, v6, v7, v0, v1, v2, v3, sha512_k((R) + (J) + 4) + w[(J) + 4]); \
    if (SCHED) sha512_sched(w, (J) + 5);                                               \
    sha512_round(v3, v4, v5, v6, v7, v0, v1, v2, sha512_k((R) + (J) + 5) + w[(J) + 5]); \
    if (SCHED) sha512_sched(w, (J) + 6);                                               \
    sha512_round(v2, v3, v4, v5, v6, v7, v0, v1, sha512_k((R) + (J) + 6) + w[(J) + 6]); \
    if (SCHED) sha512_sched(w, (J) + 7);                                               \
    sha512_round(v1, v2, v3, v4, v5, v6, v7, v0, sha512_k((R) + (J) + 7) + w[(J) + 7]); \
  } while (0)

// 80 rounds: the first 16 (no message schedule) peeled, then 4 x 16 with the schedule, so the
// rolled loop carries no per-round branch on the pass index (5 x 16 under `r > 0` compiled every
// round to a basic block of its own and spilled 4 VGPRs in the keyed prep: keyed C2 490 against
// 521 M/s, profiles/r05/s6/).  The message-schedule window w[i & 15] stays register-indexed; the
// round constants come from a uniform table (scalar loads on the device).
TMED_HD void sha512_compress(uint64_t st[8], uint64_t w[16]) {
  uint64_t v0 = st[0], v1 = st[1], v2 = st[2], v3 = st[3], v4 = st[4], v5 = st[5], v6 = st[6], v7 = st[7];
  TMED_SHA_8ROUNDS(0, 0, false);
  TMED_SHA_8ROUNDS(0, 8, false);
#pragma unroll 1
  for (int r = 16; r < 80; r += 16) {
    TMED_SHA_8ROUNDS(r, 0, true);
    TMED_SHA_8ROUNDS(r, 8, true);
  }
  st[0] += v0; st[1] += v1; st[2] += v2; st[3] += v3; st[4] += v4; st[5] += v5; st[6] += v6; st[7] += v7;
}
#undef TMED_SHA_8ROUNDS

TMED_HD uint32_t bswap32(uint32_t x) {
  return (x >> 24) | ((x >> 8) & 0xff00u) | ((x << 8) & 0xff0000u) | (x << 24);
}

// Message reader: big-endian 32-bit groups of M (any byte alignment) from aligned dword
// loads.  On the device one v_perm_b32 per group realigns and byte-swaps (the selector
// depends only on the lane's misalignment r); dwords past the last one that overlaps M
// are never read.
struct MsgReader {
  const uint32_t *base;  // M rounded down to a dword boundary (never read past ndw dwords)
  uint32_t ndw;          // aligned dwords overlapping M
  uint32_t r;            // misalignment of M in bytes
  const uint8_t *m;
  uint32_t mlen;
  TMED_HDM MsgReader(const uint8_t *m_, uint32_t mlen_) : m(m_), mlen(mlen_) {
    const uintptr_t a = (uintptr_t)m_;
    r = (uint32_t)(a & 3u);
    base = (const uint32_t *)(a - r);
    ndw = (r + mlen_ + 3u) >> 2;
  }
  // bytes M[o .. o+3] (o % 4 == 0) as a big-endian word; bytes past M are unspecified
  // (the caller masks them).
  TMED_HDM uint32_t be32(uint32_t o) const {
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t q = o >> 2;
    const uint32_t lo = q < ndw ? base[q] : 0u;
    const uint32_t hi = (q + 1) < ndw ? base[q + 1] : 0u;
    const uint32_t sel = (r << 24) | ((r + 1) << 16) | ((r + 2) << 8) | (r + 3);
    return __builtin_amdgcn_perm(hi, lo, sel);
#else
    uint32_t v = 0;
    for (uint32_t i = 0; i < 4; i++) v = (v << 8) | (o + i < mlen ? m[o + i] : 0u);
    return v;
#endif
  }
};

// Big-endian 64-bit word of the padded virtual stream  P0 || P1 || M || 0x80 || 0* || len128
// at byte position pos (multiple of 8).  npre = 0, 32 or 64 bytes of register prefix
// (p0 then p1, LE words).  total = npre + |M|, padded = 128 * nblocks.
TMED_HD uint64_t sha512_stream_word(const uint32_t p0[8], const uint32_t p1[8], int npre, const MsgReader &rd,
                                    uint32_t pos, uint32_t padded_len) {
  const uint32_t total = (uint32_t)npre + rd.mlen;
  if (pos + 8 <= (uint32_t)npre) {
    const uint32_t q = pos >> 2;  // word index into the 64-byte prefix
    const uint32_t lo = q < 8 ? p0[q] : p1[q - 8];
    const uint32_t hi = (q + 1) < 8 ? p0[q + 1] : p1[q + 1 - 8];
    return ((uint64_t)bswap32(lo) << 32) | bswap32(hi);
  }
  if (pos + 8 == padded_len) return (uint64_t)total * 8u;  // length (low 64 bits of len128)
  const uint32_t mo = pos - (uint32_t)npre;                // npre and pos are multiples of 8
  const int32_t nv = (int32_t)rd.mlen - (int32_t)mo;       // message bytes in this word
  uint64_t v = 0;
  if (nv > 0) v = ((uint64_t)rd.be32(mo) << 32) | rd.be32(mo + 4);
  if (nv < 8) {
    if (nv > 0) v &= ~(~0ull >> (8 * nv));
    if (nv >= 0) v |= 0x80ull << (56 - 8 * nv);
  }
  return v;
}

// digest = SHA-512(P0 || P1 || M) as 16 LE 32-bit words of the 64-byte digest
// (i.e. ready for sc_reduce512).
TMED_HD void sha512_stream(uint32_t out[16], const uint32_t p0[8], const uint32_t p1[8], int npre,
                           const uint8_t *m, uint32_t mlen) {
  const uint32_t total = (uint32_t)npre + mlen;
  const uint32_t nblocks = (total + 17 + 127) >> 7;
  const uint32_t padded = nblocks << 7;
  const MsgReader rd(m, mlen);
  uint64_t st[8];
  sha512_init(st);
#pragma unroll 1
  for (uint32_t b = 0; b < nblocks; b++) {
    uint64_t w[16];
#pragma unroll
    for (int t = 0; t < 16; t++) w[t] = sha512_stream_word(p0, p1, npre, rd, b * 128 + 8 * t, padded);
    sha512_compress(st, w);
  }
#pragma unroll
  for (int i = 0; i < 8; i++) {
    out[2 * i] = bswap32((uint32_t)(st[i] >> 32));
    out[2 * i + 1] = bswap32((uint32_t)st[i]);
  }
}

// SHA-512(P0 || P1 || M) for M at the start of a 16-B aligned sign-bytes slot (kernels.h
// kVoteSlot = 256 B, readable in full): each 128-B block's message bytes arrive as dwordx4 loads
// (4 for block 0, 8 for block 1) instead of two dword loads per 8-byte word through MsgReader —
// the key-cached prep kernel waited on those loads for about half of its wave time (PMC
// wait_inst_any 0.49).  Bytes past M in the slot are masked exactly as sha512_stream_word does.
// Messages needing a third block (|M| > 175) take sha512_stream.
TMED_HD uint64_t sha512_slot_word(uint32_t a, uint32_t b, int32_t nv) {
  uint64_t v = nv > 0 ? (((uint64_t)bswap32(a) << 32) | bswap32(b)) : 0ull;
  if (nv < 8) {
    if (nv > 0) v &= ~(~0ull >> (8 * nv));
    if (nv >= 0) v |= 0x80ull << (56 - 8 * nv);
  }
  return v;
}

TMED_HD void sha512_stream_slot(uint32_t out[16], const uint32_t p0[8], const uint32_t p1[8], const uint8_t *m,
                                uint32_t mlen) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t total = 64u + mlen;
  const uint32_t nblocks = (total + 17u + 127u) >> 7;
  if (nblocks > 2) {
    sha512_stream(out, p0, p1, 64, m, mlen);
    return;
  }
  const uint4 *q = reinterpret_cast<const uint4 *>(m);
  uint64_t st[8];
  sha512_init(st);
  {
    uint4 c[4];
#pragma unroll
    for (int k = 0; k < 4; k++) c[k] = q[k];  // M[0, 64)
    uint64_t w[16];
#pragma unroll
    for (int t = 0; t < 4; t++) {  // the 64-byte prefix: w[0..3] = P0, w[4..7] = P1
      const uint64_t a = ((uint64_t)bswap32(p0[2 * t]) << 32) | bswap32(p0[2 * t + 1]);
      const uint64_t b = ((uint64_t)bswap32(p1[2 * t]) << 32) | bswap32(p1[2 * t + 1]);
      w[t] = a;
      w[4 + t] = b;
    }
#pragma unroll
    for (int t = 0; t < 8; t++) {
      const uint4 cc = c[t >> 1];
      const uint32_t x = (t & 1) ? cc.z : cc.x, y = (t & 1) ? cc.w : cc.y;
      w[8 + t] = sha512_slot_word(x, y, (int32_t)mlen - 8 * t);
    }
    if (nblocks == 1) w[15] = (uint64_t)total * 8u;
    sha512_compress(st, w);
  }
  if (nblocks == 2) {
    uint4 c[8];
#pragma unroll
    for (int k = 0; k < 8; k++) c[k] = q[4 + k];  // M[64, 192)
    uint64_t w[16];
#pragma unroll
    for (int t = 0; t < 16; t++) {
      const uint4 cc = c[t >> 1];
      const uint32_t x = (t & 1) ? cc.z : cc.x, y = (t & 1) ? cc.w : cc.y;
      w[t] = sha512_slot_word(x, y, (int32_t)mlen - 64 - 8 * t);
    }
    w[15] = (uint64_t)total * 8u;
    sha512_compress(st, w);
  }
#pragma unroll
  for (int i = 0; i < 8; i++) {
    out[2 * i] = bswap32((uint32_t)(st[i] >> 32));
    out[2 * i + 1] = bswap32((uint32_t)st[i]);
  }
#else
  sha512_stream(out, p0, p1, 64, m, mlen);
#endif
}

}  // namespace tmed
