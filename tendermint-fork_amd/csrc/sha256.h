// sha256.h — SHA-256 for the Merkle kernels (one message per lane).
//
// Replaces crypto/tmhash.Sum (crypto/tmhash/hash.go:19-22, Go crypto/sha256) as used by the
// reference's RFC-6962 Merkle tree (crypto/merkle/hash.go:19-27):
//   leafHash(x)     = SHA-256(0x00 || x)
//   innerHash(l, r) = SHA-256(0x01 || l || r)
//   emptyHash()     = SHA-256("")
// Digests are carried as 8 state words (big-endian word values) between tree levels; bytes
// only at the API boundary.
#pragma once
#include "sha512.h"  // MsgReader, bswap32

namespace tmed {

#if defined(__HIPCC__)
__constant__ static const uint32_t kSha256K[64] = {
#else
static const uint32_t kSha256K[64] = {
#endif
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

TMED_HD uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

TMED_HD void sha256_init(uint32_t st[8]) {
  st[0] = 0x6a09e667u; st[1] = 0xbb67ae85u; st[2] = 0x3c6ef372u; st[3] = 0xa54ff53au;
  st[4] = 0x510e527fu; st[5] = 0x9b05688cu; st[6] = 0x1f83d9abu; st[7] = 0x5be0cd19u;
}

// 64 rounds as 4 x 16 (register-indexed schedule window), constants from a uniform table.
TMED_HD void sha256_compress(uint32_t st[8], uint32_t w[16]) {
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll 1
  for (int r = 0; r < 64; r += 16) {
#pragma unroll
    for (int j = 0; j < 16; j++) {
      if (r > 0) {
        const uint32_t w15 = w[(j + 1) & 15], w2 = w[(j + 14) & 15];
        const uint32_t s0 = rotr32(w15, 7) ^ rotr32(w15, 18) ^ (w15 >> 3);
        const uint32_t s1 = rotr32(w2, 17) ^ rotr32(w2, 19) ^ (w2 >> 10);
        w[j] += s0 + w[(j + 9) & 15] + s1;
      }
      const uint32_t S1 = rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25);
      const uint32_t ch = (e & f) ^ (~e & g);
      const uint32_t t1 = h + S1 + ch + kSha256K[r + j] + w[j];
      const uint32_t S0 = rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22);
      const uint32_t mj = (a & b) ^ (c & (a ^ b));
      h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + S0 + mj;
    }
  }
  st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

// SHA-256(prefix || M): npre = 1 prepends the byte `prefix` (0x00 for a Merkle leaf),
// npre = 0 hashes M alone.  M is read from global memory in aligned dwords (MsgReader;
// nothing past M's last dword is read).
TMED_HD void sha256_prefixed(uint32_t st[8], int npre, uint8_t prefix, const uint8_t *m, uint32_t mlen) {
  const MsgReader rd(m, mlen);
  const uint32_t total = (uint32_t)npre + mlen;
  const uint32_t nblocks = (total + 8 + 1 + 63) >> 6;
  sha256_init(st);
#if defined(__HIP_DEVICE_COMPILE__)
  // Device: each 64-byte block is 17 aligned dwords of M (stream byte p is M[p - npre] at
  // aligned offset r + p - npre), realigned by one v_perm_b32 per word with a lane-constant
  // selector; the next block's dwords are loaded before the current block is compressed, so
  // a long leaf (a 64 KiB part) streams instead of waiting on every load.
  const int32_t sh = (int32_t)rd.r - npre;                     // aligned offset of stream byte 0
  const uint32_t s = (uint32_t)sh & 3u;
  const uint32_t sel = (s << 24) | ((s + 1) << 16) | ((s + 2) << 8) | (s + 3);
  auto fetch = [&](uint32_t b, uint32_t D[17]) {
    const int32_t q0 = (sh + (int32_t)(64 * b)) >> 2;          // floor division (sh may be -1)
#pragma unroll
    for (int k = 0; k < 17; k++) {
      const int32_t q = q0 + k;
      D[k] = (q >= 0 && (uint32_t)q < rd.ndw) ? rd.base[q] : 0u;
    }
  };
  uint32_t Dn[17];
  fetch(0, Dn);
#pragma unroll 1
  for (uint32_t b = 0; b < nblocks; b++) {
    uint32_t D[17], w[16];
#pragma unroll
    for (int k = 0; k < 17; k++) D[k] = Dn[k];
    if (b + 1 < nblocks) fetch(b + 1, Dn);
#pragma unroll
    for (int t = 0; t < 16; t++) {
      const uint32_t pos = b * 64 + 4 * t;
      uint32_t v = __builtin_amdgcn_perm(D[t + 1], D[t], sel);
      if (npre && pos == 0) v = ((uint32_t)prefix << 24) | (v & 0x00ffffffu);
      const int32_t nv = (int32_t)total - (int32_t)pos;
      if (nv < 4) {
        if (nv > 0) v &= ~(0xffffffffu >> (8 * nv));
        else v = 0;
        if (nv >= 0) v |= 0x80u << (24 - 8 * nv);
      }
      if (b == nblocks - 1 && t == 14) v = total >> 29;
      if (b == nblocks - 1 && t == 15) v = total << 3;
      w[t] = v;
    }
    sha256_compress(st, w);
  }
  return;
#endif
  uint32_t prev = 0;  // npre = 1: be32 of M[pos-4 .. pos) (its low byte opens the next word)
#pragma unroll 1
  for (uint32_t b = 0; b < nblocks; b++) {
    uint32_t w[16];
#pragma unroll
    for (int t = 0; t < 16; t++) {
      const uint32_t pos = b * 64 + 4 * t;  // stream position of the word
      uint32_t v;
      if (npre) {
        // stream bytes pos..pos+3 = prefix-or-M[pos-1], M[pos .. pos+2]
        const uint32_t cur = (pos < mlen) ? rd.be32(pos) : 0u;
        v = ((pos == 0 ? (uint32_t)prefix : prev) << 24) | (cur >> 8);
        prev = cur;
      } else {
        v = (pos < mlen) ? rd.be32(pos) : 0u;
      }
      // stream bytes at positions >= total: 0x80 then zeros
      const int32_t nv = (int32_t)total - (int32_t)pos;
      if (nv < 4) {
        if (nv > 0) v &= ~(0xffffffffu >> (8 * nv));
        else v = 0;
        if (nv >= 0) v |= 0x80u << (24 - 8 * nv);
      }
      if (b == nblocks - 1 && t == 14) v = total >> 29;     // bit length, high word
      if (b == nblocks - 1 && t == 15) v = total << 3;      // bit length, low word
      w[t] = v;
    }
    sha256_compress(st, w);
  }
}

// innerHash(l, r) = SHA-256(0x01 || l || r) on digests held as state words.
TMED_HD void sha256_inner(uint32_t st[8], const uint32_t l[8], const uint32_t r[8]) {
  uint32_t w[16];
  w[0] = 0x01000000u | (l[0] >> 8);
#pragma unroll
  for (int i = 1; i < 8; i++) w[i] = (l[i - 1] << 24) | (l[i] >> 8);
  w[8] = (l[7] << 24) | (r[0] >> 8);
#pragma unroll
  for (int i = 9; i < 16; i++) w[i] = (r[i - 9] << 24) | (r[i - 8] >> 8);
  sha256_init(st);
  sha256_compress(st, w);
  // second block: r's last byte, 0x80, zeros, bit length 65 * 8 = 520
  w[0] = (r[7] << 24) | 0x00800000u;
#pragma unroll
  for (int i = 1; i < 15; i++) w[i] = 0;
  w[15] = 520;
  sha256_compress(st, w);
}

}  // namespace tmed
