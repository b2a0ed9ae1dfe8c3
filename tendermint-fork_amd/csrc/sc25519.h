// sc25519.h — scalars mod L = 2^252 + 27742317777372353535851937790883648493.
//
// Replaces Go 1.18 edwards25519.Scalar.SetUniformBytes (k = SHA-512(R||A||M)
// mod L) and Scalar.SetCanonicalBytes (reject S >= L), reached from
// crypto/ed25519/ed25519.go:154 in the reference; plus MultiplyAdd for the
// RFC 8032 signer that generates synthetic commits (ed25519.go:57-60).
//
// 32-bit limbs, little-endian.  Reduction is Barrett with mu = floor(2^512/L):
// q = floor(x*mu / 2^512) is at most one below floor(x/L), so one
// conditional subtraction finishes.  Every limb product is one
// v_mad_u64_u32 ((2^32-1)^2 + 2(2^32-1) fits in 64 bits).
#pragma once
#include "fe25519.h"

namespace tmed {

// 32-bit add / subtract with carry (device: the carry-chain builtins, which become one
// v_addc / v_subb each; the 64-bit spelling costs a sign extension and register moves per word).
TMED_HD uint32_t addc32(uint32_t a, uint32_t b, uint32_t cin, uint32_t &cout) {
#if defined(__HIP_DEVICE_COMPILE__)
  unsigned int co;
  const uint32_t r = __builtin_addc(a, b, cin, &co);
  cout = co;
  return r;
#else
  const uint64_t t = (uint64_t)a + b + cin;
  cout = (uint32_t)(t >> 32);
  return (uint32_t)t;
#endif
}
TMED_HD uint32_t subb32(uint32_t a, uint32_t b, uint32_t bin, uint32_t &bout) {
#if defined(__HIP_DEVICE_COMPILE__)
  unsigned int bo;
  const uint32_t r = __builtin_subc(a, b, bin, &bo);
  bout = bo;
  return r;
#else
  const uint64_t d = (uint64_t)a - b - bin;
  bout = (uint32_t)(d >> 63);
  return (uint32_t)d;
#endif
}

TMED_HD void sc_const_L(uint32_t l[8]) {
  const uint32_t c[8] = {0x5cf5d3edu, 0x5812631au, 0xa2f79cd6u, 0x14def9deu, 0u, 0u, 0u, 0x10000000u};
#pragma unroll
  for (int i = 0; i < 8; i++) l[i] = c[i];
}

// r = x mod L for a 512-bit x (16 LE words).
TMED_HD void sc_reduce512(uint32_t r[8], const uint32_t x[16]) {
  const uint32_t mu[9] = {0x0a2c131bu, 0xed9ce5a3u, 0x086329a7u, 0x2106215du, 0xffffffebu,
                          0xffffffffu, 0xffffffffu, 0xffffffffu, 0x0000000fu};
  uint32_t L[8];
  sc_const_L(L);
  // prod = x * mu, row by row (x[i] * mu into prod[i .. i+9]; prod[i+9] is still zero when
  // row i starts); two carry chains per row as in sc_muladd.
  uint32_t prod[25];
#pragma unroll
  for (int i = 0; i < 25; i++) prod[i] = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) {
    uint32_t c1 = 0, c2 = 0, hi = 0;
#pragma unroll
    for (int j = 0; j < 9; j++) {
      const uint64_t p = (uint64_t)x[i] * mu[j];
      const uint32_t u = addc32(prod[i + j], (uint32_t)p, c1, c1);
      prod[i + j] = addc32(u, hi, c2, c2);
      hi = (uint32_t)(p >> 32);
    }
    prod[i + 9] = hi + c1 + c2;
  }
  // q = prod[16..24]; ql = q * L mod 2^288 (the words past 8 are not needed)
  uint32_t ql[9];
#pragma unroll
  for (int i = 0; i < 9; i++) ql[i] = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    uint32_t c1 = 0, c2 = 0, hi = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      if (i + j < 9) {
        const uint64_t p = (uint64_t)prod[16 + i] * L[j];
        const uint32_t u = addc32(ql[i + j], (uint32_t)p, c1, c1);
        ql[i + j] = addc32(u, hi, c2, c2);
        hi = (uint32_t)(p >> 32);
      }
    }
    if (i == 0) ql[8] = hi + c1 + c2;  // rows i >= 1 carry past word 8 only
  }
  uint32_t rr[9], t[9];
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) rr[i] = subb32(x[i], ql[i], borrow, borrow);
  // conditional subtract L (rr < 2L)
  borrow = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) t[i] = subb32(rr[i], i < 8 ? L[i] : 0u, borrow, borrow);
#pragma unroll
  for (int i = 0; i < 8; i++) r[i] = borrow ? rr[i] : t[i];
}

// Go Scalar.SetCanonicalBytes acceptance: s < L.
TMED_HD bool sc_is_canonical(const uint32_t s[8]) {
  uint32_t L[8];
  sc_const_L(L);
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t d = (uint64_t)s[i] - L[i] - borrow;
    borrow = (uint32_t)(d >> 63);
  }
  return borrow != 0;  // s - L < 0
}

// r = (a*b + c) mod L   (RFC 8032 S = r + k*a for the signer)
TMED_HD void sc_muladd(uint32_t r[8], const uint32_t a[8], const uint32_t b[8], const uint32_t c[8]) {
  uint32_t x[16];
#pragma unroll
  for (int i = 0; i < 16; i++) x[i] = i < 8 ? c[i] : 0u;
  // row i adds a[i] * b into x[i .. i+8]; x[i+8] is still zero when row i starts, so the row's
  // carry-out is just stored.  Two carry chains: low halves of a[i] b[j], high halves of a[i] b[j-1].
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint32_t c1 = 0, c2 = 0, hi = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const uint64_t p = (uint64_t)a[i] * b[j];
      const uint32_t u = addc32(x[i + j], (uint32_t)p, c1, c1);
      x[i + j] = addc32(u, hi, c2, c2);
      hi = (uint32_t)(p >> 32);
    }
    x[i + 8] = hi + c1 + c2;  // < 2^32: the row sum fits in nine words
  }
  sc_reduce512(r, x);
}

// Signed radix-16 recoding without a carry loop: r = k + 0x8888...88 (64 nibbles
// of 8).  Digit i is then nibble_i(r) - 8 in [-8, 7], and sum(digit_i 16^i) = k.
// Valid for k < 2^255 (k < L here), so r < 2^256.
TMED_HD void sc_recode16(uint32_t r[8], const uint32_t k[8]) {
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t t = (uint64_t)k[i] + 0x88888888u + c;
    r[i] = (uint32_t)t;
    c = t >> 32;
  }
}

}  // namespace tmed
