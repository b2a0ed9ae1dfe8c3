/*
 * ed25519_port.c — fast C restatement of Go 1.18 crypto/ed25519.Verify.
 *
 * TEST INFRASTRUCTURE ONLY: the checker for large parity runs and the
 * "port" CPU baseline timed by bench.py.  Never linked into the product.
 *
 * Reference chain restated (third-party to /root/reference):
 *   crypto/ed25519/ed25519.go:148-155  PubKey.VerifySignature (len(sig)!=64 -> false)
 *   golang.org/x/crypto v0.1.0 (go.mod:44) -> Go 1.18 crypto/ed25519.Verify:
 *     sig[63]&0xE0 -> reject; A = Point.SetBytes(pub) (y>=p accepted, x=0 with sign
 *     bit accepted, non-square -> reject); k = SHA-512(R||A||M) mod L;
 *     S >= L -> reject; R' = [k](-A) + [S]B (no cofactor); accept iff
 *     canonical_encode(R') == sig[0:32].
 *   Signing (fixtures): crypto/ed25519/ed25519.go:57-60 -> RFC 8032.
 *
 * Arithmetic: GF(2^255-19) in radix 2^51 (5 x u64, unsigned __int128 products),
 * extended twisted-Edwards coordinates, signed sliding windows (width 5) for
 * both scalars — the same operation shape as Go's VarTimeDoubleScalarBaseMult.
 * Single-threaded per call, like the reference; the batch entry point can fan
 * out over pthreads (used only to report an all-cores upper bound).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

typedef unsigned __int128 u128;

/* ------------------------------------------------------------------ SHA-512 */
static const uint64_t K512[80] = {
  0x428a2f98d728ae22ULL,0x7137449123ef65cdULL,0xb5c0fbcfec4d3b2fULL,0xe9b5dba58189dbbcULL,
  0x3956c25bf348b538ULL,0x59f111f1b605d019ULL,0x923f82a4af194f9bULL,0xab1c5ed5da6d8118ULL,
  0xd807aa98a3030242ULL,0x12835b0145706fbeULL,0x243185be4ee4b28cULL,0x550c7dc3d5ffb4e2ULL,
  0x72be5d74f27b896fULL,0x80deb1fe3b1696b1ULL,0x9bdc06a725c71235ULL,0xc19bf174cf692694ULL,
  0xe49b69c19ef14ad2ULL,0xefbe4786384f25e3ULL,0x0fc19dc68b8cd5b5ULL,0x240ca1cc77ac9c65ULL,
  0x2de92c6f592b0275ULL,0x4a7484aa6ea6e483ULL,0x5cb0a9dcbd41fbd4ULL,0x76f988da831153b5ULL,
  0x983e5152ee66dfabULL,0xa831c66d2db43210ULL,0xb00327c898fb213fULL,0xbf597fc7beef0ee4ULL,
  0xc6e00bf33da88fc2ULL,0xd5a79147930aa725ULL,0x06ca6351e003826fULL,0x142929670a0e6e70ULL,
  0x27b70a8546d22ffcULL,0x2e1b21385c26c926ULL,0x4d2c6dfc5ac42aedULL,0x53380d139d95b3dfULL,
  0x650a73548baf63deULL,0x766a0abb3c77b2a8ULL,0x81c2c92e47edaee6ULL,0x92722c851482353bULL,
  0xa2bfe8a14cf10364ULL,0xa81a664bbc423001ULL,0xc24b8b70d0f89791ULL,0xc76c51a30654be30ULL,
  0xd192e819d6ef5218ULL,0xd69906245565a910ULL,0xf40e35855771202aULL,0x106aa07032bbd1b8ULL,
  0x19a4c116b8d2d0c8ULL,0x1e376c085141ab53ULL,0x2748774cdf8eeb99ULL,0x34b0bcb5e19b48a8ULL,
  0x391c0cb3c5c95a63ULL,0x4ed8aa4ae3418acbULL,0x5b9cca4f7763e373ULL,0x682e6ff3d6b2b8a3ULL,
  0x748f82ee5defb2fcULL,0x78a5636f43172f60ULL,0x84c87814a1f0ab72ULL,0x8cc702081a6439ecULL,
  0x90befffa23631e28ULL,0xa4506cebde82bde9ULL,0xbef9a3f7b2c67915ULL,0xc67178f2e372532bULL,
  0xca273eceea26619cULL,0xd186b8c721c0c207ULL,0xeada7dd6cde0eb1eULL,0xf57d4f7fee6ed178ULL,
  0x06f067aa72176fbaULL,0x0a637dc5a2c898a6ULL,0x113f9804bef90daeULL,0x1b710b35131c471bULL,
  0x28db77f523047d84ULL,0x32caab7b40c72493ULL,0x3c9ebe0a15c9bebcULL,0x431d67c49c100d4cULL,
  0x4cc5d4becb3e42b6ULL,0x597f299cfc657e2aULL,0x5fcb6fab3ad6faecULL,0x6c44198c4a475817ULL};

#define ROR64(x, n) (((x) >> (n)) | ((x) << (64 - (n))))

static void sha512_block(uint64_t st[8], const uint8_t *p) {
  uint64_t w[80];
  for (int i = 0; i < 16; i++) {
    uint64_t v = 0;
    for (int j = 0; j < 8; j++) v = (v << 8) | p[8 * i + j];
    w[i] = v;
  }
  for (int i = 16; i < 80; i++) {
    uint64_t s0 = ROR64(w[i - 15], 1) ^ ROR64(w[i - 15], 8) ^ (w[i - 15] >> 7);
    uint64_t s1 = ROR64(w[i - 2], 19) ^ ROR64(w[i - 2], 61) ^ (w[i - 2] >> 6);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint64_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
  for (int i = 0; i < 80; i++) {
    uint64_t S1 = ROR64(e, 14) ^ ROR64(e, 18) ^ ROR64(e, 41);
    uint64_t ch = (e & f) ^ (~e & g);
    uint64_t t1 = h + S1 + ch + K512[i] + w[i];
    uint64_t S0 = ROR64(a, 28) ^ ROR64(a, 34) ^ ROR64(a, 39);
    uint64_t mj = (a & b) ^ (a & c) ^ (b & c);
    uint64_t t2 = S0 + mj;
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

typedef struct { uint64_t st[8]; uint8_t buf[128]; size_t nbuf; uint64_t total; } sha512_ctx;

static void sha512_init(sha512_ctx *c) {
  static const uint64_t iv[8] = {0x6a09e667f3bcc908ULL,0xbb67ae8584caa73bULL,0x3c6ef372fe94f82bULL,
    0xa54ff53a5f1d36f1ULL,0x510e527fade682d1ULL,0x9b05688c2b3e6c1fULL,0x1f83d9abfb41bd6bULL,0x5be0cd19137e2179ULL};
  memcpy(c->st, iv, sizeof iv); c->nbuf = 0; c->total = 0;
}
static void sha512_update(sha512_ctx *c, const uint8_t *p, size_t n) {
  c->total += n;
  while (n) {
    size_t k = 128 - c->nbuf; if (k > n) k = n;
    memcpy(c->buf + c->nbuf, p, k); c->nbuf += k; p += k; n -= k;
    if (c->nbuf == 128) { sha512_block(c->st, c->buf); c->nbuf = 0; }
  }
}
static void sha512_final(sha512_ctx *c, uint8_t out[64]) {
  uint64_t bits = c->total * 8;
  uint8_t pad = 0x80; sha512_update(c, &pad, 1);
  uint8_t z = 0; while (c->nbuf != 112) sha512_update(c, &z, 1);
  uint8_t len[16] = {0};
  for (int i = 0; i < 8; i++) len[15 - i] = (uint8_t)(bits >> (8 * i));
  sha512_update(c, len, 16);
  for (int i = 0; i < 8; i++) for (int j = 0; j < 8; j++) out[8 * i + j] = (uint8_t)(c->st[i] >> (56 - 8 * j));
}

/* ------------------------------------------------------------ GF(2^255-19) */
typedef struct { uint64_t v[5]; } fe;
#define M51 ((1ULL << 51) - 1)

static uint64_t ld64(const uint8_t *p) { uint64_t v = 0; for (int i = 7; i >= 0; i--) v = (v << 8) | p[i]; return v; }

static void fe_frombytes(fe *h, const uint8_t s[32]) { /* bit 255 ignored, y >= p accepted */
  uint64_t w0 = ld64(s), w1 = ld64(s + 8), w2 = ld64(s + 16), w3 = ld64(s + 24);
  h->v[0] = w0 & M51;
  h->v[1] = ((w0 >> 51) | (w1 << 13)) & M51;
  h->v[2] = ((w1 >> 38) | (w2 << 26)) & M51;
  h->v[3] = ((w2 >> 25) | (w3 << 39)) & M51;
  h->v[4] = (w3 >> 12) & M51;
}
static void fe_carry(fe *h) {
  uint64_t c;
  c = h->v[0] >> 51; h->v[0] &= M51; h->v[1] += c;
  c = h->v[1] >> 51; h->v[1] &= M51; h->v[2] += c;
  c = h->v[2] >> 51; h->v[2] &= M51; h->v[3] += c;
  c = h->v[3] >> 51; h->v[3] &= M51; h->v[4] += c;
  c = h->v[4] >> 51; h->v[4] &= M51; h->v[0] += 19 * c;
  c = h->v[0] >> 51; h->v[0] &= M51; h->v[1] += c;
}
static void fe_tobytes(uint8_t s[32], const fe *f) {
  fe t = *f; fe_carry(&t); fe_carry(&t);
  uint64_t q = (t.v[0] + 19) >> 51;
  q = (t.v[1] + q) >> 51; q = (t.v[2] + q) >> 51; q = (t.v[3] + q) >> 51; q = (t.v[4] + q) >> 51;
  t.v[0] += 19 * q;
  uint64_t c;
  c = t.v[0] >> 51; t.v[0] &= M51; t.v[1] += c;
  c = t.v[1] >> 51; t.v[1] &= M51; t.v[2] += c;
  c = t.v[2] >> 51; t.v[2] &= M51; t.v[3] += c;
  c = t.v[3] >> 51; t.v[3] &= M51; t.v[4] += c;
  t.v[4] &= M51;
  uint64_t w0 = t.v[0] | (t.v[1] << 51);
  uint64_t w1 = (t.v[1] >> 13) | (t.v[2] << 38);
  uint64_t w2 = (t.v[2] >> 26) | (t.v[3] << 25);
  uint64_t w3 = (t.v[3] >> 39) | (t.v[4] << 12);
  for (int i = 0; i < 8; i++) { s[i] = (uint8_t)(w0 >> 8 * i); s[8 + i] = (uint8_t)(w1 >> 8 * i);
    s[16 + i] = (uint8_t)(w2 >> 8 * i); s[24 + i] = (uint8_t)(w3 >> 8 * i); }
}
static void fe_0(fe *h) { memset(h, 0, sizeof *h); }
static void fe_1(fe *h) { fe_0(h); h->v[0] = 1; }
static void fe_add(fe *h, const fe *f, const fe *g) { for (int i = 0; i < 5; i++) h->v[i] = f->v[i] + g->v[i]; fe_carry(h); }
static void fe_sub(fe *h, const fe *f, const fe *g) { /* f + 4p - g, inputs carried (< 2^52) */
  h->v[0] = f->v[0] + 0x1FFFFFFFFFFFB4ULL - g->v[0];
  for (int i = 1; i < 5; i++) h->v[i] = f->v[i] + 0x1FFFFFFFFFFFFCULL - g->v[i];
  fe_carry(h);
}
static void fe_neg(fe *h, const fe *f) { fe z; fe_0(&z); fe_sub(h, &z, f); }
static void fe_mul(fe *h, const fe *f, const fe *g) {
  uint64_t f0 = f->v[0], f1 = f->v[1], f2 = f->v[2], f3 = f->v[3], f4 = f->v[4];
  uint64_t g0 = g->v[0], g1 = g->v[1], g2 = g->v[2], g3 = g->v[3], g4 = g->v[4];
  uint64_t g1_19 = 19 * g1, g2_19 = 19 * g2, g3_19 = 19 * g3, g4_19 = 19 * g4;
  u128 r0 = (u128)f0 * g0 + (u128)f1 * g4_19 + (u128)f2 * g3_19 + (u128)f3 * g2_19 + (u128)f4 * g1_19;
  u128 r1 = (u128)f0 * g1 + (u128)f1 * g0 + (u128)f2 * g4_19 + (u128)f3 * g3_19 + (u128)f4 * g2_19;
  u128 r2 = (u128)f0 * g2 + (u128)f1 * g1 + (u128)f2 * g0 + (u128)f3 * g4_19 + (u128)f4 * g3_19;
  u128 r3 = (u128)f0 * g3 + (u128)f1 * g2 + (u128)f2 * g1 + (u128)f3 * g0 + (u128)f4 * g4_19;
  u128 r4 = (u128)f0 * g4 + (u128)f1 * g3 + (u128)f2 * g2 + (u128)f3 * g1 + (u128)f4 * g0;
  uint64_t c;
  c = (uint64_t)(r0 >> 51); r1 += c; uint64_t h0 = (uint64_t)r0 & M51;
  c = (uint64_t)(r1 >> 51); r2 += c; uint64_t h1 = (uint64_t)r1 & M51;
  c = (uint64_t)(r2 >> 51); r3 += c; uint64_t h2 = (uint64_t)r2 & M51;
  c = (uint64_t)(r3 >> 51); r4 += c; uint64_t h3 = (uint64_t)r3 & M51;
  c = (uint64_t)(r4 >> 51); uint64_t h4 = (uint64_t)r4 & M51;
  h0 += c * 19; c = h0 >> 51; h0 &= M51; h1 += c;
  h->v[0] = h0; h->v[1] = h1; h->v[2] = h2; h->v[3] = h3; h->v[4] = h4;
}
static void fe_sq(fe *h, const fe *f) { fe_mul(h, f, f); }
static void fe_sqn(fe *h, const fe *f, int n) { fe_sq(h, f); for (int i = 1; i < n; i++) fe_sq(h, h); }

/* z^(2^250-1) helper shared by invert and pow22523 */
static void fe_pow250(fe *z250, fe *z11, const fe *z) {
  fe z2, z9, t, z5_0, z10_0, z20_0, z50_0, z100_0;
  fe_sq(&z2, z);
  fe_sqn(&t, &z2, 2); fe_mul(&z9, &t, z);
  fe_mul(z11, &z9, &z2);
  fe_sq(&t, z11); fe_mul(&z5_0, &t, &z9);               /* 2^5 - 1 */
  fe_sqn(&t, &z5_0, 5); fe_mul(&z10_0, &t, &z5_0);      /* 2^10 - 1 */
  fe_sqn(&t, &z10_0, 10); fe_mul(&z20_0, &t, &z10_0);   /* 2^20 - 1 */
  fe_sqn(&t, &z20_0, 20); fe_mul(&t, &t, &z20_0);       /* 2^40 - 1 */
  fe_sqn(&t, &t, 10); fe_mul(&z50_0, &t, &z10_0);       /* 2^50 - 1 */
  fe_sqn(&t, &z50_0, 50); fe_mul(&z100_0, &t, &z50_0);  /* 2^100 - 1 */
  fe_sqn(&t, &z100_0, 100); fe_mul(&t, &t, &z100_0);    /* 2^200 - 1 */
  fe_sqn(&t, &t, 50); fe_mul(z250, &t, &z50_0);         /* 2^250 - 1 */
}
static void fe_invert(fe *out, const fe *z) { /* z^(p-2) = z^(2^255-21) */
  fe z250, z11, t;
  fe_pow250(&z250, &z11, z);
  fe_sqn(&t, &z250, 5); fe_mul(out, &t, &z11);
}
static void fe_pow22523(fe *out, const fe *z) { /* z^((p-5)/8) = z^(2^252-3) */
  fe z250, z11, t;
  fe_pow250(&z250, &z11, z);
  fe_sqn(&t, &z250, 2); fe_mul(out, &t, z);
}
static int fe_isneg(const fe *f) { uint8_t s[32]; fe_tobytes(s, f); return s[0] & 1; }
static int fe_eq(const fe *f, const fe *g) { uint8_t a[32], b[32]; fe_tobytes(a, f); fe_tobytes(b, g); return memcmp(a, b, 32) == 0; }

static const uint8_t D_BYTES[32] = {0xa3,0x78,0x59,0x13,0xca,0x4d,0xeb,0x75,0xab,0xd8,0x41,0x41,0x4d,0x0a,0x70,0x00,
                                    0x98,0xe8,0x79,0x77,0x79,0x40,0xc7,0x8c,0x73,0xfe,0x6f,0x2b,0xee,0x6c,0x03,0x52};
static const uint8_t SQRTM1_BYTES[32] = {0xb0,0xa0,0x0e,0x4a,0x27,0x1b,0xee,0xc4,0x78,0xe4,0x2f,0xad,0x06,0x18,0x43,0x2f,
                                         0xa7,0xd7,0xfb,0x3d,0x99,0x00,0x4d,0x2b,0x0b,0xdf,0xc1,0x4f,0x80,0x24,0x83,0x2b};
static const uint8_t BY_BYTES[32] = {0x58,0x66,0x66,0x66,0x66,0x66,0x66,0x66,0x66,0x66,0x66,0x66,0x66,0x66,0x66,0x66,
                                     0x66,0x66,0x66,0x66,0x66,0x66,0x66,0x66,0x66,0x66,0x66,0x66,0x66,0x66,0x66,0x66};

static fe FE_D, FE_D2, FE_SQRTM1;

/* ------------------------------------------------------------------ points */
typedef struct { fe X, Y, Z, T; } ge_p3;
typedef struct { fe X, Y, Z, T; } ge_p1p1;   /* ((X:Z), (Y:T)) */
typedef struct { fe X, Y, Z; } ge_p2;
typedef struct { fe YpX, YmX, Z, T2d; } ge_cached;

static void p3_0(ge_p3 *h) { fe_0(&h->X); fe_1(&h->Y); fe_1(&h->Z); fe_0(&h->T); }
static void p1p1_to_p2(ge_p2 *r, const ge_p1p1 *p) { fe_mul(&r->X, &p->X, &p->T); fe_mul(&r->Y, &p->Y, &p->Z); fe_mul(&r->Z, &p->Z, &p->T); }
static void p1p1_to_p3(ge_p3 *r, const ge_p1p1 *p) { fe_mul(&r->X, &p->X, &p->T); fe_mul(&r->Y, &p->Y, &p->Z);
  fe_mul(&r->Z, &p->Z, &p->T); fe_mul(&r->T, &p->X, &p->Y); }
static void p3_to_cached(ge_cached *r, const ge_p3 *p) { fe_add(&r->YpX, &p->Y, &p->X); fe_sub(&r->YmX, &p->Y, &p->X);
  r->Z = p->Z; fe_mul(&r->T2d, &p->T, &FE_D2); }
static void p2_dbl(ge_p1p1 *r, const ge_p2 *p) {
  fe xx, yy, b, a, t;
  fe_sq(&xx, &p->X); fe_sq(&yy, &p->Y); fe_sq(&b, &p->Z); fe_add(&b, &b, &b);
  fe_add(&t, &p->X, &p->Y); fe_sq(&a, &t);
  fe_add(&r->Y, &yy, &xx); fe_sub(&r->Z, &yy, &xx); fe_sub(&r->X, &a, &r->Y); fe_sub(&r->T, &b, &r->Z);
}
static void p3_dbl(ge_p1p1 *r, const ge_p3 *p) { ge_p2 q = {p->X, p->Y, p->Z}; p2_dbl(r, &q); }
static void ge_add(ge_p1p1 *r, const ge_p3 *p, const ge_cached *q, int neg) {
  fe a, b, c, d, t;
  fe_add(&t, &p->Y, &p->X); fe_mul(&a, &t, neg ? &q->YmX : &q->YpX);
  fe_sub(&t, &p->Y, &p->X); fe_mul(&b, &t, neg ? &q->YpX : &q->YmX);
  fe_mul(&c, &q->T2d, &p->T);
  fe_mul(&d, &p->Z, &q->Z); fe_add(&d, &d, &d);
  fe_sub(&r->X, &a, &b); fe_add(&r->Y, &a, &b);
  if (neg) { fe_sub(&r->Z, &d, &c); fe_add(&r->T, &d, &c); } else { fe_add(&r->Z, &d, &c); fe_sub(&r->T, &d, &c); }
}

/* Go Point.SetBytes (permissive decode), returns 0 on success. */
static int ge_frombytes(ge_p3 *h, const uint8_t s[32]) {
  fe y, u, v, v3, v7, r, chk, uneg, t;
  fe_frombytes(&y, s);
  fe_sq(&u, &y); fe_mul(&v, &u, &FE_D); fe one; fe_1(&one);
  fe_sub(&u, &u, &one); fe_add(&v, &v, &one);
  /* SqrtRatio(u, v) */
  fe_sq(&t, &v); fe_mul(&v3, &t, &v);
  fe_sq(&t, &v3); fe_mul(&v7, &t, &v);
  fe_mul(&t, &u, &v7); fe_pow22523(&t, &t);
  fe_mul(&r, &u, &v3); fe_mul(&r, &r, &t);
  fe_sq(&t, &r); fe_mul(&chk, &v, &t);
  fe_neg(&uneg, &u);
  int correct = fe_eq(&chk, &u);
  int flipped = fe_eq(&chk, &uneg);
  fe_mul(&t, &uneg, &FE_SQRTM1);
  int flipped_i = fe_eq(&chk, &t);
  if (flipped || flipped_i) fe_mul(&r, &r, &FE_SQRTM1);
  if (fe_isneg(&r)) fe_neg(&r, &r);
  if (!(correct || flipped)) return -1;
  if (s[31] >> 7) fe_neg(&r, &r);
  h->X = r; h->Y = y; fe_1(&h->Z); fe_mul(&h->T, &r, &y);
  return 0;
}
static void ge_tobytes(uint8_t s[32], const fe *X, const fe *Y, const fe *Z) {
  fe zi, x, y;
  fe_invert(&zi, Z); fe_mul(&x, X, &zi); fe_mul(&y, Y, &zi);
  fe_tobytes(s, &y); s[31] |= (uint8_t)(fe_isneg(&x) << 7);
}

/* ------------------------------------------------------------ scalars mod L */
/* L = 2^252 + 27742317777372353535851937790883648493, 64-bit limbs LE */
static const uint64_t LL[4] = {0x5812631a5cf5d3edULL, 0x14def9dea2f79cd6ULL, 0x0ULL, 0x1000000000000000ULL};
/* MU = floor(2^512 / L), 5 limbs */
static const uint64_t MU[5] = {0xed9ce5a30a2c131bULL, 0x2106215d086329a7ULL, 0xffffffffffffffebULL, 0xffffffffffffffffULL, 0xfULL};

/* x: 8 limbs (512-bit LE) -> r = x mod L (4 limbs) via Barrett with mu = floor(2^512/L). */
static void sc_reduce512(uint64_t r[4], const uint64_t x[8]) {
  uint64_t prod[13] = {0};
  for (int i = 0; i < 8; i++) {
    u128 c = 0;
    for (int j = 0; j < 5; j++) {
      c += (u128)x[i] * MU[j] + prod[i + j];
      prod[i + j] = (uint64_t)c; c >>= 64;
    }
    prod[i + 5] += (uint64_t)c;
  }
  /* q = prod >> 512 = limbs 8..12 (q < 2^261) */
  const uint64_t *q = prod + 8;
  uint64_t ql[5] = {0};  /* low 320 bits of q*L */
  for (int i = 0; i < 5; i++) {
    u128 c = 0;
    for (int j = 0; j < 4 && i + j < 5; j++) {
      c += (u128)q[i] * LL[j] + ql[i + j];
      ql[i + j] = (uint64_t)c; c >>= 64;
    }
    if (i + 4 < 5) ql[i + 4] += (uint64_t)c;
  }
  uint64_t rr[5]; u128 bw = 0; /* rr = x - q*L (mod 2^320), < 2L */
  for (int i = 0; i < 5; i++) {
    u128 d = (u128)x[i] - ql[i] - (uint64_t)bw;
    rr[i] = (uint64_t)d; bw = (d >> 64) ? 1 : 0;
  }
  for (int it = 0; it < 2; it++) { /* conditional subtract L */
    uint64_t t[5]; u128 b2 = 0;
    for (int i = 0; i < 5; i++) {
      u128 d = (u128)rr[i] - (i < 4 ? LL[i] : 0) - (uint64_t)b2;
      t[i] = (uint64_t)d; b2 = (d >> 64) ? 1 : 0;
    }
    if (!b2) memcpy(rr, t, sizeof t);
  }
  memcpy(r, rr, 32);
}
static void sc_from_bytes64(uint64_t r[4], const uint8_t h[64]) {
  uint64_t x[8]; for (int i = 0; i < 8; i++) x[i] = ld64(h + 8 * i);
  sc_reduce512(r, x);
}
static int sc_is_canonical(const uint8_t s[32]) {
  uint64_t v[4]; for (int i = 0; i < 4; i++) v[i] = ld64(s + 8 * i);
  for (int i = 3; i >= 0; i--) { if (v[i] < LL[i]) return 1; if (v[i] > LL[i]) return 0; }
  return 0; /* == L */
}
static void sc_muladd(uint64_t r[4], const uint64_t a[4], const uint64_t b[4], const uint64_t c[4]) {
  uint64_t x[8] = {0};
  for (int i = 0; i < 4; i++) { u128 cc = 0;
    for (int j = 0; j < 4; j++) { cc += (u128)a[i] * b[j] + x[i + j]; x[i + j] = (uint64_t)cc; cc >>= 64; }
    x[i + 4] = (uint64_t)cc; }
  u128 cc = 0;
  for (int i = 0; i < 8; i++) { cc += (u128)x[i] + (i < 4 ? c[i] : 0); x[i] = (uint64_t)cc; cc >>= 64; }
  sc_reduce512(r, x);
}
static void sc_tobytes(uint8_t s[32], const uint64_t v[4]) { for (int i = 0; i < 32; i++) s[i] = (uint8_t)(v[i / 8] >> (8 * (i % 8))); }

/* ------------------------------------------------- double-scalar multiplication */
static void slide(signed char *r, const uint8_t *a) {
  for (int i = 0; i < 256; ++i) r[i] = 1 & (a[i >> 3] >> (i & 7));
  for (int i = 0; i < 256; ++i) {
    if (!r[i]) continue;
    for (int b = 1; b <= 6 && i + b < 256; ++b) {
      if (!r[i + b]) continue;
      if (r[i] + (r[i + b] << b) <= 15) { r[i] += r[i + b] << b; r[i + b] = 0; }
      else if (r[i] - (r[i + b] << b) >= -15) {
        r[i] -= r[i + b] << b;
        for (int k = i + b; k < 256; ++k) { if (!r[k]) { r[k] = 1; break; } r[k] = 0; }
      } else break;
    }
  }
}

static ge_cached B_TAB[8];  /* B, 3B, ..., 15B */
static ge_p3 BASE;
static pthread_once_t init_once = PTHREAD_ONCE_INIT;

static void build_odd_table(ge_cached tab[8], const ge_p3 *p) {
  ge_p1p1 t; ge_p3 p2, cur;
  p3_to_cached(&tab[0], p);
  p3_dbl(&t, p); p1p1_to_p3(&p2, &t);
  cur = *p;
  ge_cached c2; p3_to_cached(&c2, &p2);
  for (int i = 1; i < 8; i++) { ge_add(&t, &cur, &c2, 0); p1p1_to_p3(&cur, &t); p3_to_cached(&tab[i], &cur); }
}

static void do_init(void) {
  fe_frombytes(&FE_D, D_BYTES); fe_add(&FE_D2, &FE_D, &FE_D); fe_frombytes(&FE_SQRTM1, SQRTM1_BYTES);
  uint8_t by[32]; memcpy(by, BY_BYTES, 32); /* x of B is even -> sign bit 0 */
  ge_frombytes(&BASE, by);
  build_odd_table(B_TAB, &BASE);
}

/* r = [a]P + [b]B, output as p2 */
static void double_scalarmult(ge_p2 *r, const uint8_t a[32], const ge_p3 *P, const uint8_t b[32]) {
  signed char as[256], bs[256];
  ge_cached Ai[8]; ge_p1p1 t; ge_p3 u;
  slide(as, a); slide(bs, b);
  build_odd_table(Ai, P);
  fe_0(&r->X); fe_1(&r->Y); fe_1(&r->Z);
  int i = 255;
  for (; i >= 0; --i) if (as[i] || bs[i]) break;
  for (; i >= 0; --i) {
    p2_dbl(&t, r);
    if (as[i] > 0) { p1p1_to_p3(&u, &t); ge_add(&t, &u, &Ai[as[i] / 2], 0); }
    else if (as[i] < 0) { p1p1_to_p3(&u, &t); ge_add(&t, &u, &Ai[(-as[i]) / 2], 1); }
    if (bs[i] > 0) { p1p1_to_p3(&u, &t); ge_add(&t, &u, &B_TAB[bs[i] / 2], 0); }
    else if (bs[i] < 0) { p1p1_to_p3(&u, &t); ge_add(&t, &u, &B_TAB[(-bs[i]) / 2], 1); }
    p1p1_to_p2(r, &t);
  }
}

/* ------------------------------------------------------------------ public */
int port_verify(const uint8_t *pub, const uint8_t *msg, size_t mlen, const uint8_t *sig, size_t siglen) {
  pthread_once(&init_once, do_init);
  if (siglen != 64) return 0;                 /* crypto/ed25519/ed25519.go:150 */
  if (sig[63] & 0xE0) return 0;
  ge_p3 A;
  if (ge_frombytes(&A, pub) != 0) return 0;
  sha512_ctx c; uint8_t h[64];
  sha512_init(&c); sha512_update(&c, sig, 32); sha512_update(&c, pub, 32); sha512_update(&c, msg, mlen); sha512_final(&c, h);
  uint64_t k[4]; sc_from_bytes64(k, h);
  if (!sc_is_canonical(sig + 32)) return 0;
  uint8_t kb[32]; sc_tobytes(kb, k);
  ge_p3 negA = A; fe_neg(&negA.X, &A.X); fe_neg(&negA.T, &A.T);
  ge_p2 R; double_scalarmult(&R, kb, &negA, sig + 32);
  uint8_t rb[32]; ge_tobytes(rb, &R.X, &R.Y, &R.Z);
  return memcmp(rb, sig, 32) == 0;
}

/* ZIP-215 (the opt-in cofactored mode; spec/core/encoding.md:52-54 names it, the reference's code
 * does not use it): A and R decoded permissively (Go SetBytes: y >= p and x = 0 with the sign bit
 * accepted), S < L, k = SHA-512(R_bytes || A_bytes || M) mod L, accept iff [8]([S]B - [k]A - R) = O.
 * Parity of this rule with the reference is unpinned (no ZIP-215 code or vectors in it). */
int port_verify_zip215(const uint8_t *pub, const uint8_t *msg, size_t mlen, const uint8_t *sig, size_t siglen) {
  pthread_once(&init_once, do_init);
  if (siglen != 64) return 0;
  ge_p3 A, R;
  if (ge_frombytes(&A, pub) != 0) return 0;
  if (ge_frombytes(&R, sig) != 0) return 0;
  if (!sc_is_canonical(sig + 32)) return 0;
  sha512_ctx c; uint8_t h[64];
  sha512_init(&c); sha512_update(&c, sig, 32); sha512_update(&c, pub, 32); sha512_update(&c, msg, mlen); sha512_final(&c, h);
  uint64_t k[4]; sc_from_bytes64(k, h);
  uint8_t kb[32]; sc_tobytes(kb, k);
  ge_p3 negA = A; fe_neg(&negA.X, &A.X); fe_neg(&negA.T, &A.T);
  ge_p2 Q; double_scalarmult(&Q, kb, &negA, sig + 32);  /* [S]B - [k]A */
  ge_p3 q3;                                               /* (X:Y:Z) -> (XZ : YZ : Z^2 : XY) */
  fe_mul(&q3.X, &Q.X, &Q.Z); fe_mul(&q3.Y, &Q.Y, &Q.Z); fe_mul(&q3.Z, &Q.Z, &Q.Z); fe_mul(&q3.T, &Q.X, &Q.Y);
  ge_cached rc; p3_to_cached(&rc, &R);
  ge_p1p1 t; ge_add(&t, &q3, &rc, 1);                     /* - R */
  ge_p2 d; p1p1_to_p2(&d, &t);
  for (int i = 0; i < 3; i++) { p2_dbl(&t, &d); p1p1_to_p2(&d, &t); }
  fe zero; fe_0(&zero);
  return fe_eq(&d.X, &zero) && fe_eq(&d.Y, &d.Z);
}

static void scalarmult_base(uint8_t out[32], const uint8_t s[32]) {
  uint8_t zero[32] = {0}; ge_p2 R; ge_p3 id; p3_0(&id);
  double_scalarmult(&R, zero, &id, s);
  ge_tobytes(out, &R.X, &R.Y, &R.Z);
}

void port_pubkey_from_seed(const uint8_t seed[32], uint8_t pub[32]) {
  pthread_once(&init_once, do_init);
  sha512_ctx c; uint8_t h[64];
  sha512_init(&c); sha512_update(&c, seed, 32); sha512_final(&c, h);
  h[0] &= 248; h[31] &= 127; h[31] |= 64;
  uint64_t a[4], x[8] = {0}; for (int i = 0; i < 4; i++) x[i] = ld64(h + 8 * i);
  sc_reduce512(a, x); uint8_t ab[32]; sc_tobytes(ab, a);
  scalarmult_base(pub, ab);
}

void port_sign(const uint8_t seed[32], const uint8_t *msg, size_t mlen, uint8_t sig[64]) {
  pthread_once(&init_once, do_init);
  sha512_ctx c; uint8_t h[64], rh[64], kh[64], pub[32];
  sha512_init(&c); sha512_update(&c, seed, 32); sha512_final(&c, h);
  h[0] &= 248; h[31] &= 127; h[31] |= 64;
  uint64_t a[4], x[8] = {0}; for (int i = 0; i < 4; i++) x[i] = ld64(h + 8 * i);
  sc_reduce512(a, x); uint8_t ab[32]; sc_tobytes(ab, a);
  scalarmult_base(pub, ab);
  sha512_init(&c); sha512_update(&c, h + 32, 32); sha512_update(&c, msg, mlen); sha512_final(&c, rh);
  uint64_t r[4]; sc_from_bytes64(r, rh); uint8_t rb[32]; sc_tobytes(rb, r);
  scalarmult_base(sig, rb);
  sha512_init(&c); sha512_update(&c, sig, 32); sha512_update(&c, pub, 32); sha512_update(&c, msg, mlen); sha512_final(&c, kh);
  uint64_t k[4], s[4]; sc_from_bytes64(k, kh);
  sc_muladd(s, k, a, r);
  sc_tobytes(sig + 32, s);
}

/* SHA-512 and mod-L helpers exported for unit tests of the GPU kernels. */
void port_sha512(const uint8_t *m, size_t n, uint8_t out[64]) { sha512_ctx c; sha512_init(&c); sha512_update(&c, m, n); sha512_final(&c, out); }
void port_sc_reduce64(const uint8_t h[64], uint8_t out[32]) { uint64_t r[4]; sc_from_bytes64(r, h); sc_tobytes(out, r); }

/* ------------------------------------------------------------------ batch */
typedef struct {
  const uint8_t *pub, *sig, *msg; const uint64_t *off; const uint32_t *siglen;
  uint8_t *out; size_t lo, hi; int mode; const uint8_t *seeds; uint8_t *sig_out, *pub_out;
} job_t;

static void *worker(void *p) {
  job_t *j = (job_t *)p;
  for (size_t i = j->lo; i < j->hi; i++) {
    const uint8_t *m = j->msg + j->off[i]; size_t ml = (size_t)(j->off[i + 1] - j->off[i]);
    if (j->mode == 0) j->out[i] = (uint8_t)port_verify(j->pub + 32 * i, m, ml, j->sig + 64 * i, j->siglen ? j->siglen[i] : 64);
    else if (j->mode == 2) j->out[i] = (uint8_t)port_verify_zip215(j->pub + 32 * i, m, ml, j->sig + 64 * i, j->siglen ? j->siglen[i] : 64);
    else { port_sign(j->seeds + 32 * i, m, ml, j->sig_out + 64 * i); port_pubkey_from_seed(j->seeds + 32 * i, j->pub_out + 32 * i); }
  }
  return NULL;
}

static void run_jobs(job_t base, size_t n, int nthreads) {
  pthread_once(&init_once, do_init);
  if (nthreads < 1) nthreads = 1;
  if (nthreads == 1 || n < 2) { base.lo = 0; base.hi = n; worker(&base); return; }
  pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * nthreads);
  job_t *jobs = (job_t *)malloc(sizeof(job_t) * nthreads);
  for (int t = 0; t < nthreads; t++) {
    jobs[t] = base; jobs[t].lo = n * t / nthreads; jobs[t].hi = n * (t + 1) / nthreads;
    pthread_create(&th[t], NULL, worker, &jobs[t]);
  }
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  free(th); free(jobs);
}

/* Verify n tuples; msgs concatenated with offsets off[0..n]; siglen may be NULL (all 64). */
void port_verify_batch(const uint8_t *pub, const uint8_t *sig, const uint32_t *siglen, const uint8_t *msg,
                       const uint64_t *off, size_t n, uint8_t *out, int nthreads) {
  job_t b; memset(&b, 0, sizeof b);
  b.pub = pub; b.sig = sig; b.siglen = siglen; b.msg = msg; b.off = off; b.out = out; b.mode = 0;
  run_jobs(b, n, nthreads);
}

/* The same under the ZIP-215 rule (port_verify_zip215). */
void port_verify_batch_zip215(const uint8_t *pub, const uint8_t *sig, const uint32_t *siglen, const uint8_t *msg,
                              const uint64_t *off, size_t n, uint8_t *out, int nthreads) {
  job_t b; memset(&b, 0, sizeof b);
  b.pub = pub; b.sig = sig; b.siglen = siglen; b.msg = msg; b.off = off; b.out = out; b.mode = 2;
  run_jobs(b, n, nthreads);
}

/* Sign n messages with n seeds (RFC 8032), also emitting public keys. */
void port_sign_batch(const uint8_t *seeds, const uint8_t *msg, const uint64_t *off, size_t n,
                     uint8_t *sig_out, uint8_t *pub_out, int nthreads) {
  job_t b; memset(&b, 0, sizeof b);
  b.seeds = seeds; b.msg = msg; b.off = off; b.sig_out = sig_out; b.pub_out = pub_out; b.mode = 1;
  run_jobs(b, n, nthreads);
}
