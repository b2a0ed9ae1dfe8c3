// kernels.hip — gfx950 kernels: batch ed25519 verify and RFC 8032 sign.
//
// One signature per lane (64 per wave).  The work per signature is ~2.7e5
// 32x32->64 integer multiply-adds, entirely VALU; HBM traffic
// is ~212 B per verify, so the kernel is bound by integer-VALU issue, not by
// memory and not by MFMA (which has no 32x32->64 integer path).
//
// Memory layout
//   pub   n x 32 B, sig n x 64 B (16-B aligned rows -> dwordx4 loads)
//   msgs  concatenated bytes, off[n+1] u32
//   slab  per-lane variable-base table: 9 cached points x 160 B, stored as
//         [entry j][chunk q (16 B)][lane slot] so that lanes of a wave that pick
//         the same entry read contiguous 16-B chunks.
//   btab  9 niels multiples of B, staged once per workgroup in LDS (1080 B).
#include "kernels.h"
#include "verify_core.h"

namespace tmed {

struct SlabTab {
  int4 *base;
  uint32_t stride;  // lane slots in the slab
  uint32_t slot;

  __device__ __forceinline__ void store(int j, const ge_cached &c) const {
    const fe *fs[4] = {&c.YpX, &c.YmX, &c.Z, &c.T2d};
#pragma unroll
    for (int q = 0; q < 10; q++) {
      int32_t w[4];
#pragma unroll
      for (int e = 0; e < 4; e++) {
        const int f = 4 * q + e;
        w[e] = fs[f / 10]->v[f % 10];
      }
      base[(size_t)(j * 10 + q) * stride + slot] = make_int4(w[0], w[1], w[2], w[3]);
    }
  }
  __device__ __forceinline__ void load(int j, ge_cached &c) const {
    fe *fs[4] = {&c.YpX, &c.YmX, &c.Z, &c.T2d};
#pragma unroll
    for (int q = 0; q < 10; q++) {
      const int4 v = base[(size_t)(j * 10 + q) * stride + slot];
      const int32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int e = 0; e < 4; e++) {
        const int f = 4 * q + e;
        fs[f / 10]->v[f % 10] = w[e];
      }
    }
  }
};

struct LdsBTab {
  const ge_niels *t;
  __device__ __forceinline__ void load(int j, ge_niels &n) const { n = t[j]; }
};

constexpr int kBTabEntries = 129;  // j*B, j = 0..128 (niels) — 15.5 KB of LDS

__device__ __forceinline__ void stage_btab(ge_niels *sbt, const ge_niels *btab_g) {
  int32_t *dst = reinterpret_cast<int32_t *>(sbt);
  const int32_t *src = reinterpret_cast<const int32_t *>(btab_g);
  for (int i = threadIdx.x; i < kBTabEntries * 30; i += blockDim.x) dst[i] = src[i];
  __syncthreads();
}

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

// Phase 1: SHA-512(R||A||M) mod L, S < L, A = Point.SetBytes(pub)  (one lane per signature
// of the chunk [base, base + count)).
__global__ __launch_bounds__(kThreadsPerBlock) void verify_prep_kernel(
    const uint8_t *__restrict__ pub, const uint8_t *__restrict__ sig, const uint8_t *__restrict__ msgs,
    const uint32_t *__restrict__ off, uint32_t base, uint32_t count, int4 *__restrict__ prep, uint32_t stride) {
  const uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x;
  if (slot >= count) return;
  const uint32_t i = base + slot;
  uint32_t pw[8], sw[16], k[8], s[8];
  load_row_words(pw, pub + 32 * (size_t)i, 2);
  load_row_words(sw, sig + 64 * (size_t)i, 4);
  const uint32_t o0 = off[i], o1 = off[i + 1];
  ge_p3 A;
  const bool ok = verify_prep(pw, sw, msgs + o0, o1 - o0, k, s, A);
  prep_store(prep, stride, slot, k, s, A, ok);
}

// Phase 2: table of -A, Straus [k](-A) + [s]B, encode, compare with R.
// WAVES = minimum waves per SIMD the register allocation must allow.
template <int WAVES>
__global__ __launch_bounds__(kThreadsPerBlock, WAVES) void verify_main_kernel(
    const uint8_t *__restrict__ sig, uint32_t base, uint32_t count, const int4 *__restrict__ prep,
    uint32_t stride, int4 *__restrict__ slab, const ge_niels *__restrict__ btab_g, uint8_t *__restrict__ out) {
  __shared__ ge_niels sbt[kBTabEntries];
  stage_btab(sbt, btab_g);
  const uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x;
  if (slot >= count) return;
  const uint32_t i = base + slot;
  uint32_t k[8], s[8], Rw[8];
  ge_p3 A;
  const bool ok = prep_load(prep, stride, slot, k, s, A);
  load_row_words(Rw, sig + 64 * (size_t)i, 2);
  SlabTab tab{slab, stride, slot};
  const LdsBTab bt{sbt};
  out[i] = (verify_main(k, s, A, Rw, tab, bt) && ok) ? 1 : 0;
}

__global__ __launch_bounds__(kThreadsPerBlock) void sign_kernel(
    const uint8_t *__restrict__ seeds, const uint8_t *__restrict__ msgs, const uint32_t *__restrict__ off,
    uint32_t n, uint8_t *__restrict__ sig_out, uint8_t *__restrict__ pub_out, int4 *__restrict__ slab,
    uint32_t slab_stride, const ge_niels *__restrict__ btab_g) {
  __shared__ ge_niels sbt[kBTabEntries];
  stage_btab(sbt, btab_g);
  const uint32_t gtid = blockIdx.x * blockDim.x + threadIdx.x;
  const LdsBTab bt{sbt};
  for (uint32_t i = gtid; i < n; i += gridDim.x * blockDim.x) {
    uint32_t seed[8], sg[16], pb[8];
    load_row_words(seed, seeds + 32 * (size_t)i, 2);
    const uint32_t o0 = off[i], o1 = off[i + 1];
    SlabTab t{slab, slab_stride, gtid};
    sign_one(sg, pb, seed, msgs + o0, o1 - o0, t, bt);
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
                         uint32_t n, uint8_t *out, int4 *slab, uint32_t slab_stride, const ge_niels *btab,
                         int4 *prep, hipStream_t stream, uint32_t chunk, int main_waves) {
  // Chunks of at most slab_stride signatures: the per-lane tables (slab) and the
  // prep hand-off are sized for one chunk.
  if (chunk == 0 || chunk > slab_stride) chunk = slab_stride;
  for (uint32_t base = 0; base < n; base += chunk) {
    const uint32_t count = (n - base) < chunk ? (n - base) : chunk;
    const uint32_t blocks = (count + kThreadsPerBlock - 1) / kThreadsPerBlock;
    hipLaunchKernelGGL(verify_prep_kernel, dim3(blocks), dim3(kThreadsPerBlock), 0, stream, pub, sig, msgs, off,
                       base, count, prep, slab_stride);
    if (main_waves >= 3)
      hipLaunchKernelGGL(verify_main_kernel<3>, dim3(blocks), dim3(kThreadsPerBlock), 0, stream, sig, base, count,
                         prep, slab_stride, slab, btab, out);
    else
      hipLaunchKernelGGL(verify_main_kernel<2>, dim3(blocks), dim3(kThreadsPerBlock), 0, stream, sig, base, count,
                         prep, slab_stride, slab, btab, out);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_sign(const uint8_t *seeds, const uint8_t *msgs, const uint32_t *off, uint32_t n, uint8_t *sig_out,
                       uint8_t *pub_out, int4 *slab, uint32_t slab_stride, const ge_niels *btab,
                       hipStream_t stream) {
  const uint32_t grid = grid_for(n, slab_stride / kThreadsPerBlock);
  hipLaunchKernelGGL(sign_kernel, dim3(grid), dim3(kThreadsPerBlock), 0, stream, seeds, msgs, off, n, sig_out,
                     pub_out, slab, slab_stride, btab);
  return hipGetLastError();
}

void host_build_btab(ge_niels out[129]) { build_btab_niels(out); }

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

// One workgroup per (key, window); lane j computes (j+1) * base (verify_core.h comb_entry).
__global__ __launch_bounds__(128) void comb_fill_kernel(const int32_t *__restrict__ bases, uint32_t n,
                                                       int4 *__restrict__ comb) {
  const uint32_t kw = blockIdx.x;  // key * 32 + window
  const uint32_t j = threadIdx.x + 1;  // 1..128
  ge_p3 P;
  p3_load(P, bases + (size_t)kw * 40);
  ge_niels e;
  comb_entry(e, P, j);
  int4 *row = comb + (size_t)kw * kCombEntries * kCombEntryInt4;
  niels_store(row + (size_t)j * kCombEntryInt4, e);
  if (threadIdx.x == 0) {
    ge_niels id;
    ge_niels_0(id);
    niels_store(row, id);
  }
}

struct GlobalComb {
  const int4 *base;  // 32 windows x 129 entries x 8 int4
  __device__ __forceinline__ void load(int w, int j, ge_niels &e) const {
    niels_load(e, base + ((size_t)w * kCombEntries + j) * kCombEntryInt4);
  }
};

__global__ __launch_bounds__(kThreadsPerBlock) void verify_keyset_prep_kernel(
    const uint32_t *__restrict__ val_idx, const uint8_t *__restrict__ key_pub, const uint8_t *__restrict__ key_ok,
    const uint8_t *__restrict__ sig, const uint8_t *__restrict__ msgs, const uint32_t *__restrict__ off,
    uint32_t base, uint32_t count, int4 *__restrict__ prep, uint32_t stride) {
  const uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x;
  if (slot >= count) return;
  const uint32_t i = base + slot;
  const uint32_t v = val_idx[i];
  uint32_t pw[8], sw[16], k[8], s[8];
  load_row_words(pw, key_pub + 32 * (size_t)v, 2);
  load_row_words(sw, sig + 64 * (size_t)i, 4);
  const uint32_t o0 = off[i], o1 = off[i + 1];
  const bool ok = verify_prep_comb(pw, key_ok[v] != 0, sw, msgs + o0, o1 - o0, k, s);
  ge_p3 dummy;
  ge_p3_0(dummy);
  prep_store(prep, stride, slot, k, s, dummy, ok);
}

__global__ __launch_bounds__(kThreadsPerBlock, 2) void verify_keyset_main_kernel(
    const uint32_t *__restrict__ val_idx, const int4 *__restrict__ acomb, const int4 *__restrict__ bcomb,
    const uint8_t *__restrict__ sig, uint32_t base, uint32_t count, const int4 *__restrict__ prep, uint32_t stride,
    uint8_t *__restrict__ out) {
  const uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x;
  if (slot >= count) return;
  const uint32_t i = base + slot;
  const uint32_t v = val_idx[i];
  uint32_t k[8], s[8], Rw[8];
  int32_t w[40];
#pragma unroll
  for (int q = 0; q < 5; q++) {  // k, s, (A unused), ok at word 36
    const int4 x = prep[(size_t)q * stride + slot];
    w[4 * q] = x.x; w[4 * q + 1] = x.y; w[4 * q + 2] = x.z; w[4 * q + 3] = x.w;
  }
  const bool ok = prep[(size_t)9 * stride + slot].x != 0;
#pragma unroll
  for (int j = 0; j < 8; j++) { k[j] = (uint32_t)w[j]; s[j] = (uint32_t)w[8 + j]; }
  load_row_words(Rw, sig + 64 * (size_t)i, 2);
  const GlobalComb ac{acomb + (size_t)v * kCombWindows * kCombEntries * kCombEntryInt4};
  const GlobalComb bc{bcomb};
  out[i] = (verify_main_comb(k, s, Rw, ac, bc) && ok) ? 1 : 0;
}

hipError_t launch_comb_bases(const uint8_t *pubs, uint32_t n, int negate, uint8_t *ok, int32_t *bases,
                             hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(comb_bases_kernel, dim3((n + 63) / 64), dim3(64), 0, stream, pubs, n, negate, ok, bases);
  return hipGetLastError();
}

hipError_t launch_comb_fill(const int32_t *bases, uint32_t n, int4 *comb, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(comb_fill_kernel, dim3(n * kCombWindows), dim3(128), 0, stream, bases, n, comb);
  return hipGetLastError();
}

hipError_t launch_verify_keyset(const uint32_t *val_idx, const uint8_t *key_pub, const uint8_t *key_ok,
                                const int4 *acomb, const int4 *bcomb, const uint8_t *sig, const uint8_t *msgs,
                                const uint32_t *off, uint32_t n, uint8_t *out, int4 *prep, uint32_t stride,
                                hipStream_t stream) {
  for (uint32_t base = 0; base < n; base += stride) {
    const uint32_t count = (n - base) < stride ? (n - base) : stride;
    const uint32_t blocks = (count + kThreadsPerBlock - 1) / kThreadsPerBlock;
    hipLaunchKernelGGL(verify_keyset_prep_kernel, dim3(blocks), dim3(kThreadsPerBlock), 0, stream, val_idx, key_pub,
                       key_ok, sig, msgs, off, base, count, prep, stride);
    hipLaunchKernelGGL(verify_keyset_main_kernel, dim3(blocks), dim3(kThreadsPerBlock), 0, stream, val_idx, acomb,
                       bcomb, sig, base, count, prep, stride, out);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace tmed
