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

__global__ __launch_bounds__(kThreadsPerBlock) void verify_kernel(
    const uint8_t *__restrict__ pub, const uint8_t *__restrict__ sig, const uint8_t *__restrict__ msgs,
    const uint32_t *__restrict__ off, uint32_t n, uint8_t *__restrict__ out, int4 *__restrict__ slab,
    uint32_t slab_stride, const ge_niels *__restrict__ btab_g) {
  __shared__ ge_niels sbt[9];
  {
    int32_t *dst = reinterpret_cast<int32_t *>(sbt);
    const int32_t *src = reinterpret_cast<const int32_t *>(btab_g);
    for (int i = threadIdx.x; i < 9 * 30; i += blockDim.x) dst[i] = src[i];
  }
  __syncthreads();
  const uint32_t gtid = blockIdx.x * blockDim.x + threadIdx.x;
  const SlabTab tab{slab, slab_stride, gtid};
  const LdsBTab bt{sbt};
  for (uint32_t i = gtid; i < n; i += gridDim.x * blockDim.x) {
    uint32_t pw[8], sw[16];
    load_row_words(pw, pub + 32 * (size_t)i, 2);
    load_row_words(sw, sig + 64 * (size_t)i, 4);
    const uint32_t o0 = off[i], o1 = off[i + 1];
    SlabTab t = tab;
    out[i] = verify_one(pw, sw, msgs + o0, o1 - o0, t, bt) ? 1 : 0;
  }
}

__global__ __launch_bounds__(kThreadsPerBlock) void sign_kernel(
    const uint8_t *__restrict__ seeds, const uint8_t *__restrict__ msgs, const uint32_t *__restrict__ off,
    uint32_t n, uint8_t *__restrict__ sig_out, uint8_t *__restrict__ pub_out, int4 *__restrict__ slab,
    uint32_t slab_stride, const ge_niels *__restrict__ btab_g) {
  __shared__ ge_niels sbt[9];
  {
    int32_t *dst = reinterpret_cast<int32_t *>(sbt);
    const int32_t *src = reinterpret_cast<const int32_t *>(btab_g);
    for (int i = threadIdx.x; i < 9 * 30; i += blockDim.x) dst[i] = src[i];
  }
  __syncthreads();
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
                         hipStream_t stream) {
  const uint32_t grid = grid_for(n, slab_stride / kThreadsPerBlock);
  hipLaunchKernelGGL(verify_kernel, dim3(grid), dim3(kThreadsPerBlock), 0, stream, pub, sig, msgs, off, n, out,
                     slab, slab_stride, btab);
  return hipGetLastError();
}

hipError_t launch_sign(const uint8_t *seeds, const uint8_t *msgs, const uint32_t *off, uint32_t n, uint8_t *sig_out,
                       uint8_t *pub_out, int4 *slab, uint32_t slab_stride, const ge_niels *btab,
                       hipStream_t stream) {
  const uint32_t grid = grid_for(n, slab_stride / kThreadsPerBlock);
  hipLaunchKernelGGL(sign_kernel, dim3(grid), dim3(kThreadsPerBlock), 0, stream, seeds, msgs, off, n, sig_out,
                     pub_out, slab, slab_stride, btab);
  return hipGetLastError();
}

void host_build_btab(ge_niels out[9]) { build_btab_niels(out); }

}  // namespace tmed
