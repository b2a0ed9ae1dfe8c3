// Probe of the HIP virtual-memory calls on the box (round 5, the key pool grown in place): which
// of hipMemCreate / hipMemMap / hipMemSetAccess accepts a second physical chunk mapped at an offset
// inside one reserved range, for small and multi-GB chunks, and whether a kernel then sees the data.
// Build: hipcc --offload-arch=gfx950 -O2 profiles/r05/recipes/vmm_probe.cpp -o profiles/r05/recipes/vmm_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include <vector>

__global__ void fill(uint32_t *p, size_t n, uint32_t tag) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = tag ^ (uint32_t)i;
}
__global__ void check(const uint32_t *p, size_t n, uint32_t tag, unsigned long long *bad) {
  unsigned long long b = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    b += p[i] != (tag ^ (uint32_t)i);
  if (b) atomicAdd(bad, b);
}

static hipMemAllocationProp prop() {
  hipMemAllocationProp p;
  memset(&p, 0, sizeof p);
  p.type = hipMemAllocationTypePinned;
  p.location.type = hipMemLocationTypeDevice;
  p.location.id = 0;
  return p;
}

// reserve `total`, map chunks of the given sizes one after another; setaccess per chunk (mode 0)
// or over everything mapped so far (mode 1)
static void run(const char *name, size_t total, std::vector<size_t> chunks, int mode) {
  hipMemAllocationProp p = prop();
  void *base = nullptr;
  hipError_t e = hipMemAddressReserve(&base, total, 0, nullptr, 0);
  printf("%s: reserve %zu MB -> %s\n", name, total >> 20, hipGetErrorString(e));
  if (e != hipSuccess) return;
  size_t off = 0;
  std::vector<std::pair<hipMemGenericAllocationHandle_t, size_t>> hs;
  for (size_t sz : chunks) {
    hipMemGenericAllocationHandle_t h;
    hipError_t ec = hipMemCreate(&h, sz, &p, 0);
    hipError_t em = ec == hipSuccess ? hipMemMap((char *)base + off, sz, 0, h, 0) : ec;
    hipMemAccessDesc ad;
    memset(&ad, 0, sizeof ad);
    ad.location = p.location;
    ad.flags = hipMemAccessFlagsProtReadWrite;
    hipError_t ea = em == hipSuccess ? (mode == 0 ? hipMemSetAccess((char *)base + off, sz, &ad, 1)
                                                 : hipMemSetAccess(base, off + sz, &ad, 1))
                                     : em;
    printf("  chunk at +%zu MB, %zu MB: create %s, map %s, access %s\n", off >> 20, sz >> 20, hipGetErrorString(ec),
           hipGetErrorString(em), hipGetErrorString(ea));
    (void)hipGetLastError();
    if (ec == hipSuccess) hs.emplace_back(h, em == hipSuccess ? sz : 0);
    if (ea != hipSuccess) break;
    off += sz;
  }
  if (off) {
    unsigned long long *bad;
    (void)hipMalloc(&bad, 8);
    (void)hipMemset(bad, 0, 8);
    fill<<<1024, 256>>>((uint32_t *)base, off / 4, 0x5eed);
    check<<<1024, 256>>>((const uint32_t *)base, off / 4, 0x5eed, bad);
    unsigned long long h = 0;
    hipError_t ek = hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost);
    printf("  kernel over %zu MB mapped: %s, %llu mismatches\n", off >> 20, hipGetErrorString(ek), h);
    (void)hipFree(bad);
  }
  size_t o2 = 0;
  for (auto &x : hs) {
    if (x.second) (void)hipMemUnmap((char *)base + o2, x.second);
    (void)hipMemRelease(x.first);
    o2 += x.second;
  }
  (void)hipMemAddressFree(base, total);
  (void)hipGetLastError();
}

int main() {
  hipMemAllocationProp p = prop();
  size_t gmin = 0, grec = 0;
  (void)hipMemGetAllocationGranularity(&gmin, &p, hipMemAllocationGranularityMinimum);
  (void)hipMemGetAllocationGranularity(&grec, &p, hipMemAllocationGranularityRecommended);
  printf("granularity min %zu rec %zu\n", gmin, grec);
  const size_t MB = 1 << 20, GB = 1ull << 30;
  run("small per-chunk access", 64 * MB, {2 * MB, 2 * MB, 4 * MB}, 0);
  run("small whole access", 64 * MB, {2 * MB, 2 * MB, 4 * MB}, 1);
  run("rec-gran chunks", 16 * grec, {grec, grec, 2 * grec}, 0);
  run("GB chunks per-chunk", 32 * GB, {5 * GB + 256 * MB, 5 * GB + 512 * MB}, 0);
  run("GB chunks whole", 32 * GB, {5 * GB + 256 * MB, 5 * GB + 512 * MB}, 1);
  run("odd size", 32 * GB, {5280 * MB + 2 * MB, 5380 * MB}, 0);
  // the key pool's own sizes (radix-256 comb 528,384 B a key: 10,000 keys, then 10,176 more)
  run("pool 4K-multiple", 26 * GB, {10000ull * 528384, 10176ull * 528384}, 0);
  const size_t M2 = 2 * MB;
  run("pool 2M-rounded", 26 * GB, {(10000ull * 528384 + M2 - 1) / M2 * M2, (10176ull * 528384 + M2 - 1) / M2 * M2}, 0);
  run("small 4K-multiple", 1 * GB, {64ull * 528384, 64ull * 528384}, 0);
  run("4K offset under 4G", 8 * GB, {3 * GB + 4096, 1 * GB}, 0);
  run("4K offset over 4G", 16 * GB, {5 * GB + 4096, 1 * GB}, 0);
  run("2M offset over 4G, 4K size", 16 * GB, {5 * GB, 1 * GB + 4096}, 0);
  return 0;
}
