// tmed_capi.hip — C ABI (include/tmed25519.h) over the gfx950 kernels.
//
// Host runtime: one context per GPU (one process per GPU), a private HIP
// stream, grow-only device buffers and pinned host staging buffers reused
// across calls, and a mutex so a context can be shared by concurrent callers
// (the reference's callers — blocksync, light client, evidence pool — run on
// different goroutines; ValidatorSet itself is not goroutine-safe,
// types/validator_set.go:49, so no shared mutable state crosses the seam).
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <string>

#include "../../include/tmed25519.h"
#include "kernels.h"

#include "ctx.h"

using namespace tmed;

extern "C" {

int tmed_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

const char *tmed_strerror(int code) {
  switch (code) {
    case TMED_OK: return "ok";
    case TMED_EINVAL: return "invalid argument";
    case TMED_ENODEV: return "no usable gfx950 HIP device";
    case TMED_EHIP: return "HIP runtime error";
    case TMED_ENOMEM: return "out of memory";
    case TMED_ENOKEYSET: return "unknown key-set handle";
    case TMED_EINTERNAL: return "internal error (host-side exception in the library)";
    default: return "unknown error";
  }
}

// The fixed-base tables of B too large to keep per context, the same for every context of a device:
// built by the first context that needs them, shared, freed with the last.
//   kind 0: the radix-2^26 tables of the default path (kernels.h kB26Bytes, 8.6 GB), at tmed_init;
//   kind 1: the radix-2^24 comb of the key-cached throughput kernel (kB24Bytes, 11.8 GB), at the
//           context's first tmed_keyset_load.
// TMED_B26=0 / TMED_B24=0, or an allocation that fails, leaves that path on the context's own
// radix-2^16 comb (same decisions).
namespace {
struct BShare {
  int4 *p = nullptr;
  int refs = 0;
};
std::mutex g_bshare_mu;
BShare g_bshare[2][64];
}  // namespace

// Pinned caller memory (tmed_host_alloc / tmed_host_register): [start, end) ranges, looked up per
// candidate run while a large seam batch is staged (host_pinned, ctx.h).
namespace {
std::mutex g_pin_mu;
std::map<uintptr_t, uintptr_t> g_pinned;  // start -> end
}  // namespace

extern "C++" {
namespace tmed {
bool host_pinned(const void *p, size_t bytes) {
  const uintptr_t a = (uintptr_t)p, b = a + bytes;
  std::lock_guard<std::mutex> lk(g_pin_mu);
  auto it = g_pinned.upper_bound(a);
  if (it == g_pinned.begin()) return false;
  --it;
  return a >= it->first && b <= it->second;
}
}  // namespace tmed
}

static bool env_off(const char *name) {
  const char *v = getenv(name);
  return v && v[0] == '0';
}

static int4 *bshare_acquire(int kind, int device, const int4 *comb16, hipStream_t s) {
  if (device < 0 || device >= 64) return nullptr;
  std::lock_guard<std::mutex> lk(g_bshare_mu);
  BShare &b = g_bshare[kind][device];
  if (!b.p) {
    int4 *p = nullptr;
    if (hipMalloc((void **)&p, kind == 0 ? kB26Bytes : kB24Bytes) != hipSuccess) {
      (void)hipGetLastError();
      return nullptr;
    }
    const hipError_t e = kind == 0 ? launch_build_b26(comb16, p, s) : launch_build_b24(comb16, p, s);
    if (e != hipSuccess || hipStreamSynchronize(s) != hipSuccess) {
      (void)hipFree(p);
      return nullptr;
    }
    b.p = p;
  }
  b.refs++;
  return b.p;
}

static void bshare_release(int kind, int device, int4 *p) {
  if (!p) return;
  std::lock_guard<std::mutex> lk(g_bshare_mu);
  BShare &b = g_bshare[kind][device];
  if (b.p == p && --b.refs == 0) {
    (void)hipFree(b.p);
    b.p = nullptr;
  }
}

extern "C++" {
namespace tmed {
const int4 *ctx_bcomb24(tmed_ctx *c) {
  if (!c->b24_tried && c->b24_on) {
    c->b24_tried = true;
    c->d_b24 = bshare_acquire(1, c->device, c->d_bcomb16, c->stream);
  }
  return c->d_b24;
}
}  // namespace tmed
}  // extern "C++"

int tmed_init(int device, tmed_ctx **out) {
  if (!out) return TMED_EINVAL;
  *out = nullptr;
  int ndev = tmed_device_count();
  if (device < 0 || device >= ndev) return TMED_ENODEV;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return TMED_EHIP;
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return TMED_ENODEV;  // code objects are gfx950-only
  if (hipSetDevice(device) != hipSuccess) return TMED_EHIP;
  tmed_ctx *c = new tmed_ctx();
  c->device = device;
  hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreate(&c->ev0);
  if (e == hipSuccess) e = hipEventCreate(&c->ev1);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->scratch_ev, hipEventDisableTiming);
  // Lane slots for the per-lane tables and the prep hand-off: 2^20 signatures per
  // prep/main pair (default path: 3.0 GB slab of two tables + 369 MB hand-off, of the 288 GB
  // HBM), so a BASELINE C2 batch is one launch of each kernel: +2.6 % over 131,072-signature
  // chunks, which paid a drain/ramp bubble per launch (profiles/r01/session2/variants_chunk.txt).
  // Both sizes are kept multiples of the block size (every lane of a launched block owns a slot
  // of the slab; a zero size would never make progress).
  auto round_up = [](uint32_t v) {
    if (v < kThreadsPerBlock) v = kThreadsPerBlock;
    if (v > (1u << 24)) v = 1u << 24;
    return (v + kThreadsPerBlock - 1) / kThreadsPerBlock * kThreadsPerBlock;
  };
  c->slab_slots = 4096 * kThreadsPerBlock;
  c->chunk = c->slab_slots;
  if (const char *v = getenv("TMED_SLAB_SLOTS")) c->slab_slots = round_up((uint32_t)strtoul(v, nullptr, 10));
  c->chunk = c->slab_slots;
  if (const char *v = getenv("TMED_CHUNK")) c->chunk = std::min(c->slab_slots, round_up((uint32_t)strtoul(v, nullptr, 10)));
  if (const char *v = getenv("TMED_MAIN_WAVES")) c->main_waves = atoi(v) == 5 ? 5 : 6;
  if (const char *v = getenv("TMED_LAT_MAX")) c->lat_max = (uint32_t)strtoul(v, nullptr, 10);
  if (c->lat_max > kLatMax) c->lat_max = kLatMax;
  if (const char *v = getenv("TMED_GLAT_MAX")) c->glat_max = (uint32_t)strtoul(v, nullptr, 10);
  if (c->glat_max > kGLatMax) c->glat_max = kGLatMax;
  if (e == hipSuccess)
    e = hipMalloc((void **)&c->d_slab, (size_t)c->slab_slots * kSlabSlotBytes * slab_tables(c->main_waves));
  if (e == hipSuccess) e = hipMalloc((void **)&c->d_prep, (size_t)c->slab_slots * kPrepSlotBytes + kPrepTailBytes);
  if (e == hipSuccess) e = hipMalloc((void **)&c->d_fin, kFinBytes);          // 128 MB: projective R'
  if (e == hipSuccess) e = hipMalloc((void **)&c->d_fin_pre, kFinPreBytes);   // 48 MB: prefix products
  if (e == hipSuccess) e = hipMalloc((void **)&c->d_glat, kGLatHandBytes);     // 20 MB: latency-mode hand-off
  // Shared signed radix-256 comb of +B (528 KB, L2-resident) for the key-cached path.
  uint8_t *d_bpub = nullptr, *d_bok = nullptr;
  const uint8_t benc[32] = {0x58, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66,
                            0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66,
                            0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66};
  if (e == hipSuccess) e = hipMalloc((void **)&c->d_b16, kB16Bytes);
  if (e == hipSuccess) e = launch_build_b16(c->d_b16, c->stream);
  if (e == hipSuccess) e = hipMalloc((void **)&c->d_bcomb16, kBComb16Bytes);
  {
    static int32_t bases[16 * 40];
    static std::once_flag bases_once;
    std::call_once(bases_once, [] { host_bcomb16_bases(bases); });
    int32_t *d_bases = nullptr;
    if (e == hipSuccess) e = hipMalloc((void **)&d_bases, sizeof(bases));
    if (e == hipSuccess) e = hipMemcpy(d_bases, bases, sizeof(bases), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = launch_build_bcomb16(d_bases, c->d_bcomb16, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (d_bases) (void)hipFree(d_bases);
  }
  // TMED_B26 / TMED_B24 are read here, per context (a process may hold contexts of both kinds)
  if (e == hipSuccess && !env_off("TMED_B26")) c->d_b26 = bshare_acquire(0, device, c->d_bcomb16, c->stream);
  c->b24_on = !env_off("TMED_B24");
  c->acomb_on = !env_off("TMED_KS_ACOMB");
  if (const char *v = getenv("TMED_TEST_FAIL_KS_ALLOC")) c->test_fail_ks_alloc = atoi(v);
  c->kc_on = !env_off("TMED_KEYCACHE");
  if (const char *v = getenv("TMED_KEYCACHE_GB")) c->kc_budget = (size_t)strtoull(v, nullptr, 10) << 30;
  if (e == hipSuccess) e = hipMalloc((void **)&c->d_bcomb, kCombBytesPerKey);
  if (e == hipSuccess) e = hipMalloc((void **)&d_bpub, 32);
  if (e == hipSuccess) e = hipMalloc((void **)&d_bok, 1);
  if (e == hipSuccess) e = hipMemcpy(d_bpub, benc, 32, hipMemcpyHostToDevice);
  int rc = map_err(e);
  if (rc == TMED_OK) rc = build_comb(c, d_bpub, 1, /*negate=*/0, d_bok, c->d_bcomb);
  if (d_bpub) (void)hipFree(d_bpub);
  if (d_bok) (void)hipFree(d_bok);
  if (rc != TMED_OK) {
    tmed_destroy(c);
    return rc;
  }
  *out = c;
  return TMED_OK;
}

void tmed_destroy(tmed_ctx *c) {
  if (!c) return;
  hipSetDevice(c->device);
  if (c->stream) hipStreamSynchronize(c->stream);
  if (c->copy_stream) hipStreamSynchronize(c->copy_stream);
  bs_destroy(c);  // submitted blocksync windows never waited for (their cache pins go with them)
  // The key-build worker (woken by any generic call that queued keys, and by bs_destroy's
  // unpins) uses the staging buffers, events and streams below: join it before anything is freed.
  keycache_destroy(c);
  if (c->stream) hipStreamSynchronize(c->stream);
  if (c->lane1.s) hipStreamSynchronize(c->lane1.s);
  lane_release(c->lane1);
  for (DevBuf *b : {&c->d_a, &c->d_b, &c->d_msg, &c->d_off, &c->d_out, &c->d_c}) b->release();
  for (HostBuf *b : {&c->h_a, &c->h_b, &c->h_msg, &c->h_off, &c->h_out, &c->h_c}) b->release();
  for (DevBuf *b : {&c->d_merkle_a, &c->d_merkle_b, &c->d_merkle_idx, &c->d_korder, &c->d_zip, &c->d_kbases})
    b->release();
  c->h_kup.release();
  if (c->kup_ev) hipEventDestroy(c->kup_ev);
  c->h_zip.release();
  if (c->zip_ev) hipEventDestroy(c->zip_ev);
  if (c->trace_t0) hipEventDestroy(c->trace_t0);
  for (VoteSlot &v : c->vslot) {
    for (DevBuf *b : {&v.d_votes, &v.d_vmsg, &v.d_off, &v.d_out}) b->release();
    for (HostBuf *b : {&v.h_votes, &v.h_out}) b->release();
    if (v.ev0) hipEventDestroy(v.ev0);
    if (v.ev1) hipEventDestroy(v.ev1);
    if (v.done) hipEventDestroy(v.done);
    if (v.copied) hipEventDestroy(v.copied);
    if (v.cp0) hipEventDestroy(v.cp0);
    if (v.cp1) hipEventDestroy(v.cp1);
  }
  for (auto &kv : c->keysets) free_keyset(kv.second);
  c->keysets.clear();
  if (c->scratch_ev) hipEventDestroy(c->scratch_ev);
  if (c->d_bcomb) hipFree(c->d_bcomb);
  if (c->d_b16) hipFree(c->d_b16);
  if (c->d_bcomb16) hipFree(c->d_bcomb16);
  bshare_release(0, c->device, c->d_b26);
  bshare_release(1, c->device, c->d_b24);
  if (c->d_slab) hipFree(c->d_slab);
  if (c->d_prep) hipFree(c->d_prep);
  if (c->d_fin) hipFree(c->d_fin);
  if (c->d_fin_pre) hipFree(c->d_fin_pre);
  if (c->d_glat) hipFree(c->d_glat);
  if (c->ev0) hipEventDestroy(c->ev0);
  if (c->ev1) hipEventDestroy(c->ev1);
  if (c->stream) hipStreamDestroy(c->stream);
  if (c->copy_stream) hipStreamDestroy(c->copy_stream);
  delete c;
}

float tmed_last_kernel_ms(tmed_ctx *c) { return c ? c->last_ms : 0.f; }

int tmed_set_kernel_timing(tmed_ctx *c, int on) {
  if (!c) return TMED_EINVAL;
  std::lock_guard<std::mutex> lk(c->mu);
  (void)hipSetDevice(c->device);
  if (on && !c->timing)
    for (auto &e : c->timer.ev)
      if (hipEventCreate(&e) != hipSuccess) return TMED_EHIP;
  if (!on && c->timing)
    for (auto &e : c->timer.ev) (void)hipEventDestroy(e);
  c->timing = on != 0;
  c->timer.n = 0;
  return TMED_OK;
}

int tmed_kernel_times(tmed_ctx *c, float ms[3], int launches[3]) {
  if (!c || !ms || !launches || !c->timing) return TMED_EINVAL;
  for (int k = 0; k < 3; k++) { ms[k] = 0.f; launches[k] = 0; }
  if (c->timer.n > 0 && hipEventSynchronize(c->timer.ev[c->timer.n - 1]) != hipSuccess) return TMED_EHIP;
  for (int i = 1; i < c->timer.n; i++) {
    const int k = c->timer.kind[i];
    if (k < 0 || k > 2) continue;
    float t = 0.f;
    (void)hipEventElapsedTime(&t, c->timer.ev[i - 1], c->timer.ev[i]);
    ms[k] += t;
    launches[k] += 1;
  }
  return TMED_OK;
}

int tmed_verify_batch_device(tmed_ctx *c, const uint8_t *d_pub, const uint8_t *d_sig, const uint8_t *d_msgs,
                             const uint32_t *d_off, size_t n, uint8_t *d_out, void *stream) {
  if (!c) return TMED_EINVAL;
  if (n == 0) return TMED_OK;
  if (!d_pub || !d_sig || !d_msgs || !d_off || !d_out || n > 0xffffffffu) return TMED_EINVAL;
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  std::lock_guard<std::mutex> lk(c->mu);
  hipSetDevice(c->device);
  if (c->timing) c->timer.n = 0;
  hipError_t e = scratch_acquire(c, s);
  // (one lane: split over the two kernel lanes in halves, a 2^20 batch ran at the same rate —
  // 107.8 against 108.4 M/s over three alternating runs, profiles/r04/s14/ — and is not done)
  if (e == hipSuccess)
    e = generic_verify(c, d_pub, d_sig, d_msgs, d_off, (uint32_t)n, d_out, s, false, c->timing ? &c->timer : nullptr);
  if (e == hipSuccess) e = scratch_release(c, s);
  return map_err(e);
}

int tmed_host_alloc(size_t bytes, void **p) {
  if (!p || bytes == 0) return TMED_EINVAL;
  *p = nullptr;
  if (hipHostMalloc(p, bytes, hipHostMallocDefault) != hipSuccess || !*p) return TMED_ENOMEM;
  std::lock_guard<std::mutex> lk(g_pin_mu);
  g_pinned[(uintptr_t)*p] = (uintptr_t)*p + bytes;
  return TMED_OK;
}

int tmed_host_free(void *p) {
  if (!p) return TMED_OK;
  {
    std::lock_guard<std::mutex> lk(g_pin_mu);
    if (!g_pinned.erase((uintptr_t)p)) return TMED_EINVAL;
  }
  return hipHostFree(p) == hipSuccess ? TMED_OK : TMED_EHIP;
}

int tmed_host_register(void *p, size_t bytes) {
  if (!p || bytes == 0) return TMED_EINVAL;
  if (hipHostRegister(p, bytes, hipHostRegisterDefault) != hipSuccess) return TMED_EHIP;
  std::lock_guard<std::mutex> lk(g_pin_mu);
  g_pinned[(uintptr_t)p] = (uintptr_t)p + bytes;
  return TMED_OK;
}

int tmed_host_unregister(void *p) {
  {
    std::lock_guard<std::mutex> lk(g_pin_mu);
    if (!p || !g_pinned.erase((uintptr_t)p)) return TMED_EINVAL;
  }
  return hipHostUnregister(p) == hipSuccess ? TMED_OK : TMED_EHIP;
}

int tmed_b_window_bits(const tmed_ctx *c) { return c && c->d_b26 ? 26 : 16; }
int tmed_keyset_b_window_bits(const tmed_ctx *c) { return c && c->d_b24 ? 24 : 16; }
int tmed_keyset_a_window_bits(tmed_ctx *c, uint64_t handle) {
  if (!c) return -1;
  std::lock_guard<std::mutex> lk(c->mu);
  const Keyset *k = find_keyset(c, handle);
  if (!k) return -1;
  return !k->comba.empty() && k->comba_n == k->n && c->d_b24 ? kCombABits : 8;
}

int tmed_keyset_comb_entry(tmed_ctx *c, uint64_t handle, uint32_t key, int radix_bits, uint32_t window, uint32_t j,
                           int32_t out[30]) {
  if (!c || !out) return TMED_EINVAL;
  std::lock_guard<std::mutex> lk(c->mu);
  const Keyset *k = find_keyset(c, handle);
  if (!k || key >= k->n) return TMED_EINVAL;
  const int4 *src;
  if (radix_bits == 8) {
    if (window >= (uint32_t)kCombWindows || j >= kCombEntries) return TMED_EINVAL;
    src = k->comb_row(key, (size_t)window * kCombEntries + j);
  } else if (radix_bits == kCombABits) {
    if (k->comba.empty() || key >= k->comba_n || window >= (uint32_t)kCombAWindows) return TMED_EINVAL;
    if (j >= (window + 1 == (uint32_t)kCombAWindows ? kCombATopEntries : kCombAEntries)) return TMED_EINVAL;
    src = k->comba_row_of(key, comba_row((int)window, j));
  } else {
    return TMED_EINVAL;
  }
  int4 row[kCombEntryInt4];
  // the builds are queued on the context stream / the key worker's stream: drain both first
  if (hipStreamSynchronize(c->stream) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return TMED_EHIP;
  if (hipMemcpy(row, src, sizeof(row), hipMemcpyDeviceToHost) != hipSuccess) return TMED_EHIP;
  const int32_t *w = reinterpret_cast<const int32_t *>(row);
  for (int i = 0; i < 30; i++) out[i] = w[i];
  return TMED_OK;
}

int tmed_window_stats(tmed_ctx *c, uint32_t lane_hist[65], uint32_t wave_hist[65]) {
  if (!c || !lane_hist || !wave_hist) return TMED_EINVAL;
  std::lock_guard<std::mutex> lk(c->mu);
  for (int w = 0; w < 65; w++) lane_hist[w] = wave_hist[w] = 0;
  if (c->last_hs_count == 0) return TMED_OK;
  (void)hipSetDevice(c->device);
  uint32_t *d = nullptr;
  hipError_t e = hipMalloc((void **)&d, 2 * 65 * sizeof(uint32_t));
  if (e == hipSuccess) e = scratch_acquire(c, c->stream);
  if (e == hipSuccess) e = launch_window_stats(c->d_prep, c->slab_slots, c->last_hs_count, d, c->stream);
  if (e == hipSuccess) e = scratch_release(c, c->stream);
  uint32_t h[130];
  if (e == hipSuccess) e = hipMemcpyAsync(h, d, sizeof h, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (d) (void)hipFree(d);
  if (e != hipSuccess) return map_err(e);
  for (int w = 0; w < 65; w++) { lane_hist[w] = h[w]; wave_hist[w] = h[65 + w]; }
  return TMED_OK;
}

int tmed_sign_batch_device(tmed_ctx *c, const uint8_t *d_seeds, const uint8_t *d_msgs, const uint32_t *d_off,
                           size_t n, uint8_t *d_sig_out, uint8_t *d_pub_out, void *stream) {
  if (!c) return TMED_EINVAL;
  if (n == 0) return TMED_OK;
  if (!d_seeds || !d_msgs || !d_off || !d_sig_out || !d_pub_out || n > 0xffffffffu) return TMED_EINVAL;
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  hipSetDevice(c->device);
  return map_err(launch_sign(d_seeds, d_msgs, d_off, (uint32_t)n, d_sig_out, d_pub_out, c->d_bcomb, s));
}

static int check_offsets(const uint32_t *off, size_t n) {
  for (size_t i = 0; i < n; i++)
    if (off[i + 1] < off[i]) return TMED_EINVAL;
  return TMED_OK;
}

int tmed_verify_batch(tmed_ctx *c, const uint8_t *pub, const uint8_t *sig, const uint32_t *sig_lens,
                      const uint8_t *msgs, const uint32_t *off, size_t n, uint8_t *out) {
  if (!c || !out) return TMED_EINVAL;
  if (n == 0) return TMED_OK;
  if (!pub || !sig || !off || n > 0xffffffffu) return TMED_EINVAL;
  if (check_offsets(off, n) != TMED_OK) return TMED_EINVAL;
  const size_t mbytes = off[n];
  if (mbytes && !msgs) return TMED_EINVAL;
  std::lock_guard<std::mutex> lk(c->mu);
  hipSetDevice(c->device);
  hipError_t e = hipSuccess;
  const size_t moff_bytes = (n + 1) * 4;
  for (auto &pr : {std::make_pair(&c->d_a, n * 32), std::make_pair(&c->d_b, n * 64),
                   std::make_pair(&c->d_msg, mbytes + 16), std::make_pair(&c->d_off, moff_bytes),
                   std::make_pair(&c->d_out, n)})
    if (e == hipSuccess) e = pr.first->ensure(pr.second);
  for (auto &pr : {std::make_pair(&c->h_a, n * 32), std::make_pair(&c->h_b, n * 64),
                   std::make_pair(&c->h_msg, mbytes + 16), std::make_pair(&c->h_off, moff_bytes),
                   std::make_pair(&c->h_out, n)})
    if (e == hipSuccess) e = pr.first->ensure(pr.second);
  if (e != hipSuccess) return map_err(e);
  // Stage into pinned memory (the caller's buffers may be GC-managed Go memory).
  memcpy(c->h_a.p, pub, n * 32);
  memcpy(c->h_b.p, sig, n * 64);
  if (mbytes) memcpy(c->h_msg.p, msgs, mbytes);
  memcpy(c->h_off.p, off, moff_bytes);
  hipStream_t s = c->stream;
  e = hipMemcpyAsync(c->d_a.p, c->h_a.p, n * 32, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipMemcpyAsync(c->d_b.p, c->h_b.p, n * 64, hipMemcpyHostToDevice, s);
  if (e == hipSuccess && mbytes) e = hipMemcpyAsync(c->d_msg.p, c->h_msg.p, mbytes, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipMemcpyAsync(c->d_off.p, c->h_off.p, moff_bytes, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = scratch_acquire(c, s);
  // a small (latency-mode) batch skips the kernel-time events unless timing is on: they add
  // ~8 us to the call (see votes_enqueue)
  const bool timed = c->timing || n > kLatencyUntimedMax;
  if (e == hipSuccess && timed) e = hipEventRecord(c->ev0, s);
  if (e == hipSuccess)
    e = generic_verify(c, (const uint8_t *)c->d_a.p, (const uint8_t *)c->d_b.p, (const uint8_t *)c->d_msg.p,
                       (const uint32_t *)c->d_off.p, (uint32_t)n, (uint8_t *)c->d_out.p, s, false, nullptr);
  if (e == hipSuccess && timed) e = hipEventRecord(c->ev1, s);
  if (e == hipSuccess) e = scratch_release(c, s);
  if (e == hipSuccess) e = hipMemcpyAsync(c->h_out.p, c->d_out.p, n, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return map_err(e);
  c->last_ms = 0.f;
  if (timed) hipEventElapsedTime(&c->last_ms, c->ev0, c->ev1);
  memcpy(out, c->h_out.p, n);
  if (sig_lens)
    for (size_t i = 0; i < n; i++)
      if (sig_lens[i] != 64) out[i] = 0;  // crypto/ed25519/ed25519.go:150-152
  return TMED_OK;
}

int tmed_sign_batch(tmed_ctx *c, const uint8_t *seeds, const uint8_t *msgs, const uint32_t *off, size_t n,
                    uint8_t *sigs_out, uint8_t *pubs_out) {
  if (!c || !sigs_out || !pubs_out) return TMED_EINVAL;
  if (n == 0) return TMED_OK;
  if (!seeds || !off || n > 0xffffffffu) return TMED_EINVAL;
  if (check_offsets(off, n) != TMED_OK) return TMED_EINVAL;
  const size_t mbytes = off[n];
  if (mbytes && !msgs) return TMED_EINVAL;
  std::lock_guard<std::mutex> lk(c->mu);
  hipSetDevice(c->device);
  hipError_t e = hipSuccess;
  const size_t moff_bytes = (n + 1) * 4;
  for (auto &pr : {std::make_pair(&c->d_a, n * 32), std::make_pair(&c->d_b, n * 64),
                   std::make_pair(&c->d_msg, mbytes + 16), std::make_pair(&c->d_off, moff_bytes),
                   std::make_pair(&c->d_c, n * 32)})
    if (e == hipSuccess) e = pr.first->ensure(pr.second);
  if (e != hipSuccess) return map_err(e);
  hipStream_t s = c->stream;
  e = hipMemcpyAsync(c->d_a.p, seeds, n * 32, hipMemcpyHostToDevice, s);
  if (e == hipSuccess && mbytes) e = hipMemcpyAsync(c->d_msg.p, msgs, mbytes, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipMemcpyAsync(c->d_off.p, off, moff_bytes, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipEventRecord(c->ev0, s);
  if (e == hipSuccess)
    e = launch_sign((const uint8_t *)c->d_a.p, (const uint8_t *)c->d_msg.p, (const uint32_t *)c->d_off.p,
                    (uint32_t)n, (uint8_t *)c->d_b.p, (uint8_t *)c->d_c.p, c->d_bcomb, s);
  if (e == hipSuccess) e = hipEventRecord(c->ev1, s);
  if (e == hipSuccess) e = hipMemcpyAsync(sigs_out, c->d_b.p, n * 64, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipMemcpyAsync(pubs_out, c->d_c.p, n * 32, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return map_err(e);
  hipEventElapsedTime(&c->last_ms, c->ev0, c->ev1);
  return TMED_OK;
}

}  // extern "C"
