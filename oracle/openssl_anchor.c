/* openssl_anchor.c — OpenSSL 3 EVP_DigestVerify(ED25519) over a batch (TEST INFRASTRUCTURE /
 * CPU-BASELINE ONLY).
 *
 * The independent CPU anchor BASELINE.md plans beside the C restatement (oracle/ed25519_port.c):
 * an implementation the builder did not write, timed on the same sample by bench.py's
 * cpu_baseline leg.  It is NOT the reference semantics (Go 1.18 crypto/ed25519.Verify, SURVEY.md
 * §8a V0): its decisions are reported, never used as the checker.  Same batch layout as
 * port_verify_batch: pubs n x 32, sigs n x 64, message i = msgs[off[i] .. off[i+1]).
 */
#include <openssl/evp.h>
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>

static void run(const uint8_t *pubs, const uint8_t *sigs, const uint8_t *msgs, const uint64_t *off, size_t lo,
                size_t hi, uint8_t *out) {
  EVP_MD_CTX *c = EVP_MD_CTX_new();
  for (size_t i = lo; i < hi; i++) {
    EVP_PKEY *k = EVP_PKEY_new_raw_public_key(EVP_PKEY_ED25519, NULL, pubs + 32 * i, 32);
    int ok = 0;
    if (k && EVP_DigestVerifyInit(c, NULL, NULL, NULL, k) == 1)
      ok = EVP_DigestVerify(c, sigs + 64 * i, 64, msgs + off[i], (size_t)(off[i + 1] - off[i])) == 1;
    out[i] = (uint8_t)ok;
    EVP_PKEY_free(k);
    EVP_MD_CTX_reset(c);
  }
  EVP_MD_CTX_free(c);
}

struct job {
  const uint8_t *pubs, *sigs, *msgs;
  const uint64_t *off;
  size_t lo, hi;
  uint8_t *out;
};

static void *worker(void *p) {
  struct job *j = (struct job *)p;
  run(j->pubs, j->sigs, j->msgs, j->off, j->lo, j->hi, j->out);
  return NULL;
}

void ossl_verify_batch(const uint8_t *pubs, const uint8_t *sigs, const uint8_t *msgs, const uint64_t *off, size_t n,
                       uint8_t *out, int nthreads) {
  if (nthreads <= 1 || n < 64) {
    run(pubs, sigs, msgs, off, 0, n, out);
    return;
  }
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  struct job jobs[256];
  for (int t = 0; t < nthreads; t++) {
    jobs[t] = (struct job){pubs, sigs, msgs, off, n * t / nthreads, n * (t + 1) / nthreads, out};
    pthread_create(&th[t], NULL, worker, &jobs[t]);
  }
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
}
