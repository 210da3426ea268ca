/*
 * sodium_batch.c -- TEST / BASELINE INFRASTRUCTURE ONLY.
 *
 * Times (and records verdicts of) libsodium 1.0.18
 * crypto_sign_ed25519_verify_detached -- the exact function the reference's
 * hot path ends in (stp_core/crypto/nacl_wrappers.py:86-108 ->
 * libnacl.crypto_sign_open -> libsodium) -- over a batch in the edv C-ABI
 * layout, with one pthread per requested core.  Used for (a) the libsodium
 * verdict bitmask of the big parity corpus, computed in the build container,
 * and (b) bench.py's cpu_baseline leg ("kind": "reference") on the GPU box's
 * host cores.  libsodium is the image's own /opt/conda/lib/libsodium.so.23, not
 * anything shipped inside the reference.
 */
#include <pthread.h>
#include <stdint.h>
#include <sodium.h>

typedef struct {
  const uint8_t *sigs, *pks, *msgs;
  const uint64_t *off;
  uint8_t *accept;
  uint64_t lo, hi;
} sjob;

static void *sworker(void *arg) {
  sjob *j = (sjob *)arg;
  for (uint64_t i = j->lo; i < j->hi; i++)
    j->accept[i] = crypto_sign_ed25519_verify_detached(j->sigs + 64 * i, j->msgs + j->off[i],
                                                       j->off[i + 1] - j->off[i], j->pks + 32 * i) == 0;
  return 0;
}

const char *sb_version(void) { return sodium_version_string(); }

int sb_verify_batch(const uint8_t *sigs, const uint8_t *pks, const uint8_t *msgs, const uint64_t *off, uint64_t n,
                    uint8_t *accept, int threads) {
  if (sodium_init() < 0) return -1;
  if (threads < 1) threads = 1;
  if (threads > 512) threads = 512;
  pthread_t th[512];
  sjob jobs[512];
  for (int t = 0; t < threads; t++) {
    jobs[t] = (sjob){sigs, pks, msgs, off, accept, n * t / threads, n * (t + 1) / threads};
    if (pthread_create(&th[t], 0, sworker, &jobs[t])) return -1;
  }
  for (int t = 0; t < threads; t++) pthread_join(th[t], 0);
  return 0;
}
