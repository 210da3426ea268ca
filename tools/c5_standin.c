/* Stand-in device calls for tools/profile_c5_host.py (harness only, never a
 * product path): edv_verify_digest_batch_async / edv_wait_async-compatible
 * functions that accept every request and hash the messages with the SHA-256
 * batch function set by standin_set_sha256 (the kernel's SHA-256 compiled for
 * the CPU, libedv_hostcheck.so's hc_sha256_batch), all in C so that the
 * stand-in allocates no Python objects and its time can be taken out. */
#include <stdint.h>
#include <string.h>
#include <time.h>

typedef int (*sha_fn)(const uint8_t*, const uint64_t*, uint64_t, uint8_t*, uint32_t);
static sha_fn g_sha;
static double g_s;

void standin_set_sha256(void* f) { g_sha = (sha_fn)f; }
double standin_seconds(void) { return g_s; }
void standin_reset(void) { g_s = 0; }

int standin_submit(const uint8_t* sigs, const uint8_t* pks, const uint8_t* msgs, const uint64_t* off, uint64_t n,
                   uint8_t* acc, uint8_t* digests, int device, int64_t* ticket) {
  struct timespec a, b;
  clock_gettime(CLOCK_MONOTONIC, &a);
  (void)sigs; (void)pks; (void)device;
  memset(acc, 1, n);
  int r = 0;
  if (digests) r = g_sha(msgs, off, n, digests, 0);
  *ticket = 0;
  clock_gettime(CLOCK_MONOTONIC, &b);
  g_s += (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
  return r;
}

int standin_wait(int device, int64_t ticket) { (void)device; (void)ticket; return 0; }
int standin_query(int device, int64_t ticket) { (void)device; (void)ticket; return 0; }
