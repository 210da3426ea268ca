/*
 * edv_measure.h -- measurement entry points of libedv_measure.so, the
 * benchmark/profiling build of the verifier (same sources as libedv.so,
 * compiled with -DEDV_MEASUREMENT_API).  The product library libedv.so does
 * NOT export these: a Node binds include/edv.h only.  bench.py and the
 * profiling tools load libedv_measure.so beside the product library (a
 * second set of device contexts in the same process; device pointers from
 * either library are interchangeable) to time kernels on the kernels' own
 * stream, and the GPU tests use its fault hook.  Every edv.h entry point is
 * exported too, with the product's verdicts.
 */
#ifndef EDV_MEASURE_H
#define EDV_MEASURE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/*
 * Launches the verify kernels `iters` times on device-resident inputs between
 * two HIP events recorded on the kernels' own stream; elapsed milliseconds of
 * the whole region.
 */
int edv_time_batch_dev(const uint8_t *d_sigs, const uint8_t *d_pks, const uint8_t *d_msgs,
                       const uint64_t *d_msg_off, uint64_t msg_base, uint64_t n, uint8_t *d_accept, int device,
                       int iters, float *ms_out);

/*
 * Average per-launch milliseconds of the two kernels of one batch (n <= chunk),
 * each bracketed by HIP events on the kernels' stream: prep (checks,
 * decompression, SHA-512, [S]B, tables) and main (the joint walk).  The
 * length-bucketing pass runs before each pair, outside the events.
 */
int edv_profile_batch_dev(const uint8_t *d_sigs, const uint8_t *d_pks, const uint8_t *d_msgs,
                          const uint64_t *d_msg_off, uint64_t msg_base, uint64_t n, uint8_t *d_accept, int device,
                          int iters, float *ms_prep, float *ms_main);

/*
 * edv_profile_batch_dev with, when flush_bytes > 0, a kernel between prep and
 * main that reads and rewrites a flush_bytes buffer (larger than the 256 MiB
 * Infinity Cache: the prep kernel's tables are evicted before main reads
 * them); ms_flush = that kernel's time.
 */
int edv_profile_batch_dev_flush(const uint8_t *d_sigs, const uint8_t *d_pks, const uint8_t *d_msgs,
                                const uint64_t *d_msg_off, uint64_t msg_base, uint64_t n, uint8_t *d_accept,
                                int device, int iters, uint64_t flush_bytes, float *ms_prep, float *ms_flush,
                                float *ms_main);

/*
 * The prep kernel's sides timed apart (n <= chunk, uniform message length):
 * ms[0] hash side alone, ms[1] A side alone, ms[2] R side alone, ms[3] all
 * three in one launch (the product's launch), ms[4] the two point sides in one
 * launch; averages over `iters` launches each, HIP events on the kernels'
 * stream.  The verdicts of such a call are not complete (main is not run).
 */
int edv_profile_prep_sides(const uint8_t *d_sigs, const uint8_t *d_pks, const uint8_t *d_msgs,
                           const uint64_t *d_msg_off, uint64_t msg_base, uint64_t n, uint8_t *d_accept, int device,
                           int iters, float ms[5]);

/*
 * Fault hook for the GPU tests of the asynchronous path: the submission that
 * will receive `ticket` on `device` launches no kernels and reports EDV_E_HIP
 * when it completes (edv_wait_async, or a later submission reusing its slot),
 * as a batch whose done event failed would.  ticket < 0 disarms.
 */
int edv_test_fail_async(int device, int64_t ticket);

#ifdef __cplusplus
}
#endif
#endif /* EDV_MEASURE_H */
