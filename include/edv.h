/*
 * edv.h -- C-ABI of the MI355X (gfx950) batch Ed25519 verifier (libedv.so).
 *
 * Drop-in boundary for Plenum's client-request authentication hot path.  In the
 * reference every request signature ends in ONE call:
 *
 *   stp_core/crypto/nacl_wrappers.py:232-242  Verifier.verify(signature, msg)
 *       -> VerifyKey.verify(signature + msg)           nacl_wrappers.py:86-108
 *       -> libnacl.crypto_sign_open(sm, pk)            (libsodium 1.0.18)
 *
 * made once per signature from NaclAuthNr.authenticate_multi
 * (plenum/server/client_authn.py:83-113) through DidVerifier.verify
 * (plenum/common/verifier.py:54-55).  edv_verify_batch replaces a whole batch of
 * those calls; the Python shim (indy-plenum_amd/nacl_wrappers.py, client_authn.py,
 * req_authenticator.py) keeps the reference's per-request semantics above it.
 *
 * Verdict contract: accept[i] == 1 iff libsodium 1.0.18
 * crypto_sign_ed25519_verify_detached(sig_i, msg_i, len_i, pk_i) == 0, bit for
 * bit (strict S < L, small-order R/A blocklist, canonical A, cofactorless
 * equation).  The reference's positional sig||msg split (crypto_sign_open on
 * signature + msg) is applied by the caller before this layer (see
 * INTEGRATION.md); every sig here is exactly 64 bytes.
 *
 * All entry points return 0 on success or a negative EDV_E_* code, never
 * throw, and keep no pointer to caller memory after returning (except
 * edv_verify_batch_async, until edv_wait_async -- or edv_query_async returning
 * anything but EDV_PENDING -- for that batch).
 */
#ifndef EDV_H
#define EDV_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define EDV_OK 0
#define EDV_E_ARG -1   /* bad argument (null pointer with n > 0, bad offsets) */
#define EDV_E_NODEV -2 /* no usable gfx950 device in device_mask */
#define EDV_E_HIP -3   /* HIP runtime error (text: edv_last_error) */
#define EDV_E_OOM -4   /* device or pinned allocation failed */

/*
 * Verify n detached signatures held in HOST memory; synchronous.
 * A device's shard of up to one chunk (2^18 requests, edv_set_chunk) is
 * copied field by field: signatures, keys and offsets first (the point sides
 * of the prep kernel start on them), then the messages (their hash side
 * starts as each slice lands), then the main kernel, which writes the
 * verdicts straight into page-locked host memory (no D2H copy).  A larger
 * shard alternates two streams of half-chunk sub-batches, so the copies of
 * one overlap the kernels of the other.  A shard of at most 16,384 requests
 * (a Node's prod, one Verifier.verify) takes the latency path instead
 * (edv_set_latency_path): one kernel launch with sixteen lanes per signature
 * (eight above 4,096 requests);
 * pinned inputs are copied by DMA straight from the caller's buffers (one copy
 * when sigs, pks and msg_off lie in one region in that order, then the
 * messages), pageable ones are packed into the library's pinned staging and
 * read there by the kernel.  On the batch path, inputs in pinned memory (e.g.
 * from edv_host_alloc) are copied to the device directly; pageable inputs are
 * first staged through the library's pinned buffers by a parallel memcpy
 * (EDV_COPY_THREADS threads, default 8).
 *   sigs     n x 64 bytes (R || S), contiguous
 *   pks      n x 32 bytes (A), contiguous
 *   msgs     concatenated messages; message i = msgs[msg_off[i] .. msg_off[i+1])
 *   msg_off  n + 1 non-decreasing byte offsets
 *   accept   out: n bytes, 1 = accept, 0 = reject
 *   device_mask  bit d selects device d; 0 = all visible devices.  The batch is
 *            split by request index into contiguous shards, one per device and
 *            one host thread each (edv_shard_split: equal counts, or equal
 *            estimated cost when SHA-512 block counts differ); no inter-device
 *            traffic; each shard's accept bytes land in its slice.
 * Replaces: a loop of nacl_wrappers.Verifier.verify (nacl_wrappers.py:232-242).
 */
int edv_verify_batch(const uint8_t *sigs, const uint8_t *pks, const uint8_t *msgs, const uint64_t *msg_off,
                     uint64_t n, uint8_t *accept, uint32_t device_mask);

/*
 * Asynchronous form of edv_verify_batch on one device (the batched call site of
 * plenum/server/client_authn.py:92-112 when the Node verifies one batch per prod
 * and keeps going): queues the H2D copies, the kernels and the D2H of the
 * verdicts and returns a ticket at once.  Batches take eight slots in turn,
 * so batch k+1's copies (and, for pageable inputs, its staging memcpy, done in
 * this call) run while batch k computes: back to back, the host path then runs
 * at the kernels' rate rather than copy + kernels.  The caller's buffers must
 * stay valid and unchanged, and `accept` unread, until edv_wait_async(device,
 * ticket) (or edv_query_async) returns 0; a submission waits for the batch eight submissions back
 * (completing it as edv_wait_async would) before reusing its slot.  Same
 * verdicts, arguments and alignment rules as edv_verify_batch.
 */
int edv_verify_batch_async(const uint8_t *sigs, const uint8_t *pks, const uint8_t *msgs, const uint64_t *msg_off,
                           uint64_t n, uint8_t *accept, int device, int64_t *ticket);
/* Wait for batch `ticket` of `device` and hand over its verdicts (0 at once if
 * it already was); EDV_E_ARG for a ticket never issued.  Fails closed: `accept`
 * is zeroed at submission (an unfilled buffer rejects), and once a batch has
 * failed, every wait for a ticket at or below it that is no longer pending
 * returns EDV_E_HIP, however many batches fail later. */
int edv_wait_async(int device, int64_t ticket);
/* edv_wait_async without the wait: EDV_PENDING while batch `ticket` of `device`
 * is still on the GPU (nothing changes), else exactly what edv_wait_async
 * returns, with the verdicts handed over.  Lets a Node hand a prod's batch over
 * in the same prod when the GPU is already done, and at its next prod if not. */
#define EDV_PENDING 1
int edv_query_async(int device, int64_t ticket);
/*
 * edv_verify_batch_async that also returns, when `digests` is not NULL, the
 * SHA-256 of every message (digests: n x 32 bytes, same lifetime rules as
 * `accept`), computed on the device from the bytes already copied for the
 * verify.  For a request whose signing bytes are its signingState's
 * serialization these are Request.getDigest (plenum/common/request.py:71-72),
 * which the Node computes per request next to the signature check
 * (plenum/server/node.py:2093-2147); the caller decides which requests that
 * holds for.  Ticket and wait as for edv_verify_batch_async.
 */
int edv_verify_digest_batch_async(const uint8_t *sigs, const uint8_t *pks, const uint8_t *msgs,
                                  const uint64_t *msg_off, uint64_t n, uint8_t *accept, uint8_t *digests, int device,
                                  int64_t *ticket);

/*
 * Same verdicts for inputs already resident in device memory of `device`;
 * asynchronous on `stream` (a hipStream_t, NULL = the library's own stream of
 * that device, which is then synchronised before returning).  Offsets are
 * absolute into d_msgs minus msg_base (so a shard may pass the global offset
 * array slice unchanged).
 * Alignment (EDV_E_ARG otherwise): d_sigs and d_pks 16-byte aligned (read as
 * 16-byte vectors), d_msg_off 8-byte aligned.  d_msgs may have any alignment:
 * message bytes are read as aligned 32-bit words, so the kernels touch up to
 * 3 bytes before a message start (never across a page) and up to 16 bytes past
 * the last message byte, which must be readable.
 * Launches on different streams never share the library's per-device scratch
 * concurrently: each one is ordered after the previous user of the scratch.
 */
int edv_verify_batch_dev(const uint8_t *d_sigs, const uint8_t *d_pks, const uint8_t *d_msgs,
                         const uint64_t *d_msg_off, uint64_t msg_base, uint64_t n, uint8_t *d_accept,
                         int device, void *stream);

/* Per-call SHA-512 length-bucket hint for the device paths (overrides the
 * device mode of edv_set_length_buckets for this call only). */
#define EDV_FLAG_UNIFORM_LENGTH 1u /* every message has the same SHA-512 block count: no buckets */
#define EDV_FLAG_BUCKETS 2u        /* always bucket by block count */
#define EDV_FLAG_SPLIT_PREP 4u     /* edv_verify_batch_dev_pipelined only: the hash side of batch k+1's
                                      prep runs beside batch k's main kernel, the point sides after it */
int edv_verify_batch_dev_flags(const uint8_t *d_sigs, const uint8_t *d_pks, const uint8_t *d_msgs,
                               const uint64_t *d_msg_off, uint64_t msg_base, uint64_t n, uint8_t *d_accept,
                               int device, void *stream, uint32_t flags);

/*
 * Batch SHA-256: out[32 i .. 32 i + 32) = SHA-256 of message i
 * (msgs/msg_off as in edv_verify_batch).  Host buffers, synchronous, sharded over
 * device_mask like edv_verify_batch.  Replaces, per request,
 * plenum/common/request.py:71-72 Request.getDigest (sha256 of the signing bytes,
 * hex-encoded by the caller) and plenum/server/domain_req_handler.py:166-167
 * nym_to_state_key (sha256 of the DID string).
 */
int edv_sha256_batch(const uint8_t *msgs, const uint64_t *msg_off, uint64_t n, uint8_t *out, uint32_t device_mask);
/* Device-resident form, async on `stream` (NULL = library stream, synchronised);
 * d_msgs readable 8 bytes past the last message byte; d_out n x 32 bytes. */
int edv_sha256_batch_dev(const uint8_t *d_msgs, const uint64_t *d_msg_off, uint64_t msg_base, uint64_t n,
                         uint8_t *d_out, int device, void *stream);

/*
 * Pipelined submission of device-resident batches (a continuous stream of
 * client batches, e.g. one per Node prod): enqueues the batch and returns
 * without waiting.  Consecutive submissions alternate between two internal
 * state sets, with the prep kernel (checks, decompression, SHA-512, table) of
 * batch k+1 on one library stream and the main kernel (the joint walk) of
 * batch k on another, so both can run on the SIMDs at once (measured on
 * MI355X at C2 after round 5's kernels it is slower than sequential batches,
 * 91.8-92.3 M against 98.3-98.6 M verifies/s: profiles/r05/ab_modes_s16.jsonl;
 * with EDV_FLAG_SPLIT_PREP it pays at C4's long messages).  Work
 * already queued on the library stream (edv_stream) is ordered before the
 * batch; inputs must stay unchanged and each batch's d_accept must not be
 * reused or read until edv_pipeline_sync(device) returns.  Same verdicts as
 * edv_verify_batch_dev.
 */
int edv_verify_batch_dev_pipelined(const uint8_t *d_sigs, const uint8_t *d_pks, const uint8_t *d_msgs,
                                   const uint64_t *d_msg_off, uint64_t msg_base, uint64_t n, uint8_t *d_accept,
                                   int device, uint32_t flags);
/* Wait until every pipelined batch submitted on `device` has its verdicts. */
int edv_pipeline_sync(int device);

/* (Kernel timing and fault injection are not part of this ABI: they live in
 * the benchmark build libedv_measure.so, include/edv_measure.h.) */

/* Signatures per prep/main kernel pair on `device` (0 = default 2^18; rounded
 * down to a multiple of 256).  Tuning/testing knob: verdicts never depend on it. */
int edv_set_chunk(int device, uint64_t chunk);

/* Message slices of a synchronous edv_verify_batch shard that fits one chunk
 * (1..8; 0 = default: one per 65,536 requests, so one at C2): the messages are
 * copied in that many slices by request, and each slice's SHA-512 / scalar
 * side runs as soon as it has landed, so only the last slice's remains after
 * the copy.  Tuning knob: verdicts never depend on it. */
int edv_set_host_slices(int device, int slices);

/* The latency path: every batch of at most max_requests requests (default and
 * at most 16,384; 0 = never) on `device` -- synchronous, asynchronous and
 * device-resident calls alike -- runs as ONE kernel launch with several lanes
 * per signature (edv_quad.hip; each point doubling and addition split over a
 * quad of lanes, operands exchanged by DPP): up to 4,096 requests sixteen lanes
 * (per scalar a doubler wave running the 16^j P chain and an adder wave
 * summing per-digit buckets), above that eight (two table walks).  Below one
 * wave per SIMD the batch kernels (one signature per lane) take a lane's whole
 * serial chain whatever n is; this path divides that chain instead (0.18-0.21
 * ms of kernel on MI355X against ~0.55 ms).  Tuning knob: verdicts never
 * depend on it. */
int edv_set_latency_path(int device, uint64_t max_requests);

/* SHA-512 length buckets of the device paths (a counting sort of each chunk by
 * block count, so a wave of the prep kernel hashes equally long messages):
 * 0 = never (a caller whose messages all have one length saves three small
 * launches per chunk), 1 = always, 2 = auto (default: on for device-resident
 * batches; the host path buckets only when lengths differ).  Tuning knob:
 * verdicts never depend on it. */
int edv_set_length_buckets(int device, int mode);

/*
 * Batch Ed25519 signing for synthetic load generation,
 * device-resident: seeds n x 32 B -> pks n x 32 B and detached sigs n x 64 B
 * over the given messages; RFC 8032 deterministic, byte-identical to libsodium
 * crypto_sign_seed_keypair + crypto_sign_detached.  Counterpart of the
 * reference's client-side signing (stp_core/crypto/nacl_wrappers.py:162-176
 * SigningKey.sign, plenum/common/signer_did.py:122-129).  Async on `stream`
 * (NULL = library stream, synchronised before returning).
 */
int edv_sign_batch_dev(const uint8_t *d_seeds, const uint8_t *d_msgs, const uint64_t *d_msg_off, uint64_t msg_base,
                       uint64_t n, uint8_t *d_pks, uint8_t *d_sigs, int device, void *stream);

/* The library's own HIP stream of `device` (so callers can enqueue several
 * edv_*_dev calls asynchronously on it) and a wait for everything on it. */
int edv_stream(int device, void **out);
int edv_sync(int device);

/* Number of visible gfx950 devices (0 if none).  EDV_VIRTUAL_DEVICES=k (a
 * testing knob) presents k logical devices mapped round-robin onto the physical
 * ones, each with its own context, so the multi-device path runs on one GPU. */
int edv_device_count(void);

/*
 * Device placement on a multi-GPU node.  edv_verify_batch / edv_sha256_batch
 * split a batch only into shards of at least 65,536 requests (one wave per SIMD
 * of a whole MI355X: a smaller shard takes as long as a full one; EDV_MIN_SHARD
 * overrides), so a Node-sized batch (a prod of a few hundred requests, or one
 * Verifier.verify) runs whole on ONE device, on the calling thread, and no
 * other device is initialised.  Devices are chosen the same way for one shard
 * and for 2..7 shards of a mid-sized batch: initialised devices with nothing
 * running first, then devices not yet initialised (order starting at pid mod
 * devices), then the least-loaded (load = synchronous calls placed there +
 * asynchronous batches still running on the GPU, waited for or not); concurrent
 * calls see each other's choices.  edv_pick_device returns that choice for one
 * shard; the Node's asynchronous path asks it for the device of each
 * submission (edv_verify_batch_async takes the device explicitly).
 * edv_pick_device returns that device's index (or a negative EDV_E_* code);
 * edv_context_count: devices whose context (streams, scratch, [S]B tables) exists.
 * Reference: the per-request call being placed, nacl_wrappers.py:232-242, made
 * per prod (plenum/server/node.py:1026-1049, stp_core/config.py:28).
 */
int edv_pick_device(uint32_t device_mask);

/*
 * Accept bytes -> accept bitmask on the device: d_bits[i / 8] bit (i % 8) =
 * (d_accept[i] != 0), ceil(n / 8) bytes (numpy.packbits(..., bitorder="little")).
 * What a multi-GPU run gathers to the host: N/8 bytes per shard.
 * Asynchronous on `stream` if given, else synchronous on the library stream;
 * either way ordered after every verify already launched on `device` (any
 * stream, pipelined submissions included).
 */
int edv_pack_bits_dev(const uint8_t *d_accept, uint64_t n, uint8_t *d_bits, int device, void *stream);
int edv_context_count(void);

/*
 * Device memory the library holds for `device` in this process, in bytes:
 * out[0] total, out[1] the [S]B tables (shared by the logical devices of one
 * GPU), out[2] chunk scratch of the ordinary paths, out[3] the asynchronous
 * slots (inputs and small-batch scratch), out[4] the pipelined state sets,
 * out[5] input buffers of the synchronous path, out[6] the signer's comb
 * table.  Scratch grows with the largest batch seen (up to one chunk), so a
 * Node that verifies prods of a few hundred requests holds a few hundred MB;
 * 0 for a device whose context does not exist yet.  (What a Node process
 * costs a GPU it shares with other Node processes: scripts/start_plenum_node
 * runs one Node per process.)
 */
int edv_context_memory(int device, uint64_t out[7]);

/*
 * The shard split edv_verify_batch uses (host only, no GPU needed): bounds[0..g]
 * with shard k = requests [bounds[k], bounds[k+1]).  Equal request counts
 * (n*k/g) when every message has the same SHA-512 block count; otherwise equal
 * estimated cost, sum over the shard of (40 + SHA-512 blocks of R||A||M), where
 * 40 blocks is the fixed per-verify work of SURVEY.md section 8d's W(m).
 */
int edv_shard_split(const uint64_t *msg_off, uint64_t n, uint32_t g, uint64_t *bounds);

/* Pinned (page-locked, portable) host memory: inputs packed here are copied to
 * the device by DMA without the staging memcpy. */
int edv_host_alloc(uint64_t bytes, void **out);
int edv_host_free(void *p);

/* Device memory helpers so a host without PyTorch can stage inputs. */
int edv_dev_alloc(int device, uint64_t bytes, void **out);
int edv_dev_free(int device, void *p);
int edv_h2d(int device, void *dst, const void *src, uint64_t bytes);
int edv_d2h(int device, void *dst, const void *src, uint64_t bytes);

/* Library/version string, e.g. "edv 0.1.0 gfx950". */
const char *edv_version(void);

/* Text of the last error raised on the calling thread ("" if none). */
const char *edv_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* EDV_H */
