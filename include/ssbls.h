/* ssbls.h -- C ABI of the MI355X threshold-BLS batch engine (libssbls.so, gfx950).
 *
 * This is the drop-in boundary for SafeStake's threshold-BLS hot path.  Each entry point names
 * the reference interface it replaces (paths relative to the SafeStakeOperator repository):
 *
 *   ssb_threshold_aggregate_batch  <- GenericThresholdSignature::threshold_aggregate
 *                                     (src/crypto/generic_threshold.rs:132-175), batched over
 *                                     independent (validator, signing-root) jobs
 *   ssb_unsafe_aggregate_batch     <- TThresholdSignature::unsafe_aggregate /
 *                                     BlstThresholdSignature::unsafe_aggregate
 *                                     (src/crypto/generic_threshold.rs:177-179,
 *                                      src/crypto/impls/blst.rs:67-87)
 *   ssb_verify_batch               <- bls::Signature::verify(pk, msg) as called per share at
 *                                     src/crypto/generic_threshold.rs:156 (blst verify with
 *                                     sig_groupcheck=true, pk_validate=false; same convention
 *                                     as src/network/io_committee.rs:536-539)
 *   ssb_hash_to_g2                 <- the hash_to_G2 blst runs inside verify/sign with the DST of
 *                                     src/crypto/impls/blst.rs:11
 *   ssb_lagrange_coeffs            <- lagrange_coeffs (src/crypto/impls/blst.rs:19-39)
 *   ssb_feldman_verify_batch       <- DKG::share_verification (src/crypto/dkg.rs:433-450):
 *                                     blst_p1_mult(h, s) == CommittedPoly::eval(party)
 *                                     (src/math/polynomial.rs:68-81), batched
 *   ssb_dleq_verify_batch          <- DKG::dleq_verify (src/crypto/dkg.rs:674-692), batched
 *   ssb_pk_validate_batch          <- bls::PublicKey::deserialize (key_validate) + serialize, as
 *                                     the reference deserializes operator / validator keys
 *                                     (src/validation/operator_committee_definitions.rs:47-56)
 *   ssb_decode_wire_sigs           <- bincode::deserialize::<Signature>(&data) on a received
 *                                     partial signature (src/validation/operator.rs:108; the
 *                                     records are written by bincode::serialize(&sig),
 *                                     src/node/dvfcore.rs:245-251), batched
 *
 * Conventions
 *   - Signatures are 96-byte compressed G2 points, public keys 48-byte compressed G1 points
 *     (ZCash encoding, as Signature::serialize / PublicKey::serialize).  Roots are 32 bytes.
 *   - Public keys are PRE-VALIDATED by the caller (lighthouse PublicKey::deserialize does
 *     key_validate; verify passes pk_validate=false).  A public key that does not decode, or
 *     decodes to infinity, makes its share invalid (verdict 0).
 *   - A signature that does not decode (blst BAD_ENCODING / POINT_NOT_ON_CURVE), is not in G2,
 *     or is the point at infinity yields verdict 0, exactly as blst verify returns false.
 *   - Verification is by random linear combination, as lighthouse's verify_signature_sets
 *     (RAND_BITS = 64, src/crypto/impls/blst.rs:12): one final exponentiation per batch, a failing
 *     batch is resolved by exact group tests, so every verdict equals the single-signature verify
 *     result.  The 64-bit scalars come from a 256-bit key drawn from the OS CSPRNG (getrandom) for
 *     EVERY call, inside the library, after the inputs are handed over (ChaCha12 of the key and the
 *     share index); `rlc_seed` is only XORed into that key.  The key never leaves the library, so a
 *     sender cannot craft shares whose errors cancel in the combination (see
 *     ssb_set_rlc_deterministic for the one exception).
 *   - Host-pointer functions copy inputs to the device and results back; they are synchronous
 *     (ssb_threshold_aggregate_batch_submit / ssb_batch_wait is the asynchronous form).
 *     The *_dev variants take DEVICE pointers -- or device-mapped pinned host memory
 *     (hipHostMalloc(.., hipHostMallocMapped)), which the kernels then read and write in place
 *     over PCIe -- and a hipStream_t (as void*), enqueue everything on that stream and return
 *     without synchronising.
 *   - Return value of every function: SSB_OK or a negative SSB_E* code (ssb_last_error() has
 *     the message).  No C++ exception crosses this ABI.  A context is thread-safe: every entry
 *     point holds the context's lock while it enqueues its work, so the threads of a process can
 *     share ONE context (the collector's worker, direct callers, key registration).  The synchronous
 *     entry points (ssb_unsafe_aggregate_batch, ssb_sign_batch, ssb_sk_to_pk_batch,
 *     ssb_pk_validate_batch, ssb_lagrange_coeffs, ssb_hash_to_g2*, ssb_verify_batch,
 *     ssb_decode_wire_sigs, ssb_feldman_verify_batch, ssb_dleq_verify_batch) run one at a time per
 *     context, on an idle pipeline slot when there is one, and wait for their results OUTSIDE the
 *     lock, so the other threads' batches keep launching meanwhile.  ssb_last_error is the message of
 *     the context's last failed call, copied per calling thread (read it on the thread that got the
 *     error before another call on the context fails).  ssb_destroy must not race with other calls
 *     on the context.
 */
#ifndef SSBLS_H
#define SSBLS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SSB_OK 0
#define SSB_EINVAL (-1)  /* bad argument (null pointer, size, t == 0, dst too long) */
#define SSB_EHIP (-2)    /* HIP runtime error (no device, launch failure, ...) */
#define SSB_ENOMEM (-3)  /* device allocation failed */

/* Per-job status tags (DvfError variants, src/utils/error.rs:12-60) */
#define SSB_DVF_OK 0
#define SSB_DVF_DIFFERENT_LENGTH 1            /* err = {x, y} (host-side wrapper only) */
#define SSB_DVF_INSUFFICIENT_SIGNATURES 2     /* err = {got, expected} */
#define SSB_DVF_INVALID_OPERATOR_ID 3         /* err = {id, 0} */
#define SSB_DVF_INSUFFICIENT_VALID_SIGNATURES 4 /* err = {got, expected} */
#define SSB_DVF_BAD_SIGNATURE_ENCODING 5      /* unsafe_aggregate only: a share does not decode
                                                 (the reference's unwrap() would panic) */
#define SSB_DVF_INVALID_JOB 6                 /* *_dev entry points only: t[j] == 0, t[j] > SSB_MAX_T,
                                                 share_off[j+1] < share_off[j] or > n_shares;
                                                 err = {t, share count}.  The host-pointer entry
                                                 points refuse such a batch with SSB_EINVAL. */
#define SSB_DVF_ENGINE_ERROR 7                /* the job's batch did not complete (HIP error): no
                                                 output; err[0] = the hipError_t.  Never a reference
                                                 result -- a lost batch never reads as SSB_DVF_OK. */

/* Maximum threshold t supported per job, and maximum DST length. */
#define SSB_MAX_T 64
#define SSB_MAX_DST 255

typedef struct ssb_ctx ssb_ctx;

int ssb_create(ssb_ctx** out, int device_ordinal);
void ssb_destroy(ssb_ctx* ctx);
const char* ssb_last_error(const ssb_ctx* ctx);
/* Slots x streams-per-slot limits: the HIP runtime reserves scratch on every hardware queue for the
 * largest kernel that queue has run, and 8 slots x 3 streams exhausted it on an MI355X
 * (HSA_STATUS_ERROR_OUT_OF_RESOURCES: the side streams run the large-scratch kernels) while
 * one-stream slots run clean up to SSB_MAX_SLOT_STREAMS (20: with round 3's kernels, whose
 * largest batch-path private segment is 2.4 KB per lane, 24 one-stream slots failed the same way). */
#define SSB_MAX_SLOT_STREAMS 20
#define SSB_MAX_THREE_STREAM_SLOTS 5
/* SSB_OK if `depth` slots of `streams` streams are a supported configuration (streams 1 or 3,
 * depth x streams <= SSB_MAX_SLOT_STREAMS, three-stream slots at most SSB_MAX_THREE_STREAM_SLOTS),
 * SSB_EINVAL otherwise.  No GPU needed; ssb_set_pipeline_depth / ssb_set_slot_streams refuse what
 * this refuses. */
int ssb_check_pipeline_config(int depth, int streams);
/* Hardware queues the HIP runtime gives this process: GPU_MAX_HW_QUEUES from the environment (HIP
 * reads it when it initialises, so the process must set it BEFORE its first HIP call; at most 32),
 * else HIP's default, 4.  Every stream of a pipeline slot needs a queue of its own, or independent
 * batches serialise on shared queues: ssb_set_pipeline_depth / ssb_set_slot_streams refuse a
 * configuration of more than (budget - 1) slot streams (SSB_EINVAL, the reason in ssb_last_error),
 * and ssb_collector_create lowers its in_flight to fit (with a warning on stderr).  Read at
 * ssb_create. */
int ssb_hw_queue_budget(void);
/* Number of pipeline slots (1..20, default 1; depth x streams per slot at most ssb_hw_queue_budget() - 1).
 * Each slot owns its streams and workspace; calls of
 * ssb_threshold_aggregate_batch_dev go to the slots round robin, so up to `depth` independent
 * batches are in flight and overlap on the device (e.g. the duties of consecutive slots).  Each
 * call's outputs are ready when the caller's `stream` reaches them. */
int ssb_set_pipeline_depth(ssb_ctx* ctx, int depth);
/* Streams per slot: 3 (default) overlaps hash_to_G2 and the G1 side with the main chain inside a
 * batch (lowest single-batch latency); 1 runs each batch in order on one stream, so one hardware
 * queue per slot and more slots within the HIP runtime's per-queue scratch reservations (highest
 * throughput with many batches in flight).  Re-creates the slots' streams. */
int ssb_set_slot_streams(ssb_ctx* ctx, int streams);
/* TESTS / REPRODUCIBLE PROFILING ONLY.  on = 1: the RLC key of every later call is expanded from
 * the caller's rlc_seed alone (splitmix64), so the scalars are a public function of the seed and
 * crafted shares CAN cancel -- never use this on untrusted input.  on = 0 (the default): a fresh
 * getrandom() key per call. */
int ssb_set_rlc_deterministic(ssb_ctx* ctx, int on);
/* The main stream of pipeline slot `slot` (hipStream_t as void*), e.g. to pass it back as the
 * `stream` of ssb_threshold_aggregate_batch_dev so a caller adds no hardware queue of its own.
 * A *_dev call whose `stream` is a slot's main stream runs on THAT slot; any other stream gets the
 * next slot round robin. */
void* ssb_slot_stream(ssb_ctx* ctx, int slot);
/* Profiling aid: enqueue on `stream` a one-wave kernel that waits until the device word *flag is
 * non-zero (or about max_us microseconds have passed), so batches enqueued behind it on several
 * streams start together -- a kernel-trace of a pipelined run then shows the device timeline
 * rather than the profiler's per-launch host overhead.  Not used by the product path. */
int ssb_debug_hold(void* stream, const uint32_t* flag, uint32_t max_us);
/* Device-side kernel timing with hipEvents recorded on the engine's stream around each launch,
 * only while timing is on (off by default: no events in the production path).
 * ssb_kernel_timing(ctx, 1) clears and starts accumulating every launch (ssb_kernel_time returns
 * the total and the launch count); ssb_kernel_timing(ctx, 2) records the last launch of each
 * stage only (ssb_last_kernel_ms); ssb_kernel_timing(ctx, 0) stops. */
int ssb_last_kernel_ms(const ssb_ctx* ctx, const char* kernel_name, float* ms);
int ssb_kernel_timing(ssb_ctx* ctx, int on);
int ssb_kernel_time(ssb_ctx* ctx, const char* kernel_name, float* total_ms, int* launches);

/* hash_to_G2 of n 32-byte messages; out: n x 192 bytes (blst_p2_serialize layout). */
/* DKG / VSS share verification: verdicts[i] = ([s_i]h == C_{i,0} + sum_{k>=1} [ids[i]^k mod r] C_{i,k}).
 * commitments48: n * t compressed G1 points (check i's polynomial commitments C_{i,0..t-1}, as
 * CommittedPoly::to_bytes without its u32 count); shares32: n 32-byte LITTLE-endian scalars
 * (bytes_to_blst_scalar; the low 255 bits are used, as blst_p1_mult(.., 255)); h48: the
 * commitment base (the reference's another_p1_generator(), hash_to_G1 of "dvf another
 * generator"), compressed.  A commitment that does not decode counts as the identity (the
 * reference ignores blst_p1_uncompress's error and keeps the zeroed point, polynomial.rs:109-111);
 * one that decodes to a point outside G1 gives verdict 0 (blst_p1_mult's GLV result on such a point
 * is implementation-defined); an h that does not decode gives verdict 0. */
int ssb_feldman_verify_batch(ssb_ctx* ctx, size_t n, size_t t, const uint8_t* commitments48, const uint64_t* ids,
                             const uint8_t* shares32, const uint8_t* h48, uint8_t* verdicts);

/* DLEQ (Chaum-Pedersen) proof verification: verdicts[i] = 1 iff c_i equals hash_points_to_blst_scalar
 * (x1, y1, x2, y2, t1, t2) with t_h = [r_i] x_h + [c_i] y_h -- the reference's "hash" is the 288-byte
 * concatenation of the compressed points read as one little-endian integer mod r
 * (src/utils/blst_utils.rs:273-278).  points48: n x (x1, y1, x2, y2), 48-byte compressed G1 each;
 * c32 / r32: the proof scalars, 32 bytes little endian (compared byte for byte, as blst_scalar ==). */
int ssb_dleq_verify_batch(ssb_ctx* ctx, size_t n, const uint8_t* points48, const uint8_t* c32, const uint8_t* r32,
                          uint8_t* verdicts);

/* Wire-format partial signatures -> 96-byte compressed signatures.  Record i (at wire + i*stride,
 * stride >= 202) is bincode(bls::Signature): u64 LE length 194, then "0x" and 192 hex digits of the
 * compressed point.  status[i]: 0 ok, 1 length field is not 194, 2 no "0x" prefix, 3 a non-hex
 * digit, 4 the bytes do not decompress to a curve point (bad flags, x >= p, off the curve; the
 * infinity encoding IS a valid Signature).  Any non-zero status is a record the reference drops --
 * bincode::deserialize::<Signature> fails, "Deserialize failed", operator.rs:108-113 -- so a caller
 * leaves that share out of its job (out96[i] is then meaningless).  The subgroup check stays with
 * verify (sig_groupcheck), as in the reference. */
int ssb_decode_wire_sigs(ssb_ctx* ctx, size_t n, const uint8_t* wire, size_t stride, uint8_t* out96,
                         int32_t* status);
/* device pointers, enqueued on `stream` (hipStream_t as void*), no synchronisation */
int ssb_decode_wire_sigs_dev(ssb_ctx* ctx, size_t n, const uint8_t* wire, size_t stride, uint8_t* out96,
                             int32_t* status, void* stream);

int ssb_hash_to_g2(ssb_ctx* ctx, size_t n, const uint8_t* msgs32, const uint8_t* dst, size_t dst_len,
                   uint8_t* out192);
/* Same for messages shorter than a root: message i is the first msg_len[i] <= 32 bytes of the
 * 32-byte slot msgs32 + 32 i (RFC 9380's test vectors, e.g. the empty message of Appendix K.2). */
int ssb_hash_to_g2_msgs(ssb_ctx* ctx, size_t n, const uint8_t* msgs32, const uint8_t* msg_len, const uint8_t* dst,
                        size_t dst_len, uint8_t* out192);

/* verdicts[i] = Signature::verify(pk48[i], roots32[root_idx[i]]) for sig96[i]  (1/0). */
int ssb_verify_batch(ssb_ctx* ctx, size_t n, const uint8_t* pk48, const uint8_t* sig96,
                     const uint32_t* root_idx, size_t n_roots, const uint8_t* roots32,
                     const uint8_t* dst, size_t dst_len, uint64_t rlc_seed, uint8_t* verdicts);

/* Same, device pointers, enqueued on the next pipeline slot after `stream` (hipStream_t; NULL =
 * default); the verdicts are ready when `stream` reaches them.  Root indices >= n_roots give
 * verdict 0.  The _cached variant takes per-share indices into the ssb_pk_cache_set table.  With
 * the validators' master keys and the combined signatures this is the combined-signature
 * verify (a-8), batched across validators by RLC. */
int ssb_verify_batch_dev(ssb_ctx* ctx, size_t n, const uint8_t* pk48, const uint8_t* sig96, const uint32_t* root_idx,
                         size_t n_roots, const uint8_t* roots32, const uint8_t* dst, size_t dst_len, uint64_t rlc_seed,
                         uint8_t* verdicts, void* stream);
int ssb_verify_batch_cached_dev(ssb_ctx* ctx, size_t n, const uint32_t* pk_index, const uint8_t* sig96,
                                const uint32_t* root_idx, size_t n_roots, const uint8_t* roots32, const uint8_t* dst,
                                size_t dst_len, uint64_t rlc_seed, uint8_t* verdicts, void* stream);

/* Batched threshold_aggregate.  Job j owns shares [share_off[j], share_off[j+1]) of sig96 /
 * pk48 / ids (input order = the reference's scan order), threshold t[j], and signs
 * roots32[job_root[j]].  Per job: out_status[j] (SSB_DVF_*), out_err[2j..2j+1] (error fields),
 * out_sig96[j] (combined signature, on SSB_DVF_OK).  share_verdicts (may be NULL) receives the
 * verify result of EVERY share (the reference stops verifying at the t-th valid share; the
 * combined signature is identical because every valid share lies on the same polynomial). */
int ssb_threshold_aggregate_batch(ssb_ctx* ctx, size_t n_jobs, const uint32_t* share_off,
                                  const uint32_t* t, const uint8_t* sig96, const uint8_t* pk48,
                                  const uint64_t* ids, const uint32_t* job_root, size_t n_roots,
                                  const uint8_t* roots32, const uint8_t* dst, size_t dst_len,
                                  uint64_t rlc_seed, uint8_t* out_sig96, int32_t* out_status,
                                  uint64_t* out_err, uint8_t* share_verdicts);

/* Asynchronous form of ssb_threshold_aggregate_batch (same arguments and checks, plus `ticket`):
 * the inputs are copied into the next pipeline slot's pinned, device-mapped staging buffer (a host
 * memcpy; the caller's input buffers are free again on return), the batch is enqueued on that slot
 * with its kernels reading the staging buffer in place over PCIe and writing their outputs there
 * (zero-copy: no copy kernels, no copy queues), and the call returns.  ssb_batch_wait(ctx, ticket)
 * blocks until the batch is done and copies its outputs to out_sig96 / out_status / out_err /
 * share_verdicts, which the caller keeps valid until then.  A slot's previous host batch is
 * delivered the same way before the slot is reused, so with ssb_set_pipeline_depth(S) up to S
 * batches are in flight.  ssb_threshold_aggregate_batch = submit + wait. */
int ssb_threshold_aggregate_batch_submit(ssb_ctx* ctx, size_t n_jobs, const uint32_t* share_off,
                                         const uint32_t* t, const uint8_t* sig96, const uint8_t* pk48,
                                         const uint64_t* ids, const uint32_t* job_root, size_t n_roots,
                                         const uint8_t* roots32, const uint8_t* dst, size_t dst_len,
                                         uint64_t rlc_seed, uint8_t* out_sig96, int32_t* out_status,
                                         uint64_t* out_err, uint8_t* share_verdicts, uint64_t* ticket);
/* Same with public keys as indices into the ssb_pk_cache_set table (ssb_threshold_aggregate_batch_cached_dev). */
int ssb_threshold_aggregate_batch_cached_submit(ssb_ctx* ctx, size_t n_jobs, const uint32_t* share_off,
                                                const uint32_t* t, const uint8_t* sig96, const uint32_t* pk_index,
                                                const uint64_t* ids, const uint32_t* job_root, size_t n_roots,
                                                const uint8_t* roots32, const uint8_t* dst, size_t dst_len,
                                                uint64_t rlc_seed, uint8_t* out_sig96, int32_t* out_status,
                                                uint64_t* out_err, uint8_t* share_verdicts, uint64_t* ticket);
/* Wait for a submitted batch and deliver its outputs (SSB_OK at once if already delivered;
 * SSB_EHIP if the batch did not complete -- its statuses are then SSB_DVF_ENGINE_ERROR).
 * LIFETIME: the library keeps the output pointers a _submit call received and writes into them
 * when the batch is delivered -- inside ssb_batch_wait, or earlier inside any later call that
 * delivers the slot's pending batch (the next submit to that slot, ssb_set_pipeline_depth,
 * ssb_set_slot_streams, ssb_pk_cache_set / _add when they wait, ssb_kernel_timing, ssb_destroy).
 * The caller keeps out_sig96 / out_status / out_err / share_verdicts valid until ssb_batch_wait
 * on the ticket has returned. */
int ssb_batch_wait(ssb_ctx* ctx, uint64_t ticket);

/* ---- Per-slot collector --------------------------------------------------------
 * The batched caller in front of ssb_threshold_aggregate_batch_cached_dev that SafeStake's per-duty
 * tasks use instead of one threshold_aggregate call each (HotstuffOperatorCommittee::sign,
 * src/validation/impls/hotstuff.rs:141-169; the call at :165-166).  Any number of threads submit
 * jobs concurrently (lock-free reservation in the open window, the job's bytes copied straight into
 * the window's pinned, device-mapped buffer); one worker thread closes a window when it holds
 * max_jobs jobs / max_shares shares, when its first job has waited window_us, or on flush, and
 * launches it on the next of `in_flight` one-stream pipeline slots with the public keys from the key
 * table (ssb_pk_cache_add).  Up to `in_flight` windows run on the device while the next one fills;
 * every job's result is exactly threshold_aggregate's for that job alone (generic_threshold.rs:132-175).
 * The collector sets the context to one-stream slots at pipeline depth in_flight (and leaves it so
 * after ssb_collector_destroy).  While a collector is attached the slot configuration is its own:
 * ssb_set_pipeline_depth / ssb_set_slot_streams return SSB_EINVAL, and a second collector on the
 * context must use the same in_flight.  The context stays usable by other threads while the
 * collector exists -- every entry point takes the context's lock -- so ONE context per process serves
 * the collector, direct calls (unsafe_aggregate, signing, key validation) and key registration. */
typedef struct ssb_collector ssb_collector;
typedef struct ssb_job_result {
  uint8_t sig96[96];     /* the combined signature (status SSB_DVF_OK) */
  uint64_t err[2];       /* DvfError fields of the status (ssbls.h status tags) */
  uint64_t verdicts;     /* bit i: share i's verify result (the first 64 shares) */
  int32_t status;        /* SSB_DVF_* ; SSB_DVF_ENGINE_ERROR when the job's batch failed (rc) */
  int32_t rc;            /* SSB_OK, or the negative SSB_E* code of the job's batch */
  uint32_t n_shares;
  uint32_t done;         /* 0 while pending; 1 (written last, release) when the fields are final */
  uint64_t absent;       /* wire collectors: bit i set when share i's record did not deserialize -- the
                            share was dropped from the job as the reference drops it (verdict 0) */
} ssb_job_result;
/* Called on the collector's worker thread when a job's result is final (after `done` is set); must
 * not block or call ssb_collector_* functions (e.g. complete a future / send on a channel and
 * return).  With a callback the result must stay valid until the callback has returned. */
typedef void (*ssb_job_done_fn)(void* user, const ssb_job_result* result);

/* in_flight: 1..SSB_MAX_SLOT_STREAMS one-stream pipeline slots; up to 2 x in_flight windows are on the
 * device (one running and one queued per slot, so a slot's stream never idles while the worker
 * delivers); max_shares: share capacity of a window (>= 64); window_us: how long the first job of a
 * window waits for company. */
int ssb_collector_create(ssb_ctx* ctx, uint32_t max_jobs, uint32_t max_shares, uint32_t window_us, int in_flight,
                         ssb_collector** out);
/* Flags of ssb_collector_create2.  SSB_COLLECTOR_WIRE: the windows hold every share as a wire record
 * (bincode(bls::Signature), 202 bytes), and ssb_collector_submit_wire takes the bytes a remote
 * operator sent -- no CPU deserialization on the receive path (src/validation/operator.rs:108); the
 * window runs as one ssb_threshold_aggregate_batch_wire_cached_dev batch, so a record that does not
 * deserialize makes its share absent (ssb_job_result.absent), exactly the reference's drop.  A
 * compressed share submitted with ssb_collector_submit is stored as its record (bincode::serialize).
 * max_jobs <= 2^20, max_shares <= 2^26.  in_flight above ssb_hw_queue_budget() - 1 is lowered to it
 * (with a warning on stderr). */
#define SSB_COLLECTOR_WIRE 1u
int ssb_collector_create2(ssb_ctx* ctx, uint32_t max_jobs, uint32_t max_shares, uint32_t window_us, int in_flight,
                          uint32_t flags, ssb_collector** out);
/* Drains: every submitted job is delivered before it returns.  The context stays usable. */
void ssb_collector_destroy(ssb_collector* col);
/* ssb_pk_cache_add through the collector (serialised with its launches). */
int ssb_collector_register_keys(ssb_collector* col, size_t n, const uint8_t* pk48, uint32_t* out_index);
/* One threshold_aggregate job: t, n shares (1 <= t <= SSB_MAX_T, n <= 64; the caller has done the
 * reference's two DifferentLength checks), sig96[n], pk_index[n] (rows of the key table), ids[n],
 * the 32-byte signing root.  `result` (caller-owned, valid until done) receives the outcome; `cb`
 * (may be NULL) is then called with `user`.  Thread-safe; blocks only while every window buffer is
 * busy (back-pressure). */
int ssb_collector_submit(ssb_collector* col, uint32_t t, uint32_t n, const uint8_t* sig96, const uint32_t* pk_index,
                         const uint64_t* ids, const uint8_t* root32, ssb_job_result* result, ssb_job_done_fn cb,
                         void* user);
/* A job whose shares are the wire records as received (a SSB_COLLECTOR_WIRE collector): share i is
 * wire[i] (wire_len[i] bytes).  As bincode::deserialize (bincode 1.3.3, trailing bytes allowed) the
 * first 202 bytes are decoded and any further bytes ignored; a shorter record, or a NULL one, never
 * deserializes: the share is absent.  Otherwise as ssb_collector_submit; the bytes are copied before
 * it returns. */
int ssb_collector_submit_wire(ssb_collector* col, uint32_t t, uint32_t n, const uint8_t* const* wire,
                              const size_t* wire_len, const uint32_t* pk_index, const uint64_t* ids,
                              const uint8_t* root32, ssb_job_result* result, ssb_job_done_fn cb, void* user);
/* Block until result->done (the job must have been submitted to this collector). */
int ssb_collector_wait(ssb_collector* col, const ssb_job_result* result);
/* Close the open window now and wait until every job submitted before the call is delivered. */
int ssb_collector_flush(ssb_collector* col);
/* Counters since creation: windows launched, jobs and shares delivered. */
int ssb_collector_stats(ssb_collector* col, uint64_t* windows, uint64_t* jobs, uint64_t* shares);
/* Worker-thread profile since creation: time closing + launching windows, delivering results, and
 * waiting for a device window to free up (every window on the device busy), and how many submits
 * waited for a new window. */
int ssb_collector_profile(ssb_collector* col, double* seal_ms, double* deliver_ms, double* backpressure_ms,
                          uint64_t* full_waits);

/* Same, all array arguments are device pointers; `stream` is a hipStream_t (NULL = default).
 * The caller owns the job shapes: share_off must be non-decreasing with share_off[n_jobs] ==
 * n_shares and 1 <= t[j] <= SSB_MAX_T; a job that breaks this (the library cannot check device
 * arrays without a synchronisation) gets status SSB_DVF_INVALID_JOB and no output, and never makes
 * a kernel index outside the batch. */
int ssb_threshold_aggregate_batch_dev(ssb_ctx* ctx, size_t n_jobs, size_t n_shares,
                                      const uint32_t* share_off, const uint32_t* t,
                                      const uint8_t* sig96, const uint8_t* pk48, const uint64_t* ids,
                                      const uint32_t* job_root, size_t n_roots, const uint8_t* roots32,
                                      const uint8_t* dst, size_t dst_len, uint64_t rlc_seed,
                                      uint8_t* out_sig96, int32_t* out_status, uint64_t* out_err,
                                      uint8_t* share_verdicts, void* stream);

/* Decoded public keys.  ssb_pk_cache_set decompresses n public keys once (synchronous) into the
 * context's table (replacing any previous table), the way lighthouse's PublicKey holds the
 * decompressed point; ssb_threshold_aggregate_batch_cached_dev then takes, per share, an index
 * into that table instead of 48 compressed bytes.  A key that does not decode, decodes to
 * infinity, or an index >= n makes the share invalid (verdict 0), as in the compressed path. */
int ssb_pk_cache_set(ssb_ctx* ctx, size_t n, const uint8_t* pk48);
/* Incremental registration (a committee's operator keys when it is built: DvfSigner::spawn,
 * src/node/dvfcore.rs:144-235, OperatorCommittee::from_definition, src/validation/operator_committees.rs:13-30):
 * out_index[i] = the table row of pk48[i].  A key already in the table (from this call, an earlier
 * add, or a _set) keeps its row; new keys are decoded (and their merged-MSM bases precomputed) into
 * rows after the existing ones, so indices stay stable and batches already in flight are unaffected.
 * Synchronous; when the table's capacity doubles it first waits for every in-flight batch. */
int ssb_pk_cache_add(ssb_ctx* ctx, size_t n, const uint8_t* pk48, uint32_t* out_index);
int ssb_threshold_aggregate_batch_cached_dev(ssb_ctx* ctx, size_t n_jobs, size_t n_shares,
                                             const uint32_t* share_off, const uint32_t* t,
                                             const uint8_t* sig96, const uint32_t* pk_index,
                                             const uint64_t* ids, const uint32_t* job_root, size_t n_roots,
                                             const uint8_t* roots32, const uint8_t* dst, size_t dst_len,
                                             uint64_t rlc_seed, uint8_t* out_sig96, int32_t* out_status,
                                             uint64_t* out_err, uint8_t* share_verdicts, void* stream);

/* The same with the partial signatures as WIRE RECORDS, the bytes a remote operator sends: record i at
 * wire + i * stride (stride >= 202) is bincode(bls::Signature) (ssb_decode_wire_sigs), decoded and
 * decompressed on the device -- the CPU never deserializes the share (RemoteOperator::sign,
 * src/validation/operator.rs:108).  A record that does not deserialize (share_wire_status[i]: 1 length,
 * 2 prefix, 3 hex digit, 4 not a curve point; 0 ok) makes its share ABSENT, as the reference drops it
 * before threshold_aggregate (operator.rs:108-131, the `.flatten()` of hotstuff.rs:150-155): it does not
 * count towards the job's share count -- InsufficientSignatures{got: present shares, expected: t} --
 * and the scan never meets it (verdict 0).  share_wire_status: n_shares int32, device. */
int ssb_threshold_aggregate_batch_wire_cached_dev(ssb_ctx* ctx, size_t n_jobs, size_t n_shares,
                                                  const uint32_t* share_off, const uint32_t* t,
                                                  const uint8_t* wire, size_t stride, const uint32_t* pk_index,
                                                  const uint64_t* ids, const uint32_t* job_root, size_t n_roots,
                                                  const uint8_t* roots32, const uint8_t* dst, size_t dst_len,
                                                  uint64_t rlc_seed, uint8_t* out_sig96, int32_t* out_status,
                                                  uint64_t* out_err, uint8_t* share_verdicts,
                                                  int32_t* share_wire_status, void* stream);

/* Batched unsafe_aggregate: job j combines ALL its shares [share_off[j], share_off[j+1]) with
 * Lagrange coefficients of its ids (t = share count), starting from infinity. */
int ssb_unsafe_aggregate_batch(ssb_ctx* ctx, size_t n_jobs, const uint32_t* share_off,
                               const uint8_t* sig96, const uint64_t* ids, uint8_t* out_sig96,
                               int32_t* out_status);

/* Batched local partial signing (SecretKey::sign = H(m)*sk, src/node/dvfcore.rs:241-243):
 * out_sig96[i] = compress(sk_i * hash_to_G2(roots32[root_idx[i]])), sk as 32-byte little-endian
 * scalars (< r).  Also the synthetic-input generator of bench.py. */
int ssb_sign_batch(ssb_ctx* ctx, size_t n, const uint8_t* sk32le, const uint32_t* root_idx, size_t n_roots,
                   const uint8_t* roots32, const uint8_t* dst, size_t dst_len, uint8_t* out_sig96);

/* SecretKey::public_key: out_pk48[i] = compress(sk_i * g1). */
int ssb_sk_to_pk_batch(ssb_ctx* ctx, size_t n, const uint8_t* sk32le, uint8_t* out_pk48);

/* bls::PublicKey::deserialize + PublicKey::serialize (lighthouse; blst key_validate), batched: out_valid[i]
 * = 1 iff pk48[i] decodes (ZCash flags, x < p, on the curve), is not infinity and lies in G1; then
 * out_pk48[i] is its recompression (equal to the input for a canonical encoding), else zeros.  The
 * keys every other entry point takes are expected to have passed this (registration time; pinned
 * by the keys the reference's own sources deserialize, tests/golden/reference_kats.json). */
int ssb_pk_validate_batch(ssb_ctx* ctx, size_t n, const uint8_t* pk48, uint8_t* out_valid, uint8_t* out_pk48);

/* lagrange_coeffs for one id set: out 32-byte little-endian scalars (blst_scalar.b layout). */
int ssb_lagrange_coeffs(ssb_ctx* ctx, size_t t, const uint64_t* ids, uint8_t* out32);

/* ---- Local-signing window -----------------------------------------------------
 * The batched form of DvfSigner::local_sign_and_store's SecretKey::sign (src/node/dvfcore.rs:241-251),
 * which every duty reaches once per validator (src/validation/signing_method.rs:318; selection proofs
 * and RANDAO reveals included, :269-292).  Submissions from any number of threads join the open
 * window; a worker thread closes it at max_jobs submissions or window_us after its first (or on
 * flush) -- a window holds at most max_jobs: what arrives while one is being signed opens the next --
 * signs it with ONE ssb_sign_batch (each distinct root hashed once) and completes every
 * submission: sig96 = compress([sk] hash_to_G2(root)) with the POP DST of src/crypto/impls/blst.rs:11,
 * byte for byte SecretKey::sign's output.  The keys are wiped from the library's buffers once used. */
typedef struct ssb_signer ssb_signer;
typedef struct ssb_sign_result {
  uint8_t sig96[96];   /* the signature (rc == SSB_OK) */
  int32_t rc;          /* SSB_OK, or the window's ssb_sign_batch error */
  uint32_t done;       /* 0 while pending; 1 (written last, release) when final */
} ssb_sign_result;
/* Called on the signer's worker thread after `done` is set; must not block or call ssb_signer_*. */
typedef void (*ssb_sign_done_fn)(void* user, const ssb_sign_result* result);
int ssb_signer_create(ssb_ctx* ctx, uint32_t max_jobs, uint32_t window_us, ssb_signer** out);
/* Drains: every submission is signed and delivered before it returns. */
void ssb_signer_destroy(ssb_signer* s);
/* One signature: sk32le the secret scalar (32 bytes little-endian, 0 < sk < r -- a lighthouse
 * SecretKey's bytes reversed), root32 the signing root; `result` (caller-owned, valid until done)
 * receives it, then `cb` (may be NULL) is called with `user`.  Thread-safe; the key is copied. */
int ssb_signer_submit(ssb_signer* s, const uint8_t* sk32le, const uint8_t* root32, ssb_sign_result* result,
                      ssb_sign_done_fn cb, void* user);
int ssb_signer_wait(ssb_signer* s, const ssb_sign_result* result);
/* Close the open window now and wait until every submission made before the call is delivered. */
int ssb_signer_flush(ssb_signer* s);
int ssb_signer_stats(ssb_signer* s, uint64_t* windows, uint64_t* signatures);

#ifdef __cplusplus
}
#endif
#endif /* SSBLS_H */
