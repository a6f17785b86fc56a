/*
 * stl.h -- C ABI of libstl, the MI355X (gfx950) batched Ed25519
 * transaction-signature verifier for stellard.
 *
 * Drop-in boundary (reference = hfeeki/stellard, libsodium not vendored):
 *
 *   lower boundary replaced: libsodium
 *     int crypto_sign_verify_detached(const unsigned char *sig,
 *                                     const unsigned char *m,
 *                                     unsigned long long mlen,
 *                                     const unsigned char *pk);
 *     called at src/ripple_data/protocol/RippleAddress.cpp:196-197 and
 *     src/ripple_data/crypto/StellarPublicKey.cpp:73-74
 *   upper boundary mirrored:
 *     bool RippleAddress::verifySignature(uint256 const&, Blob const&) const
 *       src/ripple_data/protocol/RippleAddress.cpp:190-200 (= verify && S<L)
 *     bool SerializedTransaction::checkSign(const RippleAddress&) const
 *       src/ripple_app/misc/SerializedTransaction.cpp:220-230
 *       (= SHA512Half(signing preimage) then verifySignature)
 *
 * Conventions: plain pointers and sizes, caller-owned host buffers, no
 * exceptions across the ABI, nothing retained after return.  Accept bitmaps
 * are ceil(n/8) bytes, bit i = byte i>>3, bit (i & 7), LSB first; a set bit
 * means ACCEPT under stellard's composite predicate (verify && S < L).
 *
 * Return codes: STL_OK (0) or a negative error.  On error the bitmap is
 * undefined and the caller MUST fall back to its own per-signature check --
 * a device error is never reported as a reject.  libstl itself has no CPU
 * verify path.
 */
#ifndef STL_H
#define STL_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define STL_ABI_VERSION 3

/* ---- return codes ---- */
#define STL_OK 0
#define STL_EINVAL (-22)   /* bad argument (null pointer with n > 0, bad flags, bad length) */
#define STL_ENODEV (-19)   /* no gfx950 device available / not initialised */
#define STL_ENOMEM (-12)   /* device or host allocation failed */
#define STL_EHIP (-1000)   /* HIP runtime error (kernel launch, copy, sync) */
#define STL_ERCCL (-1001)  /* RCCL missing, communicator setup or a collective failed */

/* ---- flags ---- */
/* Accept predicate of crypto_sign_verify_detached to reproduce.  Default is
 * the container's executable oracle, libsodium 1.0.18 (S < L, R and A not of
 * small order, A canonical).  STELLARD_1_0_0 reproduces the ref10-era
 * predicate of the libsodium the reference pins (Dockerfile:9-10): only
 * (sig[63] & 0xE0) == 0, plus a reject of the all-zero key (as some 1.0.x
 * releases did).  Parity for it is unpinned offline; where
 * the offline restatement cannot be pinned the policy errs toward reject,
 * which is the safe side -- the caller re-checks every reject serially. */
#define STL_POLICY_SODIUM_1_0_18 0x0u
#define STL_POLICY_STELLARD_1_0_0 0x1u
#define STL_POLICY_MASK 0x1u
/* stellard's crypto_sign_check_S_lt_l (RippleAddress.cpp:226-252) is always
 * applied (composite predicate); the flag exists for ABI symmetry. */
#define STL_REQUIRE_S_LT_L 0x2u
/* Check every signature with full-length scalars ([S]B - [k]A, 253-bit
 * chain) instead of the half-size-scalar equation.
 * Same accept bits, about 1.6x slower; a cross-check / reference mode. */
#define STL_FULL_LENGTH 0x4u
/* Decode each distinct public key of a batch once (stellard's signers repeat:
 * the configs-1/5 shape is 1,000 accounts for 100k transactions).  Same
 * accept bits; costs a hash pass and extra device workspace: about 270 MB
 * (stl_kernels.h kDedupBytes: hash slots, key arrays, decoded keys, shared and
 * wide key tables), allocated once per device for the host batch API and once
 * per (device, stream) -- per library stream too, and for at most
 * STL_TUNE_STREAM_WORKSPACES caller streams -- for the device-resident API.
 * Does not pay when keys are all distinct.  Chunks small enough for lane
 * pairs or quads (STL_ONE_LANE below) run on them instead: latency-bound
 * there, the pairs and quads are faster. */
#define STL_DEDUP_KEYS 0x8u
/* The host batch calls (stl_ed25519_verify_batch, stl_tx_verify_batch, the
 * blob calls) choose STL_DEDUP_KEYS by themselves for every 64K-row chunk in
 * which a host-side sample of 1,024 evenly spaced keys shows at least a fifth
 * repeating an earlier one (about 40 us per chunk, overlapped with the earlier
 * chunks' kernels); this flag turns the automatic choice off (A/B and callers
 * that know their keys are distinct).  The device-resident verify and
 * checkSign calls choose by feedback instead (their keys are in HBM): each
 * call ends with a one-workgroup sample of 2,048 keys on the caller's stream
 * (dedup when at least a quarter repeat), and the next call on that stream
 * follows that sample's verdict (no synchronisation; a stream's first call
 * runs without dedup).  The bits never depend on the choice. */
#define STL_NO_AUTO_DEDUP 0x20u
/* Small chunks run each signature on two lanes, which ends a launch that
 * cannot fill the device sooner: the main kernel up to
 * a quarter of the device's resident lanes (one pair wave per SIMD; 32,768
 * signatures on 256 CUs), on eight lanes (two lane quads) up to one quad wave
 * per SIMD (8,192 signatures) and on four (two duos) up to one duo wave per
 * SIMD (16,384; STL_TUNE_QUAD), the point decoding on pairs up to half of
 * them.  Same accept bits; this flag turns both off (A/B and
 * tests). */
#define STL_ONE_LANE 0x10u
/* TEST-ONLY: the raw crypto_sign_verify_detached predicate of the selected
 * policy, without stellard's S < L -- what RippleAddress_test expects of the
 * bare libsodium call (RippleAddress.cpp:838-845: under the 1.0.0 policy a
 * signature with S + L verifies).  stellard's accept is always the composite;
 * never set this outside tests. */
#define STL_DEBUG_RAW_PREDICATE 0x80000000u

/* stl_config.flags.  By default every device of a host batch call copies its
 * slice of the accept bitmap to the host.  With STL_CFG_RCCL_GATHER the slices
 * are gathered on device 0 with RCCL over xGMI (ncclGather / grouped
 * send-recv into one buffer, any device count) and copied to the host once;
 * stl_init returns STL_ERCCL if that communicator cannot be built.  (Opt-in
 * until a multi-GPU run has compared the gathered bitmaps: the one-process-
 * per-GPU gather, stl_bitmap_gather_device, is the measured path.) */
#define STL_CFG_RCCL_GATHER 0x1u /* gather the bitmap over RCCL (in-process communicator) */
#define STL_CFG_NO_RCCL 0x2u     /* never use RCCL: every device copies its slice to the host */

/* The caller's own single-signature check, libsodium's signature:
 * stellard passes crypto_sign_verify_detached (libstl never links it). */
typedef int (*stl_verify_fn)(const unsigned char *sig, const unsigned char *m, unsigned long long mlen,
                             const unsigned char *pk);

typedef struct stl_config {
  uint32_t struct_size;       /* sizeof(stl_config); the 16-byte ABI-1 and 24-byte ABI-2 structs
                                 are accepted too */
  int32_t device_count;       /* devices to use; <= 0 = all visible */
  int32_t first_device;       /* first HIP ordinal to use */
  uint32_t flags;             /* STL_CFG_* */
  int32_t shards_per_device;  /* ABI 2: host batch shards per device, each on its own host
                                 thread (<= 0 = 1; more than 1 forces the per-device copy) */
  uint32_t reserved;          /* 0 */
  stl_verify_fn fallback_verify; /* ABI 3, may be NULL: with it, stl_ed25519_verify_detached
                                    answers a device failure (ENODEV, ENOMEM, EHIP, ERCCL)
                                    with fallback_verify(...) == 0 && S < L, so it returns
                                    only 0 or -1 -- libsodium's convention.  Registered even
                                    when stl_init itself then fails for want of a device. */
} stl_config;

/* Replaces/augments sodium_init() (src/ripple_app/ripple_app.cpp:129-132).
 * Idempotent; cfg may be NULL (all devices).  Thread-safe.  When libstl is
 * already running (an earlier stl_init, or the implicit one of a first entry-
 * point call) a cfg still registers its fallback_verify and returns STL_OK if
 * it asks for the live device set, gather mode and shard count, STL_EINVAL
 * otherwise (stl_shutdown first to change them).  Environment
 * overrides: STL_DEVICES (device count), STL_SHARDS_PER_DEVICE, STL_RCCL
 * (1 = as STL_CFG_RCCL_GATHER, 0 = as STL_CFG_NO_RCCL), STL_FAULT_AFTER
 * (stl_debug_fault_after). */
int stl_init(const stl_config *cfg);
void stl_shutdown(void);
int stl_device_count(void);
const char *stl_version(void);
const char *stl_strerror(int rc);

/* Same signature as libsodium's crypto_sign_verify_detached (0 = accept,
 * -1 = reject), plus stellard's S<L: i.e. exactly
 * RippleAddress::verifySignature's bool as 0/-1.  Runs on the GPU (batch of
 * one).  A device failure returns a value < -1 -- unless stl_config's
 * fallback_verify was registered, in which case the call answers with it and
 * only ever returns 0 or -1.  Only with a fallback registered is this a
 * literal drop-in for `crypto_sign_verify_detached(...) == 0` at
 * RippleAddress.cpp:196-197: without one a device error must be told apart
 * from a reject by the caller (rc < -1).  STL_EINVAL (a NULL pointer) is
 * returned either way; a message longer than 2^32 - 1 bytes is STL_EINVAL
 * without a fallback and the fallback's answer (&& S < L) with one.
 * LATENCY: a signature's chain runs on eight GPU lanes (two lane quads), so a
 * call is latency-bound: 295 us per call on MI355X against libsodium's 31 us
 * (round 4; 489 us on lane pairs in round 2), and concurrent calls
 * serialise on the device (tools/latency.py).
 * Callers that verify one signature at a time (stellard's JobQueue workers)
 * keep libsodium, or submit through stl_batcher_* when many requests are in
 * flight; this entry point is the drop-in for correctness, not for speed. */
int stl_ed25519_verify_detached(const uint8_t *sig, const uint8_t *m, unsigned long long mlen,
                                const uint8_t *pk);

/* n signatures over 32-byte messages (the stellard signing hash).
 * sig: n*64 bytes (R || S), msg: n*32, pk: n*32 -- caller host memory.
 * Sharded by index over the initialised devices (contiguous, 64-aligned). */
int stl_ed25519_verify_batch(const uint8_t *sig, const uint8_t *msg, const uint8_t *pk, size_t n,
                             uint8_t *accept_bitmap, uint32_t flags);

/* checkSign equivalent: msg_i = SHA512Half(preimage_i), then verify.
 * preimage_i = preimages[offset[i] .. offset[i]+len[i]) and already includes
 * the 4-byte "STX\0" prefix (HashPrefix::txSign, HashPrefix.cpp:30).  Any
 * prefixed preimage works the same way, e.g. a consensus proposal's 76-byte
 * "PRP\0" || seq || closeTime || prevLedger || position
 * (LedgerProposal::getSigningHash, LedgerProposal.cpp:54-65).  Offsets may
 * come in any order; with several devices the rows are split into
 * contiguous 64-aligned shards of about equal preimage bytes. */
int stl_tx_verify_batch(const uint8_t *preimages, const uint64_t *offset, const uint32_t *len,
                        const uint8_t *sig, const uint8_t *pk, size_t n, uint8_t *accept_bitmap,
                        uint32_t flags);

/* ---- device-resident entry points (asynchronous on the caller's stream) ----
 * All pointers are device pointers on the current HIP device; stream is a
 * hipStream_t (NULL = default stream).  The bitmap is written as
 * ceil(n/64) little-endian 64-bit words (same bit order as above). */
int stl_ed25519_verify_batch_device(const uint8_t *d_sig, const uint8_t *d_msg, const uint8_t *d_pk,
                                    size_t n, uint64_t *d_bitmap_words, uint32_t flags, void *stream);

/* SHA512Half over n preimages -> d_msg (n*32 bytes). */
int stl_tx_hash_batch_device(const uint8_t *d_preimages, const uint64_t *d_offset, const uint32_t *d_len,
                             size_t n, uint8_t *d_msg, void *stream);

/* Device-resident checkSign: SHA512Half(preimage_i) then verify, over rows in
 * HBM (preimages as stl_tx_verify_batch's; d_sig n*64, d_pk n*32).  Cut into
 * the verify's chunks and spread over the caller's stream and one of libstl's,
 * each chunk's hashing right before its verify, so the hashing overlaps the
 * other stream's kernels.  Bits = stl_tx_hash_batch_device followed by
 * stl_ed25519_verify_batch_device on the same stream. */
int stl_tx_verify_batch_device(const uint8_t *d_preimages, const uint64_t *d_offset, const uint32_t *d_len,
                               const uint8_t *d_sig, const uint8_t *d_pk, size_t n, uint64_t *d_bitmap_words,
                               uint32_t flags, void *stream);

/* ---- serialized transactions ----
 * checkSign straight from serialized transactions -- the bytes of
 * TMTransaction.rawTransaction, or what STObject::add writes: n blobs at
 * blobs[offset[i] .. offset[i]+len[i]), each the full transaction including
 * its TxnSignature field.  Replaces, per transaction, the
 * SerializedTransaction(SerializerIterator&) -> getSigningHash ->
 * checkSign sequence (SerializedTransaction.cpp:65-92,162-165,192-230) and
 * getTransactionID (SerializedTransaction.cpp:167-171).  The device splices
 * the signing preimage out of the blob ("STX\0" || blob minus TxnSignature,
 * Signature, TxnSignatures), which equals the reference's re-serialisation
 * when the blob is in canonical form; it checks that form and DEFERS every
 * blob it cannot prove canonical (stellard_amd/csrc/stl_txblob.h lists the
 * rules).  It also restates the constructor's template checks
 * (SerializedTransaction.cpp:79-91: TransactionType present with a TxFormats
 * template, required fields present, no field outside the template), so
 * STL_TX_OK implies the reference constructs the transaction; raw wire bytes
 * are a safe input.  Validations (STL_BLOB_VALIDATION) with a field outside
 * SerializedValidation's template are deferred (the reference drops such a
 * field from the signing hash).  Per-transaction status: */
#define STL_TX_OK 0        /* accept bit = checkSign(); tx_id valid */
#define STL_TX_DEFERRED 1  /* accept bit 0; caller runs its own checkSign; tx_id zero */
#define STL_TX_MALFORMED 2 /* SigningPubKey not 32 B or TxnSignature not 64 B: checkSign()
                              is false (RippleAddress.cpp:192-194); accept bit 0; tx_id valid */

/* status: n bytes or NULL; tx_id: n*32 bytes (SHA512Half("TXN\0" || blob)) or NULL. */
int stl_tx_blob_verify_batch(const uint8_t *blobs, const uint64_t *offset, const uint32_t *len, size_t n,
                             uint8_t *accept_bitmap, uint8_t *status, uint8_t *tx_id, uint32_t flags);

/* The same over other signed STObjects.  kind:
 *   STL_BLOB_TRANSACTION  as stl_tx_blob_verify_batch ("STX\0", TxnSignature;
 *                         id = SHA512Half("TXN\0" || blob))
 *   STL_BLOB_VALIDATION   SerializedValidation::isValid(getSigningHash()):
 *                         SHA512Half("VAL\0" || blob minus Signature) checked
 *                         against SigningPubKey / Signature
 *                         (SerializedValidation.cpp:70-73,96-110,
 *                         HashPrefix.cpp:31); id = SHA512Half(blob), the
 *                         suppression key of PeerImp::recvValidation
 *                         (PeerImp.cpp:1148-1155); blobs shorter than 50 bytes
 *                         (PeerImp.cpp:1134) are deferred. */
#define STL_BLOB_TRANSACTION 0u
#define STL_BLOB_VALIDATION 1u
int stl_signed_blob_verify_batch(uint32_t kind, const uint8_t *blobs, const uint64_t *offset, const uint32_t *len,
                                 size_t n, uint8_t *accept_bitmap, uint8_t *status, uint8_t *id, uint32_t flags);

/* Device-resident first half: writes the verify inputs (d_msg n*32, d_sig
 * n*64, d_pk n*32; a deferred or malformed transaction gets a signature that
 * always rejects), d_status (n bytes) and, if d_tx_id is not NULL, the
 * transaction IDs (n*32).  Follow with stl_ed25519_verify_batch_device on the
 * same stream. */
int stl_tx_blob_prepare_device(const uint8_t *d_blobs, const uint64_t *d_offset, const uint32_t *d_len,
                               size_t n, uint8_t *d_msg, uint8_t *d_sig, uint8_t *d_pk, uint8_t *d_tx_id,
                               uint8_t *d_status, void *stream);
int stl_signed_blob_prepare_device(uint32_t kind, const uint8_t *d_blobs, const uint64_t *d_offset,
                                   const uint32_t *d_len, size_t n, uint8_t *d_msg, uint8_t *d_sig, uint8_t *d_pk,
                                   uint8_t *d_id, uint8_t *d_status, void *stream);
/* The whole device-resident check from serialized objects in one call: the
 * blob pass and the verify chunk by chunk over two streams (as
 * stl_tx_verify_batch_device); d_status (n bytes) required, d_id (n*32) may be
 * NULL.  Bits and status = stl_signed_blob_prepare_device followed by
 * stl_ed25519_verify_batch_device. */
int stl_signed_blob_verify_batch_device(uint32_t kind, const uint8_t *d_blobs, const uint64_t *d_offset,
                                        const uint32_t *d_len, size_t n, uint64_t *d_bitmap_words, uint8_t *d_status,
                                        uint8_t *d_id, uint32_t flags, void *stream);

/* ---- multi-GPU: one process per GPU ----
 * Verification shards by index with no exchange; the accept bitmaps are
 * gathered with RCCL over xGMI.  rank r owns signatures
 * [r*w*64, (r+1)*w*64) of the whole batch, w = words_per_rank (see
 * stl_shard_range).  Setup: rank 0 calls stl_comm_unique_id and hands the
 * 128 bytes to every rank out of band (stellard: its own config; the bench:
 * torch.distributed over TCP); then every rank calls stl_comm_init_rank on its
 * initialised device, which blocks until all ranks have joined -- or until the
 * RCCL deadline (STL_RCCL_TIMEOUT_S at stl_init, default 120 s, or
 * STL_TUNE_RCCL_TIMEOUT_MS) passes: the communicator is then built
 * nonblocking (ncclCommInitRankConfig, blocking = 0) and polled
 * (ncclCommGetAsyncError); on the deadline it is aborted and the call returns
 * STL_ERCCL, and a later stl_comm_init_rank may try again. */
int stl_comm_unique_id(uint8_t id[128]);
int stl_comm_init_rank(int nranks, int rank, const uint8_t id[128]);
void stl_comm_destroy(void);
/* Aborts the communicator (ncclCommAbort: outstanding collectives end without
 * waiting for peers) -- the teardown after a failed or timed-out gather. */
void stl_comm_abort(void);
/* hipStreamSynchronize(stream) with the RCCL deadline (timeout_ms, or the
 * library's when <= 0) on the gather: the work queued on the stream ahead of
 * the last stl_bitmap_gather(v)_device is waited for first (a lapse of 10x the
 * deadline, or of the library's deadline if longer, there is STL_EHIP and
 * keeps the communicator), then, while the
 * stream has not drained, the communicator's asynchronous error is polled; an
 * RCCL error or the deadline aborts the communicator (which ends a stalled
 * gather's kernels) and returns STL_ERCCL, so a rank whose peers never arrive
 * can fall back instead of hanging.  A gather whose enqueue fails or times
 * out aborts the communicator the same way. */
int stl_comm_sync(void *stream, int timeout_ms);
/* What RCCL itself reports for the communicator libstl gathers over
 * (ncclCommCount / ncclCommUserRank): the one-process-per-GPU communicator of
 * stl_comm_init_rank if there is one, else the in-process communicator of
 * stl_init (the rank of the calling thread's current device).  STL_ERCCL when
 * there is neither. */
int stl_comm_info(int *nranks, int *rank);
/* root >= 0: ncclGather of every rank's d_words (words_per_rank u64 words)
 * into d_all_words on rank root (nranks*words_per_rank words, rank order;
 * other ranks may pass NULL); root < 0: ncclAllGather (every rank receives).
 * Asynchronous on stream. */
int stl_bitmap_gather_device(const uint64_t *d_words, size_t words_per_rank, uint64_t *d_all_words, int root,
                             void *stream);

/* Variable-size gather (byte-balanced shards: config 5's ledger split by
 * preimage bytes, stl_shard_range_bytes; or any unequal index shards): rank r
 * holds d_words = word_offsets[r+1] - word_offsets[r] (= nwords) u64 words,
 * which land at word word_offsets[r] of d_all_words on rank root.
 * word_offsets: nranks+1 host entries, identical on every rank.  Grouped
 * ncclSend / ncclRecv (the root's own slice is a device copy); asynchronous
 * on stream.  STL_EINVAL if nwords disagrees with the offsets.  The argument
 * checks are local to each rank and run before the group is posted: a rank
 * that gets STL_EINVAL (its nwords, or a NULL d_all_words on the root) does
 * not join, and its peers then block in their send / recv -- every rank must
 * pass the same word_offsets and its own slice's size. */
int stl_bitmap_gatherv_device(const uint64_t *d_words, size_t nwords, uint64_t *d_all_words,
                              const uint64_t *word_offsets, int root, void *stream);

/* Shard of [0, n) that rank r of g owns: contiguous, whole 64-signature
 * bitmap words (the layout stl_bitmap_gather_device assumes and the host
 * batch calls use across devices). */
void stl_shard_range(size_t n, int r, int g, size_t *lo, size_t *hi);
/* Byte-balanced shard for variable-length rows (config 5: preimages or blobs
 * of 100 B - 4 KB): boundaries at the 64-aligned row where the prefix sum of
 * len crosses r/g of the total -- each then moved to the nearest multiple of
 * the verify step (one main-kernel wave per SIMD of the first device: 65,536
 * rows on 256 CUs; 65,536 before stl_init) when that moves its byte prefix by
 * at most 2.5 % of one rank's share: the device-resident verify's time rises
 * in steps of that many rows, so a shard just past a step would pay a whole
 * extra step (config 5's 2^20 rows over 2, 4, 8 ranks: exactly 2^20 / g each). */
void stl_shard_range_bytes(const uint32_t *len, size_t n, int r, int g, size_t *lo, size_t *hi);

/* ---- request aggregator ----
 * stellard checks transactions one at a time on JobQueue workers
 * (jtTRANSACTION: PeerImp.cpp:64-73, NetworkOPs.cpp:298-320) and has an unused
 * batching hook, TxQueue::addEntryForSigCheck (TxQueue.h:32-33).  An
 * aggregator takes single requests from any thread and runs them as device
 * batches: a batch starts when max_batch requests are pending or the oldest
 * has waited max_delay_us.  Each request completes through its callback, on
 * the aggregator's worker thread, with one verdict: */
#define STL_VERDICT_REJECT 0
#define STL_VERDICT_ACCEPT 1
#define STL_VERDICT_DEFER 2 /* serialized tx not decided on the device (STL_TX_DEFERRED) */
/* or a negative STL_E* code: the batch failed, run your own check. */
typedef void (*stl_verdict_fn)(void *ctx, int verdict);
typedef struct stl_batcher stl_batcher;

/* flags: policy bits as for the batch calls.  NULL on bad arguments. */
stl_batcher *stl_batcher_create(uint32_t max_batch, uint32_t max_delay_us, uint32_t flags);
/* RippleAddress::verifySignature(hash, sig) for one signature (copied). */
int stl_batcher_submit(stl_batcher *b, const uint8_t *sig, const uint8_t *msg32, const uint8_t *pk,
                       stl_verdict_fn fn, void *ctx);
/* SerializedTransaction::checkSign for one serialized transaction (copied). */
int stl_batcher_submit_tx(stl_batcher *b, const uint8_t *blob, size_t len, stl_verdict_fn fn, void *ctx);
/* Returns when every request submitted before the call has completed.
 * Callbacks run on the aggregator's worker thread and must not call
 * stl_batcher_flush or stl_batcher_destroy on their own aggregator. */
void stl_batcher_flush(stl_batcher *b);
void stl_batcher_stats(stl_batcher *b, uint64_t *submitted, uint64_t *completed, uint64_t *batches);
/* Completes every pending request, then frees the aggregator. */
void stl_batcher_destroy(stl_batcher *b);

/* ---- statistics and tracing (metrics) ----
 * Cumulative since stl_init / stl_reset_stats.  Host side: entry-point calls
 * (the host batch / tx / blob calls), signatures submitted, calls that
 * returned < 0, wall time inside them and in the multi-GPU gather.  Device
 * side (every verify launch, host and device entry points): accept bits
 * written and signatures checked by the full-length fallback path.  Reading
 * the device counters synchronises the devices.  STL_TRACE=1 in the
 * environment at stl_init prints one JSON line per host call on stderr. */
typedef struct stl_stats {
  uint32_t struct_size; /* sizeof(stl_stats) */
  uint32_t reserved;
  uint64_t batches, signatures, errors;
  uint64_t host_ns, gather_ns;
  uint64_t accepted, full_length_lanes;
  /* Phase timing (stl_set_phase_timing(1) or STL_PHASE_TIMING=1; zero when
   * off): summed kernel time of the verify phases, measured with HIP events
   * recorded on the launch stream between the phases of every chunk (at most
   * 2^20 signatures; a timed launch runs its chunks one after another) --
   * [0] phase 1 (the whole of it when it runs as one kernel, the default;
   * SHA-512 + lattice when split, STL_TUNE_FUSED_PREP 0), [1] the point
   * decompression kernel when split and the key-dedup kernels, [2] main
   * (Straus loop), [3] fallback -- and the number of chunks timed. */
  uint64_t phase_ns[4];
  uint64_t phase_chunks;
  /* host batch chunks and device-resident calls that chose STL_DEDUP_KEYS by
   * themselves (STL_NO_AUTO_DEDUP above); a struct without this field
   * (struct_size = its offset) is accepted */
  uint64_t auto_dedup_chunks;
} stl_stats;
int stl_get_stats(stl_stats *out);
void stl_reset_stats(void);
/* Enables (on != 0) or disables the phase timing of stl_stats for launches
 * made after the call; returns the previous setting.  Off by default: two
 * event records per phase and chunk. */
int stl_set_phase_timing(int on);

/* ---- testing hooks ----
 * Fault injection: after `calls` further HIP/RCCL calls made by libstl the
 * next one reports failure without running (one shot); calls < 0 disarms.
 * Every entry point then returns < 0 (never a reject bitmap) and the batcher
 * delivers the negative code as the verdict. */
void stl_debug_fault_after(long long calls);
/* Verify with a given k = H(R||A||M) mod L (d_k: n*32 bytes) instead of
 * hashing: drives contrived k (the lattice reduction's full-length fallback)
 * next to ordinary lanes in one wave. */
int stl_debug_verify_k_device(const uint8_t *d_sig, const uint8_t *d_k, const uint8_t *d_pk, size_t n,
                              uint64_t *d_bitmap_words, uint32_t flags, void *stream);
/* Execution tuning, process-wide, for A/B experiments and tests: every setting
 * gives the same accept bits.  Returns the previous value, or STL_EINVAL for
 * an unknown key or a value out of range; value -1 only reads the setting.
 * Takes effect for launches made after the call. */
#define STL_TUNE_FUSED_PREP 0 /* 1 (default): phase 1 (SHA-512, lattice, decodings) as one kernel; 0: two */
#define STL_TUNE_MAIN_QUEUE 1 /* 1 (default): the main kernel's waves pull 64-signature units from a
                                 counter; 0: static grid stride */
#define STL_TUNE_STREAMS 2    /* 1..4: a device-resident verify call runs its chunks on this many
                                 concurrent streams (the caller's plus the library's own, forked
                                 and joined by events; not under stl_set_phase_timing) */
#define STL_TUNE_CHUNK_LOG2 3 /* 15..20: log2 of the signatures per chunk when STL_TUNE_STREAMS > 1;
                                 0 (default): round(n / 2^18) equal chunks, at least two */
#define STL_TUNE_BYTE_SHARDS 4 /* 1: host preimage / blob batches take the byte-balanced shard path even
                                  as one shard (test hook: runs the grouped-gather placement and
                                  rank 0's device copy on one GPU under STL_CFG_RCCL_GATHER) */
#define STL_TUNE_QUAD 5        /* lane groups for the smallest chunks' main kernel, bits: 1 = chunks of
                                  at most one wave per SIMD at eight lanes per signature run on lane
                                  quads (each group formula's four products one per lane), 2 = the
                                  next ones up to one wave per SIMD at four lanes on lane duos (two
                                  products per lane); 3 (default) both, 0 lane pairs only */
#define STL_TUNE_STREAM_WORKSPACES 6 /* 1..64 (default 8, env STL_MAX_STREAM_WORKSPACES): caller streams
                                        per device whose context (verify workspace ~0.44 GB, hash
                                        queue, checkSign scratch) libstl keeps; the least recently
                                        used one beyond it is evicted, its buffers kept as a spare
                                        for the next new caller stream (no device synchronisation) */
#define STL_TUNE_LONG_HASH 8        /* 0..62 (default 8; 0 off): in calls of at most two lane-pair chunks
                                        (65,536 rows on 256 CUs), up to 1,024 of the longest preimages
                                        of more than this many SHA-512 blocks are hashed one per wave
                                        (schedules expanded side by side, rounds reading them from
                                        LDS): the longest row sets a small ledger's hash latency */
#define STL_TUNE_SHARED_KEYS 9       /* 0 / 1 (default 1): with STL_DEDUP_KEYS (or the automatic choice) a
                                        device-resident call of several chunks builds ONE key table for
                                        all of them (the first chunk builds it, the others wait for it),
                                        instead of one per chunk */
#define STL_TUNE_WIDE_MIN_ROWS 10     /* 0..2^20 (default 0): a key table of fewer rows (STL_DEDUP_KEYS or the
                                        automatic choice) builds the 9-entry per-key tables only, never
                                        the wide 137-entry ones (whose build a short call waits for) */
#define STL_TUNE_R_AHEAD 11          /* 0 / 1 (default 1): a one-call checkSign with a shared key table
                                        decodes every row's R on its own stream beside the key table's
                                        build, and the chunks' phase 1 then only combines the two */
#define STL_TUNE_FIRST_CHUNK 12      /* 0..2^20, a multiple of 64 (default 0): a device-resident verify over
                                        several streams starts with a chunk of this many rows (smaller
                                        than the others): the launch's first phase 1 has no main
                                        kernel to overlap */
#define STL_TUNE_RCCL_TIMEOUT_MS 7 /* 1..3,600,000 (default 120,000; env STL_RCCL_TIMEOUT_S): deadline of
                                      stl_comm_init_rank and stl_comm_sync */
int stl_debug_tuning(int key, int value);
/* Caller-stream contexts libstl currently keeps on the current device. */
int stl_debug_stream_contexts(void);
/* Measurement only (bench.py clock_ghz): enqueues nwg one-wave workgroups on
 * `stream`; workgroup i writes d_out[4i..4i+3] = {shader cycle counter
 * (s_memtime), 100 MHz counter (s_memrealtime), XCC_ID register, HW_ID
 * register}.  Two stamps around a timed region give its average shader clock
 * per XCD.  STL_EINVAL for a null d_out or nwg > 65,536. */
int stl_debug_clock_stamp(uint64_t *d_out, uint32_t nwg, void *stream);

/* Drops libstl's context of a caller stream on the current device -- its
 * verify workspace, hash queue, checkSign scratch and events -- without
 * waiting for anything: the buffers join the device's spare list (at most
 * STL_TUNE_STREAM_WORKSPACES sets; stl_shutdown frees them), and the next new
 * caller stream adopts a set, its first kernels ordered on the device behind
 * the last kernels that used it.  Call it before destroying a stream the
 * library has run on, or let the per-device cap evict the least recently
 * used context the same way.  A call still running on that stream keeps the
 * context until it returns.  STL_EINVAL for one of libstl's own pool streams;
 * STL_OK if there is none. */
int stl_release_stream(void *stream);

/* Synthetic-data helpers (RippleAddress::sign, RippleAddress.cpp:254-263;
 * EdKeyPair::setSeed, EdKeyPair.cpp:25-33): RFC 8032 keypair from a 32-byte
 * seed and a detached signature over a 32-byte message. */
int stl_ed25519_sign_batch_device(const uint8_t *d_seed, const uint8_t *d_msg, size_t n, uint8_t *d_pk,
                                  uint8_t *d_sig, void *stream);
/* Test data only: the same rows, then row i with d_cls[i] in 1..11 mutated
 * into SURVEY.md Appendix-B class B<cls> with the 32-bit parameter
 * d_param[i] (the construction of tests/datasets.py, stated in
 * stl_kernels.hip adversarial_row: bit flips, S+L, S >= 2^253, small-order
 * keys and R, mixed-order keys re-signed over A+T, non-canonical and off-curve
 * keys, non-canonical R); d_msg_out receives every row's message (d_cls[i] = 0
 * leaves the row honest). */
int stl_debug_sign_adversarial_device(const uint8_t *d_seed, const uint8_t *d_msg, const uint8_t *d_cls,
                                      const uint32_t *d_param, size_t n, uint8_t *d_pk, uint8_t *d_sig,
                                      uint8_t *d_msg_out, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* STL_H */
