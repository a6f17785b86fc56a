/*
 * stl_oracle.h -- CPU restatement of stellard's transaction-signature check.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product path (stellard_amd/, the
 * libstl C ABI) may include, link or call this code.  It is used by tests/,
 * by __graft_entry__.smoke() and by bench.py's cpu_baseline leg, and only as
 * the checker.
 *
 * What it restates (reference = /root/reference, libsodium is NOT vendored):
 *   - RippleAddress::verifySignature      src/ripple_data/protocol/RippleAddress.cpp:190-200
 *     = crypto_sign_verify_detached(sig, hash, 32, pk) == 0  &&  S < L
 *   - crypto_sign_check_S_lt_l            RippleAddress.cpp:226-245
 *   - crypto_sign_verify_detached         libsodium 1.0.18 (container copy,
 *     /opt/conda/lib/libsodium.so; the reference pins 1.0.0, Dockerfile:9-10).
 *     Published algorithm (RFC 8032 sec. 5.1.7 + libsodium's pre-checks):
 *       S canonical, R not small order, A canonical, A not small order,
 *       A decompresses, k = SHA-512(R||A||M) mod L,
 *       accept iff encode([k](-A) + [S]B) == R (32-byte compare).
 *   - SHA512Half                          src/ripple_data/protocol/Serializer.cpp:354-360
 *   - STObject::getSigningHash            src/ripple_data/protocol/SerializedObject.cpp:444-450
 *
 * Parity pin: tests/test_oracle_golden.py checks this restatement against the
 * golden vectors in tests/golden/ (expected bits produced by libsodium 1.0.18
 * by tests/golden/make_golden.py) and against the RippleAddress_test KATs
 * (RippleAddress.cpp:812-845).
 */
#ifndef STL_ORACLE_H
#define STL_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Same policy bits as include/stl.h */
#define ORACLE_POLICY_SODIUM_1_0_18 0u
#define ORACLE_POLICY_STELLARD_1_0_0 1u

void oracle_sha512(const uint8_t *in, size_t len, uint8_t out[64]);

/* 0 = accept, -1 = reject.  Composite stellard predicate (verify && S<L). */
int oracle_verify(const uint8_t sig[64], const uint8_t *m, size_t mlen,
                  const uint8_t pk[32], uint32_t policy);

/* Raw libsodium-1.0.18-equivalent verify (no stellard S<L wrapper). */
int oracle_verify_raw(const uint8_t sig[64], const uint8_t *m, size_t mlen,
                      const uint8_t pk[32], uint32_t policy);

/* crypto_sign_check_S_lt_l (RippleAddress.cpp:226-245): 0 if S < L else -1 */
int oracle_check_S_lt_l(const uint8_t S[32]);

/* RFC 8032 key generation / signing (used to build KATs, never to verify). */
void oracle_seed_keypair(uint8_t pk[32], uint8_t sk[64], const uint8_t seed[32]);
void oracle_sign(uint8_t sig[64], const uint8_t *m, size_t mlen, const uint8_t sk[64]);

/* Batch over SoA buffers: sig n*64, msg n*32, pk n*32; bitmap ceil(n/8),
 * bit i = byte i>>3, bit i&7 (LSB first).  Threads: 0 = all online CPUs. */
void oracle_verify_batch(const uint8_t *sig, const uint8_t *msg, const uint8_t *pk,
                         size_t n, uint8_t *bitmap, uint32_t policy, int threads);

/* checkSign over signing preimages (SerializedTransaction.cpp:220-230):
 * msg_i = SHA512Half(preimage_i), then oracle_verify. */
void oracle_tx_verify_batch(const uint8_t *preimages, const uint64_t *offset,
                            const uint32_t *len, const uint8_t *sig, const uint8_t *pk,
                            size_t n, uint8_t *bitmap, uint32_t policy, int threads);

/* ---- serialized transactions (stl_oracle_tx.c) ----
 * The reference's deserialise + re-serialise of one transaction blob
 * (SerializedTransaction(SerializerIterator&), STObject::set/add).
 * Returns 0 when the blob deserialises (and has a TransactionType, no
 * duplicate top-level field), -1 where the reference constructor throws.
 * signing: "STX\0" || add(s, false); full: add(s, true); both up to cap bytes. */
typedef struct oracle_txinfo {
  size_t signing_len, full_len;
  long pk_len, sig_len;      /* top-level SigningPubKey / TxnSignature payload sizes, -1 absent */
  uint8_t pk[64], sig[64];   /* their first bytes */
  int max_depth;             /* deepest nesting level reached (top-level fields = 0) */
  int all_declared;          /* every field code declared in SerializeDeclarations.h */
  int stopped_early;         /* a top-level 0xE1 ended the parse before the blob end */
} oracle_txinfo;
int oracle_tx_blob(const uint8_t *blob, size_t len, uint8_t *signing, uint8_t *full, size_t cap,
                   oracle_txinfo *info);

/* The same for other signed STObjects: kind 0 = transaction (as above),
 * kind 1 = validation ("VAL\0" prefix, signature in sfSignature, no
 * TransactionType, at least 50 bytes: SerializedValidation.cpp:22-34,96-110,
 * PeerImp.cpp:1134). */
int oracle_signed_blob(uint32_t kind, const uint8_t *blob, size_t len, uint8_t *signing, uint8_t *full, size_t cap,
                       oracle_txinfo *info);

/* checkSign over serialized transactions: bit = deserialises && |pk| = 32 &&
 * |sig| = 64 && verify(SHA512Half(signing)).  tx_id (n*32, may be NULL):
 * SHA512Half("TXN\0" || full), zero where the blob does not deserialise. */
void oracle_tx_blob_verify_batch(const uint8_t *blobs, const uint64_t *offset, const uint32_t *len, size_t n,
                                 uint8_t *bitmap, uint8_t *tx_id, uint32_t policy, int threads);
/* kind-generic batch; for kind 1 the id is SHA512Half(raw blob), the
 * suppression key of PeerImp::recvValidation (PeerImp.cpp:1148-1155). */
void oracle_signed_blob_verify_batch(uint32_t kind, const uint8_t *blobs, const uint64_t *offset, const uint32_t *len,
                                     size_t n, uint8_t *bitmap, uint8_t *tx_id, uint32_t policy, int threads);

/* Instrumentation: field multiplications / squarings executed by the last
 * single-threaded oracle_verify call (for the frozen work model). */
void oracle_op_counts(uint64_t *muls, uint64_t *sqs);
int oracle_decode_op_counts(const uint8_t pk[32], uint64_t *muls, uint64_t *sqs);

#ifdef __cplusplus
}
#endif
#endif
