/*
 * ref_sodium.c -- the reference's own verify path, restated at the call level
 * and linked against the real dependency it uses.  TEST INFRASTRUCTURE ONLY.
 *
 * stellard compiles this path from RippleAddress.cpp / SerializedTransaction.cpp
 * (which cannot be built here: Boost 1.55 and protobuf are absent, see
 * DESIGN.md), so this harness makes the same two library calls the reference
 * makes, in the same order, with the same composite predicate:
 *
 *   SerializedTransaction::checkSign(pk)      SerializedTransaction.cpp:220-230
 *     hash = SHA512Half(preimage)             Serializer.cpp:354-360  (OpenSSL SHA512)
 *     RippleAddress::verifySignature          RippleAddress.cpp:190-200
 *       crypto_sign_verify_detached(sig, hash, 32, pk) == 0      (libsodium)
 *       && crypto_sign_check_S_lt_l(sig+32) == 0                 RippleAddress.cpp:226-245
 *
 * libsodium: /opt/conda/lib/libsodium.so (1.0.18; the reference pins 1.0.0,
 * Dockerfile:9-10).  OpenSSL: system libcrypto.so.3.
 * Built by oracle/Makefile into oracle/_ref/libsodium_ref.so.
 */
#include <openssl/sha.h>
#include <pthread.h>
#include <sodium.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

static int check_S_lt_l(const unsigned char *S) {
  static const unsigned char l[32] = {0xed, 0xd3, 0xf5, 0x5c, 0x1a, 0x63, 0x12, 0x58, 0xd6, 0x9c, 0xf7,
                                      0xa2, 0xde, 0xf9, 0xde, 0x14, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00,
                                      0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x10};
  unsigned char c = 0, n = 1;
  unsigned int i = 32;
  do {
    i--;
    c |= ((S[i] - l[i]) >> 8) & n;
    n &= ((S[i] ^ l[i]) - 1) >> 8;
  } while (i != 0);
  return -(c == 0);
}

int ref_init(void) { return sodium_init() < 0 ? -1 : 0; }

const char *ref_sodium_version(void) { return sodium_version_string(); }

/* raw libsodium verdict (0 / -1), no stellard wrapper */
int ref_crypto_sign_verify_detached(const unsigned char *sig, const unsigned char *m, unsigned long long mlen,
                                    const unsigned char *pk) {
  return crypto_sign_verify_detached(sig, m, mlen, pk);
}

/* RippleAddress::verifySignature: 1 accept, 0 reject */
int ref_verify_signature(const unsigned char *sig, const unsigned char *hash32, const unsigned char *pk) {
  int verified = crypto_sign_verify_detached(sig, hash32, 32, pk) == 0;
  int canonical = check_S_lt_l(sig + 32) == 0;
  return verified && canonical;
}

void ref_sha512_half(const unsigned char *data, size_t len, unsigned char out[32]) {
  unsigned char j[64];
  SHA512(data, len, j);
  memcpy(out, j, 32);
}

int ref_seed_keypair(unsigned char *pk, unsigned char *sk, const unsigned char *seed) {
  return crypto_sign_seed_keypair(pk, sk, seed);
}

int ref_sign_detached(unsigned char *sig, const unsigned char *m, unsigned long long mlen, const unsigned char *sk) {
  return crypto_sign_detached(sig, NULL, m, mlen, sk);
}

typedef struct {
  const uint8_t *sig, *msg, *pk, *pre;
  const uint64_t *off;
  const uint32_t *len;
  size_t lo, hi;
  uint8_t *bits;
} job_t;

static void *worker(void *arg) {
  job_t *j = (job_t *)arg;
  for (size_t i = j->lo; i < j->hi; ++i) {
    unsigned char hash[32];
    const unsigned char *m = j->msg + 32 * i;
    if (j->pre) {
      ref_sha512_half(j->pre + j->off[i], j->len[i], hash);
      m = hash;
    }
    j->bits[i] = (uint8_t)ref_verify_signature(j->sig + 64 * i, m, j->pk + 32 * i);
  }
  return NULL;
}

static void run(job_t proto, size_t n, uint8_t *bitmap, int threads) {
  if (threads <= 0) threads = (int)sysconf(_SC_NPROCESSORS_ONLN);
  if (threads > 512) threads = 512;
  if ((size_t)threads > n) threads = n ? (int)n : 1;
  uint8_t *bits = (uint8_t *)calloc(n ? n : 1, 1);
  pthread_t tid[512];
  job_t jobs[512];
  size_t chunk = (n + threads - 1) / threads;
  for (int t = 0; t < threads; ++t) {
    jobs[t] = proto;
    jobs[t].lo = (size_t)t * chunk < n ? (size_t)t * chunk : n;
    jobs[t].hi = jobs[t].lo + chunk < n ? jobs[t].lo + chunk : n;
    jobs[t].bits = bits;
    pthread_create(&tid[t], NULL, worker, &jobs[t]);
  }
  for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
  memset(bitmap, 0, (n + 7) / 8);
  for (size_t i = 0; i < n; ++i)
    if (bits[i]) bitmap[i >> 3] |= (uint8_t)(1u << (i & 7));
  free(bits);
}

/* Batch of RippleAddress::verifySignature over SoA buffers. */
void ref_verify_batch(const uint8_t *sig, const uint8_t *msg, const uint8_t *pk, size_t n, uint8_t *bitmap,
                      int threads) {
  job_t p = {sig, msg, pk, NULL, NULL, NULL, 0, 0, NULL};
  run(p, n, bitmap, threads);
}

/* Batch of SerializedTransaction::checkSign over signing preimages. */
void ref_tx_verify_batch(const uint8_t *pre, const uint64_t *off, const uint32_t *len, const uint8_t *sig,
                         const uint8_t *pk, size_t n, uint8_t *bitmap, int threads) {
  job_t p = {sig, NULL, pk, pre, off, len, 0, 0, NULL};
  run(p, n, bitmap, threads);
}

/* Synthetic data for the committed bitmap digests (tests/golden/make_digests.py):
 * keypair from seed_i (crypto_sign_seed_keypair, EdKeyPair::setSeed,
 * EdKeyPair.cpp:25-33) and a detached signature over the 32-byte msg_i
 * (RippleAddress::sign, RippleAddress.cpp:254-263).  RFC 8032 signing is
 * deterministic, so the GPU signer reproduces these bytes on the box. */
typedef struct {
  const uint8_t *seed, *msg;
  uint8_t *pk, *sig;
  size_t lo, hi;
} sign_job_t;

static void *sign_worker(void *arg) {
  sign_job_t *j = (sign_job_t *)arg;
  unsigned char sk[64];
  for (size_t i = j->lo; i < j->hi; ++i) {
    crypto_sign_seed_keypair(j->pk + 32 * i, sk, j->seed + 32 * i);
    crypto_sign_detached(j->sig + 64 * i, NULL, j->msg + 32 * i, 32, sk);
  }
  sodium_memzero(sk, sizeof sk);
  return NULL;
}

void ref_sign_batch(const uint8_t *seed, const uint8_t *msg, size_t n, uint8_t *pk, uint8_t *sig, int threads) {
  if (threads <= 0) threads = (int)sysconf(_SC_NPROCESSORS_ONLN);
  if (threads > 512) threads = 512;
  if ((size_t)threads > n) threads = n ? (int)n : 1;
  pthread_t tid[512];
  sign_job_t jobs[512];
  size_t chunk = (n + threads - 1) / threads;
  for (int t = 0; t < threads; ++t) {
    jobs[t].seed = seed;
    jobs[t].msg = msg;
    jobs[t].pk = pk;
    jobs[t].sig = sig;
    jobs[t].lo = (size_t)t * chunk < n ? (size_t)t * chunk : n;
    jobs[t].hi = jobs[t].lo + chunk < n ? jobs[t].lo + chunk : n;
    pthread_create(&tid[t], NULL, sign_worker, &jobs[t]);
  }
  for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
}

/* Group operations for the adversarial rows of the committed datasets
 * (tests/datasets.py: B6 R = [S]B, B8 A' = A + T). */
int ref_scalarmult_base_noclamp(unsigned char *q, const unsigned char *n) {
  return crypto_scalarmult_ed25519_base_noclamp(q, n);
}

int ref_point_add(unsigned char *r, const unsigned char *p, const unsigned char *q) {
  return crypto_core_ed25519_add(r, p, q);
}
