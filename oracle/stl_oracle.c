/*
 * stl_oracle.c -- CPU restatement of the stellard checkSign / libsodium verify
 * path.  TEST INFRASTRUCTURE ONLY (see stl_oracle.h): never linked into the
 * product library.
 *
 * Structure follows the published ref10 Ed25519 algorithm that libsodium's
 * crypto_sign_ed25519_verify_detached uses (libsodium 1.0.18,
 * crypto_sign/ed25519/ref10/open.c + crypto_core/ed25519/ref10/ed25519_ref10.c;
 * not vendored by the reference -- called at RippleAddress.cpp:196-197 and
 * StellarPublicKey.cpp:73-74).  The field is restated in radix 2^51 with
 * unsigned __int128 products (not ref10's 10x25.5 limbs): same values, same
 * operation counts (one fe_mul / fe_sq per ref10 call).
 */
#include "stl_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

typedef unsigned __int128 u128;

/* ------------------------------------------------------------------ */
/* SHA-512 (FIPS 180-4).  Used for SHA512Half (Serializer.cpp:354-360, */
/* OpenSSL SHA512) and for k = H(R||A||M) inside libsodium verify.      */
/* ------------------------------------------------------------------ */
static const uint64_t K512[80] = {
    0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL,
    0x3956c25bf348b538ULL, 0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL,
    0xd807aa98a3030242ULL, 0x12835b0145706fbeULL, 0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL,
    0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL, 0xc19bf174cf692694ULL,
    0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
    0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL,
    0x983e5152ee66dfabULL, 0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL,
    0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL, 0x06ca6351e003826fULL, 0x142929670a0e6e70ULL,
    0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL, 0x53380d139d95b3dfULL,
    0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
    0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL,
    0xd192e819d6ef5218ULL, 0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL,
    0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL, 0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL,
    0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL, 0x682e6ff3d6b2b8a3ULL,
    0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
    0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL,
    0xca273eceea26619cULL, 0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL,
    0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL, 0x113f9804bef90daeULL, 0x1b710b35131c471bULL,
    0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL, 0x431d67c49c100d4cULL,
    0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL};

static inline uint64_t ror64(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

static void sha512_block(uint64_t st[8], const uint8_t *p) {
  uint64_t w[80];
  for (int i = 0; i < 16; ++i) {
    uint64_t v = 0;
    for (int j = 0; j < 8; ++j) v = (v << 8) | p[8 * i + j];
    w[i] = v;
  }
  for (int i = 16; i < 80; ++i) {
    uint64_t s0 = ror64(w[i - 15], 1) ^ ror64(w[i - 15], 8) ^ (w[i - 15] >> 7);
    uint64_t s1 = ror64(w[i - 2], 19) ^ ror64(w[i - 2], 61) ^ (w[i - 2] >> 6);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint64_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
  for (int i = 0; i < 80; ++i) {
    uint64_t S1 = ror64(e, 14) ^ ror64(e, 18) ^ ror64(e, 41);
    uint64_t ch = (e & f) ^ (~e & g);
    uint64_t t1 = h + S1 + ch + K512[i] + w[i];
    uint64_t S0 = ror64(a, 28) ^ ror64(a, 34) ^ ror64(a, 39);
    uint64_t mj = (a & b) ^ (a & c) ^ (b & c);
    uint64_t t2 = S0 + mj;
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  st[0] += a; st[1] += b; st[2] += c; st[3] += d;
  st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

typedef struct {
  uint64_t st[8];
  uint8_t buf[128];
  size_t fill;
  uint64_t total;
} sha512_ctx;

static void sha512_init(sha512_ctx *c) {
  static const uint64_t iv[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                                 0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                                 0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
  memcpy(c->st, iv, sizeof iv);
  c->fill = 0;
  c->total = 0;
}

static void sha512_update(sha512_ctx *c, const uint8_t *p, size_t n) {
  c->total += n;
  while (n) {
    size_t take = 128 - c->fill;
    if (take > n) take = n;
    memcpy(c->buf + c->fill, p, take);
    c->fill += take; p += take; n -= take;
    if (c->fill == 128) { sha512_block(c->st, c->buf); c->fill = 0; }
  }
}

static void sha512_final(sha512_ctx *c, uint8_t out[64]) {
  uint64_t bits = c->total * 8;
  uint8_t pad = 0x80;
  sha512_update(c, &pad, 1);
  uint8_t z = 0;
  while (c->fill != 112) sha512_update(c, &z, 1);
  uint8_t len[16] = {0};
  for (int i = 0; i < 8; ++i) len[15 - i] = (uint8_t)(bits >> (8 * i));
  sha512_update(c, len, 16);
  for (int i = 0; i < 8; ++i)
    for (int j = 0; j < 8; ++j) out[8 * i + j] = (uint8_t)(c->st[i] >> (56 - 8 * j));
}

void oracle_sha512(const uint8_t *in, size_t len, uint8_t out[64]) {
  sha512_ctx c;
  sha512_init(&c);
  sha512_update(&c, in, len);
  sha512_final(&c, out);
}

/* ------------------------------------------------------------------ */
/* GF(2^255-19), radix 2^51.                                           */
/* ------------------------------------------------------------------ */
typedef struct { uint64_t v[5]; } fe;

static __thread uint64_t g_muls, g_sqs;
static uint64_t g_last_muls, g_last_sqs;
#define MASK51 ((1ULL << 51) - 1)

static void fe_0(fe *h) { memset(h, 0, sizeof *h); }
static void fe_1(fe *h) { fe_0(h); h->v[0] = 1; }
static void fe_copy(fe *h, const fe *f) { *h = *f; }

static void fe_carry(fe *h) {
  uint64_t c;
  for (int i = 0; i < 4; ++i) { c = h->v[i] >> 51; h->v[i] &= MASK51; h->v[i + 1] += c; }
  c = h->v[4] >> 51; h->v[4] &= MASK51; h->v[0] += 19 * c;
  c = h->v[0] >> 51; h->v[0] &= MASK51; h->v[1] += c;
}

static void fe_add(fe *h, const fe *f, const fe *g) {
  for (int i = 0; i < 5; ++i) h->v[i] = f->v[i] + g->v[i];
  fe_carry(h);
}

/* f - g + 4p keeps every limb positive for carried inputs (< 2^52). */
static void fe_sub(fe *h, const fe *f, const fe *g) {
  static const uint64_t p4[5] = {0x1FFFFFFFFFFFB4ULL, 0x1FFFFFFFFFFFFCULL, 0x1FFFFFFFFFFFFCULL,
                                 0x1FFFFFFFFFFFFCULL, 0x1FFFFFFFFFFFFCULL};
  for (int i = 0; i < 5; ++i) h->v[i] = f->v[i] + p4[i] - g->v[i];
  fe_carry(h);
}

static void fe_neg(fe *h, const fe *f) { fe z; fe_0(&z); fe_sub(h, &z, f); }

static void fe_mul(fe *h, const fe *f, const fe *g) {
  ++g_muls;
  const uint64_t *a = f->v, *b = g->v;
  u128 t[5];
  uint64_t b19[5];
  for (int i = 0; i < 5; ++i) b19[i] = 19 * b[i];
  t[0] = (u128)a[0] * b[0] + (u128)a[1] * b19[4] + (u128)a[2] * b19[3] + (u128)a[3] * b19[2] + (u128)a[4] * b19[1];
  t[1] = (u128)a[0] * b[1] + (u128)a[1] * b[0] + (u128)a[2] * b19[4] + (u128)a[3] * b19[3] + (u128)a[4] * b19[2];
  t[2] = (u128)a[0] * b[2] + (u128)a[1] * b[1] + (u128)a[2] * b[0] + (u128)a[3] * b19[4] + (u128)a[4] * b19[3];
  t[3] = (u128)a[0] * b[3] + (u128)a[1] * b[2] + (u128)a[2] * b[1] + (u128)a[3] * b[0] + (u128)a[4] * b19[4];
  t[4] = (u128)a[0] * b[4] + (u128)a[1] * b[3] + (u128)a[2] * b[2] + (u128)a[3] * b[1] + (u128)a[4] * b[0];
  uint64_t r[5], c = 0;
  for (int i = 0; i < 5; ++i) {
    t[i] += c;
    r[i] = (uint64_t)t[i] & MASK51;
    c = (uint64_t)(t[i] >> 51);
  }
  r[0] += 19 * c;
  c = r[0] >> 51; r[0] &= MASK51; r[1] += c;
  memcpy(h->v, r, sizeof r);
}

static void fe_sq(fe *h, const fe *f) {
  fe_mul(h, f, f);
  --g_muls;
  ++g_sqs;
}

/* Full reduction to the canonical representative in [0, p). */
static void fe_tobytes(uint8_t s[32], const fe *f) {
  fe h = *f;
  fe_carry(&h);
  fe_carry(&h);
  fe_carry(&h);
  /* now h < 2^255 + small; compute q = 1 iff h >= p */
  uint64_t q = (h.v[0] + 19) >> 51;
  q = (h.v[1] + q) >> 51;
  q = (h.v[2] + q) >> 51;
  q = (h.v[3] + q) >> 51;
  q = (h.v[4] + q) >> 51;
  h.v[0] += 19 * q;
  uint64_t c;
  for (int i = 0; i < 4; ++i) { c = h.v[i] >> 51; h.v[i] &= MASK51; h.v[i + 1] += c; }
  h.v[4] &= MASK51;
  /* pack 255 bits little-endian */
  uint8_t out[32] = {0};
  for (int bit = 0, i = 0; i < 5; ++i, bit += 51) {
    for (int j = 0; j < 51; ++j) {
      int pos = bit + j;
      if (pos >= 256) break;
      if ((h.v[i] >> j) & 1) out[pos >> 3] |= (uint8_t)(1u << (pos & 7));
    }
  }
  memcpy(s, out, 32);
}

/* Load 255 bits (bit 255 ignored, no reduction -- as ref10 fe_frombytes). */
static void fe_frombytes(fe *h, const uint8_t s[32]) {
  fe_0(h);
  for (int pos = 0; pos < 255; ++pos)
    if ((s[pos >> 3] >> (pos & 7)) & 1) h->v[pos / 51] |= 1ULL << (pos % 51);
}

static int fe_iszero(const fe *f) {
  uint8_t s[32];
  fe_tobytes(s, f);
  uint8_t d = 0;
  for (int i = 0; i < 32; ++i) d |= s[i];
  return d == 0;
}

static int fe_isnegative(const fe *f) {
  uint8_t s[32];
  fe_tobytes(s, f);
  return s[0] & 1;
}

/* ref10 addition chains: z^(p-2) and z^((p-5)/8).  254/250 squarings. */
static void fe_sqn(fe *h, const fe *f, int n) {
  fe_sq(h, f);
  for (int i = 1; i < n; ++i) fe_sq(h, h);
}

static void fe_invert(fe *out, const fe *z) {
  fe t0, t1, t2, t3;
  fe_sq(&t0, z);
  fe_sqn(&t1, &t0, 2);
  fe_mul(&t1, z, &t1);
  fe_mul(&t0, &t0, &t1);
  fe_sq(&t2, &t0);
  fe_mul(&t1, &t1, &t2);
  fe_sqn(&t2, &t1, 5);
  fe_mul(&t1, &t2, &t1);
  fe_sqn(&t2, &t1, 10);
  fe_mul(&t2, &t2, &t1);
  fe_sqn(&t3, &t2, 20);
  fe_mul(&t2, &t3, &t2);
  fe_sqn(&t2, &t2, 10);
  fe_mul(&t1, &t2, &t1);
  fe_sqn(&t2, &t1, 50);
  fe_mul(&t2, &t2, &t1);
  fe_sqn(&t3, &t2, 100);
  fe_mul(&t2, &t3, &t2);
  fe_sqn(&t2, &t2, 50);
  fe_mul(&t1, &t2, &t1);
  fe_sqn(&t1, &t1, 5);
  fe_mul(out, &t1, &t0);
}

static void fe_pow22523(fe *out, const fe *z) {
  fe t0, t1, t2;
  fe_sq(&t0, z);
  fe_sqn(&t1, &t0, 2);
  fe_mul(&t1, z, &t1);
  fe_mul(&t0, &t0, &t1);
  fe_sq(&t0, &t0);
  fe_mul(&t0, &t1, &t0);
  fe_sqn(&t1, &t0, 5);
  fe_mul(&t0, &t1, &t0);
  fe_sqn(&t1, &t0, 10);
  fe_mul(&t1, &t1, &t0);
  fe_sqn(&t2, &t1, 20);
  fe_mul(&t1, &t2, &t1);
  fe_sqn(&t1, &t1, 10);
  fe_mul(&t0, &t1, &t0);
  fe_sqn(&t1, &t0, 50);
  fe_mul(&t1, &t1, &t0);
  fe_sqn(&t2, &t1, 100);
  fe_mul(&t1, &t2, &t1);
  fe_sqn(&t1, &t1, 50);
  fe_mul(&t0, &t1, &t0);
  fe_sqn(&t0, &t0, 2);
  fe_mul(out, &t0, z);
}

/* ------------------------------------------------------------------ */
/* Curve constants, derived at first use (no magic limb tables).        */
/* ------------------------------------------------------------------ */
static fe C_d, C_d2, C_sqrtm1;
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static void fe_from_u64(fe *h, uint64_t x) { fe_0(h); h->v[0] = x & MASK51; h->v[1] = x >> 51; }

/* ------------------------------------------------------------------ */
/* Group elements (ref10 representations).                              */
/* ------------------------------------------------------------------ */
typedef struct { fe X, Y, Z; } ge_p2;
typedef struct { fe X, Y, Z, T; } ge_p3;
typedef struct { fe X, Y, Z, T; } ge_p1p1;
typedef struct { fe yplusx, yminusx, xy2d; } ge_precomp;
typedef struct { fe YplusX, YminusX, Z, T2d; } ge_cached;

static void ge_p3_0(ge_p3 *h) { fe_0(&h->X); fe_1(&h->Y); fe_1(&h->Z); fe_0(&h->T); }
static void ge_p2_0(ge_p2 *h) { fe_0(&h->X); fe_1(&h->Y); fe_1(&h->Z); }

static void ge_p1p1_to_p2(ge_p2 *r, const ge_p1p1 *p) {
  fe_mul(&r->X, &p->X, &p->T);
  fe_mul(&r->Y, &p->Y, &p->Z);
  fe_mul(&r->Z, &p->Z, &p->T);
}

static void ge_p1p1_to_p3(ge_p3 *r, const ge_p1p1 *p) {
  fe_mul(&r->X, &p->X, &p->T);
  fe_mul(&r->Y, &p->Y, &p->Z);
  fe_mul(&r->Z, &p->Z, &p->T);
  fe_mul(&r->T, &p->X, &p->Y);
}

static void ge_p3_to_p2(ge_p2 *r, const ge_p3 *p) { r->X = p->X; r->Y = p->Y; r->Z = p->Z; }

static void ge_p3_to_cached(ge_cached *r, const ge_p3 *p) {
  fe_add(&r->YplusX, &p->Y, &p->X);
  fe_sub(&r->YminusX, &p->Y, &p->X);
  fe_copy(&r->Z, &p->Z);
  fe_mul(&r->T2d, &p->T, &C_d2);
}

/* dbl-2008-hwcd for a = -1 */
static void ge_p2_dbl(ge_p1p1 *r, const ge_p2 *p) {
  fe t0;
  fe_sq(&r->X, &p->X);
  fe_sq(&r->Z, &p->Y);
  fe_sq(&r->T, &p->Z);
  fe_add(&r->T, &r->T, &r->T);
  fe_add(&r->Y, &p->X, &p->Y);
  fe_sq(&t0, &r->Y);
  fe_add(&r->Y, &r->Z, &r->X);
  fe_sub(&r->Z, &r->Z, &r->X);
  fe_sub(&r->X, &t0, &r->Y);
  fe_sub(&r->T, &r->T, &r->Z);
}

static void ge_p3_dbl(ge_p1p1 *r, const ge_p3 *p) {
  ge_p2 q;
  ge_p3_to_p2(&q, p);
  ge_p2_dbl(r, &q);
}

/* add-2008-hwcd-3 (unified) */
static void ge_add(ge_p1p1 *r, const ge_p3 *p, const ge_cached *q) {
  fe t0;
  fe_add(&r->X, &p->Y, &p->X);
  fe_sub(&r->Y, &p->Y, &p->X);
  fe_mul(&r->Z, &r->X, &q->YplusX);
  fe_mul(&r->Y, &r->Y, &q->YminusX);
  fe_mul(&r->T, &q->T2d, &p->T);
  fe_mul(&r->X, &p->Z, &q->Z);
  fe_add(&t0, &r->X, &r->X);
  fe_sub(&r->X, &r->Z, &r->Y);
  fe_add(&r->Y, &r->Z, &r->Y);
  fe_add(&r->Z, &t0, &r->T);
  fe_sub(&r->T, &t0, &r->T);
}

static void ge_sub(ge_p1p1 *r, const ge_p3 *p, const ge_cached *q) {
  fe t0;
  fe_add(&r->X, &p->Y, &p->X);
  fe_sub(&r->Y, &p->Y, &p->X);
  fe_mul(&r->Z, &r->X, &q->YminusX);
  fe_mul(&r->Y, &r->Y, &q->YplusX);
  fe_mul(&r->T, &q->T2d, &p->T);
  fe_mul(&r->X, &p->Z, &q->Z);
  fe_add(&t0, &r->X, &r->X);
  fe_sub(&r->X, &r->Z, &r->Y);
  fe_add(&r->Y, &r->Z, &r->Y);
  fe_sub(&r->Z, &t0, &r->T);
  fe_add(&r->T, &t0, &r->T);
}

static void ge_madd(ge_p1p1 *r, const ge_p3 *p, const ge_precomp *q) {
  fe t0;
  fe_add(&r->X, &p->Y, &p->X);
  fe_sub(&r->Y, &p->Y, &p->X);
  fe_mul(&r->Z, &r->X, &q->yplusx);
  fe_mul(&r->Y, &r->Y, &q->yminusx);
  fe_mul(&r->T, &q->xy2d, &p->T);
  fe_add(&t0, &p->Z, &p->Z);
  fe_sub(&r->X, &r->Z, &r->Y);
  fe_add(&r->Y, &r->Z, &r->Y);
  fe_add(&r->Z, &t0, &r->T);
  fe_sub(&r->T, &t0, &r->T);
}

static void ge_msub(ge_p1p1 *r, const ge_p3 *p, const ge_precomp *q) {
  fe t0;
  fe_add(&r->X, &p->Y, &p->X);
  fe_sub(&r->Y, &p->Y, &p->X);
  fe_mul(&r->Z, &r->X, &q->yminusx);
  fe_mul(&r->Y, &r->Y, &q->yplusx);
  fe_mul(&r->T, &q->xy2d, &p->T);
  fe_add(&t0, &p->Z, &p->Z);
  fe_sub(&r->X, &r->Z, &r->Y);
  fe_add(&r->Y, &r->Z, &r->Y);
  fe_sub(&r->Z, &t0, &r->T);
  fe_add(&r->T, &t0, &r->T);
}

static void ge_tobytes(uint8_t s[32], const ge_p2 *h) {
  fe recip, x, y;
  fe_invert(&recip, &h->Z);
  fe_mul(&x, &h->X, &recip);
  fe_mul(&y, &h->Y, &recip);
  fe_tobytes(s, &y);
  s[31] ^= (uint8_t)(fe_isnegative(&x) << 7);
}

static void ge_p3_tobytes(uint8_t s[32], const ge_p3 *h) {
  ge_p2 q;
  ge_p3_to_p2(&q, h);
  ge_tobytes(s, &q);
}

/* ge25519_frombytes_negate_vartime: decodes -A.  Returns -1 when y^2-1 over
 * d*y^2+1 is not a square.  Note: x == 0 with the sign bit set is NOT
 * rejected (libsodium 1.0.18 behaviour); such points are small order and are
 * caught by the blocklist under the 1.0.18 policy. */
static int ge_frombytes_negate_vartime(ge_p3 *h, const uint8_t s[32]) {
  fe u, v, v3, vxx, check;
  fe_frombytes(&h->Y, s);
  fe_1(&h->Z);
  fe_sq(&u, &h->Y);
  fe_mul(&v, &u, &C_d);
  fe_sub(&u, &u, &h->Z);
  fe_add(&v, &v, &h->Z);
  fe_sq(&v3, &v);
  fe_mul(&v3, &v3, &v);
  fe_sq(&h->X, &v3);
  fe_mul(&h->X, &h->X, &v);
  fe_mul(&h->X, &h->X, &u);
  fe_pow22523(&h->X, &h->X);
  fe_mul(&h->X, &h->X, &v3);
  fe_mul(&h->X, &h->X, &u);
  fe_sq(&vxx, &h->X);
  fe_mul(&vxx, &vxx, &v);
  fe_sub(&check, &vxx, &u);
  if (!fe_iszero(&check)) {
    fe_add(&check, &vxx, &u);
    if (!fe_iszero(&check)) return -1;
    fe_mul(&h->X, &h->X, &C_sqrtm1);
  }
  if (fe_isnegative(&h->X) == (s[31] >> 7)) fe_neg(&h->X, &h->X);
  fe_mul(&h->T, &h->X, &h->Y);
  return 0;
}

/* ------------------------------------------------------------------ */
/* Scalars mod L = 2^252 + 27742317777372353535851937790883648493.      */
/* Restated as plain long division on 64-bit words (ref10 uses a        */
/* 21-bit-limb Barrett-like reduction; the value is the same).          */
/* ------------------------------------------------------------------ */
static const uint64_t L64[4] = {0x5812631a5cf5d3edULL, 0x14def9dea2f79cd6ULL, 0x0ULL, 0x1000000000000000ULL};

/* x (nw words, little endian) mod L -> 32 bytes */
static void sc_mod(uint8_t out[32], const uint64_t *x, int nw) {
  uint64_t r[5] = {0, 0, 0, 0, 0};  /* remainder < 2L < 2^254, 5th word for shifting */
  for (int bit = nw * 64 - 1; bit >= 0; --bit) {
    /* r = 2r + bit */
    uint64_t c = (x[bit >> 6] >> (bit & 63)) & 1;
    for (int i = 0; i < 5; ++i) {
      uint64_t nc = r[i] >> 63;
      r[i] = (r[i] << 1) | c;
      c = nc;
    }
    /* if r >= L: r -= L */
    int ge = 0;
    if (r[4]) ge = 1;
    else {
      ge = 1;
      for (int i = 3; i >= 0; --i) {
        if (r[i] != L64[i]) { ge = r[i] > L64[i]; break; }
      }
    }
    if (ge) {
      uint64_t borrow = 0;
      for (int i = 0; i < 4; ++i) {
        u128 d = (u128)r[i] - L64[i] - borrow;
        r[i] = (uint64_t)d;
        borrow = (uint64_t)(d >> 64) & 1;
      }
      r[4] -= borrow;
    }
  }
  for (int i = 0; i < 32; ++i) out[i] = (uint8_t)(r[i >> 3] >> (8 * (i & 7)));
}

static void load_words(uint64_t *w, const uint8_t *b, int nbytes) {
  for (int i = 0; i < nbytes / 8; ++i) {
    uint64_t v = 0;
    for (int j = 7; j >= 0; --j) v = (v << 8) | b[8 * i + j];
    w[i] = v;
  }
}

static void sc_reduce64(uint8_t out[32], const uint8_t h[64]) {
  uint64_t w[8];
  load_words(w, h, 64);
  sc_mod(out, w, 8);
}

/* (a*b + c) mod L */
static void sc_muladd(uint8_t s[32], const uint8_t a[32], const uint8_t b[32], const uint8_t c[32]) {
  uint64_t A[4], B[4], C[4], P[9] = {0};
  load_words(A, a, 32); load_words(B, b, 32); load_words(C, c, 32);
  for (int i = 0; i < 4; ++i) {
    uint64_t carry = 0;
    for (int j = 0; j < 4; ++j) {
      u128 t = (u128)A[i] * B[j] + P[i + j] + carry;
      P[i + j] = (uint64_t)t;
      carry = (uint64_t)(t >> 64);
    }
    P[i + 4] += carry;
  }
  uint64_t carry = 0;
  for (int i = 0; i < 9; ++i) {
    u128 t = (u128)P[i] + (i < 4 ? C[i] : 0) + carry;
    P[i] = (uint64_t)t;
    carry = (uint64_t)(t >> 64);
  }
  sc_mod(s, P, 9);
}

int oracle_check_S_lt_l(const uint8_t S[32]) {
  /* constant-time compare, as RippleAddress.cpp:226-245 */
  static const uint8_t l[32] = {0xed, 0xd3, 0xf5, 0x5c, 0x1a, 0x63, 0x12, 0x58, 0xd6, 0x9c, 0xf7,
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

/* ------------------------------------------------------------------ */
/* Base point odd multiples and the double-scalar multiplication        */
/* (ge25519_double_scalarmult_vartime: sliding windows, w = 5).          */
/* ------------------------------------------------------------------ */
static ge_precomp Bi[8]; /* B, 3B, ..., 15B  (affine Niels) */
static ge_p3 G_B;

static void slide(signed char r[256], const uint8_t a[32]) {
  for (int i = 0; i < 256; ++i) r[i] = 1 & (a[i >> 3] >> (i & 7));
  for (int i = 0; i < 256; ++i) {
    if (!r[i]) continue;
    for (int b = 1; b <= 6 && i + b < 256; ++b) {
      if (!r[i + b]) continue;
      if (r[i] + (r[i + b] << b) <= 15) {
        r[i] += (signed char)(r[i + b] << b);
        r[i + b] = 0;
      } else if (r[i] - (r[i + b] << b) >= -15) {
        r[i] -= (signed char)(r[i + b] << b);
        for (int k = i + b; k < 256; ++k) {
          if (!r[k]) { r[k] = 1; break; }
          r[k] = 0;
        }
      } else {
        break;
      }
    }
  }
}

/* r = a*A + b*B */
static void ge_double_scalarmult_vartime(ge_p2 *r, const uint8_t a[32], const ge_p3 *A, const uint8_t b[32]) {
  signed char aslide[256], bslide[256];
  ge_cached Ai[8];
  ge_p1p1 t;
  ge_p3 u, A2;
  slide(aslide, a);
  slide(bslide, b);
  ge_p3_to_cached(&Ai[0], A);
  ge_p3_dbl(&t, A);
  ge_p1p1_to_p3(&A2, &t);
  for (int i = 0; i < 7; ++i) {
    ge_add(&t, &A2, &Ai[i]);
    ge_p1p1_to_p3(&u, &t);
    ge_p3_to_cached(&Ai[i + 1], &u);
  }
  ge_p2_0(r);
  int i;
  for (i = 255; i >= 0; --i)
    if (aslide[i] || bslide[i]) break;
  for (; i >= 0; --i) {
    ge_p2_dbl(&t, r);
    if (aslide[i] > 0) { ge_p1p1_to_p3(&u, &t); ge_add(&t, &u, &Ai[aslide[i] / 2]); }
    else if (aslide[i] < 0) { ge_p1p1_to_p3(&u, &t); ge_sub(&t, &u, &Ai[(-aslide[i]) / 2]); }
    if (bslide[i] > 0) { ge_p1p1_to_p3(&u, &t); ge_madd(&t, &u, &Bi[bslide[i] / 2]); }
    else if (bslide[i] < 0) { ge_p1p1_to_p3(&u, &t); ge_msub(&t, &u, &Bi[(-bslide[i]) / 2]); }
    ge_p1p1_to_p2(r, &t);
  }
}

/* Plain double-and-add scalar multiplication (keygen / signing only). */
static void ge_scalarmult(ge_p3 *r, const uint8_t a[32], const ge_p3 *P) {
  ge_cached pc;
  ge_p1p1 t;
  ge_p3_to_cached(&pc, P);
  ge_p3_0(r);
  for (int i = 255; i >= 0; --i) {
    ge_p3_dbl(&t, r);
    ge_p1p1_to_p3(r, &t);
    if ((a[i >> 3] >> (i & 7)) & 1) {
      ge_add(&t, r, &pc);
      ge_p1p1_to_p3(r, &t);
    }
  }
}

static void init_constants(void) {
  fe num, den, inv, t;
  /* d = -121665/121666 */
  fe_from_u64(&num, 121665);
  fe_neg(&num, &num);
  fe_from_u64(&den, 121666);
  fe_invert(&inv, &den);
  fe_mul(&C_d, &num, &inv);
  fe_add(&C_d2, &C_d, &C_d);
  /* sqrt(-1) = 2^((p-1)/4): exponent bytes of (p-1)/4 = 2^253 - 5 */
  uint8_t e[32];
  memset(e, 0xff, 32);
  e[0] = 0xfb;
  e[31] = 0x1f;
  fe two, acc;
  fe_from_u64(&two, 2);
  fe_1(&acc);
  for (int i = 255; i >= 0; --i) {
    fe_sq(&acc, &acc);
    if ((e[i >> 3] >> (i & 7)) & 1) fe_mul(&acc, &acc, &two);
  }
  C_sqrtm1 = acc;
  /* B: y = 4/5, x even  -> encoding 0x58 0x66.. 0x66 ; decode gives -B */
  uint8_t benc[32];
  memset(benc, 0x66, 32);
  benc[0] = 0x58;
  ge_p3 negB;
  ge_frombytes_negate_vartime(&negB, benc);
  G_B = negB;
  fe_neg(&G_B.X, &negB.X);
  fe_neg(&G_B.T, &negB.T);
  /* Bi[i] = (2i+1)B in affine Niels form */
  ge_p3 cur = G_B, B2;
  ge_p1p1 p;
  ge_cached cb;
  ge_p3_dbl(&p, &G_B);
  ge_p1p1_to_p3(&B2, &p);
  ge_p3_to_cached(&cb, &B2);
  for (int i = 0; i < 8; ++i) {
    fe zi, x, y;
    fe_invert(&zi, &cur.Z);
    fe_mul(&x, &cur.X, &zi);
    fe_mul(&y, &cur.Y, &zi);
    fe_add(&Bi[i].yplusx, &y, &x);
    fe_sub(&Bi[i].yminusx, &y, &x);
    fe_mul(&t, &x, &y);
    fe_mul(&Bi[i].xy2d, &t, &C_d2);
    ge_add(&p, &cur, &cb);
    ge_p1p1_to_p3(&cur, &p);
  }
  g_muls = g_sqs = 0;
}

static void ensure_init(void) { pthread_once(&g_once, init_constants); }

/* ------------------------------------------------------------------ */
/* libsodium 1.0.18 pre-checks                                          */
/* ------------------------------------------------------------------ */
static int sc_is_canonical(const uint8_t s[32]) { return oracle_check_S_lt_l(s) == 0; }

static int has_small_order(const uint8_t s[32]) {
  static const uint8_t bl[7][32] = {
      {0},
      {0x01},
      {0x26, 0xe8, 0x95, 0x8f, 0xc2, 0xb2, 0x27, 0xb0, 0x45, 0xc3, 0xf4, 0x89, 0xf2, 0xef, 0x98, 0xf0,
       0xd5, 0xdf, 0xac, 0x05, 0xd3, 0xc6, 0x33, 0x39, 0xb1, 0x38, 0x02, 0x88, 0x6d, 0x53, 0xfc, 0x05},
      {0xc7, 0x17, 0x6a, 0x70, 0x3d, 0x4d, 0xd8, 0x4f, 0xba, 0x3c, 0x0b, 0x76, 0x0d, 0x10, 0x67, 0x0f,
       0x2a, 0x20, 0x53, 0xfa, 0x2c, 0x39, 0xcc, 0xc6, 0x4e, 0xc7, 0xfd, 0x77, 0x92, 0xac, 0x03, 0x7a},
      {0xec, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff,
       0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0x7f},
      {0xed, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff,
       0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0x7f},
      {0xee, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff,
       0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0x7f}};
  for (int k = 0; k < 7; ++k) {
    int eq = 1;
    for (int j = 0; j < 31 && eq; ++j) eq = s[j] == bl[k][j];
    if (eq && (s[31] & 0x7f) == bl[k][31]) return 1;
  }
  return 0;
}

static int ge_is_canonical(const uint8_t s[32]) {
  /* non-canonical iff the 255-bit y is in [p, 2^255) */
  if ((s[31] & 0x7f) != 0x7f) return 1;
  for (int i = 30; i > 0; --i)
    if (s[i] != 0xff) return 1;
  return s[0] < 0xed;
}

int oracle_verify_raw(const uint8_t sig[64], const uint8_t *m, size_t mlen, const uint8_t pk[32],
                      uint32_t policy) {
  ensure_init();
  ge_p3 A;
  ge_p2 R;
  uint8_t h[64], k[32], rcheck[32];
  if (policy == ORACLE_POLICY_STELLARD_1_0_0) {
    if (sig[63] & 224) return -1;
    /* the all-zero key (order 4) is rejected, as some 1.0.x releases did;
     * unpinned offline, conservative (stl.h) */
    int nz = 0;
    for (int i = 0; i < 32; ++i) nz |= pk[i];
    if (!nz) return -1;
  } else {
    if (!sc_is_canonical(sig + 32) || has_small_order(sig)) return -1;
    if (!ge_is_canonical(pk) || has_small_order(pk)) return -1;
  }
  if (ge_frombytes_negate_vartime(&A, pk) != 0) return -1;
  sha512_ctx c;
  sha512_init(&c);
  sha512_update(&c, sig, 32);
  sha512_update(&c, pk, 32);
  sha512_update(&c, m, mlen);
  sha512_final(&c, h);
  sc_reduce64(k, h);
  ge_double_scalarmult_vartime(&R, k, &A, sig + 32);
  ge_tobytes(rcheck, &R);
  return memcmp(rcheck, sig, 32) == 0 ? 0 : -1;
}

int oracle_verify(const uint8_t sig[64], const uint8_t *m, size_t mlen, const uint8_t pk[32], uint32_t policy) {
  g_muls = g_sqs = 0;
  /* RippleAddress::verifySignature: verified && signatureIsCanonical */
  int v = oracle_verify_raw(sig, m, mlen, pk, policy) == 0;
  int canon = oracle_check_S_lt_l(sig + 32) == 0;
  g_last_muls = g_muls;
  g_last_sqs = g_sqs;
  return (v && canon) ? 0 : -1;
}

/* Field operations of one ge_frombytes_negate_vartime (bench.py DECODE_OPS:
 * the work model's per-kernel split).  Returns the decoder's result. */
int oracle_decode_op_counts(const uint8_t pk[32], uint64_t *muls, uint64_t *sqs) {
  ensure_init();
  ge_p3 A;
  g_muls = g_sqs = 0;
  const int rc = ge_frombytes_negate_vartime(&A, pk);
  *muls = g_muls;
  *sqs = g_sqs;
  return rc;
}

void oracle_op_counts(uint64_t *muls, uint64_t *sqs) {
  *muls = g_last_muls;
  *sqs = g_last_sqs;
}

void oracle_seed_keypair(uint8_t pk[32], uint8_t sk[64], const uint8_t seed[32]) {
  ensure_init();
  uint8_t h[64];
  oracle_sha512(seed, 32, h);
  h[0] &= 248; h[31] &= 127; h[31] |= 64;
  ge_p3 A;
  ge_scalarmult(&A, h, &G_B);
  ge_p3_tobytes(pk, &A);
  memcpy(sk, seed, 32);
  memcpy(sk + 32, pk, 32);
}

void oracle_sign(uint8_t sig[64], const uint8_t *m, size_t mlen, const uint8_t sk[64]) {
  ensure_init();
  uint8_t az[64], nonce[64], r[32], hram[64], k[32];
  static const uint8_t zero[32] = {0};
  oracle_sha512(sk, 32, az);
  az[0] &= 248; az[31] &= 127; az[31] |= 64;
  sha512_ctx c;
  sha512_init(&c);
  sha512_update(&c, az + 32, 32);
  sha512_update(&c, m, mlen);
  sha512_final(&c, nonce);
  sc_reduce64(r, nonce);
  ge_p3 R;
  ge_scalarmult(&R, r, &G_B);
  ge_p3_tobytes(sig, &R);
  sha512_init(&c);
  sha512_update(&c, sig, 32);
  sha512_update(&c, sk + 32, 32);
  sha512_update(&c, m, mlen);
  sha512_final(&c, hram);
  sc_reduce64(k, hram);
  uint8_t a[32];
  memcpy(a, az, 32);
  /* the clamped scalar is < 2^255; sc_muladd reduces everything mod L */
  sc_muladd(sig + 32, k, a, r);
  (void)zero;
}

/* ------------------------------------------------------------------ */
/* Threaded batch drivers (host-core baseline / test checker).          */
/* ------------------------------------------------------------------ */
typedef struct {
  const uint8_t *sig, *msg, *pk, *pre;
  const uint64_t *off;
  const uint32_t *len;
  size_t lo, hi;
  uint8_t *bits; /* one byte per item, folded into the bitmap afterwards */
  uint32_t policy;
} job_t;

static void *verify_worker(void *arg) {
  job_t *j = (job_t *)arg;
  for (size_t i = j->lo; i < j->hi; ++i) {
    uint8_t hash[64];
    const uint8_t *m;
    if (j->pre) {
      oracle_sha512(j->pre + j->off[i], j->len[i], hash); /* SHA512Half */
      m = hash;
    } else {
      m = j->msg + 32 * i;
    }
    j->bits[i] = oracle_verify(j->sig + 64 * i, m, 32, j->pk + 32 * i, j->policy) == 0;
  }
  return NULL;
}

static void run_batch(job_t proto, size_t n, uint8_t *bitmap, int threads) {
  ensure_init();
  if (threads <= 0) threads = (int)sysconf(_SC_NPROCESSORS_ONLN);
  if (threads < 1) threads = 1;
  if ((size_t)threads > n) threads = n ? (int)n : 1;
  uint8_t *bits = (uint8_t *)calloc(n ? n : 1, 1);
  pthread_t tid[512];
  job_t jobs[512];
  if (threads > 512) threads = 512;
  size_t chunk = (n + threads - 1) / threads;
  for (int t = 0; t < threads; ++t) {
    jobs[t] = proto;
    jobs[t].lo = (size_t)t * chunk < n ? (size_t)t * chunk : n;
    jobs[t].hi = jobs[t].lo + chunk < n ? jobs[t].lo + chunk : n;
    jobs[t].bits = bits;
    pthread_create(&tid[t], NULL, verify_worker, &jobs[t]);
  }
  for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
  memset(bitmap, 0, (n + 7) / 8);
  for (size_t i = 0; i < n; ++i)
    if (bits[i]) bitmap[i >> 3] |= (uint8_t)(1u << (i & 7));
  free(bits);
}

void oracle_verify_batch(const uint8_t *sig, const uint8_t *msg, const uint8_t *pk, size_t n, uint8_t *bitmap,
                         uint32_t policy, int threads) {
  job_t p = {sig, msg, pk, NULL, NULL, NULL, 0, 0, NULL, policy};
  run_batch(p, n, bitmap, threads);
}

void oracle_tx_verify_batch(const uint8_t *preimages, const uint64_t *offset, const uint32_t *len,
                            const uint8_t *sig, const uint8_t *pk, size_t n, uint8_t *bitmap, uint32_t policy,
                            int threads) {
  job_t p = {sig, NULL, pk, preimages, offset, len, 0, 0, NULL, policy};
  run_batch(p, n, bitmap, threads);
}
