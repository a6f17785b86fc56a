// stl_sign.h -- RFC 8032 signing and the adversarial rows of the full-size
// parity datasets.  SYNTHETIC DATA ONLY: the bench's signatures and the
// tests' regenerated datasets come from here; nothing on the verify path
// calls it.  STL_HD so the host test harness (tests/native/hostemu.cpp) runs
// the same code the GPU's sign kernel runs.
//
//   sign_row          keypair from a 32-byte seed (EdKeyPair::setSeed,
//                     EdKeyPair.cpp:25-33) and a detached signature over a
//                     32-byte message (RippleAddress::sign, RippleAddress.cpp:254-263)
//   adversarial_row   SURVEY.md Appendix-B class B1..B11 built from a row's
//                     own honest signature (tests/datasets.py states the same
//                     construction over libsodium; the committed input digests
//                     pin the two against each other)
//
// Every table lookup and runtime-indexed word below is an unrolled select, so
// the row stays in registers (no private-memory arrays, no constant-memory
// pointers).
#pragma once
#include "stl_verify_core.h"

namespace stl {

// SHA-512 of a short word-aligned input (nwords even, nwords*4 <= 108 bytes).
STL_HD void sha512_short(uint32_t out[16], const uint32_t* in, int nwords) {
  uint64_t st[8], w[16];
  sha512_init(st);
#pragma unroll
  for (int j = 0; j < 16; ++j) w[j] = 0;
  for (int j = 0; j < nwords / 2; ++j) w[j] = be64_from_le32(in[2 * j], in[2 * j + 1]);
  w[nwords / 2] = 0x8000000000000000ULL;
  w[15] = (uint64_t)nwords * 32;
  sha512_compress(st, w);
  sha512_digest_le32(out, st);
}

// Honest row: A = [a]B, R = [r]B, S = r + k*a mod L; also returns the clamped
// secret scalar a (not reduced) and the nonce r.
STL_HD void sign_row(uint32_t A[8], uint32_t R[8], uint32_t S[8], uint32_t a[8], uint32_t r[8], const uint32_t sd[8],
                     const uint32_t M[8], const TableView& tv, const uint32_t* btab) {
  uint32_t h[16];
  sha512_short(h, sd, 8);
#pragma unroll
  for (int q = 0; q < 8; ++q) a[q] = h[q];
  a[0] &= 0xfffffff8u;                         // clamp: h[0] &= 248
  a[7] = (a[7] & 0x7fffffffu) | 0x40000000u;   // h[31] &= 127; h[31] |= 64
  uint32_t x[16], a_red[8], zero[8], pre[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) x[q] = q < 8 ? a[q] : 0u;
  sc_reduce64(a_red, x);
#pragma unroll
  for (int q = 0; q < 8; ++q) zero[q] = 0;
  ge_p3 id;
  ge_p3_0(id);
  ge_p2 P;
  double_scalarmult(P, id, zero, a_red, tv, btab);  // A = [a]B
  ge_tobytes(A, P);
  // r = SHA-512(h[32..63] || M) mod L
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    pre[q] = h[8 + q];
    pre[8 + q] = M[q];
  }
  uint32_t rh[16];
  sha512_short(rh, pre, 16);
  sc_reduce64(r, rh);
  double_scalarmult(P, id, zero, r, tv, btab);  // R = [r]B
  ge_tobytes(R, P);
  uint32_t kh[16], k[8];
  sha512_hram32(kh, R, A, M);
  sc_reduce64(k, kh);
  sc_muladd(S, k, a, r);  // S = r + k a mod L
}

// The 14 encodings of points of order dividing 8 (both sign bits; y = p and
// p + 1), sorted as tests/datasets.py SMALL_ORDER sorts them.
STL_HD void adv_small_order(uint32_t out[8], uint32_t idx) {
  const uint32_t t[14][8] = {
      {0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u},
      {0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x80000000u},
      {0x00000001u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u},
      {0x00000001u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x80000000u},
      {0x8f95e826u, 0xb027b2c2u, 0x89f4c345u, 0xf098eff2u, 0x05acdfd5u, 0x3933c6d3u, 0x880238b1u, 0x05fc536du},
      {0x8f95e826u, 0xb027b2c2u, 0x89f4c345u, 0xf098eff2u, 0x05acdfd5u, 0x3933c6d3u, 0x880238b1u, 0x85fc536du},
      {0x706a17c7u, 0x4fd84d3du, 0x760b3cbau, 0x0f67100du, 0xfa53202au, 0xc6cc392cu, 0x77fdc74eu, 0x7a03ac92u},
      {0x706a17c7u, 0x4fd84d3du, 0x760b3cbau, 0x0f67100du, 0xfa53202au, 0xc6cc392cu, 0x77fdc74eu, 0xfa03ac92u},
      {0xffffffecu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0x7fffffffu},
      {0xffffffecu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu},
      {0xffffffedu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0x7fffffffu},
      {0xffffffedu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu},
      {0xffffffeeu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0x7fffffffu},
      {0xffffffeeu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu}};
#pragma unroll
  for (uint32_t e = 0; e < 14; ++e)
#pragma unroll
    for (int i = 0; i < 8; ++i) out[i] = e == idx ? t[e][i] : out[i];
}

// i * T8 for i = 1..7 (T8 = the order-8 point encoded 26e8...05), as
// tests/datasets.py TORSION[1..7]
STL_HD void adv_torsion(uint32_t out[8], uint32_t i) {
  const uint32_t t[7][8] = {
      {0x8f95e826u, 0xb027b2c2u, 0x89f4c345u, 0xf098eff2u, 0x05acdfd5u, 0x3933c6d3u, 0x880238b1u, 0x05fc536du},
      {0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u},
      {0x706a17c7u, 0x4fd84d3du, 0x760b3cbau, 0x0f67100du, 0xfa53202au, 0xc6cc392cu, 0x77fdc74eu, 0x7a03ac92u},
      {0xffffffecu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0x7fffffffu},
      {0x706a17c7u, 0x4fd84d3du, 0x760b3cbau, 0x0f67100du, 0xfa53202au, 0xc6cc392cu, 0x77fdc74eu, 0xfa03ac92u},
      {0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x80000000u},
      {0x8f95e826u, 0xb027b2c2u, 0x89f4c345u, 0xf098eff2u, 0x05acdfd5u, 0x3933c6d3u, 0x880238b1u, 0x85fc536du}};
#pragma unroll
  for (uint32_t e = 0; e < 7; ++e)
#pragma unroll
    for (int k = 0; k < 8; ++k) out[k] = e + 1 == i ? t[e][k] : out[k];
}

// Non-canonical encodings of the identity: y = p + 1; y = 1 with the sign
// bit; y = p + 1 with the sign bit (tests/datasets.py NONCANON_R).
STL_HD void adv_noncanon_r(uint32_t out[8], uint32_t idx) {
  out[0] = idx == 1 ? 0x00000001u : 0xffffffeeu;
#pragma unroll
  for (int i = 1; i < 7; ++i) out[i] = idx == 1 ? 0u : 0xffffffffu;
  out[7] = idx == 0 ? 0x7fffffffu : (idx == 1 ? 0x80000000u : 0xffffffffu);
}

// w[idx >> 2] ^= v << 8*(idx & 3): flip bits of byte `idx` of a 32-byte row
STL_HD void adv_xor_byte(uint32_t w[8], uint32_t idx, uint32_t v) {
#pragma unroll
  for (uint32_t i = 0; i < 8; ++i) w[i] ^= i == (idx >> 2) ? v << (8 * (idx & 3u)) : 0u;
}

// x (8 words) += y, mod 2^256
STL_HD void adv_add256(uint32_t x[8], const uint32_t y[8]) {
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    c += (uint64_t)x[i] + y[i];
    x[i] = (uint32_t)c;
    c >>= 32;
  }
}

STL_HD int adv_clz32(uint32_t v) {
  int n = 0;
#pragma unroll
  for (int b = 31; b >= 0; --b) {
    if ((v >> b) & 1u) break;
    ++n;
  }
  return n;
}

// Clears the highest set bit of S among bits [0, 252) masked by `mask`;
// returns false if there is none.
STL_HD bool adv_clear_top(uint32_t S[8], const uint32_t mask[8]) {
  int hw = -1;
  uint32_t hv = 0;
#pragma unroll
  for (int w = 0; w < 8; ++w) {
    const uint32_t v = S[w] & mask[w];
    if (v != 0) {
      hw = w;
      hv = v;
    }
  }
  if (hw < 0) return false;
  const uint32_t top = 1u << (31 - adv_clz32(hv));
#pragma unroll
  for (int w = 0; w < 8; ++w) S[w] &= w == hw ? ~top : 0xffffffffu;
  return true;
}

// Mutates one honest row (A, R, S, M; a the clamped secret scalar, r the
// nonce) into Appendix-B class c with the 32-bit parameter u:
//   1 B1   msg byte u%32 ^= 1 << ((u>>5)&7)
//   2 B2   R   byte u%32 ^= 1 << ((u>>5)&7)
//   3 B3   clear the first set bit of S at or below bit u%252, scanning down
//          (wrapping from 0 to 251): S stays < L
//   4 B4   S += L
//   5 B5   sig[63] |= {0xE0, 0x80, 0x40, 0x20}[u%4] (S >= 2^253)
//   6 B6   pk = small-order encoding u%14, R = encode([S]B)
//   7 B7   R = small-order encoding u%14, S = k*a mod L, k = H(R||A||M) mod L
//   8 B8   pk = A' = A + (1 + u%7)*T8, S = r + k*a, k = H(R||A'||M)
//   9 B9   pk = p + 2 + u%17 (non-canonical y), sign bit (u>>8)&1
//  10 B10  pk = y + j | sign, the first j in 1..64 with y + j < p not on the curve
//  11 B11  u even: R's sign bit flipped; u odd: R = non-canonical identity
//          (u>>1)%3, S = k*a
STL_HD void adversarial_row(uint32_t c, uint32_t u, uint32_t A[8], uint32_t R[8], uint32_t S[8], uint32_t M[8],
                            const uint32_t a[8], const uint32_t r[8], const TableView& tv, const uint32_t* btab) {
  const uint32_t byte = u % 32u, bit = 1u << ((u >> 5) & 7u);
  uint32_t zero[8], k[8], h[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) zero[i] = 0;
  if (c == 1) {
    adv_xor_byte(M, byte, bit);
  } else if (c == 2) {
    adv_xor_byte(R, byte, bit);
  } else if (c == 3) {
    const uint32_t b0 = u % 252u;
    uint32_t le[8], all[8];  // bits [0, b0] and [0, 252)
#pragma unroll
    for (uint32_t w = 0; w < 8; ++w) {
      const uint32_t lo = 32 * w;
      le[w] = b0 >= lo + 31 ? 0xffffffffu : (b0 < lo ? 0u : (0xffffffffu >> (31 - (b0 - lo))));
      all[w] = w == 7 ? 0x0fffffffu : 0xffffffffu;
    }
    if (!adv_clear_top(S, le)) adv_clear_top(S, all);
  } else if (c == 4) {
    uint32_t Lw[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) Lw[i] = sc_L(i);
    adv_add256(S, Lw);
  } else if (c == 5) {
    const uint32_t m = u % 4u;
    S[7] |= (m == 0 ? 0xE0u : (m == 1 ? 0x80u : (m == 2 ? 0x40u : 0x20u))) << 24;
  } else if (c == 6) {
    adv_small_order(A, u % 14u);
    ge_p3 id;
    ge_p3_0(id);
    ge_p2 P;
    double_scalarmult(P, id, zero, S, tv, btab);  // [S]B
    ge_tobytes(R, P);
  } else if (c == 7 || c == 11) {
    if (c == 11 && (u & 1u) == 0) {
      R[7] ^= 0x80000000u;
    } else {
      if (c == 7)
        adv_small_order(R, u % 14u);
      else
        adv_noncanon_r(R, (u >> 1) % 3u);
      sha512_hram32(h, R, A, M);
      sc_reduce64(k, h);
      sc_muladd(S, k, a, zero);  // [S]B - [k]A = O
    }
  } else if (c == 8) {
    uint32_t T[8];
    adv_torsion(T, 1u + u % 7u);
    ge_p3 nA, nT;
    ge_frombytes_negate_vartime(nA, A);
    ge_frombytes_negate_vartime(nT, T);
    ge_cached cT;
    ge_p3_to_cached(cT, nT);
    ge_p1p1 t;
    ge_add_cached(t, nA, cT);  // -(A + T)
    ge_p2 s;
    ge_p1p1_to_p2(s, t);
    fe nx;
    fe_neg(nx, s.X);
    s.X = nx;
    ge_tobytes(A, s);
    sha512_hram32(h, R, A, M);
    sc_reduce64(k, h);
    sc_muladd(S, k, a, r);
  } else if (c == 9) {
    const uint32_t j = 2u + u % 17u;
#pragma unroll
    for (int i = 0; i < 8; ++i) A[i] = i == 0 ? 0xffffffedu + j : (i == 7 ? 0x7fffffffu : 0xffffffffu);
    A[7] |= ((u >> 8) & 1u) << 31;
  } else if (c == 10) {
    const uint32_t sign = A[7] & 0x80000000u;
    uint32_t y[8], one[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      y[i] = A[i];
      one[i] = i == 0 ? 1u : 0u;
    }
    y[7] &= 0x7fffffffu;
    for (uint32_t j = 1; j <= 64u; ++j) {
      adv_add256(y, one);
      if (!point_is_canonical(y) || (y[7] >> 31) != 0) continue;
      uint32_t cand[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) cand[i] = y[i];
      cand[7] |= sign;
      ge_p3 tmp;
      if (!ge_frombytes_negate_vartime(tmp, cand)) {
#pragma unroll
        for (int i = 0; i < 8; ++i) A[i] = cand[i];
        break;
      }
    }
  }
}

}  // namespace stl
